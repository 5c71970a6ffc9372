// Sample encode prelude (config C's 16 mixed nullable columns) for `make jitcheck`.
#define MJE_BS 2
#define MJE_CAP 71
#define MJE_NCOLS 16
#define MJE_NUTF8 2
#define MJE_STAGE 32768
#define MJE_SCAN_PER 1024
#define MJE_COLS(X) X(0, 9, 0, 0) X(1, 1, 1, 0) X(2, 2, 2, 0) X(3, 4, 4, 0) X(4, 8, 8, 0) X(5, 1, 16, 0) X(6, 2, 17, 0) X(7, 4, 19, 0) X(8, 8, 23, 0) X(9, 4, 31, 0) X(10, 8, 35, 0) X(11, 0, 43, 0) X(12, 0, 47, 1) X(13, 4, 51, 0) X(14, 8, 55, 0) X(15, 8, 63, 0)
