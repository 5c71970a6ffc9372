// Sample encode prelude (config E: 10 x f32) for `make jitcheck`.
#define MJE_BS 2
#define MJE_CAP 40
#define MJE_NCOLS 10
#define MJE_NUTF8 0
#define MJE_STAGE 32768
#define MJE_COLS(X) X(0, 4, 0, 0) X(1, 4, 4, 0) X(2, 4, 8, 0) X(3, 4, 12, 0) X(4, 4, 16, 0) X(5, 4, 20, 0) X(6, 4, 24, 0) X(7, 4, 28, 0) X(8, 4, 32, 0) X(9, 4, 36, 0)
