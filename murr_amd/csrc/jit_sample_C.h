// Sample prelude (config C: 16 mixed nullable columns, 2 utf8) for `make jitcheck`;
// generated from murr_amd.schema.SegmentSchema as murr_jit.cpp's prelude() does.
#define MJ_BS 2
#define MJ_FIX 73
#define MJ_NCOLS 16
#define MJ_NUTF8 2
#define MJ_COLS(X) X(0, 9, 2, 0) X(1, 1, 3, 0) X(2, 2, 4, 0) X(3, 4, 6, 0) X(4, 8, 10, 0) X(5, 1, 18, 0) X(6, 2, 19, 0) X(7, 4, 21, 0) X(8, 8, 25, 0) X(9, 4, 33, 0) X(10, 8, 37, 0) X(11, 0, 45, 0) X(12, 0, 49, 1) X(13, 4, 53, 0) X(14, 8, 57, 0) X(15, 8, 65, 0)
#define MJ_OUT_NT_LAYOUT 1
