// Sample prelude (config B: f32 + utf8, bs 1) for `make jitcheck`; the real
// prelude is generated per segment layout by murr_jit.cpp.
#define MJ_BS 1
#define MJ_FIX 9
#define MJ_NCOLS 2
#define MJ_NUTF8 1
#define MJ_COLS(X) X(0, 4, 1, 0) X(1, 0, 5, 0)
