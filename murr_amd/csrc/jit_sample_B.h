// Sample prelude (config B: f32 + utf8, bs 1) for `make jitcheck`; the real
// prelude is generated per launch layout by murr_jit.cpp.
#define MJ_NW 5
#define MJ_R 2
#define MJ_SLOTS 2
#define MJ_STAGE 12288
#define MJ_BS 1
#define MJ_NPROJ 2
#define MJ_NUTF8 1
#define MJ_FIXED(X) X(0, 4, 1, 0)
#define MJ_UTF8(X) X(1, 0, 5, 1)
#define MJ_COL_FO 1, 5
#define MJ_COL_BIT 0, 1
#define MJ_COL_WID 4, 0
