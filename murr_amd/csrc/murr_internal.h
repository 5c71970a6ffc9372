// murr_internal.h — device descriptors shared by the kernels (murr_kernels.hip)
// and the host side of the C ABI (murr_abi.cpp).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace murr {

// Threads per encode workgroup (4 waves).
constexpr uint32_t kTile = 256;
// Decode workgroup: kDW waves (kDT threads); a decode tile is kDT * KMAX rows.
constexpr uint32_t kDW = 8, kDT = 64 * kDW;
// Bytes of assembled rows an encode tile stages through LDS.  Tiles whose
// byte span exceeds the stage read / write HBM directly (the "global" path).
constexpr uint32_t kStage = 32768;
// Default decode stage (bytes of row blobs per tile held in LDS).
constexpr uint32_t kDecStage = 36864;
// Projected columns per decode call (10 bits in the packed error key).
constexpr uint32_t kMaxProj = 1024;


struct DecBlock {             // one block (batch read) of row blobs
    const uint8_t* data;
    const uint64_t* row_off;  // n_rows + 1
    uint64_t n_rows;
    uint64_t tile_base;       // first global tile of this block
};

struct DecProj {              // one projected column
    uint32_t dtype, bit, offset, width;
    uint32_t is_utf8, uslot;  // uslot = ordinal among projected utf8 columns
};

struct DecOut {               // one output Arrow array (block, column)
    uint8_t* values;
    uint8_t* validity;
    int32_t* offsets;
    uint64_t values_cap;
};

struct DecodeArgs {
    const DecBlock* blocks;
    const DecProj* proj;
    const DecOut* outs;          // [nblocks * nproj]
    uint64_t* lookback;          // [nutf8 * total_tiles] tile aggregates + 1
    uint64_t* prev;              // [grid * nutf8] each workgroup's last inclusive prefix
    unsigned long long* nulls;   // [nblocks * nproj]
    unsigned long long* lens;    // [nblocks * nproj] utf8 data bytes
    unsigned long long* err;     // max of ~key (0 = no error)
    unsigned long long* stamps;  // [8] cycle sums per phase (MURR_DEBUG_DECODE & 8 only)
    uint64_t total_tiles;
    uint32_t nblocks, nproj, nutf8, bs, cap, stage;
    uint32_t debug;              // ablation switches (MURR_DEBUG_DECODE), 0 in production
    uint32_t rows_per_tile;      // multiple of 256
    uint32_t cell_cols;          // utf8 columns whose cells phase A caches in LDS
    uint32_t local;              // 1: block-local mode (a workgroup owns whole blocks)
    // LDS plan (byte offsets), filled by launch_decode: buffer b of the two
    // tile buffers starts at b * lds_buf; inside it the chunk prefixes at 0,
    // the row-offset slice at lds_rowoff, the blob stage at lds_stage.
    uint32_t lds_rowoff, lds_stage, lds_buf, lds_nulls, lds_w, lds_mine, lds_st, lds_cell, lds_total;
};

struct EncCol {               // one Arrow input column, segment order
    const uint8_t* values;
    const uint8_t* validity;
    const int32_t* offsets;
    uint64_t offset;
    uint32_t dtype, index, soff, width;
};

struct EncodeArgs {
    const EncCol* cols;
    uint8_t* out;
    uint64_t* row_off;           // n_rows + 1
    uint64_t* lookback;          // [total_tiles]
    unsigned long long* err;     // max of ~key
    uint64_t n_rows, out_cap, total_tiles;
    uint32_t ncols, nutf8, bs, cap;
};

// Packed first-error key: block(18) | row(32) | column(10) | status(4); the
// smallest key is the reference's first error (row-major, then column).
__host__ __device__ inline uint64_t err_key(uint64_t block, uint64_t row, uint32_t col,
                                            uint32_t status) {
    if (row > 0xFFFFFFFFull) row = 0xFFFFFFFFull;
    if (block > 0x3FFFFull) block = 0x3FFFFull;
    return (block << 46) | (row << 14) | ((uint64_t)(col & 0x3FF) << 4) | (status & 0xF);
}

uint32_t decode_lds_bytes(uint32_t stage, uint32_t nproj, uint32_t nutf8, uint32_t rows_per_tile,
                          uint32_t cell_cols);
hipError_t launch_decode(const DecodeArgs& a, uint32_t grid, hipStream_t s);
hipError_t launch_encode(const EncodeArgs& a, uint32_t grid, hipStream_t s);
int decode_blocks_per_cu(uint32_t lds, uint32_t rows_per_tile);
int encode_blocks_per_cu();

}  // namespace murr
