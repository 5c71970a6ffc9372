// murr_internal.h — device descriptors shared by the kernels (murr_kernels.hip)
// and the host side of the C ABI (murr_abi.cpp).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/murr_codec.h"

namespace murr {

// Threads per encode workgroup (4 waves).
constexpr uint32_t kTile = 256;
// JIT encode scan: tiles per workgroup of its group passes (a multiple of
// 1024; murr_jit_encode.hip MJE_SCAN_PER).  1024 spreads the pass that also
// derives tile totals from the offsets over more CUs than 4096 did.
constexpr uint32_t kEncScanPer = 1024;
// Bytes of assembled rows an encode tile stages through LDS.  Tiles whose
// byte span exceeds the stage read / write HBM directly (the "global" path).
constexpr uint32_t kStage = 32768;
// Default decode stage (bytes of row blobs per tile held in LDS).
constexpr uint32_t kDecStage = 36864;
// Workspace head: the error word, then phase-stamp slots of tuning builds
// (err[2 .. 2 + kStampSlots)), then eight spare 64-B lines (round 4's
// per-XCD claim counters, removed in round 5), then the per-(block, column)
// counters.
constexpr uint32_t kStampSlots = 16;
constexpr uint32_t kPoolWord = 2 + kStampSlots, kPoolStride = 8;
constexpr uint64_t kErrBytes = 8 * (kPoolWord + 8 * kPoolStride);
// Projected columns per decode call (10 bits in the packed error key).
constexpr uint32_t kMaxProj = 1024;


struct DecBlock {             // one block (batch read) of row blobs
    const uint8_t* data;
    const uint64_t* row_off;  // n_rows + 1 (u64, or u32 when ro32: then really a const uint32_t*)
    uint64_t n_rows;
    uint64_t tile_base;       // first global tile of this block
    const uint64_t* uidx;     // its utf8 index (murr_utf8_index) or null (JIT kernel only)
    uint32_t ro32, pad;       // row_off holds u32 offsets (murr_block_t.row_off32; JIT kernel only)
};
static_assert(sizeof(DecBlock) == 48, "mj::Blk layout");
// The offsets of a public block as the kernels take them.
inline DecBlock dec_block(const murr_block_t& b, uint64_t tile_base, const uint64_t* uidx) {
    return DecBlock{b.data, b.row_off32 ? (const uint64_t*)(const void*)b.row_off32 : b.row_off, b.n_rows, tile_base,
                    uidx, b.row_off32 ? 1u : 0u, 0u};
}

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
    uint64_t* lookback;          // [nutf8 * total_tiles] tile aggregates + 1 (window mode)
    unsigned long long* nulls;   // [nblocks * nproj]
    unsigned long long* lens;    // [nblocks * nproj] utf8 data bytes
    unsigned long long* err;     // max of ~key (0 = no error)
    uint64_t total_tiles;
    uint32_t nblocks, nproj, nutf8, bs;
    uint32_t stage;              // blob bytes a slot stages (multiple of 1 KiB)
    uint32_t rows_per_tile;      // rows per fill: 64 * chunks per sub-tile * consumer waves
    uint32_t local;              // 1: block-local mode (a workgroup owns whole blocks)
    uint32_t ufix[2];            // projection index of utf8 columns 0 and 1
    // loader ring: slots, fills in flight, LDS-DMA instructions per fill
    // (row offsets, blob stage), bytes per slot
    uint32_t nslots, depth, dro, dst, slot_bytes;
    // LDS plan (byte offsets), filled by decode_lds_plan: inside a slot the
    // row-offset slice at lds_ro and the stage at lds_stage; after the slots
    // the ready flags / free counters, span ring, look-back ring (flags,
    // aggregates, inclusive prefixes), per-wave null counters, a DMA scratch
    // and the per-slot fill aggregates of window mode (sums, counters).
    uint32_t lds_ro, lds_stage, lds_ready, lds_free, lds_span, lds_lbf, lds_lba, lds_lbi, lds_nulls, lds_scratch,
        lds_fa, lds_fc, lds_total;
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
    uint64_t* row_off;           // n_rows + 1, written as row_base + offset in out
    uint64_t* lookback;          // [total_tiles]
    unsigned long long* err;     // max of ~key
    uint64_t n_rows, out_cap, total_tiles;
    uint32_t ncols, nutf8, bs, cap;
    uint64_t row_base;
};

// Packed first-error key: block(18) | row(32) | column(10) | status(4); the
// smallest key is the reference's first error (row-major, then column).
__host__ __device__ inline uint64_t err_key(uint64_t block, uint64_t row, uint32_t col,
                                            uint32_t status) {
    if (row > 0xFFFFFFFFull) row = 0xFFFFFFFFull;
    if (block > 0x3FFFFull) block = 0x3FFFFull;
    return (block << 46) | (row << 14) | ((uint64_t)(col & 0x3FF) << 4) | (status & 0xF);
}

// Layout-specialised decode kernel (murr_jit.cpp, murr_jit_kernel.hip): one
// module per segment layout holds every tile shape; the projection is a
// kernel argument.
constexpr uint32_t kJitShapes = 4;
// waves x 64-row chunks per decode wave x LDS ring slots (murr_jit_kernel.hip
// MJ_KERNEL instantiates each; a 3-slot ring measured no faster on B or C;
// 5x4 and 7x2 measured slower on B than 5x3; so did one 1024-thread
// workgroup per CU with 1920-row tiles (16x2: 1.16 vs 0.74 ms), 13x2 and 9x3
// at two per CU, although a bare LDS-DMA stream of this byte mix runs fastest
// at one workgroup per CU with 32 KiB tiles: tools/ubench/lds_mix*.hip)
constexpr uint32_t kJitShapeTab[kJitShapes][3] = {{5, 2, 2}, {5, 1, 2}, {3, 1, 2}, {5, 3, 2}};
struct JitShapeK {
    hipFunction_t fn = nullptr, fn_split = nullptr;  // local / split mode kernels
    uint32_t nw = 0, r = 0, tr = 0;  // waves (nw-1 decode, 1 loads), chunks per decode wave, rows per tile
    uint32_t nslot = 2;              // LDS ring slots (nslot - 1 tiles in flight)
    uint64_t uid = 0;                // unique per compiled module shape (never reused: keys per-kernel caches,
                                     // which must not outlive an unloaded module whose address is reused)
};
struct JitLayout {
    JitShapeK shapes[kJitShapes];
    uint32_t ncols = 0;
};
struct JitSeg {                    // = mj::Seg: rows [r_begin, r_end) of block b (split mode)
    uint32_t b, first;             // first: index of the block's first segment
    uint64_t r_begin, r_end;
};
struct JitArgsHead {               // = mj::Args without its trailing slot[] (murr_jit_kernel.hip)
    const DecBlock* blocks;
    const DecOut* outs;            // [nblocks][nproj]
    const uint32_t* order;         // unused
    const JitSeg* segs;            // split mode: segments; local mode: (virtual) blocks
    const uint16_t* slot_tab;      // [ncols] output position per column (0xFFFF = not decoded)
    const uint16_t* projcols;      // [nproj] column per output position
    unsigned long long* nulls;
    unsigned long long* lens;
    unsigned long long* err;
    unsigned long long* flags;     // split mode: [nseg][max(nutf8, 1)] look-back granules, then a claim word
    uint8_t* sink;
    uint64_t nseg;
    uint32_t nblocks, nproj, norder, mode;  // mode: 0 local, 1 split
    uint32_t stage, report;
    uint32_t emit;                 // split mode: a second pass writes utf8 cells
    uint32_t ulog;                 // log2 of the utf8 index stride
    unsigned int* abort_word;      // split mode: a timed-out wait aborts the launch (zeroed)
    unsigned int* zero_next;       // prepared launches: the other counter set, zeroed by this launch
    uint32_t zero_words, rb_words;
    unsigned int* ticket;          // prepared launches: workgroups finished (in the counter set)
    unsigned long long* rb_host;   // prepared launches: pinned read-back + done flag (last round only)
    uint32_t fast;                 // the loader's fast start: cut and split launches (murr_jit_kernel.hip)
    uint32_t pad_;
};
static_assert(sizeof(JitArgsHead) == 176, "mj::Args layout");
// The compiled layout (cached; least recently used beyond 64 are retired).
// pin: the caller will launch from it and calls jit_layout_unpin after the
// launch is enqueued; until then no eviction unloads its module.
const JitLayout* jit_layout(int device, const murr_segment_t* seg, std::string* why, bool pin = false);
void jit_layout_unpin(const JitLayout* k);
size_t jit_layout_cached();  // layouts held in memory (tests)
size_t jit_layout_limit(size_t n);  // set the in-memory bound (n > 0) and return it
uint32_t jit_lds_bytes(uint32_t nw, uint32_t r, uint32_t nslot, uint32_t stage, uint32_t nutf8);
hipError_t jit_decode_launch(const JitShapeK& k, bool split, const void* args, size_t bytes, uint32_t grid,
                             uint32_t lds, hipStream_t s);

// Run-time specialised encode kernel (murr_jit.cpp, murr_jit_encode.hip).
struct JitEncKernel {
    hipFunction_t fn, fn_sizes, fn_scan;  // encode; tile sizes and their scan (utf8 layouts)
    int bpc;        // resident workgroups per CU
    uint32_t tile;  // rows per tile = threads per workgroup (jit_encode_tile)
};
struct EncCol;
// stage: LDS bytes of a tile's blobs (jit_encode_stage), a compile-time size.
uint32_t jit_encode_stage(uint64_t n_rows, uint64_t blob_cap, uint32_t tile);
// LDS bytes per wave for the encode's string staging (murr_jit_encode.hip
// MJE_SBW): a wave's 64 rows of string bytes over every utf8 column with
// headroom, in powers of two from 512 to 4096; 0 without utf8 columns.
uint32_t jit_encode_sbw(uint64_t n_rows, uint64_t blob_cap, uint32_t fixed, uint32_t nutf8);
// tile: rows per encode tile (jit_encode_tile: 256).
uint32_t jit_encode_tile(uint64_t n_rows, uint64_t blob_cap);
const JitEncKernel* jit_encode_kernel(int device, uint32_t bs, uint32_t cap, const EncCol* cols, uint32_t ncols,
                                      uint32_t stage, uint32_t tile, uint32_t sbw, std::string* why);
struct EncodeArgs;
// Tile totals of utf8 layouts: kEncSizesPass (murr_jit_encode_sizes, exact),
// kEncSizesInline (no utf8 column has a validity buffer: the scan computes
// them from the offsets, exact), kEncSizesEstimate (the scan estimates them
// from the offsets and validity popcounts; exact when every null string is
// empty, checked by the encode kernel).
enum : uint32_t { kEncSizesPass = 0, kEncSizesInline = 1, kEncSizesEstimate = 2 };
constexpr int kEncStRecount = 12;  // murr_jit_encode.hip kStRecount
hipError_t jit_encode_launch(const JitEncKernel* k, const EncodeArgs& a, uint32_t grid, hipStream_t s,
                             uint32_t sizes);

void decode_lds_plan(DecodeArgs& a, uint32_t nw, uint32_t kc, uint32_t slots, uint32_t depth);
bool decode_shape_ok(uint32_t nw, uint32_t kc);
hipError_t launch_decode(const DecodeArgs& a, uint32_t nw, uint32_t kc, uint32_t grid, hipStream_t s);
int decode_blocks_per_cu(uint32_t nw, uint32_t kc, uint32_t lds);
hipError_t launch_encode(const EncodeArgs& a, uint32_t grid, hipStream_t s);
int encode_blocks_per_cu();

// RocksDB data blocks (murr_sst.hip, murr_sst_decode).
struct SstBlock {                  // = murr_sst_block_t
    const uint8_t* data;
    uint64_t size;
    uint32_t compression, pad;
};
// A tier-0 block's HBM slot: up to 1 KiB uncompressed plus a pad the
// thread-per-block inflate may overrun into (murr_sst.hip, tmatch).
constexpr uint64_t kSstSlot = 1024 + 64;
struct SstArgs {
    const SstBlock* blocks;
    uint64_t nblocks;
    uint32_t* tier;                // [nblocks] 0 / 1: LDS slot tier; 2: one thread, through raw
    uint64_t* ulen;                // [nblocks] uncompressed size of a tier-2 block (0 otherwise)
    uint64_t* uoff;                // [nblocks] its placement in raw (prefix of ulen)
    uint8_t* raw;                  // tier-2 blocks uncompressed, back to back
    uint8_t* slots;                // [nblocks][kSstSlot] compressed tier-0 blocks, inflated by sst_count
    uint32_t* rlen;                // [nblocks] uncompressed size of a tier-0/1 block
    uint32_t* list;                // tier-1 blocks, *nlist of them
    uint32_t* nlist;
    uint64_t *ne, *kb, *vb;        // [nblocks] entries / key bytes / value bytes
    uint64_t *eoff, *koff, *voff;  // [nblocks] their exclusive prefixes
    uint8_t* keys;                 // user keys back to back
    int32_t* key_off;              // [entries + 1]
    uint8_t* vals;                 // values (row blobs) back to back
    uint64_t* val_off;             // [entries + 1]
    uint64_t* seqs;
    uint8_t* types;
    unsigned long long* err;
    uint32_t probe, pad;           // tuning builds (MURR_SST_PROBE): sst_count_t phase ablations; 0
};
hipError_t launch_sst_count(const SstArgs& a, hipStream_t s);      // tiers 0 and 1; flags tier 2
hipError_t launch_sst_big_count(const SstArgs& a, hipStream_t s);  // tier 2: inflate to raw, count
hipError_t launch_sst_decode(const SstArgs& a, hipStream_t s);     // tiers 0 and 1, after the scans
hipError_t launch_sst_big_decode(const SstArgs& a, hipStream_t s); // tier 2
// k <= 4 scans of n-element arrays at once: y[j] = exclusive prefix of x[j],
// its total -> *total[j]; part: k * ceil(n / 1024) scratch.
struct ScanSet {
    const uint64_t* x[4];
    uint64_t* y[4];
    uint64_t* total[4];
    uint64_t* part;
    uint32_t k, pad;
};
hipError_t launch_scan_u64_n(const ScanSet& S, uint64_t n, hipStream_t s);

// utf8 index of a block (murr_index.hip, murr_utf8_index).
constexpr uint32_t kMaxUidxCols = 64;
struct Utf8IndexArgs {
    const uint8_t* data;
    const uint64_t* row_off;
    const uint32_t* row_off32;     // or these (murr_block_t.row_off32)
    uint64_t* out;                 // [(n + stride - 1) / stride + 1][nu]
    uint64_t* part;                // scratch: [windows][nu] window sums
    uint64_t from;                 // rows before `from` are indexed already (their entries, and the
                                   // total at entry ceil(from / stride), are in out)
    uint64_t n, stride;
    uint32_t bs, nu;
    uint32_t col[kMaxUidxCols];    // segment column index of utf8 column u
    uint32_t fo[kMaxUidxCols];     // its slot's row offset (bitset_size + offset)
};
hipError_t launch_utf8_index(const Utf8IndexArgs& a, hipStream_t s);
hipError_t launch_utf8_row_lengths(const Utf8IndexArgs& a, uint32_t* out, hipStream_t s);  // rows [from, n)
uint64_t utf8_index_windows(uint64_t from, uint64_t n, uint64_t stride);  // part[] entries per column

// Device key index + row gather (murr_index.hip).
constexpr uint32_t kMissing = 0xFFFFFFFFu;
struct IndexArgs {
    const uint8_t* key_data;    // the index's own copy of the keys (Arrow utf8)
    const int32_t* key_off;     // n + 1
    uint64_t* slots;            // mask + 1 entries {tag:32 | row:32}, ~0 = empty
    uint64_t* loc;              // mask + 1 entries {key start:32 | key length:32}
    uint64_t mask;
    uint64_t n;
    uint64_t base;              // insert: keys (and rows) base .. base + n - 1
    unsigned long long* err;
    const uint8_t* q_data;      // query keys (Arrow utf8)
    const int32_t* q_off;       // nq + 1
    uint64_t nq;
    uint32_t* rows;             // out: nq rows (kMissing = not found)
    const uint8_t* blob;        // gather: the table's row blobs
    const uint64_t* row_off;    //   and their offsets (n + 1)
    uint64_t* sizes;            //   out: the block's row offsets (nq + 1)
    uint8_t* out;               //   out: the block's bytes
    uint64_t out_cap;
    uint64_t* needed;           //   out (optional): unclamped block bytes
    uint64_t* scratch;          //   scan group sums
    const uint32_t* src;        // multi-shard gather: caller query -> grouped position
    uint64_t nq_live;           // probe: queries [nq_live, nq) are misses without a lookup (a
                                //   prepared read's padding to its capacity); 0 = all nq live
    unsigned long long* lb;     // small gathers (nq <= 1024): the fused kernel's look-back words
                                //   [kGatherGroups][1 + kGatherMaxU], zero at launch; null = the
                                //   two-launch form
    unsigned long long* lb_other;  //   the other word set, zeroed by this launch for the next
    const uint32_t* ulen;       // fused gather (optional): the table's per-row utf8 string bytes
                                //   [n][nu] (murr_utf8_row_lengths), with them
    uint64_t* uidx;             //   out: the gathered block's utf8 index at stride 64
    uint32_t nu;                //   utf8 columns (1 .. kGatherMaxU)
    uint32_t nu_rc;             // slot cache: utf8 columns of ru (murr_index_cache_rows)
    uint64_t* kp;               // per slot: the key's first 16 bytes, zero-padded (written by insert)
    uint64_t* rc;               // slot cache (optional, probe): per slot {row offset, row bytes}
    uint32_t* ru;               //   and the row's utf8 string bytes [nu_rc]
    uint64_t* stamps;           // tuning builds: gather_fused's phase clocks [group][kGatherStamps]
};
constexpr uint32_t kGatherStamps = 5;  // entry, probed, look-back done, published, copied
constexpr uint32_t kGatherGroups = 16;  // 64-query groups of a fused small gather
constexpr uint32_t kGatherMaxU = 4;     // utf8 columns a fused gather indexes
constexpr uint32_t kGatherWords = kGatherGroups * (1 + kGatherMaxU);  // look-back words per set
// Shards of a multi-GPU read (murr_multi_gather): arenas, row offsets and the
// end of each shard's grouped query range.
constexpr uint32_t kMaxShards = 16;
struct MultiTab {
    uint32_t n;
    const uint8_t* arena[kMaxShards];
    const uint64_t* row_off[kMaxShards];
    uint64_t q_end[kMaxShards];
};
hipError_t launch_multi_gather(const IndexArgs& a, const MultiTab& t, bool copy, hipStream_t s);
hipError_t launch_multi_copy(const IndexArgs& a, const MultiTab& t, hipStream_t s);
hipError_t launch_index_insert(const IndexArgs& a, hipStream_t s);
// the slot cache of rows [from, a.n): rc / ru of each row's slot when the
// slot holds that row (a.rc, a.ru, a.nu_rc; row_off / ulen of the table)
hipError_t launch_index_cache_rows(const IndexArgs& a, const uint64_t* row_off, const uint32_t* ulen, uint64_t from,
                                   hipStream_t s);
hipError_t launch_index_probe(const IndexArgs& a, hipStream_t s);
hipError_t launch_index_seq(const IndexArgs& a, const uint64_t* seqs, unsigned long long* best,
                            unsigned long long* win, hipStream_t s);
uint64_t gather_scan_groups(uint64_t nq);
uint64_t gather_scratch_words(uint64_t nq);  // A.scratch (u64) a launch_gather of nq queries needs
hipError_t launch_gather(const IndexArgs& a, hipStream_t s);
hipError_t launch_gather_scan(const IndexArgs& a, hipStream_t s);  // probe + sizes + scan, no copy
hipError_t launch_gather_copy(const IndexArgs& a, hipStream_t s);  // the copy of a scanned gather
hipError_t launch_offsets_rebase(int32_t* dst, const int32_t* src, uint64_t n, int64_t add, hipStream_t s);

// Segment copies by a kernel (murr_kernels.hip copy_segs_kernel): pinned host
// <-> device over PCIe as the CUs' own loads and stores (the streaming host
// decode's transfers), `grid` workgroups at most.
struct CopySeg {
    const uint8_t* src;
    uint8_t* dst;
    uint64_t bytes;       // the length, or (len set) its bound
    const int32_t* len;   // null, or a device int32 holding the length (clamped to [0, bytes])
};
constexpr uint32_t kMaxCopySegs = 12;
struct CopyArgs {
    CopySeg seg[kMaxCopySegs];
    uint32_t nseg;
};
hipError_t launch_copy_segs(const CopySeg* segs, uint32_t n, uint32_t grid, hipStream_t s);
// Row offsets u64 <-> u32, n entries (murr_kernels.hip).
hipError_t launch_row_off_narrow(const uint64_t* in, uint32_t* out, uint64_t n, unsigned int* bad, hipStream_t s);

// Arrow IPC framing (murr_ipc.cpp, murr_ipc.hip).
enum : uint32_t { kIpcValidity = 0, kIpcOffsets = 1, kIpcValues = 2 };
struct IpcPlan {
    std::vector<uint8_t> meta;          // 0xFFFFFFFF, size, flatbuffer, padding
    std::vector<uint64_t> buf_off, buf_len;  // body buffers in IPC order (offsets from the body start)
    std::vector<uint32_t> buf_field, buf_kind;
    uint64_t body_len = 0;
};
bool ipc_align_ok(uint32_t a);
int ipc_schema(const murr_segment_t* seg, const uint32_t* proj, uint32_t nproj, const char* const* names,
               uint32_t align, std::vector<uint8_t>* out);
int ipc_batch_plan(const murr_segment_t* seg, const uint32_t* proj, uint32_t nproj, uint64_t n,
                   const uint64_t* null_counts, const uint64_t* data_lens, uint32_t align, IpcPlan* plan);
struct IpcJob {                 // copy src[0..len) to dst[0..len), zero dst[len..padded)
    const uint8_t* src;
    uint8_t* dst;
    uint64_t len, padded;
};
hipError_t launch_ipc_pack(const IpcJob* jobs, uint32_t njobs, uint64_t max_padded, hipStream_t s);

}  // namespace murr
