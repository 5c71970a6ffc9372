/*
 * murr_codec.h — C ABI of the MI355X (gfx950) row-blob codec.
 *
 * This is the drop-in boundary for murr's `src/io` encode/decode path.  Every
 * entry point names the reference interface it replaces (paths are relative to
 * the murrdb/murr source tree, v0.2.1).  Plain C: pointers, sizes and status
 * codes only; no exceptions cross this boundary.
 *
 * Naming follows the north star, not the reference:
 *   decode = row blobs -> Arrow buffers  (reference ColumnEncoder / ReadBatchBuilder)
 *   encode = Arrow buffers -> row blobs  (reference ColumnDecoder / WriteRow)
 * (src/io/codec/mod.rs:43-51; .memory/io_codec_design.md explains the inversion.)
 *
 * Row blob layout (src/io/row/write.rs:19-52, src/io/row/read.rs:22-56):
 *   [bitset: bs = ceil(C/8) bytes, bit i set <=> column i NULL, init 0xFF]
 *   [static region: capacity bytes, column i at offset_i, little endian]
 *   [payloads: per non-null utf8 column in column order: u32 len, bytes]
 * A utf8 static slot holds the payload offset relative to the static region.
 *
 * Threading: a murr_ctx_t owns one HIP stream and one workspace; calls on one
 * context must be serialised by the caller (the reference reads under
 * RwLock::read with one ReadBatchBuilder per request, src/io/table/mod.rs:127).
 * Use one context per calling thread for concurrency.  Kernels are stateless.
 */
#ifndef MURR_CODEC_H
#define MURR_CODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version.  2 (round 5): murr_block_t grew row_off32 (32 -> 40 bytes) and
 * murr_opts_t.balance became `reserved` (must be 0).  A binding checks
 * murr_abi_version() against the version it was written for before passing
 * any descriptor array, so a stale caller fails fast
 * instead of handing over arrays of the old stride. */
#define MURR_ABI_VERSION 2

/* DTypeName, same members and order as src/core/schema.rs:6-19. */
typedef enum {
    MURR_UTF8 = 0,
    MURR_BOOL = 1,
    MURR_INT8 = 2,
    MURR_INT16 = 3,
    MURR_INT32 = 4,
    MURR_INT64 = 5,
    MURR_UINT8 = 6,
    MURR_UINT16 = 7,
    MURR_UINT32 = 8,
    MURR_UINT64 = 9,
    MURR_FLOAT32 = 10,
    MURR_FLOAT64 = 11,
    MURR_NUM_DTYPES = 12
} murr_dtype_t;

/* Status codes.  MurrError variants (src/core/error.rs:4-19) map as noted. */
typedef enum {
    MURR_OK = 0,
    MURR_E_INVALID_UTF8 = 1,    /* SegmentError("invalid utf8: ..."), src/io/codec/utf8.rs:90-92 */
    MURR_E_DTYPE = 2,           /* SegmentError("expected ..., got ..."), src/io/codec/mod.rs:78-85 */
    MURR_E_BAD_COLUMN = 3,      /* SegmentError("column '...' not found"), src/io/table/mod.rs:115-123 */
    MURR_E_OFFSET_OVERFLOW = 4, /* arrow-rs StringBuilder panics past i32::MAX; we report instead */
    MURR_E_MALFORMED_ROW = 5,   /* reference panics on the out-of-bounds slice (read.rs:39-55) */
    MURR_E_CAPACITY = 6,        /* caller-provided output buffer too small (required size reported) */
    MURR_E_ARGUMENT = 7,        /* invalid argument (null pointer, bad dtype code, misaligned buffer) */
    MURR_E_NULL_KEY = 8,        /* SegmentError("null in key column"), src/io/table/mod.rs:80-82 */
    MURR_E_HIP = 9,             /* HIP runtime error; hip_error holds the hipError_t */
    MURR_E_INTERNAL = 10,       /* device protocol failure (bounded spin expired) */
    MURR_E_ARROW = 11,          /* ArrowError, e.g. RecordBatch with zero columns (read.rs:106-108) */
    MURR_E_NO_DEVICE = 12       /* no HIP device visible */
} murr_status_t;

/* First error of a call, in the reference's own order (row-major, then
 * projection order: ReadBatchBuilder::add_row loops encoders per row,
 * src/io/row/read.rs:85-91). */
typedef struct {
    int32_t  status;     /* murr_status_t */
    int32_t  hip_error;  /* hipError_t when status == MURR_E_HIP */
    uint32_t block;      /* block index inside a batched call */
    uint32_t column;     /* projected column position (decode) / segment column (encode) */
    uint64_t row;        /* row inside the block */
    uint64_t required;   /* MURR_E_CAPACITY: bytes required */
} murr_error_t;

/* SegmentColumnSchema (src/io/schema.rs:8-14), without the name. */
typedef struct {
    uint32_t index;   /* null-bit position = position among non-key columns */
    uint32_t dtype;   /* murr_dtype_t */
    uint32_t offset;  /* byte offset in the static region */
    uint32_t size;    /* DType::size() */
} murr_column_t;

/* SegmentSchema (src/io/schema.rs:16-31). */
typedef struct {
    uint32_t ncols;
    uint32_t bitset_size;  /* ceil(ncols / 8) */
    uint32_t capacity;     /* sum of sizes */
    uint32_t _pad;
    const murr_column_t* cols;
} murr_segment_t;

/* ---- layout ------------------------------------------------------------ */

/* DType::size() for each dtype (src/io/codec/<dtype>.rs `fn size`); -1 if unknown. */
int murr_dtype_size(uint32_t dtype);

/* From<&TableSchema> for SegmentSchema (src/io/schema.rs:33-54): `dtypes` are
 * the non-key columns in TableSchema (IndexMap) order.  Fills `cols_out[ncols]`
 * and `seg_out` (seg_out->cols = cols_out). */
int murr_segment_init(const uint32_t* dtypes, uint32_t ncols,
                      murr_column_t* cols_out, murr_segment_t* seg_out);

/* Bytes a validity / bool bitmap of n rows occupies in murr's output buffers:
 * ceil(n/8) rounded up to 8 (the kernels store whole 64-row words; bits past n
 * are zero, as arrow-rs leaves them). */
uint64_t murr_bitmap_bytes(uint64_t n_rows);

/* ---- context / device memory -------------------------------------------- */

typedef struct murr_ctx murr_ctx_t;

int  murr_ctx_create(int device, murr_ctx_t** out);
void murr_ctx_destroy(murr_ctx_t* ctx);
/* hipStream_t the context enqueues on (opaque pointer). */
void* murr_ctx_stream(murr_ctx_t* ctx);
/* Device time of the last decode / encode kernel(s), HIP events recorded on
 * the context stream around the kernel launches only (no copies). */
int  murr_ctx_last_kernel_ms(murr_ctx_t* ctx, float* ms);
/* Name of the kernel the last decode / encode launched: "murr_jit_decode" /
 * "murr_jit_encode" (run-time specialised) or "decode_kernel" /
 * "encode_kernel" (generic); "" before any.  A static string. */
const char* murr_ctx_last_kernel(murr_ctx_t* ctx);
int  murr_device_count(int* n);
/* Timing marks on the context's stream (benchmarks): murr_ctx_mark records
 * mark `which` (0-3) behind the work queued so far; murr_ctx_mark_ms waits for
 * mark b of context cb and returns the GPU time from mark a of context ca to
 * it (two contexts of one device: work spread over their streams). */
int murr_ctx_mark(murr_ctx_t* ctx, uint32_t which);
int murr_ctx_mark_ms(murr_ctx_t* ca, uint32_t a, murr_ctx_t* cb, uint32_t b, float* ms);

/* Kernel selection of one context, for tests and benchmarks.  All zero (the
 * state of a new context) = the library's own choice.  Set once; every later
 * call on the context reads it.  A release build reads no environment
 * variable on the decode / encode path. */
typedef struct {
    uint32_t kernel;        /* decode: 0 auto (layout-specialised, generic kernel if hiprtc
                               cannot compile the layout), 1 specialised only (a compile
                               failure is MURR_E_INTERNAL), 2 generic kernel */
    uint32_t mode;          /* specialised decode: 0 auto, 1 local (workgroups own whole
                               blocks), 2 split (segments + look-back), 3 local over blocks
                               cut on their utf8 index whenever every block can be cut */
    uint32_t shape_nw;      /* tile shape: waves per workgroup (0 = auto) ... */
    uint32_t shape_r;       /* ... and 64-row chunks per decode wave */
    uint32_t seg_tiles;     /* split mode: tiles per segment (0 = auto) */
    uint32_t vrows;         /* cut blocks: rows per virtual block (0 = auto) */
    uint32_t lds_budget;    /* LDS bytes per workgroup for the tile ring (0 = auto) */
    uint32_t stage;         /* LDS stage bytes per ring slot (0 = auto) */
    uint32_t encode_kernel; /* encode: 0 auto, 1 specialised only, 2 generic kernel */
    uint32_t verbose;       /* 1: one line per decode launch on stderr */
    uint32_t grid;          /* local mode: workgroups per launch (0 = auto: the co-resident
                               grid, each workgroup walking several (virtual) blocks);
                               0xFFFFFFFF = one workgroup per (virtual) block, handed to the
                               CUs by the hardware as workgroups finish */
    uint32_t reserved;      /* 0 (round 4's dynamic-tail switch, removed: measured slower) */
} murr_opts_t;
int murr_ctx_set_opts(murr_ctx_t* ctx, const murr_opts_t* opts);
int murr_ctx_get_opts(murr_ctx_t* ctx, murr_opts_t* opts);

/* What the context's decodes did (counters since creation). */
typedef struct {
    uint64_t decodes;        /* decode launches (murr_decode_enqueue*, a retry not counted) */
    uint64_t split_retries;  /* split-mode launches whose bounded look-back wait expired and
                                that were re-run in local mode (0 on a healthy device) */
    uint32_t last_mode;      /* last decode: 0 generic kernel, 1 local, 2 local over cut
                                blocks, 3 split (after a retry: the retry's mode) */
    uint32_t last_grid;      /* its workgroups */
    uint32_t last_shape_nw;  /* its tile shape (specialised kernel) */
    uint32_t last_shape_r;
    uint64_t readback_fallbacks;  /* prepared runs whose epilogue read-back flag never came
                                     (counts then copied back the ordinary way; 0 normally) */
    uint64_t encode_recounts;     /* encodes whose utf8 tile sizes, estimated from the offsets and
                                     validity (exact when null strings are empty), were off and
                                     recounted by a sizes pass (the encode then ran twice) */
} murr_ctx_stats_t;
int murr_ctx_stats(murr_ctx_t* ctx, murr_ctx_stats_t* out);

/* The in-memory cache of compiled segment layouts (murr_segment_prepare,
 * first decode of a layout): least recently used layouts beyond `max_layouts`
 * (default 64; 0 = leave it) are retired, their code objects unloaded only
 * after every launch that may use them has finished.  Reports the bound and
 * the layouts held.  The on-disk cache is not affected. */
int murr_jit_cache_limit(uint32_t max_layouts, uint32_t* limit, uint32_t* cached);

/* Device memory.  murr_dev_free also takes the device outputs the library
 * allocates for the caller (murr_sst_decode): those go back to the context's
 * reuse cache (at most 1 GiB, released by murr_ctx_destroy) for its next
 * call; anything else is freed.  A cached buffer is handed out again only
 * after a device synchronisation that follows its free, so work queued before
 * the free on any stream of the device (another context's scan of an adopted
 * arena, the caller's own) has finished reading it -- the guarantee hipFree
 * gives. */
int murr_dev_alloc(murr_ctx_t* ctx, uint64_t bytes, void** p);
int murr_dev_free(murr_ctx_t* ctx, void* p);
int murr_host_alloc(murr_ctx_t* ctx, uint64_t bytes, void** p); /* pinned */
int murr_host_free(murr_ctx_t* ctx, void* p);
int murr_memcpy_h2d(murr_ctx_t* ctx, void* dst, const void* src, uint64_t bytes);
int murr_memcpy_d2h(murr_ctx_t* ctx, void* dst, const void* src, uint64_t bytes);
int murr_memset_dev(murr_ctx_t* ctx, void* dst, int value, uint64_t bytes);
int murr_memcpy_d2d(murr_ctx_t* ctx, void* dst, const void* src, uint64_t bytes);
/* dst on ctx's device <- src on device src_device (xGMI peer copy when they
 * differ), enqueued on ctx's stream and waited for. */
int murr_memcpy_peer(murr_ctx_t* ctx, void* dst, const void* src, int src_device, uint64_t bytes);
int murr_sync(murr_ctx_t* ctx);

/* Compile (or load from the code-object cache) the decode and encode kernels
 * of a segment layout on the context's device.  Table::create / Table::open
 * (src/io/table/mod.rs:28-52, 131-154) are where a layout becomes known, so
 * calling this there keeps run-time compilation off the read and write paths:
 * the decode kernel is specialised on the layout only, and every projection
 * of the table (Table::read's `columns`, src/io/table/mod.rs:114-123) runs
 * the same code object.  Without it the first decode / encode of a layout
 * compiles.  Synchronous. */
int murr_segment_prepare(murr_ctx_t* ctx, const murr_segment_t* seg);

/* ---- device-resident decode (row blobs -> Arrow) ------------------------- */

/* A block = one batch read: n_rows row blobs back to back in `data`.
 * Row i is data[row_off[i] .. row_off[i+1]); an empty row is a missing key
 * (ReadBatchBuilder::add_empty, src/io/row/read.rs:93-98; a present row is
 * never empty when the segment has >= 1 column, write.rs:21).
 * `data` must be 16-byte aligned; all pointers are device pointers.
 *
 * Row offsets come in two widths.  `row_off` holds them as u64 (any block,
 * e.g. a resident table's arena past 4 GiB).  `row_off32`, when non-null,
 * holds them as u32 instead (4-byte aligned, n_rows + 1 entries, every value
 * below 2^32; `row_off` is then ignored and may be null): a batch read's block
 * is far below 4 GiB, and u32 offsets halve the index bytes the decode reads
 * (and a streamed batch sends over PCIe).  Same values, same meaning. */
typedef struct {
    const uint8_t*  data;
    const uint64_t* row_off;   /* n_rows + 1 entries, row_off[0] may be > 0 */
    uint64_t        n_rows;
    uint64_t        data_bytes; /* optional: row_off[n] - row_off[0] (0 = unknown);
                                   sizes the tiles, never read past */
    const uint32_t* row_off32; /* optional: the offsets as u32 (see above) */
} murr_block_t;

/* u64 row offsets -> u32 (device, n_rows + 1 entries each; `out` 4-byte
 * aligned).  Every offset is checked on the device: MURR_E_OFFSET_OVERFLOW
 * when one is >= 2^32, MURR_E_MALFORMED_ROW when one is below its predecessor
 * (`out` then holds unspecified values).  One kernel and a 4-byte read-back
 * on the context's stream; returns once `out` is written. */
int murr_row_off_narrow(murr_ctx_t* ctx, const uint64_t* row_off, uint64_t n_rows, uint32_t* out);

/* One output Arrow array (device pointers), arrow-rs 58 builder layout:
 *   fixed W:  values = n*W bytes, null slots zero
 *   bool:     values = bitmap (murr_bitmap_bytes(n)), null -> 0 bit
 *   utf8:     offsets = n+1 i32 starting at 0, values = string bytes (values_cap)
 *   validity: bitmap (murr_bitmap_bytes(n)), 1 = valid; the caller drops it
 *             when null_count == 0 (arrow-rs NullBufferBuilder materialises
 *             validity only after the first null), and its bytes are then
 *             unspecified (the decoder may not write them).
 * null_count / data_len are outputs. */
typedef struct {
    void*    values;
    uint8_t* validity;
    int32_t* offsets;
    uint64_t values_cap;
    uint64_t null_count;  /* out */
    uint64_t data_len;    /* out: utf8 string bytes; fixed: n*W; bool: ceil(n/8) */
} murr_array_t;

/* Batched ReadBatchBuilder::add_row/add_empty/build over device-resident
 * blocks (src/io/row/read.rs:62-110, encoders src/io/codec/primitive.rs:38-61,
 * bool_.rs:85-104, utf8.rs:85-105).  `proj[nproj]` are segment column indices
 * in request order (duplicates allowed).  `outs[b*nproj + p]` is block b,
 * projected column p.  Synchronous: returns after the stream drained and the
 * output counts are filled. */
int murr_decode_blocks(murr_ctx_t* ctx, const murr_segment_t* seg,
                       const uint32_t* proj, uint32_t nproj,
                       const murr_block_t* blocks, uint32_t nblocks,
                       murr_array_t* outs, murr_error_t* err);

/* Same as murr_decode_blocks but only enqueues; murr_decode_wait finishes it
 * (fills counts, reports errors).  One pending decode per context. */
int murr_decode_enqueue(murr_ctx_t* ctx, const murr_segment_t* seg,
                        const uint32_t* proj, uint32_t nproj,
                        const murr_block_t* blocks, uint32_t nblocks,
                        murr_array_t* outs);
int murr_decode_wait(murr_ctx_t* ctx, murr_error_t* err);

/* ---- prepared decode ---------------------------------------------------------
 * A batch read repeated over the same blocks and output buffers (a resident
 * table scanned again, a benchmark loop) prepared once: the launch shape,
 * descriptors and kernel arguments are computed and uploaded by
 * murr_decode_plan; each murr_decode_run zeroes the counters, launches, waits
 * and fills the arrays' counts exactly as murr_decode_blocks_ix would.  The
 * blocks' bytes and the output buffers may change between runs, their
 * addresses and sizes may not; `outs` is written by every run.  Free every
 * plan before its context. */
typedef struct murr_plan murr_plan_t;
int murr_decode_plan(murr_ctx_t* ctx, const murr_segment_t* seg,
                     const uint32_t* proj, uint32_t nproj,
                     const murr_block_t* blocks, uint32_t nblocks,
                     const uint64_t* const* uidx, uint32_t stride,
                     murr_array_t* outs, murr_plan_t** out);
int murr_decode_run(murr_plan_t* plan, murr_error_t* err);   /* synchronous */
/* murr_decode_run in two halves: _async launches the run on the context's
 * stream and returns; _wait waits for it and fills the arrays' counts.  One
 * run of a plan in flight at a time; runs of different plans on one context
 * queue in stream order, so a caller alternating two plans (two output sets)
 * launches the next run while the host finishes the previous one.  The
 * context's last kernel time (murr_ctx_last_kernel_ms) is that of the plan's
 * last timed run: one run in MURR_PLAN_TIME_EVERY, the first included, is
 * bracketed by timing events (an event between back-to-back launches costs
 * GPU time; plans on the generic kernel time every run).
 * When _wait returns, the run's kernel has ended: its outputs are visible to
 * the host, to other streams and to peer GPUs, not only in stream order. */
#define MURR_PLAN_TIME_EVERY 4
int murr_decode_run_async(murr_plan_t* plan);
int murr_decode_run_wait(murr_plan_t* plan, murr_error_t* err);
void murr_plan_free(murr_plan_t* plan);
/* The plan's timing period: one run in `every` (MURR_PLAN_TIME_EVERY by
 * default) is bracketed by timing events; 0 times none (a caller timing a
 * whole loop of runs with murr_ctx_mark instead). */
int murr_plan_time_every(murr_plan_t* plan, uint32_t every);

/* ---- utf8 index of a block (optional) --------------------------------------
 * For every utf8 column of the layout (column order), the string bytes of the
 * rows before row j * stride, j = 0 .. ceil(n_rows / stride): the offsets the
 * decode's utf8 arrays reach at those rows (Utf8Encoder::add_row,
 * src/io/codec/utf8.rs:86-96, with the cell rules of read.rs:45-55).  u64
 * entries, [j][nutf8].  Built once when a block is written; passed to the
 * decode beside the block, it lets many workgroups decode one large block,
 * each from a known starting offset, in one pass.  stride: a power of two in
 * [64, 2^30].  A layout without utf8 columns needs no index (len 0). */
uint64_t murr_utf8_index_len(const murr_segment_t* seg, uint64_t n_rows, uint32_t stride);
int murr_utf8_index(murr_ctx_t* ctx, const murr_segment_t* seg, const murr_block_t* block,
                    uint32_t stride, uint64_t* out /* device, murr_utf8_index_len entries */);  /* enqueue */
/* Extend an index after rows were appended to a block (MemoryStore::write
 * appends, src/io/store/memory.rs:47-60): `block` now holds n_rows rows, `out`
 * holds the index of its first `from` rows (murr_utf8_index_len(seg, from,
 * stride) entries, the last being their total) and has room for
 * murr_utf8_index_len(seg, n_rows, stride).  Reads only rows from .. n_rows.
 * from = 0 builds the whole index (= murr_utf8_index).  Enqueued. */
int murr_utf8_index_update(murr_ctx_t* ctx, const murr_segment_t* seg, const murr_block_t* block,
                           uint64_t from, uint32_t stride, uint64_t* out);
/* Per-row utf8 string bytes of a block's rows [from, n_rows): out[i * nutf8 +
 * u] (u32, device) = what row i's u-th utf8 column adds to the decode's utf8
 * offsets, by the index's cell rules (0 for a null, missing, short or
 * malformed cell).  A resident table keeps these beside its arena, extended
 * with every append, so a prepared read (murr_read_plan_new row_ulen) indexes
 * its gathered block inside the gather.  A layout without utf8 columns
 * writes nothing.  Enqueued. */
int murr_utf8_row_lengths(murr_ctx_t* ctx, const murr_segment_t* seg, const murr_block_t* block,
                          uint64_t from, uint32_t* out);
/* murr_decode_enqueue / murr_decode_blocks with an index per block (uidx[b]
 * null: block b has none; uidx null: no block has one).  Same outputs. */
int murr_decode_enqueue_ix(murr_ctx_t* ctx, const murr_segment_t* seg,
                           const uint32_t* proj, uint32_t nproj,
                           const murr_block_t* blocks, uint32_t nblocks,
                           const uint64_t* const* uidx, uint32_t stride, murr_array_t* outs);
int murr_decode_blocks_ix(murr_ctx_t* ctx, const murr_segment_t* seg,
                          const uint32_t* proj, uint32_t nproj,
                          const murr_block_t* blocks, uint32_t nblocks,
                          const uint64_t* const* uidx, uint32_t stride, murr_array_t* outs,
                          murr_error_t* err);

/* ---- device-resident encode (Arrow -> row blobs) -------------------------- */

/* One Arrow input column (device pointers).  `offset` is the Arrow array
 * offset in elements (bits for bitmaps).  validity == NULL means no nulls. */
typedef struct {
    const void*    values;    /* fixed: values; bool: bitmap; utf8: string data */
    const uint8_t* validity;
    const int32_t* offsets;   /* utf8 only */
    uint64_t       offset;
} murr_col_in_t;

/* Upper bound of the blob bytes murr_encode_batch writes for n_rows rows:
 * n*(bs+cap) + sum over utf8 columns of (4*n + utf8_data_bytes[c]).
 * utf8_data_bytes has one entry per segment column (ignored for non-utf8). */
uint64_t murr_encode_bound(const murr_segment_t* seg, uint64_t n_rows,
                           const uint64_t* utf8_data_bytes);

/* Table::write's per-row loop (src/io/table/mod.rs:97-109) over device
 * buffers: for every row, WriteRow::new (0xFF bitset, write.rs:20-28) then each
 * column's ColumnDecoder::write_to_row (primitive.rs:85-95, bool_.rs:111-117,
 * utf8.rs:113-119).  `cols[seg->ncols]` in segment order.  Writes the blobs
 * back to back into out_blob and out_row_off[n_rows+1] (row i =
 * out_blob[row_off[i]..row_off[i+1]), row_off[0] = 0).  *blob_len = bytes
 * written.  Keys stay with the caller (they are RocksDB keys, never in the blob). */
int murr_encode_batch(murr_ctx_t* ctx, const murr_segment_t* seg,
                      const murr_col_in_t* cols, uint64_t n_rows,
                      uint8_t* out_blob, uint64_t blob_cap,
                      uint64_t* out_row_off, uint64_t* blob_len,
                      murr_error_t* err);

/* murr_encode_batch writing row offsets from `row_base`: out_row_off[i] =
 * row_base + (offset of row i in out_blob), so a batch can be encoded straight
 * onto the tail of a growing blob arena whose offsets array already holds the
 * earlier rows (MemoryStore::write appends, src/io/store/memory.rs:47-60).
 * *blob_len = bytes written to out_blob. */
int murr_encode_batch_at(murr_ctx_t* ctx, const murr_segment_t* seg,
                         const murr_col_in_t* cols, uint64_t n_rows,
                         uint8_t* out_blob, uint64_t blob_cap, uint64_t* out_row_off,
                         uint64_t row_base, uint64_t* blob_len, murr_error_t* err);

/* murr_encode_batch that also writes the new block's utf8 index (uidx:
 * murr_utf8_index_len(seg, n_rows, stride) entries; unused when the layout
 * has no utf8 column), so a written block can be decoded by the whole GPU in
 * one pass (Table::write, src/io/table/mod.rs:54-112, is where a block
 * becomes known).  Synchronous, like murr_encode_batch. */
int murr_encode_batch_ix(murr_ctx_t* ctx, const murr_segment_t* seg,
                         const murr_col_in_t* cols, uint64_t n_rows,
                         uint8_t* out_blob, uint64_t blob_cap, uint64_t* out_row_off,
                         uint32_t stride, uint64_t* uidx, uint64_t* blob_len, murr_error_t* err);

/* ---- host-memory path (pinned staging + hipMemcpyAsync both ways) -------- */

/* Batched ReadBatchBuilder (src/io/row/read.rs:62-110) for the store-driven
 * read (Store::read feeds rows in caller order, src/io/store/rocksdb/mod.rs:259-266,
 * src/io/store/memory.rs:38-43).  add_row copies the pinned slice into a pinned
 * host staging block; build() = H2D + one decode launch + D2H into host
 * Arrow buffers owned by the builder (valid until murr_builder_free). */
typedef struct murr_builder murr_builder_t;

typedef struct {             /* host Arrow array produced by build() */
    const uint8_t* values;
    const uint8_t* validity; /* NULL when null_count == 0 */
    const int32_t* offsets;  /* utf8 only */
    uint64_t length;
    uint64_t null_count;
    uint64_t values_len;     /* bytes in values */
    uint32_t dtype;
    uint32_t _pad;
} murr_host_array_t;

int murr_builder_new(murr_ctx_t* ctx, const murr_segment_t* seg,
                     const uint32_t* proj, uint32_t nproj, uint64_t capacity,
                     murr_builder_t** out);
int murr_builder_add_row(murr_builder_t* b, const uint8_t* bytes, uint64_t len);
int murr_builder_add_empty(murr_builder_t* b);
/* Many rows at once: ptrs[i] == NULL is a missing key. */
int murr_builder_add_rows(murr_builder_t* b, const uint8_t* const* ptrs,
                          const uint64_t* lens, uint64_t n);
int murr_builder_build(murr_builder_t* b, murr_host_array_t* outs /* nproj */,
                       murr_error_t* err);
/* Milliseconds of the last build(): total, h2d copy, decode kernel, d2h copy. */
int murr_builder_last_timing(murr_builder_t* b, double* total_ms, float* h2d_ms,
                             float* kernel_ms, float* d2h_ms);
void murr_builder_free(murr_builder_t* b);

/* ---- streaming host decode ---------------------------------------------------
 * Batch reads back to back, host memory in and host memory out: the row blobs
 * a store hands over (the RocksDB block cache, src/io/store/rocksdb/mod.rs:
 * 259-266) go to the device, are decoded, and the Arrow buffers come back for
 * the egress (Flight DoGet, src/api/flight/mod.rs:85-87) -- pipelined, so the
 * H2D of batch i+1, the decode of batch i and the D2H of batch i-1 run at once.
 * `depth` (2..8) slots, each with its own stream, pinned staging, device
 * buffers and pinned outputs, all reused from batch to batch (nothing is
 * allocated per batch once the slots have grown to the batch size).
 *
 * murr_hstream_submit enqueues one batch (a host block: rows back to back at
 * data, row i = data[row_off[i] .. row_off[i+1]), an empty row a missing key)
 * and returns at once; murr_hstream_next waits for the oldest submitted batch
 * and points `outs` (nproj arrays) at its decoded buffers, valid until its slot
 * is submitted again (`depth` submits later).  At most `depth` batches may be
 * submitted and not yet returned (else MURR_E_ARGUMENT).  With
 * MURR_HSTREAM_PINNED the caller's data / row_off are pinned (murr_host_alloc or
 * hipHostRegister) and are copied to the device straight from there; they must
 * then stay unchanged until next() returns the batch.  Without it they are
 * copied into the slot's pinned staging first (one host memcpy) and may be
 * reused as soon as submit returns.  Errors of a batch (malformed rows, invalid
 * UTF-8, ...) are reported by the next() that returns it, as
 * ReadBatchBuilder::build (src/io/row/read.rs:100-109) would. */
typedef struct murr_hstream murr_hstream_t;
#define MURR_HSTREAM_PINNED 1u
int murr_hstream_new(murr_ctx_t* ctx, const murr_segment_t* seg, const uint32_t* proj,
                     uint32_t nproj, uint32_t depth, murr_hstream_t** out);
int murr_hstream_submit(murr_hstream_t* s, const uint8_t* data, const uint64_t* row_off,
                        uint64_t n_rows, uint32_t flags, murr_error_t* err);
/* The same batch with u32 row offsets (a block below 4 GiB, as every batch
 * read is): half the offset bytes staged and sent over PCIe, decoded as a
 * murr_block_t with row_off32. */
int murr_hstream_submit32(murr_hstream_t* s, const uint8_t* data, const uint32_t* row_off,
                          uint64_t n_rows, uint32_t flags, murr_error_t* err);
int murr_hstream_next(murr_hstream_t* s, murr_host_array_t* outs /* nproj */, murr_error_t* err);
/* Totals since creation: batches returned; the bytes each copy direction
 * moved; device milliseconds of the H2D copies, the decode kernels and the
 * D2H copies of the `timed_batches` batches timed with HIP events (every
 * eighth: the events cost host time per batch); host milliseconds spent in
 * submit and in next (API calls and waits), and of those the waits for
 * batches still on the device. */
typedef struct {
    uint64_t batches;
    double h2d_ms, kernel_ms, d2h_ms;
    uint64_t h2d_bytes, d2h_bytes;
    uint64_t timed_batches;
    double host_submit_ms, host_next_ms;
    double host_wait_ms;
} murr_hstream_stats_t;
int murr_hstream_stats(murr_hstream_t* s, murr_hstream_stats_t* out);
void murr_hstream_free(murr_hstream_t* s);

/* Host-memory encode: H2D of the Arrow buffers, murr_encode_batch, D2H of the
 * blobs.  Host input columns use the same murr_col_in_t (host pointers) plus
 * the per-column byte lengths of their buffers.  Output buffers are allocated
 * by the library (pinned) and freed with murr_host_free. */
typedef struct {
    murr_col_in_t col;       /* host pointers */
    uint64_t values_bytes;   /* bytes readable at values (from element 0) */
} murr_host_col_in_t;

int murr_encode_host(murr_ctx_t* ctx, const murr_segment_t* seg,
                     const murr_host_col_in_t* cols, uint64_t n_rows,
                     uint8_t** out_blob, uint64_t* blob_len,
                     uint64_t** out_row_off, murr_error_t* err);

/* ---- device-resident key index ------------------ */

/* The key lookups of Store::read for a table whose row blobs live in HBM:
 * replaces RocksDBStore::read's ParGet/MultiGet and its serial present/missing
 * feed (src/io/store/rocksdb/mod.rs:241-267; MemoryStore::read,
 * src/io/store/memory.rs:28-45), so lookup -> gather -> decode runs on the
 * device with no host round trip.  Keys are the table's utf8 key column
 * (src/io/table/mod.rs:70-96); row i of the index is row i of the blobs
 * murr_encode_batch wrote for the same batch. */
typedef struct murr_index murr_index_t;

#define MURR_ROW_MISSING 0xFFFFFFFFu

/* Build over n keys (device Arrow utf8: key_offsets[n+1], key_data; offset =
 * Arrow array offset in elements).  The index copies the keys.  Equal keys
 * follow put semantics: the later row wins (memory.rs:47-56).  n < 2^32 - 1.
 * Synchronous. */
int murr_index_build(murr_ctx_t* ctx, const uint8_t* key_data, const int32_t* key_offsets,
                     uint64_t key_offset, uint64_t n, murr_index_t** out, murr_error_t* err);
void murr_index_free(murr_index_t* idx);
/* Append n keys as rows idx.n .. idx.n + n - 1 (Table::write into a table that
 * already holds rows, src/io/table/mod.rs:54-112 -> Store::write,
 * src/io/store/memory.rs:47-60): a key written again now maps to its new
 * row (later write wins).  The key copy grows by doubling and the slot table
 * is rehashed only when the load would pass 1/3, so an append costs in
 * proportion to the batch (amortised).  Synchronous. */
int murr_index_append(murr_ctx_t* ctx, murr_index_t* idx, const uint8_t* key_data,
                      const int32_t* key_offsets, uint64_t key_offset, uint64_t n,
                      murr_error_t* err);
/* Resolve equal keys by sequence number instead of row: afterwards each key
 * maps to its row with the highest seqs[row] (equal sequence numbers: the
 * later row).  seqs: device array of idx.n entries.  For indexes over SST
 * entries (ResidentTable.load_sst), where RocksDB stores a key's versions
 * newest first (InternalKeyComparator: user key ascending, sequence number
 * descending) and overlapping files repeat keys in any order; the version
 * with the highest sequence number is the one a read returns.  Synchronous. */
int murr_index_prefer_seq(murr_ctx_t* ctx, murr_index_t* idx, const uint64_t* seqs, murr_error_t* err);
/* One read over a table sharded by key across GPUs (SURVEY.md §8(e) mode 2),
 * without a collective and with no host synchronisation: the caller's nq
 * query keys sit on the home GPU grouped by owner shard (shard s owns grouped
 * positions [shards[s-1].q_end, shards[s].q_end)), src[i] = the grouped
 * position of caller query i.  Each shard looks its keys up on its own
 * context's stream, all shards at once (reading the keys from home memory,
 * writing rows[p] there); the home stream waits on those lookups (events, not
 * the host), then writes the caller-order block: out_row_off (nq + 1) and the
 * rows' blobs copied straight from each shard's arena (peer reads over xGMI)
 * -- row i is the row of key i, a miss an empty row (the positional contract
 * of RocksDBStore::read, src/io/store/rocksdb/mod.rs:368-399).  out_data
 * NULL: sizes and offsets only (*needed = the block's bytes), then
 * murr_multi_gather_copy.  Offsets are clamped to out_cap; *needed (optional
 * with out_data) gets the true total.  A shard with no index (nothing written)
 * misses every key.  At most 16 shards.  Asynchronous on the home stream. */
typedef struct {
    murr_ctx_t* ctx;             /* the shard's context (its GPU and stream) */
    const murr_index_t* index;   /* its key index (NULL: empty shard) */
    const uint8_t* arena;        /* its row blobs */
    const uint64_t* row_off;     /* and their offsets */
    uint64_t q_end;              /* end of its grouped query range */
} murr_shard_read_t;
int murr_multi_gather(murr_ctx_t* home, const murr_shard_read_t* shards, uint32_t nshards,
                      const uint8_t* q_data, const int32_t* q_offsets, const uint32_t* src, uint64_t nq,
                      uint32_t* rows, uint64_t* out_row_off, uint8_t* out_data, uint64_t out_cap,
                      uint64_t* needed, murr_error_t* err);
/* The copy of a murr_multi_gather whose out_data was NULL, into out_data
 * (>= *needed bytes, 16-B aligned).  Asynchronous on the home stream. */
int murr_multi_gather_copy(murr_ctx_t* home, const murr_shard_read_t* shards, uint32_t nshards,
                           const uint32_t* src, uint64_t nq, const uint32_t* rows,
                           const uint64_t* out_row_off, uint8_t* out_data, murr_error_t* err);
/* The slot cache of a resident table's index: beside each slot, the row
 * offset and size of the row it holds (row_off, the table's n + 1 offsets)
 * and, for a layout of 1 to 4 utf8 columns, the row's string bytes (row_ulen,
 * murr_utf8_row_lengths' [n][nutf8]; NULL and 0 otherwise).  With every row
 * cached, a prepared read's probe resolves a key of up to 16 bytes in the
 * round trip that loads its slot (murr_read_plan_*).  Caches the rows added
 * since the last call (every row after a rehash or murr_index_prefer_seq);
 * call it after each append, once the table's offsets (and string bytes) hold
 * the new rows.  Enqueued. */
int murr_index_cache_rows(murr_ctx_t* ctx, murr_index_t* idx, const uint64_t* row_off,
                          const uint32_t* row_ulen, uint32_t nutf8, murr_error_t* err);
/* Rows indexed (n at build) and hash-table slots. */
int murr_index_info(const murr_index_t* idx, uint64_t* n, uint64_t* slots);

/* Enqueue on the ctx stream: rows[i] = row of query key i, or MURR_ROW_MISSING.
 * Query keys are device Arrow utf8 (q_offsets[nq+1] from element 0). */
int murr_index_lookup(murr_ctx_t* ctx, const murr_index_t* idx, const uint8_t* q_data,
                      const int32_t* q_offsets, uint64_t nq, uint32_t* rows);

/* Enqueue: lookup, then gather the hit rows of (blob, row_off) back to back
 * into a decode block in caller order: out_row_off[nq+1] (from 0), out_data
 * (16-B aligned, out_cap bytes); a miss is an empty row, i.e. add_empty
 * (rocksdb/mod.rs:262-263).  rows (optional, device u32[nq]) receives the
 * lookup.  needed (optional, device u64) receives the block bytes; offsets
 * are clamped to out_cap, so when *needed > out_cap the block is cut short
 * (rows past the cap read as missing) -- size out_cap as nq * the longest row
 * to rule that out.  Feed the result to murr_decode_enqueue as one block.
 * Two-phase form (exact sizing): out_data == NULL runs the lookup and the
 * offsets only (rows and needed required, offsets not clamped); read
 * *needed, allocate that many bytes, then murr_index_gather_copy. */
int murr_index_gather(murr_ctx_t* ctx, const murr_index_t* idx, const uint8_t* q_data,
                      const int32_t* q_offsets, uint64_t nq, const uint8_t* blob,
                      const uint64_t* row_off, uint8_t* out_data, uint64_t out_cap,
                      uint64_t* out_row_off, uint32_t* rows, uint64_t* needed);

/* Second phase of a two-phase gather: copy the rows the first phase looked up
 * (rows[nq], out_row_off[nq + 1] from murr_index_gather with out_data NULL)
 * into out_data (16-B aligned, *needed bytes).  Enqueue. */
int murr_index_gather_copy(murr_ctx_t* ctx, const uint32_t* rows, uint64_t nq, const uint8_t* blob,
                           const uint64_t* row_off, const uint64_t* out_row_off, uint8_t* out_data);

/* ---- resident read: host keys in, host Arrow arrays out ------------------- */

/* Table::read (src/io/table/mod.rs:114-129) over a table whose row blobs live
 * in HBM, as one call: replaces RocksDBStore::read's MultiGet + the
 * ReadBatchBuilder feed (src/io/store/rocksdb/mod.rs:241-267) for a resident
 * table.  The reader keeps its pinned and device scratch between reads. */
typedef struct murr_reader murr_reader_t;

int murr_reader_new(murr_ctx_t* ctx, const murr_segment_t* seg, murr_reader_t** out);
/* Keys: host Arrow utf8 (key_offsets[key_offset .. key_offset + nq], key_data).
 * The table: idx over its keys, (blob, row_off) its rows in HBM, blob_bytes
 * their total size, max_row the longest row.  One H2D of the keys, lookup +
 * gather + decode on the ctx stream, one D2H when the arrays fit 1 MiB (else
 * one per buffer, exact sizes).  outs[nproj] point into the reader's pinned
 * memory, valid until its next read or free.  A missing key is an all-null
 * row (add_empty, rocksdb/mod.rs:262-263).  Synchronous. */
int murr_reader_read(murr_reader_t* r, const murr_index_t* idx, const uint8_t* blob,
                     const uint64_t* row_off, uint64_t blob_bytes, uint64_t max_row,
                     const uint8_t* key_data, const int32_t* key_offsets, uint64_t key_offset,
                     uint64_t nq, const uint32_t* proj, uint32_t nproj,
                     murr_host_array_t* outs, murr_error_t* err);
void murr_reader_free(murr_reader_t* r);

/* Prepared resident read: Table::read (src/io/table/mod.rs:114-129 over
 * src/io/store/memory.rs:28-45) repeated with one projection and at most
 * `cap` keys -- the loop of benches/read_block.rs / read_plain.rs.  Made once
 * per (table state, projection, capacity): the gather's device work area, the
 * decode's outputs and its prepared launch (descriptors resident, counters
 * handed to pinned memory by the kernel), pinned key staging and arrays.  A
 * run enqueues lookup + gather + decode (+ the arrays to pinned memory) on the
 * ctx stream and waits once: no descriptor upload, no read-back copy, no copy
 * engine; host keys are read by the probe in place.  A run of nq <= cap keys
 * decodes cap rows (queries past nq are misses) and reports nq.  The table's
 * arena, row offsets and index must not change while the plan lives (a write
 * that appends invalidates it).  Fails with MURR_E_ARGUMENT when cap x
 * max_row passes 64 MiB (murr_reader_read sizes such reads exactly).
 * row_ulen (optional, device): the table's per-row utf8 string bytes
 * (murr_utf8_row_lengths over all its rows).  With it, and a layout of 1 to 4
 * utf8 columns and cap <= 1024, the gather also writes the gathered block's
 * utf8 index, and the decode runs in one pass instead of two. */
typedef struct murr_read_plan murr_read_plan_t;
int murr_read_plan_new(murr_ctx_t* ctx, const murr_segment_t* seg, const murr_index_t* idx,
                       const uint8_t* blob, const uint64_t* row_off, const uint32_t* row_ulen,
                       uint64_t blob_bytes, uint64_t max_row, const uint32_t* proj, uint32_t nproj,
                       uint64_t cap, murr_read_plan_t** out);
/* Keys in device memory (q_offsets[nq + 1], q_data); outs[nproj] are device
 * arrays in the plan's buffers (n = nq), valid until its next run or free.
 * Returns once the decode's counters are in (null counts, lengths, errors):
 * the arrays are ready for work queued on the context's stream
 * (murr_ctx_stream); another stream or device waits on that stream first. */
int murr_read_plan_run_device(murr_read_plan_t* plan, const uint8_t* q_data, const int32_t* q_offsets,
                              uint64_t nq, murr_array_t* outs, murr_error_t* err);
/* Keys on the host (Arrow utf8 from key_offset); outs[nproj] point into the
 * plan's pinned memory, valid until its next run or free.  Synchronous. */
int murr_read_plan_run(murr_read_plan_t* plan, const uint8_t* key_data, const int32_t* key_offsets,
                       uint64_t key_offset, uint64_t nq, murr_host_array_t* outs, murr_error_t* err);
uint64_t murr_read_plan_capacity(const murr_read_plan_t* plan);
void murr_read_plan_free(murr_read_plan_t* plan);

/* ---- RocksDB data blocks --------------------------- */

/* The data blocks of the block-based SSTs the reference's store writes
 * (src/io/store/rocksdb/block.rs:97-121: block_size 512, restart interval 8,
 * BinaryAndHash data-block index, default compression) decoded on the device
 * into their entries: the bulk read a warm-up or rehydration does before the
 * row blobs go to murr_decode_* and the keys to murr_index_build.  A block is
 * its contents as stored (the BlockHandle's bytes, without the 5-byte
 * trailer) with the trailer's compression type: 0 none, 1 Snappy (raw
 * format), 4 / 5 LZ4 / LZ4HC (varint32 length + LZ4 block); other types are
 * MURR_E_MALFORMED_ROW.  Entries come out in block order: user keys (the internal key less
 * its 8-byte trailer) as Arrow utf8, values as a decode block (values 16-B
 * aligned, value_offsets[n + 1] from 0), and each trailer's sequence number
 * and value type.  Blocks that do not parse are MURR_E_MALFORMED_ROW with the
 * first such block in err->row.  Outputs are allocated by the library (device
 * memory, through the context's reuse cache) and freed with
 * murr_sst_result_free, or one by one with murr_dev_free (to keep, e.g.,
 * values and value_offsets as a table's arena); freed ones serve the
 * context's next call without a hipMalloc.  `blocks` is a host array, or a device array (device memory from
 * murr_dev_alloc / hipMalloc: the descriptor table of a file decoded more
 * than once, uploaded once -- a 100 k-block host table costs ~0.1 ms of
 * pageable copy per call); a device table is not read by the host, so a
 * block with size > 0 and no data is MURR_E_MALFORMED_ROW there rather than
 * MURR_E_ARGUMENT.  Synchronous. */
typedef struct {
    const uint8_t* data;   /* device */
    uint64_t size;
    uint32_t compression;  /* RocksDB CompressionType: 0 none, 1 Snappy, 4 LZ4, 5 LZ4HC */
    uint32_t _pad;
} murr_sst_block_t;

typedef struct {
    uint64_t n;                /* entries */
    uint8_t* keys;             /* user key bytes */
    int32_t* key_offsets;      /* n + 1 */
    uint8_t* values;           /* value bytes (row blobs) */
    uint64_t* value_offsets;   /* n + 1 */
    uint64_t* seqs;            /* n */
    uint8_t* types;            /* n (1 = value, 0 = deletion, ...) */
    uint64_t key_bytes, value_bytes;
} murr_sst_result_t;

int murr_sst_decode(murr_ctx_t* ctx, const murr_sst_block_t* blocks, uint32_t nblocks,
                    murr_sst_result_t* out, murr_error_t* err);
void murr_sst_result_free(murr_ctx_t* ctx, murr_sst_result_t* r);

/* ---- sharding -------------------------------------------- */

/* Owner shard of each of n keys (host Arrow utf8: key_offsets[key_offset ..
 * key_offset + n], key_data): fmix64(FNV-1a 64 of the key bytes) mod nshards.
 * Writes and reads route every key to its owner, so a key lives in exactly one
 * shard and a later write of it lands where the earlier one did (later write
 * wins, src/io/store/memory.rs:47-60).  Host function, no device. */
int murr_shard_of(const uint8_t* key_data, const int32_t* key_offsets, uint64_t key_offset, uint64_t n,
                  uint32_t nshards, uint32_t* out);

/* ---- Arrow IPC framing --------------------------- */

/* The read path's last step: the HTTP fetch handler serialises the batch with
 * arrow-rs StreamWriter (schema message, record-batch message, end-of-stream;
 * src/api/http/handlers.rs:93-101) and Flight DoGet with FlightDataEncoderBuilder
 * (src/api/flight/mod.rs:85-87).  These write the same encapsulated messages
 * (0xFFFFFFFF, int32 metadata size, flatbuffer Message V5 padded to
 * `alignment`, body buffers each at a multiple of `alignment`, zero padding;
 * arrow-rs IpcWriteOptions::default() uses alignment 64, Arrow C++ 8).
 * Fields are nullable with no metadata (src/io/row/read.rs:105).  A column
 * without nulls gets a zero-length validity buffer.  Every call with out ==
 * NULL only reports *out_len; cap < *out_len returns MURR_E_CAPACITY.
 * `alignment` is a power of two in [8, 4096]. */

/* Schema message for the projected columns; names[p] is column p's name. */
int murr_ipc_schema(const murr_segment_t* seg, const uint32_t* proj, uint32_t nproj,
                    const char* const* names, uint32_t alignment, uint8_t* out,
                    uint64_t cap, uint64_t* out_len);

/* Record-batch message from the host arrays of murr_builder_build (host memory). */
int murr_ipc_batch_host(const murr_segment_t* seg, const uint32_t* proj, uint32_t nproj,
                        const murr_host_array_t* arrays, uint64_t n_rows, uint32_t alignment,
                        uint8_t* out, uint64_t cap, uint64_t* out_len);

/* Record-batch message from one block's decode outputs (device arrays whose
 * null_count / data_len murr_decode_blocks filled), packed into dev_out by one
 * kernel on the ctx stream so a single D2H copy yields the wire bytes.
 * Synchronous. */
int murr_ipc_batch_device(murr_ctx_t* ctx, const murr_segment_t* seg, const uint32_t* proj,
                          uint32_t nproj, const murr_array_t* arrays, uint64_t n_rows,
                          uint32_t alignment, uint8_t* dev_out, uint64_t cap,
                          uint64_t* out_len, murr_error_t* err);

/* End-of-stream marker (0xFFFFFFFF, 0) into out[8]; returns 8. */
uint64_t murr_ipc_eos(uint8_t* out);

/* Human-readable name of a status code. */
const char* murr_status_str(int status);

/* MURR_ABI_VERSION of the library (see the define above). */
uint32_t murr_abi_version(void);

/* ---- Arrow C Data Interface export ------------------------------------------- */

/* The Arrow C Data Interface (arrow/c/abi.h), as arrow-rs' `ffi` module and
 * pyarrow define it. */
#ifndef ARROW_C_DATA_INTERFACE
#define ARROW_C_DATA_INTERFACE
#define ARROW_FLAG_DICTIONARY_ORDERED 1
#define ARROW_FLAG_NULLABLE 2
#define ARROW_FLAG_MAP_KEYS_SORTED 4
struct ArrowSchema {
    const char* format;
    const char* name;
    const char* metadata;
    int64_t flags;
    int64_t n_children;
    struct ArrowSchema** children;
    struct ArrowSchema* dictionary;
    void (*release)(struct ArrowSchema*);
    void* private_data;
};
struct ArrowArray {
    int64_t length;
    int64_t null_count;
    int64_t offset;
    int64_t n_buffers;
    int64_t n_children;
    const void** buffers;
    struct ArrowArray** children;
    struct ArrowArray* dictionary;
    void (*release)(struct ArrowArray*);
    void* private_data;
};
#endif

/* A read's host arrays (all of one length: a build()'s, a reader's, a prepared
 * read's) as the RecordBatch ReadBatchBuilder::build returns
 * (src/io/row/read.rs:100-110): a struct array of nullable fields named
 * names[i] (Arrow C format per dtype: "u" utf8, "b" bool, "c"/"s"/"i"/"l"
 * int8-64, "C"/"S"/"I"/"L" uint8-64, "f"/"g" float32/64), for
 * arrow::ffi::from_ffi / pyarrow RecordBatch._import_from_c in one call.
 * The export owns a compacted copy of the bytes (the arrays' pinned memory is
 * reused by the next read); its release callbacks free it.  Validity is
 * exported only when null_count > 0.  out_schema may be NULL: a caller that
 * reads the same columns again keeps the schema of its first export (the
 * schema depends only on names and dtypes) and imports the array against it.
 * Host only. */
int murr_arrow_export(const murr_host_array_t* arrays, uint32_t n, const char* const* names,
                      struct ArrowArray* out_array, struct ArrowSchema* out_schema);

#ifdef __cplusplus
}
#endif
#endif /* MURR_CODEC_H */
