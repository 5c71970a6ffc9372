/*
 * murr_sst.c — CPU restatement of the RocksDB data-block read path murr's
 * store sits on (TEST INFRASTRUCTURE, like murr_oracle.c: only tests/ load it).
 *
 * SURVEY.md §8(f) rank 4.  The reference stores row blobs in RocksDB
 * (src/io/store/rocksdb/mod.rs) with BlockBasedOptions from
 * src/io/store/rocksdb/block.rs:97-121: block_size 512 (:83-85), restart
 * interval 8 (:86-88), DataBlockIndexType::BinaryAndHash (:108-111), and the
 * default compression.  RocksDB itself (librocksdb-sys 0.17.3+10.4.2,
 * Cargo.lock) and Snappy are third-party C++ not in the tree; this file
 * restates their published formats:
 *
 *  - Snappy raw format (format_description.txt of google/snappy): a varint32
 *    uncompressed length, then elements: literal (tag & 3 == 0; length - 1 in
 *    tag >> 2, or in the next 1..4 little-endian bytes for 60..63), copy with
 *    a 1-byte offset (length 4 + ((tag >> 2) & 7), offset ((tag >> 5) << 8) |
 *    next byte), copy with a 2- or 4-byte little-endian offset (length
 *    1 + (tag >> 2)).  Copies may overlap their output (offset < length).
 *    Pinned against pyarrow's Snappy codec (tests/test_sst.py).
 *
 *  - LZ4 block format (lz4_Block_format.md of lz4/lz4) as RocksDB stores it
 *    with compress_format_version 2 (every format_version >= 2): a varint32
 *    uncompressed length, then one LZ4 block of sequences: a token (literal
 *    length in the high nibble, match length - 4 in the low; 15 = more in
 *    extension bytes, each added, until one below 255), the literals, and,
 *    except in the last sequence (literals only, ends the block), a 2-byte
 *    little-endian offset and the match-length extension.  Pinned against
 *    pyarrow's lz4_raw codec (tests/test_sst.py).
 *
 *  - RocksDB data block (table/block_based/block_builder.cc, block.cc,
 *    data_block_footer.cc, data_block_hash_index.cc): entries
 *    [varint32 shared][varint32 non_shared][varint32 value_len][key delta]
 *    [value]; a restart point every `restart interval` entries stores its key
 *    whole (shared = 0); then the restart offsets (u32 each), for a
 *    BinaryAndHash block the hash buckets (u8 each) and their count (u16),
 *    and a u32 footer: num_restarts | index_type << 31.  Keys are internal
 *    keys: user key + 8-byte little-endian trailer (sequence << 8 | type).
 *    No RocksDB build exists here, so the block format is parity unpinned
 *    beyond this restatement.
 */
#include "murr_sst.h"

#include <stdlib.h>
#include <string.h>

static int get_varint32(const uint8_t** p, const uint8_t* end, uint32_t* v) {
    uint32_t r = 0;
    for (int shift = 0; shift <= 28; shift += 7) {
        if (*p >= end) return 0;
        const uint32_t b = *(*p)++;
        r |= (b & 0x7Fu) << shift;
        if (!(b & 0x80)) {
            *v = r;
            return 1;
        }
    }
    return 0;
}

int oc_snappy_uncompressed_len(const uint8_t* src, uint64_t n, uint64_t* len) {
    const uint8_t* p = src;
    uint32_t v;
    if (!get_varint32(&p, src + n, &v)) return OC_SST_E_CORRUPT;
    *len = v;
    return OC_OK;
}

int oc_snappy_decompress(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* out_len) {
    const uint8_t* p = src;
    const uint8_t* end = src + n;
    uint32_t ulen;
    if (!get_varint32(&p, end, &ulen)) return OC_SST_E_CORRUPT;
    if (ulen > cap) return OC_SST_E_CORRUPT;
    uint64_t o = 0;
    while (p < end) {
        const uint32_t tag = *p++;
        uint32_t len, off;
        switch (tag & 3) {
        case 0:  // literal
            len = tag >> 2;
            if (len >= 60) {
                const uint32_t nb = len - 59;
                if ((uint64_t)(end - p) < nb) return OC_SST_E_CORRUPT;
                len = 0;
                for (uint32_t i = 0; i < nb; i++) len |= (uint32_t)p[i] << (8 * i);
                p += nb;
            }
            len += 1;
            if ((uint64_t)(end - p) < len || o + len > ulen) return OC_SST_E_CORRUPT;
            memcpy(dst + o, p, len);
            p += len;
            o += len;
            continue;
        case 1:
            if (p >= end) return OC_SST_E_CORRUPT;
            len = 4 + ((tag >> 2) & 7);
            off = ((tag >> 5) << 8) | *p++;
            break;
        case 2:
            if (end - p < 2) return OC_SST_E_CORRUPT;
            len = 1 + (tag >> 2);
            off = (uint32_t)p[0] | ((uint32_t)p[1] << 8);
            p += 2;
            break;
        default:
            if (end - p < 4) return OC_SST_E_CORRUPT;
            len = 1 + (tag >> 2);
            off = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
            p += 4;
            break;
        }
        if (off == 0 || off > o || o + len > ulen) return OC_SST_E_CORRUPT;
        for (uint32_t i = 0; i < len; i++, o++) dst[o] = dst[o - off];  // byte order: overlap repeats
    }
    if (o != ulen) return OC_SST_E_CORRUPT;
    *out_len = o;
    return OC_OK;
}

int oc_lz4_decompress(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* out_len) {
    const uint8_t* p = src;
    const uint8_t* end = src + n;
    uint32_t ulen;
    if (!get_varint32(&p, end, &ulen)) return OC_SST_E_CORRUPT;
    if (ulen > cap) return OC_SST_E_CORRUPT;
    uint64_t o = 0;
    for (;;) {
        if (p >= end) return OC_SST_E_CORRUPT;  // the last sequence (literals only) ends the block
        const uint32_t tok = *p++;
        uint64_t lit = tok >> 4;
        if (lit == 15) {
            uint32_t b;
            do {
                if (p >= end) return OC_SST_E_CORRUPT;
                b = *p++;
                lit += b;
            } while (b == 255);
        }
        if ((uint64_t)(end - p) < lit || o + lit > ulen) return OC_SST_E_CORRUPT;
        memcpy(dst + o, p, lit);
        p += lit;
        o += lit;
        if (p == end) break;
        if (end - p < 2) return OC_SST_E_CORRUPT;
        const uint32_t off = (uint32_t)p[0] | ((uint32_t)p[1] << 8);
        p += 2;
        uint64_t ml = tok & 15;
        if (ml == 15) {
            uint32_t b;
            do {
                if (p >= end) return OC_SST_E_CORRUPT;
                b = *p++;
                ml += b;
            } while (b == 255);
        }
        ml += 4;
        if (off == 0 || off > o || o + ml > ulen) return OC_SST_E_CORRUPT;
        for (uint64_t i = 0; i < ml; i++, o++) dst[o] = dst[o - off];
    }
    if (o != ulen) return OC_SST_E_CORRUPT;
    *out_len = o;
    return OC_OK;
}

/* The block's entry region [0, limit) and restart count from its footer. */
static int block_layout(const uint8_t* b, uint64_t n, uint64_t* limit, uint32_t* nrestarts) {
    if (n < 4) return OC_SST_E_CORRUPT;
    uint32_t footer;
    memcpy(&footer, b + n - 4, 4);
    const uint32_t nr = footer & 0x7FFFFFFFu;
    uint64_t tail = 4;
    if (footer >> 31) {  // BinaryAndHash: [buckets u8 x nb][nb u16] before the footer
        if (n < 6) return OC_SST_E_CORRUPT;
        uint16_t nb;
        memcpy(&nb, b + n - 6, 2);
        tail += 2 + (uint64_t)nb;
    }
    tail += 4ull * nr;
    if (nr == 0 || tail > n) return OC_SST_E_CORRUPT;
    *limit = n - tail;
    *nrestarts = nr;
    return OC_OK;
}

/* Walk the entries (block.cc DecodeEntry); `emit` non-zero writes them out. */
static int block_walk(const uint8_t* b, uint64_t n, uint64_t* ne, uint64_t* kb, uint64_t* vb, uint8_t* keys,
                      int32_t* key_off, uint8_t* vals, uint64_t* val_off, uint64_t* seqs, uint8_t* types,
                      uint8_t* scratch, uint64_t scratch_cap) {
    uint64_t limit;
    uint32_t nr;
    int st = block_layout(b, n, &limit, &nr);
    if (st) return st;
    const uint8_t* p = b;
    const uint8_t* end = b + limit;
    uint64_t cnt = 0, kbytes = 0, vbytes = 0, klen = 0;  // klen: the previous internal key's length
    while (p < end) {
        uint32_t shared, nonshared, vlen;
        if (!get_varint32(&p, end, &shared) || !get_varint32(&p, end, &nonshared) ||
            !get_varint32(&p, end, &vlen))
            return OC_SST_E_CORRUPT;
        if (shared > klen || (uint64_t)(end - p) < (uint64_t)nonshared + vlen) return OC_SST_E_CORRUPT;
        const uint64_t ilen = (uint64_t)shared + nonshared;
        if (ilen < 8 || ilen > scratch_cap) return OC_SST_E_CORRUPT;
        memcpy(scratch + shared, p, nonshared);  // the internal key, rebuilt in place
        p += nonshared;
        if (keys) {
            memcpy(keys + kbytes, scratch, ilen - 8);
            key_off[cnt + 1] = (int32_t)(kbytes + ilen - 8);
            uint64_t trailer = 0;
            for (int i = 0; i < 8; i++) trailer |= (uint64_t)scratch[ilen - 8 + i] << (8 * i);
            seqs[cnt] = trailer >> 8;
            types[cnt] = (uint8_t)(trailer & 0xFF);
            memcpy(vals + vbytes, p, vlen);
            val_off[cnt + 1] = vbytes + vlen;
        }
        p += vlen;
        klen = ilen;
        kbytes += ilen - 8;
        vbytes += vlen;
        cnt++;
    }
    *ne = cnt;
    *kb = kbytes;
    *vb = vbytes;
    return OC_OK;
}

int oc_block_count(const uint8_t* b, uint64_t n, uint64_t* nentries, uint64_t* key_bytes, uint64_t* value_bytes) {
    static uint8_t scratch[1 << 20];
    return block_walk(b, n, nentries, key_bytes, value_bytes, NULL, NULL, NULL, NULL, NULL, NULL, scratch,
                      sizeof scratch);
}

int oc_block_decode(const uint8_t* b, uint64_t n, uint8_t* keys, int32_t* key_off, uint8_t* vals,
                    uint64_t* val_off, uint64_t* seqs, uint8_t* types) {
    static uint8_t scratch[1 << 20];
    uint64_t ne, kb, vb;
    key_off[0] = 0;
    val_off[0] = 0;
    return block_walk(b, n, &ne, &kb, &vb, keys, key_off, vals, val_off, seqs, types, scratch, sizeof scratch);
}

/* Bulk form for the bench's CPU baseline: every block of a buffer inflated and
 * decoded (entries written to scratch and discarded), one thread; totals out. */
int oc_sst_decode_all(const uint8_t* data, const uint64_t* off, const uint64_t* size, const uint32_t* comp,
                      uint64_t nb, uint64_t* entries, uint64_t* key_bytes, uint64_t* value_bytes) {
    uint64_t cap = 1 << 16;
    uint8_t* raw = malloc(cap);
    uint8_t *keys = malloc(cap), *vals = malloc(cap);
    int32_t* koff = malloc(sizeof(int32_t) * (cap + 1));
    uint64_t *voff = malloc(8 * (cap + 1)), *seqs = malloc(8 * cap);
    uint8_t* types = malloc(cap);
    int st = OC_OK;
    *entries = *key_bytes = *value_bytes = 0;
    for (uint64_t b = 0; b < nb && st == OC_OK; b++) {
        const uint8_t* src = data + off[b];
        uint64_t n = size[b];
        if (comp[b] != 0) {
            uint64_t ulen = 0, got = 0;
            if ((st = oc_snappy_uncompressed_len(src, n, &ulen))) break;
            if (ulen > cap) { st = OC_SST_E_CORRUPT; break; }
            st = comp[b] == 1 ? oc_snappy_decompress(src, n, raw, cap, &got) : oc_lz4_decompress(src, n, raw, cap, &got);
            if (st) break;
            src = raw;
            n = got;
        }
        if (n > cap) { st = OC_SST_E_CORRUPT; break; }
        uint64_t ne, kb, vb;
        if ((st = oc_block_count(src, n, &ne, &kb, &vb))) break;
        if ((st = oc_block_decode(src, n, keys, koff, vals, voff, seqs, types))) break;
        *entries += ne;
        *key_bytes += kb;
        *value_bytes += vb;
    }
    free(raw); free(keys); free(vals); free(koff); free(voff); free(seqs); free(types);
    return st;
}
