/*
 * murr_sst.h — CPU restatement of the RocksDB data-block read path (Snappy raw
 * decompression, data-block entry decode).  TEST INFRASTRUCTURE: see
 * murr_sst.c for the formats and what pins them.
 */
#ifndef MURR_SST_H
#define MURR_SST_H

#include <stdint.h>

#include "murr_oracle.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { OC_SST_E_CORRUPT = 12 };

int oc_snappy_uncompressed_len(const uint8_t* src, uint64_t n, uint64_t* len);
int oc_snappy_decompress(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* out_len);
/* varint32 length + LZ4 block (RocksDB kLZ4Compression / kLZ4HCCompression);
 * the length prefix reads with oc_snappy_uncompressed_len. */
int oc_lz4_decompress(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* out_len);
/* Entries, user-key bytes and value bytes of one uncompressed data block. */
int oc_block_count(const uint8_t* b, uint64_t n, uint64_t* nentries, uint64_t* key_bytes, uint64_t* value_bytes);
/* The entries in block order: user keys (key_off[0..ne], from 0), values
 * (val_off[0..ne]), sequence numbers and value types from the 8-byte trailer. */
int oc_block_decode(const uint8_t* b, uint64_t n, uint8_t* keys, int32_t* key_off, uint8_t* vals,
                    uint64_t* val_off, uint64_t* seqs, uint8_t* types);

/* Every block of a buffer (blocks up to 64 KiB uncompressed), one thread:
 * the bench's CPU baseline.  Totals of entries, key and value bytes. */
int oc_sst_decode_all(const uint8_t* data, const uint64_t* off, const uint64_t* size, const uint32_t* comp,
                      uint64_t nb, uint64_t* entries, uint64_t* key_bytes, uint64_t* value_bytes);

#ifdef __cplusplus
}
#endif

#endif
