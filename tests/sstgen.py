"""RocksDB data blocks for the SST tests (TEST INFRASTRUCTURE).

A restatement of RocksDB's BlockBuilder (table/block_based/block_builder.cc)
and DataBlockFooter / DataBlockHashIndexBuilder (data_block_footer.cc,
data_block_hash_index.cc) as the reference's store configures them
(src/io/store/rocksdb/block.rs:97-121: restart interval 8, BinaryAndHash,
block_size 512): entries [varint32 shared][varint32 non_shared]
[varint32 value_len][key delta][value], a restart point (shared = 0) every
`restart_interval` entries, the restart offsets (u32), for BinaryAndHash the
hash buckets and their count (u16), then the footer num_restarts |
index_type << 31.  Keys are internal keys: user key + (seq << 8 | type) as
8 LE bytes.  The bucket contents are what a point lookup would use; the bulk
decode never reads them, so they are left as kNoEntry (255).  Snappy
compression comes from pyarrow's codec (the raw format RocksDB stores), LZ4
from pyarrow's lz4_raw behind RocksDB's varint32 length prefix.
"""
from __future__ import annotations

import numpy as np

TYPE_DELETION, TYPE_VALUE = 0, 1


def varint32(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def internal_key(user_key: bytes, seq: int, typ: int = TYPE_VALUE) -> bytes:
    return user_key + ((seq << 8) | typ).to_bytes(8, "little")


def build_block(entries, restart_interval: int = 8, hash_index: bool = True, hash_ratio: float = 0.75) -> bytes:
    """entries: [(user_key, seq, type, value)], in internal-key order."""
    buf = bytearray()
    restarts = []
    last = b""
    counter = restart_interval  # the first entry starts a restart point
    for uk, seq, typ, val in entries:
        ik = internal_key(uk, seq, typ)
        if counter >= restart_interval:
            restarts.append(len(buf))
            counter = 0
            shared = 0
        else:
            m = min(len(last), len(ik))
            shared = next((i for i in range(m) if last[i] != ik[i]), m)
        buf += varint32(shared) + varint32(len(ik) - shared) + varint32(len(val)) + ik[shared:] + val
        last = ik
        counter += 1
    if not restarts:
        restarts = [0]
    for r in restarts:
        buf += r.to_bytes(4, "little")
    footer = len(restarts)
    if hash_index:
        nb = max(1, int(len(entries) / hash_ratio)) | 1
        buf += bytes([255]) * nb + nb.to_bytes(2, "little")
        footer |= 1 << 31
    buf += footer.to_bytes(4, "little")
    return bytes(buf)


NONE, SNAPPY, LZ4 = 0, 1, 4  # RocksDB CompressionType values


def snappy(block: bytes) -> bytes:
    import pyarrow as pa
    return pa.Codec("snappy").compress(block, asbytes=True)


def lz4(block: bytes) -> bytes:
    """RocksDB's LZ4 block (compress_format_version 2): varint32 length + raw LZ4."""
    import pyarrow as pa
    return varint32(len(block)) + pa.Codec("lz4_raw").compress(block, asbytes=True)


def compress(block: bytes, compression: int) -> bytes:
    return {NONE: lambda b: b, SNAPPY: snappy, LZ4: lz4}[compression](block)


def blocks_of(entries, block_size: int = 512, **kw):
    """Cut a sorted entry list into blocks the way the flush policy does: a
    block is closed once its entries reach block_size bytes."""
    out, cur, size = [], [], 0
    for e in entries:
        cur.append(e)
        size += len(e[0]) + 8 + len(e[3]) + 3
        if size >= block_size:
            out.append(build_block(cur, **kw))
            cur, size = [], 0
    if cur:
        out.append(build_block(cur, **kw))
    return out


def random_entries(rng, n: int, max_key: int = 24, max_val: int = 120, dup_p: float = 0.0, del_p: float = 0.0):
    """n entries in internal-key order: user keys ascending with shared
    prefixes, optionally several versions of a key (seq descending)."""
    keys = set()
    while len(keys) < n:
        k = int(rng.integers(0, 10 ** 9))
        keys.add(("k%09d" % k)[: int(rng.integers(1, max_key + 1))].encode() + rng.integers(0x20, 0x7F, size=int(
            rng.integers(0, 6)), dtype=np.uint8).tobytes())
    out = []
    seq = 10 ** 6
    for uk in sorted(keys):
        versions = 1 + (int(rng.integers(1, 4)) if rng.random() < dup_p else 0)
        for v in range(versions):
            typ = TYPE_DELETION if rng.random() < del_p else TYPE_VALUE
            val = b"" if typ == TYPE_DELETION else rng.integers(0, 256, size=int(rng.integers(0, max_val + 1)),
                                                                dtype=np.uint8).tobytes()
            out.append((uk, seq - v, typ, val))
        seq -= 7
    return out
