"""RocksDB data blocks -> entries on the device (murr_sst_decode; SURVEY.md
§8(f) rank 4).

The reference keeps its row blobs in RocksDB block-based SSTs
(src/io/store/rocksdb/block.rs:97-121: block_size 512, restart interval 8,
BinaryAndHash, default compression).  A warm-up or rehydration that bulk-reads
those files hands their data blocks here: the stored block bytes (one upload of
the file, or of the blocks back to back) plus each block's (offset, size,
compression) from its BlockHandle and trailer.  The entries come back in HBM:
user keys as an Arrow utf8 column (what murr_index_build takes), values as a
decode block (what murr_decode_blocks takes), and each trailer's sequence
number and value type.  `ResidentTable.load_sst` turns them into a resident
table without a host round trip of the rows.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _abi
from .device import Context, DeviceBlock, DeviceBuffer
from .errors import raise_status

# RocksDB CompressionType values the device inflates.
NONE, SNAPPY, LZ4, LZ4HC = 0, 1, 4, 5
TYPE_DELETION, TYPE_VALUE = 0, 1
_SST_BLOCK = np.dtype([("data", np.uint64), ("size", np.uint64), ("compression", np.uint32), ("_pad", np.uint32)])
assert _SST_BLOCK.itemsize == C.sizeof(_abi.SstBlock)


@dataclass
class SstEntries:
    """murr_sst_result_t as device buffers (owned; freed with the object)."""
    n: int
    keys: DeviceBuffer
    key_offsets: DeviceBuffer
    values: DeviceBuffer
    value_offsets: DeviceBuffer
    seqs: DeviceBuffer
    types: DeviceBuffer
    key_bytes: int
    value_bytes: int

    def block(self) -> DeviceBlock:
        """The values as a decode block (row blobs back to back)."""
        return DeviceBlock(self.values, self.value_offsets, self.n, max(self.value_bytes, 16))

    def to_host(self):
        """(user keys, values, seqs, types) on the host, in block order."""
        ko = self.key_offsets.download(4 * (self.n + 1)).view(np.int32)
        vo = self.value_offsets.download(8 * (self.n + 1)).view(np.uint64)
        kd = self.keys.download(self.key_bytes).tobytes()
        vd = self.values.download(self.value_bytes).tobytes()
        keys = [kd[ko[i]:ko[i + 1]] for i in range(self.n)]
        vals = [vd[vo[i]:vo[i + 1]] for i in range(self.n)]
        seqs = self.seqs.download(8 * self.n).view(np.uint64)
        types = self.types.download(self.n)
        return keys, vals, seqs, types


def upload_blocks(ctx: Context, blocks):
    """Stored blocks [(bytes, compression)] back to back in one device buffer
    (the layout of the file's data region): (buffer, [(offset, size,
    compression)] as an int64 array)."""
    sizes = np.array([len(d) for d, _ in blocks], np.int64)
    h = np.zeros((len(blocks), 3), np.int64)
    h[:, 0] = np.cumsum(sizes) - sizes
    h[:, 1] = sizes
    h[:, 2] = [int(c) for _, c in blocks]
    host = np.frombuffer(b"".join(bytes(d) for d, _ in blocks) + bytes(16), np.uint8)
    return ctx.upload(host), h


def block_table(buf: DeviceBuffer, handles) -> np.ndarray:
    """murr_sst_block_t[] for blocks at buf + offset (handles: [(offset, size,
    compression)]), bounds-checked against the buffer."""
    h = np.asarray(handles, dtype=np.int64).reshape(-1, 3)
    nb = h.shape[0]
    bad = (h[:, 0] < 0) | (h[:, 1] < 0) | (h[:, 0] + h[:, 1] > buf.nbytes)
    if bad.any():
        i = int(np.flatnonzero(bad)[0])
        raise ValueError(f"block {i} {tuple(int(x) for x in h[i, :2])} lies outside the {buf.nbytes}-byte buffer")
    desc = np.zeros(max(nb, 1), dtype=_SST_BLOCK)
    desc["data"][:nb] = np.uint64(buf.ptr) + h[:, 0].astype(np.uint64)
    desc["size"][:nb] = h[:, 1]
    desc["compression"][:nb] = h[:, 2]
    return desc[:nb]


@dataclass
class SstTable:
    """A block table in device memory (device_table): murr_sst_decode reads
    it in place, so a file decoded more than once uploads its descriptors
    once."""
    table: DeviceBuffer
    n: int


def device_table(ctx: Context, buf: DeviceBuffer, handles) -> SstTable:
    """block_table() uploaded once to the device."""
    desc = block_table(buf, handles)
    return SstTable(ctx.upload(desc.view(np.uint8) if len(desc) else np.zeros(16, np.uint8)), len(desc))


def decode(ctx: Context, buf: DeviceBuffer, handles) -> SstEntries:
    """murr_sst_decode over blocks at buf + offset (handles: [(offset, size,
    compression)], or the block_table() made from them once for a file that is
    decoded again, or its device_table()).  A block that does not parse
    raises SegmentError (MURR_E_MALFORMED_ROW) naming the first such block."""
    if isinstance(handles, SstTable):
        ptr, n = C.cast(C.c_void_p(handles.table.ptr), C.POINTER(_abi.SstBlock)), handles.n
    else:
        desc = handles if isinstance(handles, np.ndarray) and handles.dtype == _SST_BLOCK else block_table(buf, handles)
        ptr, n = desc.ctypes.data_as(C.POINTER(_abi.SstBlock)), len(desc)
    res = _abi.SstResult()
    err = _abi.Error()
    st = ctx.L.murr_sst_decode(ctx.h, ptr, n, C.byref(res), C.byref(err))
    raise_status(st, err, "murr_sst_decode")
    n = res.n
    # each output is its own allocation: ownership moves to DeviceBuffers (murr_dev_free)
    return SstEntries(n, DeviceBuffer(ctx, res.keys, res.key_bytes + 16),
                      DeviceBuffer(ctx, res.key_offsets, 4 * (n + 1)),
                      DeviceBuffer(ctx, res.values, res.value_bytes + 16),
                      DeviceBuffer(ctx, res.value_offsets, 8 * (n + 1)),
                      DeviceBuffer(ctx, res.seqs, 8 * max(n, 1)), DeviceBuffer(ctx, res.types, max(n, 1)),
                      res.key_bytes, res.value_bytes)


def decode_host(ctx: Context, blocks) -> SstEntries:
    """decode() of host blocks [(bytes, compression)] (one upload)."""
    buf, handles = upload_blocks(ctx, blocks)
    return decode(ctx, buf, handles)
