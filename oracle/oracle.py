"""ctypes binding of the C restatement (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / CPU baseline.  The product path
(murr_amd, libmurr_codec.so) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmurr_oracle.so")

DTYPE_CODES = {"utf8": 0, "bool": 1, "int8": 2, "int16": 3, "int32": 4, "int64": 5,
               "uint8": 6, "uint16": 7, "uint32": 8, "uint64": 9, "float32": 10, "float64": 11}
SIZES = {0: 4, 1: 1, 2: 1, 3: 2, 4: 4, 5: 8, 6: 1, 7: 2, 8: 4, 9: 8, 10: 4, 11: 8}


class OcColumn(C.Structure):
    _fields_ = [("index", C.c_uint32), ("dtype", C.c_uint32), ("offset", C.c_uint32),
                ("size", C.c_uint32)]


class OcSegment(C.Structure):
    _fields_ = [("ncols", C.c_uint32), ("bitset_size", C.c_uint32), ("capacity", C.c_uint32),
                ("_pad", C.c_uint32), ("cols", C.POINTER(OcColumn))]


class OcArray(C.Structure):
    _fields_ = [("values", C.POINTER(C.c_uint8)), ("validity", C.POINTER(C.c_uint8)),
                ("offsets", C.POINTER(C.c_int32)), ("length", C.c_uint64),
                ("null_count", C.c_uint64), ("values_len", C.c_uint64), ("dtype", C.c_uint32),
                ("_pad", C.c_uint32)]


class OcColIn(C.Structure):
    _fields_ = [("values", C.c_void_p), ("validity", C.c_void_p), ("offsets", C.c_void_p),
                ("offset", C.c_uint64)]


class OcError(C.Structure):
    _fields_ = [("status", C.c_int32), ("_pad", C.c_int32), ("row", C.c_uint64),
                ("column", C.c_uint32), ("_pad2", C.c_uint32), ("message", C.c_char * 128)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.oc_segment_init.argtypes = [C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(OcColumn),
                                      C.POINTER(OcSegment)]
        L.oc_decode_block.argtypes = [C.POINTER(OcSegment), C.POINTER(C.c_uint32), C.c_uint32,
                                      C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(OcArray),
                                      C.POINTER(OcError)]
        L.oc_encode_batch.argtypes = [C.POINTER(OcSegment), C.POINTER(OcColIn), C.c_uint64,
                                      C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_uint64),
                                      C.c_void_p, C.POINTER(OcError)]
        L.oc_array_free.argtypes = [C.POINTER(OcArray)]
        L.oc_free.argtypes = [C.c_void_p]
        L.oc_utf8_valid.argtypes = [C.c_char_p, C.c_uint64, C.POINTER(C.c_uint64),
                                    C.POINTER(C.c_int)]
        L.oc_snappy_uncompressed_len.argtypes = [C.c_char_p, C.c_uint64, C.POINTER(C.c_uint64)]
        L.oc_snappy_decompress.argtypes = [C.c_char_p, C.c_uint64, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
        L.oc_lz4_decompress.argtypes = [C.c_char_p, C.c_uint64, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
        L.oc_sst_decode_all.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                         C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.oc_block_count.argtypes = [C.c_char_p, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                     C.POINTER(C.c_uint64)]
        L.oc_block_decode.argtypes = [C.c_char_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_void_p]
        L.oc_memstore_new.restype = C.c_void_p
        L.oc_memstore_new.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
        L.oc_memstore_read.argtypes = [C.c_void_p, C.POINTER(OcSegment), C.POINTER(C.c_uint32), C.c_uint32,
                                       C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(OcArray), C.POINTER(OcError)]
        L.oc_memstore_free.argtypes = [C.c_void_p]
        _lib = L
    return _lib


class Segment:
    def __init__(self, dtypes):
        codes = [DTYPE_CODES[d] if isinstance(d, str) else int(d) for d in dtypes]
        self.codes = codes
        n = len(codes)
        self._dt = (C.c_uint32 * max(n, 1))(*codes)
        self._cols = (OcColumn * max(n, 1))()
        self.seg = OcSegment()
        st = lib().oc_segment_init(self._dt, n, self._cols, C.byref(self.seg))
        if st:
            raise ValueError(f"oc_segment_init: {st}")

    @property
    def bitset_size(self):
        return self.seg.bitset_size

    @property
    def capacity(self):
        return self.seg.capacity


class OracleError(Exception):
    def __init__(self, status, row, column, message):
        super().__init__(f"status={status} row={row} column={column}: {message}")
        self.status, self.row, self.column, self.message = status, row, column, message


def _take_array(a: OcArray):
    n = a.length
    out = {"dtype": a.dtype, "length": n, "null_count": a.null_count,
           "values": C.string_at(a.values, a.values_len) if a.values_len else b"",
           "validity": C.string_at(a.validity, (n + 7) // 8) if a.validity else None,
           "offsets": None}
    if a.dtype == 0:
        out["offsets"] = np.ctypeslib.as_array(a.offsets, shape=(n + 1,)).copy()
    return out


def decode_block(seg: Segment, proj, data: bytes | np.ndarray, row_off: np.ndarray):
    """Store::read-style decode of one block through the restated ReadBatchBuilder."""
    proj = list(proj)
    np_ = len(proj)
    pj = (C.c_uint32 * max(np_, 1))(*proj)
    outs = (OcArray * max(np_, 1))()
    err = OcError()
    data = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else data
    data = np.ascontiguousarray(data, dtype=np.uint8)
    if data.size == 0:
        data = np.zeros(1, np.uint8)
    row_off = np.ascontiguousarray(row_off, dtype=np.uint64)
    n = row_off.size - 1
    st = lib().oc_decode_block(C.byref(seg.seg), pj, np_, data.ctypes.data, row_off.ctypes.data,
                               n, outs, C.byref(err))
    if st:
        raise OracleError(st, err.row, err.column, err.message.decode(errors="replace"))
    res = []
    for p in range(np_):
        res.append(_take_array(outs[p]))
        lib().oc_array_free(C.byref(outs[p]))
    return res


class MemStore:
    """MemoryStore (src/io/store/memory.rs) restated over host buffers: keys as
    an Arrow utf8/binary array (row i = key i; a repeated key maps to its
    later row), blobs back to back with row_off[n+1].  read() is Store::read:
    per key its blob into the ReadBatchBuilder or add_empty, then build()."""

    def __init__(self, keys, blob, row_off):
        import pyarrow as pa
        keys = keys if isinstance(keys, pa.Array) else pa.array(keys, pa.string())
        if keys.offset:
            keys = pa.concat_arrays([keys])
        b = keys.buffers()
        self._keys = keys  # (the store keeps pointers into these buffers)
        self._blob = np.ascontiguousarray(np.frombuffer(blob, np.uint8) if isinstance(blob, (bytes, bytearray))
                                          else blob, dtype=np.uint8)
        if self._blob.size == 0:
            self._blob = np.zeros(1, np.uint8)
        self._off = np.ascontiguousarray(row_off, dtype=np.uint64)
        n = len(keys)
        self.h = lib().oc_memstore_new(b[2].address if b[2] is not None else None, b[1].address, n,
                                       self._blob.ctypes.data, self._off.ctypes.data)
        if not self.h:
            raise MemoryError("oc_memstore_new")

    def read_raw(self, seg: Segment, proj, nproj: int, q_data: int, q_off: int, nq: int, outs, err) -> int:
        """The timed call: keys as raw Arrow buffers; outs[nproj] owned by the caller."""
        return lib().oc_memstore_read(self.h, C.byref(seg.seg), proj, nproj, q_data, q_off, nq, outs,
                                      C.byref(err))

    def read(self, seg: Segment, proj, keys):
        import pyarrow as pa
        q = keys if isinstance(keys, pa.Array) else pa.array(keys, pa.string())
        if q.offset:
            q = pa.concat_arrays([q])
        qb = q.buffers()
        proj = list(proj)
        pj = (C.c_uint32 * max(len(proj), 1))(*proj)
        outs = (OcArray * max(len(proj), 1))()
        err = OcError()
        st = self.read_raw(seg, pj, len(proj), qb[2].address if qb[2] is not None and len(q) else None,
                           qb[1].address if len(q) else None, len(q), outs, err)
        if st:
            raise OracleError(st, err.row, err.column, err.message.decode(errors="replace"))
        res = []
        for p in range(len(proj)):
            res.append(_take_array(outs[p]))
            lib().oc_array_free(C.byref(outs[p]))
        return res

    def close(self):
        if self.h:
            lib().oc_memstore_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def encode_batch(seg: Segment, cols, n: int):
    """cols: per segment column a dict of numpy/bytes buffers
    {values, validity (or None), offsets (utf8), offset}.  Returns (blob, row_off)."""
    keep = []
    cin = (OcColIn * max(len(cols), 1))()
    for i, c in enumerate(cols):
        def ptr(b):
            if b is None:
                return None
            a = np.frombuffer(b, dtype=np.uint8) if isinstance(b, (bytes, bytearray)) else b
            a = np.ascontiguousarray(a)
            if a.size == 0:
                a = np.zeros(8, np.uint8)
            keep.append(a)
            return a.ctypes.data
        cin[i].values = ptr(c.get("values"))
        cin[i].validity = ptr(c.get("validity"))
        cin[i].offsets = ptr(c.get("offsets"))
        cin[i].offset = int(c.get("offset", 0))
    blob = C.POINTER(C.c_uint8)()
    blen = C.c_uint64()
    row_off = np.zeros(n + 1, np.uint64)
    err = OcError()
    st = lib().oc_encode_batch(C.byref(seg.seg), cin, n, C.byref(blob), C.byref(blen),
                               row_off.ctypes.data, C.byref(err))
    if st:
        raise OracleError(st, err.row, err.column, err.message.decode(errors="replace"))
    out = np.frombuffer(C.string_at(blob, blen.value), dtype=np.uint8).copy()
    lib().oc_free(blob)
    return out, row_off


def utf8_valid(b: bytes):
    vut = C.c_uint64()
    el = C.c_int()
    ok = lib().oc_utf8_valid(b, len(b), C.byref(vut), C.byref(el))
    return bool(ok), vut.value, el.value


# ---- RocksDB data blocks (murr_sst.c) ------------------------------------------

SST_E_CORRUPT = 12


def _inflate(fn, src: bytes, what: str) -> bytes:
    n = C.c_uint64()
    st = lib().oc_snappy_uncompressed_len(src, len(src), C.byref(n))
    if st:
        raise OracleError(st, 0, 0, what)
    out = C.create_string_buffer(max(n.value, 1))
    got = C.c_uint64()
    st = fn(src, len(src), out, n.value, C.byref(got))
    if st:
        raise OracleError(st, 0, 0, what)
    return out.raw[:got.value]


def snappy_decompress(src: bytes) -> bytes:
    """Raw Snappy (the restatement in murr_sst.c)."""
    return _inflate(lib().oc_snappy_decompress, src, "corrupt snappy")


def lz4_decompress(src: bytes) -> bytes:
    """varint32 length + LZ4 block, as RocksDB stores LZ4 blocks (murr_sst.c)."""
    return _inflate(lib().oc_lz4_decompress, src, "corrupt lz4")


def sst_decode_all(data: np.ndarray, handles: np.ndarray):
    """Every block of `data` (handles: int64 [nb, 3] offset, size, compression)
    inflated and decoded in C, one thread: (entries, key bytes, value bytes)."""
    data = np.ascontiguousarray(data, np.uint8)
    off = np.ascontiguousarray(handles[:, 0], np.uint64)
    size = np.ascontiguousarray(handles[:, 1], np.uint64)
    comp = np.ascontiguousarray(handles[:, 2], np.uint32)
    ne, kb, vb = C.c_uint64(), C.c_uint64(), C.c_uint64()
    st = lib().oc_sst_decode_all(data.ctypes.data, off.ctypes.data, size.ctypes.data, comp.ctypes.data, len(off),
                                 C.byref(ne), C.byref(kb), C.byref(vb))
    if st:
        raise OracleError(st, 0, 0, "corrupt block")
    return ne.value, kb.value, vb.value


def block_contents(stored: bytes, compression: int) -> bytes:
    """A stored data block's uncompressed contents (0 none, 1 Snappy, 4/5 LZ4)."""
    if compression == 0:
        return stored
    if compression == 1:
        return snappy_decompress(stored)
    if compression in (4, 5):
        return lz4_decompress(stored)
    raise OracleError(12, 0, 0, f"unsupported compression {compression}")


def block_decode(block: bytes):
    """Entries of one uncompressed RocksDB data block, in block order:
    (user keys, values, sequence numbers, value types)."""
    ne, kb, vb = C.c_uint64(), C.c_uint64(), C.c_uint64()
    st = lib().oc_block_count(block, len(block), C.byref(ne), C.byref(kb), C.byref(vb))
    if st:
        raise OracleError(st, 0, 0, "corrupt block")
    n = ne.value
    keys = C.create_string_buffer(max(kb.value, 1))
    vals = C.create_string_buffer(max(vb.value, 1))
    koff = np.zeros(n + 1, np.int32)
    voff = np.zeros(n + 1, np.uint64)
    seqs = np.zeros(max(n, 1), np.uint64)
    types = np.zeros(max(n, 1), np.uint8)
    st = lib().oc_block_decode(block, len(block), keys, koff.ctypes.data, vals, voff.ctypes.data,
                               seqs.ctypes.data, types.ctypes.data)
    if st:
        raise OracleError(st, 0, 0, "corrupt block")
    kr, vr = keys.raw, vals.raw
    return ([kr[koff[i]:koff[i + 1]] for i in range(n)], [vr[int(voff[i]):int(voff[i + 1])] for i in range(n)],
            seqs[:n].copy(), types[:n].copy())
