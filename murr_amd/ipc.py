"""Arrow IPC framing of read results.

The reference serialises a read with arrow-rs's IPC writers: the HTTP fetch
handler with ``StreamWriter`` (schema message, one record-batch message,
end-of-stream; src/api/http/handlers.rs:93-101) and Flight DoGet with
``FlightDataEncoderBuilder`` (src/api/flight/mod.rs:85-87).  Here the messages
come from the C ABI (``murr_ipc_*``, murr_amd/csrc/murr_ipc.cpp): the host
variant frames a builder's host arrays, the device variant packs one decoded
block into a single HBM buffer (murr_amd/csrc/murr_ipc.hip) so the host gets
the wire bytes with one D2H copy.

Alignment 64 is arrow-rs ``IpcWriteOptions::default()``; 8 is Arrow C++'s.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from .errors import raise_status
from .schema import SegmentColumnSchema, SegmentSchema

ALIGN_ARROW_RS = 64


def _proj(segment: SegmentSchema, columns):
    cols = [c if isinstance(c, SegmentColumnSchema) else segment.columns[int(c)] for c in columns]
    pj = (C.c_uint32 * max(len(cols), 1))(*[c.index for c in cols])
    return cols, pj


def schema_message(segment: SegmentSchema, columns, alignment: int = ALIGN_ARROW_RS) -> bytes:
    """Encapsulated Schema message for the requested columns (request order)."""
    L = _abi.lib()
    cols, pj = _proj(segment, columns)
    names = (C.c_char_p * max(len(cols), 1))(*[c.name.encode() for c in cols])
    n = C.c_uint64()
    raise_status(L.murr_ipc_schema(C.byref(segment.c), pj, len(cols), names, alignment, None, 0, C.byref(n)),
                 what="murr_ipc_schema")
    buf = C.create_string_buffer(n.value)
    raise_status(L.murr_ipc_schema(C.byref(segment.c), pj, len(cols), names, alignment, buf, n.value,
                                   C.byref(n)), what="murr_ipc_schema")
    return buf.raw[: n.value]


def batch_message_host(segment: SegmentSchema, columns, host_arrays, n_rows: int,
                       alignment: int = ALIGN_ARROW_RS) -> bytes:
    """Encapsulated RecordBatch message from murr_host_array_t outputs."""
    L = _abi.lib()
    cols, pj = _proj(segment, columns)
    n = C.c_uint64()
    raise_status(L.murr_ipc_batch_host(C.byref(segment.c), pj, len(cols), host_arrays, n_rows, alignment,
                                       None, 0, C.byref(n)), what="murr_ipc_batch_host")
    buf = C.create_string_buffer(max(n.value, 1))
    raise_status(L.murr_ipc_batch_host(C.byref(segment.c), pj, len(cols), host_arrays, n_rows, alignment,
                                       buf, n.value, C.byref(n)), what="murr_ipc_batch_host")
    return buf.raw[: n.value]


def batch_message_device(ctx, segment: SegmentSchema, proj, outs, block: int, n_rows: int,
                         alignment: int = ALIGN_ARROW_RS, dev_out=None):
    """Pack block `block` of DecodeOutputs into one device buffer.

    Returns (DeviceBuffer, length); the message is bytes [0, length)."""
    L = ctx.L
    proj = list(proj)
    pj = (C.c_uint32 * max(len(proj), 1))(*proj)
    arrays = C.cast(C.byref(outs.arrays, block * len(proj) * C.sizeof(_abi.Array)), C.POINTER(_abi.Array))
    n = C.c_uint64()
    err = _abi.Error()
    raise_status(L.murr_ipc_batch_device(ctx.h, C.byref(segment.c), pj, len(proj), arrays, n_rows, alignment,
                                         None, 0, C.byref(n), C.byref(err)), err, "murr_ipc_batch_device")
    if dev_out is None or dev_out.nbytes < n.value:
        dev_out = ctx.alloc(max(n.value, 16))
    raise_status(L.murr_ipc_batch_device(ctx.h, C.byref(segment.c), pj, len(proj), arrays, n_rows, alignment,
                                         dev_out.ptr, dev_out.nbytes, C.byref(n), C.byref(err)), err,
                 "murr_ipc_batch_device")
    return dev_out, n.value


def eos() -> bytes:
    """End-of-stream marker (StreamWriter::finish)."""
    out = (C.c_uint8 * 8)()
    _abi.lib().murr_ipc_eos(out)
    return bytes(out)


def stream(schema_msg: bytes, *batch_msgs) -> bytes:
    """An IPC stream: schema, record batches, end-of-stream (handlers.rs:93-101)."""
    return b"".join([schema_msg, *[bytes(m) for m in batch_msgs], eos()])


def download_message(ctx, dev_buf, length: int) -> bytes:
    out = np.empty(length, dtype=np.uint8)
    if length:
        raise_status(ctx.L.murr_memcpy_d2h(ctx.h, out.ctypes.data, dev_buf.ptr, length), what="d2h")
    return out.tobytes()
