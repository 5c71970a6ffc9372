"""MurrError variants (src/core/error.rs:4-19) and the C-ABI status mapping."""
from __future__ import annotations

from . import _abi


class MurrError(Exception):
    """Base of every error the reference's `MurrError` enum can carry."""


class ConfigParsingError(MurrError): pass
class IoError(MurrError): pass
class ArrowError(MurrError): pass
class TableNotFound(MurrError): pass
class TableAlreadyExists(MurrError): pass
class TableError(MurrError): pass
class SegmentError(MurrError): pass


class DeviceError(MurrError):
    """HIP runtime / device protocol failure (no reference counterpart)."""


def raise_status(st: int, err=None, what: str = ""):
    """Map a murr_status_t (+ murr_error_t) to the reference's error variant."""
    if st == _abi.OK:
        return
    loc = ""
    if err is not None:
        loc = f" (block {err.block}, row {err.row}, column {err.column})"
    msg = f"{what}{': ' if what else ''}{_abi.status_str(st)}{loc}"
    if st in (_abi.E_INVALID_UTF8, _abi.E_DTYPE, _abi.E_BAD_COLUMN, _abi.E_NULL_KEY,
              _abi.E_MALFORMED_ROW):
        raise SegmentError(msg)
    if st == _abi.E_ARROW:
        raise ArrowError(msg)
    if st == _abi.E_OFFSET_OVERFLOW:
        # arrow-rs panics here ("byte array offset overflow"); we surface it.
        raise ArrowError(msg)
    if st == _abi.E_HIP and err is not None:
        msg += f" hipError={err.hip_error}"
    raise DeviceError(msg) if st in (_abi.E_HIP, _abi.E_INTERNAL, _abi.E_NO_DEVICE) else MurrError(msg)
