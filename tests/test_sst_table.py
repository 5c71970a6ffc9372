"""The SST block table the host builds for murr_sst_decode (CPU: no device
calls): descriptors at buffer + offset with size and compression, bounds
checked against the buffer, the struct layout the C ABI reads."""
import ctypes as C
from types import SimpleNamespace

import numpy as np
import pytest

from murr_amd import _abi, sst


def test_block_table_fields_and_layout():
    buf = SimpleNamespace(ptr=0x7F0000001000, nbytes=1000)
    h = [(0, 100, sst.SNAPPY), (100, 0, sst.NONE), (100, 900, sst.LZ4)]
    t = sst.block_table(buf, h)
    assert t.dtype.itemsize == C.sizeof(_abi.SstBlock) == 24
    assert t["data"].tolist() == [buf.ptr, buf.ptr + 100, buf.ptr + 100]
    assert t["size"].tolist() == [100, 0, 900]
    assert t["compression"].tolist() == [1, 0, 4]
    assert len(sst.block_table(buf, np.zeros((0, 3), np.int64))) == 0


@pytest.mark.parametrize("bad", [(-1, 10, 1), (995, 10, 1), (0, 1001, 0), (10, -5, 1)])
def test_block_table_bounds(bad):
    buf = SimpleNamespace(ptr=4096, nbytes=1000)
    with pytest.raises(ValueError, match=r"block 1 "):
        sst.block_table(buf, [(0, 10, 1), bad])
