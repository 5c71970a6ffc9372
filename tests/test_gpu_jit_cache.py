"""The in-memory cache of compiled segment layouts (murr_jit.cpp): layouts
beyond the bound are retired least-recently-used first, a retired layout's
code object is never unloaded under a launch that may use it, and a layout
used again after its eviction compiles (or loads from disk) again.  With the
bound lowered to 3 and 8 layouts decoded in turn, every decode must still
match the oracle."""
import ctypes as C

import numpy as np
import pytest

import oracle as O
from golden_util import assert_array_equal
from randgen import random_columns
from murr_amd import _abi, synth
from murr_amd.device import Context, DeviceBlock, decode_blocks, download_array
from murr_amd.schema import DTypeName as D, SegmentSchema

pytestmark = pytest.mark.gpu

LAYOUTS = [[D.Float32], [D.Int8, D.Utf8], [D.Utf8, D.Float64], [D.Bool, D.Int16, D.Utf8], [D.UInt64],
           [D.Utf8, D.Utf8, D.Int32], [D.Float32, D.Float32, D.Bool], [D.Int64, D.UInt8, D.Utf8, D.UInt16]]


def limit(n=0):
    lim, cached = C.c_uint32(), C.c_uint32()
    assert _abi.lib().murr_jit_cache_limit(n, C.byref(lim), C.byref(cached)) == 0
    return lim.value, cached.value


def test_lru_eviction_keeps_decodes_correct():
    old, _ = limit()
    ctx = Context(0)
    ctx.set_opts(kernel="jit")  # a compile failure is an error, never the generic fallback
    try:
        limit(3)
        rng = np.random.default_rng(7)
        for rnd in range(2):
            for li, dtypes in enumerate(LAYOUTS):
                n = 777 + 100 * li
                cols = random_columns(rng, dtypes, n, null_p=0.2, max_str=9)
                oseg = O.Segment([int(d) for d in dtypes])
                data, off = O.encode_batch(oseg, synth.oracle_cols(cols), n)
                seg = SegmentSchema([(f"c{i}", d) for i, d in enumerate(dtypes)])
                proj = list(range(len(dtypes)))[::-1]
                outs = decode_blocks(ctx, seg, proj, [DeviceBlock.upload(ctx, data, off)])
                assert ctx.last_kernel() == "murr_jit_decode"
                want = O.decode_block(oseg, proj, data, off)
                for p, ci in enumerate(proj):
                    got = download_array(ctx, outs.array(0, p), int(dtypes[ci]), n)
                    assert_array_equal(got, want[p], f"round {rnd} layout {li} proj {p}")
                lim, cached = limit()
                assert lim == 3 and cached <= 3, (lim, cached)
    finally:
        limit(old)
        ctx.close()
