"""Projections never compile on the read path.

Table::read takes an arbitrary column list per request
(src/io/table/mod.rs:114-129).  The decode kernel is specialised on the
segment layout only (murr_jit_kernel.hip); the table compiles it once at open
(murr_segment_prepare) and every projection -- subsets, permutations,
duplicates -- runs the same code object.  A never-seen projection's first read
must therefore cost about what a repeated one costs (a hiprtc compile takes
seconds; preparing the projection's read plan, a millisecond at most), and must
decode exactly like the builder path over MemoryStore."""
import time

import numpy as np
import pytest

from murr_amd.resident import ResidentTable
from murr_amd.row import default_context

from test_gpu_resident import C_DTYPES, assert_same, batch_c, expected, schema_c

pytestmark = pytest.mark.gpu


def test_new_projection_first_read_costs_no_compile():
    ctx = default_context()
    ctx.set_opts(kernel="jit")  # a JIT failure is an error here
    rt = ResidentTable(schema_c(), ctx)  # compiles the layout (or loads it)
    batch = batch_c(20_000)
    rt.write(batch)
    rng = np.random.default_rng(5)
    keys = [f"key{i}" for i in rng.integers(0, 21_000, size=1000)]
    names = [f"c{i}" for i in range(len(C_DTYPES))]
    rt.read(keys, names)  # first read: buffers, first launches
    warm = []
    for _ in range(5):
        t0 = time.perf_counter()
        rt.read(keys, names)
        warm.append(time.perf_counter() - t0)
    warm_s = float(np.median(warm))
    projections = [["c3"], ["c12", "c0"], names[::-1], ["c11", "c11", "c5", "c11"],
                   [names[i] for i in rng.permutation(16)[:7]], ["c15", "c14", "c13", "c12", "c1"]]
    for cols in projections:
        t0 = time.perf_counter()
        got = rt.read(keys, cols)
        first = time.perf_counter() - t0
        assert_same(got, expected([batch], keys, cols))
        # no compile (seconds): within 20 ms of a warm read of every column --
        # the first read of a projection prepares its read plan, whose pinned
        # and device buffers may be new allocations (~1 ms on some boxes)
        assert first < warm_s + 20e-3, (cols, first, warm_s)
    ctx.set_opts()
