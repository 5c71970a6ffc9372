"""bench.py's host-side pieces, CPU only: the PMC traffic reader (only the
timed kernel's dispatches count; FETCH_SIZE doubled per the gfx950
correction, MI355X_MICROARCH.md §HBM) and the projection argument."""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
import bench  # noqa: E402


def write_pmc(path, counter, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for d, k, v in rows:
            w.writerow({"Dispatch_Id": d, "Kernel_Name": k, "Counter_Name": counter, "Counter_Value": v})


def test_traffic_counts_only_the_timed_kernel(tmp_path):
    f, w = str(tmp_path / "fetch.csv"), str(tmp_path / "write.csv")
    # two dispatches of the timed kernel (one split into two XCD rows), one of
    # the untimed split-mode variant and a copy kernel: only the first count
    write_pmc(f, "FETCH_SIZE", [(1, "murr_jit_decode_3x1", 400.0), (1, "murr_jit_decode_3x1", 100.0),
                                (2, "murr_jit_decode_3x1", 500.0), (3, "murr_jit_decode_split_3x1", 9000.0),
                                (4, "__amd_rocclr_copyBuffer", 7.0)])
    write_pmc(w, "WRITE_SIZE", [(1, "murr_jit_decode_3x1", 300.0), (2, "murr_jit_decode_3x1", 300.0),
                                (3, "murr_jit_decode_split_3x1", 300.0)])
    got = bench.pmc_traffic(f"{f},{w}", "murr_jit_decode_3x1")
    assert got == round((2 * 500.0 + 300.0) * 1024)
    # without a kernel filter every decode dispatch counts (the old reading)
    assert bench.pmc_traffic(f"{f},{w}") == round((2 * (500 + 500 + 9000) / 3 + 300.0) * 1024)


def test_traffic_missing_file_is_none(tmp_path):
    assert bench.pmc_traffic(str(tmp_path / "nope.csv"), "x") is None
    assert bench.pmc_traffic(None) is None


def test_traffic_pass_is_never_nested(monkeypatch):
    # a bench already under rocprofv3 leaves the counters to it
    monkeypatch.setenv("ROCPROF_COUNTERS", "FETCH_SIZE")
    assert bench.measure_traffic(None, "murr_jit_decode_5x3") is None


def test_parse_proj():
    assert bench.parse_proj(None, 3) == [0, 1, 2]
    assert bench.parse_proj("rev", 3) == [2, 1, 0]
    assert bench.parse_proj("4,0,4", 5) == [4, 0, 4]
