"""Host code under AddressSanitizer / UndefinedBehaviorSanitizer (CPU only; no
GPU sanitizer exists on this pool): tools/asan/arrow_export_check.cpp drives
murr_arrow_export (the Arrow C Data Interface export of a read's batch)
through every dtype, nulls, empty and zero-column batches and a rejection,
reads every exported byte back and releases the export; and the Arrow IPC
host framing (murr_ipc_schema / murr_ipc_batch_host) at three alignments."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_arrow_export_under_asan(tmp_path):
    exe = str(tmp_path / "arrow_export_check")
    cmd = [HIPCC, "-O1", "-g", "-std=c++17", "-Xarch_host", "-fsanitize=address", "-Xarch_host",
           "-fsanitize=undefined", "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "murr_amd", "csrc"),
           os.path.join(ROOT, "tools", "asan", "arrow_export_check.cpp"),
           os.path.join(ROOT, "murr_amd", "csrc", "murr_arrow.cpp"),
           os.path.join(ROOT, "murr_amd", "csrc", "murr_ipc.cpp"), "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "arrow_export_check: ok" in out.stdout
