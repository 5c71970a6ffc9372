"""The layout-specialised decode kernel's code object, checked offline (CPU:
hipcc cross-compiles gfx950): with the sample prelude of config B's layout
(murr_amd/csrc/jit_sample_B.h) no kernel may use scratch memory.  A local
array passed by pointer into a helper once put a stack slot and a
`scratch_load` + `s_waitcnt vmcnt(0)` into the decode loop -- waiting on every
store in flight each chunk (config B 0.73 -> 1.22 ms, round 5)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "murr_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("sample", ["jit_sample_B.h", "jit_sample_C.h"])
def test_decode_kernels_use_no_scratch(tmp_path, sample):
    out = tmp_path / "k.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-include", os.path.join(CSRC, sample),
                    "-S", "--cuda-device-only", "-o", str(out), os.path.join(CSRC, "murr_jit_kernel.hip")],
                   check=True, capture_output=True, timeout=600)
    # assembled too: operand errors of inline asm (e.g. the constant-bus
    # limit) show only when the assembler sees them, and at run time hiprtc
    # would fall back to the generic kernel for that layout
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-include", os.path.join(CSRC, sample),
                    "-c", "--cuda-device-only", "-o", str(tmp_path / "k.o"), os.path.join(CSRC, "murr_jit_kernel.hip")],
                   check=True, capture_output=True, timeout=600)
    asm = out.read_text()
    names = re.findall(r"\.name:\s+(murr_jit_decode\w*)", asm)
    sizes = re.findall(r"\.private_segment_fixed_size:\s+(\d+)", asm)
    assert names and len(names) == len(sizes), (names, sizes)
    assert all(int(x) == 0 for x in sizes), dict(zip(names, sizes))
    assert "scratch_load" not in asm and "scratch_store" not in asm
