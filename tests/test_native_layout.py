"""Host build of the fused kernels' index arithmetic under AddressSanitizer + UBSan.

``tests/native/test_layout.cpp`` includes the engine's own layout code (fedmi/ops/csrc/fl_layout.h),
replays every LDS address the bf16 / fp32 round kernels compute for 288 model shapes and checks
bounds, overlap and alignment; each region is an exact-size heap allocation, so ASan flags any
out-of-region index.  Runs on the CPU (no GPU needed)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not available")
def test_kernel_layouts_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "test_layout")
    cmd = ["hipcc", "-O1", "-g", "-std=c++17", "-Xarch_host", "-fsanitize=address", "-Xarch_host",
           "-fsanitize=undefined", "-fno-omit-frame-pointer", "-I" + os.path.join(ROOT, "fedmi", "ops", "csrc"),
           os.path.join(ROOT, "tests", "native", "test_layout.cpp"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "failures: 0" in r.stdout and "layouts checked: " in r.stdout
