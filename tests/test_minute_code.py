"""minute_code (merkleTree.ts:33 key = minute.toString(3), coded as base-4
digits) -- the fast three-division form the kernels use, checked on the host
against the plain digit loop (tools/minute_code_check.hip)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_minute_code_fast_equals_digit_loop(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    exe = str(tmp_path / "mc")
    subprocess.run([hipcc, "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tools", "minute_code_check.hip"), "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad 0" in out.stdout
