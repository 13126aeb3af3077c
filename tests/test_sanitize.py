"""Host-side race detection (the reference's `go test -race`, Makefile:34-36): the C++
runtime (ShareQueue, MinerBase job switching, CpuMiner cursor, AEAD, scrypt/HMAC/PBKDF2) built under
TSan and ASan+UBSan, driven by tools/sanitize/stress_runtime.cpp. The stress asserts the job-epoch
protocol: every share names an issued epoch, rebuilds from that epoch's template, meets that epoch's
target, and is never emitted twice across re-issues / pause-resume. A libFuzzer stage (ASan + UBSan) then
checks the native SV2 frame scanner against a reference decoder and the CPU hash paths on arbitrary input."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.mark.skipif(not (os.path.exists(CLANG) or shutil.which("clang++")), reason="no clang++")
def test_runtime_under_tsan_and_asan(tmp_path):
    env = dict(os.environ, OTEDAMA_SANITIZE_OUT=str(tmp_path))
    if not os.path.exists(CLANG):
        env["CXX"] = shutil.which("clang++")
    r = subprocess.run(["bash", str(ROOT / "tools" / "sanitize" / "run.sh"), "2"], env=env,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-6000:])
    assert "sanitize: tsan + asan/ubsan + fuzz clean" in r.stdout
    assert r.stdout.count("runtime stress: all checks passed") == 2
