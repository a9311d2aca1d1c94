"""Host ASan + UBSan over the library's CPU-side code (SURVEY.md §5 'race detection / sanitizers': host
ASan/UBSan on the C-ABI shim in CPU tests).

tests/asan/host_fuzz.cpp is compiled with g++ -fsanitize=address,undefined together with the host sources of
libdcamd that take untrusted input or build tables without a GPU -- csrc/json_mini.h (config.json, safetensors
headers, the tuned GEMM table), csrc/safetensors_mini.h (the native session's weight reader) and
csrc/host_tables.cpp (DDIM / Adam tables, timestep embedding, cross-attention fold) -- and run on crafted and
mutated inputs.  Any sanitizer report, crash or wrong rejection fails the test.  The GPU kernels are not
covered here (GPU ASan is not available on this pool).
"""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "depth_completion_amd" / "csrc"


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_under_asan_ubsan(tmp_path):
    exe = tmp_path / "host_fuzz"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-static-libasan", "-I", str(CSRC), "-I", str(ROOT / "include"),
           str(ROOT / "tests" / "asan" / "host_fuzz.cpp"), str(CSRC / "host_tables.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=24")
    r = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, timeout=600, env=env)
    report = r.stdout + r.stderr
    assert r.returncode == 0, report[-4000:]
    assert "runtime error" not in report and "AddressSanitizer" not in report, report[-4000:]
    assert "clean (0 failures)" in r.stdout
