"""Host C++ of libbpperm under ASan + UBSan and under TSan:
tests/c/host_sanitize.cpp is compiled with the library's host sources
(Keccak, 8-way Keccak, circuit) and run on the CPU.  The GPU kernels are not
sanitized (GPU ASan / xnack are unavailable on the pool)."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "bulletproof-perm_amd" / "csrc"
SRCS = [ROOT / "tests" / "c" / "host_sanitize.cpp", *sorted((CSRC / "host").glob("*.cpp"))]


def _build_run(tmp_path, name, flags, env_extra):
    exe = tmp_path / name
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread", "-march=x86-64-v3",
           "-I", str(CSRC), *flags, *map(str, SRCS), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, BPP_HOST_THREADS="4", **env_extra)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert r.stdout.strip() == "ok"


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not installed")
def test_host_asan_ubsan(tmp_path):
    _build_run(tmp_path, "host_asan", ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"],
               {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "UBSAN_OPTIONS": "print_stacktrace=1"})


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not installed")
def test_host_tsan(tmp_path):
    _build_run(tmp_path, "host_tsan", ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1"})


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not installed")
def test_from_wide_fast_path_matches_montgomery_form(tmp_path):
    """hsc::from_wide (the 2^252 = -delta folding used for every wide draw and
    challenge) equals the Montgomery-form reduction on 2 M inputs, under
    UBSan (signed shifts / carries)."""
    exe = tmp_path / "from_wide"
    cmd = ["g++", "-std=c++17", "-O2", "-g", "-march=x86-64-v3", "-fsanitize=undefined", "-fno-sanitize-recover=all",
           "-I", str(CSRC), str(ROOT / "tests" / "c" / "from_wide_check.cpp"), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "mismatches: 0" in r.stdout, (r.stdout + r.stderr)[-2000:]


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not installed")
def test_invert_vartime_matches_fermat(tmp_path):
    """hsc::invert_vartime (binary extended Euclid, the IPA challenges'
    inversions) equals hsc::invert (a^(l-2)) on ~200 K random, sparse and
    edge scalars, and batch_invert's vartime form equals its constant-time
    form, under UBSan."""
    exe = tmp_path / "invert"
    cmd = ["g++", "-std=c++17", "-O2", "-g", "-march=x86-64-v3", "-fsanitize=undefined", "-fno-sanitize-recover=all",
           "-I", str(CSRC), str(ROOT / "tests" / "c" / "invert_check.cpp"), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "mismatches: 0" in r.stdout, (r.stdout + r.stderr)[-2000:]


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not installed")
def test_ge_sum_x8_matches_scalar_chain(tmp_path):
    """h25519::ge_sum_x8 (the IPA split rounds' J-partial sums on AVX-512
    IFMA) encodes to the same bytes as one scalar ge_add chain per point, for
    n = 1..64 points of J = 2..64 terms (identity terms included), under
    UBSan; skipped inside the program on a CPU without IFMA."""
    exe = tmp_path / "ge_sum"
    cmd = ["g++", "-std=c++17", "-O2", "-g", "-march=x86-64-v3", "-fsanitize=undefined", "-fno-sanitize-recover=all",
           "-I", str(CSRC), str(ROOT / "tests" / "c" / "ge_sum_check.cpp"), str(CSRC / "host" / "encode_x8.cpp"),
           "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "mismatches: 0" in r.stdout, (r.stdout + r.stderr)[-2000:]
