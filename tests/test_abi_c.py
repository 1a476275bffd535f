"""Compiles tests/c/abi_host.c against include/bpperm.h with gcc, links it to
the product's libbpperm.so and runs it (host-side entry points only: no GPU
here).  This is the C-level caller the boundary is for."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not installed")
def test_c_caller_through_header(tmp_path):
    from bpperm import _lib
    libdir = _lib.LIB_PATH.parent
    exe = tmp_path / "abi_host"
    cmd = ["gcc", "-std=c11", "-Wall", "-Werror", "-I", str(ROOT / "include"), str(ROOT / "tests" / "c" / "abi_host.c"),
           "-o", str(exe), f"-L{libdir}", "-lbpperm", f"-Wl,-rpath,{libdir}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip() == "ok"


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not installed")
def test_c_caller_transcript_kat(tmp_path):
    """tests/c/merlin_min.h -- the caller-owned transcript abi_gpu.c puts
    behind bpp_transcript_hooks -- reproduces merlin's "simple transcript"
    known answer, so the GPU test's transcript is an independent Merlin."""
    exe = tmp_path / "merlin_kat"
    r = subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Werror", str(ROOT / "tests" / "c" / "merlin_kat.c"),
                        "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=30)
    assert r.stdout.strip() == "d5a21972d0d5fe320c0d263fac7fffb8145aa640af6e9bca177c03c7efcf0615"
