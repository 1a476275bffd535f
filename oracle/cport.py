"""ctypes harness for oracle/c/dalek_port.c — TEST / CPU-BASELINE ONLY.

`build()` compiles the serial C restatement of dalek-ng's MSM with gcc into
oracle/c/libdalekport.so (git-ignored; travels to the GPU box in the
snapshot).  `bench_msm()` is bench.py's `cpu_baseline` leg ("kind": "port").
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os
import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRC = HERE / "c" / "dalek_port.c"
LIB = HERE / "c" / "libdalekport.so"
L = 2**252 + 27742317777372353535851937790883648493

_lib = None


def build(force: bool = False) -> Path:
    if force or not LIB.exists() or LIB.stat().st_mtime < SRC.stat().st_mtime:
        cmd = ["gcc", "-O3", "-march=x86-64-v3", "-mtune=native", "-shared", "-fPIC", "-o", str(LIB), str(SRC)]
        subprocess.run(cmd, check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        _lib = C.CDLL(str(LIB))
        _lib.port_msm.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t, C.c_char_p]
        _lib.port_msm.restype = C.c_int
        _lib.port_time_msm.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t, C.c_int, C.c_char_p]
        _lib.port_time_msm.restype = C.c_double
        _lib.port_from_uniform.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p]
        _lib.port_from_uniform.restype = C.c_int
    return _lib


def msm(scalars: bytes, points: bytes) -> bytes:
    n = len(scalars) // 32
    out = C.create_string_buffer(32)
    rc = lib().port_msm(scalars, points, n, out)
    if rc != 0:
        raise ValueError(f"invalid point encoding at {-rc - 1}")
    return out.raw


def from_uniform(bytes64: bytes) -> bytes:
    n = len(bytes64) // 64
    out = C.create_string_buffer(32 * n)
    lib().port_from_uniform(bytes64, n, out)
    return out.raw


def synth(n: int, seed: int):
    raw = hashlib.shake_256(b"cpu-scalars" + seed.to_bytes(8, "little")).digest(64 * n)
    sc = b"".join((int.from_bytes(raw[64 * i: 64 * i + 64], "little") % L).to_bytes(32, "little") for i in range(n))
    pts = from_uniform(hashlib.shake_256(b"cpu-points" + seed.to_bytes(8, "little")).digest(64 * n))
    return sc, pts


def bench_msm(log2n: int = 16, seconds: float = 15.0) -> dict:
    """Time dalek-style serial Pippenger (w=8 at this size) on one core."""
    n = 1 << log2n
    sc, pts = synth(n, 7)
    out = C.create_string_buffer(32)
    t1 = lib().port_time_msm(sc, pts, n, 1, out)
    reps = max(1, int(seconds / max(t1, 1e-6)))
    t = lib().port_time_msm(sc, pts, n, reps, out) if reps > 1 else t1
    return {"value": n * reps / t, "unit": "pairs/s", "cores": 1, "kind": "port",
            "sample": f"{reps} x 2^{log2n}-pair MSM (dalek-ng 4.1.1 Pippenger w=8 restated in C, 1 thread), {t:.1f} s"}
