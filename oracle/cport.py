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
PERM_SRC = HERE / "c" / "perm_cpu.c"
PERM_LIB = HERE / "c" / "libpermcpu.so"
L = 2**252 + 27742317777372353535851937790883648493

_lib = None


def build(force: bool = False) -> Path:
    if force or not LIB.exists() or LIB.stat().st_mtime < SRC.stat().st_mtime:
        cmd = ["gcc", "-O3", "-march=x86-64-v3", "-mtune=native", "-shared", "-fPIC", "-o", str(LIB), str(SRC)]
        subprocess.run(cmd, check=True)
    newest = max(SRC.stat().st_mtime, PERM_SRC.stat().st_mtime)
    if force or not PERM_LIB.exists() or PERM_LIB.stat().st_mtime < newest:
        cmd = ["gcc", "-O3", "-march=x86-64-v3", "-mtune=native", "-shared", "-fPIC", "-I", str(SRC.parent), "-o",
               str(PERM_LIB), str(PERM_SRC)]
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


def _chunks(n: int, parts: int):
    return [(n * i // parts, n * (i + 1) // parts) for i in range(parts)]


def from_uniform_threads(bytes64: bytes, threads: int | None = None) -> bytes:
    """from_uniform over `threads` workers (ctypes drops the GIL)."""
    import concurrent.futures as cf
    n = len(bytes64) // 64
    threads = max(1, min(threads or host_cores(), n or 1))
    with cf.ThreadPoolExecutor(threads) as ex:
        outs = list(ex.map(lambda ab: from_uniform(bytes64[64 * ab[0]: 64 * ab[1]]), _chunks(n, threads)))
    return b"".join(outs)


def msm_threads(scalars: bytes, points: bytes, threads: int | None = None) -> bytes:
    """Exact MSM on all host cores: the terms split into `threads` chunks,
    each a serial dalek-style MSM (port_msm), the chunk results decoded and
    summed with the Python spec oracle.  Test / golden-generation only."""
    import concurrent.futures as cf

    from oracle import ristretto as r255
    n = len(scalars) // 32
    threads = max(1, min(threads or host_cores(), n or 1))
    with cf.ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(lambda ab: msm(scalars[32 * ab[0]: 32 * ab[1]], points[32 * ab[0]: 32 * ab[1]]),
                            _chunks(n, threads)))
    acc = r255.IDENTITY
    for p in parts:
        acc = r255.ed_add(acc, r255.decode(p))
    return r255.encode(acc)


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


# ------------------------------------------------------------ CPU prover port
_plib = None


def perm_lib():
    global _plib
    if _plib is None:
        if not PERM_LIB.exists():
            build()
        _plib = C.CDLL(str(PERM_LIB))
        _plib.cpu_perm_setup.argtypes = [C.c_uint32]
        _plib.cpu_perm_proof_len.argtypes = [C.c_uint32]
        _plib.cpu_perm_proof_len.restype = C.c_size_t
        _plib.cpu_perm_prove.argtypes = [C.c_uint32, C.c_uint64, C.c_char_p, C.c_size_t, C.c_char_p, C.c_char_p]
        _plib.cpu_perm_time.argtypes = [C.c_uint32, C.c_uint64, C.c_int, C.c_char_p, C.c_size_t]
        _plib.cpu_perm_time.restype = C.c_double
    return _plib


def cpu_prove(k: int, seed: int, label: bytes = b"bp-perm"):
    """-> (proof bytes, [V_j]) from the serial C prover (perm_cpu.c)."""
    lib_ = perm_lib()
    assert lib_.cpu_perm_setup(k) == 0
    pl = lib_.cpu_perm_proof_len(k)
    pf = C.create_string_buffer(pl)
    V = C.create_string_buffer(32 * (2 * k + 1))
    assert lib_.cpu_perm_prove(k, seed, label, len(label), pf, V) == 0
    raw = V.raw
    return pf.raw, [raw[32 * j: 32 * j + 32] for j in range(2 * k + 1)]


def host_cores() -> int:
    """CPUs this process may use: the cgroup quota when one is set (the GPU
    box reports 256 CPUs but grants 16), else the affinity mask."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            return max(1, int(int(q) / int(p)))
    except Exception:
        pass
    return len(os.sched_getaffinity(0))


def bench_prove(k: int = 52, seconds: float = 10.0, threads: int = 1, label: bytes = b"bp-perm") -> dict:
    """52-card proofs/s of the serial C prover: `threads` workers (one proof
    at a time each, ctypes releases the GIL), ~`seconds` of wall time."""
    import threading
    lib_ = perm_lib()
    assert lib_.cpu_perm_setup(k) == 0
    t1 = lib_.cpu_perm_time(k, 10_000, 1, label, len(label))
    per = max(1, int(seconds / max(t1, 1e-6)))
    secs = [0.0] * threads

    def work(i):
        secs[i] = lib_.cpu_perm_time(k, 1_000_000 * (i + 1), per, label, len(label))

    th = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = max(secs)
    return {"value": threads * per / wall, "unit": "proofs/s", "cores": threads, "kind": "port",
            "sample": f"{threads} x {per} {k}-card proofs (serial C restatement: dalek-ng Straus/Pippenger MSMs, "
                      f"bulletproofs folding IPA, merlin), {wall:.1f} s"}


def bench_msm_threads(log2n: int = 16, seconds: float = 10.0, threads: int = 1) -> dict:
    """All-cores MSM baseline: `threads` independent 2^log2n MSMs in parallel."""
    import threading
    n = 1 << log2n
    sc, pts = synth(n, 7)
    out = C.create_string_buffer(32)
    t1 = lib().port_time_msm(sc, pts, n, 1, out)
    reps = max(1, int(seconds / max(t1, 1e-6)))
    secs = [0.0] * threads

    def work(i):
        o = C.create_string_buffer(32)
        secs[i] = lib().port_time_msm(sc, pts, n, reps, o)

    th = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = max(secs)
    return {"value": threads * n * reps / wall, "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"{threads} threads x {reps} x 2^{log2n}-pair MSM, {wall:.1f} s"}


# ------------------------------------------------------------ config 2 (commit + IPA)
def config2_inputs(n: int = 1024, seed: int = 1):
    """bench.py bench_config2's inputs (tests/golden/make_golden.py
    config2_inputs): SHAKE256("config2" || le64 seed) read as 64-byte wide
    scalars aL[n], aR[n], alpha, then 64 bytes for Q = from_uniform."""
    xof = hashlib.shake_256(b"config2" + seed.to_bytes(8, "little")).digest((2 * n + 1) * 64 + 64)
    sc = b"".join((int.from_bytes(xof[64 * i: 64 * i + 64], "little") % L).to_bytes(32, "little")
                  for i in range(2 * n + 1))
    return sc, xof[(2 * n + 1) * 64:]


def _c2lib():
    lib_ = perm_lib()
    lib_.cpu_config2_setup.argtypes = [C.c_uint32]
    lib_.cpu_config2.argtypes = [C.c_uint32, C.c_char_p, C.c_char_p, C.c_char_p, C.c_size_t, C.c_char_p]
    lib_.cpu_config2_time.argtypes = [C.c_uint32, C.c_char_p, C.c_char_p, C.c_char_p, C.c_size_t, C.c_int]
    lib_.cpu_config2_time.restype = C.c_double
    return lib_


def cpu_config2(n: int = 1024, seed: int = 1, label: bytes = b"config2") -> dict:
    """Config 2 through the serial C port (dalek-style MSMs, bulletproofs'
    folding IPA): A, L/R, a, b as hex (the fields of protocol.json config2)."""
    lib_ = _c2lib()
    assert lib_.cpu_config2_setup(n) == 0
    sc, q = config2_inputs(n, seed)
    lg = n.bit_length() - 1
    out = C.create_string_buffer(32 * (1 + 2 * lg + 2))
    assert lib_.cpu_config2(n, sc, q, label, len(label), out) == 0
    raw = out.raw
    return {"A": raw[:32].hex(), "L": [raw[32 + 64 * j: 64 + 64 * j].hex() for j in range(lg)],
            "R": [raw[64 + 64 * j: 96 + 64 * j].hex() for j in range(lg)],
            "a": raw[32 + 64 * lg: 64 + 64 * lg].hex(), "b": raw[64 + 64 * lg: 96 + 64 * lg].hex()}


def bench_config2(n: int = 1024, seed: int = 1, seconds: float = 5.0, threads: int = 1,
                  label: bytes = b"config2") -> dict:
    """Config 2 runs/s of the serial C port on `threads` host cores (each
    thread repeats the whole commit + IPA one at a time)."""
    import threading
    lib_ = _c2lib()
    assert lib_.cpu_config2_setup(n) == 0
    sc, q = config2_inputs(n, seed)
    t1 = lib_.cpu_config2_time(n, sc, q, label, len(label), 1)
    per = max(1, int(seconds / max(t1, 1e-6)))
    secs = [0.0] * threads

    def work(i):
        secs[i] = lib_.cpu_config2_time(n, sc, q, label, len(label), per)

    th = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = max(secs)
    return {"value": wall / per * 1e3, "unit": "ms", "runs_per_sec": threads * per / wall, "cores": threads,
            "kind": "port",
            "sample": f"{threads} x {per} runs of n = {n} vector commitment + IPA (dalek-ng Straus/Pippenger, "
                      f"bulletproofs folding IPA, merlin, restated in C), {wall:.1f} s"}
