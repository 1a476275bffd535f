"""Build libbpperm.so (HIP for gfx950 + host C++) in-tree.

    python bulletproof-perm_amd/build.py [--debug]

Every .hip under csrc/ is compiled with hipcc --offload-arch=gfx950 (host/*.cpp
with the host C++ compiler, g++ by default)
into build/ and linked into bpperm/libbpperm.so next to the ctypes wrapper,
so the shared object travels with a gpurun snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build"
OUT = ROOT / "bpperm" / "libbpperm.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
HOSTCXX = os.environ.get("BPP_HOSTCXX", "g++")
ARCH = os.environ.get("BPP_ARCH", "gfx950")


def sources():
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("host/*.cpp")))


def dep_headers():
    """Every file a source may include: a change to any of them rebuilds every
    object (the generated csrc/fe10_ops.inc included, tools/gen_fe10.py)."""
    return sorted(list(CSRC.glob("*.cuh")) + list(CSRC.glob("*.h")) + list(CSRC.glob("*.inc")) +
                  list(CSRC.glob("host/*.h")) + list(CSRC.glob("host/*.inc")) +
                  [ROOT.parent / "include" / "bpperm.h"])


def _compile(src: Path, flags, bdir: Path = BUILD) -> Path:
    obj = bdir / (src.relative_to(CSRC).as_posix().replace("/", "_") + ".o")
    deps = [src] + dep_headers()
    if obj.exists() and obj.stat().st_mtime >= max(d.stat().st_mtime for d in deps):
        return obj
    if src.suffix == ".hip":
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", *flags, "-x", "hip", "-c", str(src), "-o",
               str(obj)]
    else:  # host-only C++ (Keccak, circuit): the host compiler, no device pass
        hflags = [f for f in flags if f not in ("-Xarch_host", "-Wno-pass-failed")]
        cmd = [HOSTCXX, "-fPIC", "-std=c++17", *hflags, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(debug: bool = False, jobs: int | None = None, variant: str = "", defines=()) -> Path:
    """variant: build an A/B copy with extra -D defines into
    build/<variant>/ and bpperm/variants/libbpperm_<variant>.so (select it
    with BPP_LIB=...)."""
    bdir = BUILD / variant if variant else BUILD
    out = ROOT / "bpperm" / "variants" / f"libbpperm_{variant}.so" if variant else OUT
    bdir.mkdir(parents=True, exist_ok=True)
    out.parent.mkdir(exist_ok=True)
    flags = ["-O1", "-g"] if debug else ["-O3"]
    # host code (transcripts, scalar algebra, Keccak): x86-64-v3 (BMI2 mulx,
    # rorx) - 1.7x on Keccak-f in a microbenchmark; the GPU box hosts are EPYC
    flags += ["-Wno-unused-result", "-Wno-pass-failed", "-pthread", "-Xarch_host", "-march=x86-64-v3"]
    flags += [f"-D{d}" for d in defines]
    srcs = sources()
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, flags, bdir), srcs))
    if out.exists() and out.stat().st_mtime >= max(o.stat().st_mtime for o in objs):
        return out
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", str(out), *map(str, objs)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return out


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--variant", default="")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    a = ap.parse_args()
    print(build(debug=a.debug, variant=a.variant, defines=a.defines))
