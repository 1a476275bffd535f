"""Build libbpperm.so (HIP for gfx950 + host C++) in-tree.

    python bulletproof-perm_amd/build.py [--debug]

Every .hip / .cpp under csrc/ is compiled with hipcc --offload-arch=gfx950
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
ARCH = os.environ.get("BPP_ARCH", "gfx950")


def sources():
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("host/*.cpp")))


def _compile(src: Path, flags) -> Path:
    obj = BUILD / (src.relative_to(CSRC).as_posix().replace("/", "_") + ".o")
    deps = [src] + list(CSRC.glob("*.cuh")) + list(CSRC.glob("*.h")) + list(CSRC.glob("host/*.h")) + \
        [ROOT.parent / "include" / "bpperm.h"]
    if obj.exists() and obj.stat().st_mtime >= max(d.stat().st_mtime for d in deps):
        return obj
    lang = ["-x", "hip"] if src.suffix == ".hip" else []
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", *flags, *lang, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(debug: bool = False, jobs: int | None = None) -> Path:
    BUILD.mkdir(exist_ok=True)
    flags = ["-O1", "-g"] if debug else ["-O3"]
    flags += ["-Wno-unused-result", "-Wno-pass-failed", "-pthread"]
    srcs = sources()
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, flags), srcs))
    if OUT.exists() and OUT.stat().st_mtime >= max(o.stat().st_mtime for o in objs):
        return OUT
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", str(OUT), *map(str, objs)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return OUT


if __name__ == "__main__":
    print(build(debug="--debug" in sys.argv))
