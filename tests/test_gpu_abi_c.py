"""A C program calls the GPU entry points of include/bpperm.h directly
(tests/c/abi_gpu.c: bpp_ctx_create, bpp_gens_create, bpp_msm,
bpp_vec_commit, bpp_ipa_prove / bpp_ipa_verify, bpp_perm_prove_batch_entropy
/ bpp_perm_verify_batch) -- the boundary as a Rust `extern "C"` shim would
use it, with no ctypes layer in between.  Expected values:
tests/golden/msm.json, tests/golden/protocol.json config2, and the oracle's
permutation proofs (k = 4) from 32-byte seeds (oracle/bulletproofs.py ac_prove).
Reference call sites: circuit_lib.rs:187-229 (commitments), :478-585
(verify); the IPA is bulletproofs 4.0.0's."""
import hashlib
import json
import shutil
import subprocess
from pathlib import Path

import pytest

from oracle import bulletproofs as bp, ristretto as r255

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
L = r255.L


def _inputs(path: Path, k: int = 52):
    cases = json.loads((ROOT / "tests" / "golden" / "msm.json").read_text())["cases"]
    gold = json.loads((ROOT / "tests" / "golden" / "protocol.json").read_text())["config2"]
    lines = []
    for n in (64, 1024):
        c = next(c for c in cases if c["n"] == n)
        lines += [f"msm{n}_scalars {c['scalars']}", f"msm{n}_points {c['points']}", f"msm{n}_result {c['result']}"]
    n, seed = gold["n"], gold["seed"]
    xof = hashlib.shake_256(b"config2" + seed.to_bytes(8, "little")).digest((2 * n + 1) * 64 + 64)
    wide = [int.from_bytes(xof[64 * i: 64 * i + 64], "little") % L for i in range(2 * n + 1)]
    aL, aR, alpha = wide[:n], wide[n:2 * n], wide[2 * n]
    sb = lambda x: r255.scalar_bytes(x).hex()  # noqa: E731
    # the caller's scalar algebra: y from the same Merlin transcript, y^-i
    from oracle.merlin import Transcript
    tr = Transcript(b"config2")
    tr.append_point(b"A", bytes.fromhex(gold["A"]))
    y = tr.challenge_scalar(b"y")
    yi = pow(y, -1, L)
    hf = [pow(yi, i, L) for i in range(n)]
    cab = sum(x * z for x, z in zip(aL, aR)) % L
    psc = aL + [(x * h) % L for x, h in zip(aR, hf)] + [cab]
    lines += [f"c2_n {n.to_bytes(4, 'little').hex()}", "c2_aL " + "".join(sb(x) for x in aL),
              "c2_aR " + "".join(sb(x) for x in aR), f"c2_alpha {sb(alpha)}",
              f"c2_q64 {xof[(2 * n + 1) * 64:].hex()}", f"c2_A {gold['A']}", f"c2_y {sb(y)}",
              "c2_hf " + "".join(sb(x) for x in hf), "c2_L " + "".join(gold["L"]), "c2_R " + "".join(gold["R"]),
              f"c2_a {gold['a']}", f"c2_b {gold['b']}", "c2_P_scalars " + "".join(sb(x) for x in psc)]
    seeds = [hashlib.sha256(b"abi-gpu-%d" % i).digest() for i in range(2)]
    proofs, Vs = [], []
    for s in seeds:
        pf, _ = bp.ac_prove(k, s)
        proofs.append(pf.to_bytes())
        Vs.append(b"".join(pf.V))
    lines += [f"perm_k {k.to_bytes(4, 'little').hex()}", "perm_seeds32 " + b"".join(seeds).hex(),
              "perm_proofs " + b"".join(proofs).hex(), "perm_V " + b"".join(Vs).hex()]
    path.write_text("\n".join(lines) + "\n")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not installed")
def test_c_caller_gpu_entry_points(tmp_path):
    from bpperm import _lib
    libdir = _lib.LIB_PATH.parent
    exe = tmp_path / "abi_gpu"
    cmd = ["gcc", "-std=c11", "-O1", "-Wall", "-Werror", "-I", str(ROOT / "include"),
           str(ROOT / "tests" / "c" / "abi_gpu.c"), "-o", str(exe), f"-L{libdir}", "-lbpperm",
           f"-Wl,-rpath,{libdir}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    inp = tmp_path / "inputs.txt"
    _inputs(inp, k=4)
    r = subprocess.run([str(exe), str(inp)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip() == "ok"
