"""The serial C restatement of dalek's MSM (oracle/c, the CPU baseline) agrees
with the Python spec oracle and with the golden vectors."""
import json
from pathlib import Path

import pytest

from oracle import cport, ristretto as r255
from oracle.merlin import Rng

GOLD = json.loads((Path(__file__).parent / "golden" / "msm.json").read_text())["cases"]


@pytest.fixture(scope="module", autouse=True)
def _built():
    cport.build()


@pytest.mark.parametrize("case", GOLD, ids=lambda c: f"n{c['n']}-{c['seed']}")
def test_cport_matches_golden(case):
    pts = bytes.fromhex(case["points"])
    assert cport.from_uniform(bytes.fromhex(case["uniform"])) == pts
    assert cport.msm(bytes.fromhex(case["scalars"]), pts).hex() == case["result"]


@pytest.mark.parametrize("case", [c for c in GOLD if c["n"] <= 64], ids=lambda c: f"n{c['n']}-{c['seed']}")
def test_python_oracle_reproduces_golden(case):
    n = case["n"]
    pts = [r255.decode(bytes.fromhex(case["points"][64 * i: 64 * i + 64])) for i in range(n)]
    sc = [int.from_bytes(bytes.fromhex(case["scalars"][64 * i: 64 * i + 64]), "little") for i in range(n)]
    assert r255.encode(r255.msm(sc, pts)).hex() == case["result"]


def test_cport_straus_pippenger_boundary_consistent():
    rng = Rng(11)
    raw = b"".join(rng.bytes(64) for _ in range(190))
    pts = cport.from_uniform(raw)
    sc = b"".join(r255.scalar_bytes(rng.scalar()) for _ in range(190))
    # 189 terms (Straus) + last term == 190 terms (Pippenger)
    a = cport.msm(sc[: 189 * 32], pts[: 189 * 32])
    b = cport.msm(sc[189 * 32:], pts[189 * 32:])
    s = r255.ed_add(r255.decode(a), r255.decode(b))
    assert r255.encode(s) == cport.msm(sc, pts)


def test_cpu_prover_matches_golden_52_card():
    """The serial C prover (oracle/c/perm_cpu.c: dalek-style MSMs, folding IPA)
    reproduces the committed 52-card proof bytes (config 1, seed 0) — an
    independent second restatement agreeing with the Python oracle."""
    import json
    from pathlib import Path
    g = json.loads((Path(__file__).parent / "golden" / "protocol.json").read_text())["config1"]
    pf, V = cport.cpu_prove(g["k"], g["seed"], g["label"].encode() if isinstance(g["label"], str) else b"bp-perm")
    assert pf.hex() == g["proof"]
    assert [v.hex() for v in V] == g["V"]


@pytest.mark.parametrize("k,seed", [(2, 7), (3, 8), (6, 9)])
def test_cpu_prover_matches_python_oracle(k, seed):
    from oracle import bulletproofs as bp
    want, _ = bp.ac_prove(k, seed)
    pf, V = cport.cpu_prove(k, seed)
    assert pf == want.to_bytes() and V == want.V


def test_cport_threaded_helpers_match_serial():
    """msm_threads / from_uniform_threads (the golden generator's all-cores
    path) equal the serial port."""
    raw = b"".join(Rng(5, b"thr").bytes(64) for _ in range(1))  # seed material
    import hashlib
    raw = hashlib.shake_256(raw).digest(64 * 3000)
    pts = cport.from_uniform(raw)
    assert cport.from_uniform_threads(raw, threads=7) == pts
    sc = b"".join((int.from_bytes(hashlib.sha512(i.to_bytes(4, "little")).digest(), "little") % r255.L)
                  .to_bytes(32, "little") for i in range(3000))
    assert cport.msm_threads(sc, pts, threads=5) == cport.msm(sc, pts)


def test_bench_golden_is_prefix_consistent():
    """tests/golden/bench_msm.json (make_bench_golden.py): the world-1 entry
    of the bench's inputs at a reduced size reproduces from the serial port,
    and the file covers N = 1, 2, 4, 8 with distinct results."""
    import bench
    gold = json.loads((Path(__file__).parent / "golden" / "bench_msm.json").read_text())
    assert gold["log2n"] == 20 and sorted(gold["world"]) == ["1", "2", "4", "8"]
    res = {v["result"] for v in gold["world"].values()} | {v["result2"] for v in gold["world"].values()}
    assert len(res) == 8
    # the generator's own path on a 2^10 slice: threaded == serial
    n = 1 << 10
    pts = cport.from_uniform(bench.synth_point_bytes(n, 3))
    sc = bench.synth_scalars(n, 2)
    assert cport.msm_threads(sc, pts, threads=3) == cport.msm(sc, pts)


def test_cpu_config2_matches_golden():
    """The C port's config 2 (2049-term commitment + folding IPA at n = 1024,
    bench.py's config2 cpu_baseline) reproduces tests/golden/protocol.json
    config2, which the Python oracle generated: A, all 10 L/R pairs, a, b."""
    gold = json.loads((Path(__file__).parent / "golden" / "protocol.json").read_text())["config2"]
    got = cport.cpu_config2(gold["n"], gold["seed"])
    for key in ("A", "L", "R", "a", "b"):
        assert got[key] == gold[key], key
