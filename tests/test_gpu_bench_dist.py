"""bench.py's own N > 1 path, rehearsed on one GPU before a driver SCALE run
meets it: torch.distributed.run starts two ranks (each its own process, the
launcher started before any GPU call in them) that share cuda:0 and exchange
over gloo (BPP_DIST_BACKEND=gloo stands in for RCCL, which needs one GPU per
rank).  Asserts the 2-rank MSM (2^20 pairs per rank, bucket windows split)
equals the C-port golden for world 2 (tests/golden/bench_msm.json), the
proofs of both ranks verify, and both config-5 splits (windows, proofs)
accept the batch and reject a tampered one; config 5's single 2^22-term MSM
with its windows split over the two ranks equals the world-4 golden; and
config 4 as one job (proofs sharded over the ranks, one batch verification
by the proof split) verifies and refuses a tampered proof."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_gloo(tmp_path):
    env = dict(os.environ, BPP_DIST_BACKEND="gloo", TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(ROOT / "bench.py"),
           "--gpus", "2", "--steps", "4", "--warmup", "1", "--log2n", "20", "--no-cpu",
           "--proofs-per-gpu", "64", "--proof-streams", "2", "--proof-steps", "2",
           "--verify-proofs", "512", "--verify-steps", "1", "--job-proofs", "256", "--job-reps", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["config"]["pairs"] == 2 << 20
    assert d["result_ok"] is True, d["result_prefix"]
    assert d["pipelined_matches_serial"] is True
    assert d["proofs"]["all_verified"] is True and d["proofs"]["n_gpus"] == 2
    v = d["verify_batch"]
    assert set(v["splits"]) == {"windows", "windows_sharded", "proofs"}
    assert all(s["all_verified"] for s in v["splits"].values())
    assert v["rejects_tampered"] is True
    # config 5's one 2^22-term MSM, windows split over the two ranks (strong)
    m = d["msm_2e22"]
    assert m["n_gpus"] == 2 and m["pairs"] == 1 << 22 and m["scaling"] == "strong"
    assert m["result_ok"] is True
    # config 4 as one job: 256 proofs over the two ranks, one batch verification
    j = d["proofs"]["job"]
    assert j["proofs"] == 256 and j["proofs_per_rank"] == 128 and j["n_gpus"] == 2
    assert j["all_verified"] is True and j["rejects_tampered"] is True
