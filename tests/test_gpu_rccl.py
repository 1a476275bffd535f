"""The multi-GPU collective paths over RCCL itself (every
`nccl` branch of bpperm/dist.py and bench.py had only run over gloo): a
world-1 "nccl" process group on the box's one GPU drives bpperm.dist's MSM
window split, the three config-5 splits (the sharded one through
all_gather_into_tensor, the RCCL-only branch of gather_blocks) and the
config-4 job's own-slice verification with device tensors
(tools/rccl_world1.py, in its own process).  A world of 1 exchanges nothing
between GPUs, but every collective is an RCCL call on the device; the N > 1
exchange itself is rehearsed over gloo (test_gpu_bench_dist.py,
test_dist_*_gloo.py).  Reference: circuit_lib.rs:478-585 (verify)."""
import json
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def test_dist_paths_over_rccl_world1():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "rccl_world1.py"), "--port", str(port)],
                       capture_output=True, text=True, timeout=240)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0 and line, r.stdout[-2000:] + r.stderr[-3000:]
    d = json.loads(line[-1])
    assert d["backend"] == "nccl" and d["world"] == 1
    assert d["ok"] is True, d
