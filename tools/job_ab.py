"""Config-4 job shape study (one GPU): bench.py's job leg (1024 proofs proved
+ batch-verified) for several sub-batch sizes and job sizes, printed one line
per configuration.  The per-rank job of an N-GPU run is the 1024 / N-proof
job here plus the partial exchange.
    python tools/job_ab.py "1024:32,1024:64,1024:128,128:64" """
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for spec in sys.argv[1].split(","):
    tot, jb = spec.split(":")
    cmd = [sys.executable, str(ROOT / "bench.py"), "--no-cpu", "--steps", "2", "--warmup", "1", "--proof-steps", "1",
           "--proofs-per-gpu", "64", "--proof-streams", "32", "--verify-proofs", "0", "--no-extra",
           "--job-proofs", tot, "--job-batch", jb, "--job-reps", "5"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode:
        print(spec, "failed", r.stderr[-500:])
        sys.exit(1)
    j = json.loads(r.stdout.strip().splitlines()[-1])["proofs"]["job"]
    print(f"proofs {tot:>5} batch {jb:>4}: {j['ms_per_job']:.3f} ms per job ({j['value'] / 1e3:.1f} K proofs/s), "
          f"prove {j['prove_ms_rank0']:.3f} verify {j['verify_ms_rank0']:.3f}, {j['sub_batches_in_flight']} in flight, "
          f"ok {j['all_verified']} rejects {j['rejects_tampered']}", flush=True)
