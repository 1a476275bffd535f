"""Aggregate 52-card proofs/s with T host threads, each driving its own
context (own stream) over batches of B proofs: do batches in flight overlap
one batch's host phases with another's GPU phases?"""
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "bulletproof-perm_amd"))
import os  # noqa: E402

if os.environ.get("WITH_TORCH"):
    import torch
import bpperm  # noqa: E402

if os.environ.get("HOST_TUNING", "1") != "0":  # as bench.py (bpp_host_tuning); HOST_TUNING=0 leaves malloc alone
    bpperm.host_tuning(malloc=True)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
T = int(sys.argv[2]) if len(sys.argv) > 2 else 2
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 6
provers = []
shared = None
for t in range(T):
    ctx = bpperm.Context(0)
    if os.environ.get("SHARED_GENS"):  # one resident generator set for every context
        shared = shared or bpperm.Gens(ctx, 128)
        g = shared
    else:
        g = bpperm.Gens(ctx, 128)
    pr = bpperm.PermProver(g, 52, ctx=ctx)
    pr.prove_batch(list(range(B)))
    pr.prove_batch(list(range(B)))
    provers.append(pr)


def work(t):
    for r in range(reps):
        provers[t].prove_batch(list(range(B * (r + 10 * t), B * (r + 10 * t + 1))))


if os.environ.get("WITH_TORCH"):
    torch.cuda.synchronize()
import resource  # noqa: E402
PHASES = ["pb_rng", "pb_pedersen_V", "pb_pedersen_Vx_witness", "pb_msm_AI_AO_S", "pb_host_poly",
          "pb_pedersen_T_lr", "pb_ipa", "ipa_host", "ipa_msm", "ped_d2h", "msm_direct", "ipa_round_dt", "double_encode"]
if os.environ.get("PHASES"):  # per-phase wall time of a batch under the in-flight load
    for pr in provers:
        pr.ctx.profile(True)
        pr.ctx.profile_reset()
hp = None
if os.environ.get("HOSTPROF"):  # CPU sampling of the timed region (tools/hostprof)
    import ctypes
    hp = ctypes.CDLL(str(ROOT / "tools" / "hostprof" / "libhostprof.so"))
    hp.hp_stop.argtypes = [ctypes.c_char_p]
    hp.hp_stop.restype = ctypes.c_long
    hp.hp_start(2000)
th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
ru0 = resource.getrusage(resource.RUSAGE_SELF)
t0 = time.perf_counter()
for x in th:
    x.start()
for x in th:
    x.join()
el = time.perf_counter() - t0
if hp is not None:
    print("hostprof samples:", hp.hp_stop(os.environ["HOSTPROF"].encode()))
ru1 = resource.getrusage(resource.RUSAGE_SELF)
cpu = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
print(f"B={B} T={T}: {T * reps * B / el:.0f} proofs/s ({el / (T * reps) * 1e3:.3f} ms per batch), "
      f"host CPU {cpu / el:.1f} cores busy, {cpu / (T * reps * B) * 1e6:.1f} us CPU per proof")
if os.environ.get("PHASES"):
    for ph in PHASES:
        tot = 0.0
        for pr in provers:
            try:
                tot += pr.ctx.profile_get(ph)[0]
            except Exception:
                pass
        print(f"  {ph:24s} {tot / (T * reps):8.3f} ms per batch under load")
