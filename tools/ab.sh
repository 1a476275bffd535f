# Interleaved A/B runs on the GPU box: one leg, several configurations.
# Usage (on the box, from the repo root):
#   bash tools/ab.sh LEG "CFG" "CFG" ...
# A CFG is a space-separated list of VAR=VAL settings exported for that run;
# LIB=NAME selects bulletproof-perm_amd/bpperm/variants/libbpperm_NAME.so
# (build.py --variant NAME -D ...; LIB=default = the product library).
# Legs:
#   msm    2^20 MSM stream (bench.py headline leg; STEPS, INFLIGHT)
#   msmv   the same plus the config-5 verification leg
#   full   the whole bench line without CPU baselines
#   prove  in-flight prover proofs/s (tools/prove_inflight_exp.py B T R;
#          B, T, R may be set per CFG: defaults 256 x 16, 16 batches a stream)
#   one    one prover batch alone (prove_inflight_exp.py B 1 8)
# REPS (default 2; 3 for prove) interleaved passes over the CFGs.
# Examples:
#   bash tools/ab.sh msm "LIB=default" "LIB=w2"              (was ab_msm.sh)
#   bash tools/ab.sh msmv "BPP_MSM_LONE_RLOG=2" "BPP_MSM_LONE_RLOG=4"
#   bash tools/ab.sh full "BPP_BENCH_HW_QUEUES=4" "BPP_BENCH_HW_QUEUES=8"   (bench.py sets GPU_MAX_HW_QUEUES from it)
#   bash tools/ab.sh prove "B=256 T=16 BPP_HOST_THREADS=4" "B=384 T=11"
#   bash tools/ab.sh prove "GPU_MAX_HW_QUEUES=8 T=12" "BPP_IPA_DEVICE_MERLIN=1"
#   STEPS=120 bash tools/ab.sh msm "INFLIGHT=3" "INFLIGHT=4 BPP_BENCH_HW_QUEUES=12"
#   bash tools/ab.sh msmv "BENCH_ARGS=--verify-streams=2" "BENCH_ARGS=--verify-streams=3"
# (BENCH_ARGS: extra bench.py arguments, comma-separated)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp SHARED_GENS=1
LEG=$1; shift
[ "$LEG" = prove ] && DEF_REPS=3 || DEF_REPS=2
V=bulletproof-perm_amd/bpperm/variants
summ() {  # bench line -> one summary line
  python3 - "$1" "$2" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); cfg = sys.argv[2]
s = d["stage_ms"]
out = [cfg.ljust(44), "msm %.4f ms" % d["ms_per_step"], "lat %.3f" % d["latency_ms_per_msm"],
       "acc %.3f red %.3f" % (s["msm_accumulate"], s["msm_reduce"]), "ok %s" % d["result_ok"]]
v = d.get("verify_batch")
if v:
    sp = v["splits"]
    out.append("c5 %.3f ms x2 %.3f ms (red %.3f acc %.3f) %s" % (sp["single"]["ms_per_batch"],
               sp.get("streams", {}).get("ms_per_batch", 0), v["stage_ms"]["msm_reduce"],
               v["stage_ms"]["msm_accumulate"], v["rejects_tampered"] and sp["single"]["all_verified"]))
p = d.get("proofs")
if p:
    out.append("proofs %.0f K vb %.0f K" % (p["value"] / 1e3, p["verify_batch_proofs_per_sec"] / 1e3))
hs = d.get("host_scalars")
if hs:
    out.append("host %.2f pinned %.2f" % (hs["pipelined"]["pageable"]["vs_resident_pipelined"],
                                          hs["pipelined"]["pinned"]["vs_resident_pipelined"]))
print(" ".join(out))
EOF
}
for rep in $(seq 1 ${REPS:-$DEF_REPS}); do
for cfg in "$@"; do
  (
    for kv in $cfg; do
      case $kv in
        LIB=default) export BPP_LIB= ;;
        LIB=*) export BPP_LIB=$V/libbpperm_${kv#LIB=}.so ;;
        *) export "$kv" ;;
      esac
    done
    case $LEG in
      msm|msmv|full)
        args="--no-cpu --steps ${STEPS:-20} --warmup ${WARMUP:-2} --inflight ${INFLIGHT:-3}"
        [ $LEG = full ] || args="$args --proofs-per-gpu 0"
        [ $LEG = msm ] && args="$args --verify-proofs 0"
        args="$args --no-extra ${BENCH_ARGS//,/ }"
        timeout -k 10 300 python bench.py $args > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
        summ gpurun_out/ab.json "$cfg" ;;
      prove)
        echo -n "$cfg: "; timeout -k 10 150 python tools/prove_inflight_exp.py ${B:-256} ${T:-16} ${R:-16} 2>/dev/null ;;
      one)
        echo -n "$cfg one batch: "; timeout -k 10 120 python tools/prove_inflight_exp.py ${B:-256} 1 8 2>/dev/null ;;
      *) echo "unknown leg $LEG"; exit 2 ;;
    esac
  ) || exit 1
done; done
