# Prover regime studies (one GPU call each).  Usage on the box:
#   bash tools/gpu_prover_study.sh MODE [TAG]
#   phases      per-phase wall time of one batch (8 pool threads), 1 and 8 in flight
#   batch       phase breakdown at B = 128 / 512 and proofs/s over B x in flight
#   hostcpu     one batch with ONE host thread (host-only phases = CPU time)
#   sensitivity timing-only variants ipanw / bothnw / burn20 (build them first:
#               build.py --variant ipanw -D EXP_IPA_NOWALK; bothnw adds
#               -D EXP_DT_NOWALK; burn20 -D EXP_HOST_BURN_US=20)
#   syncwait    hardware queues 4 vs 8, pool 8 vs 16 threads
#   gaps        kernel + copy timeline of warm 128-proof batches
#               (tools/trace_gaps.py reads it)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp SHARED_GENS=1
MODE=${1:?mode}
OUT=gpurun_out/${2:-study_$MODE}
mkdir -p $OUT
case $MODE in
phases)
  PHASES=1 timeout -k 10 120 python tools/prove_inflight_exp.py 128 1 8 || exit 1
  PHASES=1 timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 16 || exit 1 ;;
batch)
  for B in 128 512; do timeout -k 10 120 python tools/prove_phases.py $B 4 || exit 1; done
  for bt in "128 8 12" "256 4 8" "256 8 6" "512 2 6" "512 4 4" "1024 2 3"; do
    set -- $bt; timeout -k 10 120 python tools/prove_inflight_exp.py $1 $2 $3 || exit 1
  done ;;
hostcpu)
  BPP_HOST_THREADS=1 BPP_POOL_SPIN_US=0 timeout -k 10 120 python tools/prove_phases.py 128 4 || exit 1
  for sp in 300 0; do echo -n "spin=$sp "; BPP_POOL_SPIN_US=$sp timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 12 || exit 1; done ;;
sensitivity)
  B=128 T=12 bash tools/ab.sh prove LIB=default LIB=ipanw LIB=bothnw LIB=burn20 || exit 1 ;;
gaps)
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT -o run --output-format csv -- python3 tools/prove_phases.py 128 3 > $OUT/log.txt 2>&1 || exit 1
  python3 tools/trace_gaps.py $OUT ;;
syncwait)
  for rep in 1 2; do for cfg in "4 8" "8 8" "4 16"; do set -- $cfg
    echo -n "hwq=$1 threads=$2 "; GPU_MAX_HW_QUEUES=$1 BPP_HOST_THREADS=$2 timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 12 || exit 1
  done; done ;;
*) echo "unknown mode $MODE"; exit 2 ;;
esac
