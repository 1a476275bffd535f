# Kernel traces of one B-proof batch (default 256) (tools/prove_batch_once.py) for
# library variants.  Usage: bash tools/gpu_trace_ab.sh TAG default VARIANT ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
for v in "$@"; do
  if [ "$v" = default ]; then lib=""; else lib="bulletproof-perm_amd/bpperm/variants/libbpperm_$v.so"; fi
  BPP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/$v -o run --output-format csv -- python3 tools/prove_batch_once.py ${B:-256} > gpurun_out/$TAG/$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
  echo "== $v"; python3 tools/kstats.py -n 16 gpurun_out/$TAG/$v/run_kernel_stats.csv
done
