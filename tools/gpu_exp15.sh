# FE_MADC_ASM (opaque mad chains) vs the default on the 2^20 MSM
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
V=bulletproof-perm_amd/bpperm/variants/libbpperm_asm.so
BPP_LIB=$V timeout -k 10 200 python -u -m pytest tests/test_gpu_msm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_asm.txt 2>&1 || { tail -20 gpurun_out/t_asm.txt; exit 1; }
tail -1 gpurun_out/t_asm.txt
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 40 --no-cpu --proofs-per-gpu 0 > gpurun_out/b_ab.json 2> gpurun_out/b_ab.err || { tail -5 gpurun_out/b_ab.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/b_ab.json')); s=d['stage_ms']
print('$label'.ljust(10), 'piped', round(d['ms_per_step'],4), 'lat', round(d['latency_ms_per_msm'],4), 'acc', round(s['msm_accumulate'],4), 'red', round(s['msm_reduce'],4), d['pipelined_matches_serial'], d['result_prefix'])"
}
for pass in 1 2 3; do run base X=0; run asm BPP_LIB=$V; done
