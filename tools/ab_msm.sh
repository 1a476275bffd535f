# A/B the 2^20 MSM across library variants (build.py --variant NAME -D ...).
# Usage on the box: bash tools/ab_msm.sh default w5 asm ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ "$v" = default ]; then lib=""; else lib="bulletproof-perm_amd/bpperm/variants/libbpperm_$v.so"; fi
  BPP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --proofs-per-gpu 0 --verify-proofs 0 --steps 20 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "variant $v failed"; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); s=d['stage_ms']; print('$v', d['result_prefix'], d.get('result_ok'), round(d['ms_per_step'],3), 'lat', round(d['latency_ms_per_msm'],3), 'ms/MSM', {k: round(x,3) for k,x in s.items()})"
done
