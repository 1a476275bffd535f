# A/B the 2^20 MSM across environment settings: each arg is "NAME:VAR=VAL[,VAR=VAL]" or "NAME:".
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 200 python bench.py --no-cpu --proofs-per-gpu 0 --steps 20 > gpurun_out/abe_$name.json 2> gpurun_out/abe_$name.err ) || { echo "variant $name failed"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/abe_$name.json')); s=d['stage_ms']; print('$name', round(d['ms_per_step'],3), 'ms/MSM', d['result_prefix'], {k: round(x,3) for k,x in s.items()})"
done
