set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05t; mkdir -p $O
true
true
for rep in 1 2; do for cfg in BPP_COPY_THREADS=4 BPP_COPY_THREADS=6 BPP_COPY_THREADS=8; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu --proofs-per-gpu 0 --no-extra --steps 10 > $O/bv.json 2> $O/bv.err || { tail $O/bv.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bv.json'));v=d['verify_batch'];h=d['host_scalars'];print('$cfg'.ljust(18),{k:round(x['ms_per_batch'],3) for k,x in v['splits'].items()}, 'upl', round(v['stage_ms']['verify_upload'],3), 'host lat', round(h['latency_host_scalars_ms'],3), 'pipe', round(h['pipelined']['pageable']['vs_resident_pipelined'],3))"
done; done
