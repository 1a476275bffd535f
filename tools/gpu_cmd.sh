set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05vs; mkdir -p $O
for rep in 1 2; do for vs in 4 6 8; do
  timeout -k 10 300 python bench.py --no-cpu --proofs-per-gpu 0 --no-extra --steps 10 --verify-streams $vs > $O/bv.json 2> $O/bv.err || { tail $O/bv.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bv.json'));v=d['verify_batch'];print('streams=$vs',{k:round(x['ms_per_batch'],3) for k,x in v['splits'].items()}, round(v['value']/1e6,3), v['rejects_tampered'])"
done; done 2>&1 | tee $O/ab.txt
