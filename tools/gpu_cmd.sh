set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05aa; mkdir -p $O
V=bulletproof-perm_amd/bpperm/variants
for rep in 1 2; do for cfg in X=1 BPP_LIB=$V/libbpperm_vs5.so BPP_LIB=$V/libbpperm_vs6.so; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu --proofs-per-gpu 0 --no-extra --steps 10 > $O/bv.json 2> $O/bv.err || { tail $O/bv.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bv.json'));v=d['verify_batch'];print('$cfg'.split('/')[-1].ljust(20),{k:round(x['ms_per_batch'],3) for k,x in v['splits'].items()}, round(v['stage_ms']['verify_scalars'],3), v['rejects_tampered'])"
done; done
