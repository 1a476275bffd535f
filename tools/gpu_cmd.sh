set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05k; mkdir -p $O
for rep in 1 2; do for cfg in BPP_VERIFY_PIECE_KB=0 X=1 BPP_VERIFY_PIECE_KB=512 BPP_COPY_THREADS=8 "BPP_COPY_THREADS=8 BPP_VERIFY_PIECE_KB=512" BPP_COPY_THREADS=12; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu --proofs-per-gpu 0 --no-extra --steps 10 > $O/bv.json 2> $O/bv.err || { tail $O/bv.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bv.json'));v=d['verify_batch'];print('$cfg'.ljust(44),{k:round(x['ms_per_batch'],3) for k,x in v['splits'].items()}, round(v['stage_ms']['verify_upload'],3))"
done; done
