# prover throughput: standalone vs with torch loaded vs inside bench.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
echo -n "plain "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 12 || exit 1
echo -n "torch "; WITH_TORCH=1 timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 12 || exit 1
echo -n "torch omp1 "; OMP_NUM_THREADS=1 WITH_TORCH=1 timeout -k 10 120 python tools/prove_inflight_exp.py 128 8 12 || exit 1
timeout -k 10 200 python bench.py --steps 5 --no-cpu --proof-steps 12 > gpurun_out/b_p.json 2> gpurun_out/b_p.err || { tail -5 gpurun_out/b_p.err; exit 1; }
python -c "import json; p=json.load(open('gpurun_out/b_p.json'))['proofs']; print('bench', round(p['value']), round(p['latency_ms_per_batch'],3))"
OMP_NUM_THREADS=1 timeout -k 10 200 python bench.py --steps 5 --no-cpu --proof-steps 12 > gpurun_out/b_p.json 2> gpurun_out/b_p.err || { tail -5 gpurun_out/b_p.err; exit 1; }
python -c "import json; p=json.load(open('gpurun_out/b_p.json'))['proofs']; print('bench omp1', round(p['value']), round(p['latency_ms_per_batch'],3))"
