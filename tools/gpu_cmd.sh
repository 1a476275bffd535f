set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06g; mkdir -p $O
bash tools/gpu_pmc_prover.sh r06 || exit 1
bash tools/gpu_pmc_prover.sh r06 msm || exit 1
# bench.py's N = 4 path rehearsed: four ranks on the one GPU over gloo
BPP_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29655 bench.py --gpus 4 --steps 4 --warmup 1 --no-cpu --proofs-per-gpu 64 --proof-streams 2 --proof-steps 2 --verify-proofs 512 --verify-steps 1 --job-reps 1 > $O/bench_n4_gloo.json 2> $O/bench_n4_gloo.err || { tail -20 $O/bench_n4_gloo.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_n4_gloo.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['result_ok'], d['msm_2e22']['result_ok'], d['proofs']['job']['all_verified'], d['proofs']['job']['rejects_tampered'], {k: v['all_verified'] for k, v in d['verify_batch']['splits'].items()}, d['verify_batch']['rejects_tampered'])"
