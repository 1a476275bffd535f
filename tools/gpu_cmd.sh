set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r05d
REPS=3 STEPS=60 bash tools/ab.sh msm "LIB=old" "LIB=sw" "LIB=default" > gpurun_out/r05d/ab.txt 2>&1; cat gpurun_out/r05d/ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "verify or dist or perm or abi or config4 or compat" > gpurun_out/r05d/tests.txt 2>&1 || { tail -40 gpurun_out/r05d/tests.txt; exit 1; }
tail -1 gpurun_out/r05d/tests.txt
timeout -k 10 300 python bench.py --no-cpu --proofs-per-gpu 0 --no-extra --steps 10 > gpurun_out/r05d/bench_v.json 2> gpurun_out/r05d/bench_v.err || { tail gpurun_out/r05d/bench_v.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r05d/bench_v.json'));v=d['verify_batch'];print(v['splits'],v['stage_ms'])"
