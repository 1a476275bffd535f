set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.txt 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 10 > gpurun_out/bench.txt 2>&1 || { echo "bench failed"; exit 1; }
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --no-cpu > gpurun_out/prof_log.txt 2>&1 || { echo "rocprof failed"; exit 1; }
echo done
