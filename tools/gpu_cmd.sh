set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06e; mkdir -p $O
bash tools/gpu_r06.sh r06e tests bench || exit 1
timeout -k 10 120 python3 tools/prove_phases.py 32 8 > $O/phases32.txt 2>&1 || { tail $O/phases32.txt; exit 1; }
timeout -k 10 120 python3 tools/prove_phases.py 128 8 > $O/phases128.txt 2>&1 || { tail $O/phases128.txt; exit 1; }
cat $O/phases32.txt $O/phases128.txt
