# Round-4 closing A/B call: the -m gpu suite on the current build, then the
# accumulate micro-changes (default / ACC_NEG_CARRY / + ACC_HEAVY_DIV = the
# former loop) on the 2^20 stream, then the staging copy pool's size on the
# config-5 batch.  Usage (on the box): bash tools/gpu_ab_r04g.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04g
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04g/tests.txt 2>&1 || { tail -30 gpurun_out/r04g/tests.txt; exit 1; }
tail -1 gpurun_out/r04g/tests.txt
STEPS=60 REPS=3 bash tools/ab.sh msm "LIB=default" "LIB=accneg" "LIB=accold" > gpurun_out/r04g/acc_ab.txt 2>&1 || { tail gpurun_out/r04g/acc_ab.txt; exit 1; }
cat gpurun_out/r04g/acc_ab.txt | tail -9
NOTRACE=1 REPS=3 bash tools/verify_ab.sh cp "BPP_COPY_THREADS=8" "BPP_COPY_THREADS=4" > gpurun_out/r04g/cp_ab.txt 2>&1 || { tail gpurun_out/r04g/cp_ab.txt; exit 1; }
echo done
