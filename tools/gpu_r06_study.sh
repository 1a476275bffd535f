# Round-6 study: MSM parity of the current build, the accumulate A/B, config-4
# job shapes, k_dt_msm pair A/B at the bench's prover shape, and the
# translation / latency counters of the prover's gathers.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06_study; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_msm.py tests/test_gpu_msm_large.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/msm_tests.txt 2>&1 || { tail -30 $O/msm_tests.txt; exit 1; }
tail -1 $O/msm_tests.txt
STEPS=60 INFLIGHT=4 REPS=3 BPP_BENCH_HW_QUEUES=8 timeout -k 10 400 bash tools/ab.sh msm "LIB=default" "LIB=parkold" > $O/acc_park_ab.txt 2>&1 || { tail $O/acc_park_ab.txt; exit 1; }
cat $O/acc_park_ab.txt
timeout -k 10 400 python3 tools/job_ab.py "1024:32,1024:64,1024:128,1024:256,512:64,256:64,128:32,128:64,128:128" > $O/job_ab.txt 2>&1 || { tail $O/job_ab.txt; exit 1; }
cat $O/job_ab.txt
GPU_MAX_HW_QUEUES=8 REPS=3 timeout -k 10 500 bash tools/ab.sh prove "B=384 T=32 R=12 BPP_DT_PAIR=1" "B=384 T=32 R=12 BPP_DT_PAIR=0" > $O/dt_pair_ab.txt 2>&1 || { tail $O/dt_pair_ab.txt; exit 1; }
cat $O/dt_pair_ab.txt
timeout -k 10 600 bash tools/gpu_tlb_prover.sh r06 "BPP_DT_PAIR=1" "BPP_DT_PAIR=0" > $O/tlb.txt 2>&1 || { tail $O/tlb.txt; exit 1; }
python3 tools/tlb_summary.py gpurun_out/tlb_r06 > $O/tlb_prover.json && echo tlb ok
