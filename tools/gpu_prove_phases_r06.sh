# round 6: prover batch phases after the IPA round work (B = 128, 16), the config-4 job, perm parity
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06w; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_perm.py tests/test_gpu_config4.py tests/test_gpu_protocol.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 200 python3 tools/prove_phases.py 128 5 > $O/phases128.txt 2>&1 || { tail $O/phases128.txt; exit 1; }
timeout -k 10 200 python3 tools/prove_phases.py 16 5 > $O/phases16.txt 2>&1 || { tail $O/phases16.txt; exit 1; }
timeout -k 10 200 python3 tools/job_ab.py 1024:0,128:0 2>&1 | tee $O/job.txt
cat $O/phases128.txt $O/phases16.txt
