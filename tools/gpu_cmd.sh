set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r05kt; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/new -o run --output-format csv -- python3 tools/prove_batch_once.py 384 > $O/new.log 2>&1 || { tail $O/new.log; exit 1; }
BPP_IPA_LR=0 BPP_PED_DBL=0 BPP_DT_PAIR=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/old -o run --output-format csv -- python3 tools/prove_batch_once.py 384 > $O/old.log 2>&1 || { tail $O/old.log; exit 1; }
for d in new old; do python3 tools/kstats.py -n 14 $(find $O/$d -name "*kernel_stats.csv"); done
