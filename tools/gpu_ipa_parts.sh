# round 6: where a config-2 round's ~50 us go -- the split round with the walk + tree (default), without the tree (notree), without both (nowalk); timing only
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06parts; mkdir -p $O
for v in default notree nowalk; do
  ( [ $v != default ] && export BPP_LIB=bulletproof-perm_amd/bpperm/variants/libbpperm_$v.so
    timeout -k 10 200 rocprofv3 --kernel-trace -d $O/$v -o run --output-format csv -- python3 tools/config2_once.py 5 > $O/${v}_log.txt 2>&1 ) || { tail $O/${v}_log.txt; exit 1; }
  python3 - "$O/$v" "$v" <<'PY'
import csv, sys
d = [float(r["End_Timestamp"]) - float(r["Start_Timestamp"]) for r in csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv")) if "k_ipa_round_dt" in r["Kernel_Name"]]
d = d[-50:]
print(sys.argv[2], "k_ipa_round_dt launches", len(d), "mean %.1f us" % (sum(d) / len(d) / 1e3))
PY
done | tee $O/parts.txt
