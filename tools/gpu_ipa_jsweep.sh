# round 6: J (blocks per L/R MSM) and TG sweep for config 2 after the split prologue
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06q; mkdir -p $O
for rep in 1 2; do
for cfg in "J=16" "J=8" "J=32" "J=64" "J=32,TG=8" "J=64,TG=8" "J=32,TG=16"; do
  ( j=${cfg#J=}; j=${j%%,*}; export BPP_IPA_SPLIT=$j
    case $cfg in *TG=*) export BPP_IPA_TG=${cfg##*TG=};; esac
    echo "$cfg: $(timeout -k 10 120 python3 tools/config2_once.py 20 2>/dev/null)" ) || exit 1
done; done | tee $O/c2_jsweep.txt
