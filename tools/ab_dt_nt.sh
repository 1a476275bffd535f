cd $GRAFT_REPO_ROOT
for nt in 64 128 256 512; do BPP_DT_NT=$nt BPP_PROVE_STREAMS=1 timeout -k 10 120 python tools/pb_threads.py 128 2>&1 | head -1 | sed "s/^/nt=$nt /"; done
