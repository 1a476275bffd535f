cd $GRAFT_REPO_ROOT
for t in 8 12 16; do for b in 128 512; do BPP_HOST_THREADS=$t BPP_PROVE_STREAMS=1 timeout -k 10 120 python tools/pb_threads.py $b 2>&1 | head -1 | sed "s/^/threads=$t /"; done; done
