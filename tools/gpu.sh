#!/bin/bash
# Build in this container (fail loudly), then run a command on the GPU box.
# Usage: tools/gpu.sh TIMEOUT 'command'
set -o pipefail
cd /root/repo
python bulletproof-perm_amd/build.py > /tmp/bpp_build.log 2>&1 || { tail -20 /tmp/bpp_build.log; echo "BUILD FAILED"; exit 1; }
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
