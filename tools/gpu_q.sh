#!/bin/bash
# tools/gpu.sh, resubmitted while the pool reports no free box (exit 3) or a
# transient preparation failure before anything ran (status "transient",
# rc null); any run of the command itself is never repeated.
# Usage: tools/gpu_q.sh TIMEOUT 'command'
for i in $(seq 1 ${GPU_Q_TRIES:-8}); do
  /root/repo/tools/gpu.sh "$1" "$2"
  rc=$?
  st=$(python3 -c "import json;d=json.load(open('/root/repo/gpurun_out/.last_call.json'));print(d.get('status'), d.get('rc'))" 2>/dev/null)
  if [ $rc -eq 3 ] || [ "$st" = "transient None" ]; then sleep 90; continue; fi
  exit $rc
done
exit 3
