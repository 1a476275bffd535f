# Host placement of the prover: the GPU's NUMA node and local CPUs, and
# 12-in-flight proofs/s unpinned vs pinned to CPUs of that node.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export SHARED_GENS=1
bus=$(python3 -c "import torch; p=torch.cuda.get_device_properties(0); print('%04x:%02x:%02x.0' % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id))")
dev=/sys/bus/pci/devices/$bus
echo "gpu $bus numa $(cat $dev/numa_node) local $(cat $dev/local_cpulist)"
lscpu | grep -E "^(Socket|NUMA node|Thread|Core|Model name)" || true
local=$(cat $dev/local_cpulist)
first=$(python3 -c "
s='$local'; c=[]
for r in s.split(','):
    a,_,b=r.partition('-'); c+=range(int(a),int(b or a)+1)
print(','.join(map(str,c[:${NC:-24}])))")
echo "pin set $first"
for rep in 1 2 3; do
  echo -n "free:   "; timeout -k 10 120 python tools/prove_inflight_exp.py 128 ${T:-12} 16 || exit 1
  echo -n "pinned: "; timeout -k 10 120 taskset -c $first python tools/prove_inflight_exp.py 128 ${T:-12} 16 || exit 1
done
