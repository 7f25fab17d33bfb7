#!/bin/bash
# The GPU box's CPU / NUMA topology, the visible GPU's NUMA node and PCI bus, and this
# process's CPU / memory masks (round 6: why the host gather pool is bound to the GPU's node;
# profiles/r06/validator/box_topology.txt).  Usage (on the box): bash tools/topo_probe.sh
set -o pipefail
mkdir -p gpurun_out/topo
{
echo "nproc: $(nproc)"; python3 -c "import os; a=os.sched_getaffinity(0); print('affinity', len(a), min(a), max(a))"
lscpu | grep -i "socket\|numa\|model name\|^CPU(s)\|Thread\|Core"
which numactl && numactl -H | head -20
for d in /sys/class/drm/card*/device; do echo "$d numa_node=$(cat $d/numa_node 2>/dev/null) vendor=$(cat $d/vendor 2>/dev/null)"; done
rocm-smi --showbus 2>/dev/null | head -20
cat /proc/self/status | grep -i "cpus_allowed_list\|mems_allowed_list"
echo "OMP=$OMP_NUM_THREADS"
} > gpurun_out/topo/topo.txt 2>&1
cat gpurun_out/topo/topo.txt
