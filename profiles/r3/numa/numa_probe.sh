#!/bin/bash
# NUMA layout of the GPU box: the GPU's node, node CPU lists, distances, memory per node.
for c in /sys/class/drm/card*/device; do echo "$c vendor=$(cat $c/vendor 2>/dev/null) numa=$(cat $c/numa_node 2>/dev/null) bdf=$(basename $(readlink -f $c))"; done
for n in /sys/devices/system/node/node*; do echo "$(basename $n) cpus=$(cat $n/cpulist) dist=$(cat $n/distance) mem=$(grep MemTotal $n/meminfo | awk '{print $4,$5}')"; done
echo "affinity: $(python3 -c 'import os; a=sorted(os.sched_getaffinity(0)); print(len(a), a[:4], a[-4:])')"
lscpu | grep -iE "socket|numa|thread|core|L3" | head -12
