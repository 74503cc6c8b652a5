#!/bin/bash
# the box's NUMA layout and the GPU's node (for the multi-rank host-memory placement question)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/numa
{
  echo "== nodes"; ls -d /sys/devices/system/node/node* 2>/dev/null
  for n in /sys/devices/system/node/node*; do echo "$n cpus: $(cat $n/cpulist 2>/dev/null) mem: $(grep MemTotal $n/meminfo 2>/dev/null)"; done
  echo "== gpu numa"; for c in /sys/class/drm/card*/device/numa_node; do echo "$c: $(cat $c)"; done
  echo "== affinity"; python3 -c "import os; a=sorted(os.sched_getaffinity(0)); print(len(a), a[:4], a[-4:])"
  echo "== cpu.max"; cat /sys/fs/cgroup/cpu.max 2>/dev/null
  echo "== lscpu"; lscpu 2>/dev/null | head -30
} > gpurun_out/numa/info.txt 2>&1
python3 -c "
import ctypes, sys
sys.path.insert(0, 'genome-assembly-using-overlap-graphs_amd')
import torch
print('pci', torch.cuda.get_device_properties(0))
" >> gpurun_out/numa/info.txt 2>&1
true
