#!/bin/bash
# Host-side facts of the GPU box that bear on the host-buffer stage, then a traced stage run.
echo "nproc $(nproc)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo "cpuset $(cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null)"
echo "affinity $(python3 -c 'import os; s=sorted(os.sched_getaffinity(0)); print(len(s), s[:8], s[-4:])')"
bus=$(rocm-smi --showbus 2>/dev/null | grep -o '[0-9a-f]\{4\}:[0-9a-f]\{2\}:[0-9a-f]\{2\}\.[0-9]' | head -1)
echo "gpu bus $bus local_cpulist $(cat /sys/bus/pci/devices/$bus/local_cpulist 2>/dev/null) numa $(cat /sys/bus/pci/devices/$bus/numa_node 2>/dev/null)"
grep -m1 "model name" /proc/cpuinfo; uptime
