#!/usr/bin/env bash
# Host facts for the CPU baseline: CPU model, nproc, the
# process's CPU affinity and the cgroup CPU quota.
echo "nproc: $(nproc)"
python3 -c 'import os; print("affinity:", len(os.sched_getaffinity(0)))'
lscpu | grep -E "Model name|^CPU\(s\)|Socket|Thread|NUMA node\(s\)" || true
for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpuset.cpus.effective /sys/fs/cgroup/cpu/cpu.cfs_quota_us; do
  [ -r "$f" ] && echo "$f: $(cat $f)"
done
free -g | head -2
