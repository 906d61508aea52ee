#!/bin/bash
# Host facts of a GPU box that shape the daemon's behaviour: CPU quota and throttling of this cgroup,
# NUMA balancing, transparent huge pages.
echo "== nproc $(nproc)"; cat /proc/sys/kernel/numa_balancing 2>&1 | sed 's/^/numa_balancing /'
cg=$(awk -F: '$1=="0"{print $3}' /proc/self/cgroup); echo "cgroup $cg"
for d in /sys/fs/cgroup$cg /sys/fs/cgroup; do echo "dir $d"; for f in cpu.max cpu.stat cpu.weight cpuset.cpus.effective memory.max; do echo "-- $f"; cat $d/$f 2>&1 || true; done; done
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag 2>&1
