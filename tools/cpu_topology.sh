#!/bin/bash
# The CPUs this process may run on and what they are: the cgroup's CPU quota, the affinity list, and for
# each allowed CPU its core and SMT siblings (so "16 CPUs" can be told apart as 16 cores or 8 cores x 2).
echo "nproc=$(nproc) online=$(cat /sys/devices/system/cpu/online)"
for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpuset.cpus.effective /sys/fs/cgroup/cpu/cpu.cfs_quota_us; do
  [ -r $f ] && echo "$f: $(cat $f)"
done
aff=$(python3 -c "import os; print(','.join(map(str, sorted(os.sched_getaffinity(0)))))")
echo "affinity: $aff"
python3 - <<'PY'
import os
cpus = sorted(os.sched_getaffinity(0))
cores = {}
for c in cpus[:512]:
    base = f"/sys/devices/system/cpu/cpu{c}/topology"
    try:
        core = open(f"{base}/core_id").read().strip()
        pkg = open(f"{base}/physical_package_id").read().strip()
        sib = open(f"{base}/thread_siblings_list").read().strip()
    except OSError:
        continue
    cores.setdefault((pkg, core), []).append(c)
print(f"allowed cpus {len(cpus)}, distinct physical cores among them {len(cores)}")
smt = [v for v in cores.values() if len(v) > 1]
print(f"cores with 2+ allowed SMT siblings: {len(smt)} e.g. {smt[:4]}")
PY
grep -m1 "model name" /proc/cpuinfo
