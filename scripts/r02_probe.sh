#!/bin/bash
# Round-2 first look: the box's CPU share (nproc, affinity, cgroup quota) and
# the unchanged bench at a >= 1 GB ring of distinct batches vs the 2-batch ring.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
{
  echo "nproc=$(nproc)"
  python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count())'
  cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cgroup v2 cpu.max"
  grep -m1 "model name" /proc/cpuinfo
} > gpurun_out/r02_box.txt 2>&1
cat gpurun_out/r02_box.txt
timeout -k 10 300 python3 bench.py --no-cpu --batches 2 > gpurun_out/r02_b2.log 2>&1 || exit $?
tail -c 400 gpurun_out/r02_b2.log; echo
timeout -k 10 400 python3 bench.py --no-cpu --batches 24 --steps 20 --warmup 3 > gpurun_out/r02_b24.log 2>&1 || exit $?
tail -c 400 gpurun_out/r02_b24.log; echo
