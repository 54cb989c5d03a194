#!/bin/bash
# round 4: the box's CPU share (affinity, cgroup quota) and the replica timeline at 16 / 15 / 12 / 8 host threads.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"
cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -E "Cpus_allowed_list" /proc/self/status
for t in 16 15 12 8; do
  PBFT_REPLICA_THREADS=$t timeout -k 10 200 python -u tools/replica_probe.py 6 > gpurun_out/probe_t$t.json 2> gpurun_out/probe_t$t.err || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/probe_t$t.json')); print($t, {k: d[k] for k in ('ms_per_round','ms_per_round_min_max','push_many_ms','flush_ms','flush_submit_ms')})"
done
