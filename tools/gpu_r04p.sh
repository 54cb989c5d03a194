#!/bin/bash
# round 4: host topology of the box (NUMA nodes, the GPU's node) and the replica round with its threads on the
# GPU's node vs unrestricted.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
cat /sys/devices/system/node/online; for n in /sys/devices/system/node/node*; do echo "$n $(cat $n/cpulist)"; done
python3 - <<'PY'
import glob, os
for d in glob.glob('/sys/class/drm/card*/device'):
    try:
        print(d, 'numa_node', open(d + '/numa_node').read().strip(), os.path.basename(os.path.realpath(d)))
    except OSError:
        pass
print('affinity', sorted(os.sched_getaffinity(0))[:8], '...', len(os.sched_getaffinity(0)))
PY
NODE=$(python3 -c "
import glob
for d in glob.glob('/sys/class/drm/card*/device/numa_node'):
    v = open(d).read().strip()
    if v not in ('-1', ''): print(v); break
")
echo "gpu node: $NODE"
CPUS=$(cat /sys/devices/system/node/node${NODE:-0}/cpulist)
for mode in free node free node; do
  if [ $mode = node ]; then
    timeout -k 10 200 taskset -c $CPUS python -u tools/replica_probe.py 8 > gpurun_out/probe_p_$mode.json 2>/dev/null || exit $?
  else
    timeout -k 10 200 python -u tools/replica_probe.py 8 > gpurun_out/probe_p_$mode.json 2>/dev/null || exit $?
  fi
  python3 -c "import json; d=json.load(open('gpurun_out/probe_p_$mode.json')); print('$mode', {k: round(d[k],3) for k in ('ms_per_round','push_many_ms','flush_ms','flush_submit_ms')})"
done
