#!/bin/bash
# r02 profiles: PMC passes of the headline command + kernel-trace stats of the same command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_pmc_cur.sh > gpurun_out/pmc.log 2>&1; rc=$?; tail -45 gpurun_out/pmc.log
[ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --no-extras > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { echo "rocprof failed"; tail -30 gpurun_out/prof.err; exit 1; }
cat gpurun_out/prof_bench.json
cut -c1-160 gpurun_out/prof/run_kernel_stats.csv
