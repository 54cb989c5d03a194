#!/bin/bash
# Round-2 measurement set on one GPU: parity tests, smoke, bench line, rocprofv3 kernel-trace summary of the
# headline command, kernel split by batch size, then the PMC passes (tools/gpu_pmc_cur.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
grep -cE "PASSED" gpurun_out/pytest_gpu.log; tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cut -c1-400 gpurun_out/bench.json
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --no-extras > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { echo "rocprof failed"; tail -30 gpurun_out/prof.err; exit 1; }
cut -c1-200 gpurun_out/prof_bench.json
cut -c1-160 gpurun_out/prof/run_kernel_stats.csv
rm -rf gpurun_out/prof_sizes
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sizes -o run -- python3 tools/size_probe.py --sizes 4096,131072,1048576 --widths 0 --trees 7 > gpurun_out/sizes.json 2> gpurun_out/sizes.err || { echo "size probe failed"; tail -20 gpurun_out/sizes.err; exit 1; }
cat gpurun_out/sizes.json
bash tools/gpu_pmc_cur.sh
