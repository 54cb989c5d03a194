set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/e1.json 2>&1 || exit 1
PBFT_KEY_TABLE_BUDGET_MB=0 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --latency-iters 0 > gpurun_out/e2.json 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/e3 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --latency-iters 0 > gpurun_out/e3.out 2>&1 || exit 1
python3 -c "import json;[print(json.loads(open(f).read().strip().splitlines()[-1])['value'], json.loads(open(f).read().strip().splitlines()[-1])['roofline']['kernel_avg_ms']) for f in ['gpurun_out/e1.json','gpurun_out/e2.json']]"
python3 tools/pmc_summary.py gpurun_out/e3 1048576 3.05
