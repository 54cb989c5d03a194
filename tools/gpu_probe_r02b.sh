export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/pt.log 2>&1; tail -3 gpurun_out/pt.log
timeout -k 10 300 python3 tools/size_probe.py --sizes 131072,524288,1048576 --widths 4,8,16 > gpurun_out/p13.json 2>gpurun_out/p13.err; cat gpurun_out/p13.json; tail -2 gpurun_out/p13.err
PBFT_KEY_TABLE_BUDGET_MB=100000 timeout -k 10 300 python3 tools/size_probe.py --sizes 131072,1048576 --widths 4,16 > gpurun_out/p14.json 2>gpurun_out/p14.err; cat gpurun_out/p14.json
timeout -k 10 300 python3 tools/size_probe.py --sizes 131072,1048576 --widths 4,16 > gpurun_out/p13b.json 2>gpurun_out/p13b.err; cat gpurun_out/p13b.json
