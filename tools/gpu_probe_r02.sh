export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/pt.log 2>&1; tail -3 gpurun_out/pt.log
timeout -k 10 300 python tools/ab.py pbft_amd/libpbft_verify.so build/ab/libpbft_finexp.so --sizes 131072,262144,1048576 --rounds 6 > gpurun_out/ab.log 2>&1; cat gpurun_out/ab.log | grep N=
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/probe2 -o run -- python3 tools/size_probe.py --sizes 131072,262144,524288,1048576 > gpurun_out/probe2.json 2>/dev/null; cat gpurun_out/probe2.json
timeout -k 10 300 python3 tools/size_probe.py --split-below 0 --sizes 2048,4096,8192,16384,32768,65536 --widths 1,4 > gpurun_out/probe3.json 2>/dev/null; cat gpurun_out/probe3.json
timeout -k 10 300 python3 tools/size_probe.py --sizes 2048,4096,8192,16384,32768 --widths 4 > gpurun_out/probe4.json 2>/dev/null; cat gpurun_out/probe4.json
