set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py -x -v -m gpu -k "api_edges or async or every_lane or clone or multi_shards or config2" --timeout 300 --timeout-method thread > gpurun_out/pt_r05b.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pt_r05b.log | tail -5; [ $rc -ne 0 ] && exit $rc
PBFT_LAUNCH_TRACE=1000 timeout -k 10 200 python -u tools/stall_probe.py 5 1.0 1 > gpurun_out/stall_r05b_import.log 2>&1 || exit $?
PBFT_LAUNCH_TRACE=1000 timeout -k 10 200 python -u tools/stall_probe.py 5 1.0 0 > gpurun_out/stall_r05b_import_pageable.log 2>&1 || exit $?
PBFT_HOST_IMPORT=0 PBFT_LAUNCH_TRACE=1000 timeout -k 10 200 python -u tools/stall_probe.py 3 1.0 1 > gpurun_out/stall_r05b_copies.log 2>&1 || exit $?
grep -E "^rep|batches|launch-stall" gpurun_out/stall_r05b_*.log
