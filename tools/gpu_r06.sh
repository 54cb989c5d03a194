#!/bin/bash
# r06 GPU step: replica GPU tests, the changed verify tests, the ingress probe, the finish stamps at the 131k shard.
# usage: tools/gpu_r06.sh TAG [steps...]   steps: replica verify ingress finstamps (default: all)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-run}; shift; D=gpurun_out/r06_$TAG; mkdir -p $D
STEPS=${@:-replica verify ingress finstamps}
for s in $STEPS; do
  case $s in
    replica) timeout -k 10 480 python -u -m pytest tests/test_gpu_replica.py -x -v --timeout 300 --timeout-method thread > $D/replica_tests.log 2>&1 ;;
    verify) timeout -k 10 400 python -u -m pytest tests/test_gpu_verify.py -x -v -k "prio_match or staged_and_pageable or update_keys" --timeout 300 --timeout-method thread > $D/verify_tests.log 2>&1 ;;
    gputests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/gpu_tests.log 2>&1 ;;
    ingress) timeout -k 10 480 python -u tools/ingress_probe.py > $D/ingress.json 2> $D/ingress.err ;;
    finstamps) echo "finstamps: build/ab variants are gpurun-ignored since r06 (rebuild with tools/build_variant.sh and drop ./build/ab from .gpurunignore)"; false ;;
    bench) timeout -k 10 600 python -u bench.py > $D/bench.json 2> $D/bench.err ;;
    finvar) timeout -k 10 400 python -u tools/ab.py build/ab/libpbft_finbase.so build/ab/libpbft_finpre.so build/ab/libpbft_findpp.so build/ab/libpbft_finpar.so build/ab/libpbft_finboth.so --replicas 16 --seqs 32768 --sizes 131072,1048576 --rounds 8 --iters 20 > $D/finvar.txt 2>&1 ;;
    step) timeout -k 10 120 tools/microbench/step_study > $D/step_study.txt 2>&1 ;;
    hostinfo) { nproc; cat /sys/fs/cgroup/cpu.max; python -c "import os; print(len(os.sched_getaffinity(0)))"; grep -m1 "model name" /proc/cpuinfo; for n in /sys/devices/system/node/node*; do echo "$n $(cat $n/cpulist)"; grep -E "MemTotal|MemFree" $n/meminfo; done; cat /sys/class/drm/card*/device/numa_node 2>/dev/null | head -3; cat /sys/kernel/mm/transparent_hugepage/enabled; cat /proc/sys/kernel/numa_balancing; } > $D/hostinfo.txt 2>&1; true ;;
    threads) timeout -k 10 400 python -u tools/ingress_probe.py --skip-ingress-leg --rounds 36 --flush-ab PBFT_REPLICA_THREADS=16,15,12,8 > $D/threads.json 2> $D/threads.err ;;
    hostbw) timeout -k 10 120 tools/microbench/host_bw > $D/host_bw.txt 2>&1 ;;
    tail) timeout -k 10 400 python -u tools/ingress_probe.py --skip-ingress-leg --rounds 40 > $D/tail.json 2> $D/tail.err ;;
    tasksab) timeout -k 10 400 python -u tools/ingress_probe.py --skip-ingress-leg --rounds 40 --flush-ab PBFT_PUSH_TASKS=1,8,4,16 > $D/tasksab.json 2> $D/tasksab.err ;;
    partialab) timeout -k 10 400 python -u tools/ingress_probe.py --skip-ingress-leg --rounds 40 --flush-ab PBFT_ADOPT_PARTIAL=0,1 > $D/partialab.json 2> $D/partialab.err ;;
    dppab) timeout -k 10 400 python -u tools/ab.py build/ab/libpbft_finbase.so build/ab/libpbft_findpp.so --replicas 16 --seqs 32768 --sizes 131072 --rounds 24 --iters 20 > $D/dppab.txt 2>&1 ;;
    timeline) timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D/tl -o tl -- python3 tools/ingress_probe.py --skip-ingress-leg --rounds 4 > $D/timeline.out 2>&1 ;;
    pieceab) timeout -k 10 400 python -u tools/ingress_probe.py --skip-ingress-leg --rounds 40 --flush-ab PBFT_MANY_PIECE=131072,262144 > $D/pieceab.json 2> $D/pieceab.err ;;
    benchprof) timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $D/benchprof -o bench -- python3 bench.py > $D/benchprof.json 2> $D/benchprof.err && rm -f $D/benchprof/bench_kernel_trace.csv ;;
    heat) timeout -k 10 300 python -u tools/replica_heat_probe.py > $D/heat.json 2> $D/heat.err ;;
    replonly) timeout -k 10 300 python -u bench.py --replica-only --no-cpu > $D/replonly.json 2> $D/replonly.err ;;
    pfab) timeout -k 10 400 python -u tools/ingress_probe.py --skip-ingress-leg --rounds 40 --flush-ab PBFT_APPLY_PREFETCH=1,2,4,0 > $D/pfab.json 2> $D/pfab.err ;;
    hostprof) rm -f $D/ingress_samples.txt; PBFT_INGRESS_PROFILE=$PWD/$D/ingress_samples.txt timeout -k 10 480 python -u tools/ingress_probe.py --skip-flush-leg > $D/hostprof.json 2> $D/hostprof.err && timeout -k 10 300 python tools/ingress_profile.py $D/ingress_samples.txt > $D/ingress_profile.txt 2>&1 ;;
    ntab) for k in 1 0 1 0; do PBFT_STREAM_STORES=$k timeout -k 10 480 python -u tools/ingress_probe.py --modes records_64 > $D/nt_$k.$RANDOM.json 2>> $D/ntab.err || exit 1; done ;;
    numaab) for k in 0 1 0 1 0 1 0 1; do PBFT_NUMA_BIND=$k timeout -k 10 300 python -u tools/ingress_probe.py --skip-ingress-leg --rounds 20 > $D/numa_$k.$RANDOM.json 2>> $D/numaab.err || exit 1; done ;;
    pmu) timeout -k 10 30 tools/microbench/pmu_probe > $D/pmu.txt 2>&1; true ;;
    smoke) timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 ;;
  esac
  rc=$?
  echo "step $s rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $D/*.log $D/*.err 2>/dev/null | tail -20; exit $rc; }
done
exit 0
