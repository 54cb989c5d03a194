#!/bin/bash
# finish phase stamps of the table-divsteps builds (PBFT_FIN_STAMPS), 131k and 262k
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
PBFT_KEY_TABLE_BUDGET_MB=20000 timeout -k 10 300 python tools/ab.py ${1:-build/ab/libpbft_tabst.so build/ab/libpbft_tabfm2st.so} --sizes ${2:-131072,262144} --rounds 6 > gpurun_out/ab_st.log 2>&1; rc=$?
grep -E "N=|stamps|Error|error" gpurun_out/ab_st.log; exit $rc
