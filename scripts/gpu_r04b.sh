#!/bin/bash
# Headline parity diagnosis: current library, one wave per problem (CMPC_QP_PAIR=0), round-3 library.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 python scripts/diag_headline.py cur > gpurun_out/diag_cur.log 2>&1 || { tail -20 gpurun_out/diag_cur.log; exit 1; }
cat gpurun_out/diag_cur.log
CMPC_QP_PAIR=0 timeout -k 10 200 python scripts/diag_headline.py onewave > gpurun_out/diag_onewave.log 2>&1 || { tail -20 gpurun_out/diag_onewave.log; exit 1; }
cat gpurun_out/diag_onewave.log
CMPC_LIB_VARIANT=r03 timeout -k 10 200 python scripts/diag_headline.py r03 > gpurun_out/diag_r03.log 2>&1 || { tail -20 gpurun_out/diag_r03.log; exit 1; }
cat gpurun_out/diag_r03.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_qp_pair.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_pair.log 2>&1 || { tail -40 gpurun_out/pytest_pair.log; exit 1; }
tail -2 gpurun_out/pytest_pair.log
bash scripts/gpu_ab.sh r03 || exit 1
