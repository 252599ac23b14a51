#!/bin/bash
# Round 4: per-phase cycle stamps of the one-wave QP (diagnostic build), metric config, unsplit.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
CMPC_QP_SPLIT=0 timeout -k 10 300 python scripts/stamps.py trot 100 1024 1 > gpurun_out/stamps_r04.log 2>&1 || { tail -20 gpurun_out/stamps_r04.log; exit 1; }
cat gpurun_out/stamps_r04.log
