#!/bin/bash
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 scripts/pair_diag.py > gpurun_out/pair_diag.log 2>&1; rc=$?
cat gpurun_out/pair_diag.log; exit $rc
