#!/bin/bash
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 scripts/straggler.py trot 100 1024 8 > gpurun_out/pair_model.log 2>&1; rc=$?
cat gpurun_out/pair_model.log; exit $rc
