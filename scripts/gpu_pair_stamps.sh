#!/bin/bash
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 python3 scripts/pair_stamps.py 100 1024 > gpurun_out/pair_stamps.log 2>&1; rc=$?
cat gpurun_out/pair_stamps.log; exit $rc
