#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 python scripts/stamps.py trot 100 256 > gpurun_out/stamps_c2.log 2>&1 || { tail -20 gpurun_out/stamps_c2.log; exit 1; }
cat gpurun_out/stamps_c2.log
timeout -k 10 200 python scripts/stamps.py talos 200 512 > gpurun_out/stamps_c4.log 2>&1 || { tail -20 gpurun_out/stamps_c4.log; exit 1; }
cat gpurun_out/stamps_c4.log
