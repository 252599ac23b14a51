#!/bin/bash
# Step fraction (fraction-to-boundary) sweep over the metric batch and the BASELINE C4 / C5 /
# C3 batches (Newton steps, statuses, QP time), plus the new contact-plan GPU test.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_contact_plans.py tests/test_gpu_gusto.py -q --timeout 200 --timeout-method thread > gpurun_out/pt_small.log 2>&1 || { tail -30 gpurun_out/pt_small.log; exit 1; }
tail -1 gpurun_out/pt_small.log
timeout -k 10 200 python scripts/qp_exits.py trot 100 1024 2 fp64 eta=0.995 eta=0.998 eta=0.999 > gpurun_out/eta_trot.log 2>&1 &&
timeout -k 10 300 python scripts/qp_exits.py talos 200 512 2 fp64 eta=0.995 eta=0.998 eta=0.999 > gpurun_out/eta_talos.log 2>&1 &&
timeout -k 10 200 python scripts/qp_exits.py mixed 150 1024 1 fp64 eta=0.995 eta=0.998 eta=0.999 > gpurun_out/eta_mixed.log 2>&1 &&
timeout -k 10 200 python scripts/qp_exits.py bound 100 1024 1 fp32 eta=0.995 eta=0.998 eta=0.999 > gpurun_out/eta_bound32.log 2>&1
rc=$?
grep -h "^eps\|^iter" gpurun_out/eta_*.log
exit $rc
