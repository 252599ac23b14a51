#!/bin/bash
# Round 4, first GPU session: smoke, the new headline / hand-over tests, the whole GPU suite, a
# same-box A/B against the round-3 library (CMPC_LIB_VARIANT=r03), the stamp profile and one full
# bench line (no CPU baseline).  Every GPU step is time-limited; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_qp_pair.py -x -v --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_new.log 2>&1 || { tail -40 gpurun_out/pytest_new.log; exit 1; }
tail -2 gpurun_out/pytest_new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash scripts/gpu_ab.sh r03 || exit 1
timeout -k 10 200 python scripts/stamps.py trot 100 1024 > gpurun_out/stamps.log 2>&1 || { tail -20 gpurun_out/stamps.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
