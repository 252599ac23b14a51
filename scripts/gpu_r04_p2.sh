#!/bin/bash
# Round 4: second polishing attempt one Newton step after a rejected guess.  Headline + split parity
# tests first, then the metric, C2 (polishing 3e-8 default and 1e-7), C5, and the Newton histogram.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_qp_split.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/p2_tests.log 2>&1 || { tail -30 gpurun_out/p2_tests.log; exit 1; }
tail -3 gpurun_out/p2_tests.log
run() {   # run <tag> <env> <bench args...>
    local tag=$1 envv=$2; shift 2
    env $envv timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 "$@" > gpurun_out/p2b_$tag.json 2> gpurun_out/p2b_$tag.err \
        || { tail -5 gpurun_out/p2b_$tag.err; return 1; }
}
run m X=0 || exit 1
run c2 X=0 --batch 256 || exit 1
run c2_1e7 CMPC_QP_POLISH_EPS=1e-7 --batch 256 || exit 1
run c5 X=0 --config mixed --N 150 || exit 1
run s128 X=0 --batch 128 || exit 1
run s128_1e7 CMPC_QP_POLISH_EPS=1e-7 --batch 128 || exit 1
python3 - <<'PY'
import json
for t in ('m', 'c2', 'c2_1e7', 'c5', 's128', 's128_1e7'):
    d = json.load(open('gpurun_out/p2b_%s.json' % t))
    print(t, round(d['value']), d['roofline']['kernel'], 'ms/step %.3f qp_ms %.3f' % (d['ms_per_step'], d['phase_ms_per_step']['qp_ms']),
          'newton %.3f' % d['qp_ipm_iterations_mean'], 'status', d['qp_exit']['status_counts'],
          'merit %.3f' % d['qp_exit']['merit_max'], 'pol +%d -%d' % (d['qp_exit']['polish_accepted'], d['qp_exit']['polish_rejected']),
          'frac %.3f' % d['roofline']['frac'])
PY
timeout -k 10 300 python3 scripts/diag_newton_hist.py > gpurun_out/p2_newton_hist.log 2>&1 || exit 1
cat gpurun_out/p2_newton_hist.log
