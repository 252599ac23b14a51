#!/bin/bash
# Same-box A/B of the default library against CMPC_LIB_VARIANT=$1 on the metric config: bench
# lines A, B, A, B (no CPU baseline, no extra legs), so box-to-box clock differences cancel.
# Further arguments go to bench.py (e.g. --config talos --N 200 --batch 512).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
V=${1:-old}
shift
EXTRA="$*"
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras $EXTRA > gpurun_out/bench_a$i.json 2> gpurun_out/bench_a$i.err || { tail -20 gpurun_out/bench_a$i.err; exit 1; }
  CMPC_LIB_VARIANT=$V timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras $EXTRA > gpurun_out/bench_b$i.json 2> gpurun_out/bench_b$i.err || { tail -20 gpurun_out/bench_b$i.err; exit 1; }
done
python - <<'PY'
import json
for t in ('a1', 'b1', 'a2', 'b2'):
    d = json.load(open('gpurun_out/bench_%s.json' % t))
    print(t, round(d['value']), 'qp_ms %.3f' % d['phase_ms_per_step']['qp_ms'], 'ms/step %.3f' % d['ms_per_step'])
PY
