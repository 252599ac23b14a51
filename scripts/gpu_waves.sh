#!/bin/bash
# Two-wave QP workgroups: the waves test, the GPU suite, then C2 / C4 and the metric config.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_qp_waves.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_waves.log 2>&1 || { tail -40 gpurun_out/pytest_waves.log; exit 1; }
tail -3 gpurun_out/pytest_waves.log
bash scripts/gpu_tests.sh || exit 1
for a in "c2 --config trot --N 100 --batch 256" "c4 --config talos --N 200 --batch 512" "m --config trot --N 100 --batch 1024"; do
    set -- $a; n=$1; shift
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras "$@" > gpurun_out/w_$n.json 2> gpurun_out/w_$n.err || { tail -20 gpurun_out/w_$n.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']), d['phase_ms_per_step'], d['roofline']['frac'])" gpurun_out/w_$n.json
done
