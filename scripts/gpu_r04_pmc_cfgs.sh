#!/bin/bash
# Round 4: PMC HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes, steady state after two
# warm-up launches) of BASELINE C4 (TALOS N=200 x 512) and the 8-GPU shard (trot N=100 x 128).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export CMPC_HEAD=${CMPC_HEAD:-?}
pmc() {   # pmc <name> <counter> <bench args>
    local name=$1 ctr=$2; shift 2
    timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_r04f_$name -o pmc -- \
        python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-extras "$@" > gpurun_out/pmc_bench_r04f_$name.log 2>&1 \
        || { tail -20 gpurun_out/pmc_bench_r04f_$name.log; return 1; }
}
pmc C4_FETCH_SIZE FETCH_SIZE --config talos --N 200 --batch 512 || exit 1
pmc C4_WRITE_SIZE WRITE_SIZE --config talos --N 200 --batch 512 || exit 1
pmc S128_FETCH_SIZE FETCH_SIZE --batch 128 || exit 1
pmc S128_WRITE_SIZE WRITE_SIZE --batch 128 || exit 1
export PMC_BENCH_CMD="python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-extras --config talos --N 200 --batch 512"
python3 scripts/pmc_traffic.py gpurun_out/pmc_r04f_C4_FETCH_SIZE gpurun_out/pmc_r04f_C4_WRITE_SIZE gpurun_out/qp_pmc_traffic_c4_r04f.json || exit 1
export PMC_BENCH_CMD="python3 bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-extras --batch 128"
python3 scripts/pmc_traffic.py gpurun_out/pmc_r04f_S128_FETCH_SIZE gpurun_out/pmc_r04f_S128_WRITE_SIZE gpurun_out/qp_pmc_traffic_s128_r04f.json || exit 1
grep -h '"hbm_bytes_per_launch"\|"kernel"' gpurun_out/qp_pmc_traffic_c4_r04f.json gpurun_out/qp_pmc_traffic_s128_r04f.json
