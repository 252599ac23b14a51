set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python scripts/qp_exits.py talos 200 512 2 fp64 1e-11 1e-10 1e-9 1e-8 > gpurun_out/eps_talos.log 2>&1 &&
timeout -k 10 200 python scripts/qp_exits.py trot 100 1024 2 fp64 1e-11 1e-10 1e-9 1e-8 > gpurun_out/eps_trot.log 2>&1 &&
timeout -k 10 200 python scripts/qp_exits.py bound 100 1024 2 fp32 1e-6 1e-5 > gpurun_out/eps_bound32.log 2>&1 &&
timeout -k 10 200 python scripts/qp_exits.py mixed 150 1024 1 fp64 1e-11 1e-9 > gpurun_out/eps_mixed.log 2>&1
cat gpurun_out/eps_*.log
