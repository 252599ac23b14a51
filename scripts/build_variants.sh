#!/bin/bash
# Diagnostic variants of the QP kernel (timing experiments only; results may be wrong):
#   libcmpc_x<k>.so built with -DCMPC_STAMPS -DPT_EXP=<k> (schur_pt.hpp).  CPU-side build.
set -e
cd "$(dirname "$0")/../centroidal-mpc_amd/csrc"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wall -Wno-unused-result"
for k in "$@"; do
  /opt/rocm/bin/hipcc $F -DCMPC_STAMPS -DPT_EXP=$k -c qp_ipm.hip -o /tmp/qp_x$k.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC linearize_diag.o linearize_lane.o assemble.o /tmp/qp_x$k.o scp.o contact_plan.o cmpc_api.o comm.o load_qp.o -o ../cmpc/libcmpc_x$k.so -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
