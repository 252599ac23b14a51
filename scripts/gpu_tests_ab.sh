#!/bin/bash
# GPU suite on the default build, then the same-box A/B against CMPC_LIB_VARIANT=$1 (scripts/gpu_ab.sh).
set -o pipefail
bash scripts/gpu_tests.sh || exit 1
bash scripts/gpu_ab.sh "${1:-old}"
