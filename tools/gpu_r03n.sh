#!/bin/bash
# A/B: head (committed) vs cur (encode prologue loads in one round trip, P0 / P[f0+n] with the columns, decode record bases with the DMA)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
VARIANTS="head cur head cur" ROUNDS=1 bash tools/ab_bench_legs.sh || exit 3
CONFIGS="3 4" VARIANTS="head cur head cur" KERNELS="enc_lds|decode" bash tools/ab_lib.sh || exit 4
