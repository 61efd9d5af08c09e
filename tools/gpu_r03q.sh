#!/bin/bash
# filter A/B: rows per tile (8 / 4) x tile order (ticket / blockIdx)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
CONFIGS="3 4" VARIANTS="cur r4 r4b r8b cur r4 r4b r8b" KERNELS="filter" bash tools/ab_lib.sh || exit 4
