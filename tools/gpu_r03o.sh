#!/bin/bash
# A/B of the mode-1 encode prologue / P0 variants (compaction encode) on configs 3 and 4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
CONFIGS="3 4" VARIANTS="head cur v1 v2 v12 head cur v1 v2 v12" KERNELS="enc_lds" bash tools/ab_lib.sh || exit 4
