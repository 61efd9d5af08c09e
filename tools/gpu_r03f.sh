#!/bin/bash
# round 3: unaligned LDS field access + encode span copies -- parity tests of the
# codec and the compaction job, then A/B against the previous build (lib/ab/head)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r03f
timeout -k 10 900 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_fuzz.py tests/test_gpu_host.py tests/test_gpu_streams.py \
  tests/test_gpu_table.py tests/test_gpu_lookup.py tests/test_gpu_open.py tests/test_gpu_compact.py tests/test_gpu_files.py \
  tests/test_gpu_cpp_boundary.py "tests/test_gpu_configs.py::test_config_full_size_vs_reference" \
  -x -q --timeout 300 --timeout-method thread > gpurun_out/r03f/pytest.log 2>&1 || { tail -30 gpurun_out/r03f/pytest.log; exit 3; }
tail -1 gpurun_out/r03f/pytest.log
VARIANTS="head cur" ROUNDS=2 bash tools/ab_bench_legs.sh || exit 4
VARIANTS="head cur" CONFIGS="3 5" KERNELS="enc_lds|decode" bash tools/ab_lib.sh
