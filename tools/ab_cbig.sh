#!/bin/bash
# A/B of the compaction large-block encode: SSTC_CBIG=0 listed for enc_emit_kernel
# (a workgroup per block), 1 encoded by the enc_lds_kernel<1> wave that met it.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/abb
SSTC_CBIG=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_files.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abb/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/abb/pytest.log; exit 3; }
tail -1 gpurun_out/abb/pytest.log
for c in 5 3; do
for v in 0 1; do
  SSTC_CBIG=$v timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/abb/t$c$v -o trace --output-format csv -- python3 tools/bench_compact.py --config $c --steps 5 --no-ref --no-files > gpurun_out/abb/b$c$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/abb/b$c$v.log; exit 4; }
  echo "== config $c SSTC_CBIG=$v $(grep -o '"device_s_median": [0-9.e-]*' gpurun_out/abb/b$c$v.log) $(grep -o '"matches_reference_fixture": [^]]*' gpurun_out/abb/b$c$v.log)"
  python3 tools/trace_compact.py $(find gpurun_out/abb/t$c$v -name "*kernel_trace.csv" | head -1) | grep -E "enc_|span"
done
done
