#!/bin/bash
# A/B of the encode offsets (SSTC_ENCOFF unset/1: block sums + block scan + P per block, 3: one pass with LDS-staged sizes)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/abe
SSTC_ENCOFF=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_table.py tests/test_gpu_cpp_boundary.py tests/test_abi.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abe/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/abe/pytest.log; exit 3; }
tail -1 gpurun_out/abe/pytest.log
for r in 1 2; do
for v in 1 3; do
  SSTC_ENCOFF=$v timeout -k 10 120 python tools/ab_enc_big.py > gpurun_out/abe/z$v$r.log 2>&1 || { echo "zipf failed"; tail -5 gpurun_out/abe/z$v$r.log; exit 5; }
  echo "zipf encode v=$v: $(tail -1 gpurun_out/abe/z$v$r.log)"
  SSTC_ENCOFF=$v timeout -k 10 300 python bench.py --steps 40 --no-cpu-baseline --no-e2e --no-hbm-variant > gpurun_out/abe/b$v$r.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/abe/b$v$r.log; exit 4; }
  echo "== SSTC_ENCOFF=$v run $r"; python3 -c "
import json; d=json.loads(open('gpurun_out/abe/b$v$r.log').read().strip().splitlines()[-1]); e=d['legs']['encode']; print({k: e[k] for k in e if k not in ('roofline',)}, e['roofline'].get('frac'))"
done
done
