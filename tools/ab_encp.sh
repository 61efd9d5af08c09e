#!/bin/bash
# A/B of the records -> blocks entry offsets: scanned in the block's wave
# (default) vs the P pass (SSTC_ENC_P=1)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/abp
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_table.py tests/test_gpu_cpp_boundary.py tests/test_gpu_streams.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abp/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/abp/pytest.log; exit 3; }
tail -1 gpurun_out/abp/pytest.log
for r in 1 2; do
for v in 0 1; do
  if [ $v = 1 ]; then export SSTC_ENC_P=1; else unset SSTC_ENC_P; fi
  timeout -k 10 120 python tools/ab_enc_big.py > gpurun_out/abp/z$v$r.log 2>&1 || { echo "zipf failed"; tail -5 gpurun_out/abp/z$v$r.log; exit 5; }
  echo "zipf encode P=$v: $(tail -1 gpurun_out/abp/z$v$r.log)"
  timeout -k 10 300 python bench.py --steps 40 --no-cpu-baseline --no-e2e --no-hbm-variant > gpurun_out/abp/b$v$r.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/abp/b$v$r.log; exit 4; }
  echo "== P=$v run $r"; python3 -c "
import json; d=json.loads(open('gpurun_out/abp/b$v$r.log').read().strip().splitlines()[-1]); e=d['legs']['encode']; print(e['ms'], e['roofline'].get('frac'), d['value'])"
done
done
for v in 0 1; do
  if [ $v = 1 ]; then export SSTC_ENC_P=1; else unset SSTC_ENC_P; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abp/trace$v -o trace --output-format csv -- python3 bench.py --steps 20 --no-cpu-baseline --no-e2e --no-hbm-variant > gpurun_out/abp/trace$v.log 2>&1 || { echo "trace failed"; exit 6; }
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/abp/trace$v/trace_kernel_stats.csv')):
    if 'enc' in r['Name'] or 'scan' in r['Name']: print('P=$v', r['Name'][:50], r['Calls'], r['AverageNs'], r['MinNs'])"
done
