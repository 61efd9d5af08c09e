#!/bin/bash
# A/B of library builds (tools/ab_build.sh) on bench.py (value + decode / encode legs),
# alternating variants ROUNDS times.  VARIANTS="base x y" bash tools/ab_bench.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/abb
for r in $(seq ${ROUNDS:-2}); do
for v in ${VARIANTS:-base cur}; do
  if [ $v = cur ]; then unset SSTC_LIB_PATH; else export SSTC_LIB_PATH=$PWD/lsm-kv-storage_amd/lib/ab/$v/libsstcodec.so; fi
  timeout -k 10 300 python bench.py --steps 40 --no-cpu-baseline --no-e2e --no-hbm-variant > gpurun_out/abb/b$v$r.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/abb/b$v$r.log; exit 4; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/abb/b$v$r.log').read().strip().splitlines()[-1]); L=d['legs']
print('$v run $r value', d['value'], 'rt frac', d['roofline']['frac'], 'decode ms', L['decode']['ms'], 'encode ms', L['encode']['ms'], 'verified', L['encode']['verified'])"
done
done
