#!/bin/bash
# bench legs (round trip, decode, encode, 1 GiB variant) for library variants:
#   VARIANTS="head cur" ROUNDS=2 bash tools/ab_bench_legs.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/abl_legs
for r in $(seq ${ROUNDS:-2}); do
for v in ${VARIANTS:-head cur}; do
  if [ $v = cur ]; then unset SSTC_LIB_PATH; else export SSTC_LIB_PATH=$PWD/lsm-kv-storage_amd/lib/ab/$v/libsstcodec.so; fi
  timeout -k 10 300 python3 bench.py --steps 20 --no-e2e --no-cpu-baseline --no-compact > gpurun_out/abl_legs/$v.$r.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/abl_legs/$v.$r.log; exit 4; }
  python3 - gpurun_out/abl_legs/$v.$r.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
L = d["legs"]
print(f"{sys.argv[2]:8s} rt {d['roofline']['launch_ms_events']:.4f} ms frac {d['roofline']['frac']:.4f} | 1GiB {d['roofline']['hbm_1gib']['launch_ms_events']:.4f} frac {d['roofline']['hbm_1gib']['frac']:.4f} | decode {L['decode']['ms']:.4f} frac {L['decode']['roofline']['frac']:.4f} | encode {L['encode']['ms']:.4f} frac {L['encode']['roofline']['frac']:.4f}")
PY
done
done
