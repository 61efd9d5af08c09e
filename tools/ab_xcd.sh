#!/bin/bash
# A/B of the XCD-aware block order (SSTC_XCD bit 0: rt_kernel, bit 1: decode +
# enc_lds) on config 3 compaction and the config-2 bench (+ its 1 GiB variant).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_compact.py -q -x > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 3; }
tail -1 gpurun_out/pt.log
cd /tmp
SSTC_XCD=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/ab0 -o t --output-format csv -- python3 $R/tools/bench_compact.py --no-ref --no-files --steps 2 > $R/gpurun_out/ab0.log 2>&1 || exit 4
echo "== compaction XCD=0"; python3 $R/tools/trace_compact.py $(ls $R/gpurun_out/ab0/*kernel_trace.csv) | head -5
SSTC_XCD=2 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/ab2 -o t --output-format csv -- python3 $R/tools/bench_compact.py --no-ref --no-files --steps 2 > $R/gpurun_out/ab2.log 2>&1 || exit 5
echo "== compaction XCD=2"; python3 $R/tools/trace_compact.py $(ls $R/gpurun_out/ab2/*kernel_trace.csv) | head -5
cd $R
for x in 0 1; do
  for nb in 65536 262144; do
    SSTC_XCD=$x timeout -k 10 300 python bench.py --steps 30 --blocks $nb --no-cpu-baseline --no-e2e > gpurun_out/bench_x${x}_${nb}.log 2>&1 || exit 6
    echo "rt XCD=$x blocks=$nb: $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_x${x}_${nb}.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['launch_ms_events'])")"
  done
done
