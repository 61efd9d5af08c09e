"""bench.py's rank path over RCCL on the box's one GPU: torch.distributed.run
with one rank and SSTC_PG_SINGLE=1, so init_ranks builds a real "nccl"
(RCCL) process group with device_id, and the config-4 leg runs its
GpuCompaction rank path (own 128-SST shard built through the flush-path
TableBuilder, one sstc_compact job per step, outputs checked against
config4_rank0) with the barrier, max / sum and all_gather going through
RCCL.  Ranks > 1 need more GPUs than the box has: the driver's scaling run
covers them; tests/test_bench_launch.py covers 2-3 ranks over gloo."""
import json
import os
import socket
import subprocess
import sys

import pytest
from conftest import ROOT

pytestmark = pytest.mark.gpu


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(600)
def test_bench_rank_path_over_rccl_one_gpu():
    env = dict(os.environ, SSTC_PG_SINGLE="1", HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "3", "--warmup", "1", "--blocks", "4096", "--no-cpu-baseline", "--no-e2e",
           "--no-hbm-variant", "--no-legs", "--no-compact", "--no-files-leg", "--c4-steps", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=540, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert "[sstc] process group: nccl, world 1" in r.stderr
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    c4 = line["legs"]["compact_config4"]
    assert c4["n_gpus"] == 1 and len(c4["per_rank"]) == 1
    assert c4["per_rank"][0]["verified_vs_reference"] is True
    assert c4["GiBps_aggregate"] > 0
