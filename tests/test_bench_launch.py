"""CPU: `bench.py --gpus N` launches its own N ranks.

The launcher (sstcodec/launch.py) starts torch.distributed.run as a child
process, each rank joins the group and checks WORLD_SIZE == N; --plumbing
swaps the GPU step for a host copy over gloo so the whole rank / barrier /
gather / aggregate path runs here.  The JSON must report n_gpus == N and one
entry per rank, and a mismatched external world size must be refused."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(args, env_extra=None):
    env = os.environ.copy()
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                          text=True, timeout=240, env=env, cwd=ROOT)


@pytest.mark.parametrize("n", [2, 3])
def test_bench_launches_n_ranks(n):
    r = run_bench(["--gpus", str(n), "--plumbing", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert [p["rank"] for p in out["per_rank"]] == list(range(n))
    assert [p["shard_tag"] for p in out["per_rank"]] == list(range(n))  # each rank ran its own shard
    assert out["value"] > 0
    # the config-4 leg's rank path: rank r merged its own 128-SST shard of
    # workload.config_inputs(4, r), the shards' key ranges are disjoint and
    # consecutive, the aggregate is over all ranks
    c4 = out["compact_config4"]
    assert c4["n_gpus"] == n and [p["rank"] for p in c4["per_rank"]] == list(range(n))
    per = 128 * 64
    assert [p["key_index_range"] for p in c4["per_rank"]] == [[r * per, (r + 1) * per - 1] for r in range(n)]
    assert c4["GiBps_aggregate"] > 0 and all(p["GiBps"] > 0 for p in c4["per_rank"])


def test_bench_refuses_world_mismatch():
    # an external launcher with WORLD_SIZE=1 while --gpus 2 was asked for
    r = run_bench(["--gpus", "2", "--plumbing", "--steps", "1"],
                  {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)
