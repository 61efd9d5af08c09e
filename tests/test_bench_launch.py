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

import numpy as np
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


def test_one_rank_process_group_under_a_launcher():
    """SSTC_PG_SINGLE=1 under torch.distributed.run: a one-rank process group
    is built (gloo here; tests/test_gpu_bench_rank.py does the same with
    RCCL on the GPU box), and the collectives run through it."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = os.environ.copy()
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["SSTC_PG_SINGLE"] = "1"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                        "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
                        "--gpus", "1", "--plumbing", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "[sstc] process group: gloo, world 1" in r.stderr
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 1 and out["compact_config4"]["n_gpus"] == 1


def test_bench_refuses_world_mismatch():
    # an external launcher with WORLD_SIZE=1 while --gpus 2 was asked for
    r = run_bench(["--gpus", "2", "--plumbing", "--steps", "1"],
                  {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)


# ---------------------------------------------------------------------------
# bench.py's GpuCompaction / time_job / config4_leg rank path over gloo, with a
# host stand-in for the device job: the class's input build + hash check, its
# run() call shape (sstc_compact's arguments), outputs(), the timing, the gather
# and the aggregation run as in the GPU bench; only the codec underneath is the
# oracle (test infrastructure).
class _HostLib:
    """sstc_compact / open_tables / _stream with sstc_compact's argument list,
    computed by the oracle restatement and written through the pointers."""

    def __init__(self, tables, T, limit):
        self.tables, self.T, self.limit = tables, T, limit

    def sstc_compact(self, h, src, bo, bl, nb, tfb, ntables, prm, dst, cap, toff, tlen, max_t, res):
        import ctypes
        from oracle import Oracle
        prm = prm._obj
        assert (prm.block_threshold, prm.table_limit, prm.base_level) == (self.T, self.limit, 1)
        assert ntables == len(self.tables) and nb > 0
        outs, _ = Oracle().compact(self.tables, self.T, self.limit, 1)
        offs = np.cumsum([0] + [o.size for o in outs]).astype(np.int64)
        assert offs[-1] <= cap and len(outs) <= max_t
        blob = np.concatenate(outs)
        ctypes.memmove(dst.value, blob.ctypes.data, blob.size)
        ctypes.memmove(toff.value, offs.ctypes.data, offs.nbytes)
        lens = np.diff(offs)
        ctypes.memmove(tlen.value, lens.ctypes.data, lens.nbytes)
        r = res._obj
        r.tables_out = len(outs)
        r.bytes_out = int(offs[-1])
        return 0


class _HostCodec:
    def __init__(self, lib):
        self.lib = lib
        self.h = None

    def _stream(self):
        pass

    def open_tables(self, src, sizes, strict=False):
        import torch
        from oracle import Oracle
        orc = Oracle()
        img = src.numpy()
        bo, bl, tfb, at = [], [], [0], 0
        for sz in sizes:
            idx = orc.table_index(img[at:at + sz])
            bo += [int(x) + at for x in idx["blk_off"]]
            bl += [int(x) for x in idx["blk_len"]]
            tfb.append(len(bo))
            at += sz
        return {"blk_off": torch.tensor(bo, dtype=torch.int64), "blk_len": torch.tensor(bl, dtype=torch.int64),
                "table_first_block": np.asarray(tfb, np.uint64)}


def _c4_worker(rank, world, port, q):
    import hashlib
    import tempfile
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "lsm-kv-storage_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import sstcodec.table
        from oracle import Oracle
        from sstcodec import launch
        from sstcodec import workload as W
        orc = Oracle()

        def host_build(codec, path, rec, T=4096):  # the flush-path builder's stand-in
            img = orc.table_build(rec, T)
            img.tofile(path)
            return img.size + 1, None

        sstcodec.table.build_table = host_build
        ranks = launch.Ranks(world, rank, rank, None, "gloo")
        keys = 64
        sets = {r: W.config_inputs(4, r, keys=keys) for r in range(world)}
        tables = {r: [orc.table_build(x, 4096) for x in sets[r]] for r in range(world)}

        def fixture(r):  # what the reference's hashes would say, from the restatement
            outs, _ = orc.compact(tables[r], 4096, 32 << 20, 1)
            sha = lambda a: hashlib.sha256(a.tobytes()).hexdigest()  # noqa: E731
            return {"inputs": [{"sha256": sha(t), "file_size": t.size + 1} for t in tables[r]],
                    "outputs_base1": [{"sha256": sha(o), "file_size": o.size + 1} for o in outs]}

        td = tempfile.mkdtemp()
        make = lambda r: bench.GpuCompaction(_HostCodec(_HostLib(tables[r], 4096, 32 << 20)),  # noqa: E731
                                             torch.device("cpu"), None, td, sets[r], fixture(r))
        leg = bench.config4_leg(ranks, make, 2, fixture)
        q.put((rank, leg))
    finally:
        dist.destroy_process_group()


def test_config4_leg_gpu_compaction_rank_path_over_gloo():
    """Two ranks over gloo run bench.config4_leg with bench.GpuCompaction itself
    (a host stand-in for the codec): every rank builds and hash-checks its own
    shard, times K calls between barriers, verifies its outputs, and rank 0
    gathers per-rank rows and the max-over-ranks aggregate."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_c4_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    leg = res[0]
    assert leg["n_gpus"] == world and [p["rank"] for p in leg["per_rank"]] == [0, 1]
    assert all(p["verified_vs_reference"] is True for p in leg["per_rank"])
    assert leg["GiBps_aggregate"] > 0 and leg["ms_per_call_max"] >= max(p["ms_per_call"] for p in leg["per_rank"])
    assert leg["per_rank"][0]["input_bytes"] > 0 and leg["per_rank"][1]["output_bytes"] > 0
