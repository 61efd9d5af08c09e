"""CPU, world_size 2 (gloo): the sharding and aggregation the multi-GPU bench
uses — disjoint, complete SST shards; max-over-ranks timing; weak-scaling
aggregate = sum of per-rank bytes / max time.  Each rank also runs the CPU
oracle round trip over its shard to show shards are independent (no exchange)."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "lsm-kv-storage_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import Oracle
        from sstcodec import shard
        from sstcodec import workload as W
        mine = shard.sst_shard(1024, world, rank)
        # each rank encodes + round-trips only its own SSTs (4 tiny ones here)
        import time
        orc = Oracle()
        dist.barrier()
        t0 = time.perf_counter()
        lo, hi = shard.record_range(rank, 500)
        rec = W.uniform_records(500, key_index=np.arange(lo, hi, dtype=np.uint64), seed=1 + rank)
        first = W.segment(rec, 4096)
        src, off, ln = orc.encode_blocks(rec, first)
        dst, out_len, status, bad = orc.roundtrip(src, off, ln, 1)
        ok = bad == 0 and np.array_equal(dst, src)
        t = time.perf_counter() - t0  # this rank's measured wall time for its shard
        tmax = shard.max_over_ranks(t)
        total = shard.sum_over_ranks(float(src.size))
        gathered = [None] * world
        dist.all_gather_object(gathered, (mine[0], mine[-1], len(mine), lo, hi, t))
        q.put((rank, ok, tmax, total, gathered))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, tmax, total, gathered in res:
        assert ok
        (a0, a1, an, lo0, hi0, ta), (b0, b1, bn, lo1, hi1, tb) = gathered
        assert ta > 0 and tb > 0 and tmax == max(ta, tb)  # max over the ranks' measured times
        assert a0 == 0 and a1 + 1 == b0 and b1 == 1023 and an == bn == 512  # disjoint + complete
        assert hi0 == lo1  # disjoint key ranges
        assert total > 0


def test_shard_sizes():
    from sstcodec import shard
    for n in (0, 1, 7, 1024):
        for w in (1, 2, 3, 8):
            parts = [shard.sst_shard(n, w, r) for r in range(w)]
            flat = [x for p in parts for x in p]
            assert flat == list(range(n))
            assert max(map(len, parts)) - min(map(len, parts)) <= 1
