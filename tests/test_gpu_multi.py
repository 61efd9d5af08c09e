"""In-process multi-device compaction (sstc_compact_files_multi, SURVEY.md
§7 step 6 / §8(e)): key-range-disjoint shards, one host thread + context +
pipe per device, no data across devices, outputs in shard order with the ids
of the shards compacted one after another.  On this one-GPU box the "devices"
are several contexts on device 0, each with its own stream: the same code
path the engine would drive with one context per GPU.

Every shard's outputs must equal what an independent compaction of that shard
writes: the oracle's (small shards) and the reference's own compaction of the
BASELINE config-4 shards (tests/golden/compaction_configs.json
config4_rank{r})."""
import hashlib
import json
import os

import numpy as np
import pytest
from conftest import GOLDEN
from sstcodec import workload as W

pytestmark = pytest.mark.gpu
CONFIGS = json.load(open(os.path.join(GOLDEN, "compaction_configs.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint8).tobytes()).hexdigest()


def make_pipes(n):
    import torch
    import sstcodec
    codecs, pipes, streams = [], [], []
    for _ in range(n):
        c = sstcodec.Codec(0)
        st = torch.cuda.Stream(device=0)
        with torch.cuda.stream(st):
            c._stream()  # a stream of its own per context: the shards' device jobs overlap
        codecs.append(c)
        streams.append(st)
        pipes.append(sstcodec.FilePipe(c, io_threads=4))
    return codecs, pipes, streams


def close(codecs, pipes):
    for p in pipes:
        p.close()
    for c in codecs:
        c.close()


def small_shards(tmp_path, oracle, n_shards, per_shard=6, keys=3000):
    shards, want = [], []
    for r in range(n_shards):
        sets = W.config_inputs(4, rank=r, ssts=per_shard, keys=keys)
        files = [oracle.table_build(x, 4096) for x in sets]
        sh = []
        for i, f in enumerate(files):
            p = str(tmp_path / f"s{r}_{i}.sst")
            f.tofile(p)
            sh.append((p, f.size + 1))
        shards.append(sh)
        outs, _ = oracle.compact(files, 4096, 1 << 20, 1)  # ~1 MiB tables: several per shard
        want.append(outs)
    return shards, want


@pytest.mark.parametrize("n_pipes,n_shards", [(2, 2), (3, 4), (4, 4), (2, 5)])
def test_multi_small_shards_vs_oracle(oracle, tmp_path, n_pipes, n_shards):
    from sstcodec.codec import compact_files_multi
    shards, want = small_shards(tmp_path, oracle, n_shards)
    codecs, pipes, _ = make_pipes(n_pipes)
    try:
        od = tmp_path / "out"
        od.mkdir()
        outs, tm = compact_files_multi(pipes, shards, str(od) + "/", 1000, 4096, 1 << 20, 1, fsync=False)
    finally:
        close(codecs, pipes)
    flat = [w for ws in want for w in ws]
    assert len(tm) == n_shards and len(outs) == len(flat) > n_shards
    assert [o[0] for o in outs] == list(range(1000, 1000 + len(flat)))  # ids continue shard to shard
    for (sid, fs, lo, hi), w in zip(outs, flat):
        img = np.fromfile(str(od / f"{sid}.sst"), np.uint8)
        assert fs == img.size + 1 == w.size + 1 and np.array_equal(img, w)
    # shard order = key order (the shards are key-range-disjoint and ascending)
    keys = [(lo, hi) for _, _, lo, hi in outs]
    assert all(a[1] < b[0] for a, b in zip(keys, keys[1:]))


def test_multi_failing_shard(oracle, tmp_path):
    """A shard that cannot be read fails the call with its error; the shards
    after it write nothing, the ones before it complete."""
    import sstcodec
    from sstcodec.codec import compact_files_multi
    shards, want = small_shards(tmp_path, oracle, 3)
    shards[1][2] = (str(tmp_path / "missing.sst"), shards[1][2][1])
    codecs, pipes, _ = make_pipes(3)
    try:
        od = tmp_path / "out"
        od.mkdir()
        with pytest.raises(sstcodec.SstcError, match="shard 1") as e:
            compact_files_multi(pipes, shards, str(od) + "/", 1, 4096, 1 << 20, 1, fsync=False)
    finally:
        close(codecs, pipes)
    written = sorted(int(f.split(".")[0]) for f in os.listdir(od))
    assert written == list(range(1, 1 + len(want[0])))  # shard 0 only
    for sid in written:
        assert np.array_equal(np.fromfile(str(od / f"{sid}.sst"), np.uint8), want[0][sid - 1])
    assert [o[0] for o in e.value.outs] == written  # and reported


def _run_multi(tmp_path, shards, n_pipes, **kw):
    from sstcodec.codec import compact_files_multi
    codecs, pipes, _ = make_pipes(n_pipes)
    od = tmp_path / "out"
    try:
        return compact_files_multi(pipes, shards, str(od) + "/", 1, 4096, 1 << 20, 1, **kw)
    finally:
        close(codecs, pipes)


@pytest.mark.parametrize("fsync", [False, True])
def test_multi_store_failure_stops_later_shards(oracle, tmp_path, fsync):
    """a shard whose WRITE fails (its first output path is a
    directory) fails the call; the shards after it write nothing, the one
    before it completes and is reported (fsync on: the O_DIRECT writes)."""
    import sstcodec
    shards, want = small_shards(tmp_path, oracle, 4)
    od = tmp_path / "out"
    od.mkdir()
    n0 = len(want[0])
    os.mkdir(od / f"{1 + n0}.sst")  # shard 1's first output
    with pytest.raises(sstcodec.SstcError, match="shard 1") as e:
        _run_multi(tmp_path, shards, 4, fsync=fsync)
    files = sorted(int(f.split(".")[0]) for f in os.listdir(od) if os.path.isfile(od / f))
    assert max(files) <= n0 + len(want[1])  # nothing of shards 2 and 3
    assert [o[0] for o in e.value.outs] == list(range(1, 1 + n0))  # shard 0: complete and reported
    for sid in range(1, 1 + n0):
        assert np.array_equal(np.fromfile(str(od / f"{sid}.sst"), np.uint8), want[0][sid - 1])


def test_multi_max_outs_across_shards(oracle, tmp_path):
    """max_outs holds per shard but not for the call: the shard
    that would pass it fails before touching a file; the shards before it are
    written and reported, the ones after write nothing."""
    import sstcodec
    shards, want = small_shards(tmp_path, oracle, 3)
    n0, n1 = len(want[0]), len(want[1])
    assert n1 > 1
    (tmp_path / "out").mkdir()
    with pytest.raises(sstcodec.SstcError, match="max_outs") as e:
        _run_multi(tmp_path, shards, 3, fsync=False, max_outs=n0 + n1 - 1)
    files = sorted(int(f.split(".")[0]) for f in os.listdir(tmp_path / "out"))
    assert files == list(range(1, 1 + n0)) and [o[0] for o in e.value.outs] == files


@pytest.mark.timeout(600)
def test_multi_config4_shards_vs_reference(tmp_path):
    """BASELINE config 4's ranks 0 and 1 (128 SSTs x 100 k records each, built by
    the flush-path TableBuilder and hash-checked against the reference
    TableBuilder's files) as two shards on two contexts: every output equal to
    the reference's compaction of that shard (config4_rank0/1)."""
    import sstcodec
    from sstcodec.codec import compact_files_multi
    from sstcodec.table import build_table
    codec = sstcodec.Codec(0)
    shards = []
    try:
        for rank in (0, 1):
            case = CONFIGS[f"config4_rank{rank}"]
            sh = []
            for i, rec in enumerate(W.config_inputs(**case["gen"])):
                p = str(tmp_path / f"r{rank}_{i}.sst")
                fs, _ = build_table(codec, p, rec, case["block_threshold"])
                assert fs == case["inputs"][i]["file_size"]
                sh.append((p, fs))
            shards.append(sh)
    finally:
        codec.close()
    codecs, pipes, _ = make_pipes(2)
    try:
        od = tmp_path / "out"
        od.mkdir()
        outs, tm = compact_files_multi(pipes, shards, str(od) + "/", 1, 4096, 32 << 20, 1, fsync=False)
    finally:
        close(codecs, pipes)
    want = CONFIGS["config4_rank0"]["outputs_base1"] + CONFIGS["config4_rank1"]["outputs_base1"]
    assert len(outs) == len(want)
    for (sid, fs, _, _), w in zip(outs, want):
        img = np.fromfile(str(od / f"{sid}.sst"), np.uint8)
        assert fs == w["file_size"] and sha(img) == w["sha256"], f"output {sid}"
    print("config4 ranks 0+1 on two contexts:", [round(t["total_s"], 3) for t in tm], flush=True)
