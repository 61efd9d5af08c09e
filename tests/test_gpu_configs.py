"""BASELINE configs 3, 3-overlap, 4 (rank-0 shard) and 5 at their full size on the
GPU, against the reference's own outputs (tests/golden/compaction_configs.json,
made by tests/golden/make_golden_configs.py from oracle/_ref: the reference's
TableBuilder for the inputs, its MergeIterator + TableReaderIterator +
TableBuilder under the DoCompactJob loop of /root/reference/db/compact.cc:232-322
for the outputs).

Per case, on the box:
  1. the input record sets are regenerated from the recorded parameters
     (sstcodec.workload.config_inputs) and written by this framework's own
     flush-path sstc::TableBuilder (GPU encode): every input file must hash to
     the reference TableBuilder's bytes (table_builder.cc:35-211 at scale);
  2. sstc_compact (device job) over the resident images: every output SST must
     hash to the reference's output and have its GetFileSize();
  3. sstc_compact_files (file -> file pipeline) over the input files: the same.
Config 3 crosses the 32 MiB output split (compact.cc:290) 27 times.
"""
import hashlib
import json
import os

import numpy as np
import pytest
from conftest import GOLDEN
from sstcodec import workload as W

pytestmark = pytest.mark.gpu
CASES = json.load(open(os.path.join(GOLDEN, "compaction_configs.json")))


@pytest.fixture(scope="module")
def codec():
    import sstcodec
    return sstcodec.Codec(0)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint8).tobytes()).hexdigest()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name", ["config5", "config3_overlap", "config3", "config4_rank0"])
def test_config_full_size_vs_reference(codec, tmp_path, name):
    import torch
    import sstcodec
    from sstcodec.table import build_table

    case = CASES[name]
    want = case["outputs_base1"]
    # 1. inputs through the flush-path TableBuilder, equal to the reference's files
    paths, sizes, imgs = [], [], []
    for i, rec in enumerate(W.config_inputs(**case["gen"])):
        p = str(tmp_path / f"in{i}.sst")
        fs, _ = build_table(codec, p, rec, case["block_threshold"])
        img = np.fromfile(p, np.uint8)
        w = case["inputs"][i]
        assert fs == w["file_size"] == img.size + 1, f"input {i}: GetFileSize"
        assert sha(img) == w["sha256"], f"input {i} differs from the reference TableBuilder's file"
        paths.append(p)
        sizes.append(fs)
        imgs.append(img)
    print(f"{name}: {len(imgs)} inputs equal to the reference's", flush=True)

    # 2. device-resident compaction job
    outs, res = codec.compact(imgs, case["block_threshold"], case["table_limit"], 1)
    del imgs
    assert res.tables_out == len(outs) == len(want)
    for t, (o, w) in enumerate(zip(outs, want)):
        assert o.size + 1 == w["file_size"], f"output {t}: GetFileSize"
        assert sha(o) == w["sha256"], f"output {t} differs from the reference's"
    del outs
    torch.cuda.empty_cache()
    print(f"{name}: device job -> {len(want)} outputs equal to the reference's", flush=True)

    # 3. file -> file pipeline
    pipe = sstcodec.FilePipe(codec, io_threads=8)
    try:
        od = tmp_path / "out"
        od.mkdir()
        fouts, _ = pipe.compact_files(paths, sizes, str(od) + "/", 1, case["block_threshold"],
                                      case["table_limit"], 1, fsync=False)
    finally:
        pipe.close()
    assert len(fouts) == len(want)
    for (sid, fsize, _, _), w in zip(fouts, want):
        p = str(od / f"{sid}.sst")
        img = np.fromfile(p, np.uint8)
        assert fsize == w["file_size"] == img.size + 1
        assert sha(img) == w["sha256"], f"file output {sid} differs from the reference's"
        os.remove(p)
    print(f"{name}: file pipeline -> {len(want)} outputs equal to the reference's", flush=True)


@pytest.mark.timeout(300)
def test_lookup_config3_vs_reference(codec, oracle):
    """sstc_get_batch at full size: 40 000 seeded point lookups over the 8
    config-3 SSTs (8 x 151.6 MB resident, block indexes from sstc_open_tables)
    give the reference TableReader::GetValue's types, value lengths and values
    (hashes in compaction_configs.json)."""
    import sstcodec
    case = CASES["lookup_config3"]
    tables = [oracle.table_build(r, 4096) for r in W.config_inputs(3)]
    for t, img in enumerate(tables):
        assert img.size + 1 == case["inputs"][t]["file_size"]
    qt, qk = W.config3_lookup_queries(case["queries"], case["seed"])
    keys = [bytes(k) for k in W.fixed_keys(qk).reshape(-1, 16)]
    lk = sstcodec.Lookup(codec, tables)
    typ, vo, vl, _ = lk.get(qt, keys)
    whole = np.concatenate(tables)
    del tables
    vlens = np.where(typ == 0, vl, 0).astype(np.uint32)
    vals = b"".join(bytes(whole[int(o):int(o) + int(n)]) for o, n, t in zip(vo, vl, typ) if t == 0)
    assert hashlib.sha256(typ.astype(np.uint32).tobytes()).hexdigest() == case["types_sha256"]
    assert hashlib.sha256(vlens.tobytes()).hexdigest() == case["val_len_sha256"]
    assert hashlib.sha256(vals).hexdigest() == case["values_sha256"]


@pytest.mark.timeout(900)
def test_config4_all_shards_vs_reference(codec, tmp_path):
    """BASELINE config 4 whole: 1024 SSTs, 128 per GPU.  Ranks 1-7's shards
    (rank 0 is test_config_full_size_vs_reference) run one after another on
    this GPU through the same device job each rank runs in bench
    (tools/bench_compact.py --config 4): inputs written by sstc::TableBuilder
    and hash-checked against the reference TableBuilder's files, every output
    SST's SHA-256 and GetFileSize() equal to the reference's compaction of
    that shard (compaction_configs.json config4_rank1..7)."""
    import torch
    from sstcodec.table import build_table
    for rank in range(1, 8):
        case = CASES[f"config4_rank{rank}"]
        imgs = []
        for i, rec in enumerate(W.config_inputs(**case["gen"])):
            p = str(tmp_path / f"r{rank}_in{i}.sst")
            fs, _ = build_table(codec, p, rec, case["block_threshold"])
            img = np.fromfile(p, np.uint8)
            os.remove(p)
            w = case["inputs"][i]
            assert fs == w["file_size"] and sha(img) == w["sha256"], f"rank {rank} input {i}"
            imgs.append(img)
        outs, res = codec.compact(imgs, case["block_threshold"], case["table_limit"], 1)
        del imgs
        want = case["outputs_base1"]
        assert res.tables_out == len(outs) == len(want)
        for t, (o, w) in enumerate(zip(outs, want)):
            assert o.size + 1 == w["file_size"] and sha(o) == w["sha256"], f"rank {rank} output {t}"
        del outs
        torch.cuda.empty_cache()
        print(f"config4 rank {rank}: 128 inputs -> {len(want)} outputs equal to the reference's", flush=True)
