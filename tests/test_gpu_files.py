"""GPU file-to-file compaction (sstc_compact_files): input SST files on disk ->
output SST files, byte-identical to the oracle compaction and to the
reference's own outputs (tests/golden/compaction.json), with the
VersionEdit::AddNewFiles metadata (GetFileSize, smallest / largest key)."""
import hashlib
import json
import os

import numpy as np
import pytest
from conftest import GOLDEN
from sstcodec import workload as W

pytestmark = pytest.mark.gpu
CASES = json.load(open(os.path.join(GOLDEN, "compaction.json")))


@pytest.fixture(scope="module")
def pipe():
    import sstcodec
    codec = sstcodec.Codec(0)
    return sstcodec.FilePipe(codec, io_threads=4)


def write_inputs(tmp_path, files):
    paths, sizes = [], []
    for i, f in enumerate(files):
        p = str(tmp_path / f"in{i}.sst")
        f.tofile(p)
        paths.append(p)
        sizes.append(f.size + 1)  # GetFileSize() convention
    return paths, sizes


def first_last_key(img):
    foot = img[-40:].view(np.uint64)
    nb, moff = int(foot[0]), int(foot[1])
    m = img[moff:].tobytes()
    p, lo, hi = 0, b"", b""
    for i in range(nb):
        fk = int.from_bytes(m[p:p + 4], "little")
        lk = int.from_bytes(m[p + 4 + fk:p + 8 + fk], "little")
        if i == 0:
            lo = m[p + 4:p + 4 + fk]
        hi = m[p + 8 + fk:p + 8 + fk + lk]
        p += 24 + fk + lk
    return lo, hi


@pytest.mark.parametrize("name", ["split", "zipf", "dups"])
def test_files_match_reference(pipe, oracle, tmp_path, name):
    case = CASES[name]
    sets = W.compaction_inputs(case["k"], case["n_per"], case["key_space"], vmax=case["vmax"],
                               distinct=case["distinct"], **case.get("gen", {}))
    files = [oracle.table_build(r, case["block_threshold"]) for r in sets]
    paths, sizes = write_inputs(tmp_path, files)
    od = tmp_path / "out"
    od.mkdir()
    for base in (1, 0):
        outs, tm = pipe.compact_files(paths, sizes, str(od) + "/", 100, case["block_threshold"],
                                      case["table_limit"], base)
        want = case[f"outputs_base{base}"]
        assert [o[0] for o in outs] == list(range(100, 100 + len(want)))
        for (sid, fsize, lo, hi), w in zip(outs, want):
            img = np.fromfile(str(od / f"{sid}.sst"), np.uint8)
            assert fsize == w["file_size"] == img.size + 1
            assert hashlib.sha256(img.tobytes()).hexdigest() == w["sha256"]
            assert (lo, hi) == first_last_key(img)
        assert tm["total_s"] >= tm["compact_s"] > 0


def test_files_vs_oracle_many_inputs(pipe, oracle, tmp_path):
    sets = W.compaction_inputs(13, 700, 3000, seed=8, vmax=300, p_delete=0.3)
    files = [oracle.table_build(r, 4096) for r in sets]
    paths, sizes = write_inputs(tmp_path, files)
    want, _ = oracle.compact(files, 4096, 40_000, 1)
    outs, _ = pipe.compact_files(paths, sizes, str(tmp_path) + "/o", 7, 4096, 40_000, 1, fsync=False)
    assert len(outs) == len(want)
    for (sid, fsize, lo, hi), w in zip(outs, want):
        img = np.fromfile(str(tmp_path / f"o{sid}.sst"), np.uint8)
        assert np.array_equal(img, w) and fsize == w.size + 1


def test_files_empty_and_errors(pipe, oracle, tmp_path):
    # no input: one empty output table (40 B footer, as DoCompactJob's first TableBuilder)
    outs, _ = pipe.compact_files([], [], str(tmp_path) + "/e", 1)
    assert len(outs) == 1 and outs[0][1] == 41
    # truncated input file: rejected, nothing written
    f = oracle.table_build(W.compaction_inputs(1, 200, 400, seed=3)[0], 4096)
    p = str(tmp_path / "bad.sst")
    f[:-7].tofile(p)
    with pytest.raises(Exception):
        pipe.compact_files([p], [f.size + 1], str(tmp_path) + "/x", 1)
    with pytest.raises(Exception):
        pipe.compact_files([str(tmp_path / "missing.sst")], [1000], str(tmp_path) + "/x", 1)


def test_files_capacity_retry_and_bound(oracle, tmp_path):
    """sstc_compact_files' capacity retry (compact_files.cpp): a first attempt
    forced one byte short of the output goes through SSTC_E_CAPACITY, the
    retry at the device-reported size writes the reference's files; a
    device-reported size past the input-derived bound is SSTC_E_INTERNAL
    (nothing is allocated for it, no file is written)."""
    import sstcodec
    case = CASES["split"]
    sets = W.compaction_inputs(case["k"], case["n_per"], case["key_space"], vmax=case["vmax"],
                               distinct=case["distinct"], **case.get("gen", {}))
    files = [oracle.table_build(r, case["block_threshold"]) for r in sets]
    paths, sizes = write_inputs(tmp_path, files)
    want = case["outputs_base1"]
    need = sum(w["file_size"] - 1 for w in want)
    codec = sstcodec.Codec(0)
    p = sstcodec.FilePipe(codec, io_threads=2)
    try:
        for first in (1, need - 1, need):
            od = tmp_path / f"out{first}"
            od.mkdir()
            assert p.lib.sstc__pipe_set_test_caps(p.h, first, 0) == 0
            outs, _ = p.compact_files(paths, sizes, str(od) + "/", 100, case["block_threshold"], case["table_limit"], 1)
            assert [o[1] for o in outs] == [w["file_size"] for w in want]
            for (sid, fs, lo, hi), w in zip(outs, want):
                img = np.fromfile(str(od / f"{sid}.sst"), np.uint8)
                assert hashlib.sha256(img.tobytes()).hexdigest() == w["sha256"]
        od = tmp_path / "bound"
        od.mkdir()
        assert p.lib.sstc__pipe_set_test_caps(p.h, 1, 1024) == 0
        with pytest.raises(sstcodec.SstcError, match="bound from the input"):
            p.compact_files(paths, sizes, str(od) + "/", 100, case["block_threshold"], case["table_limit"], 1)
        assert not os.listdir(od)
        # the pipe still works afterwards
        assert p.lib.sstc__pipe_set_test_caps(p.h, 0, 0) == 0
        od = tmp_path / "after"
        od.mkdir()
        outs, _ = p.compact_files(paths, sizes, str(od) + "/", 100, case["block_threshold"], case["table_limit"], 1)
        assert [o[1] for o in outs] == [w["file_size"] for w in want]
    finally:
        p.close()
        codec.close()


def test_files_refuse_differing_ties(pipe, tmp_path):
    """SSTC_E_TIE_ORDER through the file pipeline: inputs
    holding equal (key, txn) records with different contents in different
    tables are refused before any output file is created; identical copies
    compact as the reference does."""
    from conftest import load_golden, tie_case
    from sstcodec._lib import SSTC_E_TIE_ORDER, SstcError
    g = load_golden("compact_ties.npz")
    ins, _ = tie_case(g, "diff", 1)
    paths, sizes = write_inputs(tmp_path, ins)
    od = tmp_path / "out"
    od.mkdir()
    with pytest.raises(SstcError) as e:
        pipe.compact_files(paths, sizes, str(od) + "/", 100, 4096, 6000, 1)
    assert e.value.code == SSTC_E_TIE_ORDER
    assert os.listdir(od) == []
    ins, want = tie_case(g, "same", 1)
    paths, sizes = write_inputs(tmp_path, ins)
    outs, _ = pipe.compact_files(paths, sizes, str(od) + "/", 100, 4096, 6000, 1)
    got = [np.fromfile(str(od / f"{sid}.sst"), np.uint8) for sid, _, _, _ in outs]
    assert len(got) == len(want) and all(np.array_equal(a, b) for a, b in zip(got, want))
