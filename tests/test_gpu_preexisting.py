"""GPU: output SST paths that already exist (SURVEY.md §7 quirk list).

The reference opens an existing output file WITHOUT O_TRUNC
(`io/linux_file.cc:99-119`, `LinuxWriteOnlyFile::Open`: `O_WRONLY` only when
`access(F_OK)` succeeds) and writes the table with `pwrite` from offset 0
(`sstable/table_builder.cc:62-99,147-177`).  A pre-existing file longer than
the new table therefore keeps its stale tail; a shorter one is overwritten and
extended.  Both writers of this build -- the flush-path `sstc::TableBuilder`
and the compaction file pipeline `sstc_compact_files` -- reproduce that, and
the test compares the WHOLE on-disk file (stale tail included) with what the
reference's own TableBuilder (`oracle/_ref`, compiled from the reference's
sources) leaves on an identical pre-existing file.  `GetFileSize()` is the
table's bytes + 1 in both, whatever the file's length on disk."""
import os
import json

import numpy as np
import pytest
from conftest import GOLDEN
from sstcodec import workload as W

pytestmark = pytest.mark.gpu
CASES = json.load(open(os.path.join(GOLDEN, "compaction.json")))


@pytest.fixture(scope="module")
def codec():
    import sstcodec
    return sstcodec.Codec(0)


def _stale(rng, n):
    return rng.integers(0, 256, n, dtype=np.uint8)


def test_table_builder_keeps_stale_tail(codec, reflib, tmp_path):
    """sstc::TableBuilder over a longer and a shorter pre-existing file vs the
    reference TableBuilder over the same files."""
    from sstcodec.table import build_table
    rng = np.random.default_rng(41)
    rec = W.mixed_records(3000, seed=41, max_val=500)
    for name, extra in (("longer", 7777), ("shorter", None), ("absent", 0)):
        ours, ref = str(tmp_path / f"ours_{name}.sst"), str(tmp_path / f"ref_{name}.sst")
        if name != "absent":
            probe = str(tmp_path / "probe.sst")
            fs_probe = reflib.table_build(probe, rec, 4096)
            os.unlink(probe)
            size = fs_probe - 1 + extra if extra else (fs_probe - 1) // 3
            stale = _stale(rng, size)
            stale.tofile(ours)
            stale.tofile(ref)
        fs_ref = reflib.table_build(ref, rec, 4096)
        fs, _ = build_table(codec, ours, rec, 4096)
        a, b = np.fromfile(ours, np.uint8), np.fromfile(ref, np.uint8)
        assert fs == fs_ref, name
        assert a.size == b.size and np.array_equal(a, b), name
        if name == "longer":  # the reference really left the tail behind
            assert b.size == fs_ref - 1 + extra and np.array_equal(b[fs_ref - 1:], stale[fs_ref - 1:])
        else:
            assert b.size == fs_ref - 1


@pytest.mark.parametrize("name", ["split"])
def test_compact_files_keep_stale_tail(codec, oracle, reflib, tmp_path, name):
    """sstc_compact_files writing over pre-existing output files (longer,
    shorter and absent ones, plus a path past the last output) vs the
    reference's own compaction loop (oracle/_ref/ref_compact: MergeIterator +
    TableBuilder) over identical pre-existing files."""
    import sstcodec
    from oracle import ref_compact
    case = CASES[name]
    sets = W.compaction_inputs(case["k"], case["n_per"], case["key_space"], vmax=case["vmax"],
                               distinct=case["distinct"], **case.get("gen", {}))
    files = [oracle.table_build(r, case["block_threshold"]) for r in sets]
    paths, sizes = [], []
    for i, f in enumerate(files):
        p = str(tmp_path / f"in{i}.sst")
        f.tofile(p)
        paths.append(p)
        sizes.append(f.size + 1)
    want = case["outputs_base1"]
    rng = np.random.default_rng(7)
    ours, refd = tmp_path / "ours", tmp_path / "ref"
    ours.mkdir()
    refd.mkdir()
    stale = {}
    for k, w in enumerate(want + [5000]):  # one more path than outputs: left alone by both
        if k == len(want) - 2:
            continue  # absent: created by both
        n = w["file_size"] - 1 + 4096 + 13 * k if isinstance(w, dict) and k % 2 == 0 else \
            (w["file_size"] // 2 if isinstance(w, dict) else w)
        stale[k] = _stale(rng, n)
        stale[k].tofile(str(ours / f"{k}.sst"))
        stale[k].tofile(str(refd / f"{k}.sst"))
    ref_out = ref_compact(list(zip(paths, sizes)), str(refd), case["block_threshold"], case["table_limit"], 1)
    assert [s for _, s in ref_out] == [w["file_size"] for w in want]
    pipe = sstcodec.FilePipe(codec, io_threads=4)
    outs, _ = pipe.compact_files(paths, sizes, str(ours) + "/", 0, case["block_threshold"], case["table_limit"], 1)
    assert [o[1] for o in outs] == [w["file_size"] for w in want]
    longer = 0
    for k in range(len(want) + 1):
        a, b = np.fromfile(str(ours / f"{k}.sst"), np.uint8), np.fromfile(str(refd / f"{k}.sst"), np.uint8)
        assert a.size == b.size and np.array_equal(a, b), k
        if k < len(want) and k in stale and stale[k].size > want[k]["file_size"] - 1:
            longer += 1
            assert b.size == stale[k].size  # the tail survived in the reference's file too
    assert longer >= 2
    assert np.array_equal(np.fromfile(str(ours / f"{len(want)}.sst"), np.uint8), stale[len(want)])
