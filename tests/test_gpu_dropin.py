"""The drop-in of INTEGRATION.md, run: oracle/_ref/compact_dropin is
/root/reference/db/compact.cc (Compact::PickCompact -> DoCompactJob) AND
/root/reference/db/merge_iterator.cc compiled UNCHANGED with include/dropin/
first on the include path, so
  * every input table is read through the drop-in
    kvs::sstable::TableReaderIterator (include/dropin/sstable/
    table_reader_iterator.h): the whole table decoded in one GPU call
    (sstc_count_records + sstc_decode_blocks), and
  * every output SST is built by sstc::TableBuilder (blocks encoded on this
    GPU at Finish()).
Its outputs must be the reference's own bytes.  (The binaries are built in the
container by `make -C oracle dropin`, see
tests/test_oracle_aswritten.py::test_dropin_builds_unmodified_compact_cc, and
travel with the tree like libsstcodec.so.)

Expected bytes: the fixed-semantics outputs of tests/golden/aswritten.json
(the reference's MergeIterator + TableReaderIterator + TableBuilder under the
DoCompactJob loop with an owned last key).  The as-written reference's
`last_current_key` view dangles once its block is freed (compact.cc:250,
table_reader_iterator.cc:148); the drop-in iterator owns its decoded table
for its whole life, so the unchanged compact.cc runs the intended semantics on
every case, including the ones where the reference as written keeps stale
duplicates or crashes (config 5, probe5000, config3_overlap, cj_zipf).
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest
from conftest import GOLDEN, ROOT, load_golden, tie_case

sys.path.insert(0, GOLDEN)
import make_golden_aswritten as G  # noqa: E402

pytestmark = pytest.mark.gpu
MANIFEST = json.load(open(os.path.join(GOLDEN, "aswritten.json")))
CJ = json.load(open(os.path.join(GOLDEN, "compaction.json")))
EXE = os.path.join(ROOT, "oracle", "_ref", "compact_dropin")
REF_EXE = os.path.join(ROOT, "oracle", "_ref", "ref_pick_compact")
RUNNABLE = [n for n, c in MANIFEST.items() if isinstance(c, dict) and "fixed_outputs" in c]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint8).tobytes()).hexdigest()


def need(exe):
    if not os.path.exists(exe):
        pytest.skip(f"{os.path.relpath(exe, ROOT)} not built (needs /root/reference at build time)")


def first_last_key(img):
    from oracle import Oracle
    orc = Oracle()
    idx = orc.table_index(img)
    keys = []
    for o, ln in ((int(idx["blk_off"][0]), int(idx["blk_len"][0])), (int(idx["blk_off"][-1]), int(idx["blk_len"][-1]))):
        st, d = orc.decode_block(img[o:o + ln], 1)
        assert st == 0
        j = 0 if not keys else len(d["type"]) - 1
        ko, kl = int(d["key_off"][j]), int(d["key_len"][j])
        keys.append(img[o + ko:o + ko + kl].tobytes())
    return keys[0], keys[1]


def build_inputs(tmp_path, sets, T):
    import sstcodec
    from sstcodec.table import build_table
    codec = sstcodec.Codec(0)
    out = []
    try:
        for i, rec in enumerate(sets):
            p = str(tmp_path / f"in{i}.sst")
            fs, _ = build_table(codec, p, rec, T)
            out.append((p, fs, rec))
    finally:
        codec.close()
    return out


def case_inputs(name):
    fac, T, limit, _ = G.CASES[name]
    if fac is None:
        return G.compaction_json_inputs(name[3:])
    return fac(), T, limit


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", RUNNABLE)
def test_unmodified_compact_cc_gpu_decode_and_encode(tmp_path, name):
    """Compact::PickCompact as written, with GPU decode (drop-in
    TableReaderIterator), the device merge (drop-in MergeIterator) and GPU
    encode (drop-in TableBuilder): every output file, GetFileSize() and
    VersionEdit key range equal to the reference's."""
    _pick_compact_case(tmp_path, name, {})


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", [n for n in ("config5", "config3") if n in RUNNABLE])
def test_unmodified_compact_cc_download_failure_falls_back(tmp_path, name):
    """The merged records' download failing midway (test hook
    SSTC_TEST_DOWNLOAD_FAIL_AT: after the first 32 K-record chunk) does not
    fail the compaction: the drop-in MergeIterator replays the reference's
    heaps to its position and walks on with them, the builders mix resident
    references with copied records, and the outputs are still the
    reference's."""
    r = _pick_compact_case(tmp_path, name, {"SSTC_TEST_DOWNLOAD_FAIL_AT": "1"})
    assert "heap mode from record 32768" in r.stderr, r.stderr[-2000:]


def _pick_compact_case(tmp_path, name, env):
    need(EXE)
    from oracle import table_key_range
    case = MANIFEST[name]
    sets, T, limit = case_inputs(name)
    ins = build_inputs(tmp_path, sets, T)
    del sets
    args = [EXE, str(tmp_path / "db"), str(T), str(limit)]
    (tmp_path / "db").mkdir()
    for (p, fs, rec), want in zip(ins, case["inputs"]):
        assert fs == want["file_size"] and sha(np.fromfile(p, np.uint8)) == want["sha256"]
        lo, hi = table_key_range(rec)
        args += [p, str(fs), lo.hex() or "-", hi.hex() or "-"]
    ins = None
    r = subprocess.run(args, capture_output=True, text=True, timeout=540, env=dict(os.environ, **env))
    assert r.returncode == 0, r.stderr[-2000:]
    if name in TIMED and os.path.exists(REF_EXE) and not env:  # the same PickCompact as written (CPU decode + encode)
        t_gpu = pick_time(r.stdout)
        d = tmp_path / "db_ref"
        d.mkdir()
        rr = subprocess.run([REF_EXE, str(d)] + args[2:], capture_output=True, text=True, timeout=540,
                            env=dict(os.environ, GLIBC_TUNABLES=G.NO_TRIM))  # config 5 as written needs the heap mapped
        assert rr.returncode == 0, rr.stderr[-1000:]
        print(f"TIMING {name}: PickCompact with the drop-in GPU decode + encode {t_gpu:.3f} s "
              f"(codec context opened before it in {pick_time(r.stdout, 'init'):.3f} s), "
              f"the reference as written {pick_time(rr.stdout):.3f} s", flush=True)
    picked, outs = G.parse_pick_output(r.stdout)
    assert picked == list(range(1, len(case["inputs"]) + 1))
    got = []
    for p, fs, lo, hi in outs:
        img = np.fromfile(p, np.uint8)
        got.append((sha(img), fs))
        assert (lo, hi) == first_last_key(img)  # what VersionEdit::AddNewFiles recorded
    assert got == [(o["sha256"], o["file_size"]) for o in case["fixed_outputs"]]
    print(f"{name}: db/compact.cc unchanged over the drop-ins, GPU decode + merge + encode -> "
          f"{len(outs)} outputs equal to the reference's", flush=True)
    return r


TIMED = ("config3", "config4_rank0", "config5")
ASAN_EXE = os.path.join(ROOT, "oracle", "_ref", "compact_dropin_asan")
# tools/build_asan.sh: the same harness with libsstcodec.so's own host code
# (TableBuilder, DecodeTable, the compaction job's host side) under ASan too
ASAN_LIB_EXE = os.path.join(ROOT, "oracle", "_ref", "compact_dropin_asan_lib")
ASAN_ENV = {"ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1"}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("exe", [ASAN_EXE, ASAN_LIB_EXE], ids=["engine", "engine+lib"])
@pytest.mark.parametrize("name", [n for n in ("cj_small", "cj_zipf", "probe100", "config5") if n in RUNNABLE])
def test_dropin_host_code_under_asan(tmp_path, name, exe):
    """The drop-in's host code -- the unmodified compact.cc / merge_iterator.cc
    and the drop-in iterator over its mapped data sections -- built with
    AddressSanitizer (`make -C oracle dropin-asan`; libsstcodec.so itself
    uninstrumented): no report, outputs the reference's.  Includes cj_zipf and
    config 5, where the reference as written reads freed memory
    (compact.cc:250, aswritten.json)."""
    need(exe)
    from oracle import table_key_range
    case = MANIFEST[name]
    sets, T, limit = case_inputs(name)
    ins = build_inputs(tmp_path, sets, T)
    args = [exe, str(tmp_path / "db"), str(T), str(limit)]
    (tmp_path / "db").mkdir()
    for p, fs, rec in ins:
        lo, hi = table_key_range(rec)
        args += [p, str(fs), lo.hex() or "-", hi.hex() or "-"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=540, env=dict(os.environ, **ASAN_ENV))
    assert "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    assert r.returncode == 0, r.stderr[-2000:]
    _, outs = G.parse_pick_output(r.stdout)
    got = [(sha(np.fromfile(p, np.uint8)), fs) for p, fs, _, _ in outs]
    assert got == [(o["sha256"], o["file_size"]) for o in case["fixed_outputs"]]


@pytest.mark.parametrize("name", [n for n in ("cj_small", "probe100") if n in RUNNABLE])
def test_unmodified_compact_cc_read_path(tmp_path, name):
    """The drop-in iterator's fallback when its table cannot be mapped: the
    data section read through the TableReader's own file object
    (SSTC_DROPIN_NO_MAP forces it; SSTC_DROPIN_HEAP_MERGE makes the drop-in
    MergeIterator walk the table iterators, as it does when the device merge
    cannot take the inputs), outputs still the reference's."""
    need(EXE)
    from oracle import table_key_range
    case = MANIFEST[name]
    sets, T, limit = case_inputs(name)
    ins = build_inputs(tmp_path, sets, T)
    args = [EXE, str(tmp_path / "db"), str(T), str(limit)]
    (tmp_path / "db").mkdir()
    for p, fs, rec in ins:
        lo, hi = table_key_range(rec)
        args += [p, str(fs), lo.hex() or "-", hi.hex() or "-"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, SSTC_DROPIN_NO_MAP="1", SSTC_TRACE_HOST="1", SSTC_DROPIN_HEAP_MERGE="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "iterator read data section" in r.stderr and "iterator map data section" not in r.stderr
    _, outs = G.parse_pick_output(r.stdout)
    got = [(sha(np.fromfile(p, np.uint8)), fs) for p, fs, _, _ in outs]
    assert got == [(o["sha256"], o["file_size"]) for o in case["fixed_outputs"]]


def pick_time(stdout, tag="time"):
    return float(next(ln.split()[1] for ln in stdout.splitlines() if ln.startswith(tag + " ")))


def run_loop(exe, tmp_path, files, T, limit, base, tag):
    od = tmp_path / f"out_{tag}_{base}"
    od.mkdir()
    args = [exe, "--loop", str(od), str(T), str(limit), str(base)]
    for i, f in enumerate(files):
        p = str(tmp_path / f"{tag}_in{i}.sst")
        f.tofile(p)
        args += [p, str(f.size + 1)]
    r = subprocess.run(args, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    _, outs = G.parse_pick_output(r.stdout)
    res = []
    for p, fs, lo, hi in outs:
        img = np.fromfile(p, np.uint8)
        assert (lo, hi) == first_last_key(img)
        res.append((img, fs))
    return res


@pytest.mark.parametrize("name", sorted(CJ))
@pytest.mark.parametrize("base", [1, 0])
def test_merge_iterator_over_dropin_readers(oracle, tmp_path, name, base):
    """The reference's own db::MergeIterator over drop-in TableReaderIterators
    (made as Compact::CreateMergeIterator makes them, through the
    TableReaderCache), the DoCompactJob loop at any table limit and both
    IsBaseLevelForKey answers: every compaction.json case, bit-exact."""
    need(EXE)
    from sstcodec import workload as W
    case = CJ[name]
    sets = W.compaction_inputs(case["k"], case["n_per"], case["key_space"], vmax=case["vmax"],
                               distinct=case["distinct"], **case.get("gen", {}))
    files = [oracle.table_build(r, case["block_threshold"]) for r in sets]
    outs = run_loop(EXE, tmp_path, files, case["block_threshold"], case["table_limit"], base, name)
    want = case[f"outputs_base{base}"]
    assert [(sha(i), fs) for i, fs in outs] == [(w["sha256"], w["file_size"]) for w in want]


@pytest.mark.parametrize("name", ["same", "diff"])
@pytest.mark.parametrize("base", [1, 0])
def test_merge_iterator_ties_over_dropin_readers(tmp_path, name, base):
    """Equal (key, txn) across inputs, identical AND differing copies: the
    reference's own heap pops the ties, fed by drop-in iterators, so even the
    'diff' case is the reference's bytes."""
    need(EXE)
    ins, want = tie_case(load_golden("compact_ties.npz"), name, base)
    outs = run_loop(EXE, tmp_path, ins, 4096, 6000, base, name)
    assert len(outs) == len(want)
    for (img, fs), w in zip(outs, want):
        assert np.array_equal(img, w) and fs == w.size + 1


def trace_tables(oracle, tmp_path):
    from readers_util import reader_records
    from sstcodec import workload as W
    rec = reader_records()
    big = W.mixed_records(400, seed=11, max_val=9000)  # values past a block: 1-entry blocks
    files = [oracle.table_build(rec, 4096), oracle.table_build(rec, 32768), oracle.table_build(big, 4096)]
    args = []
    for i, f in enumerate(files):
        p = str(tmp_path / f"t{i}.sst")
        f.tofile(p)
        args += [p, str(f.size + 1)]
    return args


def test_iterator_trace_equals_reference(oracle, tmp_path):
    """The same scripted walk (SeekToFirst + Next past the end, SeekToLast +
    Prev past the start and the entry cursor's wrap back, Seek to every
    block's first / last key and to keys outside the table, each followed by
    Next / Prev) through the reference's TableReaderIterator and through the
    drop-in: IsValid, key, value (incl. null vs empty views), type and txn
    (compat quirk of block_reader.cc:109-111) equal at every step."""
    need(EXE)
    need(REF_EXE)
    args = trace_tables(oracle, tmp_path)
    dumps = []
    runs = [(REF_EXE, "ref"), (EXE, "dropin")] + [(x, os.path.basename(x)) for x in (ASAN_EXE, ASAN_LIB_EXE)
                                                   if os.path.exists(x)]
    for exe, tag in runs:
        d = str(tmp_path / f"{tag}.dump")
        r = subprocess.run([exe, "--iter", d] + args, capture_output=True, text=True, timeout=240,
                           env=dict(os.environ, **ASAN_ENV))
        assert "AddressSanitizer" not in r.stderr, (tag, r.stderr[-3000:])
        assert r.returncode == 0, (tag, r.stderr[-2000:])
        dumps.append((r.stdout.strip(), open(d, "rb").read()))
    assert dumps[0][0].startswith("iter ok ") and len(dumps[0][1]) > 1_000_000
    for out, dump in dumps[1:]:  # the drop-in (and its ASan build) walk exactly as the reference does
        assert out == dumps[0][0] and dump == dumps[0][1]


def _merge_sets(name, oracle):
    """(file images, block threshold) of the --merge trace cases"""
    from sstcodec import workload as W
    if name in CJ:
        c = CJ[name]
        sets = W.compaction_inputs(c["k"], c["n_per"], c["key_space"], vmax=c["vmax"], distinct=c["distinct"],
                                   **c.get("gen", {}))
        return [oracle.table_build(r, c["block_threshold"]) for r in sets]
    if name.startswith("ties_"):
        return tie_case(load_golden("compact_ties.npz"), name[5:], 1)[0]
    if name == "versions":  # a key's versions out of txn order as read (empty-value PUTs, block_reader.cc:109-111)
        sets = W.compaction_inputs(3, 1500, 50, seed=70, p_delete=0.1, vmin=0, vmax=3, distinct=False)
        return [oracle.table_build(r, 256) for r in sets]
    if name == "ragged":  # ragged keys 0-48 B (the empty key repeats), empty values, DELETEs
        from test_gpu_compact_fuzz import ragged_sorted
        return [oracle.table_build(ragged_sorted(900 + 300 * t, 610 + t), 4096) for t in range(4)]
    if name == "one_table":
        return [oracle.table_build(W.compaction_inputs(1, 3000, 9000, seed=9)[0], 4096)]
    if name == "reftest":  # tests/test_mergeIterator.cc:65-184's data: "key<i>" -> "value<i>", txn 0
        return [oracle.table_build(_reftest_records(t), 4096) for t in range(REFTEST_TABLES)]
    raise KeyError(name)


REFTEST_TABLES, REFTEST_PER = 4, 5000


def _reftest_pairs(t):
    """table t of the reference's TableTest.MergeIterator shape: memtable t
    holds Put("key" + i, "value" + i, 0) for a consecutive range of i, flushed
    sorted by key (so "key10" < "key2")"""
    return sorted((f"key{i}".encode(), f"value{i}".encode()) for i in range(t * REFTEST_PER, (t + 1) * REFTEST_PER))


def _reftest_records(t):
    pairs = _reftest_pairs(t)
    n = len(pairs)
    kl = np.array([len(k) for k, _ in pairs], np.uint32)
    vl = np.array([len(v) for _, v in pairs], np.uint32)
    ko = np.concatenate([[0], np.cumsum(kl[:-1], dtype=np.uint64)]).astype(np.uint64)
    vo = np.concatenate([[0], np.cumsum(vl[:-1], dtype=np.uint64)]).astype(np.uint64)
    return {"type": np.zeros(n, np.uint8), "key_len": kl, "val_len": vl, "txn": np.zeros(n, np.uint64),
            "key_off": ko, "val_off": vo,
            "key_src": np.frombuffer(b"".join(k for k, _ in pairs), np.uint8).copy(),
            "val_src": np.frombuffer(b"".join(v for _, v in pairs), np.uint8).copy()}


MERGE_CASES = sorted(CJ) + ["ties_same", "ties_diff", "versions", "ragged", "one_table", "reftest"]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name", MERGE_CASES)
def test_merge_iterator_trace_equals_reference(oracle, tmp_path, name):
    """the drop-in db::MergeIterator (device merge,
    include/dropin/db/merge_iterator.h) against the reference's own
    merge_iterator.cc over the same TableReaderIterators: the whole
    SeekToFirst + Next walk (key, value incl. null vs empty views, type, txn
    as read, IsValid) and the reference's quirks after it -- SeekToLast +
    Prev gated by the MIN heap's IsValid (tests/test_mergeIterator.cc walks it
    so), a half walk then SeekToLast / Prev / Next / Seek / SeekToFirst --
    equal at every step.  The device merge serves every case but the
    differing-tie one, which takes the heap's own order (heap mode)."""
    need(EXE)
    need(REF_EXE)
    files = _merge_sets(name, oracle)
    args = []
    for i, f in enumerate(files):
        p = str(tmp_path / f"m{i}.sst")
        f.tofile(p)
        args += [p, str(f.size + 1)]
    mid = first_last_key(files[0])[1].hex() or "-"
    dumps = []
    runs = [(REF_EXE, "ref", {}), (EXE, "dropin", {"SSTC_TRACE_HOST": "1"}),
            (EXE, "heap", {"SSTC_DROPIN_HEAP_MERGE": "1"})]
    if name in ("small", "versions", "ties_diff") and os.path.exists(ASAN_EXE):
        runs.append((ASAN_EXE, "asan", ASAN_ENV))
    for exe, tag, env in runs:
        d = str(tmp_path / f"{tag}.dump")
        r = subprocess.run([exe, "--merge", d, mid] + args, capture_output=True, text=True, timeout=240,
                           env=dict(os.environ, **env))
        assert "AddressSanitizer" not in r.stderr, (tag, r.stderr[-3000:])
        assert r.returncode == 0, (tag, r.stderr[-2000:])
        if tag == "dropin":
            mode = "heap mode" if name == "ties_diff" else "device merge"
            assert f"MergeIterator over {len(files)} tables: {mode}" in r.stderr, r.stderr[-2000:]
        dumps.append((tag, r.stdout.strip(), open(d, "rb").read()))
    assert dumps[0][1].startswith("merge ok ") and len(dumps[0][2]) > 1000
    want = merge_steps(dumps[0][2])
    if name == "reftest":  # test_mergeIterator.cc's own expectations: the forward walk is the sorted
        # list of every pair, the SeekToLast + Prev loop after it is empty (IsValid reads the min heap)
        pairs = sorted(p for t in range(REFTEST_TABLES) for p in _reftest_pairs(t))
        fwd = [(x[4][1], x[5][1]) for x in want if x[0] == "N" and len(x) > 2]
        assert fwd[:len(pairs)] == pairs and len([x for x in want if x[0] == "N"]) >= len(pairs)
        first_pass = want[:want.index(("L", 0)) + 1] if ("L", 0) in want else want
        assert not any(x[0] == "P" for x in first_pass)
    for tag, out, dump in dumps[1:]:
        got = merge_steps(dump)
        bad = next((i for i, (a, b) in enumerate(zip(got, want)) if a != b), None)
        assert bad is None, (tag, bad, len(want), got[bad], want[bad])
        assert out == dumps[0][1] and dump == dumps[0][2], tag


def merge_steps(dump):
    """the --merge dump as (op, valid, type, txn, key, value) steps"""
    import struct
    out, i = [], 0

    def view():
        nonlocal i
        has, n = dump[i], struct.unpack_from("<I", dump, i + 1)[0]
        v = (has, bytes(dump[i + 5:i + 5 + n]))
        i += 5 + n
        return v
    while i < len(dump):
        op, valid = chr(dump[i]), dump[i + 1]
        i += 2
        if op in "EL" and (i >= len(dump) or chr(dump[i]) in "NPHLSF"):  # the no-read steps
            out.append((op, valid))
            continue
        typ, txn = dump[i], struct.unpack_from("<Q", dump, i + 1)[0]
        i += 9
        out.append((op, valid, typ, txn, view(), view()))
    return out
