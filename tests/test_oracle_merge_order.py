"""The merge-order model of tests/test_gpu_merge_records.py pinned on the CPU
against the reference itself: the reference's own db::MergeIterator over its
own TableReaderIterators (oracle/_ref/ref_pick_compact --merge, built from
/root/reference/db/merge_iterator.cc unchanged) walks the same inputs in
exactly the order the model builds from the oracle's block decode (key asc,
merge txn desc with the merge txn the running minimum over a key's group in its
input, lower input first, file order), txns as read included."""
import os
import subprocess

import pytest
from sstcodec import workload as W
from test_gpu_dropin import REF_EXE, merge_steps, need
from test_gpu_merge_records import _expected, fuzz_sets

CASES = {
    "overlap": lambda: W.compaction_inputs(5, 2000, 3000, seed=11, vmin=1, vmax=300),
    "versions": lambda: W.compaction_inputs(3, 1500, 50, seed=70, p_delete=0.1, vmin=0, vmax=3, distinct=False),
    "many_inputs": lambda: W.compaction_inputs(20, 400, 5000, seed=12, vmin=1, vmax=120, distinct=False),
    "one_input": lambda: W.compaction_inputs(1, 3000, 9000, seed=9),
    "empty_values": lambda: W.compaction_inputs(4, 800, 900, seed=13, vmin=0, vmax=0, distinct=False),
    "fuzz0": lambda: fuzz_sets(0),
    "fuzz3": lambda: fuzz_sets(3),
    "fuzz5": lambda: fuzz_sets(5),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_merge_order_model_equals_reference_merge_iterator(oracle, tmp_path, case):
    need(REF_EXE)
    files = [oracle.table_build(r, 4096) for r in CASES[case]()]
    args = []
    for i, img in enumerate(files):
        p = str(tmp_path / f"m{i}.sst")
        img.tofile(p)
        args += [p, str(img.size + 1)]
    dump = str(tmp_path / "ref.dump")
    r = subprocess.run([REF_EXE, "--merge", dump, "-"] + args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    want = _expected(oracle, files)
    walk = [(x[4][1], x[3]) for x in merge_steps(open(dump, "rb").read()) if x[0] == "N" and len(x) > 2]
    assert walk[:len(want)] == [(k, tx) for k, _, _, _, tx, _ in want]
    assert os.path.getsize(dump) > 0
