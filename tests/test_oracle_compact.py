"""CPU: the compaction restatement (orc_compact) against outputs of the
reference's own MergeIterator + TableBuilder (tests/golden/compaction.json,
compact_small_*.npz, made by oracle/_ref/ref_compact)."""
import hashlib
import json
import os
import tempfile

import numpy as np
import pytest
from conftest import GOLDEN, load_golden
from sstcodec import workload as W

CASES = json.load(open(os.path.join(GOLDEN, "compaction.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint8).tobytes()).hexdigest()


def build_inputs(oracle, case):
    sets = W.compaction_inputs(case["k"], case["n_per"], case["key_space"], vmax=case["vmax"],
                               distinct=case["distinct"], **case.get("gen", {}))
    return [oracle.table_build(rec, case["block_threshold"]) for rec in sets]


@pytest.mark.parametrize("name", sorted(CASES))
def test_inputs_match_reference_tablebuilder(oracle, name):
    case = CASES[name]
    files = build_inputs(oracle, case)
    for f, want in zip(files, case["inputs"]):
        assert sha(f) == want["sha256"] and f.size + 1 == want["file_size"]


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("base", [1, 0])
def test_compact_matches_reference(oracle, name, base):
    case = CASES[name]
    files = build_inputs(oracle, case)
    outs, kept = oracle.compact(files, case["block_threshold"], case["table_limit"], base)
    want = case[f"outputs_base{base}"]
    assert len(outs) == len(want)
    for o, w in zip(outs, want):
        assert o.size + 1 == w["file_size"] and sha(o) == w["sha256"]


@pytest.mark.parametrize("base", [1, 0])
def test_compact_small_bytes(oracle, base):
    g = load_golden(f"compact_small_base{base}.npz")
    ins = [g[f"in{i}"] for i in range(4)]
    outs, _ = oracle.compact(ins, 4096, 32 << 20, base)
    assert len(outs) == len([k for k in g if k.startswith("out")])
    for j, o in enumerate(outs):
        assert np.array_equal(o, g[f"out{j}"])


def test_live_ref_compact(oracle):
    from oracle import REF_COMPACT, ref_compact
    if not os.path.exists(REF_COMPACT):
        pytest.skip("reference compaction driver not built")
    sets = W.compaction_inputs(6, 700, 900, seed=99, vmax=300, p_delete=0.3)
    with tempfile.TemporaryDirectory() as td:
        ins, files = [], []
        for i, rec in enumerate(sets):
            f = oracle.table_build(rec, 4096)
            p = os.path.join(td, f"i{i}.sst")
            f.tofile(p)
            ins.append((p, f.size + 1))
            files.append(f)
        od = os.path.join(td, "o")
        os.makedirs(od)
        outs = ref_compact(ins, od, 4096, 40_000, 1)
        mine, _ = oracle.compact(files, 4096, 40_000, 1)
        assert len(outs) == len(mine) > 2
        for (p, fs), m in zip(outs, mine):
            assert np.array_equal(np.fromfile(p, np.uint8), m) and fs == m.size + 1


CONFIGS = json.load(open(os.path.join(GOLDEN, "compaction_configs.json")))


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_config_full_size_matches_reference(oracle, name):
    """BASELINE configs 3 / 3-overlap / 4 (rank-0 shard) / 5 at full size: the
    oracle's inputs equal the reference TableBuilder's files and its compaction
    equals the reference's outputs (tests/golden/make_golden_configs.py)."""
    case = CONFIGS[name]
    files = [oracle.table_build(r, case["block_threshold"]) for r in W.config_inputs(**case["gen"])]
    for f, want in zip(files, case["inputs"]):
        assert f.size + 1 == want["file_size"] and sha(f) == want["sha256"]
    outs, _ = oracle.compact(files, case["block_threshold"], case["table_limit"], 1)
    want = case["outputs_base1"]
    assert len(outs) == len(want)
    for o, w in zip(outs, want):
        assert o.size + 1 == w["file_size"] and sha(o) == w["sha256"]
