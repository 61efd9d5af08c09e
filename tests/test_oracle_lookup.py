"""CPU: the point-lookup restatement (orc_table_get: TableReader::GetValue ->
BlockReader::GetValue) against the reference's own lookups
(tests/golden/lookup.npz, made by oracle/_ref ref_table_get) and, when the
reference build is present, live on random tables with repeated keys."""
import os
import tempfile

import numpy as np
import pytest
from conftest import load_golden
from sstcodec import workload as W


def golden_queries(g, t):
    ka, ko, kl = g[f"q{t}_keys"], g[f"q{t}_key_off"], g[f"q{t}_key_len"]
    return [bytes(ka[int(o):int(o) + int(n)]) for o, n in zip(ko, kl)]


def golden_values(g, t):
    va, vo, vl = g[f"q{t}_val"], g[f"q{t}_val_off"], g[f"q{t}_val_len"]
    return [bytes(va[int(o):int(o) + int(n)]) for o, n in zip(vo, vl)]


@pytest.mark.parametrize("t", [0, 1])
def test_lookup_golden(oracle, t):
    g = load_golden("lookup.npz")
    img = g[f"sst{t}"]
    keys = golden_queries(g, t)
    typ, vo, vl, _ = oracle.table_get(img, keys)
    want_t = g[f"q{t}_type"]
    assert np.array_equal(typ, want_t)
    assert set(np.unique(want_t)) >= {0, 2} and (t == 1 or 1 in want_t)
    for i, v in enumerate(golden_values(g, t)):
        if typ[i] == 0:
            assert bytes(img[int(vo[i]):int(vo[i]) + int(vl[i])]) == v


def test_lookup_empty_table(oracle):
    img = oracle.table_build(W.compaction_inputs(1, 0, 10)[0], 4096)
    typ, _, _, blk = oracle.table_get(img, [b"a", b""])
    assert (typ == 2).all() and (blk == 2 ** 64 - 1).all()


def test_lookup_live_reference(oracle, reflib):
    for seed in range(3):
        rec = W.compaction_inputs(1, 2000, 3000, seed=30 + seed, vmax=[50, 900, 5000][seed], p_delete=0.3,
                                  distinct=seed == 1)[0]
        img = oracle.table_build(rec, [4096, 4096, 32768][seed])
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "t.sst")
            img.tofile(p)
            keys = [b"k%015d" % i for i in range(0, 3000, 1)] + [b"", b"k", b"l"]
            rt, rv = reflib.table_get(p, img.size + 1, keys)
        typ, vo, vl, _ = oracle.table_get(img, keys)
        assert np.array_equal(typ, rt)
        for i in range(len(keys)):
            if typ[i] == 0:
                assert bytes(img[int(vo[i]):int(vo[i]) + int(vl[i])]) == rv[i]


def test_lookup_config3_matches_reference(oracle):
    """40 000 seeded point lookups over the 8 config-3 SSTs (1 M keys each):
    the oracle's TableReader::GetValue restatement gives the reference's types,
    value lengths and values (tests/golden/compaction_configs.json)."""
    import hashlib
    import json
    import os
    from conftest import GOLDEN
    from sstcodec import workload as W
    case = json.load(open(os.path.join(GOLDEN, "compaction_configs.json")))["lookup_config3"]
    qt, qk = W.config3_lookup_queries(case["queries"], case["seed"])
    keys = W.fixed_keys(qk).reshape(-1, 16)
    types = np.zeros(len(qt), np.uint32)
    vlens = np.zeros(len(qt), np.uint32)
    vals = [b""] * len(qt)
    for t, rec in enumerate(W.config_inputs(3)):
        img = oracle.table_build(rec, 4096)
        assert img.size + 1 == case["inputs"][t]["file_size"]
        sel = np.flatnonzero(qt == t)
        ty, vo, vl, _ = oracle.table_get(img, [bytes(keys[j]) for j in sel])
        for j, a, o, n in zip(sel, ty, vo, vl):
            types[j] = a
            if a == 0:
                vals[j] = bytes(img[int(o):int(o) + int(n)])
                vlens[j] = n
    assert hashlib.sha256(types.tobytes()).hexdigest() == case["types_sha256"]
    assert hashlib.sha256(vlens.tobytes()).hexdigest() == case["val_len_sha256"]
    assert hashlib.sha256(b"".join(vals)).hexdigest() == case["values_sha256"]
