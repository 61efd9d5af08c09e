"""Rebuild the AS-WRITTEN reference compaction output from the build's output
plus the attributed record list (tests/golden/aswritten_<case>.npz).

db/compact.cc as written keeps some older duplicates that the build (and the
fixed-semantics fixtures) drop: its `string_view last_current_key` dangles
after a block switch (compact.cc:250,266-268).  The compaction order is the
same in both, (key asc, txn desc) (merge_iterator.h:91-95), so

    as-written stream = sort_by_merge_order(build stream  U  extra records)

and the as-written output files are that stream cut greedily at
GetDataSize() >= limit (compact.cc:289-301) and written by a TableBuilder.
Every record is an input record, named by (input table, record index); txns
are unique across the inputs of every attributed case.
"""
import numpy as np

NO_VALUE = 0xFFFFFFFF


def refs_by_txn(sets, txns):
    """(table, index) of each txn in the input record sets."""
    all_tx = np.concatenate([s["txn"].astype(np.uint64) for s in sets])
    tab = np.concatenate([np.full(len(s["txn"]), t, np.uint32) for t, s in enumerate(sets)])
    idx = np.concatenate([np.arange(len(s["txn"]), dtype=np.uint32) for s in sets])
    order = np.argsort(all_tx, kind="stable")
    pos = np.searchsorted(all_tx[order], np.asarray(txns, np.uint64))
    assert np.all(all_tx[order][pos] == np.asarray(txns, np.uint64)), "txn not in the inputs"
    return tab[order][pos], idx[order][pos]


def gather(sets, tab, idx):
    """Record set (sstcodec.workload layout) of the given input records, in order."""
    n = len(tab)
    out = {k: np.zeros(n, dt) for k, dt in (("type", np.uint8), ("key_len", np.uint32), ("val_len", np.uint32),
                                            ("txn", np.uint64))}
    kparts, vparts = [], []
    key_off = np.zeros(n, np.uint64)
    val_off = np.zeros(n, np.uint64)
    for t, s in enumerate(sets):
        sel = np.flatnonzero(tab == t)
        if sel.size == 0:
            continue
        i = idx[sel]
        for k in ("type", "key_len", "val_len", "txn"):
            out[k][sel] = s[k][i]
        # keys / values stay in their table's arenas: concatenate arenas, rebase
        kbase = sum(p.size for p in kparts)
        vbase = sum(p.size for p in vparts)
        kparts.append(s["key_src"])
        vparts.append(s["val_src"])
        key_off[sel] = s["key_off"][i].astype(np.uint64) + np.uint64(kbase)
        val_off[sel] = np.where(s["val_len"][i] == NO_VALUE, 0, s["val_off"][i].astype(np.uint64) + np.uint64(vbase))
    out["key_off"] = key_off
    out["val_off"] = val_off.astype(np.uint64)
    out["key_src"] = np.concatenate(kparts) if kparts else np.zeros(0, np.uint8)
    out["val_src"] = np.concatenate(vparts) if vparts else np.zeros(0, np.uint8)
    return out


def merge_order(rec):
    """Permutation putting records in (key asc, txn desc) order (fixed-width keys)."""
    kl = rec["key_len"]
    w = int(kl[0]) if len(kl) else 0
    assert np.all(kl == w), "merge_order handles fixed-width keys (all attributed cases)"
    keys = np.stack([rec["key_src"][rec["key_off"].astype(np.int64) + j] for j in range(w)]) if w else np.zeros((0, 0))
    cols = [~rec["txn"].astype(np.uint64)] + [keys[j] for j in range(w - 1, -1, -1)]
    return np.lexsort(cols)


def take(rec, perm):
    out = {k: rec[k][perm] for k in ("type", "key_len", "val_len", "txn", "key_off", "val_off")}
    out["key_src"], out["val_src"] = rec["key_src"], rec["val_src"]
    return out


def table_cuts(rec, limit):
    """[lo, hi) record ranges of the output tables: a table is finished right
    after the record that brings its data size (key + value bytes,
    table_builder.cc:55) to >= limit (compact.cc:289-301)."""
    vl = rec["val_len"].astype(np.uint64)
    ds = rec["key_len"].astype(np.uint64) + np.where(rec["val_len"] == NO_VALUE, np.uint64(0), vl)
    cs = np.concatenate([[0], np.cumsum(ds, dtype=np.uint64)])
    n = len(ds)
    cuts, lo = [], 0
    while lo < n:
        hi = int(np.searchsorted(cs, cs[lo] + np.uint64(limit), side="left"))  # first j with cs[j]-cs[lo] >= limit
        hi = n if hi > n else hi
        cuts.append((lo, hi))
        lo = hi
    return cuts


def slice_rec(rec, lo, hi):
    out = {k: rec[k][lo:hi] for k in ("type", "key_len", "val_len", "txn", "key_off", "val_off")}
    out["key_src"], out["val_src"] = rec["key_src"], rec["val_src"]
    return out


def aswritten_tables(sets, build_txns, extra_table, extra_index, limit):
    """Record sets of the as-written output tables: the build's kept records
    (by txn) plus the attributed extras, in merge order, cut at `limit`."""
    bt, bi = refs_by_txn(sets, build_txns)
    tab = np.concatenate([bt, np.asarray(extra_table, np.uint32)])
    idx = np.concatenate([bi, np.asarray(extra_index, np.uint32)])
    rec = gather(sets, tab, idx)
    rec = take(rec, merge_order(rec))
    return [slice_rec(rec, lo, hi) for lo, hi in table_cuts(rec, limit)]
