"""Batched point lookups (sstc_get_batch) on config-3 SSTs: 8 tables x 1 M keys
(16 B keys, 100 B values), Q random queries (half present), device-resident.

    python tools/bench_lookup.py [--queries 4000000] [--steps 5]

Baseline: the reference's TableReader::GetValue without a block cache (one
pread + BlockReader parse + binary search per lookup; oracle/_ref
ref_table_get, 1 thread) on a bounded sample of the same queries.  Results of
all queries are compared with the oracle restatement (orc_table_get).
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lsm-kv-storage_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import sstcodec  # noqa: E402
from sstcodec import workload as W  # noqa: E402
from sstcodec.table import build_table  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tables", type=int, default=8)
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--queries", type=int, default=4_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--ref-sample", type=int, default=50_000)
    args = ap.parse_args()
    codec = sstcodec.Codec(0)
    td = tempfile.mkdtemp(prefix="sstc_get_")
    tables, paths = [], []
    for s in range(args.tables):
        i = np.arange(args.keys, dtype=np.uint64)
        rec = W.uniform_records(args.keys, key_index=i * np.uint64(args.tables) + np.uint64(s), seed=s + 1,
                                txn_start=1 + s * args.keys)
        p = os.path.join(td, f"{s}.sst")
        fs, _ = build_table(codec, p, rec, 4096)
        tables.append(np.fromfile(p, np.uint8))
        paths.append((p, fs))
    lk = sstcodec.Lookup(codec, tables)
    rng = np.random.default_rng(1)
    n = args.queries
    kidx = rng.integers(0, 2 * args.keys * args.tables, n)  # half the keys exist
    qt = (kidx % args.tables).astype(np.uint32)
    keys = [b"k%015d" % (k // 2 if k % 2 == 0 else 10 ** 14 + k) for k in kidx.tolist()]
    qt = np.where(kidx % 2 == 0, (kidx // 2) % args.tables, qt).astype(np.uint32)
    ot, ov, ol, ob = lk.get(qt, keys, raw=True)  # warm-up; device arrays
    torch.cuda.synchronize()
    # timed: the lookup kernel only (queries already resident), HIP events on the codec's stream
    import ctypes
    from sstcodec._lib import check
    from sstcodec.codec import _p, _queries
    arena, off, lens = _queries(keys)
    dev = codec.device
    qt_d = torch.from_numpy(qt.view(np.int32)).to(dev)
    qk = torch.from_numpy(arena).to(dev)
    qo = torch.from_numpy(off.view(np.int64)).to(dev)
    ql = torch.from_numpy(lens.view(np.int32)).to(dev)
    idx = lk.index()
    stream = torch.cuda.current_stream(dev)
    times = []
    for _ in range(args.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        codec._stream()
        e0.record(stream)
        check(codec.lib.sstc_get_batch(codec.h, _p(lk.src), ctypes.byref(idx), _p(qt_d), _p(qk), qk.numel(), _p(qo),
                                       _p(ql), n, _p(ot), _p(ov), _p(ol), _p(ob)), "sstc_get_batch")
        e1.record(stream)
        e1.synchronize()
        times.append(e0.elapsed_time(e1) / 1e3)
    typ = ot[:n].cpu().numpy().view(np.uint32)
    out = {"workload": f"lookup: {args.tables} SSTs x {args.keys} keys (config 3 tables), {n} random queries",
           "queries": n, "hits": int((typ == 0).sum()), "gpu_s_median": float(np.median(times)),
           "gpu_lookups_per_s": n / float(np.median(times))}
    try:
        from oracle import Oracle
        orc = Oracle()
        ok = True
        vo = ov[:n].cpu().numpy().view(np.uint64)
        base = np.cumsum([0] + [t.size for t in tables])
        for t in range(args.tables):
            sel = np.nonzero(qt == t)[0]
            o_t, o_vo, _, _ = orc.table_get(tables[t], [keys[i] for i in sel])
            ok &= bool(np.array_equal(typ[sel], o_t))
            put = o_t == 0
            ok &= bool(np.array_equal(vo[sel][put] - base[t], o_vo[put]))
        out["identical_to_oracle"] = ok
        from oracle import RefLib
        ref = RefLib()
        m = min(args.ref_sample, n)
        t0 = time.perf_counter()
        for t in range(args.tables):
            sel = [i for i in range(m) if qt[i] == t]
            ref.table_get(paths[t][0], paths[t][1], [keys[i] for i in sel])
        ref_s = time.perf_counter() - t0
        out["cpu_baseline"] = {"kind": "reference", "lookups_per_s": m / ref_s, "cores": 1,
                               "sample": f"first {m} queries, TableReader::GetValue without block cache"}
    except (FileNotFoundError, OSError) as e:
        out["cpu_baseline"] = f"unavailable: {e}"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
