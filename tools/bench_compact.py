"""Config 3 (BASELINE.json): full L0->L1 compaction re-encode of 8 input SSTs x
1 M keys (16 B keys, 100 B values) on one GPU, device-resident.

    python tools/bench_compact.py [--keys 1000000] [--ssts 8] [--overlap] [--steps 3]

Inputs: SST s holds keys k%015d of i*8+s (disjoint interleave),
or with --overlap the same key set in every SST with distinct txns (exercises
the drop path).  They are written by this framework's TableBuilder (bit-exact
with the reference's, tests/test_gpu_table.py).  Timed: sstc_compact on the
resident input (decode, merge, filter, split, encode, meta, footers).
Baseline: the reference's own MergeIterator + TableBuilder driver
(oracle/_ref/ref_compact, includes its file I/O), when present; outputs are
compared by SHA-256.
"""
import argparse
import ctypes
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lsm-kv-storage_amd"))
import sstcodec  # noqa: E402
from sstcodec import workload as W  # noqa: E402
from sstcodec._lib import CompactParams, CompactResult, check  # noqa: E402
from sstcodec.codec import _table_index  # noqa: E402
from sstcodec.table import build_table  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--ssts", type=int, default=8)
    ap.add_argument("--overlap", action="store_true")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--no-ref", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    codec = sstcodec.Codec(0)
    td = tempfile.mkdtemp(prefix="sstc_c3_")
    files, paths = [], []
    t0 = time.perf_counter()
    for s in range(args.ssts):
        i = np.arange(args.keys, dtype=np.uint64)
        keys = i if args.overlap else i * np.uint64(args.ssts) + np.uint64(s)
        rec = W.uniform_records(args.keys, key_index=keys, seed=s + 1,
                                txn_start=1 + s * args.keys)
        p = os.path.join(td, f"{s}.sst")
        fs, _ = build_table(codec, p, rec, 4096)
        files.append(np.fromfile(p, np.uint8))
        paths.append((p, fs))
    gen_s = time.perf_counter() - t0
    offs, lens, tfb, base = [], [], [0], 0
    for f in files:
        o, ln = _table_index(f)
        offs.append(o + np.uint64(base))
        lens.append(ln)
        tfb.append(tfb[-1] + len(o))
        base += f.size
    src = torch.from_numpy(np.concatenate(files)).to(dev)
    bo = torch.from_numpy(np.concatenate(offs).view(np.int64)).to(dev)
    bl = torch.from_numpy(np.concatenate(lens).view(np.int64)).to(dev)
    h_tfb = np.asarray(tfb, np.uint64)
    cap = int(src.numel()) + (1 << 20)
    dst = torch.empty(cap, dtype=torch.uint8, device=dev)
    max_t = 4096
    toff = torch.zeros(max_t + 1, dtype=torch.int64, device=dev)
    tlen = torch.zeros(max_t, dtype=torch.int64, device=dev)
    prm = CompactParams(4096, 32 << 20, 1, 0)
    res = CompactResult()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def run():
        codec._stream()
        check(codec.lib.sstc_compact(codec.h, P(src), P(bo), P(bl), int(bo.numel()),
                                     h_tfb.ctypes.data_as(ctypes.c_void_p), len(files), ctypes.byref(prm), P(dst),
                                     cap, P(toff), P(tlen), max_t, ctypes.byref(res)), "sstc_compact")

    run()  # warm-up (also the verified output)
    torch.cuda.synchronize()
    times = []
    for _ in range(args.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    nt = res.tables_out
    o = toff[: nt + 1].cpu().numpy()
    d = dst[: int(o[nt])].cpu().numpy()
    gpu_hash = [hashlib.sha256(d[int(o[t]):int(o[t + 1])].tobytes()).hexdigest() for t in range(nt)]
    in_bytes = int(src.numel())
    out = {"workload": "config3" + ("-overlap" if args.overlap else ""), "ssts": args.ssts, "keys_per_sst": args.keys,
           "input_bytes": in_bytes, "records_in": res.records_in, "records_kept": res.records_kept,
           "tables_out": nt, "blocks_out": res.blocks_out, "bytes_out": res.bytes_out,
           "gpu_s_median": float(np.median(times)), "gpu_GiBps_in": in_bytes / np.median(times) / 2 ** 30,
           "input_build_s": gen_s, "output_sizes_head": [int(x) + 1 for x in tlen[:min(nt, 4)].cpu().tolist()]}
    ref = os.path.join(ROOT, "oracle", "_ref", "ref_compact")
    if not args.no_ref and os.path.exists(ref):
        od = os.path.join(td, "ref_out")
        os.makedirs(od)
        cmd = [ref, od, "4096", str(32 << 20), "1"]
        for p, fs in paths:
            cmd += [p, str(fs)]
        t0 = time.perf_counter()
        r = subprocess.run(cmd, check=True, capture_output=True, text=True)
        ref_s = time.perf_counter() - t0
        lines = [ln.rsplit(" ", 1) for ln in r.stdout.strip().splitlines()]
        ref_hash = [hashlib.sha256(open(p, "rb").read()).hexdigest() for p, _ in lines]
        out["cpu_baseline"] = {"kind": "reference", "seconds": ref_s, "GiBps_in": in_bytes / ref_s / 2 ** 30,
                               "cores": 1, "what": "reference MergeIterator + TableReaderIterator + TableBuilder "
                                                   "(oracle/_ref/ref_compact), files on local disk incl. fsync"}
        out["bit_exact_vs_reference"] = ref_hash == gpu_hash
        out["ref_tables"] = len(ref_hash)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
