"""Flush-path encode (db/db_impl.cc:403-440: memtable ->
TableBuilder): one SST of N uniform records (16 B keys / 100 B values, the
config-3 input SST) written by

  gpu  sstc::TableBuilder (AddEntry per record on the host, GPU block encode at
       Finish, one pwrite + fsync), through the C shim's batch add;
  ref  the reference's own TableBuilder (oracle/_ref, per-entry BlockBuilder,
       three pwrite64 per block, fsync), 1 thread.

Both files are compared byte for byte.  Prints one JSON line.

    python tools/bench_flush.py [--records 1000000] [--reps 3]
"""
import argparse
import hashlib
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lsm-kv-storage_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import sstcodec  # noqa: E402
from sstcodec import workload as W  # noqa: E402
from sstcodec.table import build_table  # noqa: E402


def sha(p):
    return hashlib.sha256(open(p, "rb").read()).hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    rec = W.uniform_records(args.records, seed=1)
    codec = sstcodec.Codec(0)
    out = {"records": args.records, "what": "one SST, 16 B keys / 100 B values, 4096 B blocks"}
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "gpu.sst")
        build_table(codec, p, rec, 4096)  # warm-up (context workspace, code objects)
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            fs, nb = build_table(codec, p, rec, 4096)
            ts.append(time.perf_counter() - t0)
        out["gpu"] = {"seconds_median": sorted(ts)[len(ts) // 2], "file_size": fs, "blocks": nb}
        # phase split of one more build: AddEntries (host bookkeeping) vs Finish
        # (pack + H2D + GPU encode + D2H + meta/footer + pwrite + fsync)
        import ctypes
        import numpy as np
        from sstcodec.table import _sig, _p
        from sstcodec._lib import load
        lib = _sig(load())
        r = {k: np.ascontiguousarray(v) for k, v in rec.items()}
        tb = ctypes.c_void_p()
        codec._stream()
        lib.sstc_tb_create(p.encode(), 4096, codec.h, ctypes.byref(tb))
        lib.sstc_tb_open(tb)
        t0 = time.perf_counter()
        lib.sstc_tb_add_batch(tb, args.records, _p(r["type"]), _p(r["key_len"]), _p(r["val_len"]), _p(r["txn"]),
                              _p(r["key_src"]), _p(r["key_off"]), _p(r["val_src"]), _p(r["val_off"]))
        t1 = time.perf_counter()
        lib.sstc_tb_finish(tb)
        t2 = time.perf_counter()
        lib.sstc_tb_destroy(tb)
        out["gpu"]["phases_s"] = {"add_entries": round(t1 - t0, 4), "finish": round(t2 - t1, 4)}
        try:
            from oracle import RefLib
            ref = RefLib()
            q = os.path.join(td, "ref.sst")
            t0 = time.perf_counter()
            rfs = ref.table_build(q, rec, 4096)
            out["ref"] = {"seconds": time.perf_counter() - t0, "file_size": rfs, "cores": 1,
                          "kind": "reference TableBuilder (oracle/_ref), per-entry BlockBuilder + pwrite64 per block"}
            out["bit_exact_vs_reference"] = sha(p) == sha(q) and rfs == fs
        except (FileNotFoundError, OSError):
            pass
    mb = fs / 1e6
    out["gpu"]["MBps"] = round(mb / out["gpu"]["seconds_median"], 1)
    if "ref" in out:
        out["ref"]["MBps"] = round(mb / out["ref"]["seconds"], 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
