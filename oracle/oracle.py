"""ctypes wrappers of the CPU checkers (TEST INFRASTRUCTURE ONLY).

    Oracle  -> oracle/liboracle.so       clean-room C restatement (sst_oracle.c)
    RefLib  -> oracle/_ref/libsstref.so  the reference's own sstable sources
                                          (+ ref_harness.cc), built by
                                          oracle/Makefile when /root/reference
                                          is present

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this
module, always as the checker / the CPU baseline, never as the product path.
Record sets use the layout of sstcodec.workload (numpy arrays).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libsstref.so")
NO_VALUE = 0xFFFFFFFF

_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64


def build(quiet=True):
    """Build liboracle.so (and _ref/libsstref.so when /root/reference exists)."""
    subprocess.run(["make", "-C", HERE, "-j8"], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


def _ptr(a):
    return a.ctypes.data_as(_vp) if a is not None else _vp(0)


def _rec_args(rec):
    r = {k: np.ascontiguousarray(rec[k]) for k in
         ("type", "key_len", "val_len", "txn", "key_off", "val_off", "key_src", "val_src")}
    r["type"] = r["type"].astype(np.uint8, copy=False)
    r["key_len"] = r["key_len"].astype(np.uint32, copy=False)
    r["val_len"] = r["val_len"].astype(np.uint32, copy=False)
    for k in ("txn", "key_off", "val_off"):
        r[k] = r[k].astype(np.uint64, copy=False)
    if r["key_src"].size == 0:
        r["key_src"] = np.zeros(8, np.uint8)
    if r["val_src"].size == 0:
        r["val_src"] = np.zeros(8, np.uint8)
    return r


def entry_sizes(rec):
    vl = rec["val_len"].astype(np.uint64)
    has = rec["val_len"] != NO_VALUE
    return np.uint64(13) + rec["key_len"].astype(np.uint64) + np.where(has, np.uint64(4) + vl, np.uint64(0))


def block_bytes(rec, lo=0, hi=None):
    hi = len(rec["type"]) if hi is None else hi
    s = entry_sizes({k: rec[k][lo:hi] for k in ("key_len", "val_len")})
    return int(s.sum()) + 16 * (hi - lo) + 16


class Oracle:
    """liboracle.so: the clean-room restatement."""

    def __init__(self, path=ORACLE_SO):
        if not os.path.exists(path):
            build()
        self.lib = lib = ctypes.CDLL(path)
        lib.orc_block_encode.restype = _u64
        lib.orc_block_encode.argtypes = [_u64] + [_vp] * 9
        lib.orc_block_decode.restype = ctypes.c_int
        lib.orc_block_decode.argtypes = [_vp, _u64, _u64, ctypes.c_int] + [_vp] * 7
        lib.orc_roundtrip_blocks.restype = _u64
        lib.orc_roundtrip_blocks.argtypes = [_vp, _vp, _vp, _u64, ctypes.c_int, _vp, _vp, _vp]
        lib.orc_segment.restype = _u64
        lib.orc_segment.argtypes = [_u64, _vp, _vp, _u64, _vp]
        lib.orc_table_build.restype = _u64
        lib.orc_table_build.argtypes = [_u64] + [_vp] * 8 + [_u64, _vp]
        lib.orc_table_index.restype = _u64
        lib.orc_table_index.argtypes = [_vp, _u64, _u64] + [_vp] * 8
        lib.orc_compact.restype = _u64
        lib.orc_compact.argtypes = [ctypes.c_uint32, _vp, _vp, _u64, _u64, ctypes.c_int, _vp, _u64, _vp, _u64, _vp]
        lib.orc_table_get.restype = ctypes.c_int
        lib.orc_table_get.argtypes = [_vp, _u64, _u64] + [_vp] * 7

    def encode_block(self, rec, lo=0, hi=None):
        hi = len(rec["type"]) if hi is None else hi
        r = _rec_args(rec)
        out = np.zeros(block_bytes(rec, lo, hi) + 16, np.uint8)
        sl = lambda k: _ptr(r[k][lo:]) if hi > lo else _ptr(r[k])  # noqa: E731
        n = self.lib.orc_block_encode(hi - lo, sl("type"), sl("key_len"), sl("val_len"), sl("txn"),
                                      _ptr(r["key_src"]), sl("key_off"), _ptr(r["val_src"]), sl("val_off"),
                                      _ptr(out))
        return out[:n]

    def encode_blocks(self, rec, blk_first, base=0):
        """Blocks for record ranges blk_first[b]..blk_first[b+1], back to back."""
        parts, offs, lens = [], [], []
        pos = base
        for b in range(len(blk_first) - 1):
            blk = self.encode_block(rec, int(blk_first[b]), int(blk_first[b + 1]))
            parts.append(blk)
            offs.append(pos)
            lens.append(blk.size)
            pos += blk.size
        data = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
        return data, np.asarray(offs, np.uint64), np.asarray(lens, np.uint64)

    def decode_block(self, blk, txn_mode=0, base=0):
        blk = np.ascontiguousarray(blk, dtype=np.uint8)
        cap = max(blk.size // 13 + 1, 1)
        out = {"type": np.zeros(cap, np.uint8), "key_len": np.zeros(cap, np.uint32),
               "val_len": np.zeros(cap, np.uint32), "txn": np.zeros(cap, np.uint64),
               "key_off": np.zeros(cap, np.uint64), "val_off": np.zeros(cap, np.uint64)}
        n = _u64()
        st = self.lib.orc_block_decode(_ptr(blk), blk.size, base, txn_mode, _ptr(out["type"]),
                                       _ptr(out["key_len"]), _ptr(out["val_len"]), _ptr(out["txn"]),
                                       _ptr(out["key_off"]), _ptr(out["val_off"]), ctypes.byref(n))
        k = min(n.value, cap)
        return st, {key: v[:k] for key, v in out.items()}

    def roundtrip(self, src, blk_off, blk_len, txn_mode=0):
        src = np.ascontiguousarray(src, np.uint8)
        blk_off = np.ascontiguousarray(blk_off, np.uint64)
        blk_len = np.ascontiguousarray(blk_len, np.uint64)
        dst = np.zeros_like(src)
        nb = blk_off.size
        out_len = np.zeros(max(nb, 1), np.uint64)
        status = np.zeros(max(nb, 1), np.uint32)
        bad = self.lib.orc_roundtrip_blocks(_ptr(src), _ptr(blk_off), _ptr(blk_len), nb, txn_mode, _ptr(dst),
                                            _ptr(out_len), _ptr(status))
        return dst, out_len[:nb], status[:nb], bad

    def segment(self, rec, threshold):
        r = _rec_args(rec)
        n = len(r["type"])
        first = np.zeros(n + 1, np.uint64)
        nb = self.lib.orc_segment(n, _ptr(r["key_len"]), _ptr(r["val_len"]), threshold, _ptr(first))
        return first[: nb + 1]

    def table_build(self, rec, threshold):
        r = _rec_args(rec)
        n = len(r["type"])
        args = [n, _ptr(r["type"]), _ptr(r["key_len"]), _ptr(r["val_len"]), _ptr(r["txn"]),
                _ptr(r["key_src"]), _ptr(r["key_off"]), _ptr(r["val_src"]), _ptr(r["val_off"]), threshold]
        size = self.lib.orc_table_build(*args, _vp(0))
        out = np.zeros(size, np.uint8)
        self.lib.orc_table_build(*args, _ptr(out))
        return out

    def table_index(self, file_bytes, cap=1 << 20):
        f = np.ascontiguousarray(file_bytes, np.uint8)
        cap = min(cap, f.size // 24 + 1)
        o = {k: np.zeros(cap, np.uint64) for k in ("blk_off", "blk_len", "first_key_off", "last_key_off")}
        o["first_key_len"] = np.zeros(cap, np.uint32)
        o["last_key_len"] = np.zeros(cap, np.uint32)
        mn, mx = _u64(), _u64()
        nb = self.lib.orc_table_index(_ptr(f), f.size, cap, _ptr(o["blk_off"]), _ptr(o["blk_len"]),
                                      _ptr(o["first_key_off"]), _ptr(o["first_key_len"]),
                                      _ptr(o["last_key_off"]), _ptr(o["last_key_len"]),
                                      ctypes.byref(mn), ctypes.byref(mx))
        if nb == 2 ** 64 - 1:
            return None
        k = min(nb, cap)
        res = {key: v[:k] for key, v in o.items()}
        res["nblocks"] = nb
        res["min_txn"] = mn.value
        res["max_txn"] = mx.value
        return res


def queries_arena(keys):
    """list of bytes -> (arena u8, off u64, len u32)"""
    lens = np.array([len(k) for k in keys], np.uint32)
    off = np.zeros(len(keys), np.uint64)
    if len(keys) > 1:
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    arena = np.frombuffer(b"".join(keys) + b"\0" * 8, np.uint8).copy()
    return arena, off, lens


def _table_get_oracle(self, file_bytes, keys):
    """Point lookups of TableReader::GetValue on one SST image.  Returns
    (type u32[], val_off u64[] into the image, val_len u32[], block u64[])."""
    f = np.ascontiguousarray(file_bytes, np.uint8)
    arena, off, lens = queries_arena(keys)
    n = len(keys)
    t = np.zeros(max(n, 1), np.uint32)
    vo = np.zeros(max(n, 1), np.uint64)
    vl = np.zeros(max(n, 1), np.uint32)
    blk = np.zeros(max(n, 1), np.uint64)
    rc = self.lib.orc_table_get(_ptr(f), f.size, n, _ptr(arena), _ptr(off), _ptr(lens), _ptr(t), _ptr(vo),
                                _ptr(vl), _ptr(blk))
    if rc != 0:
        return None
    return t[:n], vo[:n], vl[:n], blk[:n]


Oracle.table_get = _table_get_oracle


def _compact_oracle(self, files, block_threshold=4096, table_limit=32 << 20, base_level=1):
    """files: list of SST images (numpy u8) in iterator order.  Returns the list
    of output SST images and the kept-record count."""
    k = len(files)
    arrs = [np.ascontiguousarray(f, np.uint8) for f in files]
    ptrs = (ctypes.c_void_p * max(k, 1))(*[a.ctypes.data for a in arrs])
    sizes = np.array([a.size for a in arrs] or [0], np.uint64)
    cap = int(sum(a.size for a in arrs)) * 2 + 4096
    out = np.zeros(cap, np.uint8)
    max_t = cap // 40 + 1
    osz = np.zeros(max_t, np.uint64)
    kept = _u64()
    nt = self.lib.orc_compact(k, ptrs, _ptr(sizes), block_threshold, table_limit, base_level, _ptr(out), cap,
                              _ptr(osz), max_t, ctypes.byref(kept))
    if nt == 2 ** 64 - 1:
        raise ValueError("orc_compact failed")
    res, pos = [], 0
    for t in range(nt):
        res.append(out[pos:pos + int(osz[t])].copy())
        pos += int(osz[t])
    return res, kept.value


Oracle.compact = _compact_oracle

REF_COMPACT = os.path.join(HERE, "_ref", "ref_compact")


def ref_compact(paths_and_sizes, out_dir, block_threshold=4096, table_limit=32 << 20, base_level=1):
    """Run the reference-code compaction driver (oracle/_ref/ref_compact).
    Returns [(path, GetFileSize())]."""
    args = [REF_COMPACT, out_dir, str(block_threshold), str(table_limit), str(base_level)]
    for p, s in paths_and_sizes:
        args += [p, str(int(s))]
    r = subprocess.run(args, check=True, capture_output=True, text=True)
    out = []
    for line in r.stdout.strip().splitlines():
        p, s = line.rsplit(" ", 1)
        out.append((p, int(s)))
    return out


REF_PICK_COMPACT = os.path.join(HERE, "_ref", "ref_pick_compact")
COMPACT_DROPIN = os.path.join(HERE, "_ref", "compact_dropin")


def table_key_range(rec):
    """(smallest, largest) key of a sorted record set (what VersionEdit::AddNewFiles
    records for a flushed table, db_impl.cc:430-436)."""
    n = len(rec["type"])
    ko, kl, src = rec["key_off"], rec["key_len"], rec["key_src"]
    first = bytes(src[int(ko[0]):int(ko[0]) + int(kl[0])])
    last = bytes(src[int(ko[n - 1]):int(ko[n - 1]) + int(kl[n - 1])])
    return first, last


def ref_pick_compact(inputs, db_dir, block_threshold=4096, table_limit=32 << 20, exe=REF_PICK_COMPACT, env=None):
    """Run the reference's Compact::PickCompact (db/compact.cc compiled
    unchanged, oracle/ref_pick_compact.cc) over L0 tables 1..k.
    inputs: [(path, file_size, smallest_key_bytes, largest_key_bytes)].
    Returns (picked table ids, [(path, GetFileSize(), smallest, largest)])."""
    args = [exe, db_dir, str(block_threshold), str(table_limit)]
    for p, s, lo, hi in inputs:
        args += [p, str(int(s)), lo.hex() or "-", hi.hex() or "-"]
    r = subprocess.run(args, check=True, capture_output=True, text=True, env=env)
    picked, out = [], []
    for line in r.stdout.strip().splitlines():
        f = line.split(" ")
        if f[0] == "in":
            picked.append(int(f[1]))
        elif f[0] == "out":
            unhex = lambda h: b"" if h == "-" else bytes.fromhex(h)  # noqa: E731
            out.append((f[1], int(f[2]), unhex(f[3]), unhex(f[4])))
    return picked, out


class RefLib:
    """oracle/_ref/libsstref.so: the reference's own sstable code."""

    def __init__(self, path=REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.lib = lib = ctypes.CDLL(path)
        lib.ref_block_encode.restype = _u64
        lib.ref_block_encode.argtypes = [_u64] + [_vp] * 9
        lib.ref_block_decode.restype = _u64
        lib.ref_block_decode.argtypes = [_vp, _u64] + [_vp] * 6
        lib.ref_roundtrip_blocks.restype = _u64
        lib.ref_roundtrip_blocks.argtypes = [_vp, _vp, _vp, _u64, _vp, _vp]
        lib.ref_table_build.restype = _u64
        lib.ref_table_build.argtypes = [ctypes.c_char_p, _u64, _u64] + [_vp] * 8
        lib.ref_table_index.restype = _u64
        lib.ref_table_index.argtypes = [ctypes.c_char_p, _u64, _u64] + [_vp] * 6
        lib.ref_table_get.restype = _u64
        lib.ref_table_get.argtypes = [ctypes.c_char_p, _u64, _u64] + [_vp] * 7 + [_u64]

    def encode_block(self, rec, lo=0, hi=None):
        hi = len(rec["type"]) if hi is None else hi
        r = _rec_args(rec)
        out = np.zeros(block_bytes(rec, lo, hi) + 16, np.uint8)
        sl = lambda k: _ptr(r[k][lo:]) if hi > lo else _ptr(r[k])  # noqa: E731
        n = self.lib.ref_block_encode(hi - lo, sl("type"), sl("key_len"), sl("val_len"), sl("txn"),
                                      _ptr(r["key_src"]), sl("key_off"), _ptr(r["val_src"]), sl("val_off"),
                                      _ptr(out))
        return out[:n]

    def decode_block(self, blk):
        blk = np.ascontiguousarray(blk, np.uint8)
        cap = max(blk.size // 13 + 1, 1)
        out = {"type": np.zeros(cap, np.uint8), "key_len": np.zeros(cap, np.uint32),
               "val_len": np.zeros(cap, np.uint32), "txn": np.zeros(cap, np.uint64),
               "key_off": np.zeros(cap, np.uint64), "val_off": np.zeros(cap, np.uint64)}
        n = self.lib.ref_block_decode(_ptr(blk), blk.size, _ptr(out["type"]), _ptr(out["key_len"]),
                                      _ptr(out["val_len"]), _ptr(out["txn"]), _ptr(out["key_off"]),
                                      _ptr(out["val_off"]))
        return {k: v[:n] for k, v in out.items()}

    def roundtrip(self, src, blk_off, blk_len, dst=None):
        src = np.ascontiguousarray(src, np.uint8)
        blk_off = np.ascontiguousarray(blk_off, np.uint64)
        blk_len = np.ascontiguousarray(blk_len, np.uint64)
        if dst is None:
            dst = np.zeros_like(src)
        out_len = np.zeros(max(blk_off.size, 1), np.uint64)
        total = self.lib.ref_roundtrip_blocks(_ptr(src), _ptr(blk_off), _ptr(blk_len), blk_off.size, _ptr(dst),
                                              _ptr(out_len))
        return dst, out_len[: blk_off.size], total

    def table_build(self, path, rec, block_size=4096):
        r = _rec_args(rec)
        n = len(r["type"])
        fs = self.lib.ref_table_build(path.encode(), block_size, n, _ptr(r["type"]), _ptr(r["key_len"]),
                                      _ptr(r["val_len"]), _ptr(r["txn"]), _ptr(r["key_src"]),
                                      _ptr(r["key_off"]), _ptr(r["val_src"]), _ptr(r["val_off"]))
        return fs

    def table_index(self, path, file_size, cap=1 << 16):
        o = {"blk_off": np.zeros(cap, np.uint64), "blk_len": np.zeros(cap, np.uint64),
             "first_key_len": np.zeros(cap, np.uint32), "last_key_len": np.zeros(cap, np.uint32)}
        fk = np.zeros(4096, np.uint8)
        lk = np.zeros(4096, np.uint8)
        nb = self.lib.ref_table_index(path.encode(), file_size, cap, _ptr(o["blk_off"]), _ptr(o["blk_len"]),
                                      _ptr(o["first_key_len"]), _ptr(o["last_key_len"]), _ptr(fk), _ptr(lk))
        if nb == 2 ** 64 - 1:
            return None
        res = {k: v[:nb] for k, v in o.items()}
        res["nblocks"] = nb
        res["first_key"] = bytes(fk[: int(res["first_key_len"][0])]) if nb else b""
        res["last_key"] = bytes(lk[: int(res["last_key_len"][-1])]) if nb else b""
        return res


def _ref_table_get(self, path, file_size, keys, val_cap=1 << 26):
    """The reference's TableReader::GetValue (no cache) on an SST file.  Returns
    (type u32[], list of value bytes or None)."""
    arena, off, lens = queries_arena(keys)
    n = len(keys)
    t = np.zeros(max(n, 1), np.uint32)
    vo = np.zeros(max(n, 1), np.uint64)
    vl = np.zeros(max(n, 1), np.uint32)
    out = np.zeros(val_cap, np.uint8)
    used = self.lib.ref_table_get(path.encode(), file_size, n, _ptr(arena), _ptr(off), _ptr(lens), _ptr(t),
                                  _ptr(vo), _ptr(vl), _ptr(out), val_cap)
    if used == 2 ** 64 - 1:
        return None
    vals = [bytes(out[int(vo[i]):int(vo[i]) + int(vl[i])]) if t[i] == 0 else None for i in range(n)]
    return t[:n], vals


RefLib.table_get = _ref_table_get
