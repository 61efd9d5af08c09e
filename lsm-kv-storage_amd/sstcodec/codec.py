"""Torch-facing wrapper of the C-ABI (device buffers are torch CUDA tensors).

PyTorch here is plumbing only: it owns device memory and the stream; all codec
work runs in libsstcodec.so's HIP kernels.  u64 arrays are carried in int64
tensors and u32 arrays in int32 tensors (bit-identical; SSTC_NO_VALUE is -1).
"""
import ctypes

import torch

from . import _lib
from ._lib import Records, check, load


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _dev(t, dtype, device):
    if not torch.is_tensor(t):
        import numpy as np
        t = torch.from_numpy(np.ascontiguousarray(t).view({
            torch.uint8: np.uint8, torch.int32: np.int32, torch.int64: np.int64}[dtype]))
    if t.dtype != dtype:
        t = t.view(dtype) if t.element_size() == torch.empty((), dtype=dtype).element_size() else t.to(dtype)
    return t.to(device, non_blocking=False).contiguous()


class RecordTable:
    """SoA record table on the device (see include/sstcodec.h sstc_records)."""

    FIELDS = (("type", torch.uint8), ("key_len", torch.int32), ("val_len", torch.int32),
              ("txn", torch.int64), ("key_off", torch.int64), ("val_off", torch.int64))

    def __init__(self, n, device, tensors=None):
        self.n = int(n)
        if tensors is None:
            tensors = {k: torch.empty(max(self.n, 1), dtype=dt, device=device) for k, dt in self.FIELDS}
        self.t = tensors

    @classmethod
    def from_numpy(cls, rec, device):
        n = len(rec["type"])
        t = {k: _dev(rec[k], dt, device) for k, dt in cls.FIELDS}
        return cls(n, device, t)

    def c(self):
        return Records(*[self.t[k].data_ptr() for k, _ in self.FIELDS])

    def to_numpy(self):
        import numpy as np
        view = {torch.uint8: np.uint8, torch.int32: np.uint32, torch.int64: np.uint64}
        return {k: self.t[k][: self.n].cpu().numpy().view(view[dt]) for k, dt in self.FIELDS}


class Codec:
    """One sstc_ctx bound to a device; calls run on torch's current stream."""

    def __init__(self, device=None):
        lib = load()
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device)
        self.lib = lib
        h = ctypes.c_void_p()
        check(lib.sstc_ctx_create(int(device), ctypes.c_void_p(0), ctypes.byref(h)), "sstc_ctx_create")
        self.h = h

    def close(self):
        if self.h:
            self.lib.sstc_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        s = torch.cuda.current_stream(self.device).cuda_stream
        check(self.lib.sstc_ctx_set_stream(self.h, ctypes.c_void_p(s)), "sstc_ctx_set_stream")

    def reserve(self, max_blocks, max_records):
        self._stream()
        check(self.lib.sstc_ctx_reserve(self.h, int(max_blocks), int(max_records)), "sstc_ctx_reserve")

    def error_count(self):
        self._stream()
        v = ctypes.c_uint64()
        check(self.lib.sstc_ctx_error_count(self.h, ctypes.byref(v)), "sstc_ctx_error_count")
        return v.value

    def reset_errors(self):
        self._stream()
        check(self.lib.sstc_ctx_reset_errors(self.h), "sstc_ctx_reset_errors")

    # ---- fused round trip -------------------------------------------------
    def roundtrip(self, src, blk_off, blk_len, dst=None, txn_mode=_lib.SSTC_TXN_COMPAT,
                  out_len=None, status=None):
        nb = blk_off.numel()
        if dst is None:
            dst = torch.zeros_like(src)
        if out_len is None:
            out_len = torch.empty(max(nb, 1), dtype=torch.int64, device=self.device)
        if status is None:
            status = torch.empty(max(nb, 1), dtype=torch.int32, device=self.device)
        self._stream()
        check(self.lib.sstc_roundtrip_blocks(self.h, _p(src), _p(dst), _p(blk_off), _p(blk_len), nb,
                                             txn_mode, _p(out_len), _p(status)), "sstc_roundtrip_blocks")
        return dst, out_len, status

    def roundtrip_host(self, h_src, h_dst, blk_off, blk_len, txn_mode=_lib.SSTC_TXN_COMPAT, chunk_bytes=16 << 20):
        """sstc_roundtrip_host: blocks in host memory (u8 CPU tensors, pinned
        for full rate; numpy offsets / lengths) streamed through the device.
        Returns numpy (out_len, status)."""
        import numpy as np
        off = np.ascontiguousarray(blk_off, np.uint64)
        ln = np.ascontiguousarray(blk_len, np.uint64)
        nb = off.size
        out_len = np.zeros(max(nb, 1), np.uint64)
        status = np.zeros(max(nb, 1), np.uint32)
        vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        self._stream()
        check(self.lib.sstc_roundtrip_host(self.h, ctypes.c_void_p(h_src.data_ptr()),
                                           ctypes.c_void_p(h_dst.data_ptr()), h_src.numel(), vp(off), vp(ln), nb,
                                           txn_mode, int(chunk_bytes), vp(out_len), vp(status)),
              "sstc_roundtrip_host")
        return out_len[:nb], status[:nb]

    def roundtrip_raw(self, src, dst, blk_off, blk_len, nb, txn_mode=_lib.SSTC_TXN_COMPAT,
                      out_len=None, status=None):
        """Minimal-overhead launch for timing loops (pointers pre-resolved by caller)."""
        return self.lib.sstc_roundtrip_blocks(self.h, src, dst, blk_off, blk_len, nb, txn_mode,
                                              out_len, status)

    # ---- decode ------------------------------------------------------------
    def count(self, src, blk_off, blk_len):
        nb = blk_off.numel()
        rec_base = torch.empty(nb + 1, dtype=torch.int64, device=self.device)
        self._stream()
        check(self.lib.sstc_count_records(self.h, _p(src), _p(blk_off), _p(blk_len), nb, _p(rec_base)),
              "sstc_count_records")
        return rec_base

    def decode(self, src, blk_off, blk_len, txn_mode=_lib.SSTC_TXN_COMPAT, rec_base=None, status=None):
        nb = blk_off.numel()
        if rec_base is None:
            rec_base = self.count(src, blk_off, blk_len)
        total = int(rec_base[nb].item())
        table = RecordTable(total, self.device)
        if status is None:
            status = torch.empty(max(nb, 1), dtype=torch.int32, device=self.device)
        self._stream()
        check(self.lib.sstc_decode_blocks(self.h, _p(src), _p(blk_off), _p(blk_len), nb, _p(rec_base),
                                          table.c(), txn_mode, _p(status)), "sstc_decode_blocks")
        return table, rec_base, status

    def pack(self, table):
        """sstc_pack_records: the record table as n x 32 B sstc_record32 rows
        (uint8 tensor [n, 32]) -- what the drop-in TableReaderIterator reads."""
        out = torch.empty((max(table.n, 1), 32), dtype=torch.uint8, device=self.device)
        self._stream()
        check(self.lib.sstc_pack_records(self.h, table.c(), table.n, _p(out)), "sstc_pack_records")
        return out[: table.n]

    # ---- encode ------------------------------------------------------------
    def segment(self, table, threshold):
        n = table.n
        first = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        nb = torch.empty(1, dtype=torch.int64, device=self.device)
        self._stream()
        check(self.lib.sstc_segment_records(self.h, _p(table.t["key_len"]), _p(table.t["val_len"]), n,
                                            int(threshold), _p(first), _p(nb)), "sstc_segment_records")
        k = int(nb.item())
        return first[: k + 1]

    def encode(self, table, key_src, val_src, blk_first, out_base=0, dst=None):
        nb = blk_first.numel() - 1
        out_off = torch.empty(nb + 1, dtype=torch.int64, device=self.device)
        out_len = torch.empty(max(nb, 1), dtype=torch.int64, device=self.device)
        if dst is None:
            # exact size: data + 16 per record + 16 per block
            sizes = 13 + table.t["key_len"][: table.n].to(torch.int64)
            vl = table.t["val_len"][: table.n].to(torch.int64)
            sizes = sizes + torch.where(vl == -1, torch.zeros_like(vl), 4 + (vl & 0xFFFFFFFF))
            total = int(sizes.sum().item()) + 16 * table.n + 16 * nb + int(out_base)
            dst = torch.zeros(max(total, 1), dtype=torch.uint8, device=self.device)
        self._stream()
        check(self.lib.sstc_encode_blocks(self.h, _p(key_src), _p(val_src), table.c(), table.n, _p(blk_first),
                                          nb, int(out_base), _p(dst), _p(out_off), _p(out_len)),
              "sstc_encode_blocks")
        return dst, out_off, out_len[:nb]

    # ---- SST open ------------------------------------------------------------
    def open_tables(self, src, tab_bytes, tab_off=None, max_blocks=None, strict=False):
        """sstc_open_tables: footers + meta sections of the SST images in the
        device u8 tensor `src` (table t = src[tab_off[t] .. + tab_bytes[t]),
        tab_bytes = GetFileSize() - 1; back to back when tab_off is None)
        parsed on the device.  Returns a dict of device tensors (blk_off,
        blk_len, first_key_off, first_key_len, last_key_off, last_key_len,
        table_first_block_dev; key / block offsets absolute into src) and numpy
        table_first_block, status (SSTC_TAB_*), footer (ntables x 5).
        strict: raise unless every table is SSTC_TAB_OK."""
        import numpy as np
        nt = len(tab_bytes)
        tb = np.ascontiguousarray(tab_bytes, np.uint64)
        if tab_off is None:
            to = np.zeros(nt, np.uint64)
            if nt > 1:
                to[1:] = np.cumsum(tb[:-1])
        else:
            to = np.ascontiguousarray(tab_off, np.uint64)
        if max_blocks is None:  # every block takes >= 24 B of meta + >= 16 B of data
            max_blocks = int(tb.sum()) // 40 + 1
        dev = self.device
        cap = max(int(max_blocks), 1)
        o = {k: torch.empty(cap, dtype=torch.int64, device=dev)
             for k in ("blk_off", "blk_len", "first_key_off", "last_key_off")}
        o["first_key_len"] = torch.empty(cap, dtype=torch.int32, device=dev)
        o["last_key_len"] = torch.empty(cap, dtype=torch.int32, device=dev)
        o["table_first_block_dev"] = torch.empty(nt + 1, dtype=torch.int64, device=dev)
        tfb = np.zeros(nt + 1, np.uint64)
        status = np.zeros(max(nt, 1), np.int32)
        footer = np.zeros((max(nt, 1), 5), np.uint64)
        vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        self._stream()
        check(self.lib.sstc_open_tables(self.h, _p(src), int(src.numel()), vp(to), vp(tb), nt, int(max_blocks),
                                        _p(o["blk_off"]), _p(o["blk_len"]), _p(o["first_key_off"]),
                                        _p(o["first_key_len"]), _p(o["last_key_off"]), _p(o["last_key_len"]),
                                        _p(o["table_first_block_dev"]), vp(tfb), vp(status), vp(footer)),
              "sstc_open_tables")
        nb = int(tfb[nt])
        for k in ("blk_off", "blk_len", "first_key_off", "last_key_off", "first_key_len", "last_key_len"):
            o[k] = o[k][:nb]
        o["table_first_block"] = tfb
        o["status"] = status[:nt]
        o["footer"] = footer[:nt]
        if strict and nt and (status[:nt] != _lib.SSTC_TAB_OK).any():
            bad = int(np.flatnonzero(status[:nt])[0])
            raise _lib.SstcError(f"sstc_open_tables: table {bad} rejected (status {int(status[bad])})")
        return o

    # ---- compaction ----------------------------------------------------------
    def compact(self, tables, block_threshold=4096, table_limit=32 << 20, base_level=1,
                txn_mode=_lib.SSTC_TXN_COMPAT, probe=None):
        """Compact SST images (list of numpy u8 arrays, iterator order) on the
        GPU.  Returns (list of output SST images as numpy arrays, result).
        probe (tests): a list that receives the output buffer before the call's
        status is checked."""
        import numpy as np
        from ._lib import CompactParams, CompactResult
        if isinstance(tables, (list, tuple)):
            files = [np.ascontiguousarray(t, np.uint8) for t in tables]
        else:
            files = list(tables)
        # block index of every table: footers + meta sections parsed on the device
        src = torch.from_numpy(np.concatenate(files) if files else np.zeros(1, np.uint8)).to(self.device)
        idx = self.open_tables(src, [f.size for f in files], strict=True)
        blk_off, blk_len, h_tfb = idx["blk_off"], idx["blk_len"], idx["table_first_block"]
        cap = int(src.numel()) * 2 + 4096
        # outputs filled with junk, not zeros: the library writes every byte
        # and every table slot it reports (the reference-hash tests see any gap)
        dst = torch.full((cap,), 0xA5, dtype=torch.uint8, device=self.device)
        max_t = cap // 40 + 1
        toff = torch.full((max_t + 1,), -1, dtype=torch.int64, device=self.device)
        tlen = torch.full((max_t,), -1, dtype=torch.int64, device=self.device)
        prm = CompactParams(block_threshold, table_limit, base_level, txn_mode)
        res = CompactResult()
        self._stream()
        rc = self.lib.sstc_compact(self.h, _p(src), _p(blk_off), _p(blk_len), int(blk_off.numel()),
                                   h_tfb.ctypes.data_as(ctypes.c_void_p), len(files), ctypes.byref(prm), _p(dst),
                                   cap, _p(toff), _p(tlen), max_t, ctypes.byref(res))
        if probe is not None:
            probe.append(dst)
        check(rc, "sstc_compact")
        nt = res.tables_out
        o = toff[: nt + 1].cpu().numpy()
        d = dst[: int(o[nt])].cpu().numpy()
        return [d[int(o[t]):int(o[t + 1])] for t in range(nt)], res


    def merge_records(self, tables, txn_mode=_lib.SSTC_TXN_COMPAT, max_records=None):
        """sstc_merge_records over SST images (numpy u8 arrays, iterator
        order): MergeIterator's SeekToFirst + Next order of every record.
        Returns (records: numpy (n, 2) u64 of [key offset into the tables
        concatenated, txn as read], MergeResult).  max_records=None sizes the
        output by a first call that reports the count (SSTC_E_CAPACITY)."""
        import numpy as np
        from ._lib import SSTC_E_CAPACITY, MergeResult
        files = [np.ascontiguousarray(t, np.uint8) for t in tables]
        src = torch.from_numpy(np.concatenate(files)).to(self.device)
        idx = self.open_tables(src, [f.size for f in files], strict=True)
        blk_off, blk_len, h_tfb = idx["blk_off"], idx["blk_len"], idx["table_first_block"]
        res = MergeResult()

        def call(cap):
            out = torch.empty((max(cap, 1), 2), dtype=torch.int64, device=self.device)
            self._stream()
            rc = self.lib.sstc_merge_records(self.h, _p(src), _p(blk_off), _p(blk_len), int(blk_off.numel()),
                                             h_tfb.ctypes.data_as(ctypes.c_void_p), len(files), txn_mode, _p(out),
                                             cap, ctypes.byref(res))
            return rc, out
        if max_records is None:
            rc, out = call(0)
            if rc == SSTC_E_CAPACITY:
                rc, out = call(int(res.records))
        else:
            rc, out = call(int(max_records))
        check(rc, "sstc_merge_records")
        return out[: res.records].cpu().numpy().view(np.uint64), res


def _queries(keys):
    import numpy as np
    lens = np.array([len(k) for k in keys], np.uint32)
    off = np.zeros(len(keys), np.uint64)
    if len(keys) > 1:
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    arena = np.frombuffer(b"".join(keys) + b"\0" * 8, np.uint8).copy()
    return arena, off, lens


class Lookup:
    """Device-resident SSTs + block indexes for batched point lookups
    (sstc_get_batch): TableReader::GetValue over many tables and keys."""

    def __init__(self, codec, tables):
        import numpy as np
        self.codec = codec
        dev = codec.device
        self.src = torch.from_numpy(np.concatenate(tables) if tables else np.zeros(1, np.uint8)).to(dev)
        # block indexes parsed on the device (footer + meta section per table)
        idx = codec.open_tables(self.src, [f.size for f in tables], strict=True)
        one = lambda t: t if t.numel() else torch.zeros(1, dtype=t.dtype, device=dev)  # noqa: E731
        self.blk_off, self.blk_len = one(idx["blk_off"]), one(idx["blk_len"])
        self.lk_off, self.lk_len = one(idx["last_key_off"]), one(idx["last_key_len"])
        self.tfb = idx["table_first_block_dev"]
        self.ntables = len(tables)
        self.base = [0]
        for f in tables:
            self.base.append(self.base[-1] + f.size)

    def index(self):
        from ._lib import BlockIndex
        n = self.src.numel()
        return BlockIndex(self.blk_off.data_ptr(), self.blk_len.data_ptr(), self.lk_off.data_ptr(),
                          self.lk_len.data_ptr(), self.src.data_ptr(), self.tfb.data_ptr(), self.ntables, n, n)

    def get(self, q_table, keys, raw=False):
        """q_table: table index per query; keys: list of bytes.  Returns numpy
        (type, val_off (absolute, into the concatenated tables), val_len, block)."""
        import numpy as np
        dev = self.codec.device
        arena, off, lens = _queries(keys)
        n = len(keys)
        qt = torch.from_numpy(np.asarray(q_table, np.uint32).view(np.int32)).to(dev) if n else \
            torch.zeros(1, dtype=torch.int32, device=dev)
        qk = torch.from_numpy(arena).to(dev)
        qo = torch.from_numpy(off.view(np.int64) if n else np.zeros(1, np.int64)).to(dev)
        ql = torch.from_numpy(lens.view(np.int32) if n else np.zeros(1, np.int32)).to(dev)
        ot = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        ov = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        ol = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        ob = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        idx = self.index()
        self.codec._stream()
        check(self.codec.lib.sstc_get_batch(self.codec.h, _p(self.src), ctypes.byref(idx), _p(qt), _p(qk),
                                            qk.numel(), _p(qo), _p(ql), n, _p(ot), _p(ov), _p(ol), _p(ob)),
              "sstc_get_batch")
        if raw:
            return ot, ov, ol, ob
        return (ot[:n].cpu().numpy().view(np.uint32), ov[:n].cpu().numpy().view(np.uint64),
                ol[:n].cpu().numpy().view(np.uint32), ob[:n].cpu().numpy().view(np.uint64))


class FilePipe:
    """sstc_pipe: file-to-file compaction (input SST files -> output SST files)
    with pinned staging kept across calls."""

    def __init__(self, codec, io_threads=8):
        self.codec = codec
        self.lib = codec.lib
        h = ctypes.c_void_p()
        check(self.lib.sstc_pipe_create(codec.h, int(io_threads), ctypes.byref(h)), "sstc_pipe_create")
        self.h = h

    def close(self):
        if self.h:
            self.lib.sstc_pipe_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def compact_files(self, paths, file_sizes, out_prefix, first_sst_id, block_threshold=4096,
                      table_limit=32 << 20, base_level=1, txn_mode=_lib.SSTC_TXN_COMPAT, fsync=True,
                      max_outs=4096):
        """Returns ([(sst_id, file_size, smallest_key, largest_key)], timing dict)."""
        from ._lib import CompactParams, FileOut, FilesTiming
        n = len(paths)
        arr = (ctypes.c_char_p * max(n, 1))(*[p.encode() for p in paths])
        sizes = (ctypes.c_uint64 * max(n, 1))(*[int(x) for x in file_sizes])
        outs = (FileOut * max_outs)()
        arena = ctypes.create_string_buffer(max_outs * 2 * 4096)
        nout = ctypes.c_uint32()
        tm = FilesTiming()
        prm = CompactParams(block_threshold, table_limit, base_level, txn_mode)
        self.codec._stream()
        check(self.lib.sstc_compact_files(self.h, ctypes.cast(arr, ctypes.c_void_p), ctypes.cast(sizes, ctypes.c_void_p),
                                          n, out_prefix.encode(), int(first_sst_id), ctypes.byref(prm),
                                          1 if fsync else 0, ctypes.cast(outs, ctypes.c_void_p), max_outs,
                                          ctypes.byref(nout), ctypes.cast(arena, ctypes.c_void_p),
                                          len(arena), ctypes.byref(tm)), "sstc_compact_files")
        raw = arena.raw
        res = []
        for o in outs[: nout.value]:
            lo = raw[o.smallest_key_off:o.smallest_key_off + o.smallest_key_len]
            hi = raw[o.largest_key_off:o.largest_key_off + o.largest_key_len]
            res.append((o.sst_id, o.file_size, lo, hi))
        return res, {k: getattr(tm, k) for k, _ in FilesTiming._fields_}


def compact_files_multi(pipes, shards, out_prefix, first_sst_id, block_threshold=4096, table_limit=32 << 20,
                        base_level=1, txn_mode=_lib.SSTC_TXN_COMPAT, fsync=True, max_outs=8192):
    """sstc_compact_files_multi: shards = [[(path, GetFileSize()), ...], ...]
    (key-range-disjoint input groups), shard s on pipes[s % len(pipes)], one
    host thread per pipe.  Returns ([(sst_id, file_size, smallest, largest)]
    in shard order, [timing dict per shard])."""
    from ._lib import CompactParams, FileOut, FilesTiming
    lib = pipes[0].lib
    paths = [p for sh in shards for p, _ in sh]
    sizes = [int(fs) for sh in shards for _, fs in sh]
    first = [0]
    for sh in shards:
        first.append(first[-1] + len(sh))
    n = max(len(paths), 1)
    arr = (ctypes.c_char_p * n)(*[p.encode() for p in paths])
    sz = (ctypes.c_uint64 * n)(*sizes)
    sf = (ctypes.c_uint32 * len(first))(*first)
    ph = (ctypes.c_void_p * len(pipes))(*[p.h for p in pipes])
    outs = (FileOut * max_outs)()
    arena = ctypes.create_string_buffer(max_outs * 2 * 4096)
    nout = ctypes.c_uint32()
    tm = (FilesTiming * max(len(shards), 1))()
    prm = CompactParams(block_threshold, table_limit, base_level, txn_mode)
    rc = lib.sstc_compact_files_multi(ctypes.cast(ph, ctypes.c_void_p), len(pipes), ctypes.cast(arr, ctypes.c_void_p),
                                      ctypes.cast(sz, ctypes.c_void_p), ctypes.cast(sf, ctypes.c_void_p), len(shards),
                                      out_prefix.encode(), int(first_sst_id), ctypes.byref(prm), 1 if fsync else 0,
                                      ctypes.cast(outs, ctypes.c_void_p), max_outs, ctypes.byref(nout),
                                      ctypes.cast(arena, ctypes.c_void_p), len(arena), ctypes.cast(tm, ctypes.c_void_p))
    raw = arena.raw
    res = [(o.sst_id, o.file_size, raw[o.smallest_key_off:o.smallest_key_off + o.smallest_key_len],
            raw[o.largest_key_off:o.largest_key_off + o.largest_key_len]) for o in outs[: nout.value]]
    try:
        check(rc, "sstc_compact_files_multi")
    except _lib.SstcError as e:
        e.outs = res  # the outputs of the shards that completed before the failing one
        raise
    return res, [{k: getattr(t, k) for k, _ in FilesTiming._fields_} for t in tm[: len(shards)]]


def _table_index(f, keys=False):
    """(block offsets, block sizes[, last-key offsets, last-key lengths]) of an
    SST image: footer + meta section walk (reference table_reader.cc:52-156).
    Key offsets point into the image."""
    import numpy as np
    b = f.size
    foot = f[b - 40:].view(np.uint64)
    nb, moff, mlen = int(foot[0]), int(foot[1]), int(foot[2])
    meta = f[moff:moff + mlen].tobytes()
    offs, lens, lko, lkl = [], [], [], []
    p = 0
    for _ in range(nb):
        fk = int.from_bytes(meta[p:p + 4], "little")
        lk = int.from_bytes(meta[p + 4 + fk:p + 8 + fk], "little")
        q = p + 8 + fk + lk
        lko.append(moff + p + 8 + fk)
        lkl.append(lk)
        offs.append(int.from_bytes(meta[q:q + 8], "little"))
        lens.append(int.from_bytes(meta[q + 8:q + 16], "little"))
        p = q + 16
    if keys:
        return (np.asarray(offs, np.uint64), np.asarray(lens, np.uint64), np.asarray(lko, np.uint64),
                np.asarray(lkl, np.uint32))
    return np.asarray(offs, np.uint64), np.asarray(lens, np.uint64)
