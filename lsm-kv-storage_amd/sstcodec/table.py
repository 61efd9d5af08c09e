"""Python face of the host C++ TableBuilder / TableReader (include/sstc_table.h).

Thin ctypes wrapper over the C shim; the classes themselves are C++ (the
reference is C++).  Used by tests to hold the host framing to the reference's
SST bytes.
"""
import ctypes

import numpy as np

from ._lib import SstcError, check, load

_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64


def _sig(lib):
    if getattr(lib, "_sstc_table_sig", False):
        return lib
    P = ctypes.POINTER
    for name, res, args in [
        ("sstc_tb_create", ctypes.c_int, [ctypes.c_char_p, _u64, _vp, P(_vp)]),
        ("sstc_tb_open", ctypes.c_int, [_vp]),
        ("sstc_tb_add", ctypes.c_int, [_vp, _vp, ctypes.c_uint32, _vp, ctypes.c_uint32, _u64, ctypes.c_uint8]),
        ("sstc_tb_add_batch", ctypes.c_int, [_vp, _u64] + [_vp] * 8),
        ("sstc_tb_finish", ctypes.c_int, [_vp]),
        ("sstc_tb_file_size", _u64, [_vp]),
        ("sstc_tb_num_blocks", _u64, [_vp]),
        ("sstc_tb_destroy", ctypes.c_int, [_vp]),
        ("sstc_tr_open", ctypes.c_int, [ctypes.c_char_p, _u64, _vp, P(_vp)]),
        ("sstc_tr_num_blocks", _u64, [_vp]),
        ("sstc_tr_block_index", ctypes.c_int, [_vp, _vp, _vp]),
        ("sstc_tr_num_records", _u64, [_vp, ctypes.c_uint32]),
        ("sstc_tr_decode_all", ctypes.c_int, [_vp, ctypes.c_uint32] + [_vp] * 6),
        ("sstc_tr_destroy", ctypes.c_int, [_vp]),
    ]:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    lib._sstc_table_sig = True
    return lib


def _p(a):
    return a.ctypes.data_as(_vp)


def build_table(codec, path, rec, block_threshold=4096):
    """Write an SST through sstc::TableBuilder; returns GetFileSize()."""
    lib = _sig(load())
    codec._stream()
    tb = _vp()
    check(lib.sstc_tb_create(path.encode(), block_threshold, codec.h, ctypes.byref(tb)), "sstc_tb_create")
    try:
        check(lib.sstc_tb_open(tb), "sstc_tb_open")
        r = {k: np.ascontiguousarray(rec[k]) for k in rec}
        ks = r["key_src"] if r["key_src"].size else np.zeros(1, np.uint8)
        vs = r["val_src"] if r["val_src"].size else np.zeros(1, np.uint8)
        n = len(r["type"])
        check(lib.sstc_tb_add_batch(tb, n, _p(r["type"].astype(np.uint8)), _p(r["key_len"].astype(np.uint32)),
                                    _p(r["val_len"].astype(np.uint32)), _p(r["txn"].astype(np.uint64)), _p(ks),
                                    _p(r["key_off"].astype(np.uint64)), _p(vs), _p(r["val_off"].astype(np.uint64))),
              "sstc_tb_add_batch")
        check(lib.sstc_tb_finish(tb), "sstc_tb_finish")
        return lib.sstc_tb_file_size(tb), lib.sstc_tb_num_blocks(tb)
    finally:
        lib.sstc_tb_destroy(tb)


def read_table(codec, path, file_size, txn_mode=0):
    """Open through sstc::TableReader and decode every block on the GPU."""
    lib = _sig(load())
    codec._stream()
    tr = _vp()
    check(lib.sstc_tr_open(path.encode(), int(file_size), codec.h, ctypes.byref(tr)), "sstc_tr_open")
    try:
        nb = lib.sstc_tr_num_blocks(tr)
        off = np.zeros(max(nb, 1), np.uint64)
        ln = np.zeros(max(nb, 1), np.uint64)
        check(lib.sstc_tr_block_index(tr, _p(off), _p(ln)), "sstc_tr_block_index")
        n = lib.sstc_tr_num_records(tr, txn_mode)
        out = {"type": np.zeros(max(n, 1), np.uint8), "key_len": np.zeros(max(n, 1), np.uint32),
               "val_len": np.zeros(max(n, 1), np.uint32), "txn": np.zeros(max(n, 1), np.uint64),
               "key_off": np.zeros(max(n, 1), np.uint64), "val_off": np.zeros(max(n, 1), np.uint64)}
        st = lib.sstc_tr_decode_all(tr, txn_mode, *[_p(out[k]) for k in
                                                    ("type", "key_len", "val_len", "txn", "key_off", "val_off")])
        if st != 0:
            raise SstcError(f"sstc_tr_decode_all: status {st}")
        return {"blk_off": off[:nb], "blk_len": ln[:nb], **{k: v[:n] for k, v in out.items()}}
    finally:
        lib.sstc_tr_destroy(tr)
