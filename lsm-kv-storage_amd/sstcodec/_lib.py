"""ctypes binding of libsstcodec.so (include/sstcodec.h).

The library is loaded from the in-tree build (lsm-kv-storage_amd/lib/).  There
is no fallback: if the library is missing, or no GPU is present, calls raise.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
# SSTC_LIB_PATH: an A/B build of the same library (tools/ab_*.sh); default the in-tree build
LIB_PATH = os.environ.get("SSTC_LIB_PATH") or os.path.join(PKG_ROOT, "lib", "libsstcodec.so")
HEADER = os.path.join(os.path.dirname(PKG_ROOT), "include", "sstcodec.h")

SSTC_OK = 0
SSTC_NO_VALUE = 0xFFFFFFFF
SSTC_TXN_COMPAT = 0
SSTC_TXN_CORRECT = 1
BLK_STATUS = {0: "OK", 1: "TOO_SMALL", 2: "EMPTY", 3: "OFFSETS_RANGE", 4: "ENTRY_RANGE",
              5: "BAD_TYPE", 6: "KEY_TOO_LONG", 7: "TOO_LARGE",
              8: "NO_ROOM", 9: "COUNT_MISMATCH"}

c_u8p = ctypes.c_void_p
c_u64 = ctypes.c_uint64
c_u32 = ctypes.c_uint32
c_vp = ctypes.c_void_p


class Records(ctypes.Structure):
    """sstc_records: device pointers of the SoA record table."""
    _fields_ = [("type", c_vp), ("key_len", c_vp), ("val_len", c_vp), ("txn", c_vp),
                ("key_off", c_vp), ("val_off", c_vp)]


class CompactParams(ctypes.Structure):
    _fields_ = [("block_threshold", ctypes.c_uint64), ("table_limit", ctypes.c_uint64),
                ("base_level", ctypes.c_uint32), ("txn_mode", ctypes.c_uint32)]


class CompactResult(ctypes.Structure):
    _fields_ = [("records_in", ctypes.c_uint64), ("records_kept", ctypes.c_uint64),
                ("blocks_out", ctypes.c_uint64), ("tables_out", ctypes.c_uint64), ("bytes_out", ctypes.c_uint64)]


class MergeResult(ctypes.Structure):
    """sstc_merge_result"""
    _fields_ = [("records", ctypes.c_uint64), ("cross_ties", ctypes.c_uint64), ("tie_diffs", ctypes.c_uint64)]


class BlockIndex(ctypes.Structure):
    """sstc_block_index (device pointers)."""
    _fields_ = [("blk_off", c_vp), ("blk_len", c_vp), ("last_key_off", c_vp), ("last_key_len", c_vp),
                ("keys", c_vp), ("table_first_block", c_vp), ("ntables", ctypes.c_uint32),
                ("src_bytes", ctypes.c_uint64), ("keys_bytes", ctypes.c_uint64)]


GET_TYPES = {0: "PUT", 1: "DELETED", 2: "NOT_FOUND", 4: "BAD_BLOCK"}


class FileOut(ctypes.Structure):
    _fields_ = [("sst_id", ctypes.c_uint64), ("file_size", ctypes.c_uint64), ("smallest_key_off", ctypes.c_uint64),
                ("largest_key_off", ctypes.c_uint64), ("smallest_key_len", ctypes.c_uint32),
                ("largest_key_len", ctypes.c_uint32)]


class FilesTiming(ctypes.Structure):
    _fields_ = [("index_s", ctypes.c_double), ("load_s", ctypes.c_double), ("compact_s", ctypes.c_double),
                ("store_s", ctypes.c_double), ("total_s", ctypes.c_double)]


SSTC_E_INVALID_ARG = -1
SSTC_E_CAPACITY = -5
SSTC_E_INTERNAL = -6  # include/sstcodec.h: a device-side consistency check failed
SSTC_E_TIE_ORDER = -7  # include/sstcodec.h: equal (key, txn) records with different contents in different inputs

SSTC_TAB_OK, SSTC_TAB_BAD_FOOTER, SSTC_TAB_BAD_META, SSTC_TAB_BAD_BLOCK, SSTC_TAB_TOO_LARGE = 0, 1, 2, 3, 4


class SstcError(RuntimeError):
    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code  # the SSTC_E_* return code


_lib = None


def load():
    """Load (once) and return the ctypes library.  Raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SstcError(f"{LIB_PATH} is not built (run lsm-kv-storage_amd/build.py); "
                        "the SST codec has no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    sig = {
        "sstc_version": (c_u32, []),
        "sstc_last_error_string": (ctypes.c_char_p, []),
        "sstc_ctx_create": (ctypes.c_int, [ctypes.c_int, c_vp, P(c_vp)]),
        "sstc_ctx_destroy": (ctypes.c_int, [c_vp]),
        "sstc_ctx_set_stream": (ctypes.c_int, [c_vp, c_vp]),
        "sstc_ctx_drop_stream": (ctypes.c_int, [c_vp]),
        "sstc_ctx_reserve": (ctypes.c_int, [c_vp, c_u64, c_u64]),
        "sstc_ctx_error_count": (ctypes.c_int, [c_vp, P(c_u64)]),
        "sstc_ctx_reset_errors": (ctypes.c_int, [c_vp]),
        "sstc_count_records": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_u64, c_vp]),
        "sstc_decode_blocks": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_u64, c_vp, Records, c_u32, c_vp]),
        "sstc_pack_records": (ctypes.c_int, [c_vp, Records, c_u64, c_vp]),
        "sstc_segment_records": (ctypes.c_int, [c_vp, c_vp, c_vp, c_u64, c_u64, c_vp, c_vp]),
        "sstc_encode_blocks": (ctypes.c_int, [c_vp, c_vp, c_vp, Records, c_u64, c_vp, c_u64, c_u64,
                                              c_vp, c_vp, c_vp]),
        "sstc_roundtrip_blocks": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_u64, c_u32, c_vp, c_vp]),
        "sstc_compact": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_u64, c_vp, c_u32, P(CompactParams), c_vp, c_u64,
                                        c_vp, c_vp, c_u64, P(CompactResult)]),
        "sstc_merge_records": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_u64, c_vp, c_u32, c_u32, c_vp, c_u64,
                                              P(MergeResult)]),
        "sstc_get_batch": (ctypes.c_int, [c_vp, c_vp, P(BlockIndex), c_vp, c_vp, c_u64, c_vp, c_vp, c_u64, c_vp, c_vp,
                                          c_vp, c_vp]),
        "sstc_roundtrip_host": (ctypes.c_int, [c_vp, c_vp, c_vp, c_u64, c_vp, c_vp, c_u64, c_u32, c_u64, c_vp,
                                               c_vp]),
        "sstc_copy_probe": (ctypes.c_int, [c_vp, c_vp, c_vp, c_u64]),
        "sstc__ctx_set_fault": (ctypes.c_int, [c_vp, c_u32]),  # test hooks (sstc_api.hip), not in the header
        "sstc__ctx_seg_stats": (ctypes.c_int, [c_vp, c_vp, c_vp]),
        "sstc__ctx_set_scan_epoch": (ctypes.c_int, [c_vp, c_u32]),
        "sstc_open_tables": (ctypes.c_int, [c_vp, c_vp, c_u64, c_vp, c_vp, c_u32, c_u64, c_vp, c_vp, c_vp, c_vp,
                                            c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
        "sstc_pipe_create": (ctypes.c_int, [c_vp, c_u32, P(c_vp)]),
        "sstc_pipe_destroy": (ctypes.c_int, [c_vp]),
        "sstc__pipe_set_test_caps": (ctypes.c_int, [c_vp, c_u64, c_u64]),  # test hook (compact_files.cpp)
        "sstc_compact_files_multi": (ctypes.c_int, [c_vp, c_u32, c_vp, c_vp, c_vp, c_u32, ctypes.c_char_p, c_u64,
                                                    P(CompactParams), c_u32, c_vp, c_u32, P(c_u32), c_vp, c_u64,
                                                    c_vp]),
        "sstc_compact_files": (ctypes.c_int, [c_vp, c_vp, c_vp, c_u32, ctypes.c_char_p, c_u64, P(CompactParams),
                                              c_u32, c_vp, c_u32, P(c_u32), c_vp, c_u64, P(FilesTiming)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, what):
    if rc != SSTC_OK:
        msg = load().sstc_last_error_string()
        raise SstcError(f"{what} failed ({rc}): {msg.decode() if msg else ''}", rc)
