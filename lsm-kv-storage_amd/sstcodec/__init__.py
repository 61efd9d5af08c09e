"""sstcodec — MI355X (gfx950) SST block codec for NamHoaiNguyen/LSM-KV-Storage.

Python face of libsstcodec.so (include/sstcodec.h).  Import this package with
`lsm-kv-storage_amd/` on sys.path (the directory name is not an identifier):

    import sys; sys.path.insert(0, "<repo>/lsm-kv-storage_amd")
    import sstcodec
"""
from . import workload  # noqa: F401  (numpy only)
from ._lib import (BLK_STATUS, LIB_PATH, SSTC_NO_VALUE, SSTC_TXN_COMPAT, SSTC_TXN_CORRECT,  # noqa: F401
                   SstcError, load)


def __getattr__(name):
    # torch-facing classes are imported lazily so that CPU-only tooling can use
    # the workload generator without importing torch.
    if name in ("Codec", "RecordTable", "FilePipe", "Lookup"):
        from . import codec
        return getattr(codec, name)
    raise AttributeError(name)
