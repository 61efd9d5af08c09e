"""Reference-decoded record streams of the reader-boundary test's files.

    make -C oracle && python tests/golden/make_golden_readers.py

tests/test_gpu_cpp_boundary.py::test_cpp_block_readers_and_iterator reads two
SST files (3000 mixed records sorted by key, 4 KiB and 32 KiB blocks) through
the product's TableReader / BlockReader / TableReaderIterator and dumps the
records it saw.  Here the same files are written by the REFERENCE's
TableBuilder (oracle/_ref/libsstref.so: sstable/table_builder.cc) and read by
the reference's TableReader index and BlockReaderIterator
(sstable/table_reader.cc, sstable/block_reader_iterator.cc); the canonical dump
of that stream (tests/readers_util.py) is hashed.  Output: readers_ref.json.
"""
import hashlib
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "lsm-kv-storage_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import RefLib  # noqa: E402
from readers_util import reader_records, ref_stream  # noqa: E402


def main():
    ref = RefLib()
    rec = reader_records()
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for bs in (4096, 32768):
            p = os.path.join(td, f"r{bs}.sst")
            fs = ref.table_build(p, rec, bs)
            f = np.fromfile(p, np.uint8)
            stream, n = ref_stream(ref, p, f)
            out[str(bs)] = {"file_sha256": hashlib.sha256(f.tobytes()).hexdigest(), "file_size": int(fs),
                            "records": n, "stream_sha256": hashlib.sha256(stream).hexdigest(),
                            "stream_bytes": len(stream)}
    json.dump(out, open(os.path.join(HERE, "readers_ref.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
