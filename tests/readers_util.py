"""The record stream of an SST file in the canonical dump format (per record:
u8 type, u64 txn, u32 key length, key, u8 value-is-non-null, u32 value length,
value; little endian) that tests/cpp/readers_check.cc --readers writes from
the sstc::TableReader iterators (tests/test_gpu_dropin.py compares the two),
made from block decodes of the file's index.  With RefLib (the reference's own
TableReader index + BlockReaderIterator, oracle/_ref/libsstref.so) it is the
reference-decoded stream; with the oracle it is the restatement's."""
import struct

import numpy as np
from sstcodec import workload as W

NO_VALUE = 0xFFFFFFFF


def dump_records(blocks):
    """blocks: iterable of (block bytes, decoded dict with block-relative offsets)"""
    out = bytearray()
    n = 0
    for blk, d in blocks:
        blk = bytes(blk)
        for i in range(len(d["type"])):
            kl, vl = int(d["key_len"][i]), int(d["val_len"][i])
            ko = int(d["key_off"][i])
            out += struct.pack("<BQI", int(d["type"][i]), int(d["txn"][i]), kl) + blk[ko:ko + kl]
            if vl == NO_VALUE:
                out += struct.pack("<BI", 0, 0)
            else:
                vo = int(d["val_off"][i])
                out += struct.pack("<BI", 1, vl) + blk[vo:vo + vl]
            n += 1
    return bytes(out), n


def ref_stream(ref, path, file_bytes):
    """The reference's TableReader index + BlockReaderIterator over every block."""
    idx = ref.table_index(path, file_bytes.size + 1)
    blocks = []
    for o, ln in zip(idx["blk_off"], idx["blk_len"]):
        blk = np.ascontiguousarray(file_bytes[int(o):int(o) + int(ln)])
        blocks.append((blk, ref.decode_block(blk)))
    return dump_records(blocks)


def oracle_stream(oracle, file_bytes):
    idx = oracle.table_index(file_bytes)
    blocks = []
    for o, ln in zip(idx["blk_off"], idx["blk_len"]):
        blk = np.ascontiguousarray(file_bytes[int(o):int(o) + int(ln)])
        st, d = oracle.decode_block(blk)
        assert st == 0
        d["val_len"] = np.where(d["type"] == 1, NO_VALUE, d["val_len"]).astype(np.uint32)  # DELETE: null view
        blocks.append((blk, d))
    return dump_records(blocks)


def reader_records():
    """the reader-boundary test's records: W.mixed_records(3000, seed=5) stably sorted by key"""
    rec = W.mixed_records(3000, seed=5)
    order = np.lexsort((np.arange(3000), [bytes(rec["key_src"][int(o):int(o) + int(k)])
                                          for o, k in zip(rec["key_off"], rec["key_len"])]))
    return {k: (v[order] if v.size == 3000 else v) for k, v in rec.items()}
