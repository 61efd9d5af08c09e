"""CPU: pin the oracle (oracle/sst_oracle.c) to the reference.

(1) the known-answer vectors of the reference's own tests, restated byte for
byte; (2) the golden fixtures dumped from the reference by
tests/golden/make_golden.py; (3) live comparisons against the reference build
(oracle/_ref) when it is present.
"""
import os
import tempfile

import numpy as np
import pytest
from conftest import BLOCK_SETS, REC_KEYS, golden_records, load_golden
from sstcodec import workload as W


def u8(*chunks):
    out = []
    for c in chunks:
        out += list(c) if isinstance(c, (bytes, bytearray)) else c
    return np.array(out, np.uint8)


def le(v, n):
    return list(int(v).to_bytes(n, "little"))


# tests/test_block.cc:58-114 (BlockTest.BasicEncode)
KAT_BASIC = u8([0], le(5, 4), b"apple", le(6, 4), b"value1", [0x39, 0x30, 0, 0, 0, 0, 0, 0],
               [0], le(5, 4), b"apply", le(7, 4), b"success", [0x94, 0x26, 0, 0, 0, 0, 0, 0],
               [0], le(8, 4), b"colossus", le(7, 4), b"thunder", [0xFF, 0xFF, 0xFF, 0xFF, 0, 0, 0, 0],
               le(0, 8), le(0x1C, 8), le(0x1C, 8), le(0x1D, 8), le(0x39, 8), le(0x20, 8),
               le(3, 8), le(0x59, 8))
# tests/test_block.cc:141-176 (BlockTest.EdgeCasesEncode)
KAT_EDGE = u8([0], le(0, 4), le(0, 4), [0xA, 0, 0, 0, 0, 0, 0, 0], le(0, 8), le(0x11, 8), le(1, 8), le(0x11, 8))


def test_kat_basic(oracle):
    g = load_golden("kat_basic.npz")
    assert np.array_equal(oracle.encode_block(golden_records(g)), KAT_BASIC)
    assert np.array_equal(g["src"], KAT_BASIC)  # the reference agrees with its own test


def test_kat_edge(oracle):
    g = load_golden("kat_edge.npz")
    assert np.array_equal(oracle.encode_block(golden_records(g)), KAT_EDGE)
    assert np.array_equal(g["src"], KAT_EDGE)


def test_kat_table_mini(oracle):
    """tests/test_sst.cc:64-148: data section with txn 0, then the 230 B file.
    The test's unasserted block_index_buffer_encoded claims block size 0x86;
    the reference writes 0x99 = 89 + 48 + 16."""
    g = load_golden("table_mini.npz")
    rec = golden_records(g)
    f = oracle.table_build(rec, 4096)
    assert np.array_equal(f, g["sst"])
    assert f.size == 230 and int(g["file_size"][0]) == 231  # GetFileSize() = bytes + 1
    data = KAT_BASIC.copy()
    for e in (28, 57, 89):  # zero the three txns (test_sst.cc:64-92)
        data[e - 8:e] = 0
    assert np.array_equal(f[:89], data[:89])
    meta = u8(le(5, 4), b"apple", le(8, 4), b"colossus", le(0, 8), le(0x99, 8))
    assert np.array_equal(f[153:190], meta)
    assert np.array_equal(f[190:].view(np.uint64), np.array([1, 153, 37, 0, 0], np.uint64))


@pytest.mark.parametrize("name", BLOCK_SETS)
def test_golden_encode(oracle, name):
    g = load_golden(name)
    rec = golden_records(g)
    data, offs, lens = oracle.encode_blocks(rec, g["blk_first"])
    assert np.array_equal(data, g["src"])
    assert np.array_equal(offs, g["blk_off"]) and np.array_equal(lens, g["blk_len"])


@pytest.mark.parametrize("name", BLOCK_SETS)
def test_golden_decode(oracle, name):
    g = load_golden(name)
    rb = g["dec_rec_base"]
    for b, (o, l) in enumerate(zip(g["blk_off"], g["blk_len"])):
        st, d = oracle.decode_block(g["src"][int(o):int(o + l)], txn_mode=0, base=int(o))
        assert st == 0
        lo, hi = int(rb[b]), int(rb[b + 1])
        for k in REC_KEYS:
            assert np.array_equal(d[k], g["dec_" + k][lo:hi]), (name, b, k)


@pytest.mark.parametrize("name", BLOCK_SETS)
def test_golden_roundtrip(oracle, name):
    g = load_golden(name)
    dst, out_len, status, bad = oracle.roundtrip(g["src"], g["blk_off"], g["blk_len"], txn_mode=0)
    assert bad == 0 and (status == 0).all()
    assert np.array_equal(out_len, g["rt_len"])
    assert np.array_equal(dst, g["rt_dst"])


def test_golden_quirk_is_visible(oracle):
    """The empty-value PUTs of blocks_edge change txn in the reference's round
    trip: (txn & 0xffffffff) << 32.  CORRECT mode is the identity."""
    g = load_golden("blocks_edge.npz")
    assert not np.array_equal(g["rt_dst"], g["src"])
    b = 1  # the 70 empty-value PUTs
    lo, hi = int(g["dec_rec_base"][b]), int(g["dec_rec_base"][b + 1])
    want = (g["rec_txn"][150:220] & np.uint64(0xFFFFFFFF)) << np.uint64(32)
    assert np.array_equal(g["dec_txn"][lo:hi], want)
    dst, _, _, _ = oracle.roundtrip(g["src"], g["blk_off"], g["blk_len"], txn_mode=1)
    assert np.array_equal(dst, g["src"])


@pytest.mark.parametrize("T", [4096, 32768])
def test_golden_table(oracle, T):
    g = load_golden(f"table_mixed_{T}.npz")
    rec = golden_records(load_golden("blocks_mixed.npz"))
    f = oracle.table_build(rec, T)
    assert np.array_equal(f, g["sst"])
    idx = oracle.table_index(f)
    assert np.array_equal(idx["blk_off"], g["idx_blk_off"])
    assert np.array_equal(idx["blk_len"], g["idx_blk_len"])
    assert np.array_equal(idx["first_key_len"], g["idx_first_key_len"])
    assert np.array_equal(idx["last_key_len"], g["idx_last_key_len"])


def test_segment_matches_host_rule(oracle):
    for seed in range(4):
        rec = W.mixed_records(900, seed=seed, max_val=2000)
        for T in (4096, 8192, 32768):
            assert np.array_equal(oracle.segment(rec, T), W.segment(rec, T))


# ---- malformed blocks: codes are this framework's (the reference does not
#      validate), pinned here so the GPU kernels can be held to them ---------
def test_error_codes(oracle):
    good = KAT_BASIC.copy()
    assert oracle.decode_block(good)[0] == 0
    assert oracle.decode_block(good[:10])[0] == 1          # TOO_SMALL
    b = good.copy(); b[-16:-8] = 0
    assert oracle.decode_block(b)[0] == 2                  # EMPTY
    b = good.copy(); b[-8:] = u8(le(10_000, 8))
    assert oracle.decode_block(b)[0] == 3                  # OFFSETS_RANGE
    b = good.copy(); b[89 + 16:89 + 24] = u8(le(88, 8))
    assert oracle.decode_block(b)[0] == 4                  # ENTRY_RANGE
    b = good.copy(); b[28] = 7
    assert oracle.decode_block(b)[0] == 5                  # BAD_TYPE
    b = good.copy(); b[29:33] = u8(le(5000, 4))
    assert oracle.decode_block(b)[0] == 6                  # KEY_TOO_LONG


# ---- live comparison with the reference build (skipped without it) -------
@pytest.mark.parametrize("seed", range(3))
def test_live_reference(oracle, reflib, seed):
    rec = W.mixed_records(800, seed=100 + seed, max_val=3000)
    first = W.segment(rec, 4096)
    data, offs, lens = oracle.encode_blocks(rec, first)
    for b in range(len(first) - 1):
        blk = reflib.encode_block(rec, int(first[b]), int(first[b + 1]))
        assert np.array_equal(blk, data[int(offs[b]):int(offs[b] + lens[b])])
        d = reflib.decode_block(blk)
        st, o = oracle.decode_block(blk)
        assert st == 0 and all(np.array_equal(d[k], o[k]) for k in REC_KEYS)
    rd, rl, _ = reflib.roundtrip(data, offs, lens)
    od, ol, _, bad = oracle.roundtrip(data, offs, lens, 0)
    assert bad == 0 and np.array_equal(rd, od) and np.array_equal(rl, ol)
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "x.sst")
        fs = reflib.table_build(p, rec, 4096)
        assert np.array_equal(np.fromfile(p, np.uint8), oracle.table_build(rec, 4096))
        assert fs == os.path.getsize(p) + 1


def test_oracle_fuzz_self_consistent(oracle):
    """The corrupted-block set of tests/test_gpu_fuzz.py on the oracle alone:
    its round trip and its decode agree on every block's status (except
    NO_ROOM: a block that decodes but whose re-encoding outgrows its slot),
    and the set mixes valid blocks with several distinct fault codes."""
    from fuzz_blocks import fuzz_blocks
    src, offs, lens, _ = fuzz_blocks(oracle, 0, nrec=3000)
    _, _, st, _ = oracle.roundtrip(src, offs, lens, 0)
    dec = np.array([oracle.decode_block(src[int(o):int(o + n)], 0, int(o))[0] for o, n in zip(offs, lens)])
    no_room = st == 8  # ORC_BLK_NO_ROOM
    assert (dec[no_room] == 0).all() and no_room.any()
    assert np.array_equal(st[~no_room], dec[~no_room])
    assert (st == 0).any() and len(set(st.tolist())) >= 5
