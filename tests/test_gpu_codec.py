"""GPU parity: the HIP kernels (through the C-ABI) against the oracle and the
reference's golden fixtures.  Bit-exact everywhere (integer/byte work)."""
import os

import numpy as np
import pytest
import torch
from conftest import BLOCK_SETS, GOLDEN, REC_KEYS, golden_records, load_golden
from sstcodec import workload as W

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def codec():
    import sstcodec
    return sstcodec.Codec(0)


def t8(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.uint8)).to(DEV)


def t64(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(DEV)


def cpu_u64(t):
    return t.cpu().numpy().view(np.uint64)


def run_roundtrip(codec, src, offs, lens, mode=0, dst_fill=0):
    s = t8(src)
    d = torch.full_like(s, dst_fill)
    dst, out_len, status = codec.roundtrip(s, t64(offs), t64(lens), dst=d, txn_mode=mode)
    torch.cuda.synchronize()
    n = len(offs)
    return dst.cpu().numpy(), cpu_u64(out_len)[:n], status.cpu().numpy()[:n].astype(np.uint32)


def oracle_rt(oracle, src, offs, lens, mode=0, dst_fill=0):
    d, l, s, _ = oracle.roundtrip(src, offs, lens, mode)
    if dst_fill:
        # oracle writes into zeros; emulate a pre-filled destination
        base = np.full_like(src, dst_fill)
        for o, ln, st in zip(offs, l, s):
            if st == 0:
                base[int(o):int(o + ln)] = d[int(o):int(o + ln)]
        d = base
    return d, l, s


# ---------------------------------------------------------------- round trip
@pytest.mark.parametrize("name", BLOCK_SETS)
def test_roundtrip_golden(codec, name):
    g = load_golden(name)
    dst, out_len, status = run_roundtrip(codec, g["src"], g["blk_off"], g["blk_len"])
    assert (status == 0).all()
    assert np.array_equal(out_len, g["rt_len"])
    assert np.array_equal(dst, g["rt_dst"])
    dst1, _, _ = run_roundtrip(codec, g["src"], g["blk_off"], g["blk_len"], mode=1)
    assert np.array_equal(dst1, g["src"])


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("T", [4096, 32768])
def test_roundtrip_random_vs_oracle(codec, oracle, seed, T):
    rec = W.mixed_records(3000, seed=seed, max_val=1500 if T == 4096 else 5000)
    first = oracle.segment(rec, T)
    src, offs, lens = oracle.encode_blocks(rec, first, base=seed * 3)  # unaligned start
    src = np.concatenate([np.zeros(seed * 3, np.uint8), src, np.zeros(5, np.uint8)])
    for mode in (0, 1):
        got = run_roundtrip(codec, src, offs, lens, mode, dst_fill=0xA5)
        want = oracle_rt(oracle, src, offs, lens, mode, dst_fill=0xA5)
        assert np.array_equal(got[2], want[2])
        assert np.array_equal(got[1], want[1])
        assert np.array_equal(got[0], want[0])


def test_roundtrip_scattered_blocks(codec, oracle):
    """Blocks in arbitrary order with gaps between them (a batch gathered from
    several SSTs): every byte outside the blocks must stay untouched."""
    rec = W.mixed_records(2000, seed=42)
    first = oracle.segment(rec, 4096)
    data, offs, lens = oracle.encode_blocks(rec, first)
    rng = np.random.default_rng(0)
    order = rng.permutation(len(lens))
    gaps = rng.integers(0, 40, len(lens))
    parts, noffs, pos = [], np.zeros(len(lens), np.uint64), 0
    for g_, b in zip(gaps, order):
        parts.append(np.full(g_, 0x5A, np.uint8))
        pos += int(g_)
        noffs[b] = pos
        parts.append(data[int(offs[b]):int(offs[b] + lens[b])])
        pos += int(lens[b])
    src = np.concatenate(parts)
    got = run_roundtrip(codec, src, noffs, lens, 0, dst_fill=0x33)
    want = oracle_rt(oracle, src, noffs, lens, 0, dst_fill=0x33)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])


def test_roundtrip_non_canonical(codec, oracle):
    """Entries not packed (gap before the offset section, entries listed out of
    order): valid for the reference reader, re-encode packs them."""
    rec = W.mixed_records(40, seed=5, max_val=60)
    blk = oracle.encode_block(rec)
    n = 40
    D = int(blk[-8:].view(np.uint64)[0])
    offsec = blk[D:D + 16 * n].copy()
    # 1) 24 junk bytes between data section and offset section
    b1 = np.concatenate([blk[:D], np.full(24, 0xEE, np.uint8), offsec,
                         np.array([n], np.uint64).view(np.uint8), np.array([D + 24], np.uint64).view(np.uint8)])
    # 2) offset entries reversed (record order changes)
    rev = offsec.reshape(n, 16)[::-1].reshape(-1)
    b2 = np.concatenate([blk[:D], rev, blk[-16:]])
    src = np.concatenate([b1, np.zeros(7, np.uint8), b2])
    offs = np.array([0, b1.size + 7], np.uint64)
    lens = np.array([b1.size, b2.size], np.uint64)
    got = run_roundtrip(codec, src, offs, lens, 0, dst_fill=0x11)
    want = oracle_rt(oracle, src, offs, lens, 0, dst_fill=0x11)
    assert (got[2] == 0).all()
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0])
    assert got[1][0] == b1.size - 24


def test_roundtrip_errors(codec, oracle):
    g = load_golden("kat_basic.npz")
    good = g["src"]
    blocks = [good.copy() for _ in range(8)]
    blocks[1][-16:-8] = 0                                                   # EMPTY
    blocks[2][-8:] = np.array([10_000], np.uint64).view(np.uint8)           # OFFSETS_RANGE
    blocks[3][89 + 16:89 + 24] = np.array([88], np.uint64).view(np.uint8)   # ENTRY_RANGE
    blocks[4][28] = 7                                                       # BAD_TYPE
    blocks[5][29:33] = np.array([5000], np.uint32).view(np.uint8)           # KEY_TOO_LONG
    blocks[6] = blocks[6][:9]                                               # TOO_SMALL
    src = np.concatenate(blocks)
    lens = np.array([b.size for b in blocks], np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    codec.reset_errors()
    got = run_roundtrip(codec, src, offs, lens, 0, dst_fill=0x77)
    want = oracle_rt(oracle, src, offs, lens, 0, dst_fill=0x77)
    assert got[2].tolist() == [0, 2, 3, 4, 5, 6, 1, 0]
    assert np.array_equal(got[2], want[2])
    assert np.array_equal(got[0], want[0])
    assert codec.error_count() == 6


def test_roundtrip_empty_batch(codec):
    s = torch.zeros(16, dtype=torch.uint8, device=DEV)
    e = torch.zeros(0, dtype=torch.int64, device=DEV)
    codec.roundtrip(s, e, e)
    torch.cuda.synchronize()


# -------------------------------------------------------------------- decode
@pytest.mark.parametrize("name", BLOCK_SETS)
def test_decode_golden(codec, name):
    g = load_golden(name)
    for mode in (0, 1):
        table, rec_base, status = codec.decode(t8(g["src"]), t64(g["blk_off"]), t64(g["blk_len"]), txn_mode=mode)
        torch.cuda.synchronize()
        assert (status.cpu().numpy()[: len(g["blk_off"])] == 0).all()
        assert np.array_equal(cpu_u64(rec_base), g["dec_rec_base"])
        got = table.to_numpy()
        for k in REC_KEYS:
            want = g["dec_" + k]
            if k == "txn" and mode == 1:
                want = g["rec_txn"]  # blocks hold the records in order
            assert np.array_equal(got[k], want), (name, mode, k)


@pytest.mark.parametrize("seed", range(3))
def test_decode_random_vs_oracle(codec, oracle, seed):
    rec = W.mixed_records(5000, seed=20 + seed, max_val=900)
    first = oracle.segment(rec, 4096)
    src, offs, lens = oracle.encode_blocks(rec, first, base=1)
    src = np.concatenate([[9], src]).astype(np.uint8)
    table, rec_base, status = codec.decode(t8(src), t64(offs), t64(lens), txn_mode=1)
    got = table.to_numpy()
    # oracle per block, offsets absolute
    parts = {k: [] for k in REC_KEYS}
    for o, l in zip(offs, lens):
        st, d = oracle.decode_block(src[int(o):int(o + l)], 1, int(o))
        assert st == 0
        for k in REC_KEYS:
            parts[k].append(d[k])
    for k in REC_KEYS:
        assert np.array_equal(got[k], np.concatenate(parts[k])), k
    # decode(encode(records)) == records (keys/values compared by bytes)
    assert np.array_equal(got["txn"], rec["txn"]) and np.array_equal(got["type"], rec["type"])


@pytest.mark.parametrize("mode", [0, 1])
def test_pack_records_equals_decoded_columns(codec, oracle, mode):
    """sstc_pack_records, what the drop-in TableReaderIterator serves: every
    32 B sstc_record32 row holds the decoded record's key offset, txn (the
    compat quirk in mode 0, block_reader.cc:109-111), key length, value offset
    relative to the key (0 for a DELETE), value length (SSTC_NO_VALUE for a
    DELETE) and type -- DELETEs, empty keys and empty values included."""
    rec = W.mixed_records(6000, seed=41, max_val=700)
    first = oracle.segment(rec, 4096)
    src, offs, lens = oracle.encode_blocks(rec, first, base=3)
    src = np.concatenate([[1, 2, 3], src]).astype(np.uint8)
    table, _, status = codec.decode(t8(src), t64(offs), t64(lens), txn_mode=mode)
    assert int(status.max().item()) == 0
    rows = codec.pack(table).cpu().numpy()
    got = table.to_numpy()
    n = len(got["type"])
    assert rows.shape == (n, 32) and n == len(rec["type"])
    u64 = rows[:, :16].copy().view("<u8")
    u32 = rows[:, 16:28].copy().view("<u4")
    nv = got["val_len"] == np.uint32(0xFFFFFFFF)
    assert nv.any() and (got["val_len"] == 0).any() and (got["key_len"] == 0).any()
    assert np.array_equal(u64[:, 0], got["key_off"]) and np.array_equal(u64[:, 1], got["txn"])
    assert np.array_equal(u32[:, 0], got["key_len"]) and np.array_equal(u32[:, 2], got["val_len"])
    rel = np.where(nv, 0, got["val_off"] - got["key_off"]).astype(np.uint32)
    assert np.array_equal(u32[:, 1], rel)
    assert np.array_equal(rows[:, 28], got["type"])


# -------------------------------------------------------------------- encode
def records_table(rec):
    from sstcodec.codec import RecordTable
    return RecordTable.from_numpy(rec, torch.device(DEV))


@pytest.mark.parametrize("name", BLOCK_SETS)
def test_encode_golden(codec, name):
    g = load_golden(name)
    rec = golden_records(g)
    dst, off, ln = codec.encode(records_table(rec), t8(rec["key_src"]), t8(rec["val_src"]), t64(g["blk_first"]))
    torch.cuda.synchronize()
    assert np.array_equal(cpu_u64(ln), g["blk_len"])
    assert np.array_equal(cpu_u64(off)[:-1], g["blk_off"])
    assert np.array_equal(dst.cpu().numpy()[: g["src"].size], g["src"])


@pytest.mark.parametrize("seed", range(4))
def test_encode_random_vs_oracle(codec, oracle, seed):
    rec = W.mixed_records(4000, seed=50 + seed, max_val=3000 if seed % 2 else 200)
    T = [4096, 8192, 32768, 4096][seed]
    first = oracle.segment(rec, T)
    want, woff, wlen = oracle.encode_blocks(rec, first, base=seed)
    dst, off, ln = codec.encode(records_table(rec), t8(rec["key_src"]), t8(rec["val_src"]), t64(first),
                                out_base=seed)
    torch.cuda.synchronize()
    assert np.array_equal(cpu_u64(off)[:-1], woff) and np.array_equal(cpu_u64(ln), wlen)
    assert np.array_equal(dst.cpu().numpy()[seed:seed + want.size], want)


@pytest.mark.parametrize("seed", range(4))
def test_segment_vs_oracle(codec, oracle, seed):
    rec = W.mixed_records([1, 37, 3000, 20000][seed], seed=70 + seed, max_val=[10, 500, 5000, 300][seed])
    for T in (4096, 8192, 32768):
        want = oracle.segment(rec, T)
        got = cpu_u64(codec.segment(records_table(rec), T))
        assert np.array_equal(got, want), (seed, T)


def test_decode_then_encode_is_roundtrip(codec, oracle):
    """Unfused pipeline: decode -> (records stay in HBM) -> encode with the
    input block boundaries == fused round trip."""
    g = load_golden("blocks_mixed.npz")
    src = t8(g["src"])
    table, rec_base, status = codec.decode(src, t64(g["blk_off"]), t64(g["blk_len"]), txn_mode=0)
    dst, off, ln = codec.encode(table, src, src, rec_base)
    torch.cuda.synchronize()
    assert np.array_equal(dst.cpu().numpy()[: g["rt_dst"].size], g["rt_dst"])


# --------------------------------------------- full size (BASELINE configs)
def uniform_blocks(codec, nblocks, seed=1):
    n = nblocks * 28
    rec = W.uniform_records(n, seed=seed)
    first = np.arange(0, n + 1, 28, dtype=np.uint64)
    dst, off, ln = codec.encode(records_table(rec), t8(rec["key_src"]), t8(rec["val_src"]), t64(first))
    return rec, dst, off[:-1].contiguous(), ln


def test_config2_full_size_properties(codec, oracle):
    """65 536 x 4188 B blocks (bench.py's rank-0 input): encode(GPU) -> the
    whole buffer hashes to the reference BlockBuilder's encoding of the same
    records (tests/golden/bench_inputs.json) -> round trip -> identity; decode
    -> records equal the generator's; a sample of blocks equal the oracle's."""
    import hashlib
    import json
    nb = 65536
    rec, src, off, ln = uniform_blocks(codec, nb)
    torch.cuda.synchronize()
    assert int(ln.min()) == int(ln.max()) == 4188 and src.numel() == nb * 4188
    pins = json.load(open(os.path.join(GOLDEN, "bench_inputs.json")))["cases"]
    want_sha = [c["sha256"] for c in pins if c["rank"] == 0 and c["blocks"] == nb][0]
    assert hashlib.sha256(src.cpu().numpy().tobytes()).hexdigest() == want_sha, \
        "GPU-encoded config-2 buffer differs from the reference BlockBuilder's"
    dst, out_len, status = codec.roundtrip(src, off, ln, txn_mode=0)
    torch.cuda.synchronize()
    assert bool((status[:nb] == 0).all()) and bool((out_len[:nb] == 4188).all())
    assert torch.equal(dst, src)
    # sampled bit-exact check against the oracle encoder
    srcn = src.cpu().numpy()
    for b in (0, 1, 777, nb - 1):
        want = oracle.encode_block(rec, 28 * b, 28 * b + 28)
        assert np.array_equal(srcn[4188 * b:4188 * (b + 1)], want)
    table, rec_base, st = codec.decode(src, off, ln)
    got = table.to_numpy()
    assert np.array_equal(got["txn"], rec["txn"]) and (got["key_len"] == 16).all() and (got["val_len"] == 100).all()
    # key bytes gathered through the decoded offsets equal the generator's keys
    ko = got["key_off"][:1000].astype(np.int64)
    keys = srcn[ko[:, None] + np.arange(16)[None, :]]
    assert np.array_equal(keys.reshape(-1), rec["key_src"][:16000])


def test_roundtrip_overlapping_entries_no_room(codec, oracle):
    """Offset entries that all point at entry 0: valid to the reference reader,
    but the re-encoded block is longer than its slot -> NO_ROOM, untouched."""
    rec = W.mixed_records(30, seed=9, max_val=50)
    blk = oracle.encode_block(rec)
    D = int(blk[-8:].view(np.uint64)[0])
    big = blk.copy()
    n = 30
    offs_ = big[D:D + 16 * n].reshape(n, 16)
    offs_[:, :8] = 0  # every start -> 0
    # make entry 0 the largest so 30 copies overflow
    src = np.concatenate([big, blk])
    offs = np.array([0, big.size], np.uint64)
    lens = np.array([big.size, blk.size], np.uint64)
    got = run_roundtrip(codec, src, offs, lens, 0, dst_fill=0x42)
    want = oracle_rt(oracle, src, offs, lens, 0, dst_fill=0x42)
    assert np.array_equal(got[2], want[2]) and np.array_equal(got[0], want[0])
    assert np.array_equal(got[1], want[1])


def test_decode_count_mismatch(codec):
    g = load_golden("blocks_mixed.npz")
    rb = g["dec_rec_base"].copy()
    rb[1:] += 1  # block 0 claims one record more than its extra says
    table, _, status = codec.decode(t8(g["src"]), t64(g["blk_off"]), t64(g["blk_len"]), rec_base=t64(rb))
    torch.cuda.synchronize()
    st = status.cpu().numpy()[: len(g["blk_off"])]
    assert st[0] == 9 and (st[1:] == 0).all()


def test_roundtrip_large_blocks_streamed(codec, oracle):
    """Blocks larger than a wave's LDS slot (streamed path): 1-entry 64 KiB
    values, and 32 KiB-threshold blocks of small entries (offset section spans
    several windows), including compat txn rewrites in a large block."""
    items = []
    rng = np.random.default_rng(3)
    for i in range(12):
        items.append((0, b"big%03d" % i, rng.integers(0, 256, int(rng.integers(5000, 70000)), dtype=np.uint8).tobytes(), 10 + i))
    rec_big = _records(items)
    first_big = np.arange(0, 13, dtype=np.uint64)
    small = W.mixed_records(3000, seed=77, max_val=40, p_empty_val=0.2, p_delete=0.2)
    first_small = oracle.segment(small, 32768)
    for rec, first in ((rec_big, first_big), (small, first_small)):
        src, offs, lens = oracle.encode_blocks(rec, first, base=3)
        src = np.concatenate([np.zeros(3, np.uint8), src, np.zeros(1, np.uint8)])
        assert lens.max() > 4608
        for mode in (0, 1):
            got = run_roundtrip(codec, src, offs, lens, mode, dst_fill=0x5C)
            want = oracle_rt(oracle, src, offs, lens, mode, dst_fill=0x5C)
            assert (got[2] == 0).all()
            assert np.array_equal(got[1], want[1]) and np.array_equal(got[0], want[0])


def _records(items):
    import sys
    sys.path.insert(0, __import__("os").path.join(__import__("conftest").ROOT, "tests", "golden"))
    from make_golden import records_from_list
    return records_from_list(items)


def test_config5_zipf_blocks(codec, oracle):
    """Config 5 shape: Zipf(1.1) values clamped to [8 B, 64 KiB],
    10 % DELETE.  Most blocks hold one entry far above the 4 KiB threshold
    (streamed paths of rt_kernel and enc_emit_kernel), the rest pack small
    entries: segmentation, encode and the compat / correct round trips against
    the oracle."""
    rec = W.compaction_inputs(1, 1500, 3000, seed=11, vmin=8, vmax=65536, zipf=1.1, p_delete=0.1)[0]
    first = oracle.segment(rec, 4096)
    got_first = cpu_u64(codec.segment(records_table(rec), 4096))
    assert np.array_equal(got_first, first)
    want, woff, wlen = oracle.encode_blocks(rec, first, base=5)
    assert wlen.max() > 60000 and wlen.min() < 4608
    dst, off, ln = codec.encode(records_table(rec), t8(rec["key_src"]), t8(rec["val_src"]), t64(first),
                                out_base=5)
    torch.cuda.synchronize()
    assert np.array_equal(cpu_u64(off)[:-1], woff) and np.array_equal(cpu_u64(ln), wlen)
    img = dst.cpu().numpy()
    assert np.array_equal(img[5:5 + want.size], want)
    src = np.concatenate([np.zeros(5, np.uint8), want, np.zeros(3, np.uint8)])
    for mode in (0, 1):
        got = run_roundtrip(codec, src, woff, wlen, mode, dst_fill=0xA7)
        ref = oracle_rt(oracle, src, woff, wlen, mode, dst_fill=0xA7)
        assert (got[2] == 0).all()
        assert np.array_equal(got[1], ref[1]) and np.array_equal(got[0], ref[0])


def length_records(klen, vlen):
    """Records that carry only lengths (segmentation reads nothing else)."""
    n = len(klen)
    z = np.zeros(n, np.uint64)
    return {"type": np.zeros(n, np.uint8), "key_len": np.asarray(klen, np.uint32),
            "val_len": np.asarray(vlen, np.uint32), "txn": z, "key_off": z, "val_off": z,
            "key_src": np.zeros(1, np.uint8), "val_src": np.zeros(1, np.uint8)}


@pytest.mark.parametrize("case", ["tiny", "huge", "span_tiles", "mixed_runs", "no_value"])
def test_segment_tiles_vs_oracle(codec, oracle, case):
    """Block segmentation across many 2048-record tiles: entry windows of
    ~140 records (tiny entries), 1-record blocks (huge values), blocks that
    span several tiles (large thresholds), runs alternating between the two,
    and DELETE-shaped records without value fields."""
    rng = np.random.default_rng({"tiny": 1, "huge": 2, "span_tiles": 3, "mixed_runs": 4, "no_value": 5}[case])
    n = {"tiny": 150_000, "huge": 20_000, "span_tiles": 60_000, "mixed_runs": 80_000, "no_value": 50_000}[case]
    klen = rng.integers(0, 20, n)
    vlen = rng.integers(0, 12, n)
    if case == "huge":
        vlen = rng.integers(4000, 70_000, n)
    elif case == "mixed_runs":
        big = (np.arange(n) // 3000) % 2 == 1
        vlen = np.where(big, rng.integers(3000, 9000, n), vlen)
    elif case == "no_value":
        vlen = np.full(n, 0xFFFFFFFF)
    rec = length_records(klen, vlen)
    for T in ((4096, 1 << 20) if case == "span_tiles" else (4096, 32768)):
        want = oracle.segment(rec, T)
        got = cpu_u64(codec.segment(records_table(rec), T))
        assert np.array_equal(got, want), (case, T)


@pytest.mark.parametrize("case", ["serial_gate", "serial_fallback"])
def test_segment_serial_walk_vs_oracle(codec, oracle, case):
    """seg_walk_kernel's short-chain path (round 5): a 1024-record tile whose
    first segment predicts <= 48 segments walks its window chains serially,
    a walk past 64 segments falls back to pointer jumping.  serial_gate:
    constant-weight runs of 22 / 21 / 16 / 32-record blocks at T = 4096 (both
    sides of the 48 gate); serial_fallback: every tile starts with 600 tiny
    records (one ~565-record segment, so the gate says serial) and ends with
    424 one-record blocks (the walk passes 64 and the tile is redone by
    pointer jumping)."""
    if case == "serial_gate":
        n = 40_000
        w = np.array([190, 200, 256, 128])[(np.arange(n) // 5000) % 4]  # weight = 33 + key + value bytes
        klen, vlen, T = np.zeros(n, np.int64), w - 33, 4096
    else:
        n = 1024 * 40
        tiny = (np.arange(n) % 1024) < 600
        klen = np.zeros(n, np.int64)
        vlen = np.where(tiny, 0xFFFFFFFF, 20_000)  # no-value records weigh 29 B
        T = 16384
    rec = length_records(klen, vlen)
    want = oracle.segment(rec, T)
    got = cpu_u64(codec.segment(records_table(rec), T))
    assert np.array_equal(got, want), case
    if case == "serial_gate":  # the block lengths the runs were built for
        L = np.diff(want)
        assert {22, 21, 16, 32} <= set(L.tolist())


@pytest.mark.parametrize("case", ["uniform", "exact_fit", "one_record_blocks", "one_off_late", "one_off_first",
                                  "no_value"])
def test_segment_arithmetic_chain_vs_oracle(codec, oracle, case):
    """seg_arith_kernel / seg_arith_check_kernel (end of round 5): equal-sized
    entries take the arithmetic chain T, T + g, T + 2g, ... checked hop by hop;
    any other input must fall back to the general walk.  uniform: 149 B entries
    (config 2's shape, 28-record blocks, a short last block); exact_fit: blocks
    that reach the threshold exactly (W(q) == W(p) + T on every hop);
    one_record_blocks: values past the threshold (g = 1); one_off_late /
    one_off_first: equal entries but one record 3000 B heavier near the end /
    in the first block, so that block closes early (the chain's check fails on
    one hop / the first hop predicts the wrong g: the general walk); no_value:
    equal DELETE-shaped records."""
    n = 100_003
    klen = np.full(n, 16, np.int64)
    vlen = np.full(n, 100, np.int64)
    Ts = (4096, 32768)
    if case == "exact_fit":
        vlen[:] = 128 - 33 - 16  # weight (entry + offset entry) 33 + 16 + 79 = 128 B: T / 128 records per block
        Ts = (4096, 128 * 7)
    elif case == "one_record_blocks":
        vlen[:] = 5000
    elif case == "one_off_late":
        vlen[n - 777] += 3000
    elif case == "one_off_first":
        vlen[3] += 3000
    elif case == "no_value":
        vlen[:] = 0xFFFFFFFF
    rec = length_records(klen, vlen)
    for T in Ts:
        want = oracle.segment(rec, T)
        got = cpu_u64(codec.segment(records_table(rec), T))
        assert np.array_equal(got, want), (case, T)
        if case == "uniform":
            assert len(set(np.diff(want[:-1]).tolist())) == 1  # the arithmetic shape the fast path takes


@pytest.mark.parametrize("seed", range(3))
def test_encode_span_alignments_vs_oracle(codec, oracle, seed):
    """Keys / values at every source alignment (arena offsets shuffled, so
    spans start at any byte of a 16 B chunk), lengths 0..40 around the chunk
    and dword edges, DELETEs (no value fields), values spanning several chunk
    rounds, blocks of > 64 tiny records and blocks past an LDS slot."""
    rng = np.random.default_rng(300 + seed)
    n = 6000
    klen = rng.integers(0, 41, n).astype(np.uint32)
    vlen = rng.integers(0, 41, n).astype(np.uint32)
    big = rng.random(n) < 0.03
    vlen[big] = rng.integers(100, 6000, int(big.sum()))
    typ = (rng.random(n) < 0.15).astype(np.uint8)
    vlen[typ == 1] = W.NO_VALUE
    # arenas with gaps: every key / value at a random byte offset
    kgap = rng.integers(0, 16, n).astype(np.uint64)
    key_off = np.cumsum(klen.astype(np.uint64) + kgap) - klen.astype(np.uint64)
    vb = np.where(vlen == W.NO_VALUE, 0, vlen).astype(np.uint64)
    vgap = rng.integers(0, 16, n).astype(np.uint64)
    val_off = np.cumsum(vb + vgap) - vb
    rec = {"type": typ, "key_len": klen, "val_len": vlen, "txn": rng.integers(0, 2 ** 63, n, dtype=np.uint64),
           "key_off": key_off, "val_off": np.where(typ == 1, 0, val_off).astype(np.uint64),
           "key_src": rng.integers(0, 256, int(key_off[-1] + klen[-1]) + 1, dtype=np.uint8),
           "val_src": rng.integers(0, 256, int(val_off[-1] + vb[-1]) + 1, dtype=np.uint8)}
    T = [4096, 1024, 16384][seed]
    first = oracle.segment(rec, T)
    want, woff, wlen = oracle.encode_blocks(rec, first, base=seed * 5)
    dst, off, ln = codec.encode(records_table(rec), t8(rec["key_src"]), t8(rec["val_src"]), t64(first),
                                out_base=seed * 5)
    torch.cuda.synchronize()
    assert np.array_equal(cpu_u64(off)[:-1], woff) and np.array_equal(cpu_u64(ln), wlen)
    assert np.array_equal(dst.cpu().numpy()[seed * 5:seed * 5 + want.size], want)


def test_encode_many_blocks_of_many_records_vs_oracle(codec, oracle):
    """More than one workgroup's worth of blocks (> 2048: the one-kernel block
    offsets with the look-back over 256-block tiles) whose blocks hold ~90 tiny
    records each (past the 32 records whose loads the offsets kernel issues up
    front), a few blocks past the LDS slot, out_base unaligned."""
    rng = np.random.default_rng(808)
    n = 300_000
    klen = rng.integers(0, 13, n).astype(np.uint32)
    vlen = rng.integers(0, 13, n).astype(np.uint32)
    big = rng.random(n) < 0.0005
    vlen[big] = rng.integers(5000, 9000, int(big.sum()))
    typ = (rng.random(n) < 0.1).astype(np.uint8)
    vlen[typ == 1] = W.NO_VALUE
    key_off = np.cumsum(klen.astype(np.uint64)) - klen.astype(np.uint64)
    vb = np.where(vlen == W.NO_VALUE, 0, vlen).astype(np.uint64)
    val_off = np.cumsum(vb) - vb
    rec = {"type": typ, "key_len": klen, "val_len": vlen, "txn": rng.integers(0, 2 ** 63, n, dtype=np.uint64),
           "key_off": key_off, "val_off": np.where(typ == 1, 0, val_off).astype(np.uint64),
           "key_src": rng.integers(0, 256, int(key_off[-1] + klen[-1]) + 16, dtype=np.uint8),
           "val_src": rng.integers(0, 256, int(val_off[-1] + vb[-1]) + 16, dtype=np.uint8)}
    first = oracle.segment(rec, 4096)
    assert first.size - 1 > 2048
    want, woff, wlen = oracle.encode_blocks(rec, first, base=11)
    dst, off, ln = codec.encode(records_table(rec), t8(rec["key_src"]), t8(rec["val_src"]), t64(first),
                                out_base=11)
    torch.cuda.synchronize()
    o = cpu_u64(off)
    assert np.array_equal(o[:-1], woff) and np.array_equal(cpu_u64(ln), wlen) and int(o[-1]) == 11 + want.size
    assert np.array_equal(dst.cpu().numpy()[11:11 + want.size], want)


def test_encode_empty(codec):
    """No blocks: out_blk_off[0] = out_base, nothing written."""
    rec = W.uniform_records(0)
    first = torch.zeros(1, dtype=torch.int64, device=DEV)
    dst = torch.zeros(16, dtype=torch.uint8, device=DEV)
    d, off, ln = codec.encode(records_table(rec), t8(np.zeros(8, np.uint8)), t8(np.zeros(8, np.uint8)), first,
                              out_base=7, dst=dst)
    torch.cuda.synchronize()
    assert int(off[0]) == 7 and int(dst.abs().sum()) == 0


@pytest.mark.parametrize("nb", [5, 3000])
def test_encode_empty_blocks_null_columns(codec, oracle, nb):
    """nrec = 0 with NULL record columns and source pointers, nb empty block
    ranges (3000 > 2048: the one-kernel block offsets, which must not touch a
    record column for an empty block): every block is the 16 B image of
    BlockBuilder::EncodeExtraInfo on no entries (block_builder.cc:95-109)."""
    import ctypes
    from sstcodec._lib import Records, check
    first = torch.zeros(nb + 1, dtype=torch.int64, device=DEV)
    out_off = torch.empty(nb + 1, dtype=torch.int64, device=DEV)
    out_len = torch.empty(nb, dtype=torch.int64, device=DEV)
    base = 5
    dst = torch.full((base + 16 * nb + 16,), 0xAB, dtype=torch.uint8, device=DEV)
    codec._stream()
    null = ctypes.c_void_p(0)
    check(codec.lib.sstc_encode_blocks(codec.h, null, null, Records(0, 0, 0, 0, 0, 0), 0,
                                       ctypes.c_void_p(first.data_ptr()), nb, base, ctypes.c_void_p(dst.data_ptr()),
                                       ctypes.c_void_p(out_off.data_ptr()), ctypes.c_void_p(out_len.data_ptr())),
          "sstc_encode_blocks")
    torch.cuda.synchronize()
    rec = W.uniform_records(0)
    want, woff, wlen = oracle.encode_blocks(rec, np.zeros(nb + 1, np.uint64), base=base)
    assert want.size == 16 * nb and not want.any()
    assert np.array_equal(cpu_u64(out_off), np.append(woff, base + 16 * nb))
    assert np.array_equal(cpu_u64(out_len), wlen)
    d = dst.cpu().numpy()
    assert np.array_equal(d[base:base + 16 * nb], want)
    assert (d[:base] == 0xAB).all() and (d[base + 16 * nb:] == 0xAB).all()
