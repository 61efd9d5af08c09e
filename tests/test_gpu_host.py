"""GPU: sstc_roundtrip_host (host-resident blocks streamed through the device
in chunks over upload / kernel / download streams) against the oracle's
round trip on the corrupted-block set and on gapped, unaligned layouts."""
import numpy as np
import pytest
import torch
from fuzz_blocks import fuzz_blocks
from sstcodec import workload as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    import sstcodec
    return sstcodec.Codec(0)


def pinned(a):
    t = torch.empty(a.size, dtype=torch.uint8, pin_memory=True)
    t.numpy()[:] = a
    return t


def check_vs_oracle(codec, oracle, src, offs, lens, mode, chunk):
    h_src = pinned(src)
    h_dst = pinned(np.full(src.size, 0x5A, np.uint8))
    out_len, st = codec.roundtrip_host(h_src, h_dst, offs, lens, txn_mode=mode, chunk_bytes=chunk)
    want_d, want_len, want_st, _ = oracle.roundtrip(src, offs, lens, mode)
    assert np.array_equal(st, want_st)
    assert np.array_equal(out_len[want_st == 0], want_len[want_st == 0])
    got = h_dst.numpy()
    for o, ln, wl, s in zip(offs, lens, want_len, want_st):
        o = int(o)
        if s == 0:
            assert np.array_equal(got[o:o + int(wl)], want_d[o:o + int(wl)])
        else:  # a rejected block keeps its source bytes
            assert np.array_equal(got[o:o + int(ln)], src[o:o + int(ln)])
    return st


@pytest.mark.parametrize("seed,T,mode,chunk", [(0, 4096, 0, 4096), (1, 4096, 1, 20000), (2, 32768, 0, 1 << 20),
                                               (3, 32768, 1, 70000)])
def test_host_roundtrip_fuzz(codec, oracle, seed, T, mode, chunk):
    src, offs, lens, _ = fuzz_blocks(oracle, seed, T=T)
    st = check_vs_oracle(codec, oracle, src, offs, lens, mode, chunk)
    assert 0 < (st == 0).sum() < len(offs)


def test_host_roundtrip_gaps_unaligned(codec, oracle):
    rec = W.mixed_records(8000, seed=21, max_val=500)
    first = W.segment(rec, 4096)
    data, offs, lens = oracle.encode_blocks(rec, first)
    rng = np.random.default_rng(5)
    parts, new_off, pos = [], [], 0
    for o, ln in zip(offs, lens):
        g = int(rng.integers(0, 40))
        parts.append(rng.integers(0, 256, g, dtype=np.uint8))
        pos += g
        new_off.append(pos)
        parts.append(data[int(o):int(o + ln)])
        pos += int(ln)
    src = np.concatenate(parts)
    noff = np.asarray(new_off, np.uint64)
    for chunk in (4096, 9000, 1 << 24):
        st = check_vs_oracle(codec, oracle, src, noff, lens, 1, chunk)
        assert (st == 0).all()


def test_host_roundtrip_identity_config2_shape(codec):
    import bench
    dev = torch.device("cuda", 0)
    src, off, ln = bench.make_blocks(codec, dev, 8192, 0)
    h_src = pinned(src.cpu().numpy())
    h_dst = pinned(np.zeros(src.numel(), np.uint8))
    o = off.cpu().numpy().view(np.uint64)
    n = ln.cpu().numpy().view(np.uint64)
    out_len, st = codec.roundtrip_host(h_src, h_dst, o, n, chunk_bytes=4 << 20)
    assert (st == 0).all() and np.array_equal(out_len, n)
    assert torch.equal(h_dst, h_src)


def test_host_roundtrip_rejects_bad_layout(codec):
    src = pinned(np.zeros(10000, np.uint8))
    dst = pinned(np.zeros(10000, np.uint8))
    with pytest.raises(Exception):  # overlapping blocks
        codec.roundtrip_host(src, dst, np.array([0, 100], np.uint64), np.array([200, 200], np.uint64))
    with pytest.raises(Exception):  # past the buffer
        codec.roundtrip_host(src, dst, np.array([9000], np.uint64), np.array([2000], np.uint64))
