"""Corrupted blocks (tests/fuzz_blocks.py: bad entry counts, offset-section
starts, entry starts, type bytes, key / value lengths, random bytes, truncated
slots) through the GPU decode and round trip, against the oracle: the same
status code for every block, the same records for every block that decodes,
and the same output bytes (a failing block leaves its output slot untouched).
The status codes are this framework's (the reference asserts or reads out of
range on such blocks), so this pins GPU == oracle, not GPU == reference."""
import numpy as np
import pytest
import torch
from conftest import REC_KEYS
from fuzz_blocks import fuzz_blocks

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


CASES = [(0, 4096, 0), (1, 4096, 1), (2, 32768, 0), (3, 32768, 1)]


@pytest.mark.parametrize("seed,T,mode", CASES)
def test_roundtrip_fuzz_vs_oracle(codec, oracle, seed, T, mode):
    src, offs, lens, _ = fuzz_blocks(oracle, seed, T=T)
    d = torch.full((src.size,), 0x5A, dtype=torch.uint8, device=DEV)
    dst, out_len, status = codec.roundtrip(t8(src), t64(offs), t64(lens), dst=d, txn_mode=mode)
    torch.cuda.synchronize()
    n = len(offs)
    got_st = status.cpu().numpy()[:n].astype(np.uint32)
    got_len = out_len.cpu().numpy().view(np.uint64)[:n]
    want_d, want_len, want_st, _ = oracle.roundtrip(src, offs, lens, mode)
    assert np.array_equal(got_st, want_st)
    assert 0 < (want_st == 0).sum() < n and len(set(want_st.tolist())) >= 5  # the set really mixes faults
    assert np.array_equal(got_len, want_len)
    exp = np.full(src.size, 0x5A, np.uint8)
    for o, ln, st in zip(offs, want_len, want_st):
        if st == 0:
            exp[int(o):int(o + ln)] = want_d[int(o):int(o + ln)]
    assert np.array_equal(dst.cpu().numpy(), exp)


@pytest.mark.parametrize("seed,T,mode", CASES)
def test_decode_fuzz_vs_oracle(codec, oracle, seed, T, mode):
    src, offs, lens, _ = fuzz_blocks(oracle, seed, T=T)
    table, rec_base, status = codec.decode(t8(src), t64(offs), t64(lens), txn_mode=mode)
    got = table.to_numpy()
    rb = rec_base.cpu().numpy().view(np.uint64)
    st = status.cpu().numpy()[:len(offs)].astype(np.uint32)
    for b, (o, ln) in enumerate(zip(offs, lens)):
        want_st, want = oracle.decode_block(src[int(o):int(o + ln)], mode, int(o))
        assert st[b] == want_st, b
        if want_st == 0:
            for k in REC_KEYS:
                assert np.array_equal(got[k][int(rb[b]):int(rb[b + 1])], want[k]), (b, k)
