"""GPU: sstc_open_tables (footer + meta section parse on the device,
sstable/table_reader.cc:52-156) against the reference's own index fixtures
and the oracle's sequential walk (oracle/sst_oracle.c orc_table_index)."""
import numpy as np
import pytest
from conftest import golden_records, load_golden
from sstcodec import workload as W

pytestmark = pytest.mark.gpu

TAB_OK, TAB_BAD_FOOTER, TAB_BAD_META, TAB_BAD_BLOCK = 0, 1, 2, 3


@pytest.fixture(scope="module")
def codec():
    import sstcodec
    return sstcodec.Codec(0)


def _dev(codec, arr):
    import torch
    return torch.from_numpy(np.ascontiguousarray(arr, np.uint8)).to(codec.device)


def _place(tables, gaps):
    """Tables back to back with `gaps[t]` junk bytes before table t (unaligned)."""
    parts, offs, pos = [], [], 0
    rng = np.random.default_rng(len(tables))
    for f, g in zip(tables, gaps):
        parts.append(rng.integers(0, 256, g, dtype=np.uint8))
        pos += g
        offs.append(pos)
        parts.append(f)
        pos += f.size
    return np.concatenate(parts), np.asarray(offs, np.uint64)


def _check_vs_oracle(codec, oracle, tables, gaps=None):
    gaps = gaps or [0] * len(tables)
    src, offs = _place(tables, gaps)
    idx = codec.open_tables(_dev(codec, src), [f.size for f in tables], tab_off=offs)
    tfb = idx["table_first_block"]
    got = {k: idx[k].cpu().numpy() for k in ("blk_off", "blk_len", "first_key_off", "first_key_len",
                                             "last_key_off", "last_key_len")}
    assert np.array_equal(idx["table_first_block_dev"].cpu().numpy().view(np.uint64), tfb)
    for t, f in enumerate(tables):
        ref = oracle.table_index(f, cap=f.size // 24 + 1)
        st = int(idx["status"][t])
        if ref is None:
            assert st in (TAB_BAD_FOOTER, TAB_BAD_META), (t, st)
            continue
        assert st in (TAB_OK, TAB_BAD_BLOCK), (t, st)
        lo, hi = int(tfb[t]), int(tfb[t + 1])
        assert hi - lo == ref["nblocks"]
        base = np.uint64(offs[t])
        for k in ("blk_off", "first_key_off", "last_key_off"):
            assert np.array_equal(got[k][lo:hi].view(np.uint64), ref[k] + base), (t, k)
        assert np.array_equal(got["blk_len"][lo:hi].view(np.uint64), ref["blk_len"])
        for k in ("first_key_len", "last_key_len"):
            assert np.array_equal(got[k][lo:hi].view(np.uint32), ref[k]), (t, k)
        foot = f[f.size - 40:].view(np.uint64)
        assert np.array_equal(idx["footer"][t], foot)
        moff = int(foot[1])
        in_data = np.all((ref["blk_off"] <= moff) & (ref["blk_len"] <= moff - ref["blk_off"]))
        assert st == (TAB_OK if in_data else TAB_BAD_BLOCK)
    return idx


def fake_table(seed, nb, max_key, data_bytes=4096, p_big=0.0):
    """A table image whose meta entries have random key lengths (0 .. max_key,
    a fraction p_big of them up to 40000 B so entries span several 32 KiB
    tiles); block ranges inside the data section."""
    rng = np.random.default_rng(seed)
    fk = rng.integers(0, max_key + 1, nb)
    lk = rng.integers(0, max_key + 1, nb)
    big = rng.random(nb) < p_big
    fk[big] = rng.integers(4096, 40000, big.sum())
    parts = [rng.integers(0, 256, data_bytes, dtype=np.uint8)]
    for i in range(nb):
        bo = int(rng.integers(0, data_bytes))
        bl = int(rng.integers(0, data_bytes - bo + 1))
        parts += [np.array([fk[i]], "<u4").view(np.uint8), rng.integers(0, 256, fk[i], dtype=np.uint8),
                  np.array([lk[i]], "<u4").view(np.uint8), rng.integers(0, 256, lk[i], dtype=np.uint8),
                  np.array([bo, bl], "<u8").view(np.uint8)]
    body = np.concatenate(parts)
    foot = np.array([nb, data_bytes, body.size - data_bytes, 3, 99], "<u8").view(np.uint8)
    return np.concatenate([body, foot])


def test_open_golden_tables(codec):
    mini = load_golden("table_mini.npz")["sst"]
    g4, g32 = load_golden("table_mixed_4096.npz"), load_golden("table_mixed_32768.npz")
    idx = codec.open_tables(_dev(codec, np.concatenate([mini, g4["sst"], g32["sst"]])),
                            [mini.size, g4["sst"].size, g32["sst"].size], strict=True)
    tfb = idx["table_first_block"]
    assert list(idx["footer"][0]) == [1, 153, 37, 0, 0]  # tests/test_sst.cc footer of the 230 B table
    assert int(tfb[1]) == 1 and int(idx["blk_off"][0]) == 0 and int(idx["blk_len"][0]) == 153
    base = mini.size
    for t, g in ((1, g4), (2, g32)):
        lo, hi = int(tfb[t]), int(tfb[t + 1])
        assert np.array_equal(idx["blk_off"][lo:hi].cpu().numpy().view(np.uint64), g["idx_blk_off"] + np.uint64(base))
        assert np.array_equal(idx["blk_len"][lo:hi].cpu().numpy().view(np.uint64), g["idx_blk_len"])
        assert np.array_equal(idx["first_key_len"][lo:hi].cpu().numpy().view(np.uint32), g["idx_first_key_len"])
        assert np.array_equal(idx["last_key_len"][lo:hi].cpu().numpy().view(np.uint32), g["idx_last_key_len"])
        base += g["sst"].size


def test_open_built_tables_vs_oracle(codec, oracle):
    rec_small = W.mixed_records(20000, seed=11, max_key=48, max_val=60)
    rec_long = W.mixed_records(3000, seed=12, max_key=4096, max_val=300)
    tables = [oracle.table_build(rec_small, 64),     # ~1 record per block: meta spans many tiles
              oracle.table_build(rec_small, 4096),
              oracle.table_build(rec_long, 4096),    # entries up to 8 KiB span tile edges
              oracle.table_build(golden_records(load_golden("blocks_mixed.npz")), 4096)]
    idx = _check_vs_oracle(codec, oracle, tables, gaps=[0, 3, 17, 1])
    assert (idx["status"] == TAB_OK).all()


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_open_fake_meta_vs_oracle(codec, oracle, seed):
    # 24 B entries (empty keys): 1365 chain positions per tile, the doubling bound;
    # huge keys: the chain skips whole tiles
    tables = [fake_table(seed, 5000, 0), fake_table(seed + 10, 3000, 40, p_big=0.0),
              fake_table(seed + 20, 60, 300, p_big=0.3), fake_table(seed + 30, 1, 5)]
    _check_vs_oracle(codec, oracle, tables, gaps=[5, 0, 2, 9])


def test_open_malformed(codec, oracle):
    good = fake_table(7, 500, 30)
    f = good[good.size - 40:].view(np.uint64)
    moff, mlen = int(f[1]), int(f[2])
    cases = []
    t = good.copy()
    t[-40:-32] = np.array([501], "<u8").view(np.uint8)  # one entry more than the section holds
    cases.append(t)
    t = good.copy()
    t[-32:-24] = np.array([good.size], "<u8").view(np.uint8)  # meta offset past the image
    cases.append(t)
    t = good.copy()
    t[moff + 100] ^= 0x40  # a length field inside the chain grows past the section (or not)
    cases.append(t)
    t = good.copy()
    t[moff:moff + 4] = np.array([mlen], "<u4").view(np.uint8)  # first key runs past the section
    cases.append(t)
    cases.append(good[-30:].copy())  # shorter than a footer
    t = good.copy()
    # block range outside the data section: last 16 B of the first entry
    fkl = int(good[moff:moff + 4].view("<u4")[0])
    lkl = int(good[moff + 4 + fkl:moff + 8 + fkl].view("<u4")[0])
    t[moff + 8 + fkl + lkl:moff + 16 + fkl + lkl] = np.array([moff + 1], "<u8").view(np.uint8)
    cases.append(t)
    idx = _check_vs_oracle(codec, oracle, [good] + cases, gaps=[0] * (len(cases) + 1))
    st = list(idx["status"])
    assert st[0] == TAB_OK and st[1] == TAB_BAD_META and st[2] == TAB_BAD_FOOTER
    assert st[4] == TAB_BAD_META and st[5] == TAB_BAD_FOOTER and st[6] == TAB_BAD_BLOCK
    with pytest.raises(Exception):
        codec.open_tables(_dev(codec, good), [good.size], strict=True, max_blocks=10)


def test_open_empty(codec):
    idx = codec.open_tables(_dev(codec, np.zeros(1, np.uint8)), [])
    assert list(idx["table_first_block"]) == [0]
    nb0 = np.concatenate([np.zeros(5, np.uint8), np.array([0, 5, 0, 0, 0], "<u8").view(np.uint8)])
    idx = codec.open_tables(_dev(codec, nb0), [nb0.size], strict=True)
    assert list(idx["table_first_block"]) == [0, 0]
