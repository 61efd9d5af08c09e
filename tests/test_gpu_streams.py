"""A context used from two streams back to back (sstc_ctx_set_stream orders the
new stream after the old one: the workspace is shared by every call), and a
file pipeline created while another device is current (it binds the
context's device).  Results must equal the single-stream ones / the oracle."""
import numpy as np
import pytest
import torch
from sstcodec import workload as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    import sstcodec
    return sstcodec.Codec(0)


def _blocks(oracle, n, seed):
    rec = W.mixed_records(n, seed=seed)
    first = W.segment(rec, 4096)
    return oracle.encode_blocks(rec, first)


def test_two_streams_back_to_back(codec, oracle):
    dev = torch.device("cuda", 0)
    sets = [_blocks(oracle, 6000 + 500 * k, 70 + k) for k in range(4)]
    want = []
    for src, off, ln in sets:
        st, rec = zip(*[oracle.decode_block(src[int(o):int(o + l)], 0, int(o)) for o, l in zip(off, ln)])
        want.append({k: np.concatenate([r[k] for r in rec]) for k in rec[0]})
    dsets = [(torch.from_numpy(s).to(dev), torch.from_numpy(o.view(np.int64)).to(dev),
              torch.from_numpy(l.view(np.int64)).to(dev)) for s, o, l in sets]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    torch.cuda.synchronize()
    outs = []
    for k, (s, o, l) in enumerate(dsets):  # alternate streams: count + decode share scan / record workspace
        with torch.cuda.stream(streams[k % 2]):
            for t in (s, o, l):
                t.record_stream(streams[k % 2])
            table, rec_base, status = codec.decode(s, o, l)
            outs.append((table, rec_base, status))
    torch.cuda.synchronize()
    for (table, rec_base, status), w in zip(outs, want):
        assert int(status.abs().sum()) == 0
        got = table.to_numpy()
        for key in ("type", "key_len", "val_len", "txn", "key_off", "val_off"):
            assert np.array_equal(got[key], w[key]), key


def test_encode_two_streams(codec, oracle):
    """sstc_encode_blocks (scan workspace + large-block list) on two streams."""
    dev = torch.device("cuda", 0)
    from sstcodec.codec import RecordTable
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    res = []
    for k in range(4):
        rec = W.mixed_records(5000 + 300 * k, seed=90 + k, max_val=3000 if k % 2 else 300)
        first = W.segment(rec, 4096)
        want, _, _ = oracle.encode_blocks(rec, first)
        with torch.cuda.stream(streams[k % 2]):
            table = RecordTable.from_numpy(rec, dev)
            ks = torch.from_numpy(rec["key_src"]).to(dev)
            vs = torch.from_numpy(rec["val_src"]).to(dev)
            f = torch.from_numpy(first.view(np.int64)).to(dev)
            dst, _, _ = codec.encode(table, ks, vs, f)
            res.append((dst, want, (table, ks, vs, f)))
    torch.cuda.synchronize()
    for dst, want, _ in res:
        assert np.array_equal(dst.cpu().numpy()[: want.size], want)
