"""A context used from two streams back to back (sstc_ctx_set_stream orders the
new stream after the old one: the workspace is shared by every call).  Every
input holds more than kScanTile (2048) blocks, so the device scans run as
multi-tile decoupled look-backs whose status words are shared by the calls on
both streams.  Results must equal the oracle's.  Also: dropping a stream the
caller destroys (sstc_ctx_drop_stream) and scans across the 14-bit epoch wrap
of a context's scan workspace."""
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
    sets = [_blocks(oracle, 48_000 + 500 * k, 70 + k) for k in range(4)]
    assert all(len(o) > 2048 for _, o, _ in sets)  # multi-tile look-back scans
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
        rec = W.mixed_records(60_000 + 300 * k, seed=90 + k, max_val=3000 if k % 2 else 300)
        first = W.segment(rec, 4096)
        assert len(first) - 1 > 2048  # the block-length scan spans several tiles
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


def test_drop_stream_then_destroy(oracle):
    """sstc_ctx_drop_stream: a caller synchronizes the context's stream, drops
    it (nothing is recorded on it) and destroys it; the next
    sstc_ctx_set_stream (which records the switch on the current stream) then
    works, where without the drop it would record on a destroyed stream."""
    import ctypes
    import sstcodec
    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.device("cuda", 0)
    codec = sstcodec.Codec(0)
    src, off, ln = _blocks(oracle, 3000, 5)
    s, o, l = (torch.from_numpy(src).to(dev), torch.from_numpy(off.view(np.int64)).to(dev),
               torch.from_numpy(ln.view(np.int64)).to(dev))
    rb = torch.empty(len(off) + 1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    raw = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(raw)) == 0
    assert codec.lib.sstc_ctx_set_stream(codec.h, raw) == 0
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    assert codec.lib.sstc_count_records(codec.h, P(s), P(o), P(l), len(off), P(rb)) == 0
    assert hip.hipStreamSynchronize(raw) == 0
    assert codec.lib.sstc_ctx_drop_stream(codec.h) == 0
    assert hip.hipStreamDestroy(raw) == 0
    table, _, status = codec.decode(s, o, l)  # switches the context to torch's current stream
    torch.cuda.synchronize()
    want = sum(len(oracle.decode_block(src[int(a):int(a + b)], 0)[1]["type"]) for a, b in zip(off, ln))
    assert int(status.abs().sum()) == 0 and table.n == want == int(rb[-1])
    codec.close()


def test_scans_across_epoch_wrap(oracle):
    """A context tags its scans with a 14-bit epoch and clears the workspace
    when it wraps (sstc_api.hip next_epoch): with the epoch set just below the
    wrap (test hook sstc__ctx_set_scan_epoch), segmentation and encode calls
    across it, on inputs of several scan tiles, equal the oracle's."""
    import sstcodec
    from sstcodec.codec import RecordTable
    dev = torch.device("cuda", 0)
    codec = sstcodec.Codec(0)
    rec = W.mixed_records(50_000, seed=123, max_val=400)
    first = W.segment(rec, 4096)
    want, _, _ = oracle.encode_blocks(rec, first)
    table = RecordTable.from_numpy(rec, dev)
    ks, vs = torch.from_numpy(rec["key_src"]).to(dev), torch.from_numpy(rec["val_src"]).to(dev)
    assert codec.lib.sstc__ctx_set_scan_epoch(codec.h, (1 << 14) - 3) == 0
    for _ in range(6):  # crosses the wrap (epochs 16382, 16383 -> clear -> 1, 2, ...)
        f = codec.segment(table, 4096)
        assert np.array_equal(f.cpu().numpy().view(np.uint64), first)
        dst, _, _ = codec.encode(table, ks, vs, f)
        assert np.array_equal(dst.cpu().numpy()[: want.size], want)
    codec.close()
