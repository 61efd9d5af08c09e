

def test_reader_fixture_pins_oracle_decode(oracle):
    """tests/golden/readers_ref.json (the reference TableBuilder's files read by
    its own TableReader index + BlockReaderIterator): the oracle writes the same
    files and decodes the same record stream; live against oracle/_ref when built."""
    import hashlib
    import json
    import os
    import tempfile
    from conftest import GOLDEN
    from oracle import REF_SO, RefLib
    from readers_util import oracle_stream, reader_records, ref_stream
    want = json.load(open(os.path.join(GOLDEN, "readers_ref.json")))
    rec = reader_records()
    for bs, w in want.items():
        f = oracle.table_build(rec, int(bs))
        assert hashlib.sha256(f.tobytes()).hexdigest() == w["file_sha256"] and f.size + 1 == w["file_size"]
        stream, n = oracle_stream(oracle, f)
        assert n == w["records"] and hashlib.sha256(stream).hexdigest() == w["stream_sha256"]
        if os.path.exists(REF_SO):
            with tempfile.TemporaryDirectory() as td:
                p = os.path.join(td, "t.sst")
                f.tofile(p)
                assert ref_stream(RefLib(), p, f)[0] == stream
