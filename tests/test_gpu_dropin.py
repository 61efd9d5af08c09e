"""The drop-in of INTEGRATION.md, run: oracle/_ref/compact_dropin is
/root/reference/db/compact.cc (Compact::PickCompact -> DoCompactJob) compiled
UNCHANGED with include/dropin/sstable/table_builder.h first on the include
path, so every output SST it builds goes through sstc::TableBuilder (blocks
encoded on this GPU at Finish()).  Its outputs must be the reference's own
bytes.  (The binary is built in the container by `make -C oracle dropin`,
tests/test_oracle_aswritten.py::test_dropin_builds_unmodified_compact_cc, and
travels with the tree like libsstcodec.so.)

Cases: those whose as-written output equals the fixed semantics under both
allocator settings (tests/golden/aswritten.json), since this binary runs the
reference's dangling `last_current_key` as written (compact.cc:250)."""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest
from conftest import GOLDEN, ROOT

sys.path.insert(0, GOLDEN)
import make_golden_aswritten as G  # noqa: E402

pytestmark = pytest.mark.gpu
MANIFEST = json.load(open(os.path.join(GOLDEN, "aswritten.json")))
EXE = os.path.join(ROOT, "oracle", "_ref", "compact_dropin")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.uint8).tobytes()).hexdigest()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name", ["probe100", "config3"])
def test_reference_compaction_with_dropin_table_builder(tmp_path, name):
    if not os.path.exists(EXE):
        pytest.skip("oracle/_ref/compact_dropin not built (needs /root/reference at build time)")
    import sstcodec
    from oracle import table_key_range
    from sstcodec.table import build_table
    case = MANIFEST[name]
    assert case["no_trim_equals_fixed"] and case["default_equals_fixed"]
    fac, T, limit, _ = G.CASES[name]
    codec = sstcodec.Codec(0)
    args = [EXE, str(tmp_path / "db"), str(T), str(limit)]
    (tmp_path / "db").mkdir()
    for i, rec in enumerate(fac()):
        p = str(tmp_path / f"in{i}.sst")
        fs, _ = build_table(codec, p, rec, T)
        assert fs == case["inputs"][i]["file_size"] and sha(np.fromfile(p, np.uint8)) == case["inputs"][i]["sha256"]
        lo, hi = table_key_range(rec)
        args += [p, str(fs), lo.hex(), hi.hex()]
    codec.close()
    r = subprocess.run(args, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    picked, outs = G.parse_pick_output(r.stdout)
    assert picked == list(range(1, len(case["inputs"]) + 1))
    got = [(sha(np.fromfile(p, np.uint8)), fs) for p, fs, _, _ in outs]
    assert got == [(o["sha256"], o["file_size"]) for o in case["fixed_outputs"]]
    # and VersionEdit::AddNewFiles got the reference's key ranges
    assert [(lo.hex(), hi.hex()) for _, _, lo, hi in outs] == \
        [(o["smallest"], o["largest"]) for o in case["no_trim"]["outputs"]]
    print(f"{name}: db/compact.cc unchanged + sstc::TableBuilder -> {len(outs)} outputs equal to the reference's",
          flush=True)
