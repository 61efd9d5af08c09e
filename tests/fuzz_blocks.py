"""Corrupted-block generator shared by tests/test_gpu_fuzz.py and
tests/test_oracle.py: valid blocks from the oracle's encoder, then per block
one of nine seeded mutations (none, entry count, offset-section start, one
entry start, a type byte, a key length, a value length, random bytes, a
truncated slot)."""
import numpy as np
from sstcodec import workload as W


def fuzz_blocks(oracle, seed, nrec=6000, T=4096):
    """(src, blk_off, blk_len, mutation kind per block)."""
    rng = np.random.default_rng(seed)
    rec = W.mixed_records(nrec, seed=100 + seed, max_val=700 if T <= 4096 else 4000)
    first = oracle.segment(rec, T)
    src, offs, lens = oracle.encode_blocks(rec, first)
    src = src.copy(); lens = lens.copy()
    kinds = []
    for b in range(len(offs)):
        o, L = int(offs[b]), int(lens[b])
        k = int(rng.integers(0, 9))
        kinds.append(k)
        if k == 0:
            continue
        n = int(src[o + L - 16:o + L - 8].view(np.uint64)[0]); d = int(src[o + L - 8:o + L].view(np.uint64)[0])
        if k == 1:    # entry count
            v = rng.choice([0, n + 1, n - 1, 1 << 40, int(rng.integers(0, 2 * n + 2))])
            src[o + L - 16:o + L - 8] = np.array([v], np.uint64).view(np.uint8)
        elif k == 2:  # offset-section start
            v = rng.choice([d + 1, d - 1, L, 0, int(rng.integers(0, L + 64))])
            src[o + L - 8:o + L] = np.array([v], np.uint64).view(np.uint8)
        elif k == 3 and n:  # one entry start
            i = int(rng.integers(0, n))
            v = rng.choice([int(rng.integers(0, L)), L + 3, 0])
            src[o + d + 16 * i:o + d + 16 * i + 8] = np.array([v], np.uint64).view(np.uint8)
        elif k == 4 and n:  # an entry's type byte
            i = int(rng.integers(0, n)); s = int(src[o + d + 16 * i:o + d + 16 * i + 8].view(np.uint64)[0])
            src[o + s] = rng.choice([2, 7, 255])
        elif k == 5 and n:  # an entry's key length
            i = int(rng.integers(0, n)); s = int(src[o + d + 16 * i:o + d + 16 * i + 8].view(np.uint64)[0])
            src[o + s + 1:o + s + 5] = np.array([rng.choice([4097, L, 0xFFFFFFFF, int(rng.integers(0, 64))])], np.uint32).view(np.uint8)
        elif k == 6 and n:  # an entry's value length
            i = int(rng.integers(0, n)); s = int(src[o + d + 16 * i:o + d + 16 * i + 8].view(np.uint64)[0])
            kl = int(src[o + s + 1:o + s + 5].view(np.uint32)[0])
            if src[o + s] == 0:
                src[o + s + 5 + kl:o + s + 9 + kl] = np.array([rng.choice([L, 0xFFFFFFFF, 0, int(rng.integers(0, 900))])], np.uint32).view(np.uint8)
        elif k == 7:  # random bytes anywhere
            for _ in range(int(rng.integers(1, 4))):
                src[o + int(rng.integers(0, L))] = int(rng.integers(0, 256))
        elif k == 8:  # truncated slot
            lens[b] = max(0, L - int(rng.integers(1, 40)))
    return src, offs, lens, np.array(kinds)
