"""Deterministic synthetic record sets for the SST block codec (numpy only).

The shapes follow SURVEY.md §8(d): 16 B keys "k%015d", 100 B values drawn from
a splitmix64 stream, ascending txn ids.  A record set is a dict of numpy arrays
in the layout of include/sstcodec.h's sstc_records plus the key/value arenas:

    type u8, key_len u32, val_len u32 (NO_VALUE = no value fields), txn u64,
    key_off u64 (into key_src), val_off u64 (into val_src), key_src u8, val_src u8
"""
import numpy as np

NO_VALUE = 0xFFFFFFFF
TYPE_PUT = 0
TYPE_DELETED = 1

_GAMMA = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(seed, n, start=0):
    """n outputs of splitmix64 seeded with `seed`, from counter `start`."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (np.arange(start + 1, start + n + 1, dtype=np.uint64) * _GAMMA)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def random_bytes(seed, nbytes, start_word=0):
    words = splitmix64(seed, (nbytes + 7) // 8, start_word)
    return words.view(np.uint8)[:nbytes].copy()


def fixed_keys(index, width=16):
    """Keys "k%0{width-1}d" % index as one contiguous arena (width bytes each)."""
    index = np.asarray(index, dtype=np.uint64)
    nd = width - 1
    pw = np.uint64(10) ** np.arange(nd - 1, -1, -1, dtype=np.uint64)
    digits = (index[:, None] // pw[None, :]) % np.uint64(10)
    out = np.empty((index.size, width), dtype=np.uint8)
    out[:, 0] = ord("k")
    out[:, 1:] = (digits + np.uint64(ord("0"))).astype(np.uint8)
    return out.reshape(-1)


def uniform_records(n, key_index=None, seed=1, value_len=100, txn_start=1, key_width=16):
    """n PUT records, key_width-byte keys, value_len-byte random values."""
    if key_index is None:
        key_index = np.arange(n, dtype=np.uint64)
    key_src = fixed_keys(key_index, key_width)
    val_src = random_bytes(seed, n * value_len)
    return {
        "type": np.zeros(n, np.uint8),
        "key_len": np.full(n, key_width, np.uint32),
        "val_len": np.full(n, value_len, np.uint32),
        "txn": np.arange(txn_start, txn_start + n, dtype=np.uint64),
        "key_off": np.arange(n, dtype=np.uint64) * np.uint64(key_width),
        "val_off": np.arange(n, dtype=np.uint64) * np.uint64(value_len),
        "key_src": key_src,
        "val_src": val_src,
    }


def mixed_records(n, seed=7, max_key=48, max_val=300, p_delete=0.1, p_empty_val=0.05,
                  p_empty_key=0.02, sorted_keys=True):
    """Records with ragged keys/values, DELETEs, empty keys and empty values
    (the empty-value PUT exercises the reference's txn quirk)."""
    rng = np.random.default_rng(seed)
    klen = rng.integers(1, max_key + 1, n).astype(np.uint32)
    klen[rng.random(n) < p_empty_key] = 0
    vlen = rng.integers(1, max_val + 1, n).astype(np.uint32)
    vlen[rng.random(n) < p_empty_val] = 0
    typ = (rng.random(n) < p_delete).astype(np.uint8)
    vlen[typ == TYPE_DELETED] = NO_VALUE
    key_off = np.zeros(n, np.uint64)
    key_off[1:] = np.cumsum(klen[:-1].astype(np.uint64))
    key_src = rng.integers(0x20, 0x7F, int(klen.sum(dtype=np.uint64)) + 8, dtype=np.uint8)
    vbytes = np.where(vlen == NO_VALUE, 0, vlen).astype(np.uint64)
    val_off = np.zeros(n, np.uint64)
    val_off[1:] = np.cumsum(vbytes[:-1])
    val_src = rng.integers(0, 256, int(vbytes.sum()) + 8, dtype=np.uint8)
    val_off[typ == TYPE_DELETED] = 0
    txn = rng.integers(1, 1 << 62, n, dtype=np.uint64)
    return {
        "type": typ,
        "key_len": klen,
        "val_len": vlen,
        "txn": txn,
        "key_off": key_off,
        "val_off": val_off,
        "key_src": key_src,
        "val_src": val_src,
    }


def entry_sizes(rec):
    """Per-record entry size (reference sstable/block_builder.cc:19-21)."""
    vl = rec["val_len"].astype(np.uint64)
    has = rec["val_len"] != NO_VALUE
    return np.uint64(13) + rec["key_len"].astype(np.uint64) + np.where(has, np.uint64(4) + vl, np.uint64(0))


def segment(rec, threshold):
    """Greedy block boundaries of TableBuilder::AddEntry (table_builder.cc:57-59),
    host-side: the block closes right after the record whose cumulative
    (entry_size + 16) reaches `threshold`.  Returns the nblocks+1 boundaries."""
    w = entry_sizes(rec) + np.uint64(16)
    firsts = [0]
    acc = 0
    wl = w.tolist()
    for i, x in enumerate(wl):
        acc += x
        if acc >= threshold:
            firsts.append(i + 1)
            acc = 0
    if firsts[-1] != len(wl):
        firsts.append(len(wl))
    return np.asarray(firsts, dtype=np.uint64)


def uniform_block_layout(nblocks, per_block=28, key_len=16, val_len=100):
    """Offsets/lengths of nblocks back-to-back uniform blocks."""
    blen = per_block * (13 + key_len + 4 + val_len + 16) + 16
    off = np.arange(nblocks, dtype=np.uint64) * np.uint64(blen)
    return off, np.full(nblocks, blen, np.uint64)


CONFIG_DEFAULTS = {3: (8, 1_000_000), 4: (128, 100_000), 5: (8, 5000)}


def config_inputs(config, rank=0, ssts=None, keys=None, overlap=False, ranges=False, key_space=20000):
    """Input record sets (one per input SST, iterator order) of BASELINE.json
    configs 3-5, exactly as tests/golden/make_golden_configs.py fed them to the
    reference:

    config 3  `ssts` x `keys` uniform records; SST s holds k%015d of i*ssts+s
              (disjoint interleave), 100 B values (splitmix64 seed s+1), txns
              ascending and unique; overlap=True: the same key set i in every
              SST with distinct txns (the drop path); ranges=True: SST s holds
              one contiguous key range.
    config 4  rank r's shard of 1024 SSTs: keys [r*K, (r+1)*K), K = ssts*keys,
              SST s holds base + i*ssts + s; seeds / txns by global SST id.
    config 5  W.compaction_inputs: keys from a shared space of `key_space`,
              Zipf(1.1) values clamped to [8 B, 64 KiB], 10 % DELETE (seed 55+rank).
    """
    d_ssts, d_keys = CONFIG_DEFAULTS[config]
    ssts = ssts or d_ssts
    keys = keys or d_keys
    if config == 3:
        out = []
        for s in range(ssts):
            i = np.arange(keys, dtype=np.uint64)
            if overlap:
                k = i
            elif ranges:
                k = i + np.uint64(s * keys)
            else:
                k = i * np.uint64(ssts) + np.uint64(s)
            out.append(uniform_records(keys, key_index=k, seed=s + 1, txn_start=1 + s * keys))
        return out
    if config == 4:
        K = ssts * keys
        base = np.uint64(rank * K)
        out = []
        for s in range(ssts):
            i = np.arange(keys, dtype=np.uint64)
            g = rank * ssts + s
            out.append(uniform_records(keys, key_index=base + i * np.uint64(ssts) + np.uint64(s), seed=g + 1,
                                       txn_start=1 + g * keys))
        return out
    if config == 5:
        return compaction_inputs(ssts, keys, key_space, seed=55 + rank, vmin=8, vmax=65536, zipf=1.1, p_delete=0.1)
    raise ValueError(f"no input generator for config {config}")


def compaction_inputs(k, n_per, key_space, seed=5, p_delete=0.1, vmin=8, vmax=200, key_width=16,
                      distinct=True, zipf=None):
    """k record sets (one per input SST, iterator order), each sorted by key,
    keys drawn from a shared space of `key_space` keys (overlap across tables),
    txn ids unique across all tables (the engine's sequence numbers).  zipf:
    optional exponent for Zipf value sizes clamped to [vmin, vmax]."""
    rng = np.random.default_rng(seed)
    total = k * n_per
    txns = rng.permutation(np.arange(1, total + 1, dtype=np.uint64)) * np.uint64(7) + np.uint64(3)
    out = []
    pos = 0
    for t in range(k):
        if distinct:
            idx = np.sort(rng.choice(key_space, size=min(n_per, key_space), replace=False)).astype(np.uint64)
        else:
            idx = np.sort(rng.integers(0, key_space, n_per)).astype(np.uint64)
        n = idx.size
        key_src = fixed_keys(idx, key_width)
        if zipf:
            v = rng.zipf(zipf, n).astype(np.float64)
            vlen = np.clip(v * vmin, vmin, vmax).astype(np.uint32)
        else:
            vlen = rng.integers(vmin, vmax + 1, n).astype(np.uint32)
        typ = (rng.random(n) < p_delete).astype(np.uint8)
        vlen[typ == TYPE_DELETED] = NO_VALUE
        vb = np.where(vlen == NO_VALUE, 0, vlen).astype(np.uint64)
        val_off = np.zeros(n, np.uint64)
        val_off[1:] = np.cumsum(vb[:-1])
        val_src = random_bytes(seed * 1000 + t, int(vb.sum()) + 8)
        tx = txns[pos:pos + n].copy()
        pos += n
        if not distinct:  # duplicates inside one table: newest first (skiplist order)
            order = np.lexsort((-tx.astype(np.float64), idx))
            tx = tx[order]
        out.append({"type": typ, "key_len": np.full(n, key_width, np.uint32), "val_len": vlen, "txn": tx,
                    "key_off": np.arange(n, dtype=np.uint64) * np.uint64(key_width),
                    "val_off": np.where(typ == TYPE_DELETED, 0, val_off).astype(np.uint64),
                    "key_src": key_src, "val_src": val_src})
    return out


def cross_duplicate_inputs(k, n_per, key_space, seed=5, p_shared=0.5, p_delete=0.2, same_content=True,
                           vmax=40, key_width=16):
    """k sorted record sets in which the same (key, txn) appears in several
    tables -- the case where the merge order among equal (key, txn) records
    decides the output bytes (ShouldKeepEntry keeps them all,
    compact.cc:357-362).  Every key has one shared version (txn, type, value);
    a table that holds the key takes the shared version with probability
    p_shared, else a table-unique txn.  same_content=False: the shared txn
    comes with the table's own type / value (not reachable through the
    engine, whose txn ids are unique per write)."""
    rng = np.random.default_rng(seed)
    shared_txn = (rng.permutation(key_space).astype(np.uint64) + np.uint64(1)) * np.uint64(1000)
    shared_typ = (rng.random(key_space) < p_delete).astype(np.uint8)
    shared_vl = rng.integers(0, vmax + 1, key_space).astype(np.uint32)
    shared_seed = rng.integers(0, 1 << 30, key_space)
    out = []
    for t in range(k):
        idx = np.sort(rng.choice(key_space, size=min(n_per, key_space), replace=False))
        n = idx.size
        share = rng.random(n) < p_shared
        typ = np.where(share & same_content, shared_typ[idx], (rng.random(n) < p_delete).astype(np.uint8))
        vl = np.where(share & same_content, shared_vl[idx], rng.integers(0, vmax + 1, n)).astype(np.uint32)
        txn = np.where(share, shared_txn[idx], shared_txn[idx] + np.uint64(1 + t)).astype(np.uint64)
        vals = []
        for j in range(n):
            if typ[j] == TYPE_DELETED:
                continue
            s = int(shared_seed[idx[j]]) if (share[j] and same_content) else int(rng.integers(0, 1 << 30))
            vals.append(random_bytes(s, int(vl[j])))
        vl = np.where(typ == TYPE_DELETED, np.uint32(NO_VALUE), vl).astype(np.uint32)
        vb = np.where(vl == NO_VALUE, 0, vl).astype(np.uint64)
        val_off = np.zeros(n, np.uint64)
        val_off[1:] = np.cumsum(vb[:-1])
        val_src = np.concatenate(vals + [np.zeros(8, np.uint8)])
        out.append({"type": typ.astype(np.uint8), "key_len": np.full(n, key_width, np.uint32), "val_len": vl,
                    "txn": txn, "key_off": np.arange(n, dtype=np.uint64) * np.uint64(key_width),
                    "val_off": np.where(typ == TYPE_DELETED, 0, val_off).astype(np.uint64),
                    "key_src": fixed_keys(idx.astype(np.uint64), key_width), "val_src": val_src})
    return out


def config3_lookup_queries(n, seed=7, ssts=8, keys=1_000_000):
    """Point-lookup queries over the config-3 SSTs (SST s holds k%015d of
    i*ssts+s): (table per query, key index per query).  Half are present in
    their table, a quarter belong to another table (absent here), the rest
    lie past the last key or between keys' ranges of other sizes."""
    rng = np.random.default_rng(seed)
    t = rng.integers(0, ssts, n).astype(np.uint32)
    kind = rng.random(n)
    i = rng.integers(0, keys, n).astype(np.uint64)
    own = i * np.uint64(ssts) + t.astype(np.uint64)
    other = i * np.uint64(ssts) + ((t.astype(np.uint64) + np.uint64(1)) % np.uint64(ssts))
    past = np.uint64(ssts * keys) + rng.integers(0, 1000, n).astype(np.uint64)
    k = np.where(kind < 0.5, own, np.where(kind < 0.75, other, past))
    return t, k
