/*
 * sst_oracle.c — CPU restatement of the reference SST block codec.
 * TEST INFRASTRUCTURE ONLY (see sst_oracle.h).  Plain scalar C on purpose: it
 * is the checker, never the product.
 */
#include "sst_oracle.h"

#include <stdlib.h>
#include <string.h>

static uint32_t rd32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
static uint64_t rd64(const uint8_t *p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}
static void wr32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static void wr64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }

/* sstable/block_builder.cc:19-21 */
uint32_t orc_entry_size(uint32_t key_len, uint32_t val_len) {
  return 1u + 4u + key_len + (val_len != ORC_NO_VALUE ? 4u + val_len : 0u) + 8u;
}

/* sstable/block_builder.cc:12-109: data entries, then one 16 B offset entry
 * (start, size) per record, then extra = (num_entries, data bytes). */
uint64_t orc_block_encode(uint64_t n, const uint8_t *type, const uint32_t *key_len,
                          const uint32_t *val_len, const uint64_t *txn,
                          const uint8_t *key_src, const uint64_t *key_off,
                          const uint8_t *val_src, const uint64_t *val_off,
                          uint8_t *out) {
  uint64_t pos = 0;
  for (uint64_t i = 0; i < n; i++) { /* EncodeDataEntry :36-77 */
    out[pos] = type[i];
    wr32(out + pos + 1, key_len[i]);
    memcpy(out + pos + 5, key_src + key_off[i], key_len[i]);
    pos += 5 + (uint64_t)key_len[i];
    if (val_len[i] != ORC_NO_VALUE) {
      wr32(out + pos, val_len[i]);
      if (val_len[i]) memcpy(out + pos + 4, val_src + val_off[i], val_len[i]);
      pos += 4 + (uint64_t)val_len[i];
    }
    wr64(out + pos, txn[i]);
    pos += 8;
  }
  const uint64_t data_bytes = pos;
  uint64_t start = 0;
  for (uint64_t i = 0; i < n; i++) { /* EncodeOffsetEntry :79-93 */
    const uint64_t sz = orc_entry_size(key_len[i], val_len[i]);
    wr64(out + pos, start);
    wr64(out + pos + 8, sz);
    pos += 16;
    start += sz;
  }
  wr64(out + pos, n); /* EncodeExtraInfo :95-109 */
  wr64(out + pos + 8, data_bytes);
  return pos + 16;
}

int orc_block_count(const uint8_t *blk, uint64_t len, uint64_t *n_out) {
  *n_out = 0;
  if (len < 16) return ORC_BLK_TOO_SMALL;
  *n_out = rd64(blk + len - 16);
  return ORC_BLK_OK;
}

int orc_block_decode(const uint8_t *blk, uint64_t len, uint64_t base, int txn_mode,
                     uint8_t *type, uint32_t *key_len, uint32_t *val_len,
                     uint64_t *txn, uint64_t *key_off, uint64_t *val_off,
                     uint64_t *n_out) {
  *n_out = 0;
  if (len < 16) return ORC_BLK_TOO_SMALL;
  /* table_reader.cc:226-232: n at [size-16], offset section start at [size-8] */
  const uint64_t n = rd64(blk + len - 16);
  const uint64_t off = rd64(blk + len - 8);
  if (n == 0) return ORC_BLK_EMPTY;
  if (off > len - 16 || n > (len - 16 - off) / 16) return ORC_BLK_OFFSETS_RANGE;
  *n_out = n;
  for (uint64_t i = 0; i < n; i++) {
    /* table_reader.cc:11-20: only the start half of an offset entry is read */
    const uint64_t s = rd64(blk + off + 16 * i);
    if (s >= off || off - s < 5) return ORC_BLK_ENTRY_RANGE;
    const uint8_t t = blk[s];                      /* block_reader.cc:59-68 */
    if (t > ORC_TYPE_DELETED) return ORC_BLK_BAD_TYPE;
    const uint32_t kl = rd32(blk + s + 1);         /* block_reader.cc:70-82 */
    if (kl > ORC_MAX_KEY) return ORC_BLK_KEY_TOO_LONG;
    uint64_t p = s + 5 + kl;
    uint32_t vl = ORC_NO_VALUE;
    uint64_t vo = 0;
    if (t != ORC_TYPE_DELETED) {                   /* block_reader.cc:84-102 */
      if (p + 4 > off) return ORC_BLK_ENTRY_RANGE;
      vl = rd32(blk + p);
      vo = p + 4;
      p = vo + vl;
    }
    if (p + 8 > off) return ORC_BLK_ENTRY_RANGE;
    uint64_t tx = rd64(blk + p);                   /* block_reader.cc:104-114 */
    if (txn_mode == ORC_TXN_COMPAT && t != ORC_TYPE_DELETED && vl == 0) {
      /* value.empty() is true, so the reference reads 8 bytes at the value
       * length field: (txn & 0xffffffff) << 32 */
      tx = rd64(blk + s + 5 + kl);
    }
    type[i] = t;
    key_len[i] = kl;
    key_off[i] = base + s + 5;
    val_len[i] = vl;
    val_off[i] = t != ORC_TYPE_DELETED ? base + vo : 0;
    txn[i] = tx;
  }
  return ORC_BLK_OK;
}

/* Bounded scratch for the per-block records of the roundtrip. A block holds at
 * most (len-16)/29 entries (13 B minimal entry + 16 B offset entry). */
#define ORC_RT_MAX 65536
uint64_t orc_roundtrip_blocks(const uint8_t *src, const uint64_t *blk_off,
                              const uint64_t *blk_len, uint64_t nblocks,
                              int txn_mode, uint8_t *dst, uint64_t *out_len,
                              uint32_t *status) {
  static uint8_t type[ORC_RT_MAX];
  static uint32_t kl[ORC_RT_MAX], vl[ORC_RT_MAX];
  static uint64_t tx[ORC_RT_MAX], ko[ORC_RT_MAX], vo[ORC_RT_MAX];
  uint64_t bad = 0;
  for (uint64_t b = 0; b < nblocks; b++) {
    const uint8_t *blk = src + blk_off[b];
    uint64_t n = 0;
    int st = ORC_BLK_OK;
    if (blk_len[b] >= 16 && blk_len[b] / 29 + 1 > ORC_RT_MAX) {
      st = ORC_BLK_OFFSETS_RANGE;
    } else {
      st = orc_block_decode(blk, blk_len[b], 0, txn_mode, type, kl, vl, tx, ko, vo, &n);
    }
    if (st == ORC_BLK_OK) {
      uint64_t sz = 16 + 16 * n;
      for (uint64_t i = 0; i < n; i++) sz += orc_entry_size(kl[i], vl[i]);
      if (sz >= (1ull << 32)) st = ORC_BLK_TOO_LARGE;
      else if (sz > blk_len[b]) st = ORC_BLK_NO_ROOM; /* re-encoded in place of the input */
    }
    status[b] = (uint32_t)st;
    if (st != ORC_BLK_OK) {
      out_len[b] = 0;
      bad++;
      continue;
    }
    out_len[b] = orc_block_encode(n, type, kl, vl, tx, blk, ko, blk, vo, dst + blk_off[b]);
  }
  return bad;
}

uint64_t orc_segment(uint64_t n, const uint32_t *key_len, const uint32_t *val_len,
                     uint64_t threshold, uint64_t *blk_first) {
  uint64_t nb = 0, acc = 0;
  for (uint64_t i = 0; i < n; i++) {
    if (acc == 0) blk_first[nb++] = i;
    acc += orc_entry_size(key_len[i], val_len[i]) + 16; /* block_builder.cc:33 */
    if (acc >= threshold) acc = 0;                       /* table_builder.cc:57 */
  }
  blk_first[nb] = n;
  return nb;
}

static uint64_t meta_entry(uint8_t *out, const uint8_t *fk, uint32_t fkl,
                           const uint8_t *lk, uint32_t lkl, uint64_t off,
                           uint64_t len) {
  /* TableBuilder::AddIndexBlockEntry, sstable/table_builder.cc:101-145 */
  if (out) {
    wr32(out, fkl);
    memcpy(out + 4, fk, fkl);
    wr32(out + 4 + fkl, lkl);
    memcpy(out + 8 + fkl, lk, lkl);
    wr64(out + 8 + fkl + lkl, off);
    wr64(out + 16 + fkl + lkl, len);
  }
  return 24 + (uint64_t)fkl + lkl;
}

uint64_t orc_table_build(uint64_t n, const uint8_t *type, const uint32_t *key_len,
                         const uint32_t *val_len, const uint64_t *txn,
                         const uint8_t *key_src, const uint64_t *key_off,
                         const uint8_t *val_src, const uint64_t *val_off,
                         uint64_t threshold, uint8_t *out) {
  /* pass 1: data blocks (segmentation of AddEntry, FlushBlock :62-99) */
  uint64_t pos = 0, nb = 0, start = 0, acc = 0;
  uint64_t min_txn = UINT64_MAX, max_txn = 0;
  for (uint64_t i = 0; i < n; i++) {
    if (txn[i] < min_txn) min_txn = txn[i];
    if (txn[i] > max_txn) max_txn = txn[i];
    acc += orc_entry_size(key_len[i], val_len[i]) + 16;
    if (acc >= threshold || i + 1 == n) {
      const uint64_t m = i + 1 - start;
      uint64_t sz = 16;
      for (uint64_t j = start; j <= i; j++) sz += orc_entry_size(key_len[j], val_len[j]) + 16;
      if (out)
        orc_block_encode(m, type + start, key_len + start, val_len + start, txn + start,
                         key_src, key_off + start, val_src, val_off + start, out + pos);
      pos += sz;
      nb++;
      start = i + 1;
      acc = 0;
    }
  }
  /* pass 2: meta section (one entry per block, in block order) */
  const uint64_t meta_off = pos;
  start = 0;
  acc = 0;
  uint64_t boff = 0;
  for (uint64_t i = 0; i < n; i++) {
    acc += orc_entry_size(key_len[i], val_len[i]) + 16;
    if (acc >= threshold || i + 1 == n) {
      uint64_t sz = 16;
      for (uint64_t j = start; j <= i; j++) sz += orc_entry_size(key_len[j], val_len[j]) + 16;
      pos += meta_entry(out ? out + pos : NULL, key_src + key_off[start], key_len[start],
                        key_src + key_off[i], key_len[i], boff, sz);
      boff += sz;
      start = i + 1;
      acc = 0;
    }
  }
  const uint64_t meta_len = pos - meta_off;
  /* footer, TableBuilder::EncodeExtraInfo :179-211 */
  if (out) {
    wr64(out + pos, nb);
    wr64(out + pos + 8, meta_off);
    wr64(out + pos + 16, meta_len);
    wr64(out + pos + 24, min_txn);
    wr64(out + pos + 32, max_txn);
  }
  return pos + 40;
}

uint64_t orc_table_index(const uint8_t *file, uint64_t bytes, uint64_t cap,
                         uint64_t *blk_off, uint64_t *blk_len,
                         uint64_t *first_key_off, uint32_t *first_key_len,
                         uint64_t *last_key_off, uint32_t *last_key_len,
                         uint64_t *min_txn, uint64_t *max_txn) {
  if (bytes < 40) return UINT64_MAX;
  /* DecodeExtraInfo, sstable/table_reader.cc:52-84 (file_size - 40 - 1 with
   * file_size = bytes + 1) */
  const uint8_t *f = file + bytes - 40;
  const uint64_t nb = rd64(f), moff = rd64(f + 8), mlen = rd64(f + 16);
  *min_txn = rd64(f + 24);
  *max_txn = rd64(f + 32);
  if (moff > bytes - 40 || mlen > bytes - 40 - moff) return UINT64_MAX;
  /* FetchBlockIndexInfo :86-156, sequential length-prefixed walk */
  uint64_t p = moff;
  const uint64_t end = moff + mlen;
  for (uint64_t i = 0; i < nb; i++) {
    if (p + 4 > end) return UINT64_MAX;
    const uint32_t fkl = rd32(file + p);
    if (p + 4 + (uint64_t)fkl + 4 > end) return UINT64_MAX;
    const uint32_t lkl = rd32(file + p + 4 + fkl);
    if (p + 24 + (uint64_t)fkl + lkl > end) return UINT64_MAX;
    if (i < cap) {
      first_key_off[i] = p + 4;
      first_key_len[i] = fkl;
      last_key_off[i] = p + 8 + fkl;
      last_key_len[i] = lkl;
      blk_off[i] = rd64(file + p + 8 + fkl + lkl);
      blk_len[i] = rd64(file + p + 16 + fkl + lkl);
    }
    p += 24 + (uint64_t)fkl + lkl;
  }
  return nb;
}

/* ------------------------------------------------------------------------ */
/* Compaction (db/compact.cc:232-363), records reached through the reference  */
/* reader (COMPAT txn), merged in MergeIterator order (db/merge_iterator.h:   */
/* 91-95: key ascending, txn descending; equal (key, txn) -> lower input       */
/* table first, which the reference's std::priority_queue leaves unspecified). */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint64_t n;
  uint8_t *type;
  uint32_t *kl, *vl;
  uint64_t *tx, *ko, *vo; /* offsets into the table's file image */
  const uint8_t *file;
} orc_run;

static int key_cmp(const uint8_t *a, uint32_t al, const uint8_t *b, uint32_t bl) {
  const uint32_t m = al < bl ? al : bl;
  const int c = m ? memcmp(a, b, m) : 0;
  if (c) return c < 0 ? -1 : 1;
  return al < bl ? -1 : (al > bl ? 1 : 0);
}

static void run_free(orc_run *r) {
  free(r->type); free(r->kl); free(r->vl); free(r->tx); free(r->ko); free(r->vo);
}

static int run_load(orc_run *r, const uint8_t *file, uint64_t bytes) {
  memset(r, 0, sizeof(*r));
  r->file = file;
  uint64_t mn, mx;
  const uint64_t nb = orc_table_index(file, bytes, 0, NULL, NULL, NULL, NULL, NULL, NULL, &mn, &mx);
  if (nb == UINT64_MAX) return -1;
  uint64_t *bo = malloc((nb + 1) * 8), *bl = malloc((nb + 1) * 8), *fo = malloc((nb + 1) * 8), *lo = malloc((nb + 1) * 8);
  uint32_t *fl = malloc((nb + 1) * 4), *ll = malloc((nb + 1) * 4);
  orc_table_index(file, bytes, nb, bo, bl, fo, fl, lo, ll, &mn, &mx);
  uint64_t cap = 0;
  for (uint64_t b = 0; b < nb; b++) cap += bl[b] / 29 + 1;
  r->type = malloc(cap + 1); r->kl = malloc(4 * cap + 4); r->vl = malloc(4 * cap + 4);
  r->tx = malloc(8 * cap + 8); r->ko = malloc(8 * cap + 8); r->vo = malloc(8 * cap + 8);
  int rc = 0;
  for (uint64_t b = 0; b < nb && !rc; b++) {
    uint64_t n = 0;
    if (bo[b] > bytes || bl[b] > bytes - bo[b]) { rc = -1; break; }
    if (orc_block_decode(file + bo[b], bl[b], bo[b], ORC_TXN_COMPAT, r->type + r->n, r->kl + r->n, r->vl + r->n,
                         r->tx + r->n, r->ko + r->n, r->vo + r->n, &n) != ORC_BLK_OK) rc = -1;
    r->n += n;
  }
  free(bo); free(bl); free(fo); free(lo); free(fl); free(ll);
  return rc;
}

/* one output table under construction */
typedef struct {
  uint64_t n, cap;
  uint8_t *type;
  uint32_t *kl, *vl;
  uint64_t *tx;
  const uint8_t **kp, **vp;
} orc_pending;

static void pend_push(orc_pending *p, uint8_t t, uint32_t kl, uint32_t vl, uint64_t tx, const uint8_t *kp,
                      const uint8_t *vp) {
  if (p->n == p->cap) {
    p->cap = p->cap ? 2 * p->cap : 1024;
    p->type = realloc(p->type, p->cap); p->kl = realloc(p->kl, 4 * p->cap); p->vl = realloc(p->vl, 4 * p->cap);
    p->tx = realloc(p->tx, 8 * p->cap); p->kp = realloc(p->kp, sizeof(void *) * p->cap);
    p->vp = realloc(p->vp, sizeof(void *) * p->cap);
  }
  p->type[p->n] = t; p->kl[p->n] = kl; p->vl[p->n] = vl; p->tx[p->n] = tx; p->kp[p->n] = kp; p->vp[p->n] = vp;
  p->n++;
}

/* TableBuilder AddEntry... Finish over pointer-addressed records */
static uint64_t pend_build(const orc_pending *p, uint64_t threshold, uint8_t *out) {
  uint64_t pos = 0, nb = 0, start = 0, acc = 0, mn = UINT64_MAX, mx = 0;
  uint64_t *bstart = malloc(8 * (p->n + 1)), *bend = malloc(8 * (p->n + 1)), *blen = malloc(8 * (p->n + 1));
  for (uint64_t i = 0; i < p->n; i++) {
    if (p->tx[i] < mn) mn = p->tx[i];
    if (p->tx[i] > mx) mx = p->tx[i];
    acc += orc_entry_size(p->kl[i], p->vl[i]) + 16;
    if (acc >= threshold || i + 1 == p->n) {
      uint64_t q = pos;
      for (uint64_t j = start; j <= i; j++) {
        out[q] = p->type[j]; wr32(out + q + 1, p->kl[j]); memcpy(out + q + 5, p->kp[j], p->kl[j]);
        q += 5 + (uint64_t)p->kl[j];
        if (p->vl[j] != ORC_NO_VALUE) {
          wr32(out + q, p->vl[j]);
          if (p->vl[j]) memcpy(out + q + 4, p->vp[j], p->vl[j]);
          q += 4 + (uint64_t)p->vl[j];
        }
        wr64(out + q, p->tx[j]); q += 8;
      }
      const uint64_t data = q - pos;
      uint64_t st = 0;
      for (uint64_t j = start; j <= i; j++) {
        const uint64_t sz = orc_entry_size(p->kl[j], p->vl[j]);
        wr64(out + q, st); wr64(out + q + 8, sz); q += 16; st += sz;
      }
      wr64(out + q, i + 1 - start); wr64(out + q + 8, data); q += 16;
      bstart[nb] = start; bend[nb] = i; blen[nb] = q - pos;
      nb++; pos = q; start = i + 1; acc = 0;
    }
  }
  const uint64_t moff = pos;
  uint64_t boff = 0;
  for (uint64_t b = 0; b < nb; b++) {
    const uint64_t f = bstart[b], l = bend[b];
    pos += meta_entry(out + pos, p->kp[f], p->kl[f], p->kp[l], p->kl[l], boff, blen[b]);
    boff += blen[b];
  }
  wr64(out + pos, nb); wr64(out + pos + 8, moff); wr64(out + pos + 16, pos - moff);
  wr64(out + pos + 24, mn); wr64(out + pos + 32, mx);
  free(bstart); free(bend); free(blen);
  return pos + 40;
}

uint64_t orc_compact(uint32_t k, const uint8_t *const *files, const uint64_t *bytes, uint64_t block_threshold,
                     uint64_t table_limit, int base_level, uint8_t *out, uint64_t out_cap, uint64_t *out_size,
                     uint64_t max_tables, uint64_t *kept_records) {
  orc_run *runs = calloc(k ? k : 1, sizeof(orc_run));
  uint64_t *head = calloc(k ? k : 1, 8);
  uint64_t ntab = 0, pos = 0, kept = 0;
  int bad = 0;
  for (uint32_t t = 0; t < k; t++)
    if (run_load(&runs[t], files[t], bytes[t])) bad = 1;
  orc_pending cur = {0};
  uint64_t data_size = 0;
  const uint8_t *last_key = NULL;
  uint32_t last_kl = 0;
  uint64_t last_txn = UINT64_MAX; /* INVALID_TXN_ID */
  int first = 1;
  while (!bad) {
    int best = -1;
    for (uint32_t t = 0; t < k; t++) {
      if (head[t] >= runs[t].n) continue;
      if (best < 0) { best = (int)t; continue; }
      const orc_run *a = &runs[t], *b = &runs[best];
      const uint64_t i = head[t], j = head[best];
      const int c = key_cmp(a->file + a->ko[i], a->kl[i], b->file + b->ko[j], b->kl[j]);
      if (c < 0 || (c == 0 && a->tx[i] > b->tx[j])) best = (int)t;
    }
    if (best < 0) break;
    const orc_run *r = &runs[best];
    const uint64_t i = head[best]++;
    const uint8_t *key = r->file + r->ko[i];
    const uint32_t kl = r->kl[i];
    const uint64_t txn = r->tx[i];
    const uint8_t type = r->type[i];
    /* ShouldKeepEntry, db/compact.cc:324-363 */
    int keep;
    const int new_key = first || key_cmp(key, kl, last_key, last_kl) != 0;
    if (first) keep = 1;
    else if (new_key) keep = type == ORC_TYPE_PUT ? 1 : (base_level ? 0 : 1);
    else keep = !(last_txn > txn);
    if (new_key) { last_key = key; last_kl = kl; last_txn = txn; }
    first = 0;
    if (!keep) continue;
    kept++;
    pend_push(&cur, type, kl, r->vl[i], txn, key, r->vl[i] != ORC_NO_VALUE ? r->file + r->vo[i] : NULL);
    data_size += kl + (r->vl[i] != ORC_NO_VALUE ? r->vl[i] : 0); /* table_builder.cc:55 */
    if (data_size >= table_limit) {                               /* compact.cc:290 */
      uint64_t need = 40;
      for (uint64_t j = 0; j < cur.n; j++) need += orc_entry_size(cur.kl[j], cur.vl[j]) + 16 + 16 + 24 + 2 * cur.kl[j];
      if (pos + need > out_cap || ntab >= max_tables) { bad = 1; break; }
      out_size[ntab++] = pend_build(&cur, block_threshold, out + pos);
      pos += out_size[ntab - 1];
      cur.n = 0;
      data_size = 0;
    }
  }
  /* DoCompactJob opens its first output before the loop and finishes it even
   * when nothing was added (compact.cc:236-240, 304-310) */
  if (!bad && cur.n == 0 && ntab == 0) {
    if (out_cap < 40 || max_tables < 1) bad = 1;
    else {
      out_size[ntab++] = pend_build(&cur, block_threshold, out + pos);
      pos += out_size[ntab - 1];
    }
  }
  if (!bad && cur.n) {
    uint64_t need = 40;
    for (uint64_t j = 0; j < cur.n; j++) need += orc_entry_size(cur.kl[j], cur.vl[j]) + 16 + 16 + 24 + 2 * cur.kl[j];
    if (pos + need > out_cap || ntab >= max_tables) bad = 1;
    else {
      out_size[ntab++] = pend_build(&cur, block_threshold, out + pos);
      pos += out_size[ntab - 1];
    }
  }
  free(cur.type); free(cur.kl); free(cur.vl); free(cur.tx); free(cur.kp); free(cur.vp);
  for (uint32_t t = 0; t < k; t++) run_free(&runs[t]);
  free(runs); free(head);
  if (kept_records) *kept_records = kept;
  return bad ? UINT64_MAX : ntab;
}

/* ------------------------------------------------------------------------ */
/* Point lookup (sstable/table_reader.cc:168-210, block_reader.cc:20-57)      */
/* ------------------------------------------------------------------------ */

/* std::string_view::compare: unsigned bytes, then length */
static int sv_cmp(const uint8_t *a, uint64_t la, const uint8_t *b, uint64_t lb) {
  const uint64_t m = la < lb ? la : lb;
  for (uint64_t i = 0; i < m; i++)
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return la < lb ? -1 : (la > lb ? 1 : 0);
}

int orc_table_get(const uint8_t *file, uint64_t bytes, uint64_t nq, const uint8_t *keys,
                  const uint64_t *key_off, const uint32_t *key_len, uint32_t *out_type,
                  uint64_t *out_val_off, uint32_t *out_val_len, uint64_t *out_block) {
  uint64_t mn, mx;
  const uint64_t nb = orc_table_index(file, bytes, 0, NULL, NULL, NULL, NULL, NULL, NULL, &mn, &mx);
  if (nb == UINT64_MAX) return -1;
  uint64_t *bo = (uint64_t *)malloc(sizeof(uint64_t) * (nb + 1)), *bl = (uint64_t *)malloc(sizeof(uint64_t) * (nb + 1));
  uint64_t *fo = (uint64_t *)malloc(sizeof(uint64_t) * (nb + 1)), *lo = (uint64_t *)malloc(sizeof(uint64_t) * (nb + 1));
  uint32_t *fl = (uint32_t *)malloc(sizeof(uint32_t) * (nb + 1)), *ll = (uint32_t *)malloc(sizeof(uint32_t) * (nb + 1));
  orc_table_index(file, bytes, nb, bo, bl, fo, fl, lo, ll, &mn, &mx);
  for (uint64_t q = 0; q < nq; q++) {
    const uint8_t *key = keys + key_off[q];
    const uint64_t kl = key_len[q];
    out_type[q] = ORC_GET_NOT_FOUND;
    out_val_off[q] = 0;
    out_val_len[q] = 0;
    out_block[q] = UINT64_MAX;
    if (nb == 0) continue; /* the reference indexes block_index_[-1] here */
    /* GetBlockOffsetAndSize :191-210 */
    int64_t left = 0, right = (int64_t)nb - 1;
    while (left < right) {
      const int64_t mid = left + (right - left) / 2;
      if (sv_cmp(file + lo[mid], ll[mid], key, kl) >= 0) right = mid;
      else left = mid + 1;
    }
    const uint64_t b = (uint64_t)right;
    out_block[q] = b;
    /* CreateAndSetupDataForBlockReader :212-241 (trailer + entry starts) */
    const uint64_t L = bl[b];
    if (bo[b] > bytes || L > bytes - bo[b] || L < 16) { out_type[q] = ORC_GET_BAD; continue; }
    const uint8_t *blk = file + bo[b];
    const uint64_t n = rd64(blk + L - 16), offs = rd64(blk + L - 8);
    if (offs > L - 16 || n > (L - 16 - offs) / 16) { out_type[q] = ORC_GET_BAD; continue; }
    /* BlockReader::GetValue :20-57 */
    int64_t l2 = 0, r2 = (int64_t)n - 1;
    while (l2 <= r2) {
      const int64_t mid = l2 + (r2 - l2) / 2;
      const uint64_t s = rd64(blk + offs + 16 * (uint64_t)mid);
      if (s > offs || offs - s < 5) { out_type[q] = ORC_GET_BAD; break; }
      const uint8_t t = blk[s];
      const uint32_t ekl = rd32(blk + s + 1);
      if ((uint64_t)ekl > offs - s - 5 || t > 1) { out_type[q] = ORC_GET_BAD; break; }
      const int c = sv_cmp(blk + s + 5, ekl, key, kl);
      if (c == 0) {
        if (t == 1) {
          out_type[q] = ORC_GET_DELETED;
        } else {
          if (offs - s - 5 - ekl < 4) { out_type[q] = ORC_GET_BAD; break; }
          const uint32_t vl = rd32(blk + s + 5 + ekl);
          if ((uint64_t)vl > offs - s - 9 - ekl) { out_type[q] = ORC_GET_BAD; break; }
          out_type[q] = ORC_GET_PUT;
          out_val_off[q] = bo[b] + s + 9 + ekl;
          out_val_len[q] = vl;
        }
        break;
      } else if (c < 0) {
        l2 = mid + 1;
      } else {
        r2 = mid - 1;
      }
    }
  }
  free(bo); free(bl); free(fo); free(lo); free(fl); free(ll);
  return 0;
}
