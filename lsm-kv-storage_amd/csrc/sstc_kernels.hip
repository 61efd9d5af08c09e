// sstc_kernels.hip — CDNA4 (gfx950) kernels of the SST block codec.
//
// Kernels (each cites the reference function whose byte work it replaces):
//   rt_kernel           fused decode -> re-encode, one wave per block; small
//                       blocks staged in LDS by LDS-DMA (global_load_lds_dwordx4),
//                       large ones parsed from HBM and streamed through the
//                       wave's LDS slot (replaces the per-block work of
//                       db/compact.cc:254-302 on surviving records).
//   count_scan_kernel   per-block entry counts from the 16 B extras
//                       (TableReader::CreateAndSetupDataForBlockReader,
//                       sstable/table_reader.cc:226-232) scanned into
//                       record bases, one kernel.
//   decode_kernel       per-entry parse into a record table
//                       (BlockReader accessors, sstable/block_reader.cc:59-114).
//   enc_*_kernel        records -> blocks (BlockBuilder, block_builder.cc:12-109).
//   seg_*_kernel        greedy block / table segmentation of TableBuilder::AddEntry
//                       (table_builder.cc:57-59) and DoCompactJob (compact.cc:290):
//                       per-tile chain walks + node-level pointer jumping, or
//                       a wave hopping along few long segments.
//   scan_*_kernel       device-wide exclusive scan (u64) used by the above.
#include "sstc_device.h"
#include "sstc_launch.h"

namespace sstc {

// ---------------------------------------------------------------------------
// Entry parse, shared by every decode path.  Mirrors the reference reader
// (block_reader.cc:59-114) plus the bounds checks the reference does not do
// (their failure codes are the SSTC_BLK_* values).  Offsets are block-relative.
// ---------------------------------------------------------------------------
struct Entry {
  uint32_t code;
  uint32_t type;
  uint32_t klen;
  uint32_t vlen; // kNoValue for DELETE
  uint64_t txn;  // as decoded (compat quirk applied when asked)
  uint64_t size; // recomputed entry size
};

struct LdsReader {
  const uint8_t *img; // image byte 0 == block byte 0
  __device__ uint32_t u8(uint64_t o) const { return lds_u8(img, static_cast<uint32_t>(o)); }
  __device__ uint32_t u32(uint64_t o) const { return lds_u32u(img, static_cast<uint32_t>(o)); }
  __device__ uint64_t u64(uint64_t o) const { return lds_u64u(img, static_cast<uint32_t>(o)); }
};

struct GlobalReader {
  const uint8_t *blk;
  __device__ uint32_t u8(uint64_t o) const { return g_u8(blk + o); }
  __device__ uint32_t u32(uint64_t o) const { return g_u32u(blk + o); }
  __device__ uint64_t u64(uint64_t o) const { return g_u64u(blk + o); }
};

template <class R>
__device__ __forceinline__ Entry parse_entry(const R &rd, uint64_t s, uint64_t doff,
                                             uint32_t txn_mode) {
  Entry e;
  e.code = kBlkOk;
  e.type = 0;
  e.klen = 0;
  e.vlen = kNoValue;
  e.txn = 0;
  e.size = 0;
  if (s >= doff || doff - s < 5) {
    e.code = kBlkEntryRange;
    return e;
  }
  e.type = rd.u8(s);
  if (e.type > kTypeDeleted) {
    e.code = kBlkBadType;
    return e;
  }
  e.klen = rd.u32(s + 1);
  if (e.klen > kMaxKey) {
    e.code = kBlkKeyTooLong;
    return e;
  }
  uint64_t p = s + 5 + e.klen;
  if (e.type != kTypeDeleted) {
    if (p + 4 > doff) {
      e.code = kBlkEntryRange;
      return e;
    }
    e.vlen = rd.u32(p);
    p += 4ull + e.vlen;
  }
  if (p + 8 > doff) {
    e.code = kBlkEntryRange;
    return e;
  }
  // value.empty() test of GetTransactionIdFromDataEntry (block_reader.cc:109-111)
  const bool quirk = txn_mode == 0u && e.type != kTypeDeleted && e.vlen == 0u;
  e.txn = rd.u64(quirk ? s + 5 + e.klen : p);
  e.size = p + 8 - s;
  return e;
}

// Block-level checks on the 16 B extra (table_reader.cc:226-232).
__device__ __forceinline__ uint32_t check_extra(uint64_t len, uint64_t n, uint64_t doff) {
  if (n == 0) return kBlkEmpty;
  if (doff > len - 16 || n > (len - 16 - doff) / 16) return kBlkOffsetsRange;
  return kBlkOk;
}

// ---------------------------------------------------------------------------
// Fused round trip: ONE kernel, one wave per block, every block size.
//
//   1. a block that fits the wave's LDS slot is staged whole by LDS-DMA
//      (global_load_lds_dwordx4, 1 KiB per wave instruction); a larger block is
//      parsed straight from HBM and later streamed through the slot in windows;
//   2. decode: 16 B extra, then entries 64 per round (one lane per entry),
//      validated exactly like the oracle; a wave-wide scan of the recomputed
//      entry sizes gives each entry's re-encoded start;
//   3. re-encode.  When the starts equal the stored starts (entries packed
//      back-to-back: every block the reference writes) each entry's encoding
//      of its decoded fields already sits at its output position, except the
//      txn the compat reader rewrites, so the block is re-emitted from the
//      staged bytes with the offset section, the extra and those txns
//      regenerated.  Otherwise (entries out of order / gaps, valid for the
//      reference reader) the wave re-packs the entries one output byte at a
//      time (rare, malformed-ish input).
// ---------------------------------------------------------------------------
constexpr uint32_t kRtWaves = 4;
constexpr uint32_t kRtSlot = kRtSlotBytes;     // LDS bytes per wave
constexpr uint32_t kRtWinChunks = 256;         // 16 B chunks per streaming window

struct Pass1 {
  uint32_t st;
  bool canon;
  bool quirk; // some entry gets its txn rewritten (compat mode)
  uint64_t data; // sum of recomputed entry sizes
};

template <class R>
__device__ __forceinline__ Pass1 rt_pass1(const R &rd, uint64_t L, uint64_t n, uint64_t doff,
                                          uint32_t txn_mode) {
  Pass1 p{kBlkOk, doff + 16 * n + 16 == L, false, 0};
  const uint32_t lane = lane_id();
  for (uint64_t i0 = 0; i0 < n; i0 += kWave) {
    const uint64_t i = i0 + lane;
    Entry e{};
    uint64_t s = 0;
    if (i < n) {
      s = rd.u64(doff + 16 * i);
      e = parse_entry(rd, s, doff, txn_mode);
    }
    const uint64_t bad = __ballot(e.code != kBlkOk);
    if (bad) {
      p.st = __shfl(e.code, __ffsll(static_cast<long long>(bad)) - 1, kWave);
      return p;
    }
    const uint64_t incl = wave_incl_scan_u64(e.size);
    const bool mism = i < n && s != p.data + incl - e.size;
    p.canon = p.canon && !__any(mism);
    p.quirk = p.quirk || __any(i < n && txn_mode == 0u && e.type != kTypeDeleted && e.vlen == 0u);
    p.data += __shfl(incl, kWave - 1, kWave);
  }
  p.canon = p.canon && p.data == doff;
  return p;
}

// LDS image byte writes of a 64-bit little-endian value clipped to [lo, hi)
// (positions relative to the image).
__device__ __forceinline__ void img_put64_clipped(uint8_t *img, int64_t pos, uint64_t v, int64_t lo,
                                                  int64_t hi) {
  if (pos >= lo && pos + 8 <= hi && ((pos & 3) == 0)) {
    uint32_t *w = reinterpret_cast<uint32_t *>(img + pos);
    w[0] = static_cast<uint32_t>(v);
    w[1] = static_cast<uint32_t>(v >> 32);
    return;
  }
  for (int j = 0; j < 8; j++)
    if (pos + j >= lo && pos + j < hi) img[pos + j] = static_cast<uint8_t>(v >> (8 * j));
}

__device__ __forceinline__ void g_put64_bytes(uint8_t *p, uint64_t v) {
  for (int j = 0; j < 8; j++) p[j] = static_cast<uint8_t>(v >> (8 * j));
}

// Store image bytes [c0*16, (c0+cnt)*16) to gd at the same positions; only the
// bytes in [keep_lo, keep_hi) belong to this block (edge chunks are shared
// with the neighbouring blocks and are written byte by byte).
__device__ __forceinline__ void store_window(const uint8_t *img, uint8_t *gd, uint32_t cnt, int64_t base,
                                             int64_t keep_lo, int64_t keep_hi) {
  const uint32_t lane = lane_id();
  for (uint32_t c0 = 0; c0 < cnt; c0 += kWave) {
    const uint32_t c = c0 + lane;
    if (c >= cnt) continue;
    const int64_t lo = base + 16 * static_cast<int64_t>(c);
    if (lo >= keep_lo && lo + 16 <= keep_hi) {
      const u32x4 v = *reinterpret_cast<const u32x4 *>(img + 16 * c);
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(gd + lo));
    } else { // an edge chunk shared with a neighbouring block: only this block's bytes,
             // as dwords where they are dword-aligned (back-to-back 4188 B blocks: always)
      const int64_t x0 = lo < keep_lo ? keep_lo : lo;
      const int64_t x1 = lo + 16 < keep_hi ? lo + 16 : keep_hi;
      int64_t x = x0;
      for (; x < x1 && (x & 3); x++) gd[x] = img[x - base];
      for (; x + 4 <= x1; x += 4)
        *reinterpret_cast<uint32_t *>(gd + x) = *reinterpret_cast<const uint32_t *>(img + (x - base));
      for (; x < x1; x++) gd[x] = img[x - base];
    }
  }
}

// Non-packed block: re-pack entries into dst (byte-granular, global memory).
__device__ void rt_repack_wave(const RtArgs &a, const uint8_t *blk, uint8_t *out, uint64_t n, uint64_t doff,
                               uint64_t data, uint8_t *slot) {
  const uint32_t lane = lane_id();
  const GlobalReader rd{blk};
  uint64_t *s_src = reinterpret_cast<uint64_t *>(slot);          // 64 x 8
  uint64_t *s_out = s_src + kWave;                              // 64 x 8
  uint64_t *s_txn = s_out + kWave;                              // 64 x 8
  uint32_t *s_kl = reinterpret_cast<uint32_t *>(s_txn + kWave); // 64 x 4
  uint32_t *s_pt = s_kl + kWave;                                // 64 x 4
  uint64_t carry = 0;
  for (uint64_t i0 = 0; i0 < n; i0 += kWave) {
    const uint64_t i = i0 + lane;
    Entry e{};
    uint64_t s = 0;
    if (i < n) {
      s = rd.u64(doff + 16 * i);
      e = parse_entry(rd, s, doff, a.txn_mode);
    }
    const uint64_t incl = wave_incl_scan_u64(e.size);
    const uint64_t o = carry + incl - e.size;
    if (i < n) {
      s_src[lane] = s;
      s_out[lane] = o;
      s_txn[lane] = e.txn;
      s_kl[lane] = e.klen;
      s_pt[lane] = (a.txn_mode == 0u && e.type != kTypeDeleted && e.vlen == 0u) ? 1u : 0u;
      g_put64_bytes(out + data + 16 * i, o);
      g_put64_bytes(out + data + 16 * i + 8, e.size);
    }
    wave_lds_sync();
    const uint64_t tot = __shfl(incl, kWave - 1, kWave);
    const uint32_t wn = static_cast<uint32_t>(n - i0 < kWave ? n - i0 : kWave);
    for (uint64_t x = carry + lane; x < carry + tot; x += kWave) {
      uint32_t lo = 0, hi = wn - 1;
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (s_out[mid] <= x) lo = mid;
        else hi = mid - 1;
      }
      const uint64_t rel = x - s_out[lo];
      const uint64_t t0 = 9ull + s_kl[lo];
      out[x] = (s_pt[lo] && rel >= t0 && rel < t0 + 8) ? static_cast<uint8_t>(s_txn[lo] >> (8 * (rel - t0)))
                                                        : blk[s_src[lo] + rel];
    }
    wave_lds_sync();
    carry += tot;
  }
  if (lane == 0) {
    g_put64_bytes(out + data + 16 * n, n);
    g_put64_bytes(out + data + 16 * n + 8, data);
  }
}

__device__ __forceinline__ void rt_report(const RtArgs &a, uint64_t b, uint32_t st, uint64_t out_len) {
  if (lane_id() == 0) {
    if (a.status) a.status[b] = st;
    if (a.out_len) a.out_len[b] = st == kBlkOk ? out_len : 0;
    if (st != kBlkOk) atomicAdd(a.err_count, 1ull);
  }
}

// Issue the LDS-DMA of a small block ([off & ~15, off + L) -> img); returns the
// number of wave-level DMA instructions issued (for counted vmcnt waits).
template <int AUX = 0>
__device__ __forceinline__ uint32_t rt_stage(const uint8_t *g, uint8_t *img, uint32_t nchunk) {
  const uint32_t lane = lane_id();
  uint32_t k = 0;
  for (uint32_t c0 = 0; c0 < nchunk; c0 += kWave, k++) {
    const uint32_t c = c0 + lane;
    if (c < nchunk)
      __builtin_amdgcn_global_load_lds((gbl_void_t *)(g + 16u * c), (lds_void_t *)(img + 16u * c0), 16, 0, AUX);
  }
  return k;
}

// A block staged whole in img (image byte pad == block byte 0).
__device__ __forceinline__ void rt_small(const RtArgs &a, uint64_t b, uint8_t *img, uint64_t off, uint32_t L,
                                         uint32_t pad) {
  const uint32_t lane = lane_id();
  const LdsReader rd{img + pad};
  const uint64_t n = uniform64(rd.u64(L - 16));
  const uint64_t doff = uniform64(rd.u64(L - 8));
  uint32_t st = check_extra(L, n, doff);
  if (st != kBlkOk) return rt_report(a, b, st, 0);
  if (n <= kWave) { // one entry per lane: parse, validate and regenerate in one pass
    uint8_t *wimg = img + pad;
    const uint32_t i = lane, nn = static_cast<uint32_t>(n), dd = static_cast<uint32_t>(doff);
    Entry e{};
    uint64_t s = 0;
    if (i < nn) {
      s = rd.u64(dd + 16ull * i);
      e = parse_entry(rd, s, doff, a.txn_mode);
    }
    const uint64_t bad = __ballot(e.code != kBlkOk);
    if (bad) return rt_report(a, b, __shfl(e.code, __ffsll(static_cast<long long>(bad)) - 1, kWave), 0);
    const uint32_t sz = static_cast<uint32_t>(e.size); // < L < 2^32
    const uint32_t incl = wave_incl_scan_u32(sz);
    const uint32_t data = __shfl(incl, kWave - 1, kWave);
    const bool canon = doff + 16 * n + 16 == L && data == doff && !__any(i < nn && s != incl - sz);
    const bool qk = i < nn && a.txn_mode == 0u && e.type != kTypeDeleted && e.vlen == 0u;
    if (!canon) {
      const uint64_t out_len = data + 16 * n + 16;
      if (out_len > L) return rt_report(a, b, kBlkNoRoom, 0);
      rt_repack_wave(a, a.src + off, a.dst + off, n, doff, data, img);
      return rt_report(a, b, kBlkOk, out_len);
    }
    if (i < nn) { // offset entry (start = scan = stored start, size recomputed), compat txn
      lds_st_u64u(wimg, dd + 16u * i, incl - sz);
      lds_st_u64u(wimg, dd + 16u * i + 8u, sz);
      if (qk) lds_st_u64u(wimg, static_cast<uint32_t>(s) + 9u + e.klen, e.txn);
    }
    if (lane == 0) { // extra: n, data bytes (== doff)
      lds_st_u64u(wimg, L - 16, n);
      lds_st_u64u(wimg, L - 8, data);
    }
    wave_lds_sync();
    store_window(img, a.dst + (off - pad), (pad + L + 15u) >> 4, 0, pad, pad + L);
    return rt_report(a, b, kBlkOk, L);
  }
  const Pass1 p = rt_pass1(rd, L, n, doff, a.txn_mode);
  if (p.st != kBlkOk) return rt_report(a, b, p.st, 0);
  if (!p.canon) {
    const uint64_t out_len = p.data + 16 * n + 16;
    if (out_len > L) return rt_report(a, b, kBlkNoRoom, 0);
    rt_repack_wave(a, a.src + off, a.dst + off, n, doff, p.data, img);
    return rt_report(a, b, kBlkOk, out_len);
  }
  // re-encode in place: offset section (start, size) from the scan, extra,
  // compat txns
  uint8_t *wimg = img + pad;
  const uint32_t nn = static_cast<uint32_t>(n), dd = static_cast<uint32_t>(doff);
  uint32_t carry = 0;
  for (uint32_t i0 = 0; i0 < nn; i0 += kWave) {
    const uint32_t i = i0 + lane;
    uint32_t sz = 0;
    Entry e{};
    uint64_t s = 0;
    if (i < nn) {
      s = rd.u64(dd + 16ull * i);
      e = parse_entry(rd, s, doff, a.txn_mode);
      sz = static_cast<uint32_t>(e.size);
    }
    const uint32_t incl = wave_incl_scan_u32(sz);
    if (i < nn) {
      lds_st_u64u(wimg, dd + 16u * i, carry + incl - sz);
      lds_st_u64u(wimg, dd + 16u * i + 8u, sz);
      if (p.quirk && e.type != kTypeDeleted && e.vlen == 0u)
        lds_st_u64u(wimg, static_cast<uint32_t>(s) + 9u + e.klen, e.txn);
    }
    carry += __shfl(incl, kWave - 1, kWave);
  }
  if (lane == 0) {
    lds_st_u64u(wimg, L - 16, n);
    lds_st_u64u(wimg, L - 8, carry);
  }
  wave_lds_sync();
  store_window(img, a.dst + (off - pad), (pad + L + 15u) >> 4, 0, pad, pad + L);
  rt_report(a, b, kBlkOk, L);
}

// A block larger than the slot: parsed from HBM, streamed through img.
__device__ void rt_large(const RtArgs &a, uint64_t b, uint8_t *img, uint64_t off, uint32_t L, uint32_t pad) {
  const uint32_t lane = lane_id();
  const uint8_t *g = a.src + (off - pad);
  uint8_t *gd = a.dst + (off - pad);
  const uint32_t nchunk = (pad + L + 15u) >> 4;
  const uint8_t *blk = a.src + off;
  const GlobalReader rd{blk};
  const uint64_t n = uniform64(rd.u64(L - 16));
  const uint64_t doff = uniform64(rd.u64(L - 8));
  uint32_t st = check_extra(L, n, doff);
  if (st != kBlkOk) return rt_report(a, b, st, 0);
  const Pass1 p = rt_pass1(rd, L, n, doff, a.txn_mode);
  if (p.st != kBlkOk) return rt_report(a, b, p.st, 0);
  if (!p.canon) {
    const uint64_t out_len = p.data + 16 * n + 16;
    if (out_len > L) return rt_report(a, b, kBlkNoRoom, 0);
    rt_repack_wave(a, blk, a.dst + off, n, doff, p.data, img);
    return rt_report(a, b, kBlkOk, out_len);
  }
  const int64_t ob = static_cast<int64_t>(doff);        // offset section start (block-relative)
  const int64_t oe = ob + 16 * static_cast<int64_t>(n); // its end == L - 16
  for (uint32_t w = 0; w < nchunk; w += kRtWinChunks) {
    const uint32_t cnt = nchunk - w < kRtWinChunks ? nchunk - w : kRtWinChunks;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // previous window's stores read img
    rt_stage(g + 16ull * w, img, cnt);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // window = block bytes [wlo, whi); image byte 0 == block byte wlo
    const int64_t wlo = 16 * static_cast<int64_t>(w) - pad;
    const int64_t whi = wlo + 16 * static_cast<int64_t>(cnt);
    if (whi > ob && wlo < oe) {
      const int64_t a0 = wlo > ob ? wlo : ob;
      const int64_t a1 = whi < oe ? whi : oe;
      const uint64_t i_lo = static_cast<uint64_t>(a0 - ob) >> 4;
      const uint64_t i_hi = (static_cast<uint64_t>(a1 - ob) + 15) >> 4;
      for (uint64_t i = i_lo + lane; i < i_hi; i += kWave) {
        const uint64_t s = rd.u64(doff + 16 * i);
        const uint64_t s1 = i + 1 < n ? rd.u64(doff + 16 * (i + 1)) : doff; // packed: size = next start - start
        const int64_t pos = ob + 16 * static_cast<int64_t>(i) - wlo;
        img_put64_clipped(img, pos, s, 0, whi - wlo);
        img_put64_clipped(img, pos + 8, s1 - s, 0, whi - wlo);
      }
    }
    if (lane == 0 && whi > oe) {
      img_put64_clipped(img, oe - wlo, n, 0, whi - wlo);
      img_put64_clipped(img, oe + 8 - wlo, doff, 0, whi - wlo);
    }
    wave_lds_sync();
    store_window(img, gd, cnt, 16 * static_cast<int64_t>(w), pad, pad + static_cast<int64_t>(L));
    wave_lds_sync();
  }
  if (p.quirk) {
    // compat txn rewrites after every bulk store of this wave has landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint8_t *out = a.dst + off;
    for (uint64_t i0 = 0; i0 < n; i0 += kWave) {
      const uint64_t i = i0 + lane;
      if (i < n) {
        const uint64_t s = rd.u64(doff + 16 * i);
        const Entry e = parse_entry(rd, s, doff, a.txn_mode);
        if (e.type != kTypeDeleted && e.vlen == 0u) g_put64_bytes(out + s + 9 + e.klen, e.txn);
      }
    }
  }
  rt_report(a, b, kBlkOk, L);
}

// 0: staged small block, 1: large block, 2: error reported
__device__ __forceinline__ uint32_t rt_classify(const RtArgs &a, uint64_t b, uint64_t &off, uint32_t &L,
                                                uint32_t &pad) {
  off = uniform64(a.blk_off[b]);
  const uint64_t len = uniform64(a.blk_len[b]);
  pad = static_cast<uint32_t>(off & 15u);
  L = static_cast<uint32_t>(len);
  if (len < 16) {
    rt_report(a, b, kBlkTooSmall, 0);
    return 2;
  }
  if (len >= (1ull << 32)) {
    rt_report(a, b, kBlkTooLarge, 0);
    return 2;
  }
  return pad + L + 16 <= kRtSlot ? 0u : 1u;
}

// One block per wave, 4 waves per workgroup, grid covers every block.  The
// staging DMA uses sc0 (aux = 1): in the A/B of profiles/r01_ab_variants.md it
// was the fastest of {4, 8, 16, 2, 1 waves per WG} x {default, sc0, nt, sc0|nt}
// within noise at 256 MiB and +5 % at 1 GiB; a persistent double-buffered
// variant was 40 % slower.  The structure runs at the speed of the same
// LDS-staged copy without any parse (the parse is hidden under HBM time).
__global__ __launch_bounds__(kRtWaves *kWave, 8) void rt_kernel(RtArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kRtWaves * kRtSlot];
  const uint32_t wave = uniform(threadIdx.x / kWave);
  const uint32_t wg = a.xcd ? xcd_logical_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint64_t b = static_cast<uint64_t>(wg) * kRtWaves + wave;
  if (b >= a.nblocks) return;
  uint8_t *img = lds + wave * kRtSlot;
  uint64_t off;
  uint32_t L, pad;
  const uint32_t cls = rt_classify(a, b, off, L, pad);
  if (cls == 0) {
    rt_stage<1>(a.src + (off - pad), img, (pad + L + 15u) >> 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    rt_small(a, b, img, off, L, pad);
  } else if (cls == 1) {
    rt_large(a, b, img, off, L, pad);
  }
}


// ---------------------------------------------------------------------------
// Decode to the record table.
// ---------------------------------------------------------------------------
constexpr uint32_t kDecWaves = 4;

// Parse one block into the record table (and, when asked, the 32 B sort keys
// of the compaction merge).  R reads block bytes (LDS image or HBM).
// kSk: the compaction's variant (merge keys with their running-minimum merge
// txns; its registers stay out of the plain decode)
template <bool kSk, class R>
// base / base1: rec_base[b], rec_base[b + 1], loaded by the caller before it
// waits for the block's bytes (one dependent round trip fewer per wave)
__device__ __forceinline__ uint32_t decode_block(const DecArgs &a, const R &rd, uint64_t b, uint64_t off,
                                                 uint64_t len, uint64_t base, uint64_t base1) {
  const uint32_t lane = lane_id();
  base = uniform64(base);
  const uint64_t n = uniform64(rd.u64(len - 16));
  const uint64_t doff = uniform64(rd.u64(len - 8));
  uint32_t st = check_extra(len, n, doff);
  if (st == kBlkOk && n != uniform64(base1) - base) st = kBlkCountMismatch;
  if (st != kBlkOk) return st;
  // previous record of the block (sortedness check): carried across chunks,
  // with its merge txn (SortKey)
  uint64_t c0 = 0, c1 = 0, ctx = 0, cs = 0, ceff = 0;
  uint32_t ckl = 0;
  for (uint64_t i0 = 0; i0 < n; i0 += kWave) {
    const uint64_t i = i0 + lane;
    Entry e{};
    uint64_t s = 0;
    if (i < n) {
      s = rd.u64(doff + 16 * i);
      e = parse_entry(rd, s, doff, a.txn_mode);
    }
    const uint64_t bad = __ballot(e.code != kBlkOk);
    if (bad) return __shfl(e.code, __ffsll(static_cast<long long>(bad)) - 1, kWave);
    bool same = false; // same key as the block's previous record
    if (a.unsorted) {
      // TableBuilder requires sorted input (table_builder.h:77): a record may
      // not sort before its predecessor (key asc, then txn desc).  The
      // compaction (a.sk) checks the key order only: its merge txns absorb
      // versions of a key that are out of txn order as read
      const uint64_t k0 = i < n && e.klen ? key_prefix8(__builtin_bswap64(rd.u64(s + 5)), e.klen) : 0;
      const uint64_t k1 = i < n && e.klen > 8 ? key_prefix8(__builtin_bswap64(rd.u64(s + 13)), e.klen - 8) : 0;
      uint64_t q0 = __shfl_up(k0, 1u, kWave), q1 = __shfl_up(k1, 1u, kWave);
      uint64_t qt = __shfl_up(e.txn, 1u, kWave), qs = __shfl_up(s, 1u, kWave);
      uint32_t ql = __shfl_up(e.klen, 1u, kWave);
      if (lane == 0) {
        q0 = c0, q1 = c1, qt = ctx, qs = cs, ql = ckl;
      }
      bool viol = false;
      if (i < n && i > 0) {
        int c = k0 != q0 ? (k0 < q0 ? -1 : 1) : (k1 != q1 ? (k1 < q1 ? -1 : 1) : 0);
        if (c == 0 && e.klen > 16 && ql > 16) {
          const uint32_t m = e.klen < ql ? e.klen : ql;
          for (uint32_t j = 16; j < m && c == 0; j++) {
            const uint32_t x = rd.u8(s + 5 + j), y = rd.u8(qs + 5 + j);
            if (x != y) c = x < y ? -1 : 1;
          }
        }
        if (c == 0) c = e.klen < ql ? -1 : (e.klen > ql ? 1 : 0);
        viol = c < 0 || (c == 0 && !kSk && e.txn > qt);
        same = c == 0;
      }
      const uint64_t v = __ballot(viol);
      if (v && lane == 0) atomicAdd(a.unsorted, static_cast<unsigned long long>(__popcll(v)));
      c0 = __shfl(k0, kWave - 1, kWave), c1 = __shfl(k1, kWave - 1, kWave);
      ctx = __shfl(e.txn, kWave - 1, kWave), cs = __shfl(s, kWave - 1, kWave);
      ckl = __shfl(e.klen, kWave - 1, kWave);
    }
    // merge txn: segmented running minimum of the txns as read over the key
    // groups of the block (Hillis-Steele over (value, segment-start) pairs;
    // lanes still open after it continue the previous chunk's last group)
    uint64_t eff = e.txn;
    if (kSk && a.unsorted) {
      bool f = !same;
#pragma unroll
      for (uint32_t d = 1; d < kWave; d <<= 1) {
        const uint64_t uv = __shfl_up(eff, d, kWave);
        const bool uf = __shfl_up(static_cast<int>(f), d, kWave) != 0;
        if (lane >= d && !f) {
          eff = uv < eff ? uv : eff;
          f = uf;
        }
      }
      if (!f && i0 > 0) eff = ceff < eff ? ceff : eff;
      ceff = __shfl(eff, kWave - 1, kWave);
      if (a.inv && __any(i < n && eff != e.txn) && lane == 0) atomicOr(a.inv, kGuardInv);
    }
    if (i < n) {
      const uint64_t r = base + i;
      if (a.rx) {
        RecX x;
        x.ko = off + s + 5;
        x.vl = e.vlen;
        x.type = e.type;
        a.rx[r] = x;
      } else {
        a.out.type[r] = static_cast<uint8_t>(e.type);
        a.out.key_len[r] = e.klen;
        a.out.val_len[r] = e.vlen;
        a.out.txn[r] = e.txn;
        a.out.key_off[r] = off + s + 5;
        a.out.val_off[r] = e.type != kTypeDeleted ? off + s + 9 + e.klen : 0;
      }
      if (kSk) {
        // 16 B big-endian key prefix (a key is followed by >= 40 B of block)
        SortKey k;
        k.p0 = e.klen ? key_prefix8(__builtin_bswap64(rd.u64(s + 5)), e.klen) : 0;
        k.p1 = e.klen > 8 ? key_prefix8(__builtin_bswap64(rd.u64(s + 13)), e.klen - 8) : 0;
        k.tx = eff;
        k.kl = e.klen | (eff != e.txn ? kSkRead : 0u);
        k.id = static_cast<uint32_t>(r);
        a.sk[r] = k;
      }
    }
  }
  return kBlkOk;
}

// One wave per block; a block that fits the LDS slot is staged by LDS-DMA and
// parsed from LDS (the lane-per-entry header reads would otherwise be
// dependent HBM round trips), a larger one is parsed from HBM.
template <bool kSk>
__global__ __launch_bounds__(kDecWaves *kWave) void decode_kernel(DecArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kDecWaves * kRtSlot];
  const uint32_t wave = uniform(threadIdx.x / kWave);
  const uint32_t wg = a.xcd ? xcd_logical_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint64_t b = static_cast<uint64_t>(wg) * kDecWaves + wave;
  if (b >= a.nblocks) return;
  uint8_t *img = lds + wave * kRtSlot;
  const uint64_t off = uniform64(a.blk_off[b]);
  const uint64_t len = uniform64(a.blk_len[b]);
  const uint32_t pad = static_cast<uint32_t>(off & 15u);
  uint32_t st;
  if (len < 16) {
    st = kBlkTooSmall;
  } else if (pad + len + 16 <= kRtSlot) {
    const uint64_t base = a.rec_base[b], base1 = a.rec_base[b + 1]; // in flight with the block's DMA
    rt_stage<1>(a.src + (off - pad), img, static_cast<uint32_t>((pad + len + 15) >> 4));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st = decode_block<kSk>(a, LdsReader{img + pad}, b, off, len, base, base1);
  } else {
    st = decode_block<kSk>(a, GlobalReader{a.src + off}, b, off, len, a.rec_base[b], a.rec_base[b + 1]);
  }
  if (lane_id() == 0) {
    if (a.status) a.status[b] = st;
    if (st != kBlkOk) atomicAdd(a.err_count, 1ull);
  }
}

// ---------------------------------------------------------------------------
// Encode: records -> blocks.
// ---------------------------------------------------------------------------
// an encode of no blocks: the offset array's closing entry only
__global__ void enc_none_kernel(uint64_t out_base, uint64_t *blk_off) { blk_off[0] = out_base; }

// Encode offsets without a scan over the records: 8 lanes per block sum its
// entry sizes (block length = entries + 16 per offset entry + the 16 B extra)
// and a device scan of the block lengths gives the block offsets; the entry
// offsets inside a block are scanned by the block's own wave in
// enc_lds_kernel<0>.  Replaced the chained 1.8 M-record look-back scan + the
// closed-form offsets (config 2 encode leg -4.6 us; one kernel with a thread
// per block and a look-back over 256-block tiles was 20 us slower, 5 us slower
// with the tile's entry sizes staged in LDS; the P pass of enc_prefix 7 us:
// profiles/r02_ab/encode_ab.md).
constexpr uint32_t kBsG = 8;

__global__ __launch_bounds__(256) void enc_bsum_kernel(const uint32_t *kl, const uint32_t *vl,
                                                       const uint64_t *blk_first, uint64_t nblocks,
                                                       uint64_t *blk_len) {
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
  const uint64_t b = t / kBsG;
  const uint32_t g = static_cast<uint32_t>(t % kBsG);
  uint64_t f0 = 0, f1 = 0, sum = 0;
  if (b < nblocks) {
    f0 = blk_first[b];
    f1 = blk_first[b + 1];
    for (uint64_t r = f0 + g; r < f1; r += kBsG) sum += entry_size(kl[r], vl[r]);
  }
#pragma unroll
  for (uint32_t d = kBsG / 2; d > 0; d >>= 1) sum += __shfl_xor(sum, d, kWave); // stays inside the 8-lane group
  if (b < nblocks && g == 0) blk_len[b] = sum + 16 * (f1 - f0) + 16;
}

// One workgroup per block; each thread assembles 16-byte output chunks aligned
// to the destination address.  A chunk that lies inside one key or value span
// is funnel-shifted from five source dwords; any other chunk is assembled byte
// by byte through a per-thread LDS slot.
constexpr uint32_t kEncThreads = 256;
constexpr uint32_t kEncWaves = 4;
constexpr uint32_t kEncSlot = 4608;       // LDS image bytes per wave (enc_lds_kernel)

__device__ __forceinline__ u32x4 load16_unaligned(const uint8_t *p) {
  uint32_t sh;
  const uint32_t *w = align4_down(p, sh);
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3];
  const uint32_t w4 = sh ? w[4] : 0u;
  u32x4 v;
  v.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
  v.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
  v.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
  v.w = __builtin_amdgcn_alignbyte(w4, w3, sh);
  return v;
}

// kT threads (tid = 0..kT-1) encode block b straight to HBM (one wave:
// enc_lds_kernel's records -> blocks past its LDS slot; P holds the block's
// relative entry offsets, written by enc_wave_offsets)
template <uint32_t kT = kEncThreads>
__device__ void enc_emit_block(const EncArgs &a, uint64_t b, uint8_t *slot, uint32_t tid = threadIdx.x) {
  const uint64_t f0 = a.blk_first[b], f1 = a.blk_first[b + 1];
  const uint64_t n = f1 - f0;
  const uint64_t P0 = a.P[f0];
  const uint64_t bo = a.out_blk_off[b];
  const uint64_t L = a.out_blk_len[b];
  if ((bo & 15) + L + 16 <= kEncSlot) return; // encoded by enc_lds_kernel
  // entry bytes from the block length (P[f1] is not read: in mode 0 it belongs
  // to the next block's wave)
  const uint64_t D = L - 16 * n - 16;
  auto Pr = [&](uint64_t x) { return x < f1 ? a.P[x] - P0 : D; }; // entry offset, x in [f0, f1]
  uint8_t *dst = a.dst;
  uint8_t *my = slot + 16 * tid;

  const uint64_t c_first = bo >> 4, c_end = (bo + L + 15) >> 4;
  for (uint64_t c = c_first + tid; c < c_end; c += kT) {
    const int64_t x0 = static_cast<int64_t>(16 * c) - static_cast<int64_t>(bo);
    const uint64_t xs = x0 < 0 ? 0 : static_cast<uint64_t>(x0);
    const uint64_t xe = static_cast<uint64_t>(x0 + 16) < L ? static_cast<uint64_t>(x0 + 16) : L;
    const bool full = x0 >= 0 && static_cast<uint64_t>(x0) + 16 <= L;
    // entry cursor for the first data byte of this chunk
    uint64_t r = f0;
    if (xs < D) {
      uint64_t lo = f0, hi = f1 - 1;
      while (lo < hi) {
        const uint64_t mid = (lo + hi + 1) >> 1;
        if (a.P[mid] - P0 <= xs) lo = mid;
        else hi = mid - 1;
      }
      r = lo;
      // fast path: the whole chunk inside one key or value span
      if (full) {
        const uint64_t o = a.P[r] - P0;
        const uint32_t kl = a.in.key_len[r], vl = a.in.val_len[r];
        const uint64_t rel = xs - o;
        const uint8_t *sp = nullptr;
        if (rel >= 5 && rel + 16 <= 5ull + kl) sp = a.key_src + a.in.key_off[r] + (rel - 5);
        else if (vl != kNoValue && rel >= 9ull + kl && rel + 16 <= 9ull + kl + vl)
          sp = a.val_src + a.in.val_off[r] + (rel - 9 - kl);
        if (sp) {
          __builtin_nontemporal_store(load16_unaligned(sp), reinterpret_cast<u32x4 *>(dst + 16 * c));
          continue;
        }
      }
    }
    for (uint64_t x = xs; x < xe; x++) {
      uint32_t v;
      if (x < D) {
        while (r + 1 < f1 && a.P[r + 1] - P0 <= x) r++;
        const uint64_t rel = x - (a.P[r] - P0);
        const uint32_t kl = a.in.key_len[r], vl = a.in.val_len[r];
        if (rel == 0) v = a.in.type[r];
        else if (rel < 5) v = (kl >> (8 * (rel - 1))) & 0xFFu;
        else if (rel < 5ull + kl) v = a.key_src[a.in.key_off[r] + rel - 5];
        else if (vl != kNoValue && rel < 9ull + kl) v = (vl >> (8 * (rel - 5 - kl))) & 0xFFu;
        else if (vl != kNoValue && rel < 9ull + kl + vl) v = a.val_src[a.in.val_off[r] + rel - 9 - kl];
        else {
          const uint64_t t0 = 5ull + kl + (vl != kNoValue ? 4ull + vl : 0ull);
          v = static_cast<uint32_t>(a.in.txn[r] >> (8 * (rel - t0))) & 0xFFu;
        }
      } else if (x < D + 16 * n) {
        const uint64_t i = (x - D) >> 4, j = (x - D) & 15;
        const uint64_t val = j < 8 ? Pr(f0 + i) : Pr(f0 + i + 1) - Pr(f0 + i);
        v = static_cast<uint32_t>(val >> (8 * (j & 7))) & 0xFFu;
      } else {
        const uint64_t j = x - D - 16 * n;
        const uint64_t val = j < 8 ? n : D;
        v = static_cast<uint32_t>(val >> (8 * (j & 7))) & 0xFFu;
      }
      if (full) my[x - xs] = static_cast<uint8_t>(v);
      else dst[bo + x] = static_cast<uint8_t>(v);
    }
    if (full) {
      __builtin_nontemporal_store(*reinterpret_cast<const u32x4 *>(my),
                                  reinterpret_cast<u32x4 *>(dst + 16 * c));
    }
  }
}


// the consistency guard of one record of a compaction block (EncArgs::guard):
// inside the block image, at least its header + key, its source inside
// [5, *src_end).  Compaction only; true when unguarded.
__device__ __forceinline__ bool enc1_entry_ok(const EncArgs &a, uint64_t o, uint64_t sz, uint32_t kl, uint64_t ko,
                                              uint64_t D) {
  if (!a.guard) return true;
  const uint64_t e = *a.src_end;
  return o <= D && sz <= D - o && kl <= kMaxKey && sz >= 13ull + kl && ko >= 5 && ko - 5 <= e && sz <= e - (ko - 5);
}
__device__ __forceinline__ bool enc1_block_ok(const EncArgs &a, uint64_t bo, uint64_t L, uint64_t n) {
  if (!a.guard) return true;
  return L >= 16 * n + 16 && bo <= a.cap && L <= a.cap - bo;
}

// Large block of a compaction (records decoded from blocks held in key_src):
// every entry is already its own encoding in its input block, so the wave
// that met the block copies whole entries: each 16 B destination chunk
// (aligned) is funnel-shifted from two aligned 16 B source chunks (the source
// / destination skew is constant along the entry); the partial chunks at its
// ends and the txn (the compat reader may have changed it) go byte by byte.
// Then the offset section and the extra.

__device__ __forceinline__ u32x4 funnel16(const u32x4 &v0, const u32x4 &v1, uint32_t s) {
  const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  const uint32_t q = s >> 2, r = s & 3u;
  uint32_t o[5];
#pragma unroll
  for (uint32_t j = 0; j < 5; j++) { // o[j] = w[q + j] (q <= 3)
    const uint32_t a0 = w[j], a1 = w[j + 1], a2 = w[j + 2], a3 = w[j + 3];
    o[j] = q == 0 ? a0 : (q == 1 ? a1 : (q == 2 ? a2 : a3));
  }
  u32x4 out;
  out.x = __builtin_amdgcn_alignbyte(o[1], o[0], r);
  out.y = __builtin_amdgcn_alignbyte(o[2], o[1], r);
  out.z = __builtin_amdgcn_alignbyte(o[3], o[2], r);
  out.w = __builtin_amdgcn_alignbyte(o[4], o[3], r);
  return out;
}

// copy_span by one wave with kU chunks per lane in flight: the right-hand
// source chunk of lane l's funnel shift is lane l + 1's own chunk (a shuffle),
// for lane 63 lane 0's chunk of the next group (a broadcast), and after the
// last group one extra chunk every lane loads (the same address): one load per
// 16 B instead of two.  The source may be read up to 31 B past sp + len
// (inside its block: the txn and the offset section follow every entry).
// kU = 4 (config 5 encode 232 -> 224 us); kU = 8 is
// faster on config 5 (210 us) but its 98 VGPRs cost enc_lds_kernel<1> a wave
// per SIMD: config 3 encode 500 -> 624 us (profiles/r02_ab/encode_ab.md)
constexpr uint32_t kWaveSpanUnroll = 4;
template <uint32_t kU>
__device__ __forceinline__ void copy_span_wave(uint8_t *dp, const uint8_t *sp, uint64_t len) {
  const uint32_t lane = lane_id();
  const uintptr_t d0 = reinterpret_cast<uintptr_t>(dp), d1 = d0 + len;
  const uintptr_t cb = (d0 + 15) & ~static_cast<uintptr_t>(15), ce = d1 & ~static_cast<uintptr_t>(15);
  if (cb >= ce) {
    for (uint64_t x = lane; x < len; x += kWave) dp[x] = sp[x];
    return;
  }
  const uint64_t nch = (ce - cb) >> 4;
  const uint8_t *s0 = sp + (cb - d0);
  const uint32_t sh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(s0) & 15u);
  const u32x4 *sa = reinterpret_cast<const u32x4 *>(s0 - sh);
  u32x4 *da = reinterpret_cast<u32x4 *>(cb);
  for (uint64_t k0 = 0; k0 < nch; k0 += static_cast<uint64_t>(kWave) * kU) {
    u32x4 v[kU + 1];
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) { // clamped at nch: sa[nch] is inside the read allowance
      const uint64_t k = k0 + static_cast<uint64_t>(u) * kWave + lane;
      v[u] = sa[k < nch ? k : nch];
    }
    const uint64_t kn = k0 + static_cast<uint64_t>(kU) * kWave;
    v[kU] = sa[kn < nch ? kn : nch];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
      u32x4 nx;
      nx.x = __shfl_down(v[u].x, 1u, kWave);
      nx.y = __shfl_down(v[u].y, 1u, kWave);
      nx.z = __shfl_down(v[u].z, 1u, kWave);
      nx.w = __shfl_down(v[u].w, 1u, kWave);
      u32x4 nl;
      if (u + 1 < kU) {
        nl.x = __shfl(v[u + 1].x, 0, kWave);
        nl.y = __shfl(v[u + 1].y, 0, kWave);
        nl.z = __shfl(v[u + 1].z, 0, kWave);
        nl.w = __shfl(v[u + 1].w, 0, kWave);
      } else {
        nl = v[kU];
      }
      if (lane == kWave - 1) nx = nl;
      const uint64_t k = k0 + static_cast<uint64_t>(u) * kWave + lane;
      if (k < nch) __builtin_nontemporal_store(funnel16(v[u], nx, sh), da + k);
    }
  }
  for (uintptr_t x = d0 + lane; x < cb; x += kWave) dp[x - d0] = sp[x - d0];
  for (uintptr_t x = ce + lane; x < d1; x += kWave) dp[x - d0] = sp[x - d0];
}

// A compaction block past the LDS slot of the enc_lds_kernel<1> wave that met
// it: entries one after another, each copied by the 64 lanes.
template <uint32_t kSpanU = kWaveSpanUnroll>
__device__ bool enc_emit_block_entries_wave(const EncArgs &a, uint64_t b) {
  const uint32_t lane = lane_id();
  const uint64_t f0 = a.blk_first[b], f1 = a.blk_first[b + 1];
  const uint64_t n = f1 - f0;
  const uint64_t P0 = a.P[f0];
  const uint64_t D = a.P[f1] - P0;
  if (a.guard) { // every entry checked before the first byte goes out
    bool bad = !enc1_block_ok(a, a.out_blk_off[b], a.out_blk_len[b], n) || a.out_blk_len[b] != D + 16 * n + 16;
    for (uint64_t r = f0 + lane; r < f1 && !bad; r += kWave)
      bad = !enc1_entry_ok(a, a.P[r] - P0, a.P[r + 1] - a.P[r], a.in.key_len[r], a.in.key_off[r], D);
    if (__any(bad)) {
      if (lane == 0) atomicOr(a.guard, kGuardEntry);
      return false;
    }
  }
  uint8_t *blk = a.dst + a.out_blk_off[b];
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t r = f0 + i;
    const uint64_t o = a.P[r] - P0, sz = a.P[r + 1] - a.P[r];
    copy_span_wave<kSpanU>(blk + o, a.key_src + a.in.key_off[r] - 5, sz - 8);
    if (lane < 8) blk[o + sz - 8 + lane] = static_cast<uint8_t>(a.in.txn[r] >> (8 * lane));
  }
  for (uint64_t i = lane; i < n; i += kWave) {
    const uint64_t st = a.P[f0 + i] - P0, sz = a.P[f0 + i + 1] - a.P[f0 + i];
    uint8_t *q = blk + D + 16 * i;
    for (int j = 0; j < 8; j++) {
      q[j] = static_cast<uint8_t>(st >> (8 * j));
      q[8 + j] = static_cast<uint8_t>(sz >> (8 * j));
    }
  }
  if (lane == 0) {
    uint8_t *q = blk + D + 16 * n;
    for (int j = 0; j < 8; j++) {
      q[j] = static_cast<uint8_t>(n >> (8 * j));
      q[8 + j] = static_cast<uint8_t>(D >> (8 * j));
    }
  }
  return true;
}


// One lane copies len bytes from global src to LDS dst, both at arbitrary
// alignment: head bytes until dst is 4-aligned, then one aligned source dword
// per destination dword through a funnel shift (the source / destination byte
// skew is constant along a span), then tail bytes.
__device__ __forceinline__ void lane_copy(uint8_t *dst, const uint8_t *src, uint32_t len) {
  uint32_t i = 0;
  uint32_t head = (4u - static_cast<uint32_t>(reinterpret_cast<uintptr_t>(dst) & 3u)) & 3u;
  head = head < len ? head : len;
  for (; i < head; i++) dst[i] = src[i];
  const uint32_t nw = (len - i) >> 2;
  if (nw) {
    uint32_t sh;
    const uint32_t *w = align4_down(src + i, sh);
    uint32_t *d = reinterpret_cast<uint32_t *>(dst + i);
    if (sh == 0) {
      for (uint32_t k = 0; k < nw; k++) d[k] = w[k];
    } else {
      uint32_t lo = w[0];
      for (uint32_t k = 0; k < nw; k++) {
        const uint32_t hi = w[k + 1];
        d[k] = __builtin_amdgcn_alignbyte(hi, lo, sh);
        lo = hi;
      }
    }
    i += 4 * nw;
  }
  for (; i < len; i++) dst[i] = src[i];
}

// Small-block encode: one wave per block, the block is assembled in an LDS
// image then written with 16 B stores (as rt_kernel).  Lane per record: its
// header fields, key and value bytes (lane_copy), txn and offset entry; lane 0
// the extra.  When the records were decoded from blocks held in key_src
// (a.entries_in_src, the compaction path) each record's whole entry is one
// contiguous source range at key_off - 5 and is copied as one span (txn then
// rewritten from the record: the compat reader may have changed it).
constexpr uint32_t kEncSlotWaves = kEncWaves;

// Four destination dwords of one aligned 16 B source chunk: source bytes
// r0 + 4j .. r0 + 4j + 3 of (v, nxt) go to the LDS dword at y + 4j when that
// dword lies inside [lo, hi) (the entry's image bytes).
__device__ __forceinline__ void emit_chunk(uint8_t *img, u32x4 v, uint32_t nxt, uint32_t r0, int32_t y,
                                           int32_t lo, int32_t hi) {
  const uint32_t w[5] = {v.x, v.y, v.z, v.w, nxt};
#pragma unroll
  for (uint32_t j = 0; j < 4; j++) {
    const int32_t yy = y + 4 * static_cast<int32_t>(j);
    if (yy >= lo && yy + 4 <= hi)
      *reinterpret_cast<uint32_t *>(img + yy) = __builtin_amdgcn_alignbyte(w[j + 1], w[j], r0);
  }
}

// Compaction encode (records decoded from blocks held in key_src): every
// surviving entry is already its own encoding in its input block, so the block
// image is assembled by copying whole entries.  16 lanes per entry, each loads
// one ALIGNED 16 B source chunk (one dwordx4 per lane instead of five dword
// loads) and funnel-shifts it, with the first dword of its right neighbour's
// chunk, into the dword-aligned LDS image (aligned stores: unaligned dword
// stores of the source dwords measured 501 -> 679 us at config 3); kCopyQ
// entry quads are loaded before any is written so a lane has kCopyQ wide
// loads in flight.  Dwords that straddle an entry's ends are left to the
// record pass that follows:
// lane per record writes type + key length (the first 5 bytes), the txn (the
// last 8; the compat reader may have changed it) and the offset entry.
template <uint32_t kCopyQ>
__device__ __forceinline__ bool enc_copy_entries(const EncArgs &a, uint8_t *img, uint32_t pad, uint64_t f0,
                                                 uint32_t n, uint64_t P0, uint32_t D, uint64_t b) {
  const uint32_t lane = lane_id();
  const uint32_t g = lane & 15u, sub = lane >> 4;
  uint64_t tmin = ~0ull, tmax = 0; // the block's min / max txn (table footer, table_builder.cc:47-49)
  uint64_t kfirst = 0, klast = 0;  // key offset | key length << 40 of the first / last entry (EncArgs::bmeta)
  for (uint32_t c0 = 0; c0 < n; c0 += kWave) {
    const uint32_t nc = n - c0 < kWave ? n - c0 : kWave;
    uint32_t my_o = 0, my_sz = 0, my_kl = 0, my_ty = 0;
    uint64_t my_ko = 0, my_tx = 0;
    if (lane < nc) {
      const uint64_t r = f0 + c0 + lane;
      const uint64_t pr = a.P[r];
      my_o = static_cast<uint32_t>(pr - P0);
      my_sz = static_cast<uint32_t>(a.P[r + 1] - pr);
      my_ko = a.in.key_off[r];
      my_tx = a.in.txn[r];
      my_kl = a.in.key_len[r];
      my_ty = a.in.type[r];
    }
    if (__any(lane < nc && !enc1_entry_ok(a, my_o, my_sz, my_kl, my_ko, D))) { // the block is not written
      if (lane == 0) atomicOr(a.guard, kGuardEntry);
      return false;
    }
    for (uint32_t p0 = 0; p0 < nc; p0 += 4 * kCopyQ) {
      u32x4 v[kCopyQ];
      uint32_t r0_[kCopyQ], nch_[kCopyQ];
      int32_t y_[kCopyQ], lo_[kCopyQ], hi_[kCopyQ];
      const uint8_t *A_[kCopyQ];
#pragma unroll
      for (uint32_t q = 0; q < kCopyQ; q++) {
        const uint32_t i = p0 + 4 * q + sub;
        const int sl = static_cast<int>(i & 63u);
        const uint32_t o = __shfl(my_o, sl, kWave), sz = __shfl(my_sz, sl, kWave);
        const uint32_t klo = __shfl(static_cast<uint32_t>(my_ko), sl, kWave);
        const uint32_t khi = __shfl(static_cast<uint32_t>(my_ko >> 32), sl, kWave);
        const uint8_t *sp = a.key_src + ((static_cast<uint64_t>(khi) << 32) | klo) - 5;
        const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(sp) & 15u);
        const uint8_t *A = sp - mis;
        const uint32_t nch = i < nc ? (mis + sz + 15u) >> 4 : 0u;
        const uint32_t ds = pad + o;
        v[q] = g < nch ? *reinterpret_cast<const u32x4 *>(A + 16 * g) : u32x4{0u, 0u, 0u, 0u};
        r0_[q] = (mis - ds) & 3u;
        y_[q] = static_cast<int32_t>(ds) - static_cast<int32_t>(mis) + static_cast<int32_t>(r0_[q]);
        lo_[q] = static_cast<int32_t>(ds);
        hi_[q] = static_cast<int32_t>(ds + sz);
        nch_[q] = nch;
        A_[q] = A;
      }
#pragma unroll
      for (uint32_t q = 0; q < kCopyQ; q++) {
        const uint32_t nxt = __shfl_down(v[q].x, 1u, 16);
        if (g < 15u && g < nch_[q]) emit_chunk(img, v[q], nxt, r0_[q], y_[q] + 16 * static_cast<int32_t>(g), lo_[q], hi_[q]);
        // entries longer than 15 chunks (~230 B): further rounds of 15 chunks
        for (uint32_t c = 15u + g; c - g < nch_[q]; c += 15u) {
          const u32x4 w = c < nch_[q] ? *reinterpret_cast<const u32x4 *>(A_[q] + 16 * c) : u32x4{0u, 0u, 0u, 0u};
          const uint32_t nx = __shfl_down(w.x, 1u, 16);
          if (g < 15u && c < nch_[q]) emit_chunk(img, w, nx, r0_[q], y_[q] + 16 * static_cast<int32_t>(c), lo_[q], hi_[q]);
        }
      }
    }
    wave_lds_sync();
    if (lane < nc) { // type + key length (the first 5 bytes), the txn (the last 8), the offset entry
      uint8_t *e = img + pad + my_o;
      e[0] = static_cast<uint8_t>(my_ty);
      lds_st_u32u(e, 1, my_kl);
      lds_st_u64u(e, my_sz - 8, my_tx);
      lds_st_u64u(img, pad + D + 16 * (c0 + lane), my_o);
      lds_st_u64u(img, pad + D + 16 * (c0 + lane) + 8, my_sz);
      tmin = my_tx < tmin ? my_tx : tmin;
      tmax = my_tx > tmax ? my_tx : tmax;
    }
    if (a.bmeta) {
      if (c0 == 0) kfirst = readlane_u64(my_ko, 0) | static_cast<uint64_t>(__shfl(my_kl, 0, kWave)) << 40;
      klast = readlane_u64(my_ko, nc - 1) | static_cast<uint64_t>(__shfl(my_kl, static_cast<int>(nc - 1), kWave)) << 40;
    }
  }
  if (a.bmeta) {
    for (uint32_t d = kWave / 2; d > 0; d >>= 1) {
      const uint64_t x = __shfl_xor(tmin, d, kWave), y = __shfl_xor(tmax, d, kWave);
      tmin = x < tmin ? x : tmin;
      tmax = y > tmax ? y : tmax;
    }
    if (lane < 4) // min, max, first / last key (offset | length << 40): one store
      a.bmeta[4 * b + lane] = lane == 0 ? tmin : (lane == 1 ? tmax : (lane == 2 ? kfirst : klast));
  }
  return true;
}

// Chunk c of a span: the 16 ALIGNED source bytes v hold the span's bytes from
// offset 16 c - mis on, so source dword j belongs at image position y + 4 j
// (y = span image position - mis + 16 c: any alignment, one unaligned
// ds_write_b32 per dword -- gfx950 runs LDS in unaligned mode, see
// sstc_device.h).  Every dword that meets [lo, hi) is stored whole, the others
// go to a per-lane sink word (no branches): a dword at an end of the span also
// overwrites up to 3 bytes beyond it, which always belong to the entry's own
// header fields (klen before a key, vlen after it or before a value, txn after
// the last field: block_builder.cc:36-77) -- the record pass that follows
// rewrites every header field, so it must run after the spans.  (Replaced a
// funnel shift of every dword with its neighbour lane's first dword.)
__device__ __forceinline__ void emit_chunk_ua(uint8_t *img, uint32_t *dummy, u32x4 v, int32_t y, int32_t lo,
                                              int32_t hi) {
  // dword j at y + 4 j meets [lo, hi) iff 0 <= y + 4 j - lo + 3 < hi - lo + 3 (one unsigned compare)
  const uint32_t t = static_cast<uint32_t>(y - lo + 3), span = static_cast<uint32_t>(hi - lo + 3);
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (uint32_t j = 0; j < 4; j++) {
    uint8_t *p = t + 4 * j < span ? img + y + 4 * static_cast<int32_t>(j) : reinterpret_cast<uint8_t *>(dummy);
    __builtin_memcpy(p, &w[j], 4);
  }
}

// One pass of span copies into a block image (enc_copy_split).  Owner lane
// i < nspan holds span i = (offset into `base`, length, image position).
// Spans are copied by groups of G lanes, 64 / G spans per wave instruction:
// lane g of a group loads the ALIGNED 16 B source chunk g (chunks g + G,
// g + 2G, ... in further rounds, only when some span needs them) and stores its
// dwords at their image positions (emit_chunk_ua), so the loads are 16 B per
// lane and coalesced per span.  kQ span groups are loaded before any is stored.
template <uint32_t G, uint32_t kQ>
__device__ __forceinline__ void copy_spans(const uint8_t *base, uint8_t *img, uint32_t *dummy, uint32_t nspan,
                                           uint64_t my_off, uint32_t my_len, uint32_t my_ds, const u32x4 *safe,
                                           u32x4 *tbl) {
  constexpr uint32_t kS = kWave / G;
  const uint32_t lane = lane_id();
  const uint32_t g = lane % G, sub = lane / G;
  const uintptr_t my_addr = reinterpret_cast<uintptr_t>(base + my_off);
  const uint32_t my_nch = my_len ? ((static_cast<uint32_t>(my_addr & 15u) + my_len + 15u) >> 4) : 0u;
  const bool longs = __any(my_nch > G); // wave-uniform
  const int32_t no = -(1 << 30);
  // the owners' span tuples in the wave's LDS table: one 16 B broadcast read
  // per span group instead of four shuffles (config-2 encode leg -1 %,
  // profiles/r02_ab/encode_ab.md)
  tbl[lane] = u32x4{static_cast<uint32_t>(my_off), static_cast<uint32_t>(my_off >> 32), my_len, my_ds};
  wave_lds_sync();
  for (uint32_t p0 = 0; p0 < nspan; p0 += kS * kQ) {
    u32x4 v[kQ];
    const uint8_t *sp_[kQ];
    uint32_t len_[kQ], ds_[kQ];
#pragma unroll
    for (uint32_t q = 0; q < kQ; q++) {
      const uint32_t i = p0 + q * kS + sub;
      const int sl = static_cast<int>(i & 63u);
      const u32x4 t = tbl[sl];
      const uint32_t olo = t.x, ohi = t.y;
      len_[q] = t.z; // 0 for owners >= nspan
      ds_[q] = t.w;
      sp_[q] = base + ((static_cast<uint64_t>(ohi) << 32) | olo);
      const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(sp_[q]) & 15u);
      const uint32_t nch = len_[q] ? (mis + len_[q] + 15u) >> 4 : 0u;
      v[q] = *(g < nch ? reinterpret_cast<const u32x4 *>(sp_[q] - mis + 16 * g) : safe);
    }
#pragma unroll
    for (uint32_t q = 0; q < kQ; q++) {
      const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(sp_[q]) & 15u);
      const uint32_t len = len_[q], ds = ds_[q];
      const uint32_t nch = len ? (mis + len + 15u) >> 4 : 0u;
      const uint8_t *A = sp_[q] - mis;
      const int32_t y = static_cast<int32_t>(ds) - static_cast<int32_t>(mis);
      const int32_t lo = static_cast<int32_t>(ds), hi = static_cast<int32_t>(ds + len);
      emit_chunk_ua(img, dummy, v[q], y + 16 * static_cast<int32_t>(g), g < nch ? lo : no, g < nch ? hi : no);
      if (longs) {
        for (uint32_t c = g + G; c - g < nch; c += G) {
          const u32x4 w = c < nch ? *reinterpret_cast<const u32x4 *>(A + 16 * c) : u32x4{0u, 0u, 0u, 0u};
          if (c < nch) emit_chunk_ua(img, dummy, w, y + 16 * static_cast<int32_t>(c), lo, hi);
        }
      }
    }
  }
}

// Keys and values of up to 32 records with every source load of the round in
// flight together: the key spans (2-lane groups, one load per lane) and the
// value spans (8-lane groups, four loads per lane) are issued before any is
// stored, so a block of <= 32 records waits on one HBM round trip for its
// entry bytes instead of three (keys, then two rounds of values).  The span
// tuples go through the wave's one LDS table: key tuples, read, then value
// tuples (LDS operations of a wave complete in order).  Spans longer than the
// group (keys > 2 chunks, values > 8) finish in a loop, as in copy_spans.
__device__ __forceinline__ void copy_kv_spans(const EncArgs &a, uint8_t *img, uint32_t *dummy, uint32_t p0,
                                              uint64_t ko, uint32_t kl, uint32_t dsk, uint64_t vo, uint32_t vl,
                                              uint32_t dsv, const u32x4 *safe, u32x4 *tbl) {
  constexpr uint32_t GK = 2, GV = 8, kQV = 4;
  const uint32_t lane = lane_id();
  const int32_t no = -(1 << 30);
  const uint32_t gk = lane % GK, gv = lane % GV;
  const uint32_t kbase = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(a.key_src));
  const uint32_t vbase = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(a.val_src));
  const bool longk = __any(kl && (((kbase + static_cast<uint32_t>(ko)) & 15u) + kl + 15u) >> 4 > GK);
  const bool longv = __any(vl && (((vbase + static_cast<uint32_t>(vo)) & 15u) + vl + 15u) >> 4 > GV);
  const uint32_t kown = (p0 + lane / GK) & 63u;
  // keys: record p0 + lane / 2 (its tuple, then the value tuples, through the one table)
  tbl[lane] = u32x4{static_cast<uint32_t>(ko), static_cast<uint32_t>(ko >> 32), kl, dsk};
  wave_lds_sync();
  const u32x4 tk = tbl[kown];
  const uint32_t misk = (kbase + tk.x) & 15u;
  const uint32_t nchk = tk.z ? (misk + tk.z + 15u) >> 4 : 0u;
  const u32x4 vk = *(gk < nchk ? reinterpret_cast<const u32x4 *>(
                                     a.key_src + ((static_cast<uint64_t>(tk.y) << 32) | tk.x) - misk + 16 * gk)
                               : safe);
  const uint32_t dk = tk.w, lk = tk.z;
  wave_lds_sync();
  tbl[lane] = u32x4{static_cast<uint32_t>(vo), static_cast<uint32_t>(vo >> 32), vl, dsv};
  wave_lds_sync();
  u32x4 vv[kQV];
#pragma unroll
  for (uint32_t q = 0; q < kQV; q++) {
    const u32x4 t = tbl[(p0 + q * (kWave / GV) + lane / GV) & 63u];
    const uint32_t mis = (vbase + t.x) & 15u;
    const uint32_t nch = t.z ? (mis + t.z + 15u) >> 4 : 0u;
    vv[q] = *(gv < nch ? reinterpret_cast<const u32x4 *>(a.val_src + ((static_cast<uint64_t>(t.y) << 32) | t.x) -
                                                         mis + 16 * gv)
                       : safe);
  }
  __builtin_amdgcn_sched_barrier(0); // every load above is issued before the stores below
  { // key stores
    const int32_t y = static_cast<int32_t>(dk) - static_cast<int32_t>(misk);
    const int32_t lo = static_cast<int32_t>(dk), hi = static_cast<int32_t>(dk + lk);
    emit_chunk_ua(img, dummy, vk, y + 16 * static_cast<int32_t>(gk), gk < nchk ? lo : no, gk < nchk ? hi : no);
    if (longk) { // rare: the owner's key offset by shuffle (the table holds the value tuples now)
      const uint64_t kok = __shfl(ko, static_cast<int>(kown), kWave);
      const uint8_t *A = a.key_src + kok - misk;
      for (uint32_t c = gk + GK; c - gk < nchk; c += GK) {
        const u32x4 w = c < nchk ? *reinterpret_cast<const u32x4 *>(A + 16 * c) : u32x4{0u, 0u, 0u, 0u};
        if (c < nchk) emit_chunk_ua(img, dummy, w, y + 16 * static_cast<int32_t>(c), lo, hi);
      }
    }
  }
#pragma unroll
  for (uint32_t q = 0; q < kQV; q++) { // value stores (tuples re-read: fewer live registers)
    const u32x4 t = tbl[(p0 + q * (kWave / GV) + lane / GV) & 63u];
    const uint32_t mis = (vbase + t.x) & 15u, len = t.z, ds = t.w;
    const uint32_t nch = len ? (mis + len + 15u) >> 4 : 0u;
    const int32_t y = static_cast<int32_t>(ds) - static_cast<int32_t>(mis);
    const int32_t lo = static_cast<int32_t>(ds), hi = static_cast<int32_t>(ds + len);
    emit_chunk_ua(img, dummy, vv[q], y + 16 * static_cast<int32_t>(gv), gv < nch ? lo : no, gv < nch ? hi : no);
    if (longv) {
      const uint8_t *A = a.val_src + ((static_cast<uint64_t>(t.y) << 32) | t.x) - mis;
      for (uint32_t c = gv + GV; c - gv < nch; c += GV) {
        const u32x4 w = c < nch ? *reinterpret_cast<const u32x4 *>(A + 16 * c) : u32x4{0u, 0u, 0u, 0u};
        if (c < nch) emit_chunk_ua(img, dummy, w, y + 16 * static_cast<int32_t>(c), lo, hi);
      }
    }
  }
}

constexpr bool kFusedKV = true;

template <uint32_t GK, uint32_t GV, uint32_t kQ>
__device__ __forceinline__ void enc_copy_split(const EncArgs &a, uint8_t *img, uint32_t *dummy, uint32_t pad,
                                               uint64_t f0, uint32_t n, uint64_t P0, uint32_t D, u32x4 *tbl) {
  const uint32_t lane = lane_id();
  uint8_t *im = img + pad;
  const u32x4 *safe = reinterpret_cast<const u32x4 *>(a.P); // a valid address for masked-off loads
  uint32_t carry = 0; // entry bytes of the rounds before
  for (uint32_t c0 = 0; c0 < n; c0 += kWave) {
    const uint32_t nc = n - c0 < kWave ? n - c0 : kWave;
    const uint64_t r = f0 + c0 + (lane < nc ? lane : 0u);
    const bool on = lane < nc;
    const uint32_t kl = a.in.key_len[r], vl = a.in.val_len[r], ty = a.in.type[r];
    // entry offsets by a wave scan of the entry sizes (no P pass over HBM)
    const uint32_t sz = on ? static_cast<uint32_t>(entry_size(kl, vl)) : 0u;
    const uint32_t inc = wave_incl_scan_u32(sz);
    const uint32_t o = carry + inc - sz;
    carry += __shfl(inc, kWave - 1, kWave);
    const uint64_t ko = a.in.key_off[r], vo = a.in.val_off[r], tx = a.in.txn[r];
    const uint32_t vlen = on && vl != kNoValue ? vl : 0u;
    if (kFusedKV) { // every load of a 32-record sub-round in flight at once
      for (uint32_t p0 = 0; p0 < nc; p0 += 32)
        copy_kv_spans(a, img, dummy, p0, on ? ko : 0ull, on ? kl : 0u, pad + o + 5, vlen ? vo : 0ull, vlen,
                      pad + o + 9 + kl, safe, tbl);
    } else {
      copy_spans<GK, kQ>(a.key_src, img, dummy, nc, ko, on ? kl : 0u, pad + o + 5, safe, tbl);
      copy_spans<GV, kQ>(a.val_src, img, dummy, nc, vlen ? vo : 0ull, vlen, pad + o + 9 + kl, safe, tbl);
    }
    if (on) { // header fields, txn, offset entry (after both span passes)
      im[o] = static_cast<uint8_t>(ty);
      lds_st_u32u(im, o + 1, kl);
      lds_st_u32u(vl != kNoValue ? im : reinterpret_cast<uint8_t *>(dummy), vl != kNoValue ? o + 5 + kl : 0u, vl);
      lds_st_u64u(im, o + sz - 8, tx);
      lds_st_u64u(im, D + 16 * (c0 + lane), o);
      lds_st_u64u(im, D + 16 * (c0 + lane) + 8, sz);
    }
  }
}

// mode 0, a block past its LDS slot: its wave writes the block-relative
// entry offsets P[f0 .. f1) (a workspace no other block touches) for
// enc_emit_block, which reads them back from other lanes
__device__ void enc_wave_offsets(const EncArgs &a, uint64_t b) {
  uint64_t *P = const_cast<uint64_t *>(a.P);
  const uint32_t lane = lane_id();
  const uint64_t f0 = a.blk_first[b], n = a.blk_first[b + 1] - f0;
  uint64_t carry = 0;
  for (uint64_t c0 = 0; c0 < n; c0 += kWave) {
    const bool on = c0 + lane < n;
    const uint64_t r = f0 + c0 + (on ? lane : 0u);
    const uint64_t sz = on ? entry_size(a.in.key_len[r], a.in.val_len[r]) : 0ull;
    const uint64_t inc = wave_incl_scan_u64(sz);
    if (on) P[r] = carry + inc - sz;
    carry += __shfl(inc, kWave - 1, kWave);
  }
  __threadfence_block(); // the stores complete before any lane of the wave reads them (same CU)
}

// kMode 0: two arenas (key spans in groups of GK lanes, then value spans in
// groups of GV, kQ span groups in flight); 1: whole-entry copy (compaction),
// kQ entry quads in flight per lane for the blocks that fit the LDS slot and
// kU 16 B chunks per lane for the ones past it.  Mode 1 comes in two builds
// (launch_enc_emit picks by EncArgs::large_blocks): kQ = kU = 2 needs 59 VGPRs,
// 8 waves / SIMD (config 3 encode 525 -> 512 us, config 4 863 -> 844 us), but
// copies large blocks slower (config 5 231 -> 255 us); kQ = kU = 4 needs 79,
// 6 waves (profiles/r05/encode_ab.md)
// EncArgs::xcd == 2 (the compaction job, whose grid is a bound): 16
// consecutive workgroups per XCD chunk.  Neighbouring output blocks copy
// neighbouring entries of the same inputs (config 4: 1-entry runs from 128
// inputs), so their source lines are fetched once per L2: config 4 encode
// FETCH 3.89 -> 2.33 GB, 845 -> 832 us (profiles/r05/encode_xcd.md)
#ifndef SSTC_ENC_XCD_CHUNK
#define SSTC_ENC_XCD_CHUNK 16
#endif
constexpr uint32_t kEncXcdChunk = SSTC_ENC_XCD_CHUNK;

template <uint32_t kMode, uint32_t GK = 2, uint32_t GV = 8, uint32_t kQ = 2, uint32_t kU = kWaveSpanUnroll>
__global__ __launch_bounds__(kEncWaves *kWave) void enc_lds_kernel(EncArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kEncSlotWaves * kEncSlot];
  __shared__ uint32_t s_dummy[kMode == 0 ? kEncWaves * kWave : 1]; // per-lane sink of clipped stores
  __shared__ u32x4 s_tbl[kMode == 0 ? kEncWaves * kWave : 1]; // span tuples (copy_spans)
  const uint32_t wave = uniform(threadIdx.x / kWave);
  const uint32_t lane = lane_id();
  const uint32_t wg = a.xcd == 2   ? xcd_chunk_block(blockIdx.x, gridDim.x, kEncXcdChunk)
                      : a.xcd == 1 ? xcd_logical_block(blockIdx.x, gridDim.x)
                                   : blockIdx.x;
  const uint64_t b = static_cast<uint64_t>(wg) * kEncWaves + wave;
  if (b >= a.nblocks) return;
  uint8_t *img = lds + wave * kEncSlot;
  uint64_t bo, L64, f0_v, f1_v;
  if constexpr (kMode == 0) {
    // every load that depends on b only is issued before any of them is
    // waited for (the compiler sank the record range behind the large-block
    // branch: a dependent round trip of its own; config-2 encode leg -1.5 %)
    const uint64_t bo_v = a.out_blk_off[b], L_v = a.out_blk_len[b];
    f0_v = a.blk_first[b];
    f1_v = a.blk_first[b + 1];
    __builtin_amdgcn_sched_barrier(0); // all issued before the first use waits
    // the all-ones test is never true for a real block (a 2^64 - 1 byte
    // length); it keeps the four loads ahead of the branch
    if ((bo_v & L_v & f0_v & f1_v) == ~0ull) return;
    bo = uniform64(bo_v);
    L64 = uniform64(L_v);
  } else {
    // (the same hoisting measured 2-3 % slower for the compaction encode,
    // profiles/r03_ab/encode_prologue.md)
    const uint64_t nbl = *a.nb_dev; // the count on the device, nblocks its bound
    if (b >= nbl || nbl > a.nblocks || a.over()) return;
    bo = uniform64(a.out_blk_off[b]);
    L64 = uniform64(a.out_blk_len[b]);
  }
  const uint32_t pad = static_cast<uint32_t>(bo & 15u);
  if (pad + L64 + 16 > kEncSlot) { // large block
    { // this wave writes it straight to HBM
      if constexpr (kMode == 0) {
        enc_wave_offsets(a, b);
        enc_emit_block<kWave>(a, b, img, lane); // its LDS image holds the lanes' chunk slots
      } else {
        if (!enc_emit_block_entries_wave<kU>(a, b)) return;
        if (a.bmeta) { // the block's min / max txn (table footer), reduced by the wave
          const uint64_t f0 = a.blk_first[b], f1 = a.blk_first[b + 1];
          uint64_t mn = ~0ull, mx = 0;
          for (uint64_t r = f0 + lane; r < f1; r += kWave) {
            const uint64_t x = a.in.txn[r];
            mn = x < mn ? x : mn;
            mx = x > mx ? x : mx;
          }
          for (uint32_t d = kWave / 2; d > 0; d >>= 1) {
            const uint64_t x = __shfl_xor(mn, d, kWave), y = __shfl_xor(mx, d, kWave);
            mn = x < mn ? x : mn;
            mx = y > mx ? y : mx;
          }
          if (lane < 4) { // min, max, first / last key (offset | length << 40): one store
            const uint64_t r = lane < 2 ? 0 : (lane == 2 ? f0 : f1 - 1);
            const uint64_t k = lane < 2 ? 0 : a.in.key_off[r] | static_cast<uint64_t>(a.in.key_len[r]) << 40;
            a.bmeta[4 * b + lane] = lane == 0 ? mn : (lane == 1 ? mx : k);
          }
        }
      }
    }
    return;
  }
  const uint32_t L = static_cast<uint32_t>(L64);
  if constexpr (kMode == 1) {
    f0_v = a.blk_first[b];
    f1_v = a.blk_first[b + 1];
  }
  const uint64_t f0 = uniform64(f0_v);
  const uint32_t n = static_cast<uint32_t>(uniform64(f1_v) - f0);
  // L = D + 16 n + 16
  const uint32_t D = L - 16u * n - 16u;
  uint8_t *im = img + pad; // image byte 0 == block byte 0

  if constexpr (kMode == 1) {
    const uint64_t P0 = uniform64(a.P[f0]);
    if (!enc1_block_ok(a, bo, L64, n) || (a.guard && uniform64(a.P[f0 + n]) - P0 != D)) {
      if (lane == 0) atomicOr(a.guard, kGuardBlockRange);
      return;
    }
    if (!enc_copy_entries<kQ>(a, img, pad, f0, n, P0, D, b)) return;
  } else {
    // mode 0 scans its entry offsets in the wave
    enc_copy_split<GK, GV, kQ>(a, img, s_dummy + threadIdx.x, pad, f0, n, 0, D, s_tbl + wave * kWave);
  }
  if (lane == 0) {
    lds_st_u64u(im, D + 16 * n, n);
    lds_st_u64u(im, D + 16 * n + 8, D);
  }
  wave_lds_sync();
  store_window(img, a.dst + (bo - pad), (pad + L + 15u) >> 4, 0, pad, pad + L);
}

// ---------------------------------------------------------------------------
// Greedy segmentation (TableBuilder::AddEntry's flush rule, table_builder.cc:
// 57-59, and DoCompactJob's output split, compact.cc:290).
// J0[i] = one past the last record of a segment that starts at record i: the
// first e >= i with W(e + 1) >= W(i) + threshold, plus one, clamped to the end
// of i's output table; W(x) = Pw[x] + add * x.  The segments are the chain
// 0 -> J0[0] -> ...; J0 is nondecreasing.
//
// Many short segments (blocks): tiles of kChTile records.
//  A seg_walk_kernel: J0 of the tile by galloping in an LDS copy of W; a
//    segment that enters tile k starts in its entry window [c0, J0[c0 - 1]]
//    (J0 is monotone), and every window position walks the chain inside the
//    tile: entry -> (exit record, segments started in the tile).
//  B the window positions of all tiles are the nodes of a much smaller chain
//    (one node per tile it visits): node -> node of its exit, radix-8 pointer
//    jumping over nodes (log8 tiles levels) with segment counts.
//  C every visited tile learns its entry and the segments before it, then
//    seg_emit_kernel re-walks its part of the chain and writes the starts.
// Few long segments (output tables): seg_spec_kernel takes the hop from every
// predicted segment start in parallel (one wave per start), then
// seg_hops_kernel, one wave, follows the chain through those answers and hops
// on its own (windows around the predicted ends, a 512-ary search of W) from
// the first start that was not predicted.
// ---------------------------------------------------------------------------
constexpr uint32_t kChTile = 1024, kChThreads = 256, kChMargin = 256;
constexpr uint32_t kSegRadix = 8;
constexpr uint32_t kNoNode = 0xFFFFFFFFu;

// LDS slot of W(base + x): one pad word per 8 so that threads walking 8
// consecutive records each hit different banks
__device__ __forceinline__ uint32_t lw_slot(uint64_t x) { return static_cast<uint32_t>(x + (x >> 3)); }

struct SegW { // W(x) from an LDS window [base, base + n) or from HBM
  const uint64_t *Pw, *lw;
  uint64_t add, base, n;
  __device__ __forceinline__ uint64_t operator()(uint64_t x) const {
    return x - base < n ? lw[lw_slot(x - base)] : Pw[x] + add * x;
  }
};

// the first e in [i, lim - 1] with W(e + 1) >= W(i) + threshold, plus one; lim
// when the threshold is not reached before the clamp (the bisection then ends
// at lim - 1 by itself: W is monotone).  Every e < from (>= i) is known to
// fail: galloping starts there.
__device__ uint64_t seg_next_to(const SegW &W, uint64_t target, uint64_t lim, uint64_t from) {
  uint64_t lo = from, hi = lim - 1;
  for (uint64_t span = 1;; span <<= 1) {
    const uint64_t e = from + span - 1;
    if (e >= lim - 1) break;
    if (W(e + 1) >= target) {
      hi = e;
      break;
    }
    lo = e + 1;
  }
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (W(mid + 1) >= target) hi = mid;
    else lo = mid + 1;
  }
  return lo + 1;
}
__device__ __forceinline__ uint64_t seg_next_at(const SegW &W, uint64_t i, uint64_t lim, uint64_t threshold,
                                                uint64_t from) {
  return seg_next_to(W, W(i) + threshold, lim, from);
}

struct SegArgs {
  const uint64_t *Pw;
  uint64_t add, m, threshold;
  const uint64_t *ends, *nends; // optional clamp: ends[0..*nends], ends[*nends] = m; ends holds >= m + 1 words
  uint32_t *J0, *Fx, *Fc; // by record
  uint64_t *win;          // per tile: entry-window size (scanned into node bases)
  uint64_t *first, *d_count;
  uint64_t *zws;          // cleared here: the win scan's look-back status words
  uint64_t nz;
  uint32_t *tentry;       // cleared here: tiles + 1 entry counters
  const uint64_t *mp;     // optional: the record count on the device (m is then its bound)
  const uint64_t *skip;   // *skip != 0: the arithmetic chain held (seg_arith_*), nothing to do (null: run)
};

// table ends cached in LDS by seg_walk_kernel: ends[t0 - 1 + j], j < kEndCache
constexpr uint32_t kEndCache = 16;

__global__ __launch_bounds__(kChThreads) void seg_walk_kernel(SegArgs a) {
  constexpr uint32_t kLw = kChTile + kChMargin;
  __shared__ uint64_t lw[kLw + kLw / 8];
  __shared__ uint32_t jn[kChTile], jc[kChTile];
  __shared__ uint64_t s_wend, s_t0, s_e[kEndCache], s_ec;
  const uint32_t tid = threadIdx.x;
  const uint64_t c0 = static_cast<uint64_t>(blockIdx.x) * kChTile;
  if (a.skip && *a.skip) return;
  // the window's loads go out on the host bound a.m (Pw holds a.m + 1 words),
  // together with the device count's: one round trip instead of two
  constexpr uint32_t kFill = kLw / kChThreads;
  const uint64_t nlh = a.m + 1 - c0 < kLw ? a.m + 1 - c0 : kLw;
  uint64_t v[kFill];
#pragma unroll
  for (uint32_t r = 0; r < kFill; r++) {
    const uint32_t x = tid + r * kChThreads;
    v[r] = x < nlh ? a.Pw[c0 + x] : 0;
  }
  // in the same round trip: W(c0 - 1) for the entry window (thread 255), and
  // the table-end count with the first 64 ends (wave 0: the search below
  // starts from them when there are at most 63 ends, else it reloads)
  const uint64_t wprev = tid == kChThreads - 1 && c0 ? a.Pw[c0 - 1] + a.add * (c0 - 1) : 0;
  uint64_t ne_ld = 0, e_ld = 0;
  if (a.ends && tid < kWave) {
    ne_ld = *a.nends;
    e_ld = a.ends[tid < a.m ? tid : a.m];
  }
  const uint64_t m = a.mp ? *a.mp : a.m;
  if (tid == 0) {
    a.tentry[blockIdx.x] = 0;
    if (blockIdx.x == 0) a.tentry[gridDim.x] = 0;
    for (uint64_t z = blockIdx.x; z < a.nz; z += gridDim.x) a.zws[z] = 0;
  }
  if (c0 >= m) { // a tile past the device count (uniform): no window, no node
    if (tid == 0) a.win[blockIdx.x] = 0;
    return;
  }
  const uint64_t c1 = c0 + kChTile < m ? c0 + kChTile : m;
  const uint32_t len = static_cast<uint32_t>(c1 - c0);
  const uint64_t nl = m + 1 - c0 < kLw ? m + 1 - c0 : kLw;
  if (a.ends && tid < kWave) {
    // t0 = the first table end past the tile start (ends[0..ne] sorted, ends[ne]
    // = m > c0): a 64-ary search by wave 0, one round trip while ne < 64 (a
    // thread's binary search was log2(ne) dependent loads on every
    // workgroup's critical path); its last round leaves ends[t0 - 1 ..] in
    // the lanes, cached in LDS for the clamps below
    const uint32_t lane = tid;
    const uint64_t ne = ne_ld;
    uint64_t lo = 0, n = ne + 1, below = 0, e = 0; // answer in [lo, lo + n); ends[lo - 1] = below
    uint32_t f = 0;
    for (;;) {
      // step = ceil((n - 1) / 63) past one round: lane 63 probes lo + n - 1
      // (ends[lo + n - 1] > c0 is the invariant), so the ballot is never empty
      const uint64_t step = n <= kWave ? 1 : (n - 2) / (kWave - 1) + 1;
      const uint64_t off = static_cast<uint64_t>(lane) * step;
      const uint64_t x = step == 1 ? (lo + lane < ne ? lo + lane : ne) : lo + (off < n - 1 ? off : n - 1);
      if (lo == 0 && n <= kWave) // the first round of <= 64 ends: the loads above (x = min(lane, ne))
        e = lane <= ne ? e_ld : readlane_u64(e_ld, static_cast<uint32_t>(ne));
      else
        e = a.ends[x];
      const uint64_t gt = __ballot(e > c0); // a suffix of the lanes, lane min(n - 1, 63) at least
      // (never empty; a corrupt end list must not turn f into ~0 and send the
      // next round's loads out of range)
      f = gt ? static_cast<uint32_t>(__ffsll(static_cast<long long>(gt))) - 1u : kWave - 1;
      if (step == 1) break;
      if (f) below = readlane_u64(e, f - 1);
      const uint64_t nlo = f ? lo + static_cast<uint64_t>(f - 1) * step + 1 : lo;
      const uint64_t xf = lo + (static_cast<uint64_t>(f) * step < n - 1 ? static_cast<uint64_t>(f) * step : n - 1);
      n = xf - nlo + 1;
      lo = nlo;
    }
    const uint64_t t0 = lo + f;
    if (f) below = readlane_u64(e, f - 1);
    const int64_t j = static_cast<int64_t>(lo + lane) - static_cast<int64_t>(t0) + 1; // slot of ends[lo + lane]
    if (j >= 1 && j < static_cast<int64_t>(kEndCache) && lo + lane <= ne) s_e[j] = e;
    if (lane == 0) {
      s_e[0] = below; // ends[t0 - 1] (unused when t0 = 0)
      const uint64_t last = lo + kWave - 1 < ne ? lo + kWave - 1 : ne; // ends[t0 - 1 .. last] are cached
      const uint64_t nc = last + 2 - t0;
      s_ec = nc < kEndCache ? nc : kEndCache;
      s_t0 = t0;
    }
  }
#pragma unroll
  for (uint32_t r = 0; r < kFill; r++) {
    const uint32_t x = tid + r * kChThreads;
    if (x < nl) lw[lw_slot(x)] = v[r] + a.add * (c0 + x);
  }
  __syncthreads();
  const uint64_t t0 = a.ends ? s_t0 : 0, ec = a.ends ? s_ec : 0;
  auto end_at = [&](uint64_t t) -> uint64_t { // ends[t], t >= t0 - 1
    const uint64_t j = t + 1 - t0;
    return j < ec ? s_e[j] : a.ends[t];
  };
  const SegW W{a.Pw, lw, a.add, c0, nl};
  if (tid == kChThreads - 1) { // entry window end: J0 of the record before the tile
    const uint64_t i = c0 - 1;
    uint64_t lim = m;
    if (a.ends) // first end > c0 - 1: t0, or the one before it when it equals c0
      lim = t0 > 0 && end_at(t0 - 1) == c0 ? c0 : end_at(t0);
    s_wend = blockIdx.x ? seg_next_to(W, wprev + a.threshold, lim, i) : c0;
  }
  // J0 of kPer consecutive records per thread: gallop for the first, then from
  // the previous answer (J0 is monotone within an output table)
  constexpr uint32_t kPer = kChTile / kChThreads;
  uint64_t lim[kPer];
  {
    const uint64_t i0 = c0 + tid * kPer;
    uint64_t t = t0;
    uint64_t end = a.ends ? end_at(t) : m; // ends[ne] = m: the walks below stop at ne
#pragma unroll
    for (uint32_t r = 0; r < kPer; r++) {
      const uint64_t i = i0 + r;
      if (a.ends && i < m)
        while (end <= i) end = end_at(++t); // ends[ne] = m > i
      lim[r] = i < c1 ? end : 0;
    }
  }
  uint64_t e_prev = 0;
#pragma unroll
  for (uint32_t r = 0; r < kPer; r++) {
    const uint32_t p = tid * kPer + r;
    if (p >= len) break;
    const uint64_t i = c0 + p;
    const uint64_t j = seg_next_at(W, i, lim[r], a.threshold, r && e_prev > i ? e_prev : i);
    e_prev = j - 1;
    jn[p] = static_cast<uint32_t>(j);
    jc[p] = 1;
    a.J0[i] = static_cast<uint32_t>(j);
  }
  __syncthreads();
  const uint64_t wend = s_wend; // inclusive; >= c0
  const uint32_t nwin = static_cast<uint32_t>((wend < c1 - 1 ? wend : c1 - 1) - c0 + 1);
  // short chains (blocks of tens of records, estimated from the tile's first
  // segment): every window position walks its chain through the tile on its
  // own, no barrier per round (config 3: 65 -> 52 us, config 4: 94 -> 73 us);
  // a walk past kSerialWalk segments sends the whole tile to the pointer
  // jumping below, which long chains (large records) take from the start
  constexpr uint32_t kSerialWalk = 64;
  const uint32_t seg0 = jn[0] - static_cast<uint32_t>(c0); // >= 1
  if (len / seg0 <= kSerialWalk - kSerialWalk / 4) {
    bool long_chain = false;
    for (uint32_t p = tid; p < nwin; p += kChThreads) {
      uint32_t x = jn[p], cnt = 1;
      while (x < c1 && cnt <= kSerialWalk) {
        x = jn[x - static_cast<uint32_t>(c0)];
        cnt++;
      }
      if (x < c1) {
        long_chain = true;
      } else {
        a.Fx[c0 + p] = x;
        a.Fc[c0 + p] = cnt;
      }
    }
    if (!__syncthreads_or(long_chain)) {
      if (tid == 0) a.win[blockIdx.x] = nwin;
      return;
    }
  }
  // pointer jumping inside the tile: jn[p] -> first chain position >= c1
  // reached from p, jc[p] -> segments started on the way (p's included)
  for (;;) {
    uint32_t nx[kPer], nc[kPer];
    int moved = 0;
#pragma unroll
    for (uint32_t r = 0; r < kPer; r++) {
      const uint32_t p = tid + r * kChThreads;
      nx[r] = 0;
      nc[r] = 0;
      if (p < len) {
        nx[r] = jn[p];
        nc[r] = jc[p];
        if (nx[r] < c1) {
          const uint32_t q = nx[r] - static_cast<uint32_t>(c0);
          nc[r] += jc[q];
          nx[r] = jn[q];
          moved = 1;
        }
      }
    }
    if (!__syncthreads_or(moved)) break;
#pragma unroll
    for (uint32_t r = 0; r < kPer; r++) {
      const uint32_t p = tid + r * kChThreads;
      if (p < len) {
        jn[p] = nx[r];
        jc[p] = nc[r];
      }
    }
    __syncthreads();
  }
  for (uint32_t p = tid; p < nwin; p += kChThreads) {
    a.Fx[c0 + p] = jn[p];
    a.Fc[c0 + p] = jc[p];
  }
  if (tid == 0) a.win[blockIdx.x] = nwin;
}

struct NodeArgs {
  const uint32_t *Fx, *Fc;
  const uint64_t *base; // node base of every tile (exclusive scan of win), tiles + 1
  uint64_t m, tiles;
  uint32_t *Nx, *Nc, *Nt; // level 0: next node, segments, tile
  const uint64_t *mp;     // optional device record count
  const uint64_t *skip;   // as SegArgs::skip
};

__global__ void seg_node_kernel(NodeArgs a) {
  if (a.skip && *a.skip) return;
  const uint64_t k = blockIdx.x;
  const uint64_t b0 = a.base[k], nw = a.base[k + 1] - b0, c0 = k * kChTile;
  const uint64_t m = a.mp ? *a.mp : a.m;
  for (uint64_t o = threadIdx.x; o < nw; o += blockDim.x) {
    const uint64_t x = a.Fx[c0 + o];
    uint32_t nx = kNoNode;
    if (x < m) {
      const uint64_t t = x / kChTile;
      nx = static_cast<uint32_t>(a.base[t] + (x - t * kChTile));
    }
    a.Nx[b0 + o] = nx;
    a.Nc[b0 + o] = a.Fc[c0 + o];
    a.Nt[b0 + o] = static_cast<uint32_t>(k);
  }
}

// level k + 1 = 8 hops of level k (node count from the device)
__global__ void seg_npow_kernel(const uint32_t *Nx, const uint32_t *Nc, uint32_t *Nx1, uint32_t *Nc1,
                                const uint64_t *nnodes, const uint64_t *skip) {
  if (skip && *skip) return;
  const uint64_t n = *nnodes;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    uint32_t x = static_cast<uint32_t>(i), c = 0;
#pragma unroll
    for (uint32_t j = 0; j < kSegRadix; j++) {
      if (x == kNoNode) break;
      c += Nc[x];
      x = Nx[x];
    }
    Nx1[i] = x;
    Nc1[i] = c;
  }
}

// Visit h of the node chain from node 0: its node (tile, entry) and the
// segments before it; a visit past the chain's end meets kNoNode on its walk
// and leaves.  Thread 0 of workgroup 0 also walks the whole chain down the
// levels: the total segment count and first[total] = m.  (Round 4: one kernel
// with the depth walk instead of a one-thread launch before this one.)
__global__ void seg_nentry_kernel(const uint32_t *Nx, const uint32_t *Nc, const uint32_t *Nt, const uint64_t *base,
                                  uint32_t levels, uint64_t stride, uint64_t m, const uint64_t *mp,
                                  uint64_t tiles, uint32_t *tentry, uint32_t *tbefore, uint64_t *first,
                                  uint64_t *d_count, const uint64_t *skip) {
  if (skip && *skip) return;
  if (mp) m = *mp;
  const uint64_t h = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (h == 0) {
    if (m == 0) { // no records (an aborted compaction): no node, no segment
      *d_count = 0;
      first[0] = 0;
    } else {
      uint64_t pos = 0, tot = 0;
      for (int k = static_cast<int>(levels) - 1; k >= 0; k--) {
        const uint32_t *X = Nx + static_cast<uint64_t>(k) * stride, *C = Nc + static_cast<uint64_t>(k) * stride;
        for (uint32_t d = 1; d < kSegRadix; d++) {
          const uint32_t nx = X[pos];
          if (nx == kNoNode) break;
          tot += C[pos];
          pos = nx;
        }
      }
      tot += Nc[pos];
      *d_count = tot;
      first[tot] = m;
    }
  }
  if (m == 0 || h >= tiles) return; // (a tile is visited at most once)
  uint64_t pos = 0, before = 0, q = h;
  for (uint32_t k = 0; k < levels && q; k++, q /= kSegRadix) {
    const uint32_t *X = Nx + static_cast<uint64_t>(k) * stride, *C = Nc + static_cast<uint64_t>(k) * stride;
    for (uint32_t d = static_cast<uint32_t>(q % kSegRadix); d; d--) {
      const uint32_t nx = X[pos];
      if (nx == kNoNode) return; // past the chain's last visit
      before += C[pos];
      pos = nx;
    }
  }
  const uint32_t t = Nt[pos];
  tentry[t] = static_cast<uint32_t>(pos - base[t]) + 1; // 0 = not visited
  tbefore[t] = static_cast<uint32_t>(before);
}

// Block starts of a visited tile: the chain from its entry position, marked
// by doubling inside the tile (every marked position marks its 2^r-th
// successor, then the successor pointers double; a round that adds no mark
// leaves the marked set closed, i.e. complete), then numbered by a prefix
// count of the marks: O(log chain) barriers instead of a serial walk (a tile
// of 64 KiB values is a 2048-step chain).  Chains estimated at <= 128 steps
// (e.g. 4 KiB blocks of small records: ~73 per tile) are walked by one thread.
__global__ __launch_bounds__(kChThreads) void seg_emit_kernel(const uint32_t *J0, uint64_t m, const uint64_t *mp,
                                                              const uint32_t *tentry, const uint32_t *tbefore,
                                                              uint64_t *first, const uint64_t *skip) {
  if (skip && *skip) return;
  constexpr uint32_t kPer = kChTile / kChThreads;
  constexpr uint16_t kOut = 0xFFFF; // successor outside the tile
  constexpr uint32_t kSerialChain = 128;
  __shared__ uint16_t nx[kChTile];
  __shared__ uint8_t mk[kChTile];
  __shared__ uint32_t s_wsum[kChThreads / kWave];
  const uint64_t k = blockIdx.x;
  const uint64_t c0 = k * kChTile;
  const uint32_t tid = threadIdx.x;
  // the tile's J0 goes out on the host bound m (J0 holds m + 1 words) with the
  // entry and the device count: one round trip instead of three
  uint32_t v[kPer];
#pragma unroll
  for (uint32_t r = 0; r < kPer; r++) {
    const uint64_t x = c0 + tid + r * kChThreads;
    v[r] = J0[x < m ? x : m];
  }
  const uint32_t e = tentry[k];
  if (mp) m = *mp;
  if (!e) return; // a segment spans the whole tile (or the tile is past the device count)
  const uint64_t c1 = c0 + kChTile < m ? c0 + kChTile : m;
  const uint32_t len = static_cast<uint32_t>(c1 - c0);
  {
#pragma unroll
    for (uint32_t r = 0; r < kPer; r++) {
      const uint32_t p = tid + r * kChThreads;
      nx[p] = p < len && v[r] < c1 ? static_cast<uint16_t>(v[r] - c0) : kOut;
      mk[p] = p == e - 1;
    }
  }
  __syncthreads();
  { // short chain (estimated from its first segment): one thread walks it
    const uint32_t s0 = e - 1, q0 = nx[s0];
    const uint32_t seg = q0 == kOut ? len - s0 : q0 - s0;
    if ((len - s0) / seg <= kSerialChain) {
      if (tid == 0) {
        uint64_t b = tbefore[k];
        for (uint32_t pos = s0; pos != kOut;) {
          first[b++] = c0 + pos;
          pos = nx[pos];
        }
      }
      return;
    }
  }
  for (;;) {
    uint16_t nn[kPer];
    int added = 0;
#pragma unroll
    for (uint32_t r = 0; r < kPer; r++) {
      const uint32_t p = tid * kPer + r;
      const uint16_t q = nx[p];
      nn[r] = kOut;
      if (q != kOut) {
        if (mk[p] && !mk[q]) {
          mk[q] = 1;
          added = 1;
        }
        nn[r] = nx[q];
      }
    }
    if (!__syncthreads_or(added)) break;
#pragma unroll
    for (uint32_t r = 0; r < kPer; r++) nx[tid * kPer + r] = nn[r];
    __syncthreads();
  }
  // number the marks: kPer contiguous positions per thread, workgroup scan
  uint32_t cnt = 0;
#pragma unroll
  for (uint32_t r = 0; r < kPer; r++) cnt += mk[tid * kPer + r];
  const uint32_t incl = wave_incl_scan_u32(cnt);
  if (lane_id() == kWave - 1) s_wsum[tid / kWave] = incl;
  __syncthreads();
  uint32_t rank = incl - cnt;
  for (uint32_t w = 0; w < tid / kWave; w++) rank += s_wsum[w];
  const uint64_t b0 = tbefore[k];
#pragma unroll
  for (uint32_t r = 0; r < kPer; r++) {
    const uint32_t p = tid * kPer + r;
    if (mk[p]) first[b0 + rank++] = c0 + p;
  }
}

// few long segments: one wave follows the chain.  Each hop first probes
// kHopSpan consecutive records around pos + (previous segment length) --
// equal-sized tables end there: one coalesced round -- and falls back to a
// kHopSpan-ary search of W over the rest.  Wave-synchronous: a round is one
// batch of loads and ballots, no barrier.
constexpr uint32_t kHopProbe = 8;
constexpr uint64_t kHopSpan = static_cast<uint64_t>(kWave) * kHopProbe;

// number of x = x0 + j * step (j < kHopSpan, x <= x1) with W(x) < target
__device__ __forceinline__ uint64_t hop_below(const uint64_t *Pw, uint64_t add, uint64_t x0, uint64_t x1,
                                              uint64_t step, uint64_t target) {
  const uint32_t lane = lane_id();
  // clamped, unconditional loads: all kHopProbe in flight together (a load
  // under a branch is waited for before the branch joins)
  uint64_t w[kHopProbe];
#pragma unroll
  for (uint32_t r = 0; r < kHopProbe; r++) {
    const uint64_t x = x0 + (static_cast<uint64_t>(r) * kWave + lane) * step;
    const uint64_t xc = x <= x1 ? x : x1;
    w[r] = Pw[xc];
  }
  __builtin_amdgcn_sched_barrier(0); // keep the loads ahead of their uses
  bool b[kHopProbe];
#pragma unroll
  for (uint32_t r = 0; r < kHopProbe; r++) {
    const uint64_t x = x0 + (static_cast<uint64_t>(r) * kWave + lane) * step;
    b[r] = x <= x1 && w[r] + add * (x <= x1 ? x : x1) < target;
  }
  uint64_t nb = 0;
#pragma unroll
  for (uint32_t r = 0; r < kHopProbe; r++) nb += __popcll(__ballot(b[r]));
  return nb;
}

// exact hop from pos: the first x in [pos + 1, m] with W(x) >= target
// (W(m) >= target), probing around pos + glen first when glen is known
__device__ uint64_t hop_exact(const uint64_t *Pw, uint64_t add, uint64_t m, uint64_t pos, uint64_t glen,
                              uint64_t target) {
  uint64_t lo = pos + 1, hi = m;
  if (glen) {
    const uint64_t g0 = pos + glen > pos + 1 + kHopSpan / 2 ? pos + glen - kHopSpan / 2 : pos + 1;
    const uint64_t g1 = g0 + kHopSpan - 1 < m ? g0 + kHopSpan - 1 : m;
    const uint64_t nb = hop_below(Pw, add, g0, g1, 1, target);
    if (nb == 0) hi = g0;
    else if (g0 + nb <= g1) lo = hi = g0 + nb;
    else lo = g1 + 1;
  }
  while (hi > lo) {
    const uint64_t step = (hi - lo + kHopSpan) / kHopSpan; // ceil(span / kHopSpan)
    const uint64_t nb = hop_below(Pw, add, lo, hi, step, target);
    // probes below target form a prefix (W is monotone): answer in (lo + (nb - 1) step, lo + nb step]
    const uint64_t h2 = lo + nb * step;
    if (nb) lo = lo + (nb - 1) * step + 1;
    hi = h2 < hi ? h2 : hi;
  }
  return lo;
}

// Speculation: once a segment length is known, one round loads kHopAhead
// windows of kHopSpan records around pos + h * glen (h = 1..kHopAhead) in one
// batch and resolves up to kHopAhead hops from registers; a hop whose answer
// is not inside its window falls back to hop_exact and starts a new round.
// Equal-sized tables: ~2 load round trips per kHopAhead tables instead of 2
// per table.
constexpr uint32_t kHopAhead = 8, kSpecProbe = kHopProbe;
constexpr uint64_t kSpecSpan = kHopSpan;

// predicted segment length from the mean weight of nrec records of total
// weight rest (equal-sized records: the exact length); 0: none
__device__ __forceinline__ uint64_t hop_predict(uint64_t threshold, uint64_t nrec, uint64_t rest) {
  const uint64_t g = rest ? static_cast<uint64_t>(ceil(static_cast<double>(threshold) * static_cast<double>(nrec) /
                                                       static_cast<double>(rest)))
                          : 0;
  return g >= 1 && g <= nrec ? g : 0;
}

// Hops in parallel: a lone wave pays an address-translation walk for every
// page its probes touch, one after another (measured: ~0.9 us per output
// table, whether a round speculates 8 or 32 hops; touching the pages first
// just moves the cost), so seg_spec_kernel runs one wave per predicted
// segment start h * g on as many CUs, each taking the exact hop from there
// (spec[h]); seg_hops_kernel follows the chain through these answers while
// every hop starts where predicted (equal-sized tables: all of them) and hops
// on its own from the first one that does not.
constexpr uint32_t kSpecHops = 256;

__global__ __launch_bounds__(kWave) void seg_spec_kernel(const uint64_t *Pw, uint64_t add, uint64_t m,
                                                         const uint64_t *mp, uint64_t threshold, uint64_t *spec) {
  if (mp) m = *mp;
  if (m == 0) return;
  const uint64_t w0 = Pw[0], wm = Pw[m] + add * m;
  if (wm - w0 < threshold) return;
  const uint64_t g = hop_predict(threshold, m, wm - w0);
  const uint64_t p = static_cast<uint64_t>(blockIdx.x) * g;
  if (g == 0 || p >= m) return;
  const uint64_t target = Pw[p] + add * p + threshold;
  const uint64_t nx = wm < target ? m : hop_exact(Pw, add, m, p, g, target); // m: the last segment
  if (lane_id() == 0) spec[blockIdx.x] = nx;
}

__global__ __launch_bounds__(kWave) void seg_hops_kernel(const uint64_t *Pw, uint64_t add, uint64_t m,
                                                         const uint64_t *mp, uint64_t threshold, uint64_t *first,
                                                         uint64_t *d_count, const uint64_t *spec) {
  const uint32_t lane = lane_id();
  if (mp) m = *mp; // m = 0: no segment, first[0] = 0
  const uint64_t wm = Pw[m] + add * m;
  uint64_t pos = 0, nseg = 0, glen = 0, wpos = Pw[0];
  bool done = false;
  if (spec && m > 0 && wm - wpos >= threshold) { // the same prediction as seg_spec_kernel's
    const uint64_t g = hop_predict(threshold, m, wm - wpos);
    const uint64_t H = g ? ((m + g - 1) / g < kSpecHops ? (m + g - 1) / g : kSpecHops) : 0; // starts h g < m
    bool follow = true;
    for (uint64_t c = 0; c < H && follow; c += kWave) {
      const uint64_t nv = c + lane < H ? spec[c + lane] : 0;
      for (uint32_t j = 0; j < kWave && c + j < H; j++) {
        if (pos != (c + j) * g) { // the chain left the predicted starts
          follow = false;
          break;
        }
        const uint64_t nx = readlane_u64(nv, j);
        if (lane == 0) first[nseg] = pos;
        nseg++;
        glen = nx - pos;
        pos = nx;
        if (pos >= m) {
          follow = false;
          done = true;
          break;
        }
      }
    }
    if (!done && pos) wpos = Pw[pos] + add * pos;
  }
  while (!done) {
    if (glen == 0 && pos < m && wm - wpos >= threshold) {
      // no segment length seen yet: predict one from the mean weight of the
      // rest (equal-sized records: the first window holds the answer, no
      // exact search); a
      // window that misses falls back to the exact hop below
      glen = hop_predict(threshold, m - pos, wm - wpos);
    }
    if (glen == 0) { // no prediction: one exact hop
      if (pos >= m) break;
      if (lane == 0) first[nseg] = pos;
      nseg++;
      const uint64_t target = wpos + threshold;
      if (wm < target) break; // the last segment runs to m
      const uint64_t nx = hop_exact(Pw, add, m, pos, 0, target);
      glen = nx - pos;
      pos = nx;
      if (pos >= m) break;
      wpos = Pw[pos] + add * pos;
      continue;
    }
    uint64_t v[kHopAhead][kSpecProbe], g0s[kHopAhead];
#pragma unroll
    for (uint32_t h = 0; h < kHopAhead; h++) {
      const uint64_t e = pos + (h + 1) * glen;
      g0s[h] = e > kSpecSpan / 2 ? e - kSpecSpan / 2 : 0;
#pragma unroll
      for (uint32_t r = 0; r < kSpecProbe; r++) {
        const uint64_t x = g0s[h] + static_cast<uint64_t>(r) * kWave + lane;
        v[h][r] = Pw[x <= m ? x : m];
      }
    }
    __builtin_amdgcn_sched_barrier(0); // all kHopAhead windows in flight together
#pragma unroll
    for (uint32_t h = 0; h < kHopAhead; h++) {
#pragma unroll
      for (uint32_t r = 0; r < kSpecProbe; r++) {
        const uint64_t x = g0s[h] + static_cast<uint64_t>(r) * kWave + lane;
        // past m: >= any target (W(m) >= target)
        v[h][r] = x <= m ? v[h][r] + add * x : ~0ull;
      }
    }
#pragma unroll
    for (uint32_t h = 0; h < kHopAhead; h++) {
      if (lane == 0) first[nseg] = pos;
      nseg++;
      const uint64_t target = wpos + threshold;
      if (wm < target) {
        done = true;
        break;
      }
      uint64_t nb = 0;
#pragma unroll
      for (uint32_t r = 0; r < kSpecProbe; r++) nb += __popcll(__ballot(v[h][r] < target));
      // records of the window at or before pos are below target too, so the
      // answer is g0 + nb whenever it lies inside the window and nothing
      // before the window can be the answer
      const uint64_t g0 = g0s[h];
      uint64_t nx, wnx;
      const bool hit = nb < kSpecSpan && (nb > 0 || g0 <= pos + 1);
      if (hit) {
        nx = g0 + nb;
        uint64_t t = 0;
#pragma unroll
        for (uint32_t r = 0; r < kSpecProbe; r++)
          if (r == (nb >> 6)) t = v[h][r];
        wnx = __shfl(t, static_cast<int>(nb & (kWave - 1)), kWave);
      } else {
        nx = hop_exact(Pw, add, m, pos, glen, target);
        wnx = nx < m ? Pw[nx] + add * nx : wm;
      }
      glen = nx - pos;
      pos = nx;
      wpos = wnx;
      if (pos >= m) {
        done = true;
        break;
      }
      if (!hit) break; // re-predict from the exact answer
    }
  }
  if (lane_id() == 0) {
    first[nseg] = m;
    *d_count = nseg;
  }
}

// ---------------------------------------------------------------------------
// Device-wide exclusive scan of u64.  Up to 2048 items: one workgroup
// (scan_apply_kernel).  Beyond: single pass with decoupled look-back
// (scan_lookback_kernel, 4096 items per tile): read n, write n, instead of
// reduce-then-scan's 2 reads + 1 write and its extra launches.
// ---------------------------------------------------------------------------
constexpr uint32_t kScanThreads = 256, kScanItems = 8, kScanTile = kScanThreads * kScanItems;

__device__ __forceinline__ uint64_t wg_excl_scan_u64(uint64_t v, uint64_t &total) {
  __shared__ uint64_t sm[kScanThreads / kWave];
  const uint32_t lane = lane_id(), w = threadIdx.x / kWave;
  const uint64_t incl = wave_incl_scan_u64(v);
  if (lane == kWave - 1) sm[w] = incl;
  __syncthreads();
  uint64_t base = 0, tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanThreads / kWave; k++) {
    const uint64_t x = sm[k];
    if (k < w) base += x;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return base + incl - v;
}

// Scan inputs: a u64 array, or the entry sizes of a record table computed on
// the fly (the encode's offsets, block_builder.cc:19-21, without a sizes array).
struct ArrIn {
  const uint64_t *p;
  __device__ __forceinline__ uint64_t operator()(uint64_t i) const { return p[i]; }
};
struct EntryIn {
  const uint32_t *kl, *vl;
  uint64_t add;
  __device__ __forceinline__ uint64_t operator()(uint64_t i) const { return entry_size(kl[i], vl[i]) + add; }
};

// out[i] = carry_in + sum(in[0..i)), out[n] = carry_in + total.  in may alias out.
template <class In>
__global__ __launch_bounds__(kScanThreads) void scan_apply_kernel(In in, uint64_t n, const uint64_t *tile_base,
                                                                  uint64_t carry_in, uint64_t *out,
                                                                  const uint64_t *skip) {
  if (skip && *skip) return; // (launch_segment: the arithmetic chain held)
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * kScanTile + threadIdx.x * kScanItems;
  uint64_t v[kScanItems];
  uint64_t s = 0;
#pragma unroll
  for (uint32_t j = 0; j < kScanItems; j++) {
    v[j] = t0 + j < n ? in(t0 + j) : 0;
    s += v[j];
  }
  uint64_t tot;
  uint64_t run = wg_excl_scan_u64(s, tot) + carry_in + (tile_base ? tile_base[blockIdx.x] : 0);
#pragma unroll
  for (uint32_t j = 0; j < kScanItems; j++) {
    if (t0 + j < n) out[t0 + j] = run;
    run += v[j];
  }
  if (n == 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) out[0] = carry_in;
  } else if (t0 <= n - 1 && n - 1 < t0 + kScanItems) {
    out[n] = run; // the thread holding the last element writes the total
  }
}

// Tile status word: 2 flag bits | 14-bit epoch | 48 value bits in ONE u64,
// published and polled with agent-scope atomics (per-XCD L2s are not
// coherent; an sc1 store / sc1 load pair on a single word needs no separate
// fence).  Totals must stay below 2^48.  A word counts only when its epoch is
// the launch's: a context tags every scan on its own workspace with a new
// epoch, so stale words of earlier calls are ignored and no memset precedes
// the scan (epoch 0 = the caller cleared the words in an earlier kernel).
// Tile = workgroup id: workgroups are dispatched in id order, so every tile a
// workgroup waits on is resident or done (round 4 drew a ticket per tile from
// a device-scope counter; SSTC_SCAN_TICKET=1 builds that for A/B).
// ws = [unused, status[tiles]].
constexpr uint32_t kLbItems = 16;
#ifndef SSTC_SCAN_TICKET
#define SSTC_SCAN_TICKET 0
#endif

__device__ __forceinline__ uint32_t lb_idx(uint32_t i) { return i + (i >> 4); } // 1 pad per 16

template <class In, uint32_t kItems = kLbItems>
__global__ __launch_bounds__(kScanThreads) void scan_lookback_kernel(In in, uint64_t n, uint64_t carry_in,
                                                                     uint64_t *out, uint64_t *ws, uint32_t epoch,
                                                                     const uint64_t *skip, LbFail fail) {
  if (skip && *skip) return; // uniform: every tile returns (launch_segment: the arithmetic chain held)
  constexpr uint32_t kTile = kScanThreads * kItems;
  __shared__ uint64_t sm[kTile + kTile / 16];
  __shared__ uint64_t s_wsum[kScanThreads / kWave];
  __shared__ uint64_t s_prefix;
  const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid / kWave;
#if SSTC_SCAN_TICKET
  __shared__ uint64_t s_tile;
  if (tid == 0) {
    const uint64_t t = __hip_atomic_fetch_add(ws, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t + 1 == gridDim.x) __hip_atomic_store(ws, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_tile = t;
  }
  __syncthreads();
  const uint64_t tile = s_tile;
#else
  // tile = workgroup id (dispatched in id order: the lowest unfinished tile
  // is resident, as in ck_filter_kernel; ws[0] is unused)
  const uint64_t tile = blockIdx.x;
#endif
  const uint64_t base = tile * kTile;
  uint64_t *status = ws + 1;
#pragma unroll
  for (uint32_t j = 0; j < kItems; j++) {
    const uint32_t i = j * kScanThreads + tid;
    sm[lb_idx(i)] = base + i < n ? in(base + i) : 0;
  }
  __syncthreads();
  uint64_t v[kItems], sum = 0;
#pragma unroll
  for (uint32_t j = 0; j < kItems; j++) {
    v[j] = sm[lb_idx(tid * kItems + j)];
    sum += v[j];
  }
  const uint64_t incl = wave_incl_scan_u64(sum);
  if (lane == kWave - 1) s_wsum[w] = incl;
  __syncthreads();
  uint64_t wbase = 0, total = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanThreads / kWave; k++) {
    const uint64_t x = s_wsum[k];
    if (k < w) wbase += x;
    total += x;
  }
  if (w == 0) {
    const uint64_t prefix = lb_publish_lookback(status, tile, total, epoch, fail);
    if (lane == 0) s_prefix = prefix;
  }
  __syncthreads();
  uint64_t run = carry_in + s_prefix + wbase + incl - sum;
#pragma unroll
  for (uint32_t j = 0; j < kItems; j++) {
    sm[lb_idx(tid * kItems + j)] = run;
    run += v[j];
  }
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < kItems; j++) {
    const uint32_t i = j * kScanThreads + tid;
    if (base + i < n) out[base + i] = sm[lb_idx(i)];
  }
  if (tid == 0 && base < n && n <= base + kTile) out[n] = carry_in + s_prefix + total;
}

// Record bases of the blocks in ONE kernel (count_kernel + a scan of its
// counts were two launches): a workgroup reads the 16 B extras of kCsTile
// blocks (n and the offset section start, table_reader.cc:11-20; an extra
// that fails check_extra counts 0, as in count_kernel), scans the counts by
// decoupled look-back (tile = workgroup id, status words at ws + kCsStatus)
// and writes rec_base[0..n].
// kStart, the compaction job's first kernel (ck_start_kernel's work folded in
// as well: one launch where there were three): every tile also reduces its
// blocks' byte sum and source end into part[], and the last tile to finish
// (ws[0] is the ticket) does the job's first host hand-off -- the run starts
// rec_base[tfb[i]] to the device and the pinned host words with the input
// bytes, the error-counter snapshot, the cleared unsorted count, guard words
// and the check / footer kernels' tickets, then the sequence word the host
// spins on.  Its ws is the context's persistent region (Arena::lb), zero at
// entry (epoch 0): the last tile clears the ticket and the status words again
// once every tile has finished its look-back.
#ifndef SSTC_CS_ITEMS
#define SSTC_CS_ITEMS 8
#endif
constexpr uint32_t kCsItems = SSTC_CS_ITEMS, kCsTile = kScanThreads * kCsItems, kCsStatus = 32;

uint64_t count_scan_tiles(uint64_t nblocks) { return nblocks ? (nblocks + kCsTile - 1) / kCsTile : 1; }
uint64_t count_scan_workspace(uint64_t nblocks) { return kCsStatus + count_scan_tiles(nblocks); }

constexpr uint64_t kPartGaveUp = 1ull << 63; // part[2 t]: tile t's look-back gave up
template <bool kStart>
__global__ __launch_bounds__(kScanThreads) void count_scan_kernel(CountScanArgs a) {
  __shared__ uint64_t sm[kCsTile + kCsTile / 16];
  __shared__ uint64_t s_wsum[kScanThreads / kWave], s_bytes[kScanThreads / kWave], s_end[kScanThreads / kWave];
  __shared__ uint64_t s_prefix;
  __shared__ uint32_t s_last;
  __shared__ unsigned long long s_gave; // start: a look-back (this tile's, or any tile's in the last) gave up
  const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid / kWave;
  const uint64_t n = a.nblocks, tile = blockIdx.x, base = tile * kCsTile;
  if (kStart && tid == 0) s_gave = 0; // (read after the barriers below)
  // masked-off extras read 16 B of the ticket line no thread writes
  const uint8_t *safe = reinterpret_cast<const uint8_t *>(a.ws + 8);
  uint64_t len[kCsItems], off[kCsItems];
#pragma unroll
  for (uint32_t j = 0; j < kCsItems; j++) {
    const uint64_t i = base + j * kScanThreads + tid;
    len[j] = i < n ? a.blk_len[i] : 0;
    off[j] = i < n ? a.blk_off[i] : 0;
  }
  // every extra's loads issued before any is used (clamped, not branched)
  uint64_t xn[kCsItems], xd[kCsItems];
#pragma unroll
  for (uint32_t j = 0; j < kCsItems; j++) {
    const uint8_t *p = len[j] >= 16 ? a.src + off[j] + len[j] - 16 : safe;
    xn[j] = g_u64u(p);
    xd[j] = g_u64u(p + 8);
  }
  uint64_t bytes = 0, end = 0;
#pragma unroll
  for (uint32_t j = 0; j < kCsItems; j++) {
    const uint32_t x = j * kScanThreads + tid;
    sm[lb_idx(x)] = len[j] >= 16 && check_extra(len[j], xn[j], xd[j]) == kBlkOk ? xn[j] : 0;
    if constexpr (kStart) {
      bytes += len[j];
      const uint64_t e = base + x < n ? off[j] + len[j] : 0;
      end = e > end ? e : end;
    }
  }
  __syncthreads();
  uint64_t v[kCsItems], sum = 0;
#pragma unroll
  for (uint32_t j = 0; j < kCsItems; j++) {
    v[j] = sm[lb_idx(tid * kCsItems + j)];
    sum += v[j];
  }
  const uint64_t incl = wave_incl_scan_u64(sum);
  if (lane == kWave - 1) s_wsum[w] = incl;
  if constexpr (kStart) {
    bytes = wave_sum_u64(bytes);
    for (uint32_t d = kWave / 2; d > 0; d >>= 1) {
      const uint64_t y = __shfl_xor(end, d, kWave);
      end = y > end ? y : end;
    }
    if (lane == 0) {
      s_bytes[w] = bytes;
      s_end[w] = end;
    }
  }
  __syncthreads();
  uint64_t wbase = 0, total = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanThreads / kWave; k++) {
    const uint64_t x = s_wsum[k];
    if (k < w) wbase += x;
    total += x;
  }
  if (w == 0) {
    const uint64_t prefix = lb_publish_lookback(a.ws + kCsStatus, tile, total, a.epoch,
                                                kStart ? LbFail{&s_gave, 1} : LbFail{a.lb_fail, 0});
    if (lane == 0) s_prefix = prefix;
  }
  __syncthreads();
  uint64_t run = s_prefix + wbase + incl - sum;
#pragma unroll
  for (uint32_t j = 0; j < kCsItems; j++) {
    sm[lb_idx(tid * kCsItems + j)] = run;
    run += v[j];
  }
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < kCsItems; j++) {
    const uint32_t i = j * kScanThreads + tid;
    if (base + i < n) a.rec_base[base + i] = sm[lb_idx(i)];
  }
  // rec_base[n] = the record count: the tile holding item n - 1 (tile 0 when n = 0)
  if (tid == 0 && (n == 0 ? tile == 0 : base < n && n <= base + kCsTile)) a.rec_base[n] = s_prefix + total;
  if constexpr (kStart) {
    if (tid == 0) {
      uint64_t by = 0, e = 0;
      for (uint32_t k = 0; k < kScanThreads / kWave; k++) {
        by += s_bytes[k];
        e = s_end[k] > e ? s_end[k] : e;
      }
      a.part[2 * tile] = by | (s_gave ? kPartGaveUp : 0ull); // (block bytes < 2^63)
      a.part[2 * tile + 1] = e;
    }
    // the tile's stores drained, then released at agent scope before its
    // ticket; the last tile acquires before it reads the others' (as the
    // check kernel's long-group hand-off)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const bool last =
          __hip_atomic_fetch_add(a.ws, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1ull;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    uint64_t by = 0, e = 0, gave = 0;
    for (uint64_t p = tid; p < gridDim.x; p += kScanThreads) {
      const uint64_t b = __hip_atomic_load(a.part + 2 * p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      by += b & ~kPartGaveUp;
      gave |= b & kPartGaveUp;
      const uint64_t x = __hip_atomic_load(a.part + 2 * p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      e = x > e ? x : e;
    }
    by = wave_sum_u64(by);
    for (uint32_t d = kWave / 2; d > 0; d >>= 1) {
      const uint64_t y = __shfl_xor(e, d, kWave);
      e = y > e ? y : e;
    }
    if (lane == 0) {
      s_bytes[w] = by;
      s_end[w] = e;
    }
    if (gave) s_gave = 1;
    for (uint64_t i = tid; i < a.ntfb; i += kScanThreads) {
      const uint64_t r = __hip_atomic_load(a.rec_base + a.tfb[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      a.run_start[i] = r;
      a.host[1 + i] = r;
    }
    for (uint64_t x = tid; x < gridDim.x; x += kScanThreads) a.ws[kCsStatus + x] = 0; // for the next job
    __syncthreads();
    if (tid == 0) {
      by = 0;
      e = 0;
      for (uint32_t k = 0; k < kScanThreads / kWave; k++) {
        by += s_bytes[k];
        e = s_end[k] > e ? s_end[k] : e;
      }
      a.host[0] = s_gave ? ~0ull : by; // input block bytes (~0: the run starts are wrong)
      *a.errs = *a.err_count;
      *a.bad = 0;
      a.guard[0] = s_gave ? kGuardLookback : 0; // consistency-guard bits
      a.guard[1] = e; // the end of the source bytes the input blocks span
      for (int g = 0; g < 10; g++) a.guard[32 + 32 * g] = 0; // the check kernel's 9 tickets, the footer's
      a.ws[0] = 0; // the ticket, for the next job
    }
    __threadfence_system();
    __syncthreads();
    if (tid == 0) __hip_atomic_store(a.host + a.flag, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

hipError_t launch_count_scan(const CountScanArgs &a, bool start, hipStream_t s) {
  const uint32_t g = static_cast<uint32_t>(count_scan_tiles(a.nblocks));
  if (start) count_scan_kernel<true><<<g, kScanThreads, 0, s>>>(a);
  else count_scan_kernel<false><<<g, kScanThreads, 0, s>>>(a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Launch wrappers
// ---------------------------------------------------------------------------
static inline uint32_t grid_for(uint64_t n, uint32_t per) { return static_cast<uint32_t>((n + per - 1) / per); }



// copy ceiling probe (sstc_copy_probe): the best plain copy of the same bytes
// (one 16 B non-temporal load + store per lane, profiles/r01_ab_variants.md)
typedef uint32_t probe_u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void copy_probe_kernel(const probe_u32x4 *__restrict__ s,
                                                         probe_u32x4 *__restrict__ d, uint64_t n) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}

hipError_t launch_copy_probe(const uint8_t *src, uint8_t *dst, uint64_t n16, hipStream_t s) {
  if (n16)
    copy_probe_kernel<<<static_cast<uint32_t>((n16 + 255) / 256), 256, 0, s>>>(
        reinterpret_cast<const probe_u32x4 *>(src), reinterpret_cast<probe_u32x4 *>(dst), n16);
  return hipGetLastError();
}

hipError_t launch_roundtrip(const RtArgs &a, hipStream_t s) {
  // blocks in dispatch order: the XCD-grouped order measured +3 % at config 2
  // (256 MiB, Infinity-Cache resident) but -2.5 % on 1 GiB (profiles/r01_ab_xcd.log)
  // (persistent waves looping over blocks in one or two slots, staging through
  // VGPRs instead of LDS-DMA, and storing the staged block before the parse
  // were all slower: profiles/r02_ab/rt_ab.md, profiles/r03_ab/rt_1gib.md)
  if (a.nblocks) rt_kernel<<<grid_for(a.nblocks, kRtWaves), kRtWaves * kWave, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_decode(const DecArgs &a, hipStream_t s) {
  DecArgs b = a;
  b.xcd = 1; // XCD-grouped block order: neighbouring blocks share L2 lines (-5 % time, config 3)
  if (a.nblocks && a.sk) decode_kernel<true><<<grid_for(a.nblocks, kDecWaves), kDecWaves * kWave, 0, s>>>(b);
  else if (a.nblocks) decode_kernel<false><<<grid_for(a.nblocks, kDecWaves), kDecWaves * kWave, 0, s>>>(b);
  return hipGetLastError();
}

// SoA record table -> 32 B records (sstc_record32), one record per thread:
// 33 B of columns read, 32 B written, both coalesced
static_assert(sizeof(sstc_record32) == 32, "sstc_record32 is 32 B");
__global__ __launch_bounds__(256) void pack_records_kernel(sstc_records in, uint64_t n, sstc_record32 *out) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint64_t ko = in.key_off[i], vo = in.val_off[i], tx = in.txn[i];
    const uint32_t kl = in.key_len[i], vl = in.val_len[i], ty = in.type[i];
    const uint32_t rel = vl == kNoValue ? 0u : static_cast<uint32_t>(vo - ko);
    u32x4 *q = reinterpret_cast<u32x4 *>(out + i);
    q[0] = u32x4{static_cast<uint32_t>(ko), static_cast<uint32_t>(ko >> 32), static_cast<uint32_t>(tx),
                 static_cast<uint32_t>(tx >> 32)};
    q[1] = u32x4{kl, rel, vl, ty};
  }
}

hipError_t launch_pack_records(const sstc_records &in, uint64_t nrec, sstc_record32 *out, hipStream_t s) {
  if (nrec) pack_records_kernel<<<static_cast<uint32_t>(std::min<uint64_t>(grid_for(nrec, 256), 8192)), 256, 0, s>>>(
      in, nrec, out);
  return hipGetLastError();
}

// sized for the smallest tile any scan uses (kScanThreads x 4 items)
uint64_t scan_workspace_elems(uint64_t n) { return (n + 4 * kScanThreads - 1) / (4 * kScanThreads) + 2; }


// u64 array scans (block counts, block lengths, segmentation node counts):
// kArrItems per thread (16 / 8 / 4: the three block-level scans of config 3
// took 28.4 / 20.9 / 25.9 us); the entry-size scan keeps kLbItems
constexpr uint32_t kArrItems = 8, kArrTile = kScanThreads * kArrItems;
uint64_t scan_status_words(uint64_t n) { return n <= kScanTile ? 0 : (n + kArrTile - 1) / kArrTile + 1; }

template <class In, uint32_t kItems = kLbItems>
static hipError_t scan_any(In in, uint64_t n, uint64_t carry_in, uint64_t *out, uint64_t *ws, hipStream_t s,
                           bool ws_zeroed, uint32_t epoch, const uint64_t *skip = nullptr,
                           LbFail fail = LbFail{}) {
  constexpr uint64_t kTile = kScanThreads * kItems;
  if (n <= kScanTile) {
    scan_apply_kernel<In><<<1, kScanThreads, 0, s>>>(in, n, nullptr, carry_in, out, skip);
    return hipGetLastError();
  }
  const uint64_t tiles = (n + kTile - 1) / kTile;
  if (ws_zeroed) {
    epoch = 0;
  } else if (epoch == 0) {
    hipError_t e = hipMemsetAsync(ws, 0, (tiles + 1) * sizeof(uint64_t), s);
    if (e != hipSuccess) return e;
  }
  scan_lookback_kernel<In, kItems><<<static_cast<uint32_t>(tiles), kScanThreads, 0, s>>>(in, n, carry_in, out, ws,
                                                                                        epoch, skip, fail);
  return hipGetLastError();
}

hipError_t launch_scan(const uint64_t *in, uint64_t n, uint64_t carry_in, uint64_t *out, uint64_t *ws,
                       hipStream_t s, bool ws_zeroed, uint32_t epoch, unsigned long long *guard) {
  return scan_any<ArrIn, kArrItems>(ArrIn{in}, n, carry_in, out, ws, s, ws_zeroed, epoch, nullptr,
                                    LbFail{guard, kGuardLookback});
}

hipError_t launch_scan_entry_sizes(const uint32_t *klen, const uint32_t *vlen, uint64_t nrec, uint64_t add,
                                   uint64_t *out, uint64_t *ws, hipStream_t s, uint32_t epoch,
                                   unsigned long long *err_count) {
  // 16 items per thread: 4 and 8 were slower (37.9 / 24.8 vs 20.4 us at 1.8 M records, the look-back chain)
  return scan_any(EntryIn{klen, vlen, add}, nrec, 0, out, ws, s, false, epoch, nullptr, LbFail{err_count, 0});
}

// Block lengths and offsets of a records -> blocks encode in ONE kernel
// (enc_bsum_kernel + a block scan were two launches, ~13 us of the config-2
// encode leg): a workgroup per tile of kBoTile blocks sums every block's entry
// sizes with kBsG lanes per block -- the block bounds of all its passes, then
// the first kBoUnroll records of every lane, issued before any is used (one
// dependent round trip each) --, scans the tile's lengths, and takes the
// tile's offset from a decoupled look-back over the tiles (ticketed,
// epoch-tagged status words, as scan_lookback_kernel).  ws = [ticket,
// status[tiles]].
constexpr uint32_t kBoThreads = 1024, kBoTile = 256, kBoPasses = kBoTile * kBsG / kBoThreads, kBoUnroll = 4;
constexpr uint32_t kBoScanWaves = kBoTile / kWave;
__global__ __launch_bounds__(kBoThreads) void enc_offsets_kernel(const uint32_t *kl, const uint32_t *vl,
                                                                 const uint64_t *blk_first, uint64_t nblocks,
                                                                 uint64_t out_base, uint64_t *blk_off,
                                                                 uint64_t *blk_len, uint64_t *ws, uint32_t epoch,
                                                                 LbFail fail) {
  __shared__ uint64_t s_len[kBoTile];
  __shared__ uint64_t s_wsum[kBoScanWaves];
  __shared__ uint64_t s_tile, s_prefix;
  const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid / kWave, g = tid % kBsG;
  if (tid == 0) {
    const uint64_t t = __hip_atomic_fetch_add(ws, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t + 1 == gridDim.x) __hip_atomic_store(ws, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_tile = t;
  }
  __syncthreads();
  const uint64_t tile = s_tile, b0 = tile * kBoTile;
  uint64_t F0[kBoPasses], F1[kBoPasses];
#pragma unroll
  for (uint32_t p = 0; p < kBoPasses; p++) {
    const uint64_t b = b0 + p * (kBoThreads / kBsG) + tid / kBsG;
    const uint64_t bc = b < nblocks ? b : 0;
    F0[p] = blk_first[bc];
    F1[p] = b < nblocks ? blk_first[bc + 1] : F0[p];
  }
  uint32_t K[kBoPasses][kBoUnroll], V[kBoPasses][kBoUnroll];
#pragma unroll
  for (uint32_t p = 0; p < kBoPasses; p++) {
#pragma unroll
    for (uint32_t k = 0; k < kBoUnroll; k++) {
      // a lane past its block's records re-reads the block's first record; an
      // empty block reads nothing (nrec may be 0 with NULL record columns)
      const uint64_t r = F0[p] + g + k * kBsG;
      const uint64_t rc = r < F1[p] ? r : F0[p];
      K[p][k] = 0;
      V[p][k] = 0;
      if (F0[p] < F1[p]) {
        K[p][k] = kl[rc];
        V[p][k] = vl[rc];
      }
    }
  }
#pragma unroll
  for (uint32_t p = 0; p < kBoPasses; p++) {
    uint64_t sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kBoUnroll; k++)
      if (F0[p] + g + k * kBsG < F1[p]) sum += entry_size(K[p][k], V[p][k]);
    for (uint64_t r = F0[p] + g + kBoUnroll * kBsG; r < F1[p]; r += kBsG) sum += entry_size(kl[r], vl[r]);
#pragma unroll
    for (uint32_t d = kBsG / 2; d > 0; d >>= 1) sum += __shfl_xor(sum, d, kWave); // inside the 8-lane group
    const uint32_t lb = p * (kBoThreads / kBsG) + tid / kBsG;
    if (g == 0) s_len[lb] = b0 + lb < nblocks ? sum + 16 * (F1[p] - F0[p]) + 16 : 0;
  }
  __syncthreads();
  // the tile scan: thread tid < kBoTile holds block b0 + tid
  const uint64_t len = tid < kBoTile ? s_len[tid] : 0;
  const uint64_t incl = wave_incl_scan_u64(len);
  if (w < kBoScanWaves && lane == kWave - 1) s_wsum[w] = incl;
  __syncthreads();
  uint64_t wbase = 0, total = 0;
#pragma unroll
  for (uint32_t k = 0; k < kBoScanWaves; k++) {
    const uint64_t x = s_wsum[k];
    if (k < w) wbase += x;
    total += x;
  }
  if (w == 0) {
    const uint64_t tag = static_cast<uint64_t>(epoch) << kLbEpochShift;
    uint64_t *status = ws + 1;
    uint64_t prefix = 0;
    if (tile == 0) {
      if (lane == 0) __hip_atomic_store(&status[0], kLbInc | tag | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(&status[tile], kLbAgg | tag | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int64_t p = static_cast<int64_t>(tile) - 1; // window [p - 63, p]
      uint64_t spins = 0;
      for (;;) {
        const int64_t q = p - static_cast<int64_t>(lane);
        uint64_t st = q >= 0 ? __hip_atomic_load(&status[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : kLbInc | tag;
        if (((st >> kLbEpochShift) & 0x3FFFu) != epoch) st = 0; // a stale word: not published yet
        const uint64_t inc = __ballot((st >> 62) == 2);
        const uint32_t need = inc ? static_cast<uint32_t>(__ffsll(static_cast<long long>(inc))) : kWave;
        if (__ballot((st >> 62) == 0 && lane < need)) {
          if (++spins > kLbSpinLimit) { // a predecessor never published: give up (no hang), reported
            if (lane == 0) fail.report();
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        prefix += wave_sum_u64(lane < need ? (st & kLbVal) : 0);
        if (inc) break;
        p -= kWave;
      }
      if (lane == 0)
        __hip_atomic_store(&status[tile], kLbInc | tag | (prefix + total), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) s_prefix = prefix;
  }
  __syncthreads();
  const uint64_t b = b0 + tid;
  if (tid < kBoTile && b < nblocks) {
    const uint64_t off = out_base + s_prefix + wbase + incl - len;
    blk_off[b] = off;
    blk_len[b] = len;
    if (b + 1 == nblocks) blk_off[nblocks] = off + len;
  }
}

uint64_t enc_offsets_workspace(uint64_t nblocks) { return (nblocks + kBoTile - 1) / kBoTile + 2; }

hipError_t launch_enc_offsets(const uint32_t *kl, const uint32_t *vl, const uint64_t *blk_first, uint64_t nblocks,
                              uint64_t out_base, uint64_t *blk_off, uint64_t *blk_len, uint64_t *ws, hipStream_t s,
                              uint32_t epoch, unsigned long long *err_count) {
  if (nblocks == 0) { // blk_first may be NULL
    enc_none_kernel<<<1, 1, 0, s>>>(out_base, blk_off);
    return hipGetLastError();
  }
  if (nblocks <= kScanTile || epoch == 0) { // one workgroup's scan / no epoch: sum kernel + scan
    enc_bsum_kernel<<<grid_for(nblocks * kBsG, 256), 256, 0, s>>>(kl, vl, blk_first, nblocks, blk_len);
    return scan_any<ArrIn, kArrItems>(ArrIn{blk_len}, nblocks, out_base, blk_off, ws, s, false, epoch, nullptr,
                                      LbFail{err_count, 0});
  }
  // ws: enc_offsets_workspace(nblocks) words
  enc_offsets_kernel<<<static_cast<uint32_t>((nblocks + kBoTile - 1) / kBoTile), kBoThreads, 0, s>>>(
      kl, vl, blk_first, nblocks, out_base, blk_off, blk_len, ws, epoch, LbFail{err_count, 0});
  return hipGetLastError();
}

hipError_t launch_enc_emit(const EncArgs &a, hipStream_t s) {
  if (!a.nblocks) return hipSuccess;
  if (a.entries_in_src && (!a.nb_dev || !a.need)) return hipErrorInvalidValue; // mode 1 reads both on the device
  const uint32_t g = grid_for(a.nblocks, kEncWaves);
  // G = 8 lanes per span, 2 span groups in flight: G = 16 and kQ = 4 / 8 were
  // slower (profiles/r02_ab/encode_ab.md)
  // keys in 2-lane groups, values in 8-lane groups, 2 span groups in flight:
  // (4, 8, 2) / (2, 8, 1) / (4, 8, 4) / (2, 8, 4) and the single pass over
  // (key, value) span pairs were slower (profiles/r02_ab/encode_ab.md)
  if (!a.entries_in_src) enc_lds_kernel<0><<<g, kEncWaves * kWave, 0, s>>>(a);
  else if (a.large_blocks) enc_lds_kernel<1, 2, 8, 4, 4><<<g, kEncWaves * kWave, 0, s>>>(a);
  else enc_lds_kernel<1, 2, 8, 2, 2><<<g, kEncWaves * kWave, 0, s>>>(a);
  // blocks past an LDS slot are encoded by the wave that met them (a listed
  // pass by a workgroup per block was slower: Zipf set 329 -> 236 us, config 5
  // 319 -> 233 us; profiles/r02_ab/)
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Arithmetic block chains.  When the records of an output table have equal
// entry sizes (fixed-size keys and values, configs 2-4, db_bench's default),
// its segments all hold the same number of records but the last: the chain
// through table a is T_a, T_a + g_a, T_a + 2 g_a, ... (T_a its first record)
// up to T_{a+1}.  seg_arith_kernel predicts g_a from the table's first record
// (the least k with k w >= threshold, w = W(T_a + 1) - W(T_a)) and scans the
// predicted segment counts; seg_arith_check_kernel writes every predicted
// start and checks its hop exactly against W -- the hop from p is
// q = min(p + g_a, T_{a+1}) iff W(q - 1) < W(p) + threshold (or q - 1 = p) and,
// unless q = T_{a+1}, W(q) >= W(p) + threshold: three loads, no walk, every
// hop checked (the first included), so a wrong prediction only costs the
// fallback.  One failed check (or more than kArMax tables) clears the verdict
// word and the general chain walk above runs; when every hop checks, its
// kernels (seg_walk, the window scan, seg_node, seg_npow, seg_nentry,
// seg_emit) return at once.
// ---------------------------------------------------------------------------
constexpr uint32_t kArMax = 1024, kArThreads = 512;

struct ArithArgs {
  const uint64_t *Pw;
  uint64_t add, m, threshold;   // m: the host bound
  const uint64_t *ends, *nends; // optional table starts ends[0..*nends] (ends[*nends] = the record count)
  const uint64_t *mp;           // optional device record count
  // ar[0]: verdict (1: every predicted hop holds), ar[1]: segment count,
  // ar[2 ..]: g_a (kArMax), then the segment bases of the tables (kArMax + 1)
  uint64_t *ar;
  uint64_t *first, *d_count;
  // optional: a chain that fails (here or in the check) ORs fail_bit into
  // *fail (the compaction job's guard word: a note, or -- when the general
  // walk was not enqueued -- the bit that makes the job's writers stand down)
  unsigned long long *fail = nullptr;
  unsigned long long fail_bit = 0;
  __device__ void failed() const {
    if (fail) atomicOr(fail, fail_bit);
  }
};

__device__ __forceinline__ uint64_t ar_w(const ArithArgs &a, uint64_t x) { return a.Pw[x] + a.add * x; }

// table t's predicted hop and segment count (0: not a table the chain can take)
__device__ __forceinline__ void ar_predict(const ArithArgs &a, uint64_t t, uint64_t nt, uint64_t m, uint64_t &g,
                                           uint64_t &cnt) {
  g = cnt = 0;
  if (t >= nt) return;
  const uint64_t T0 = a.ends ? a.ends[t] : 0, T1 = a.ends ? a.ends[t + 1] : m;
  if (!(T0 < T1 && T1 <= m)) return;
  const uint64_t w = ar_w(a, T0 + 1) - ar_w(a, T0), len = T1 - T0;
  uint64_t k = w ? (a.threshold + w - 1) / w : len;
  k = k < 1 ? 1 : (k > len ? len : k);
  g = k;
  cnt = (len + k - 1) / k;
}

__global__ __launch_bounds__(kArThreads) void seg_arith_kernel(ArithArgs a) {
  __shared__ uint64_t s_w[kArThreads / kWave];
  __shared__ uint32_t s_bad;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid / kWave;
  const uint64_t m = a.mp ? *a.mp : a.m;
  const uint64_t nt = a.ends ? *a.nends : 1;
  if (m == 0 || nt == 0 || nt > kArMax) { // no records: the general path's m = 0 case; too many tables
    if (tid == 0) {
      a.ar[0] = 0;
      a.failed();
    }
    return;
  }
  if (tid == 0) s_bad = 0;
  __syncthreads();
  uint64_t *g = a.ar + 2, *tb = a.ar + 2 + kArMax;
  uint64_t g0, c0, g1, c1; // tables 2 tid, 2 tid + 1
  ar_predict(a, 2 * tid, nt, m, g0, c0);
  ar_predict(a, 2 * tid + 1, nt, m, g1, c1);
  if ((2 * tid < nt && !c0) || (2 * tid + 1 < nt && !c1)) s_bad = 1; // an empty or out-of-range table
  const uint64_t inc = wave_incl_scan_u64(c0 + c1);
  if (lane == kWave - 1) s_w[wv] = inc;
  __syncthreads();
  uint64_t before = 0, total = 0;
  for (uint32_t k = 0; k < kArThreads / kWave; k++) {
    before += k < wv ? s_w[k] : 0;
    total += s_w[k];
  }
  const uint64_t b0 = before + inc - (c0 + c1);
  if (2 * tid < nt) {
    g[2 * tid] = g0;
    tb[2 * tid] = b0;
  }
  if (2 * tid + 1 < nt) {
    g[2 * tid + 1] = g1;
    tb[2 * tid + 1] = b0 + c0;
  }
  if (tid == 0) {
    tb[nt] = total;
    a.ar[1] = total;
    a.ar[0] = s_bad ? 0 : 1;
    if (s_bad) a.failed();
    if (!s_bad) { // the general path writes both when it runs
      *a.d_count = total;
      a.first[total] = m;
    }
  }
}

__global__ __launch_bounds__(256) void seg_arith_check_kernel(ArithArgs a) {
  __shared__ uint64_t s_tb[kArMax + 1], s_t[kArMax + 1], s_g[kArMax];
  // the verdict, the count and the tables' words in one round of loads
  const uint64_t ok0 = a.ar[0], total = a.ar[1];
  const uint64_t m = a.mp ? *a.mp : a.m;
  const uint64_t nt = a.ends ? *a.nends : 1;
  const uint64_t *g = a.ar + 2, *tb = a.ar + 2 + kArMax;
  if (!ok0 || nt > kArMax) return; // not eligible, or a hop already failed: the general path writes everything
  for (uint64_t t = threadIdx.x; t <= nt; t += 256) {
    s_tb[t] = tb[t];
    s_t[t] = a.ends ? a.ends[t] : (t ? m : 0);
    if (t < nt) s_g[t] = g[t];
  }
  __syncthreads();
  bool ok = true;
  for (uint64_t h = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; h < total;
       h += static_cast<uint64_t>(gridDim.x) * 256) {
    uint64_t lo = 0, hi = nt; // the table: s_tb[lo] <= h < s_tb[lo + 1]
    while (lo + 1 < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (s_tb[mid] <= h) lo = mid;
      else hi = mid;
    }
    const uint64_t T1 = s_t[lo + 1], gg = s_g[lo];
    const uint64_t p = s_t[lo] + (h - s_tb[lo]) * gg;
    const uint64_t q = p + gg < T1 ? p + gg : T1;
    const uint64_t wp = ar_w(a, p), wq1 = ar_w(a, q - 1), wq = ar_w(a, q);
    const uint64_t target = wp + a.threshold;
    ok &= p < T1 && (q - 1 == p || wq1 < target) && (q == T1 || wq >= target);
    a.first[h] = p;
  }
  if (!ok) { // (every failing thread stores the same 0)
    a.ar[0] = 0;
    a.failed();
  }
}

namespace {
struct SegLayout { // u32 offsets into the segmentation workspace
  uint64_t tiles, levels, J0, Fx, Fc, Nx, Nc, Nt, tentry, tbefore, u64, total;
  // u64 region (8-aligned): win[tiles + 1], base[tiles + 1], nn, visits, scan
  // ws, the arithmetic chain's words (ArithArgs::ar)
  uint64_t win, base, nn, visits, sws, ar;
  explicit SegLayout(uint64_t m) {
    tiles = (m + kChTile - 1) / kChTile;
    levels = 1;
    for (uint64_t r = kSegRadix; r < tiles; r *= kSegRadix) levels++;
    const uint64_t n1 = m + 1;
    J0 = 0;
    Fx = J0 + n1;
    Fc = Fx + n1;
    Nx = Fc + n1;
    Nc = Nx + levels * n1;
    Nt = Nc + levels * n1;
    tentry = Nt + n1;
    tbefore = tentry + tiles + 1;
    u64 = (tbefore + tiles + 1 + 1) & ~uint64_t(1);
    win = 0;
    base = win + tiles + 1;
    nn = base + tiles + 1;
    visits = nn + 1;
    sws = visits + 1;
    ar = sws + scan_workspace_elems(tiles + 1) + 1;
    total = u64 + 2 * (ar + 2 + 2 * kArMax + 1 + 1);
  }
};
} // namespace

uint64_t segment_workspace_u32(uint64_t nrec) {
  return std::max<uint64_t>(SegLayout(nrec).total + 2, 2 * kSpecHops); // (the long-segment path: spec words)
}

hipError_t launch_segment(const uint64_t *Pw, uint64_t nrec, uint64_t threshold, uint32_t *J,
                          uint64_t *d_nblocks, uint64_t *blk_first, hipStream_t s, const uint64_t *ends,
                          const uint64_t *d_nends, uint64_t add, bool long_segments, const uint64_t *d_nrec,
                          SegMode mode, unsigned long long *fail) {
  if (nrec == 0) { // no records: no segment, first[0] = 0
    hipError_t e = hipMemsetAsync(d_nblocks, 0, sizeof(uint64_t), s);
    if (e == hipSuccess) e = hipMemsetAsync(blk_first, 0, sizeof(uint64_t), s);
    return e;
  }
  if (long_segments && !ends) {
    uint64_t *spec = reinterpret_cast<uint64_t *>(J); // kSpecHops words (segment_workspace_u32)
    if (spec) seg_spec_kernel<<<kSpecHops, kWave, 0, s>>>(Pw, add, nrec, d_nrec, threshold, spec);
    seg_hops_kernel<<<1, kWave, 0, s>>>(Pw, add, nrec, d_nrec, threshold, blk_first, d_nblocks, spec);
    return hipGetLastError();
  }
  const SegLayout L(nrec);
  // u64 region 8-aligned relative to J (J itself is 256-aligned by the callers' allocators)
  uint64_t *U = reinterpret_cast<uint64_t *>(J + L.u64);
  uint64_t *win = U + L.win, *base = U + L.base, *sws = U + L.sws;
  uint32_t *tentry = J + L.tentry, *tbefore = J + L.tbefore;
  const uint64_t stride = nrec + 1;
  // equal-sized entries: the arithmetic chain, checked hop by hop; the
  // general walk below runs only when a check fails (ar[0] = 0)
  uint64_t *ar = U + L.ar;
  const uint32_t pg = static_cast<uint32_t>(std::min<uint64_t>(grid_for(nrec + 1, 256), 2048));
  if (mode != SegMode::kGeneralOnly) {
    ArithArgs aa{Pw, add, nrec, threshold, ends, d_nends, d_nrec, ar, blk_first, d_nblocks};
    aa.fail = fail;
    aa.fail_bit = mode == SegMode::kArithOnly ? kGuardSplitRedo : kGuardArithFail;
    seg_arith_kernel<<<1, kArThreads, 0, s>>>(aa);
    seg_arith_check_kernel<<<pg, 256, 0, s>>>(aa);
    if (mode == SegMode::kArithOnly) return hipGetLastError(); // a failed chain: *fail |= kGuardSplitRedo
  } else {
    ar = nullptr; // no verdict: the general walk runs
  }
  SegArgs a{Pw, add, nrec, threshold, ends, d_nends, J + L.J0, J + L.Fx, J + L.Fc, win, blk_first, d_nblocks,
            sws, scan_status_words(L.tiles), tentry, d_nrec, ar};
  seg_walk_kernel<<<static_cast<uint32_t>(L.tiles), kChThreads, 0, s>>>(a);
  // base[tiles] = node count
  hipError_t e = scan_any<ArrIn, kArrItems>(ArrIn{win}, L.tiles, 0, base, sws, s, true, 0, ar,
                                            LbFail{fail, kGuardLookback});
  if (e != hipSuccess) return e;
  const uint64_t *nn = base + L.tiles;
  NodeArgs na{J + L.Fx, J + L.Fc, base, nrec, L.tiles, J + L.Nx, J + L.Nc, J + L.Nt, d_nrec, ar};
  seg_node_kernel<<<static_cast<uint32_t>(L.tiles), 256, 0, s>>>(na);
  for (uint64_t k = 0; k + 1 < L.levels; k++)
    seg_npow_kernel<<<pg, 256, 0, s>>>(J + L.Nx + k * stride, J + L.Nc + k * stride, J + L.Nx + (k + 1) * stride,
                                       J + L.Nc + (k + 1) * stride, nn, ar);
  seg_nentry_kernel<<<grid_for(L.tiles, 256), 256, 0, s>>>(J + L.Nx, J + L.Nc, J + L.Nt, base,
                                                           static_cast<uint32_t>(L.levels), stride, nrec, d_nrec,
                                                           L.tiles, tentry, tbefore, blk_first, d_nblocks, ar);
  seg_emit_kernel<<<static_cast<uint32_t>(L.tiles), kChThreads, 0, s>>>(J + L.J0, nrec, d_nrec, tentry, tbefore,
                                                                        blk_first, ar);
  return hipGetLastError();
}

} // namespace sstc
