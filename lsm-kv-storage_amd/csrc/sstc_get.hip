// sstc_get.hip — batched point lookups (include/sstcodec.h sstc_get_batch):
// TableReader::GetValue without a block cache (sstable/table_reader.cc:
// 168-210) and BlockReader::GetValue (sstable/block_reader.cc:20-57).
//
// One wave per query.  The block search (GetBlockOffsetAndSize: first block
// whose largest key >= key) is a lower bound, so any search order gives the
// reference's answer: the wave probes 64 candidates per step (a 35 k-block
// table takes 3 steps instead of 16 dependent probes).  The in-block search is
// NOT order-free when a block holds equal keys (several versions of a key):
// the reference returns the first equal entry ITS probe sequence meets.  The
// wave therefore compares the query with every entry in parallel (lane per
// entry, results in LDS) and then replays the reference's exact
// left/right/mid sequence on those results, which costs no memory round trip.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/sstcodec.h"
#include "sstc_device.h"
#include "sstc_launch.h"

namespace sstc {
namespace {

constexpr uint32_t kGetWaves = 4;
constexpr uint32_t kGetCmp = 512; // entries per block compared in parallel (more: lane-0 search)
constexpr int8_t kCmpBad = 2;

__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

// std::string_view::compare (unsigned bytes, then length): -1 / 0 / 1
__device__ int cmp_bytes(const uint8_t *a, uint32_t la, const uint8_t *b, uint32_t lb) {
  const uint32_t m = la < lb ? la : lb;
  uint32_t i = 0;
  for (; i + 4 <= m; i += 4) {
    const uint32_t x = bswap32(g_u32u(a + i)), y = bswap32(g_u32u(b + i));
    if (x != y) return x < y ? -1 : 1;
  }
  for (; i < m; i++)
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return la < lb ? -1 : (la > lb ? 1 : 0);
}

// entry i of a block: compare its key with the query; kCmpBad when the entry
// is out of range (the reference would read outside its buffer)
__device__ int8_t probe_entry(const uint8_t *base, uint64_t offs, uint64_t i, const uint8_t *key, uint32_t kl) {
  const uint64_t s = g_u64u(base + offs + 16 * i);
  if (s > offs || offs - s < 5) return kCmpBad;
  const uint32_t t = base[s];
  const uint32_t ekl = g_u32u(base + s + 1);
  if (static_cast<uint64_t>(ekl) > offs - s - 5 || t > 1) return kCmpBad;
  return static_cast<int8_t>(cmp_bytes(base + s + 5, ekl, key, kl));
}

__global__ __launch_bounds__(kGetWaves *kWave) void get_kernel(GetArgs a) {
  __shared__ int8_t s_cmp[kGetWaves][kGetCmp];
  const uint32_t wave = uniform(threadIdx.x / kWave), lane = lane_id();
  const uint64_t q = static_cast<uint64_t>(blockIdx.x) * kGetWaves + wave;
  if (q >= a.nq) return;
  const uint32_t t = uniform(a.q_table[q]);
  const uint8_t *key = a.q_keys + a.q_key_off[q];
  const uint32_t kl = uniform(a.q_key_len[q]);
  uint32_t type = SSTC_GET_NOT_FOUND, vlen = 0;
  uint64_t voff = 0, blk = ~0ull;
  if (t < a.ntables) {
    const uint64_t b0 = uniform64(a.tfb[t]), b1 = uniform64(a.tfb[t + 1]);
    if (b0 < b1) {
      // lower bound over [b0, b1 - 1): first block whose largest key >= key,
      // b1 - 1 when none is (table_reader.cc:191-210)
      uint64_t lo = b0, hi = b1 - 1;
      while (lo < hi) {
        const uint64_t step = (hi - lo + kWave - 1) / kWave;
        const uint64_t x = lo + lane * step;
        bool p = true;
        if (x < hi) p = cmp_bytes(a.keys + a.lk_off[x], a.lk_len[x], key, kl) >= 0;
        const uint64_t m = __ballot(p);
        if (m == 0) {
          lo = lo + (kWave - 1) * step + 1;
          continue;
        }
        const uint32_t f = static_cast<uint32_t>(__ffsll(static_cast<long long>(m))) - 1;
        const uint64_t xf = lo + f * step;
        if (xf < hi) hi = xf;
        if (f > 0) lo = lo + (f - 1) * step + 1;
      }
      blk = lo;
      const uint8_t *base = a.src + a.blk_off[blk];
      const uint64_t L = uniform64(a.blk_len[blk]);
      uint64_t n = 0, offs = 0;
      bool ok = L >= 16;
      if (ok) {
        n = uniform64(g_u64u(base + L - 16));
        offs = uniform64(g_u64u(base + L - 8));
        ok = offs <= L - 16 && n <= (L - 16 - offs) / 16;
      }
      int64_t found = -1;
      if (!ok) {
        type = SSTC_GET_BAD_BLOCK;
      } else if (n <= kGetCmp) {
        for (uint64_t i0 = 0; i0 < n; i0 += kWave) {
          const uint64_t i = i0 + lane;
          if (i < n) s_cmp[wave][i] = probe_entry(base, offs, i, key, kl);
        }
        wave_lds_sync();
        // BlockReader::GetValue's probe sequence (block_reader.cc:24-54)
        int64_t left = 0, right = static_cast<int64_t>(n) - 1;
        while (left <= right) {
          const int64_t mid = left + (right - left) / 2;
          const int8_t c = s_cmp[wave][mid];
          if (c == kCmpBad) {
            type = SSTC_GET_BAD_BLOCK;
            break;
          }
          if (c == 0) {
            found = mid;
            break;
          }
          if (c < 0) left = mid + 1;
          else right = mid - 1;
        }
      } else {
        // very long blocks: the same sequence, probed one entry at a time
        int64_t left = 0, right = static_cast<int64_t>(n) - 1;
        while (left <= right) {
          const int64_t mid = left + (right - left) / 2;
          const int8_t c = probe_entry(base, offs, static_cast<uint64_t>(mid), key, kl);
          if (c == kCmpBad) {
            type = SSTC_GET_BAD_BLOCK;
            break;
          }
          if (c == 0) {
            found = mid;
            break;
          }
          if (c < 0) left = mid + 1;
          else right = mid - 1;
        }
      }
      if (found >= 0) {
        const uint64_t s = g_u64u(base + offs + 16 * static_cast<uint64_t>(found));
        const uint32_t ekl = g_u32u(base + s + 1);
        if (base[s] == 1) {
          type = SSTC_GET_DELETED;
        } else if (offs - s - 5 - ekl < 4) {
          type = SSTC_GET_BAD_BLOCK;
        } else {
          const uint32_t vl = g_u32u(base + s + 5 + ekl);
          if (static_cast<uint64_t>(vl) > offs - s - 9 - ekl) {
            type = SSTC_GET_BAD_BLOCK;
          } else {
            type = SSTC_GET_PUT;
            voff = a.blk_off[blk] + s + 9 + ekl;
            vlen = vl;
          }
        }
      }
    }
  }
  if (lane == 0) {
    a.out_type[q] = type;
    a.out_val_off[q] = voff;
    a.out_val_len[q] = vlen;
    if (a.out_block) a.out_block[q] = blk;
    if (type == SSTC_GET_BAD_BLOCK) atomicAdd(a.err_count, 1ull);
  }
}

} // namespace

hipError_t launch_get(const GetArgs &a, hipStream_t s) {
  if (a.nq)
    get_kernel<<<static_cast<uint32_t>((a.nq + kGetWaves - 1) / kGetWaves), kGetWaves * kWave, 0, s>>>(a);
  return hipGetLastError();
}

} // namespace sstc
