// sstc_get.hip — batched point lookups (include/sstcodec.h sstc_get_batch):
// TableReader::GetValue without a block cache (sstable/table_reader.cc:
// 168-210) and BlockReader::GetValue (sstable/block_reader.cc:20-57).
//
// One thread per query, each running the reference's two binary searches
// with the reference's exact left/right/mid sequences: the in-block search is
// order-sensitive when a block holds several versions of a key (the first
// equal entry the probe sequence meets is returned), so it is not replaced by
// a different search order.  A wave keeps 64 independent lookups in flight,
// which hides the dependent-load latency of each search.
//
// Every global read is bounds-checked against the buffer sizes the caller
// passes (src, index keys, query keys): a corrupt index, trailer or offset
// entry answers SSTC_GET_BAD_BLOCK instead of reading outside the buffers.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/sstcodec.h"
#include "sstc_device.h"
#include "sstc_launch.h"

namespace sstc {
namespace {

constexpr uint32_t kGetThreads = 256;

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

struct Found {
  uint32_t type, vlen;
  uint64_t voff;
};

// BlockReader::GetValue (block_reader.cc:20-57) on the block at src[bo, bo+L)
__device__ Found block_get(const uint8_t *src, uint64_t bo, uint64_t L, const uint8_t *key, uint32_t kl) {
  Found r{SSTC_GET_NOT_FOUND, 0, 0};
  const uint8_t *base = src + bo;
  if (L < 16) return {SSTC_GET_BAD_BLOCK, 0, 0};
  const uint64_t n = g_u64u(base + L - 16), offs = g_u64u(base + L - 8);
  if (offs > L - 16 || n > (L - 16 - offs) / 16) return {SSTC_GET_BAD_BLOCK, 0, 0};
  int64_t left = 0, right = static_cast<int64_t>(n) - 1;
  while (left <= right) {
    const int64_t mid = left + (right - left) / 2;
    const uint64_t s = g_u64u(base + offs + 16 * static_cast<uint64_t>(mid));
    if (s > offs || offs - s < 5) return {SSTC_GET_BAD_BLOCK, 0, 0};
    const uint32_t t = base[s];
    const uint32_t ekl = g_u32u(base + s + 1);
    if (static_cast<uint64_t>(ekl) > offs - s - 5 || t > 1) return {SSTC_GET_BAD_BLOCK, 0, 0};
    const int c = cmp_bytes(base + s + 5, ekl, key, kl);
    if (c == 0) {
      if (t == 1) return {SSTC_GET_DELETED, 0, 0};
      if (offs - s - 5 - ekl < 4) return {SSTC_GET_BAD_BLOCK, 0, 0};
      const uint32_t vl = g_u32u(base + s + 5 + ekl);
      if (static_cast<uint64_t>(vl) > offs - s - 9 - ekl) return {SSTC_GET_BAD_BLOCK, 0, 0};
      return {SSTC_GET_PUT, vl, bo + s + 9 + ekl};
    }
    if (c < 0) left = mid + 1;
    else right = mid - 1;
  }
  return r;
}

__global__ __launch_bounds__(kGetThreads) void get_kernel(GetArgs a) {
  const uint64_t q = static_cast<uint64_t>(blockIdx.x) * kGetThreads + threadIdx.x;
  if (q >= a.nq) return;
  Found r{SSTC_GET_NOT_FOUND, 0, 0};
  uint64_t blk = ~0ull;
  const uint32_t t = a.q_table[q];
  const uint64_t koff = a.q_key_off[q];
  const uint32_t kl = a.q_key_len[q];
  if (koff > a.q_keys_bytes || kl > a.q_keys_bytes - koff) {
    r.type = SSTC_GET_BAD_BLOCK;
  } else if (t < a.ntables) {
    const uint8_t *key = a.q_keys + koff;
    const uint64_t total = a.tfb[a.ntables];
    const uint64_t b0 = a.tfb[t], b1 = a.tfb[t + 1];
    if (b0 > b1 || b1 > total) {
      r.type = SSTC_GET_BAD_BLOCK;
    } else if (b0 < b1) {
      // GetBlockOffsetAndSize (table_reader.cc:191-210)
      int64_t left = 0, right = static_cast<int64_t>(b1 - b0) - 1;
      bool bad = false;
      while (left < right) {
        const int64_t mid = left + (right - left) / 2;
        const uint64_t x = b0 + static_cast<uint64_t>(mid);
        const uint64_t ko = a.lk_off[x];
        const uint32_t kn = a.lk_len[x];
        if (ko > a.keys_bytes || kn > a.keys_bytes - ko) {
          bad = true;
          break;
        }
        if (cmp_bytes(a.keys + ko, kn, key, kl) >= 0) right = mid;
        else left = mid + 1;
      }
      blk = b0 + static_cast<uint64_t>(right);
      const uint64_t bo = a.blk_off[blk], L = a.blk_len[blk];
      if (bad || bo > a.src_bytes || L > a.src_bytes - bo) r.type = SSTC_GET_BAD_BLOCK;
      else r = block_get(a.src, bo, L, key, kl);
    }
  }
  a.out_type[q] = r.type;
  a.out_val_off[q] = r.voff;
  a.out_val_len[q] = r.vlen;
  if (a.out_block) a.out_block[q] = blk;
  if (r.type == SSTC_GET_BAD_BLOCK) atomicAdd(a.err_count, 1ull);
}

} // namespace

hipError_t launch_get(const GetArgs &a, hipStream_t s) {
  if (a.nq) get_kernel<<<static_cast<uint32_t>((a.nq + kGetThreads - 1) / kGetThreads), kGetThreads, 0, s>>>(a);
  return hipGetLastError();
}

} // namespace sstc
