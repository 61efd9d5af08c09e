// sstc_device.h — device-side helpers for the SST block codec kernels (gfx950).
//
// Byte-format facts used everywhere (reference sstable/block_builder.h:14-57):
// every multi-byte field is little-endian and sits at an arbitrary byte offset
// (blocks are packed back-to-back, fields follow variable-length keys), so all
// field reads go through the unaligned helpers below: two or three aligned
// dword reads + v_alignbyte_b32, never a misaligned wide access.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sstc {

constexpr uint32_t kWave = 64;
constexpr uint32_t kNoValue = 0xFFFFFFFFu;
constexpr uint32_t kTypePut = 0, kTypeDeleted = 1;
constexpr uint32_t kMaxKey = 4096;

enum BlkStatus : uint32_t {
  kBlkOk = 0,
  kBlkTooSmall = 1,
  kBlkEmpty = 2,
  kBlkOffsetsRange = 3,
  kBlkEntryRange = 4,
  kBlkBadType = 5,
  kBlkKeyTooLong = 6,
  kBlkTooLarge = 7,
  kBlkNoRoom = 8,
  kBlkCountMismatch = 9,
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// wave-uniform value -> SGPR (tells the compiler the value is uniform)
__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// ---- XCD-aware workgroup order ---------------------------------------------
// Workgroups are dispatched round-robin over the 8 XCDs (WG i runs on XCD
// i % 8), each with its own L2.  Remapping so that XCD x owns one contiguous
// range of logical workgroups keeps neighbouring blocks -- which share the
// cache lines at their boundaries -- inside one L2.  Bijective for any grid.
constexpr uint32_t kNumXcd = 8;
__device__ __forceinline__ uint32_t xcd_logical_block(uint32_t i, uint32_t n) {
  const uint32_t q = n / kNumXcd, r = n % kNumXcd, x = i % kNumXcd, k = i / kNumXcd;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

// XCD-chunked order for grids sized by a bound (the real count is on the
// device): within every run of kNumXcd * C workgroups, XCD x (= i % 8, the
// dispatch round robin) takes the x-th chunk of C consecutive logical ids, so
// neighbouring ids run at the same time behind one L2; a last partial run
// keeps dispatch order (workgroups past the real count leave)
__device__ __forceinline__ uint32_t xcd_chunk_block(uint32_t i, uint32_t n, uint32_t C) {
  const uint32_t run = kNumXcd * C, r0 = i / run * run;
  if (r0 + run > n) return i;
  const uint32_t j = i - r0;
  return r0 + (j % kNumXcd) * C + j / kNumXcd;
}

// ---- LDS image reads / writes at arbitrary byte offsets ---------------------
// Reads: aligned dwords + v_alignbyte (the image is padded by >= 16 bytes past
// its last byte).  gfx950 runs LDS in unaligned mode (the compiler's default
// target features unaligned-access-mode + unaligned-ds-access), but single
// unaligned ds_read_b32 / b64 measured slower in the LDS-bound round trip
// (profiles/r03_ab/unaligned_lds.md).  Writes: one ds_write_b32 / b64 at any
// alignment (replacing up to 8 byte stores).
__device__ __forceinline__ uint32_t lds_u8(const uint8_t *img, uint32_t off) { return img[off]; }

__device__ __forceinline__ uint32_t lds_u32u(const uint8_t *img, uint32_t off) {
  const uint32_t *w = reinterpret_cast<const uint32_t *>(img + (off & ~3u));
  return __builtin_amdgcn_alignbyte(w[1], w[0], off & 3u);
}

__device__ __forceinline__ uint64_t lds_u64u(const uint8_t *img, uint32_t off) {
  const uint32_t *w = reinterpret_cast<const uint32_t *>(img + (off & ~3u));
  const uint32_t a = w[0], b = w[1], c = w[2], sh = off & 3u;
  const uint32_t lo = __builtin_amdgcn_alignbyte(b, a, sh);
  const uint32_t hi = __builtin_amdgcn_alignbyte(c, b, sh);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

__device__ __forceinline__ void lds_st_u64u(uint8_t *img, uint32_t off, uint64_t v) {
  __builtin_memcpy(img + off, &v, 8);
}
__device__ __forceinline__ void lds_st_u32u(uint8_t *img, uint32_t off, uint32_t v) {
  __builtin_memcpy(img + off, &v, 4);
}

// ---- global reads at arbitrary byte offsets ---------------------------------
// Only dwords that hold a requested byte are touched, so a field that ends at
// the last byte of an allocation never reads past it.  The aligned pointer is
// derived by pointer arithmetic (not an integer round trip), so the compiler
// keeps the global address space and emits global_load, not flat_load (a flat
// load is waited for with vmcnt(0) lgkmcnt(0)).
__device__ __forceinline__ uint32_t g_u8(const uint8_t *p) { return *p; }

__device__ __forceinline__ const uint32_t *align4_down(const uint8_t *p, uint32_t &sh) {
  sh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p) & 3u);
  return reinterpret_cast<const uint32_t *>(p - sh);
}

__device__ __forceinline__ uint32_t g_u32u(const uint8_t *p) {
  uint32_t sh;
  const uint32_t *w = align4_down(p, sh);
  const uint32_t lo = w[0];
  const uint32_t hi = sh ? w[1] : 0u;
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

__device__ __forceinline__ uint64_t g_u64u(const uint8_t *p) {
  uint32_t sh;
  const uint32_t *w = align4_down(p, sh);
  const uint32_t x = w[0], y = w[1];
  const uint32_t z = sh ? w[2] : 0u;
  const uint32_t lo = __builtin_amdgcn_alignbyte(y, x, sh);
  const uint32_t hi = __builtin_amdgcn_alignbyte(z, y, sh);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// ---- wave-level primitives (wave64) -----------------------------------------
// Inclusive scan by DPP (no LDS round trips): row_shr 1 / 2 / 4 / 8 inside each
// 16-lane row (a lane whose source is outside its row keeps the identity, 0),
// then row_bcast:15 into rows 1 and 3 and row_bcast:31 into rows 2 and 3.
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x111, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x112, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x114, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x118, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x142, 0xa, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x143, 0xc, 0xf, false));
  return v;
}

template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) { // lanes the DPP does not write read 0
  const uint32_t lo = static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(static_cast<uint32_t>(v)), kCtrl, kRowMask, 0xf, false));
  const uint32_t hi = static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(static_cast<uint32_t>(v >> 32)), kCtrl, kRowMask, 0xf, false));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v) { // as wave_incl_scan_u32
  v += dpp_u64<0x111, 0xf>(v);
  v += dpp_u64<0x112, 0xf>(v);
  v += dpp_u64<0x114, 0xf>(v);
  v += dpp_u64<0x118, 0xf>(v);
  v += dpp_u64<0x142, 0xa>(v);
  v += dpp_u64<0x143, 0xc>(v);
  return v;
}

// decoupled look-back status word: 2 flag bits (aggregate / inclusive) | 14-bit
// epoch | 48 value bits (scan_lookback_kernel, ck_filter_kernel)
constexpr uint64_t kLbAgg = 1ull << 62, kLbInc = 2ull << 62, kLbVal = (1ull << 48) - 1;
constexpr uint32_t kLbEpochShift = 48;
constexpr uint64_t kLbSpinLimit = 1ull << 24; // never reached unless a tile died

// Where a look-back that gave up (kLbSpinLimit: a predecessor tile never
// published, e.g. a workgroup dispatched out of id order) reports it, so the
// caller rejects the wrong prefix sums instead of using them: bit != 0 ORs the
// bit into *p (a compaction guard word), bit == 0 counts into *p (a context's
// error counter).  p == nullptr: not reported.
struct LbFail {
  unsigned long long *p = nullptr;
  unsigned long long bit = 0;
  __device__ void report() const {
    if (!p) return;
    if (bit) atomicOr(p, bit);
    else atomicAdd(p, 1ull);
  }
};

__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, uint32_t l) {
  return (static_cast<uint64_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), l)) << 32) |
         __builtin_amdgcn_readlane(static_cast<uint32_t>(v), l);
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (uint32_t d = kWave / 2; d > 0; d >>= 1) v += __shfl_xor(v, d, kWave);
  return v;
}

// One wave of tile `tile`: publishes the tile's total, looks back over the
// status words of the tiles before it (64 per round) until an inclusive one,
// publishes its own inclusive prefix and returns the exclusive prefix
// (wave-uniform; tile 0: 0).  Words of another epoch are not published yet.
__device__ __forceinline__ uint64_t lb_publish_lookback(uint64_t *status, uint64_t tile, uint64_t total,
                                                        uint32_t epoch, const LbFail &fail = LbFail{}) {
  const uint32_t lane = lane_id();
  const uint64_t tag = static_cast<uint64_t>(epoch) << kLbEpochShift;
  if (tile == 0) {
    if (lane == 0) __hip_atomic_store(&status[0], kLbInc | tag | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0) __hip_atomic_store(&status[tile], kLbAgg | tag | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t prefix = 0;
  int64_t p = static_cast<int64_t>(tile) - 1; // window [p - 63, p]
  uint64_t spins = 0;
  for (;;) {
    const int64_t q = p - static_cast<int64_t>(lane);
    uint64_t st = q >= 0 ? __hip_atomic_load(&status[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kLbInc | tag;
    if (((st >> kLbEpochShift) & 0x3FFFu) != epoch) st = 0; // a stale word: not published yet
    const uint64_t inc = __ballot((st >> 62) == 2);
    const uint32_t need = inc ? static_cast<uint32_t>(__ffsll(static_cast<long long>(inc))) : kWave;
    const uint64_t zero = __ballot((st >> 62) == 0 && lane < need);
    if (zero) {
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
    __hip_atomic_store(&status[tile], kLbInc | tag | (prefix + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return prefix;
}

// LDS writes of one lane are made visible to the other lanes of the SAME wave:
// LDS executes a wave's DS instructions in order, so only a compiler barrier
// and the lgkmcnt drain are needed (no s_barrier).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Big-endian key bytes (first byte most significant) masked to the first
// `keep` bytes (keep >= 8 keeps all 8).
__device__ __forceinline__ uint64_t key_prefix8(uint64_t be, uint32_t keep) {
  return keep >= 8 ? be : (be & (~0ull << (8 * (8 - keep))));
}

// One record's entry size (reference sstable/block_builder.cc:19-21).
__device__ __forceinline__ uint64_t entry_size(uint32_t key_len, uint32_t val_len) {
  return 13ull + key_len + (val_len != kNoValue ? 4ull + val_len : 0ull);
}

} // namespace sstc
