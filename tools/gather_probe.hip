// gather_probe.hip -- HBM rate of a plain copy whose source is scattered the
// way the compaction encode's large-block reads are (diagnostic, not the
// product).  Thread per 16 B destination chunk (the copy-probe style, the most
// memory-level parallelism a copy can have); the source of chunk c is
//   contiguous   c
//   permuted     perm[c / S] * S + c % S   (S-chunk pieces in random order)
//   misaligned   the permuted address + a per-piece 1..15 B skew (unaligned 16 B loads)
//   hipcc -O3 --offload-arch=gfx950 tools/gather_probe.hip -o /tmp/gather_probe && /tmp/gather_probe [MiB]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void gather(const unsigned char *src, u32x4 *dst, size_t n, const unsigned *perm,
                                               unsigned piece, int skew) {
  const size_t c = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x;
  if (c >= n) return;
  size_t s = c;
  unsigned k = 0;
  if (perm) {
    const size_t p = c / piece;
    s = static_cast<size_t>(perm[p]) * piece + c % piece;
    k = skew ? 1 + (perm[p] % 15) : 0;
  }
  u32x4 v;
  __builtin_memcpy(&v, src + 16 * s + k, 16);
  __builtin_nontemporal_store(v, dst + c);
}

// the same copy, but every wave of a resident grid copies one contiguous run of
// the destination (kU chunks per lane per round), as enc_piece_kernel does
template <int kU>
__global__ __launch_bounds__(256) void gather_runs(const unsigned char *src, u32x4 *dst, size_t n,
                                                   const unsigned *perm, unsigned piece) {
  const size_t W = static_cast<size_t>(gridDim.x) * 4, w = static_cast<size_t>(blockIdx.x) * 4 + threadIdx.x / 64;
  const size_t c0 = n * w / W, c1 = n * (w + 1) / W;
  const unsigned lane = threadIdx.x % 64;
  for (size_t b = c0; b < c1; b += 64 * kU) {
    u32x4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      size_t c = b + u * 64 + lane;
      c = c < c1 ? c : c1 - 1;
      const size_t p = c / piece;
      const size_t s = static_cast<size_t>(perm[p]) * piece + c % piece;
      __builtin_memcpy(&v[u], src + 16 * s + 1 + (perm[p] % 15), 16);
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const size_t c = b + u * 64 + lane;
      if (c < c1) __builtin_nontemporal_store(v[u], dst + c);
    }
  }
}

int main(int argc, char **argv) {
  const size_t mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 451;
  const size_t n = mib << 16; // 16 B chunks
  unsigned char *src;
  u32x4 *dst;
  if (hipMalloc(&src, 16 * n * 2 + 64) != hipSuccess || hipMalloc(&dst, 16 * n) != hipSuccess) return 1;
  hipMemset(src, 1, 16 * n * 2 + 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (unsigned piece : {64u, 1024u, 1792u}) { // 1 KiB, 16 KiB, 28 KiB pieces
    const size_t np = (n + piece - 1) / piece;
    std::vector<unsigned> h(2 * np); // pieces drawn from a source twice the size (40 % kept)
    std::iota(h.begin(), h.end(), 0u);
    std::shuffle(h.begin(), h.end(), std::mt19937(7));
    h.resize(np);
    unsigned *perm;
    hipMalloc(&perm, 4 * np);
    hipMemcpy(perm, h.data(), 4 * np, hipMemcpyHostToDevice);
    for (int mode = 0; mode < 3; mode++) {
      if (mode == 0 && piece != 64u) continue;
      const unsigned *pp = mode ? perm : nullptr;
      float best = 1e30f;
      for (int it = 0; it < 6; it++) {
        hipEventRecord(e0);
        gather<<<static_cast<unsigned>((n + 255) / 256), 256>>>(src, dst, n, pp, piece, mode == 2);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (it) best = std::min(best, ms);
      }
      const char *name[3] = {"contiguous", "permuted", "misaligned"};
      printf("%-10s piece %5u B: %7.1f us  %.2f TB/s (read + write)\n", name[mode], 16 * piece, best * 1e3,
             2.0 * 16 * n / (best * 1e-3) / 1e12);
    }
    for (unsigned grid : {1024u, 1536u}) {
      float best = 1e30f;
      for (int it = 0; it < 6; it++) {
        hipEventRecord(e0);
        gather_runs<4><<<grid, 256>>>(src, dst, n, perm, piece);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (it) best = std::min(best, ms);
      }
      printf("wave runs  piece %5u B grid %u: %7.1f us  %.2f TB/s (read + write, misaligned)\n", 16 * piece, grid,
             best * 1e3, 2.0 * 16 * n / (best * 1e-3) / 1e12);
    }
    hipFree(perm);
  }
  return 0;
}
