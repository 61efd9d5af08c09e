// copy_probe.hip — HBM copy ceiling on this box (diagnostic, not the product):
// how fast can a plain 16 B/lane copy move the bytes rt_kernel moves?
//   hipcc -O3 --offload-arch=gfx950 tools/copy_probe.hip -o tools/copy_probe && tools/copy_probe [MiB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_kernel(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, size_t n) {
  const size_t base = (static_cast<size_t>(blockIdx.x) * 256 * U) + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const size_t i = base + static_cast<size_t>(u) * 256;
    if (i < n) v[u] = NT ? __builtin_nontemporal_load(s + i) : s[i];
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    const size_t i = base + static_cast<size_t>(u) * 256;
    if (i < n) {
      if (NT) __builtin_nontemporal_store(v[u], d + i);
      else d[i] = v[u];
    }
  }
}

template <int U, bool NT> void run(const u32x4 *s, u32x4 *d, size_t n, const char *name) {
  const unsigned grid = static_cast<unsigned>((n + 256 * U - 1) / (256 * U));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; w++) copy_kernel<U, NT><<<grid, 256>>>(s, d, n);
  const int reps = 20;
  hipEventRecord(e0);
  for (int r = 0; r < reps; r++) copy_kernel<U, NT><<<grid, 256>>>(s, d, n);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  printf("%-22s %8.1f us  %7.1f GB/s (read+write)\n", name, ms * 1e3, 2.0 * n * 16 / (ms * 1e-3) / 1e9);
}

int main(int argc, char **argv) {
  const size_t mib = argc > 1 ? atol(argv[1]) : 1047;
  const size_t n = mib * (1 << 20) / 16;
  u32x4 *s, *d;
  if (hipMalloc(&s, n * 16) != hipSuccess || hipMalloc(&d, n * 16) != hipSuccess) return 1;
  hipMemset(s, 1, n * 16);
  printf("bytes per side: %zu\n", n * 16);
  run<1, false>(s, d, n, "u1");
  run<4, false>(s, d, n, "u4");
  run<8, false>(s, d, n, "u8");
  run<1, true>(s, d, n, "u1 nt");
  run<4, true>(s, d, n, "u4 nt");
  run<8, true>(s, d, n, "u8 nt");
  run<16, true>(s, d, n, "u16 nt");
  hipFree(s);
  hipFree(d);
  return 0;
}
