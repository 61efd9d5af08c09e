// fetch_calib.hip — calibrates rocprofv3 FETCH_SIZE against known byte counts
// for the access widths the compaction job's kernels use (MI355X_MICROARCH.md:
// "FETCH_SIZE reports exactly 1/2 of the bytes of a wide coalesced streaming
// read (16 B/lane) ... other access widths are uncalibrated").
//
//   hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE -d out -o f --output-format csv -- tools/fetch_calib
//
// Each kernel reads a 1 GiB buffer (past the 256 MiB Infinity Cache) in one
// pattern and writes one word per workgroup; the program prints the bytes each
// kernel reads (the denominator) in dispatch order.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

constexpr uint64_t kBytes = 1ull << 30;

template <class T>
__global__ __launch_bounds__(256) void stream_read(const T *__restrict__ p, uint64_t n, uint64_t *out) {
  uint64_t acc = 0;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const T v = p[i];
    acc += reinterpret_cast<const uint32_t *>(&v)[0];
  }
  if (acc == 0x12345678ull) out[blockIdx.x] = acc; // never true: keeps the loads
}

// one `W`-byte read per 128 B line, lines visited in a scattered order
// (a multiplicative permutation of the line index), every line once
template <int W>
__global__ __launch_bounds__(256) void gather_lines(const uint8_t *__restrict__ p, uint64_t lines, uint64_t mul,
                                                    uint64_t *out) {
  uint64_t acc = 0;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < lines;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint64_t line = (i * mul) & (lines - 1);
    const uint8_t *q = p + line * 128 + 32; // inside the line
    if constexpr (W == 4) acc += *reinterpret_cast<const uint32_t *>(q);
    else if constexpr (W == 8) acc += *reinterpret_cast<const uint64_t *>(q);
    else acc += reinterpret_cast<const uint4 *>(q)->x;
  }
  if (acc == 0x12345678ull) out[blockIdx.x] = acc;
}

int main() {
  uint8_t *buf = nullptr;
  uint64_t *out = nullptr;
  CK(hipMalloc(&buf, kBytes));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(buf, 1, kBytes));
  CK(hipDeviceSynchronize());
  const uint32_t grid = 2048;
  const uint64_t lines = kBytes / 128;
  std::printf("kernel bytes_read\n");
  stream_read<uint4><<<grid, 256>>>(reinterpret_cast<const uint4 *>(buf), kBytes / 16, out);
  std::printf("stream16 %llu\n", (unsigned long long)kBytes);
  stream_read<uint2><<<grid, 256>>>(reinterpret_cast<const uint2 *>(buf), kBytes / 8, out);
  std::printf("stream8 %llu\n", (unsigned long long)kBytes);
  stream_read<uint32_t><<<grid, 256>>>(reinterpret_cast<const uint32_t *>(buf), kBytes / 4, out);
  std::printf("stream4 %llu\n", (unsigned long long)kBytes);
  // the line each gather touches is the unit the memory side can fetch:
  // report the touched lines' bytes (128 B) -- a 64 B sector fetch would show 1/2
  gather_lines<4><<<grid, 256>>>(buf, lines, 0x9E3779B1ull, out);
  std::printf("gather4_lines %llu\n", (unsigned long long)(lines * 128));
  gather_lines<8><<<grid, 256>>>(buf, lines, 0x9E3779B1ull, out);
  std::printf("gather8_lines %llu\n", (unsigned long long)(lines * 128));
  gather_lines<16><<<grid, 256>>>(buf, lines, 0x9E3779B1ull, out);
  std::printf("gather16_lines %llu\n", (unsigned long long)(lines * 128));
  CK(hipDeviceSynchronize());
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
