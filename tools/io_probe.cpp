// io_probe.cpp — host-side I/O costs that bound the drop-in MergeIterator path
// (maps of page-cache-hot SST files, H2D from them, D2H into pageable memory,
// pwrite + fsync of output-sized files).  Diagnostic only.
//   hipcc -O2 -std=c++20 tools/io_probe.cpp -o tools/io_probe -lpthread
//   tools/io_probe <dir> <files> <MiB per file> [writes|pin]   (writes: only the output-file section;
//   pin: only the page-locking section)
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e = (x);                                                                  \
    if (e != hipSuccess) std::printf("%s -> %s\n", #x, hipGetErrorString(e));            \
  } while (0)

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  const std::string dir = argv[1];
  const int nf = std::atoi(argv[2]);
  const size_t sz = std::strtoull(argv[3], nullptr, 10) << 20;
  std::vector<std::string> paths;
  {
    std::vector<uint8_t> buf(sz);
    for (size_t i = 0; i < sz; i++) buf[i] = static_cast<uint8_t>(i * 2654435761u >> 13);
    for (int f = 0; f < nf; f++) {
      paths.push_back(dir + "/in" + std::to_string(f) + ".sst");
      int fd = open(paths.back().c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
      if (write(fd, buf.data(), sz) != static_cast<ssize_t>(sz)) return 3;
      close(fd);
    }
  }
  const bool writes_only = argc > 4 && (std::string(argv[4]) == "writes" || std::string(argv[4]) == "pin");
  const bool pin_only = argc > 4 && std::string(argv[4]) == "pin";
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void *dev = nullptr;
  CK(hipMalloc(&dev, sz * nf));
  const double gib = static_cast<double>(sz) * nf / (1u << 30);
  auto map_all = [&](bool populate, std::vector<void *> &maps) {
    maps.assign(nf, nullptr);
    for (int f = 0; f < nf; f++) {
      int fd = open(paths[f].c_str(), O_RDONLY);
      maps[f] = mmap(nullptr, sz, PROT_READ, MAP_PRIVATE | (populate ? MAP_POPULATE : 0), fd, 0);
      close(fd);
    }
  };
  auto unmap_all = [&](std::vector<void *> &maps) {
    for (void *p : maps) munmap(p, sz);
  };
  std::vector<void *> maps;
  for (int rep = 0; rep < (writes_only ? 0 : 2); rep++) {
    double t0 = now();
    map_all(true, maps);
    double t1 = now();
    std::printf("mmap populate serial: %.1f ms (%.2f GiB)\n", (t1 - t0) * 1e3, gib);
    unmap_all(maps);
  }
  if (!writes_only) {
    maps.assign(nf, nullptr);
    double t0 = now();
    std::vector<std::thread> th;
    for (int f = 0; f < nf; f++)
      th.emplace_back([&, f] {
        int fd = open(paths[f].c_str(), O_RDONLY);
        maps[f] = mmap(nullptr, sz, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
        close(fd);
      });
    for (auto &t : th) t.join();
    std::printf("mmap populate %d threads: %.1f ms\n", nf, (now() - t0) * 1e3);
    // pageable H2D from the maps
    t0 = now();
    for (int f = 0; f < nf; f++) CK(hipMemcpyAsync(static_cast<char *>(dev) + f * sz, maps[f], sz, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    double t1 = now();
    std::printf("H2D pageable from maps: %.1f ms = %.1f GB/s\n", (t1 - t0) * 1e3, sz * nf / (t1 - t0) / 1e9);
    // again
    t0 = now();
    for (int f = 0; f < nf; f++) CK(hipMemcpyAsync(static_cast<char *>(dev) + f * sz, maps[f], sz, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    t1 = now();
    std::printf("H2D pageable from maps (2nd): %.1f ms = %.1f GB/s\n", (t1 - t0) * 1e3, sz * nf / (t1 - t0) / 1e9);
    // 4 threads, own streams
    t0 = now();
    th.clear();
    for (int q = 0; q < 4; q++)
      th.emplace_back([&, q] {
        hipStream_t sq;
        CK(hipStreamCreateWithFlags(&sq, hipStreamNonBlocking));
        for (int f = q; f < nf; f += 4)
          CK(hipMemcpyAsync(static_cast<char *>(dev) + f * sz, maps[f], sz, hipMemcpyHostToDevice, sq));
        CK(hipStreamSynchronize(sq));
        CK(hipStreamDestroy(sq));
      });
    for (auto &t : th) t.join();
    t1 = now();
    std::printf("H2D pageable 4 threads: %.1f ms = %.1f GB/s\n", (t1 - t0) * 1e3, sz * nf / (t1 - t0) / 1e9);
    // register read-only
    for (unsigned flags : {unsigned(hipHostRegisterReadOnly), unsigned(hipHostRegisterDefault)}) {
      t0 = now();
      bool ok = true;
      for (int f = 0; f < nf; f++) {
        hipError_t e = hipHostRegister(maps[f], sz, flags);
        if (e != hipSuccess) {
          std::printf("hipHostRegister(flags %u) file %d: %s\n", flags, f, hipGetErrorString(e));
          ok = false;
          (void)hipGetLastError();
          break;
        }
      }
      t1 = now();
      std::printf("hipHostRegister flags %u: %.1f ms ok %d\n", flags, (t1 - t0) * 1e3, ok);
      if (!ok) continue;
      t0 = now();
      for (int f = 0; f < nf; f++) CK(hipMemcpyAsync(static_cast<char *>(dev) + f * sz, maps[f], sz, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      t1 = now();
      std::printf("H2D registered: %.1f ms = %.1f GB/s\n", (t1 - t0) * 1e3, sz * nf / (t1 - t0) / 1e9);
      t0 = now();
      for (int f = 0; f < nf; f++) CK(hipHostUnregister(maps[f]));
      std::printf("hipHostUnregister: %.1f ms\n", (now() - t0) * 1e3);
    }
    unmap_all(maps);
  }
  // pread into a pinned ring + H2D (what sstc_compact_files does), single thread
  if (!writes_only) {
    double t0 = now();
    void *pin = nullptr;
    CK(hipHostMalloc(&pin, 64 << 20, hipHostMallocDefault));
    double t1 = now();
    std::printf("hipHostMalloc 64 MiB: %.1f ms\n", (t1 - t0) * 1e3);
    t0 = now();
    void *pin2 = nullptr;
    CK(hipHostMalloc(&pin2, size_t(1) << 30, hipHostMallocDefault));
    t1 = now();
    std::printf("hipHostMalloc 1 GiB: %.1f ms\n", (t1 - t0) * 1e3);
    t0 = now();
    CK(hipHostFree(pin2));
    std::printf("hipHostFree 1 GiB: %.1f ms\n", (now() - t0) * 1e3);
    CK(hipHostFree(pin));
  }
  // D2H of 256 MiB into pageable memory
  if (!writes_only) {
    const size_t n = size_t(256) << 20;
    double t0 = now();
    std::vector<uint8_t> h(n);
    double t1 = now();
    std::printf("vector 256 MiB alloc+zero: %.1f ms\n", (t1 - t0) * 1e3);
    t0 = now();
    CK(hipMemcpyAsync(h.data(), dev, n, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    t1 = now();
    std::printf("D2H 256 MiB pageable (touched): %.1f ms = %.1f GB/s\n", (t1 - t0) * 1e3, n / (t1 - t0) / 1e9);
    uint8_t *raw = static_cast<uint8_t *>(std::malloc(n));
    t0 = now();
    CK(hipMemcpyAsync(raw, dev, n, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    t1 = now();
    std::printf("D2H 256 MiB pageable (fresh malloc): %.1f ms = %.1f GB/s\n", (t1 - t0) * 1e3, n / (t1 - t0) / 1e9);
    std::free(raw);
  }
  // output files: 44 MB pwrite + fsync, serial and split over threads
  {
    const size_t n = 44u << 20;
    std::vector<uint8_t> img(n, 7);
    for (int rep = 0; rep < 4; rep++) {
      std::string p = dir + "/out" + std::to_string(rep) + ".sst";
      int fd = open(p.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
      double t0 = now();
      (void)!pwrite(fd, img.data(), n, 0);
      double t1 = now();
      fsync(fd);
      double t2 = now();
      close(fd);
      std::printf("44 MiB pwrite %.2f ms fsync %.2f ms\n", (t1 - t0) * 1e3, (t2 - t1) * 1e3);
    }
    for (int rep = 0; rep < 3; rep++) {
      std::string p = dir + "/outp" + std::to_string(rep) + ".sst";
      int fd = open(p.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
      double t0 = now();
      std::vector<std::thread> th;
      for (int q = 0; q < 4; q++)
        th.emplace_back([&, q] { (void)!pwrite(fd, img.data() + q * (n / 4), n / 4, q * (n / 4)); });
      for (auto &t : th) t.join();
      double t1 = now();
      fsync(fd);
      double t2 = now();
      close(fd);
      std::printf("44 MiB pwrite x4 threads %.2f ms fsync %.2f ms\n", (t1 - t0) * 1e3, (t2 - t1) * 1e3);
    }
  }
  // page locking: hipHostMalloc against an anonymous map (populated) +
  // hipHostRegister, alloc + free, and a 64 MiB H2D from each
  if (pin_only) {
    for (size_t mb : {size_t(1), size_t(8), size_t(32), size_t(64)}) {
      const size_t n = mb << 20;
      for (int rep = 0; rep < 2; rep++) {
        double t0 = now();
        void *p = nullptr;
        CK(hipHostMalloc(&p, n, hipHostMallocPortable));
        double t1 = now();
        CK(hipHostFree(p));
        double t2 = now();
        void *q = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
        double t3 = now();
        CK(hipHostRegister(q, n, hipHostRegisterPortable));
        double t4 = now();
        if (mb == 64) {
          double a = now();
          CK(hipMemcpyAsync(dev, q, n, hipMemcpyHostToDevice, s));
          CK(hipStreamSynchronize(s));
          double b = now();
          std::printf("  H2D 64 MiB from registered map: %.2f ms = %.1f GB/s\n", (b - a) * 1e3, n / (b - a) / 1e9);
        }
        CK(hipHostUnregister(q));
        munmap(q, n);
        double t5 = now();
        std::printf("%zu MiB: hipHostMalloc %.2f ms (free %.2f) | mmap+populate %.2f + hipHostRegister %.2f ms "
                    "(unregister+munmap %.2f)\n", mb, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3,
                    (t4 - t3) * 1e3, (t5 - t4) * 1e3);
      }
    }
    CK(hipFree(dev));
    std::printf("done\n");
    return 0;
  }
  // O_DIRECT writes of a 44 MB table image from page-locked memory (what
  // TableBuilder::Finish does), one pwrite, 1 MiB / 8 MiB pieces, and the
  // image split over 2 / 4 / 8 threads writing their slices at once
  {
    const size_t n = 44u << 20;
    uint8_t *img = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void **>(&img), n, hipHostMallocDefault));
    std::memset(img, 7, n);
    auto run = [&](const char *what, int threads, size_t piece) {
      for (int rep = 0; rep < 3; rep++) {
        std::string p = dir + "/outd" + std::to_string(rep) + ".sst";
        int fd = open(p.c_str(), O_CREAT | O_TRUNC | O_WRONLY | O_DIRECT, 0644);
        if (fd < 0) {
          std::printf("O_DIRECT open refused\n");
          return;
        }
        double t0 = now();
        std::vector<std::thread> th;
        const size_t slice = n / threads;
        for (int q = 0; q < threads; q++)
          th.emplace_back([&, q] {
            for (size_t at = q * slice; at < (q + 1) * slice; at += piece)
              (void)!pwrite(fd, img + at, std::min(piece, (q + 1) * slice - at), at);
          });
        for (auto &t : th) t.join();
        double t1 = now();
        fsync(fd);
        double t2 = now();
        close(fd);
        std::printf("44 MiB O_DIRECT %s: pwrite %.2f ms (%.1f GB/s) fsync %.2f ms\n", what, (t1 - t0) * 1e3,
                    n / (t1 - t0) / 1e9, (t2 - t1) * 1e3);
      }
    };
    run("1 pwrite", 1, n);
    run("8 MiB pieces", 1, 8u << 20);
    run("1 MiB pieces", 1, 1u << 20);
    run("2 threads", 2, n);
    run("4 threads", 4, n);
    run("8 threads", 8, n);
    run("4 threads 1 MiB pieces", 4, 1u << 20);
    CK(hipHostFree(img));
  }
  CK(hipFree(dev));
  std::printf("done\n");
  return 0;
}
