// compact_files.cpp — file-to-file compaction (include/sstcodec.h
// sstc_compact_files): the I/O half of Compact::DoCompactJob
// (db/compact.cc:232-322, io/linux_file.cc:138-195) around the device job
// sstc_compact.
//
//   index   one thread per input file preads the 40 B footer and the meta
//           section and walks it (TableReader, table_reader.cc:52-156);
//   load    the data sections are read in 16 MiB chunks by io_threads into
//           pinned memory and every finished chunk is copied H2D at once, so
//           file reads overlap PCIe;
//   compact sstc_compact (device; synchronous);
//   store   every output SST is copied D2H as one async copy with an event;
//           writer threads wait for their table's event, pwrite, fsync.
//
// The reference writes each block with three pwrite64 and fsyncs per output
// SST (table_builder.cc:62-99,147-211); here each output SST is one pwrite.
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "sstcodec.h"

extern "C" int sstc__fail(int code, const char *what); // sstc_api.hip: sets sstc_last_error_string
extern "C" int sstc__ctx_device(const sstc_ctx *ctx);   // sstc_api.hip: the device a context is bound to
extern "C" int sstc__ctx_sync(sstc_ctx *ctx);           // sstc_api.hip: synchronize the context's stream

struct sstc_pipe {
  sstc_ctx *ctx = nullptr;
  int device = 0;
  uint32_t io_threads = 8;
  hipStream_t stream = nullptr;
  uint8_t *h_in = nullptr, *h_out = nullptr, *d_src = nullptr, *d_dst = nullptr;
  uint64_t *d_idx = nullptr;
  uint64_t cap_h_in = 0, cap_h_out = 0, cap_d_src = 0, cap_d_dst = 0, cap_d_idx = 0;
  // test hooks (sstc__pipe_set_test_caps): the first attempt's output
  // capacity and the retry's size bound, 0 = the production values
  uint64_t test_first_cap = 0, test_bound = 0;
};

// test hook, not in the header: force the first attempt's output capacity
// (first_cap) and the retry's size bound (bound); 0 restores the production value
extern "C" int sstc__pipe_set_test_caps(sstc_pipe *pipe, uint64_t first_cap, uint64_t bound) {
  if (!pipe) return SSTC_E_INVALID_ARG;
  pipe->test_first_cap = first_cap;
  pipe->test_bound = bound;
  return SSTC_OK;
}

namespace {

using clk = std::chrono::steady_clock;
constexpr uint64_t kChunk = 16ull << 20;

double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }

uint32_t get32(const uint8_t *p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
uint64_t get64(const uint8_t *p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}

bool pread_full(int fd, uint8_t *buf, uint64_t size, uint64_t off) {
  while (size > 0) {
    const ssize_t r = ::pread(fd, buf, size, static_cast<off_t>(off));
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    buf += r;
    size -= static_cast<uint64_t>(r);
    off += static_cast<uint64_t>(r);
  }
  return true;
}

bool pwrite_full(int fd, const uint8_t *buf, uint64_t size, uint64_t off) {
  while (size > 0) {
    const ssize_t w = ::pwrite(fd, buf, size, static_cast<off_t>(off));
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return false;
    buf += w;
    size -= static_cast<uint64_t>(w);
    off += static_cast<uint64_t>(w);
  }
  return true;
}

int grow_pinned(uint8_t *&p, uint64_t &cap, uint64_t need) {
  if (p && need <= cap) return 0;
  if (p) (void)hipHostFree(p);
  p = nullptr;
  cap = 0;
  const uint64_t n = need + need / 8 + 4096;
  if (hipHostMalloc(reinterpret_cast<void **>(&p), n, hipHostMallocDefault) != hipSuccess) {
    p = nullptr;
    return -1;
  }
  cap = n;
  return 0;
}

template <class T> int grow_dev(T *&p, uint64_t &cap, uint64_t need_elems) {
  if (p && need_elems <= cap) return 0;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  const uint64_t n = need_elems + need_elems / 8 + 1024;
  if (hipMalloc(reinterpret_cast<void **>(&p), n * sizeof(T)) != hipSuccess) {
    p = nullptr;
    return -1;
  }
  cap = n;
  return 0;
}

struct InFile {
  int fd = -1;
  uint64_t bytes = 0, meta_off = 0, base = 0;
  std::vector<uint64_t> off, len;
  bool ok = false;
};

// DecodeExtraInfo + FetchBlockIndexInfo (table_reader.cc:52-156)
void index_file(InFile &f) {
  uint8_t foot[40];
  if (f.bytes < 40 || !pread_full(f.fd, foot, 40, f.bytes - 40)) return;
  const uint64_t nb = get64(foot), moff = get64(foot + 8), mlen = get64(foot + 16);
  if (moff > f.bytes - 40 || mlen > f.bytes - 40 - moff) return;
  std::vector<uint8_t> meta(mlen);
  if (mlen && !pread_full(f.fd, meta.data(), mlen, moff)) return;
  f.off.reserve(nb);
  f.len.reserve(nb);
  uint64_t p = 0;
  for (uint64_t i = 0; i < nb; i++) {
    if (p + 4 > mlen) return;
    const uint64_t fk = get32(&meta[p]);
    if (p + 8 + fk > mlen) return;
    const uint64_t lk = get32(&meta[p + 4 + fk]);
    if (p + 24 + fk + lk > mlen) return;
    const uint64_t bo = get64(&meta[p + 8 + fk + lk]), bl = get64(&meta[p + 16 + fk + lk]);
    if (bo > moff || bl > moff - bo) return;
    f.off.push_back(bo);
    f.len.push_back(bl);
    p += 24 + fk + lk;
  }
  f.meta_off = moff;
  f.ok = true;
}

// smallest / largest key of a finished table image (its first and last meta
// entries: TableBuilder::GetSmallestKey/GetLargestKey, table_builder.h:118-125)
void table_keys(const uint8_t *img, uint64_t bytes, std::string &lo, std::string &hi) {
  lo.clear();
  hi.clear();
  if (bytes < 40) return;
  const uint8_t *foot = img + bytes - 40;
  const uint64_t nb = get64(foot), moff = get64(foot + 8);
  const uint8_t *m = img + moff;
  for (uint64_t i = 0; i < nb; i++) {
    const uint32_t fk = get32(m);
    const uint32_t lk = get32(m + 4 + fk);
    if (i == 0) lo.assign(reinterpret_cast<const char *>(m + 4), fk);
    if (i + 1 == nb) hi.assign(reinterpret_cast<const char *>(m + 8 + fk), lk);
    m += 24ull + fk + lk;
  }
}

struct FdGuard {
  std::vector<InFile> &files;
  ~FdGuard() {
    for (auto &f : files)
      if (f.fd >= 0) ::close(f.fd);
  }
};

} // namespace

extern "C" {

int sstc_pipe_create(sstc_ctx *ctx, uint32_t io_threads, sstc_pipe **out) {
  if (!ctx || !out) return sstc__fail(SSTC_E_INVALID_ARG, "sstc_pipe_create: NULL argument");
  *out = nullptr;
  // the pipe's stream and buffers live on the context's device, whatever the
  // calling thread's current device is
  const int dev = sstc__ctx_device(ctx);
  if (dev < 0 || hipSetDevice(dev) != hipSuccess) return sstc__fail(SSTC_E_NO_DEVICE, "no HIP device");
  sstc_pipe *p = new sstc_pipe();
  p->ctx = ctx;
  p->device = dev;
  p->io_threads = io_threads ? io_threads : 8;
  if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess) {
    delete p;
    return sstc__fail(SSTC_E_HIP, "sstc_pipe_create: hipStreamCreate");
  }
  *out = p;
  return SSTC_OK;
}

int sstc_pipe_destroy(sstc_pipe *p) {
  if (!p) return SSTC_OK;
  (void)hipSetDevice(p->device);
  (void)hipStreamSynchronize(p->stream);
  if (p->h_in) (void)hipHostFree(p->h_in);
  if (p->h_out) (void)hipHostFree(p->h_out);
  for (void *d : {static_cast<void *>(p->d_src), static_cast<void *>(p->d_dst), static_cast<void *>(p->d_idx)})
    if (d) (void)hipFree(d);
  (void)hipStreamDestroy(p->stream);
  delete p;
  return SSTC_OK;
}

} // extern "C"

namespace {

// one compaction's outputs (sstc_file_out with key offsets into keys)
struct FilesOut {
  std::vector<sstc_file_out> outs;
  std::string keys;
  sstc_files_timing tm{};
};

// first_id(nt, key_bytes, id): called once the output tables are in host
// memory (their count nt and the bytes of their smallest + largest keys,
// what the caller's outs / key_arena receive, are known) and before any
// output file is touched; sets the first output id or returns an error code
// (then nothing is written)
using FirstId = std::function<int(uint64_t, uint64_t, uint64_t &)>;

constexpr uint64_t kDirectAlign = 4096;

// One output table: created, or opened WITHOUT O_TRUNC when the path exists
// (io/linux_file.cc:99-119, LinuxWriteOnlyFile::Open: a longer stale file
// keeps its tail past the new table's bytes, as the reference's compaction
// leaves it), then written at offset 0.  With fsync on, the 4 KiB-aligned
// part goes through a second O_DIRECT descriptor straight from the pinned
// image (no page-cache copy before the flush: the fsync'd buffered write of a
// 44 MB table cost its memcpy on top of the device write), the tail through
// the ordinary one; a file system that refuses O_DIRECT takes buffered
// writes.  img must be 4 KiB aligned for the direct part.
bool write_table(const std::string &path, const uint8_t *img, uint64_t bytes, bool do_fsync) {
  ::chmod(path.c_str(), 0644);
  const bool create = ::access(path.c_str(), F_OK) != 0;
  const int fd = ::open(path.c_str(), create ? (O_WRONLY | O_CREAT | O_TRUNC) : O_WRONLY, 0644);
  if (fd < 0) return false;
  uint64_t done = 0;
  if (do_fsync && !(reinterpret_cast<uintptr_t>(img) & (kDirectAlign - 1))) {
    const int dfd = ::open(path.c_str(), O_WRONLY | O_DIRECT | O_CLOEXEC);
    const uint64_t a = bytes & ~(kDirectAlign - 1);
    if (dfd >= 0) {
      if (a && pwrite_full(dfd, img, a, 0)) done = a;
      ::close(dfd);
    }
  }
  bool ok = done == bytes || pwrite_full(fd, img + done, bytes - done, done);
  if (ok && do_fsync && ::fsync(fd) < 0) ok = false;
  ::close(fd);
  return ok;
}

int compact_files_impl(sstc_pipe *pipe, const char *const *in_paths, const uint64_t *in_file_sizes, uint32_t n_in,
                       const char *out_prefix, const FirstId &first_id, const sstc_compact_params *params,
                       uint32_t do_fsync, uint32_t max_outs, FilesOut &result) {
  if (hipSetDevice(pipe->device) != hipSuccess) return sstc__fail(SSTC_E_HIP, "hipSetDevice");
  const auto t0 = clk::now();
  hipStream_t s = pipe->stream;
  // error exits once copies may be in flight: drain the pipe's stream (and the
  // context's, after the device job) so the next call never frees or refills
  // pinned / device staging that a pending copy or kernel still reads
  auto bail = [&](int code, const char *what) {
    (void)hipStreamSynchronize(s);
    (void)sstc__ctx_sync(pipe->ctx);
    return sstc__fail(code, what);
  };

  // ---- index: footers + meta sections, one thread per file
  std::vector<InFile> files(n_in);
  FdGuard guard{files};
  for (uint32_t i = 0; i < n_in; i++) {
    files[i].fd = ::open(in_paths[i], O_RDONLY);
    if (files[i].fd < 0 || in_file_sizes[i] < 41)
      return sstc__fail(SSTC_E_INVALID_ARG, (std::string("cannot open SST ") + in_paths[i]).c_str());
    files[i].bytes = in_file_sizes[i] - 1; // GetFileSize() = bytes + 1
  }
  {
    std::vector<std::thread> th;
    for (auto &f : files) th.emplace_back(index_file, std::ref(f));
    for (auto &t : th) t.join();
  }
  uint64_t total = 0, nblocks = 0;
  std::vector<uint64_t> tfb(1, 0);
  for (uint32_t i = 0; i < n_in; i++) {
    if (!files[i].ok) return sstc__fail(SSTC_E_INVALID_ARG, (std::string("bad SST index: ") + in_paths[i]).c_str());
    files[i].base = total;
    total += (files[i].meta_off + 255) & ~uint64_t(255);
    nblocks += files[i].off.size();
    tfb.push_back(nblocks);
  }
  const auto t1 = clk::now();

  // ---- load: chunked preads into pinned memory, each chunk copied H2D when done
  const uint64_t idx_at = (total + 255) & ~uint64_t(255);
  if (grow_pinned(pipe->h_in, pipe->cap_h_in, idx_at + 16 * nblocks + 16) ||
      grow_dev(pipe->d_src, pipe->cap_d_src, total + 16))
    return sstc__fail(SSTC_E_NOMEM, "sstc_compact_files: input staging");
  struct Chunk {
    uint32_t file;
    uint64_t off, len;
  };
  std::vector<Chunk> chunks;
  for (uint32_t i = 0; i < n_in; i++)
    for (uint64_t o = 0; o < files[i].meta_off; o += kChunk)
      chunks.push_back({i, o, std::min(kChunk, files[i].meta_off - o)});
  std::mutex mu;
  std::condition_variable cv;
  std::deque<int64_t> done; // chunk index, or -1 - index on a read failure
  std::atomic<size_t> next{0};
  const uint32_t nth = std::max<uint32_t>(1, std::min<uint32_t>(pipe->io_threads, chunks.size()));
  std::vector<std::thread> readers;
  for (uint32_t w = 0; w < nth && !chunks.empty(); w++)
    readers.emplace_back([&] {
      for (size_t c; (c = next.fetch_add(1)) < chunks.size();) {
        const Chunk &k = chunks[c];
        const bool ok = pread_full(files[k.file].fd, pipe->h_in + files[k.file].base + k.off, k.len, k.off);
        std::lock_guard<std::mutex> lk(mu);
        done.push_back(ok ? static_cast<int64_t>(c) : -1 - static_cast<int64_t>(c));
        cv.notify_one();
      }
    });
  bool read_ok = true;
  hipError_t herr = hipSuccess;
  for (size_t got = 0; got < chunks.size(); got++) {
    int64_t c;
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return !done.empty(); });
      c = done.front();
      done.pop_front();
    }
    if (c < 0) {
      read_ok = false;
      continue;
    }
    const Chunk &k = chunks[c];
    const uint64_t at = files[k.file].base + k.off;
    if (herr == hipSuccess) herr = hipMemcpyAsync(pipe->d_src + at, pipe->h_in + at, k.len, hipMemcpyHostToDevice, s);
  }
  for (auto &t : readers) t.join();
  if (!read_ok) return bail(SSTC_E_INVALID_ARG, "sstc_compact_files: input read failed");
  // block index (absolute offsets into the staged data sections)
  uint64_t *h_off = reinterpret_cast<uint64_t *>(pipe->h_in + idx_at), *h_len = h_off + nblocks;
  for (uint32_t i = 0, b = 0; i < n_in; i++)
    for (size_t j = 0; j < files[i].off.size(); j++, b++) {
      h_off[b] = files[i].base + files[i].off[j];
      h_len[b] = files[i].len[j];
    }
  const uint64_t max_tables = std::min(total / params->table_limit + 2, total / 13 + 2);
  if (grow_dev(pipe->d_idx, pipe->cap_d_idx, 2 * nblocks + 2 * max_tables + 2))
    return bail(SSTC_E_NOMEM, "sstc_compact_files: index staging");
  uint64_t *d_off = pipe->d_idx, *d_len = d_off + nblocks, *d_toff = d_len + nblocks, *d_tlen = d_toff + max_tables + 1;
  if (herr == hipSuccess && nblocks)
    herr = hipMemcpyAsync(d_off, h_off, 16 * nblocks, hipMemcpyHostToDevice, s);
  if (herr == hipSuccess) herr = hipStreamSynchronize(s);
  if (herr != hipSuccess) return bail(SSTC_E_HIP, "sstc_compact_files: H2D");
  const auto t2 = clk::now();

  // ---- compact on the device
  // Output size bound from the input alone: every surviving entry is its
  // input entry's bytes plus, at worst, a block of its own (16 B extra) and a
  // meta entry (24 B + its key twice: at most twice the entry), each output
  // table a 40 B footer; an input entry takes >= 29 B with its offset entry.
  // So output <= 2 * input + 40 B per record (<= 1.4 * input) + 40 B per table.
  // A device-reported size past it is an internal fault, never an allocation.
  const uint64_t bound = pipe->test_bound ? pipe->test_bound : 4 * total + 64 * max_tables + (1u << 20);
  sstc_compact_result res{};
  uint64_t cap = total + total / 2 + (1u << 20);
  int rc = SSTC_E_CAPACITY;
  for (int attempt = 0; attempt < 2 && rc == SSTC_E_CAPACITY; attempt++) {
    if (grow_dev(pipe->d_dst, pipe->cap_d_dst, cap)) {
      const std::string what = "sstc_compact_files: output buffer of " + std::to_string(cap) + " bytes (" +
                               std::to_string(res.tables_out) + " tables, " + std::to_string(res.blocks_out) +
                               " blocks, " + std::to_string(res.records_kept) + " records)";
      return bail(SSTC_E_NOMEM, what.c_str());
    }
    const uint64_t use = attempt == 0 && pipe->test_first_cap ? std::min(pipe->test_first_cap, pipe->cap_d_dst)
                                                               : pipe->cap_d_dst;
    rc = sstc_compact(pipe->ctx, pipe->d_src, d_off, d_len, nblocks, tfb.data(), n_in, params, pipe->d_dst, use,
                      d_toff, d_tlen, max_tables, &res);
    if (rc == SSTC_E_CAPACITY) { // the exact size is known after a capacity miss
      if (res.bytes_out <= use || res.bytes_out > bound) {
        (void)sstc__ctx_sync(pipe->ctx);
        const std::string what = "sstc_compact_files: the device reported an output size of " +
                                 std::to_string(res.bytes_out) + " bytes after a capacity miss at " +
                                 std::to_string(use) + " (bound from the input: " + std::to_string(bound) + ")";
        return sstc__fail(SSTC_E_INTERNAL, what.c_str());
      }
      cap = res.bytes_out;
    }
  }
  if (rc != SSTC_OK) { // sstc_compact set the error string
    (void)sstc__ctx_sync(pipe->ctx);
    return rc;
  }
  const auto t3 = clk::now();

  // ---- store: per-table D2H with an event (each table at a 4 KiB-aligned
  // place of the pinned staging, for the O_DIRECT writes), the tables' keys
  // read from their images, then -- once first_id has accepted the count and
  // the key bytes -- writer threads write + fsync (no output file is touched
  // before every check has passed)
  const uint64_t nt = res.tables_out;
  if (nt > max_outs) return sstc__fail(SSTC_E_CAPACITY, "sstc_compact_files: more output tables than max_outs");
  std::vector<uint64_t> toff(nt + 1), hoff(nt + 1, 0);
  if (hipMemcpy(toff.data(), d_toff, 8 * (nt + 1), hipMemcpyDeviceToHost) != hipSuccess)
    return sstc__fail(SSTC_E_HIP, "sstc_compact_files: table offsets");
  for (uint64_t t = 0; t < nt; t++)
    hoff[t + 1] = hoff[t] + (toff[t + 1] - toff[t] + kDirectAlign - 1) / kDirectAlign * kDirectAlign;
  if (grow_pinned(pipe->h_out, pipe->cap_h_out, hoff[nt] + kDirectAlign))
    return sstc__fail(SSTC_E_NOMEM, "sstc_compact_files: output staging");
  uint8_t *h_out = pipe->h_out + ((kDirectAlign - reinterpret_cast<uintptr_t>(pipe->h_out) % kDirectAlign) % kDirectAlign);
  std::vector<hipEvent_t> ev(nt);
  for (uint64_t t = 0; t < nt; t++) {
    if (hipEventCreateWithFlags(&ev[t], hipEventDisableTiming) != hipSuccess ||
        hipMemcpyAsync(h_out + hoff[t], pipe->d_dst + toff[t], toff[t + 1] - toff[t], hipMemcpyDeviceToHost,
                       s) != hipSuccess ||
        hipEventRecord(ev[t], s) != hipSuccess) {
      (void)hipStreamSynchronize(s);
      for (uint64_t u = 0; u <= t && u < nt; u++)
        if (ev[u]) (void)hipEventDestroy(ev[u]);
      return sstc__fail(SSTC_E_HIP, "sstc_compact_files: D2H");
    }
  }
  std::vector<std::string> lo(nt), hi(nt);
  std::atomic<int> werr{0};
  const uint32_t nw = static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(pipe->io_threads, nt)));
  auto parallel = [&](const std::function<void(uint64_t)> &work) {
    std::atomic<uint64_t> tnext{0};
    std::vector<std::thread> th;
    for (uint32_t w = 0; w < nw; w++)
      th.emplace_back([&] {
        (void)hipSetDevice(pipe->device);
        for (uint64_t t; (t = tnext.fetch_add(1)) < nt;) work(t);
      });
    for (auto &x : th) x.join();
  };
  parallel([&](uint64_t t) {
    if (hipEventSynchronize(ev[t]) != hipSuccess) {
      werr = 1;
      return;
    }
    table_keys(h_out + hoff[t], toff[t + 1] - toff[t], lo[t], hi[t]);
  });
  for (auto &e : ev) (void)hipEventDestroy(e);
  if (werr) return sstc__fail(SSTC_E_HIP, "sstc_compact_files: D2H of the outputs failed");
  uint64_t key_bytes = 0;
  for (uint64_t t = 0; t < nt; t++) key_bytes += lo[t].size() + hi[t].size();
  uint64_t first_sst_id = 0;
  if (const int r = first_id(nt, key_bytes, first_sst_id)) return r;
  const std::string prefix(out_prefix);
  parallel([&](uint64_t t) {
    if (!write_table(prefix + std::to_string(first_sst_id + t) + ".sst", h_out + hoff[t], toff[t + 1] - toff[t],
                     do_fsync))
      werr = 2;
  });
  if (werr) return sstc__fail(SSTC_E_INVALID_ARG, "sstc_compact_files: output write failed");
  result.outs.resize(nt);
  result.keys.clear();
  for (uint64_t t = 0; t < nt; t++) {
    sstc_file_out &o = result.outs[t];
    o.sst_id = first_sst_id + t;
    o.file_size = toff[t + 1] - toff[t] + 1;
    o.smallest_key_len = static_cast<uint32_t>(lo[t].size());
    o.largest_key_len = static_cast<uint32_t>(hi[t].size());
    o.smallest_key_off = result.keys.size();
    o.largest_key_off = result.keys.size() + lo[t].size();
    result.keys += lo[t];
    result.keys += hi[t];
  }
  const auto t4 = clk::now();
  result.tm.index_s = secs(t0, t1);
  result.tm.load_s = secs(t1, t2);
  result.tm.compact_s = secs(t2, t3);
  result.tm.store_s = secs(t3, t4);
  result.tm.total_s = secs(t0, t4);
  return SSTC_OK;
}

// copies outputs (shard after shard) into the caller's arrays
int copy_outs(const std::vector<const FilesOut *> &parts, sstc_file_out *outs, uint32_t max_outs, uint32_t *n_out,
              uint8_t *key_arena, uint64_t key_arena_cap, const char *who) {
  uint64_t n = 0, kat = 0;
  for (const FilesOut *p : parts) {
    if (n + p->outs.size() > max_outs)
      return sstc__fail(SSTC_E_CAPACITY, (std::string(who) + ": more output tables than max_outs").c_str());
    if (key_arena && kat + p->keys.size() > key_arena_cap)
      return sstc__fail(SSTC_E_CAPACITY, (std::string(who) + ": key_arena too small").c_str());
    for (sstc_file_out o : p->outs) {
      o.smallest_key_off += kat;
      o.largest_key_off += kat;
      outs[n++] = o;
    }
    if (key_arena && !p->keys.empty()) std::memcpy(key_arena + kat, p->keys.data(), p->keys.size());
    kat += p->keys.size();
  }
  *n_out = static_cast<uint32_t>(n);
  return SSTC_OK;
}

} // namespace

extern "C" {

int sstc_compact_files(sstc_pipe *pipe, const char *const *in_paths, const uint64_t *in_file_sizes,
                       uint32_t n_in, const char *out_prefix, uint64_t first_sst_id,
                       const sstc_compact_params *params, uint32_t do_fsync, sstc_file_out *outs,
                       uint32_t max_outs, uint32_t *n_out, uint8_t *key_arena, uint64_t key_arena_cap,
                       sstc_files_timing *timing) {
  if (!pipe || (n_in && (!in_paths || !in_file_sizes)) || !out_prefix || !params || !outs || !n_out)
    return sstc__fail(SSTC_E_INVALID_ARG, "sstc_compact_files: NULL argument");
  if (params->table_limit == 0 || params->block_threshold == 0)
    return sstc__fail(SSTC_E_INVALID_ARG, "sstc_compact_files: bad parameters");
  *n_out = 0;
  FilesOut r;
  const int rc = compact_files_impl(
      pipe, in_paths, in_file_sizes, n_in, out_prefix,
      [&](uint64_t nt, uint64_t key_bytes, uint64_t &id) {
        if (nt > max_outs) return sstc__fail(SSTC_E_CAPACITY, "sstc_compact_files: more output tables than max_outs");
        if (key_arena && key_bytes > key_arena_cap)
          return sstc__fail(SSTC_E_CAPACITY, "sstc_compact_files: key_arena too small");
        id = first_sst_id;
        return static_cast<int>(SSTC_OK);
      },
      params, do_fsync, max_outs, r);
  if (rc != SSTC_OK) return rc;
  if (timing) *timing = r.tm;
  return copy_outs({&r}, outs, max_outs, n_out, key_arena, key_arena_cap, "sstc_compact_files");
}

int sstc_compact_files_multi(sstc_pipe *const *pipes, uint32_t n_pipes, const char *const *in_paths,
                             const uint64_t *in_file_sizes, const uint32_t *shard_first, uint32_t n_shards,
                             const char *out_prefix, uint64_t first_sst_id, const sstc_compact_params *params,
                             uint32_t do_fsync, sstc_file_out *outs, uint32_t max_outs, uint32_t *n_out,
                             uint8_t *key_arena, uint64_t key_arena_cap, sstc_files_timing *timing) {
  const char *who = "sstc_compact_files_multi";
  if (!pipes || n_pipes == 0 || !shard_first || !out_prefix || !params || !outs || !n_out)
    return sstc__fail(SSTC_E_INVALID_ARG, "sstc_compact_files_multi: NULL argument");
  if (params->table_limit == 0 || params->block_threshold == 0)
    return sstc__fail(SSTC_E_INVALID_ARG, "sstc_compact_files_multi: bad parameters");
  *n_out = 0;
  for (uint32_t j = 0; j < n_pipes; j++) {
    if (!pipes[j]) return sstc__fail(SSTC_E_INVALID_ARG, "sstc_compact_files_multi: NULL pipe");
    for (uint32_t k = 0; k < j; k++)
      if (pipes[k] == pipes[j])
        return sstc__fail(SSTC_E_INVALID_ARG, "sstc_compact_files_multi: a pipe listed twice (one thread per pipe)");
  }
  if (shard_first[0] != 0) return sstc__fail(SSTC_E_INVALID_ARG, "sstc_compact_files_multi: shard_first[0] != 0");
  for (uint32_t s = 0; s < n_shards; s++)
    if (shard_first[s + 1] < shard_first[s])
      return sstc__fail(SSTC_E_INVALID_ARG, "sstc_compact_files_multi: shard_first not ascending");
  if (shard_first[n_shards] && (!in_paths || !in_file_sizes))
    return sstc__fail(SSTC_E_INVALID_ARG, "sstc_compact_files_multi: NULL argument");

  // the output-id chain: shard s takes the ids after shard s - 1's tables,
  // exactly the GetNextSSTId() sequence of the shards compacted one after
  // another.  A shard writes only once the shard before it has written all
  // of its outputs, and only after the call-wide checks (max_outs, key_arena
  // for the shards so far) pass; a shard that fails -- before or while
  // writing -- breaks the chain, so every shard after it writes nothing (the
  // device work of all shards still overlaps).
  std::mutex m;
  std::condition_variable cv;
  std::vector<int> state(n_shards + 1, 0); // 0 pending, 1 written, -1 broken
  std::vector<uint64_t> base(n_shards + 1, 0), kbase(n_shards + 1, 0);
  state[0] = 1;
  base[0] = first_sst_id;
  auto publish = [&](uint32_t s, int st, uint64_t b, uint64_t kb) {
    std::lock_guard<std::mutex> lk(m);
    if (state[s + 1] != 0) return;
    state[s + 1] = st;
    base[s + 1] = b;
    kbase[s + 1] = kb;
    cv.notify_all();
  };
  std::vector<FilesOut> res(n_shards);
  std::vector<int> rcs(n_shards, SSTC_OK);
  std::vector<std::string> errs(n_shards);
  std::vector<std::thread> th;
  for (uint32_t j = 0; j < std::min(n_pipes, n_shards); j++)
    th.emplace_back([&, j] {
      for (uint32_t sh = j; sh < n_shards; sh += n_pipes) {
        uint64_t my_id = 0, my_keys = 0;
        const FirstId chain = [&, sh](uint64_t nt, uint64_t key_bytes, uint64_t &id) {
          std::unique_lock<std::mutex> lk(m);
          cv.wait(lk, [&] { return state[sh] != 0; });
          if (state[sh] < 0) return sstc__fail(SSTC_E_INVALID_ARG, "sstc_compact_files_multi: an earlier shard failed");
          if (base[sh] - first_sst_id + nt > max_outs)
            return sstc__fail(SSTC_E_CAPACITY, "sstc_compact_files_multi: more output tables than max_outs");
          if (key_arena && kbase[sh] + key_bytes > key_arena_cap)
            return sstc__fail(SSTC_E_CAPACITY, "sstc_compact_files_multi: key_arena too small");
          id = my_id = base[sh];
          my_keys = kbase[sh] + key_bytes;
          return static_cast<int>(SSTC_OK);
        };
        const uint32_t f = shard_first[sh], n = shard_first[sh + 1] - f;
        rcs[sh] = compact_files_impl(pipes[j], in_paths + f, in_file_sizes + f, n, out_prefix, chain, params, do_fsync,
                                     max_outs, res[sh]);
        if (rcs[sh] != SSTC_OK) {
          errs[sh] = sstc_last_error_string(); // thread-local: carried to the caller's thread
          publish(sh, -1, 0, 0);
        } else {
          publish(sh, 1, my_id + res[sh].outs.size(), my_keys);
        }
      }
    });
  for (auto &t : th) t.join();
  if (timing)
    for (uint32_t sh = 0; sh < n_shards; sh++) timing[sh] = res[sh].tm;
  // the shards before the first failing one completed: their outputs are
  // reported (outs / n_out / key_arena) whatever the call returns
  uint32_t done = 0;
  while (done < n_shards && rcs[done] == SSTC_OK) done++;
  std::vector<const FilesOut *> parts;
  for (uint32_t sh = 0; sh < done; sh++) parts.push_back(&res[sh]);
  const int rc = copy_outs(parts, outs, max_outs, n_out, key_arena, key_arena_cap, who);
  if (done < n_shards)
    return sstc__fail(rcs[done], ("sstc_compact_files_multi: shard " + std::to_string(done) + ": " + errs[done]).c_str());
  return rc;
}

} // extern "C"
