// sst_table.cpp — host C++ mirror of the reference TableBuilder / TableReader
// over the codec C-ABI.  See include/sstc_table.h.
//
// Byte work (block serialisation, block parse) happens in the GPU kernels via
// sstc_encode_blocks / sstc_count_records / sstc_decode_blocks.  What stays on
// the host is what the reference does per block or per table, not per byte:
// block boundaries (a running sum per AddEntry), the meta section (one entry per
// block), the 40 B footer, and the file I/O.
#include "sstc_table.h"

#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <memory>
#include <stdexcept>

namespace sstc {
namespace {

uint64_t entry_size(uint32_t klen, uint32_t vlen) {
  return 13ull + klen + (vlen != SSTC_NO_VALUE ? 4ull + vlen : 0ull); // block_builder.cc:19-21
}

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

bool pwrite_all(int fd, const uint8_t *buf, size_t size, uint64_t off) {
  while (size > 0) { // io/linux_file.cc:138-157 semantics: retry on EINTR
    ssize_t w = ::pwrite64(fd, buf, size, static_cast<off64_t>(off));
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    buf += w;
    size -= static_cast<size_t>(w);
    off += static_cast<uint64_t>(w);
  }
  return true;
}

bool pread_all(int fd, uint8_t *buf, size_t size, uint64_t off) {
  while (size > 0) {
    ssize_t r = ::pread(fd, buf, size, static_cast<off64_t>(off));
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    if (r == 0) return false;
    buf += r;
    size -= static_cast<size_t>(r);
    off += static_cast<uint64_t>(r);
  }
  return true;
}

// RAII device buffer
struct DevBuf {
  void *p = nullptr;
  explicit DevBuf(size_t n) {
    if (hipMalloc(&p, n ? n : 16) != hipSuccess) throw std::runtime_error("hipMalloc failed");
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  template <class T> T *as() const { return static_cast<T *>(p); }
};

} // namespace
} // namespace sstc

extern "C" int sstc__ctx_device(const sstc_ctx *ctx); // sstc_api.hip: the device a context is bound to
extern "C" void *sstc__ctx_stream(const sstc_ctx *ctx); // sstc_api.hip: the stream a context runs on

namespace sstc {
namespace {

// Every copy runs on the context's own stream, in order with its kernels: a
// null-stream hipMemcpy would not be ordered after work on a non-blocking
// stream, and on a blocking one it would serialise every thread's builder
// (concurrent flushes, db_impl.cc:354-362, each own a context and a stream).
hipStream_t stream_of(sstc_ctx *ctx) { return static_cast<hipStream_t>(sstc__ctx_stream(ctx)); }

void h2d(sstc_ctx *ctx, void *d, const void *h, size_t n) {
  if (n && hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, stream_of(ctx)) != hipSuccess)
    throw std::runtime_error("hipMemcpyAsync H2D failed");
}

bool d2h(sstc_ctx *ctx, void *h, const void *d, size_t n) {
  return !n || hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, stream_of(ctx)) == hipSuccess;
}

bool sync(sstc_ctx *ctx) { return hipStreamSynchronize(stream_of(ctx)) == hipSuccess; }


} // namespace

namespace {
// SSTC_TRACE_HOST=1: host-side phase times on stderr (diagnostics of the C++
// drop-in paths; off by default)
bool trace_host() {
  static const bool on = std::getenv("SSTC_TRACE_HOST") != nullptr;
  return on;
}
double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
thread_local double g_pin_ms = 0;
thread_local uint64_t g_pin_bytes = 0, g_pin_calls = 0;
} // namespace

void TraceHost(const char *what, double ms) {
  if (trace_host()) std::fprintf(stderr, "[sstc] %s %.3f ms\n", what, ms);
}
bool TraceHostOn() { return trace_host(); }
double TraceNowMs() { return now_ms(); }

extern "C" void *sstc_host_alloc(uint64_t bytes, int *pinned) {
  void *p = nullptr;
  const double t0 = trace_host() ? now_ms() : 0;
  const bool ok = bytes && hipHostMalloc(&p, bytes, hipHostMallocPortable) == hipSuccess;
  if (trace_host()) {
    g_pin_ms += now_ms() - t0;
    g_pin_bytes += bytes;
    g_pin_calls++;
  }
  if (ok) {
    if (pinned) *pinned = 1;
    return p;
  }
  (void)hipGetLastError(); // no device / no pinning: ordinary memory
  if (pinned) *pinned = 0;
  return std::malloc(bytes ? bytes : 1);
}

extern "C" void sstc_host_free(void *p, int pinned) {
  if (!p) return;
  if (pinned) (void)hipHostFree(p);
  else std::free(p);
}

namespace {

void check(int rc, const char *what) {
  if (rc != SSTC_OK) throw std::runtime_error(std::string(what) + ": " + sstc_last_error_string());
}

} // namespace

// ---------------------------------------------------------------- TableBuilder
struct BuilderArena {
  HostVec<uint8_t> type, keys, vals;
  HostVec<uint32_t> kl, vl;
  HostVec<uint64_t> txn, ko, vo, first;
  void clear() {
    for (auto *v : {&type, &keys, &vals}) v->clear();
    kl.clear();
    vl.clear();
    for (auto *v : {&txn, &ko, &vo, &first}) v->clear();
  }
};

namespace {
struct DeferredFrees {
  std::vector<std::pair<void *, int>> bufs;
  void flush() {
    for (auto &[p, pinned] : bufs) sstc_host_free(p, pinned);
    bufs.clear();
  }
  ~DeferredFrees() { flush(); }
};
thread_local DeferredFrees g_deferred;
} // namespace

void DeferHostFree(void *p, int pinned) {
  if (!p) return;
  if (!pinned) {
    sstc_host_free(p, pinned); // pageable: free() does not touch the device
    return;
  }
  g_deferred.bufs.emplace_back(p, pinned);
}

void FlushDeferredHostFrees() { g_deferred.flush(); }

namespace {
// per-thread pool of builder arenas: a finished builder's pinned, faulted-in
// arrays are the next builder's (the flush / compaction threads build SST
// after SST; round 2 spent most of AddEntries in first-touch page faults)
constexpr size_t kArenaPool = 4;
thread_local std::vector<std::unique_ptr<BuilderArena>> g_arenas;

BuilderArena *take_arena() {
  if (g_arenas.empty()) return new BuilderArena();
  BuilderArena *a = g_arenas.back().release();
  g_arenas.pop_back();
  return a;
}

// a surplus arena's pinned arrays are freed with the thread's deferred frees
// (at its next Finish or exit), not in the destructor of the builder that
// returned it
struct SurplusArenas {
  std::vector<std::unique_ptr<BuilderArena>> v;
};
thread_local SurplusArenas g_surplus;

void give_arena(BuilderArena *a) {
  a->clear();
  if (g_arenas.size() < kArenaPool) g_arenas.emplace_back(a);
  else g_surplus.v.emplace_back(a);
}
} // namespace

TableBuilder::TableBuilder(std::string filename, uint64_t block_threshold, sstc_ctx *ctx)
    : filename_(std::move(filename)), threshold_(block_threshold), ctx_(ctx), arena_(take_arena()),
      type_(arena_->type), key_len_(arena_->kl), val_len_(arena_->vl), txn_(arena_->txn), key_off_(arena_->ko),
      val_off_(arena_->vo), keys_(arena_->keys), vals_(arena_->vals), blk_first_(arena_->first) {
  blk_first_.push_back(0);
}

TableBuilder::~TableBuilder() {
  if (fd_ >= 0) ::close(fd_);
  give_arena(arena_);
}

bool TableBuilder::Open() {
  // io/linux_file.cc:99-119: an existing file is opened WITHOUT O_TRUNC (stale
  // tail bytes survive a shorter rewrite); a new one is created.
  ::chmod(filename_.c_str(), 0644);
  const bool create = ::access(filename_.c_str(), F_OK) != 0;
  const int flags = create ? (O_TRUNC | O_WRONLY | O_CREAT) : O_WRONLY;
  fd_ = ::open(filename_.c_str(), flags, 0644);
  return fd_ >= 0;
}

bool TableBuilder::AdoptResident() {
  ResidentInputs *r = ResidentInputs::Active();
  if (!r || r->Device() != sstc__ctx_device(ctx_)) return false;
  res_ = r->shared_from_this();
  res_host_ = r->Host();
  res_bytes_ = r->Bytes();
  return true;
}

void TableBuilder::AddEntry(std::string_view key, std::string_view value, uint64_t txn_id,
                            uint8_t value_type) {
  // table_builder.cc:35-60
  if (table_smallest_key_.empty()) table_smallest_key_ = std::string(key);
  const uint8_t *kp = reinterpret_cast<const uint8_t *>(key.data());
  const uint8_t *vp = reinterpret_cast<const uint8_t *>(value.data());
  // views into the resident inputs (what the drop-in MergeIterator hands out):
  // offsets only, the bytes are already on the device
  if ((res_host_ || (type_.empty() && AdoptResident())) &&
      static_cast<uint64_t>(kp - res_host_) < res_bytes_ &&
      (!vp || static_cast<uint64_t>(vp - res_host_) < res_bytes_)) {
    key_off_.push_back(static_cast<uint64_t>(kp - res_host_));
    val_off_.push_back(vp ? static_cast<uint64_t>(vp - res_host_) : 0);
  } else {
    const uint64_t tag = res_host_ ? kArenaRef : 0;
    arena_recs_ += tag != 0;
    key_off_.push_back(keys_.size() | tag);
    keys_.append(kp, key.size());
    if (vp) {
      val_off_.push_back(vals_.size() | tag);
      vals_.append(vp, value.size());
    } else {
      val_off_.push_back(tag);
    }
  }
  type_.push_back(value_type);
  key_len_.push_back(static_cast<uint32_t>(key.size()));
  val_len_.push_back(vp ? static_cast<uint32_t>(value.size()) : SSTC_NO_VALUE);
  txn_.push_back(txn_id);
  if (txn_id < min_txn_) min_txn_ = txn_id;
  if (txn_id > max_txn_) max_txn_ = txn_id;
  data_size_ += key.size() + (vp ? value.size() : 0);
  block_size_ += entry_size(key_len_.back(), val_len_.back()) + 16; // block_builder.cc:33
  if (block_size_ >= threshold_) FlushBlock();
}

void TableBuilder::AddEntries(uint64_t n, const uint8_t *type, const uint32_t *key_len, const uint32_t *val_len,
                              const uint64_t *txn, const uint8_t *key_src, const uint64_t *key_off,
                              const uint8_t *val_src, const uint64_t *val_off) {
  // AddEntry's bookkeeping (table_builder.cc:35-60) in one loop: SoA appends
  // and the running block size; keys / values appended per record
  type_.reserve(type_.size() + n);
  key_len_.reserve(key_len_.size() + n);
  val_len_.reserve(val_len_.size() + n);
  txn_.reserve(txn_.size() + n);
  key_off_.reserve(key_off_.size() + n);
  val_off_.reserve(val_off_.size() + n);
  uint64_t kb = 0, vb = 0;
  for (uint64_t i = 0; i < n; i++) {
    kb += key_len[i];
    vb += val_len[i] != SSTC_NO_VALUE ? val_len[i] : 0;
  }
  keys_.reserve(keys_.size() + kb);
  vals_.reserve(vals_.size() + vb);
  const uint64_t tag = res_host_ ? kArenaRef : 0; // (a resident builder: these are arena records)
  arena_recs_ += tag ? n : 0;
  for (uint64_t i = 0; i < n; i++) {
    const uint32_t kl = key_len[i], vl = val_len[i];
    if (table_smallest_key_.empty()) table_smallest_key_.assign(reinterpret_cast<const char *>(key_src + key_off[i]), kl);
    type_.push_back(type[i]);
    key_len_.push_back(kl);
    key_off_.push_back(keys_.size() | tag);
    keys_.append(key_src + key_off[i], kl);
    if (vl != SSTC_NO_VALUE) {
      val_off_.push_back(vals_.size() | tag);
      vals_.append(val_src + val_off[i], vl);
    } else {
      val_off_.push_back(tag);
    }
    val_len_.push_back(vl);
    txn_.push_back(txn[i]);
    if (txn[i] < min_txn_) min_txn_ = txn[i];
    if (txn[i] > max_txn_) max_txn_ = txn[i];
    data_size_ += kl + (vl != SSTC_NO_VALUE ? vl : 0);
    block_size_ += entry_size(kl, vl) + 16; // block_builder.cc:33
    if (block_size_ >= threshold_) FlushBlock();
  }
}

void TableBuilder::FlushBlock() {
  if (block_size_ == 0) return; // table_builder.cc:65-68: empty block not written
  blk_first_.push_back(type_.size());
  block_size_ = 0;
}

namespace {
// per-host-thread, per-device staging reused across Finish() calls (flush /
// compaction threads each build many SSTs): one pinned host buffer and one
// device buffer on the context's device, grown when needed, so a Finish makes
// no allocation in steady state and its copies run from / into pinned memory
struct Staging {
  uint8_t *host = nullptr, *dev = nullptr;
  uint64_t host_cap = 0, dev_cap = 0;
  std::vector<hipEvent_t> ev; // one per D2H chunk of a Finish
  ~Staging() {
    if (host) (void)hipHostFree(host);
    if (dev) (void)hipFree(dev);
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  }
  hipEvent_t Event(uint64_t i) {
    while (ev.size() <= i) {
      hipEvent_t e = nullptr;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) throw std::runtime_error("hipEventCreate");
      ev.push_back(e);
    }
    return ev[i];
  }
  uint8_t *Host(uint64_t n) {
    if (n > host_cap) {
      if (host) (void)hipHostFree(host);
      host = nullptr;
      host_cap = 0;
      const uint64_t c = n + n / 4;
      if (hipHostMalloc(reinterpret_cast<void **>(&host), c, hipHostMallocDefault) != hipSuccess)
        throw std::runtime_error("hipHostMalloc failed");
      host_cap = c;
    }
    return host;
  }
  uint8_t *Dev(uint64_t n) {
    if (n > dev_cap) {
      if (dev) (void)hipFree(dev);
      dev = nullptr;
      dev_cap = 0;
      const uint64_t c = n + n / 4;
      if (hipMalloc(reinterpret_cast<void **>(&dev), c) != hipSuccess) throw std::runtime_error("hipMalloc failed");
      dev_cap = c;
    }
    return dev;
  }
};
thread_local std::map<int, Staging> g_stage; // device -> staging

// Finish() writes the file image in chunks as they arrive from the device
constexpr uint64_t kWriteChunk = 8ull << 20;
constexpr uint64_t kDirectAlign = 4096;

// Writes the image h[0, file_bytes) of an SST at offset 0: the 4 KiB-aligned
// part through a second O_DIRECT descriptor (the page-locked image goes to
// the device without a copy into the page cache: a buffered pwrite of a
// 44 MB table cost 4-5 ms of memcpy on top of the fsync), the unaligned tail
// through the builder's own descriptor.  Same bytes, same offsets, same
// durability (Finish fsyncs after); a file system without O_DIRECT, or a
// direct write it refuses, takes buffered pwrites.  SSTC_NO_DIRECT_IO=1: always buffered.
class FileWriter {
public:
  FileWriter(int fd, const std::string &path, const uint8_t *h) : fd_(fd), h_(h) {
    static const bool off = std::getenv("SSTC_NO_DIRECT_IO") != nullptr;
    if (!off && !(reinterpret_cast<uintptr_t>(h) & (kDirectAlign - 1)))
      dfd_ = ::open(path.c_str(), O_WRONLY | O_DIRECT | O_CLOEXEC);
  }
  ~FileWriter() {
    if (dfd_ >= 0) ::close(dfd_);
  }
  bool direct() const { return direct_used_; }
  // write [done_, end); `last`: end is the file's end (write the unaligned tail too)
  void WriteUpTo(uint64_t end, bool last) {
    if (dfd_ >= 0) {
      const uint64_t a = end & ~(kDirectAlign - 1);
      if (a > done_) {
        if (pwrite_all(dfd_, h_ + done_, a - done_, done_)) {
          direct_used_ = true;
          done_ = a;
        } else { // refused (alignment rules of this file system): buffered from here on
          ::close(dfd_);
          dfd_ = -1;
        }
      }
      if (!last) return;
    }
    if (end > done_ && !pwrite_all(fd_, h_ + done_, end - done_, done_))
      throw std::runtime_error("Error when flushing sstable"); // table_builder.cc:155-170
    done_ = end;
  }

private:
  int fd_, dfd_ = -1;
  const uint8_t *h_;
  uint64_t done_ = 0;
  bool direct_used_ = false;
};

// makes `dev` current for the scope and restores the caller's device
struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (dev >= 0 && dev != prev && hipSetDevice(dev) != hipSuccess) throw std::runtime_error("hipSetDevice failed");
  }
  ~DeviceScope() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

uint64_t align256(uint64_t x) { return (x + 255) & ~uint64_t(255); }
} // namespace

void TableBuilder::Finish() {
  if (fd_ < 0) throw std::runtime_error("TableBuilder::Finish: file not open");
  const double t_begin = trace_host() ? now_ms() : 0;
  double t_enc = t_begin, t_d2h = t_begin, t_write = t_begin;
  FlushBlock();
  const uint64_t n = type_.size();
  const uint64_t nb = blk_first_.size() - 1;
  uint64_t data_bytes = 16 * nb + 16 * n;
  for (uint64_t i = 0; i < n; i++) data_bytes += entry_size(key_len_[i], val_len_[i]);
  uint64_t meta_bytes = 0;
  for (uint64_t b = 0; b < nb; b++) meta_bytes += 24 + key_len_[blk_first_[b]] + key_len_[blk_first_[b + 1] - 1];
  const uint64_t file_bytes = data_bytes + meta_bytes + 40;
  if (keys_.empty()) keys_.push_back(0);
  if (vals_.empty()) vals_.push_back(0);
  // input image (SoA + arenas + block starts) packed at 256 B boundaries
  const uint64_t o_type = 0, o_kl = align256(o_type + n), o_vl = align256(o_kl + 4 * n),
                 o_txn = align256(o_vl + 4 * n), o_ko = align256(o_txn + 8 * n), o_vo = align256(o_ko + 8 * n),
                 o_first = align256(o_vo + 8 * n), o_keys = align256(o_first + 8 * (nb + 1)),
                 o_vals = align256(o_keys + keys_.size()), in_bytes = align256(o_vals + vals_.size());
  const uint64_t o_dst = in_bytes, o_off = align256(o_dst + data_bytes), o_len = align256(o_off + 8 * (nb + 1)),
                 dev_bytes = align256(o_len + 8 * nb + 8);
  // the staging lives on the context's device, whatever device the calling
  // thread has current (the encode kernel runs on the context's device)
  const int dev = sstc__ctx_device(ctx_);
  DeviceScope on_ctx_device(dev);
  Staging &stage = g_stage[dev];
  uint8_t *h = stage.Host(file_bytes + 16 * nb + 16); // the file image (blocks D2H'd straight into it)
  std::vector<uint64_t> blk_off(nb + 1), blk_len(nb);
  if (nb) {
    uint8_t *d = stage.Dev(dev_bytes);
    // the arrays are pinned (HostVec): each goes up as a true async copy,
    // ordered before the encode, with no pack copy on the host
    h2d(ctx_, d + o_type, type_.data(), n);
    h2d(ctx_, d + o_kl, key_len_.data(), 4 * n);
    h2d(ctx_, d + o_vl, val_len_.data(), 4 * n);
    h2d(ctx_, d + o_txn, txn_.data(), 8 * n);
    h2d(ctx_, d + o_first, blk_first_.data(), 8 * (nb + 1));
    const uint8_t *key_src = d + o_keys, *val_src = d + o_vals;
    std::vector<uint64_t> ko2, vo2; // (a resident builder with arena records: offsets from one base)
    if (!res_host_) {
      h2d(ctx_, d + o_ko, key_off_.data(), 8 * n);
      h2d(ctx_, d + o_vo, val_off_.data(), 8 * n);
      h2d(ctx_, d + o_keys, keys_.data(), keys_.size());
      h2d(ctx_, d + o_vals, vals_.data(), vals_.size());
    } else if (arena_recs_ == 0) {
      // every record is in the resident inputs: their device copy is the
      // source, nothing but the record columns goes up
      key_src = val_src = res_->DeviceBytes();
      h2d(ctx_, d + o_ko, key_off_.data(), 8 * n);
      h2d(ctx_, d + o_vo, val_off_.data(), 8 * n);
    } else {
      h2d(ctx_, d + o_keys, keys_.data(), keys_.size());
      h2d(ctx_, d + o_vals, vals_.data(), vals_.size());
      const uint8_t *rdev = res_->DeviceBytes();
      const uint8_t *base = std::min<const uint8_t *>({rdev, key_src, val_src});
      ko2.resize(n);
      vo2.resize(n);
      for (uint64_t i = 0; i < n; i++) {
        const uint64_t k = key_off_[i], v = val_off_[i];
        ko2[i] = k & kArenaRef ? static_cast<uint64_t>(key_src - base) + (k & ~kArenaRef)
                               : static_cast<uint64_t>(rdev - base) + k;
        vo2[i] = v & kArenaRef ? static_cast<uint64_t>(val_src - base) + (v & ~kArenaRef)
                               : static_cast<uint64_t>(rdev - base) + v;
      }
      key_src = val_src = base;
      h2d(ctx_, d + o_ko, ko2.data(), 8 * n);
      h2d(ctx_, d + o_vo, vo2.data(), 8 * n);
    }
    sstc_records rec{d + o_type, reinterpret_cast<uint32_t *>(d + o_kl), reinterpret_cast<uint32_t *>(d + o_vl),
                     reinterpret_cast<uint64_t *>(d + o_txn), reinterpret_cast<uint64_t *>(d + o_ko),
                     reinterpret_cast<uint64_t *>(d + o_vo)};
    check(sstc_encode_blocks(ctx_, key_src, val_src, rec, n, reinterpret_cast<uint64_t *>(d + o_first), nb, 0,
                             d + o_dst, reinterpret_cast<uint64_t *>(d + o_off), reinterpret_cast<uint64_t *>(d + o_len)),
          "sstc_encode_blocks");
    uint64_t errs = 0;
    check(sstc_ctx_error_count(ctx_, &errs), "sstc_ctx_error_count"); // synchronises the stream
    if (trace_host()) t_enc = now_ms();
    // the block index first (the meta section below needs it), then the
    // blocks straight into the file image in chunks, each chunk's arrival an
    // event: the file is written chunk by chunk behind the copies
    if (!d2h(ctx_, blk_off.data(), d + o_off, (nb + 1) * 8) || !d2h(ctx_, blk_len.data(), d + o_len, nb * 8))
      throw std::runtime_error("hipMemcpyAsync D2H failed");
    for (uint64_t c = 0; c * kWriteChunk < data_bytes; c++) {
      const uint64_t at = c * kWriteChunk, len = std::min(kWriteChunk, data_bytes - at);
      if (!d2h(ctx_, h + at, d + o_dst + at, len) || hipEventRecord(stage.Event(c), stream_of(ctx_)) != hipSuccess)
        throw std::runtime_error("hipMemcpyAsync D2H failed");
    }
    // (the block index is in once the first chunk's event has fired)
    if (hipEventSynchronize(stage.Event(0)) != hipSuccess) throw std::runtime_error("hipEventSynchronize failed");
  }
  // meta section: one entry per block (table_builder.cc:101-145), then the
  // footer (table_builder.cc:179-211), appended to the file image in place
  if (trace_host()) t_d2h = now_ms();
  uint8_t *w = h + data_bytes;
  auto put = [&w](const void *p, uint64_t len) {
    std::memcpy(w, p, len);
    w += len;
  };
  for (uint64_t b = 0; b < nb; b++) {
    const uint64_t f = blk_first_[b], l = blk_first_[b + 1] - 1;
    put(&key_len_[f], 4);
    put(KeyPtr(f), key_len_[f]);
    put(&key_len_[l], 4);
    put(KeyPtr(l), key_len_[l]);
    put(&blk_off[b], 8);
    put(&blk_len[b], 8);
  }
  const uint64_t meta_off = data_bytes, foot[5] = {nb, meta_off, meta_bytes, min_txn_, max_txn_};
  put(foot, 40);
  const double t_meta = trace_host() ? now_ms() : 0;
  // the data blocks as their chunks land, then the rest (table_builder.cc:
  // 155-170 writes the same bytes block by block)
  FileWriter out(fd_, filename_, h);
  for (uint64_t c = 0; nb && c * kWriteChunk < data_bytes; c++) {
    if (hipEventSynchronize(stage.Event(c)) != hipSuccess) throw std::runtime_error("hipEventSynchronize failed");
    out.WriteUpTo(std::min((c + 1) * kWriteChunk, data_bytes), false);
  }
  out.WriteUpTo(file_bytes, true);
  if (trace_host()) t_write = now_ms();
  current_offset_ = file_bytes;
  if (::fsync(fd_) < 0) throw std::runtime_error("fsync failed");
  // the stream is idle here: free what this thread's builders outgrew
  g_surplus.v.clear();
  FlushDeferredHostFrees();
  if (trace_host())
    std::fprintf(stderr,
                 "[sstc] Finish %llu records %llu B: %.3f ms (H2D + encode %.3f, D2H %.3f, meta %.3f, pwrite %.3f, "
                 "fsync %.3f%s%s); page-locked allocs so far %llu calls %llu B %.3f ms\n",
                 static_cast<unsigned long long>(type_.size()), static_cast<unsigned long long>(file_bytes),
                 now_ms() - t_begin, t_enc - t_begin, t_d2h - t_enc, t_meta - t_d2h, t_write - t_meta,
                 now_ms() - t_write, res_host_ ? (arena_recs_ ? ", resident + arena" : ", resident") : "",
                 out.direct() ? ", direct" : "",
                 static_cast<unsigned long long>(g_pin_calls), static_cast<unsigned long long>(g_pin_bytes), g_pin_ms);
}

// ----------------------------------------------------------------- TableReader
TableReader *TableReader::Open(const std::string &filename, uint64_t file_size, sstc_ctx *ctx) {
  std::unique_ptr<TableReader> tr(new TableReader());
  tr->ctx_ = ctx;
  tr->fd_ = ::open(filename.c_str(), O_RDONLY);
  if (tr->fd_ < 0 || file_size < 41) return nullptr;
  tr->bytes_ = file_size - 1;
  uint8_t foot[40];
  // DecodeExtraInfo: footer at file_size - 40 - 1 (table_reader.cc:52-84)
  if (!pread_all(tr->fd_, foot, 40, tr->bytes_ - 40)) return nullptr;
  const uint64_t nb = get64(foot), moff = get64(foot + 8), mlen = get64(foot + 16);
  tr->min_txn_ = get64(foot + 24);
  tr->max_txn_ = get64(foot + 32);
  if (moff > tr->bytes_ - 40 || mlen > tr->bytes_ - 40 - moff) return nullptr;
  tr->meta_off_ = moff;
  std::vector<uint8_t> meta(mlen);
  if (mlen && !pread_all(tr->fd_, meta.data(), mlen, moff)) return nullptr;
  // FetchBlockIndexInfo (table_reader.cc:86-156): sequential length-prefixed walk
  uint64_t p = 0;
  for (uint64_t i = 0; i < nb; i++) {
    if (p + 4 > mlen) return nullptr;
    const uint32_t fk = get32(&meta[p]);
    if (p + 8 + fk > mlen) return nullptr;
    const uint32_t lk = get32(&meta[p + 4 + fk]);
    if (p + 24 + fk + lk > mlen) return nullptr;
    BlockIndex bi;
    bi.smallest_key.assign(reinterpret_cast<const char *>(&meta[p + 4]), fk);
    bi.largest_key.assign(reinterpret_cast<const char *>(&meta[p + 8 + fk]), lk);
    bi.offset = get64(&meta[p + 8 + fk + lk]);
    bi.size = get64(&meta[p + 16 + fk + lk]);
    tr->index_.push_back(std::move(bi));
    p += 24 + fk + lk;
  }
  return tr.release();
}

TableReader::~TableReader() {
  if (fd_ >= 0) ::close(fd_);
}

namespace {
// Batched GPU decode of blocks (off[b], len[b]) inside the host bytes `data`:
// per-block record counts and status, record fields with offsets into data.
using HostRecords = DecodedBlocks;

} // namespace

namespace {
// per-host-thread, per-device decode staging, grow-only (a reader thread
// decodes table after table: no hipMalloc / hipFree per table)
struct DecStage {
  uint8_t *dev = nullptr;
  uint64_t cap = 0;
  ~DecStage() {
    if (dev) (void)hipFree(dev);
  }
  uint8_t *get(uint64_t n) {
    if (n > cap) {
      if (dev) (void)hipFree(dev);
      dev = nullptr;
      cap = 0;
      const uint64_t c = n + n / 4;
      if (hipMalloc(reinterpret_cast<void **>(&dev), c) != hipSuccess) throw std::runtime_error("hipMalloc failed");
      cap = c;
    }
    return dev;
  }
};
// device -> staging: the input bytes + block index, and the record arrays
// (sized by the real record count, known after the count kernel)
thread_local std::map<int, DecStage> g_dec, g_dec_rec;
} // namespace

namespace {
// H2D of the bytes and the block index, count + decode on the device; on
// SSTC_OK `base` holds the per-block record bases (host) and `rec` / `d_st`
// the device record table and block codes (in the thread's staging region)
int decode_on_device(sstc_ctx *ctx, const uint8_t *data, uint64_t bytes, const uint64_t *off, const uint64_t *len,
                     uint64_t nb, uint32_t txn_mode, std::vector<uint64_t> &base, sstc_records &rec,
                     uint32_t *&d_st, uint8_t *&d_extra, uint64_t extra_per_rec) {
  if (!ctx || (bytes && !data) || (nb && (!off || !len))) return SSTC_E_INVALID_ARG;
  uint64_t sum_len = 0;
  for (uint64_t b = 0; b < nb; b++) {
    if (off[b] > bytes || len[b] > bytes - off[b]) return SSTC_E_INVALID_ARG;
    sum_len += len[b];
  }
  static const uint8_t kZero[16] = {};
  const int dev = sstc__ctx_device(ctx);
  DeviceScope on_ctx_device(dev);
  // one device region for the bytes, the block index, the counts and the
  // block codes; the record arrays in a second one sized by the real count
  // (the count kernel takes a trailer's n only when 16 n + 16 <= the block's
  // length, so n <= nmax; round 5 sized them by nmax: ~4x the records of
  // 150 B entries, 65 B each with the packed rows)
  const uint64_t nmax = sum_len / 16 + 1;
  const uint64_t o_src = 0, o_off = align256(bytes + 16), o_len = align256(o_off + 8 * nb),
                 o_base = align256(o_len + 8 * nb), o_st = align256(o_base + 8 * (nb + 1)),
                 total = align256(o_st + 4 * nb + 4);
  uint8_t *d = g_dec[dev].get(total);
  h2d(ctx, d + o_src, bytes ? data : kZero, bytes ? bytes : 1);
  h2d(ctx, d + o_off, off, nb * 8);
  h2d(ctx, d + o_len, len, nb * 8);
  auto *d_off = reinterpret_cast<uint64_t *>(d + o_off), *d_len = reinterpret_cast<uint64_t *>(d + o_len),
       *d_base = reinterpret_cast<uint64_t *>(d + o_base);
  check(sstc_count_records(ctx, d + o_src, d_off, d_len, nb, d_base), "sstc_count_records");
  base.resize(nb + 1);
  if (!d2h(ctx, base.data(), d_base, (nb + 1) * 8) || !sync(ctx)) return SSTC_E_HIP;
  const uint64_t n = base[nb];
  if (n > nmax) return SSTC_E_INVALID_ARG; // blocks claiming more entries than their bytes hold
  const uint64_t r_type = 0, r_kl = align256(n + 1), r_vl = align256(r_kl + 4 * n + 4),
                 r_txn = align256(r_vl + 4 * n + 4), r_ko = align256(r_txn + 8 * n + 8),
                 r_vo = align256(r_ko + 8 * n + 8), r_x = align256(r_vo + 8 * n + 8),
                 r_total = align256(r_x + extra_per_rec * n + 16);
  uint8_t *r = g_dec_rec[dev].get(r_total);
  rec = sstc_records{r + r_type, reinterpret_cast<uint32_t *>(r + r_kl), reinterpret_cast<uint32_t *>(r + r_vl),
                     reinterpret_cast<uint64_t *>(r + r_txn), reinterpret_cast<uint64_t *>(r + r_ko),
                     reinterpret_cast<uint64_t *>(r + r_vo)};
  d_st = reinterpret_cast<uint32_t *>(d + o_st);
  d_extra = r + r_x;
  check(sstc_decode_blocks(ctx, d + o_src, d_off, d_len, nb, d_base, rec, txn_mode, d_st), "sstc_decode_blocks");
  return SSTC_OK;
}
} // namespace

int DecodeBlocks(sstc_ctx *ctx, const uint8_t *data, uint64_t bytes, const uint64_t *off, const uint64_t *len,
                 uint64_t nb, uint32_t txn_mode, DecodedBlocks &out) {
  try {
    sstc_records rec{};
    uint32_t *d_st = nullptr;
    uint8_t *d_x = nullptr;
    if (int r = decode_on_device(ctx, data, bytes, off, len, nb, txn_mode, out.base, rec, d_st, d_x, 0)) return r;
    const uint64_t n = out.base[nb];
    out.status.resize(nb);
    out.type.resize(n);
    out.key_len.resize(n);
    out.val_len.resize(n);
    out.txn.resize(n);
    out.key_off.resize(n);
    out.val_off.resize(n);
    bool ok = d2h(ctx, out.status.data(), d_st, nb * 4) && d2h(ctx, out.type.data(), rec.type, n) &&
              d2h(ctx, out.key_len.data(), rec.key_len, 4 * n) && d2h(ctx, out.val_len.data(), rec.val_len, 4 * n) &&
              d2h(ctx, out.txn.data(), rec.txn, 8 * n) && d2h(ctx, out.key_off.data(), rec.key_off, 8 * n) &&
              d2h(ctx, out.val_off.data(), rec.val_off, 8 * n);
    ok = sync(ctx) && ok;
    return ok ? SSTC_OK : SSTC_E_HIP;
  } catch (const std::exception &) {
    return SSTC_E_HIP;
  }
}

int DecodeTable(sstc_ctx *ctx, const uint8_t *data, uint64_t bytes, const uint64_t *off, const uint64_t *len,
                uint64_t nb, uint32_t txn_mode, DecodedTable &out) {
  try {
    sstc_records rec{};
    uint32_t *d_st = nullptr;
    uint8_t *d_x = nullptr;
    if (int r = decode_on_device(ctx, data, bytes, off, len, nb, txn_mode, out.base, rec, d_st, d_x,
                                 sizeof(sstc_record32)))
      return r;
    const uint64_t n = out.base[nb];
    auto *d_rec = reinterpret_cast<sstc_record32 *>(d_x);
    check(sstc_pack_records(ctx, rec, n, d_rec), "sstc_pack_records");
    out.status.resize(nb);
    out.n = n;
    out.rec.reset(new sstc_record32[n ? n : 1]); // default-initialised: the copy below fills it
    bool ok = d2h(ctx, out.status.data(), d_st, nb * 4) && d2h(ctx, out.rec.get(), d_rec, n * sizeof(sstc_record32));
    ok = sync(ctx) && ok;
    return ok ? SSTC_OK : SSTC_E_HIP;
  } catch (const std::exception &) {
    return SSTC_E_HIP;
  }
}

namespace {
int decode_host(sstc_ctx *ctx, std::vector<uint8_t> &data, const std::vector<uint64_t> &off,
                const std::vector<uint64_t> &len, uint32_t txn_mode, HostRecords &out) {
  return DecodeBlocks(ctx, data.data(), data.size(), off.data(), len.data(), off.size(), txn_mode, out);
}

struct CtxHolder { // one context + one non-blocking stream per host thread, destroyed at thread exit
  sstc_ctx *ctx = nullptr;
  hipStream_t stream = nullptr;
  ~CtxHolder() {
    if (ctx) sstc_ctx_destroy(ctx); // synchronises the stream
    if (stream) (void)hipStreamDestroy(stream);
  }
};
} // namespace

sstc_ctx *ThreadContext() {
  thread_local CtxHolder h;
  if (!h.ctx) {
    int dev = 0;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
      throw std::runtime_error("no HIP device: libsstcodec has no CPU path");
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    // its own stream: concurrent builders on pool threads overlap on the GPU
    // instead of queueing on the null stream
    if (hipStreamCreateWithFlags(&h.stream, hipStreamNonBlocking) != hipSuccess)
      throw std::runtime_error("hipStreamCreateWithFlags failed");
    check(sstc_ctx_create(dev, h.stream, &h.ctx), "sstc_ctx_create");
    // the runtime's pageable-copy paths set themselves up on first use (~10 ms
    // each way): once here, when the engine opens the codec, not inside the
    // first compaction's merge (ResidentInputs uploads from the file maps and
    // downloads into ordinary memory)
    void *d = nullptr;
    uint64_t word = 0;
    if (hipMalloc(&d, 64) == hipSuccess) {
      (void)hipMemcpyAsync(d, &word, 8, hipMemcpyHostToDevice, h.stream);
      (void)hipMemcpyAsync(&word, d, 8, hipMemcpyDeviceToHost, h.stream);
      (void)hipStreamSynchronize(h.stream);
      (void)hipFree(d);
    }
  }
  return h.ctx;
}

int TableReader::DecodeAll(uint32_t txn_mode, std::vector<uint8_t> &data, std::vector<uint8_t> &type,
                           std::vector<uint32_t> &key_len, std::vector<uint32_t> &val_len,
                           std::vector<uint64_t> &txn, std::vector<uint64_t> &key_off,
                           std::vector<uint64_t> &val_off) {
  const uint64_t nb = index_.size();
  data.resize(meta_off_);
  if (meta_off_ && !pread_all(fd_, data.data(), meta_off_, 0)) return SSTC_E_INVALID_ARG;
  std::vector<uint64_t> off(nb), len(nb);
  for (uint64_t b = 0; b < nb; b++) {
    off[b] = index_[b].offset;
    len[b] = index_[b].size;
    if (off[b] > meta_off_ || len[b] > meta_off_ - off[b]) return SSTC_E_INVALID_ARG;
  }
  HostRecords r;
  if (int rc = decode_host(ctx_, data, off, len, txn_mode, r)) return rc;
  type = std::move(r.type);
  key_len = std::move(r.key_len);
  val_len = std::move(r.val_len);
  txn = std::move(r.txn);
  key_off = std::move(r.key_off);
  val_off = std::move(r.val_off);
  for (uint64_t b = 0; b < nb; b++)
    if (r.status[b] != SSTC_BLK_OK) return static_cast<int>(r.status[b]);
  return SSTC_BLK_OK;
}

std::vector<std::unique_ptr<BlockReader>> TableReader::CreateAndSetupDataForBlockReaders(
    const std::vector<std::pair<BlockOffset, uint64_t>> &blocks, uint32_t txn_mode) const {
  // table_reader.cc:212-241 for every block: pread, then ONE batched decode
  const uint64_t nb = blocks.size();
  std::vector<std::unique_ptr<BlockReader>> out(nb);
  std::vector<uint64_t> off, len, which;
  std::vector<uint8_t> data;
  for (uint64_t b = 0; b < nb; b++) {
    const auto [o, l] = blocks[b];
    if (o > bytes_ || l > bytes_ - o) continue; // read failure -> nullptr (table_reader.cc:218-224)
    const uint64_t at = data.size();
    data.resize(at + l);
    if (l && !pread_all(fd_, data.data() + at, l, o)) {
      data.resize(at);
      continue;
    }
    off.push_back(at);
    len.push_back(l);
    which.push_back(b);
  }
  if (which.empty()) return out;
  HostRecords r;
  check(decode_host(ctx_, data, off, len, txn_mode, r), "block decode");
  for (uint64_t k = 0; k < which.size(); k++) {
    auto br = std::unique_ptr<BlockReader>(new BlockReader());
    br->buf_.assign(data.begin() + off[k], data.begin() + off[k] + len[k]);
    br->status_ = static_cast<int>(r.status[k]);
    for (uint64_t i = r.base[k]; i < r.base[k + 1]; i++) {
      br->type_.push_back(r.type[i]);
      br->key_len_.push_back(r.key_len[i]);
      br->val_len_.push_back(r.val_len[i]);
      br->txn_.push_back(r.txn[i]);
      br->key_off_.push_back(r.key_off[i] - off[k]);
      br->val_off_.push_back(r.val_len[i] == SSTC_NO_VALUE ? 0 : r.val_off[i] - off[k]);
    }
    out[which[k]] = std::move(br);
  }
  return out;
}

std::unique_ptr<BlockReader> TableReader::CreateAndSetupDataForBlockReader(BlockOffset offset, uint64_t block_size,
                                                                           uint32_t txn_mode) const {
  auto v = CreateAndSetupDataForBlockReaders({{offset, block_size}}, txn_mode);
  return std::move(v[0]);
}

// ---------------------------------------------------------- TableReaderIterator
void TableReaderIterator::Load() {
  if (loaded_) return;
  loaded_ = true;
  status_ = table_->DecodeAll(txn_mode_, data_, type_, key_len_, val_len_, txn_, key_off_, val_off_);
  n_ = status_ == SSTC_BLK_OK ? type_.size() : 0;
}

void TableReaderIterator::Seek(std::string_view key) {
  Load();
  uint64_t lo = 0, hi = n_; // first entry with key >= `key` (entries are key-ascending)
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    pos_ = mid;
    if (GetKey() < key) lo = mid + 1;
    else hi = mid;
  }
  pos_ = lo;
}

} // namespace sstc

// ----------------------------------------------------------------------- C shim
struct sstc_table_builder {
  sstc::TableBuilder tb;
};
struct sstc_table_reader {
  std::unique_ptr<sstc::TableReader> tr;
  uint32_t cached_mode = 0xFFFFFFFFu;
  std::vector<uint8_t> data, type;
  std::vector<uint32_t> kl, vl;
  std::vector<uint64_t> txn, ko, vo;
  int status = 0;
};

extern "C" {

int sstc_tb_create(const char *path, uint64_t block_threshold, sstc_ctx *ctx, sstc_table_builder **out) {
  if (!path || !ctx || !out || block_threshold == 0) return SSTC_E_INVALID_ARG;
  *out = new sstc_table_builder{sstc::TableBuilder(path, block_threshold, ctx)};
  return SSTC_OK;
}

int sstc_tb_open(sstc_table_builder *tb) {
  if (!tb) return SSTC_E_INVALID_ARG;
  return tb->tb.Open() ? SSTC_OK : SSTC_E_INVALID_ARG;
}

int sstc_tb_add(sstc_table_builder *tb, const uint8_t *key, uint32_t key_len, const uint8_t *val,
                uint32_t val_len, uint64_t txn, uint8_t type) {
  if (!tb || (!key && key_len)) return SSTC_E_INVALID_ARG;
  static const char kEmpty[1] = {0};
  std::string_view k(key ? reinterpret_cast<const char *>(key) : kEmpty, key_len);
  std::string_view v = val ? std::string_view(reinterpret_cast<const char *>(val), val_len) : std::string_view{};
  tb->tb.AddEntry(k, v, txn, type);
  return SSTC_OK;
}

int sstc_tb_add_batch(sstc_table_builder *tb, uint64_t n, const uint8_t *type, const uint32_t *key_len,
                      const uint32_t *val_len, const uint64_t *txn, const uint8_t *key_src,
                      const uint64_t *key_off, const uint8_t *val_src, const uint64_t *val_off) {
  if (!tb || (n && (!type || !key_len || !val_len || !txn || !key_off || !val_off))) return SSTC_E_INVALID_ARG;
  tb->tb.AddEntries(n, type, key_len, val_len, txn, key_src, key_off, val_src, val_off);
  return SSTC_OK;
}

int sstc_tb_finish(sstc_table_builder *tb) {
  if (!tb) return SSTC_E_INVALID_ARG;
  try {
    tb->tb.Finish();
  } catch (const std::exception &) {
    return SSTC_E_HIP;
  }
  return SSTC_OK;
}

uint64_t sstc_tb_file_size(const sstc_table_builder *tb) { return tb ? tb->tb.GetFileSize() : 0; }
uint64_t sstc_tb_num_blocks(const sstc_table_builder *tb) { return tb ? tb->tb.GetNumBlocks() : 0; }

int sstc_tb_destroy(sstc_table_builder *tb) {
  delete tb;
  return SSTC_OK;
}

int sstc_tr_open(const char *path, uint64_t file_size, sstc_ctx *ctx, sstc_table_reader **out) {
  if (!path || !ctx || !out) return SSTC_E_INVALID_ARG;
  sstc::TableReader *r = sstc::TableReader::Open(path, file_size, ctx);
  if (!r) return SSTC_E_INVALID_ARG;
  *out = new sstc_table_reader();
  (*out)->tr.reset(r);
  return SSTC_OK;
}

uint64_t sstc_tr_num_blocks(const sstc_table_reader *tr) { return tr ? tr->tr->GetBlockIndex().size() : 0; }

int sstc_tr_block_index(const sstc_table_reader *tr, uint64_t *blk_off, uint64_t *blk_len) {
  if (!tr || !blk_off || !blk_len) return SSTC_E_INVALID_ARG;
  const auto &idx = tr->tr->GetBlockIndex();
  for (size_t i = 0; i < idx.size(); i++) {
    blk_off[i] = idx[i].offset;
    blk_len[i] = idx[i].size;
  }
  return SSTC_OK;
}

static int tr_decode(sstc_table_reader *tr, uint32_t mode) {
  if (tr->cached_mode == mode) return tr->status;
  try {
    tr->status = tr->tr->DecodeAll(mode, tr->data, tr->type, tr->kl, tr->vl, tr->txn, tr->ko, tr->vo);
  } catch (const std::exception &) {
    tr->status = SSTC_E_HIP;
  }
  tr->cached_mode = mode;
  return tr->status;
}

uint64_t sstc_tr_num_records(sstc_table_reader *tr, uint32_t txn_mode) {
  if (!tr || tr_decode(tr, txn_mode) < 0) return 0;
  return tr->type.size();
}

int sstc_tr_decode_all(sstc_table_reader *tr, uint32_t txn_mode, uint8_t *type, uint32_t *key_len,
                       uint32_t *val_len, uint64_t *txn, uint64_t *key_off, uint64_t *val_off) {
  if (!tr) return SSTC_E_INVALID_ARG;
  const int st = tr_decode(tr, txn_mode);
  const size_t n = tr->type.size();
  if (n) {
    std::memcpy(type, tr->type.data(), n);
    std::memcpy(key_len, tr->kl.data(), 4 * n);
    std::memcpy(val_len, tr->vl.data(), 4 * n);
    std::memcpy(txn, tr->txn.data(), 8 * n);
    std::memcpy(key_off, tr->ko.data(), 8 * n);
    std::memcpy(val_off, tr->vo.data(), 8 * n);
  }
  return st;
}

int sstc_tr_destroy(sstc_table_reader *tr) {
  delete tr;
  return SSTC_OK;
}

} // extern "C"
