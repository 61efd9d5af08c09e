// resident.cpp — sstc::ResidentInputs (include/sstc_table.h): the input SSTs
// of one merge mapped into one host range, uploaded once, and merged on the
// device into the order db::MergeIterator walks them
// (db/merge_iterator.cc:34-46,79-92 over the iterators of
// db/compact.cc:186-230).
//
// Host range: a PROT_NONE reservation with every input file mapped read-only
// at a page-aligned offset inside it (MAP_FIXED), so one pointer range covers
// all inputs and a view's offset in the range is also its offset in the
// device copy.  The maps are the page cache itself: no read into fresh memory
// (a page fault and a zeroed page per 4 KiB), no host copy; the upload is one
// H2D per table straight from its map.
#include "sstc_table.h"

#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <map>
#include <stdexcept>

extern "C" int sstc__ctx_device(const sstc_ctx *ctx);   // sstc_api.hip
extern "C" void *sstc__ctx_stream(const sstc_ctx *ctx); // sstc_api.hip

namespace sstc {
namespace {

constexpr uint64_t kPage = 4096;

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// per-thread, per-device grow-only device buffer for the merged records (only
// needed until they are downloaded)
struct RecStage {
  void *p = nullptr;
  uint64_t cap = 0;
  ~RecStage() {
    if (p) (void)hipFree(p);
  }
};
thread_local std::map<int, RecStage> g_rec_stage;

thread_local ResidentInputs *g_active = nullptr;

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

} // namespace

ResidentInputs *ResidentInputs::Active() { return g_active; }
void ResidentInputs::Activate() { g_active = this; }
void ResidentInputs::Deactivate() {
  if (g_active == this) g_active = nullptr;
}

ResidentInputs::~ResidentInputs() {
  const double t0 = TraceHostOn() ? now_ms() : 0;
  struct Trace {
    double t0;
    ~Trace() {
      if (t0 > 0) TraceHost("resident inputs: teardown (device copy freed, maps unmapped)", now_ms() - t0);
    }
  } trace{t0};
  Deactivate();
  if (helper_.joinable()) helper_.join();
  if (drec_ || dev_) {
    DeviceScope on(device_);
    RecStage &stage = g_rec_stage[device_];
    if (drec_ && !stage.p) { // lent back to this thread's merge buffer
      stage.p = drec_;
      stage.cap = drec_cap_;
    } else if (drec_) {
      (void)hipFree(drec_);
    }
    if (dev_) (void)hipFree(dev_);
  }
  if (host_) munmap(host_, bytes_);
}

// the helper thread: records device -> host in chunks, a small first one so
// the walk starts early, each published by ready_ once it has landed
void ResidentInputs::Download() {
  try {
    DeviceScope on(device_);
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) throw std::runtime_error("stream");
    // test hook: the download fails once this many records are down (the
    // drop-in MergeIterator must continue on the heaps)
    static const char *fail_at_env = std::getenv("SSTC_TEST_DOWNLOAD_FAIL_AT");
    const uint64_t fail_at = fail_at_env ? std::strtoull(fail_at_env, nullptr, 10) : ~0ull;
    uint64_t done = 0, chunk = 1ull << 15;
    while (done < n_) {
      if (done >= fail_at) throw std::runtime_error("test hook: download stopped");
      const uint64_t k = std::min(chunk, n_ - done);
      if (hipMemcpyAsync(rec_.get() + done, static_cast<sstc_merged_record *>(drec_) + done,
                         k * sizeof(sstc_merged_record), hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
        throw std::runtime_error("D2H");
      done += k;
      ready_.store(done, std::memory_order_release);
      chunk = std::min<uint64_t>(chunk * 4, 1ull << 20);
    }
    (void)hipStreamDestroy(s);
  } catch (const std::exception &) {
    failed_.store(1, std::memory_order_release);
  }
}

uint64_t ResidentInputs::WaitRecords(uint64_t k) {
  k = std::min(k, n_);
  for (uint64_t spins = 0;; spins++) {
    const uint64_t r = ready_.load(std::memory_order_acquire);
    if (r >= k) return r;
    if (failed_.load(std::memory_order_acquire)) throw std::runtime_error("ResidentInputs: D2H of the merged records failed");
    if (spins > 64) std::this_thread::yield();
  }
}

uint32_t ResidentInputs::InputOf(uint64_t key_off) const {
  // last table whose range starts at or before the offset
  const auto it = std::upper_bound(table_base_.begin(), table_base_.end(), key_off);
  return static_cast<uint32_t>(it - table_base_.begin()) - 1;
}

std::shared_ptr<ResidentInputs> ResidentInputs::Create(sstc_ctx *ctx, const std::vector<Input> &inputs,
                                                       uint32_t txn_mode, std::string *why) {
  auto fail = [why](std::string w) -> std::shared_ptr<ResidentInputs> {
    if (why) *why = std::move(w);
    return nullptr;
  };
  if (!ctx || inputs.empty()) return fail("no inputs");
  const double t0 = now_ms();
  std::shared_ptr<ResidentInputs> r(new ResidentInputs());
  // layout: table t's file bytes [0, hi_t) at table_base_[t], page aligned
  const uint32_t nt = static_cast<uint32_t>(inputs.size());
  std::vector<uint64_t> hi(nt), lo(nt);
  uint64_t total = 0, nblocks = 0;
  for (uint32_t t = 0; t < nt; t++) {
    const Input &in = inputs[t];
    if (in.off.empty() || in.off.size() != in.len.size()) return fail("an input table has no blocks");
    lo[t] = UINT64_MAX;
    for (size_t b = 0; b < in.off.size(); b++) {
      lo[t] = std::min(lo[t], in.off[b]);
      hi[t] = std::max(hi[t], in.off[b] + in.len[b]);
    }
    r->table_base_.push_back(total);
    total += (hi[t] + kPage - 1) / kPage * kPage;
    nblocks += in.off.size();
  }
  void *range = mmap(nullptr, total, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  if (range == MAP_FAILED) return fail("cannot reserve the host range");
  r->host_ = static_cast<uint8_t *>(range);
  r->bytes_ = total;
  // the maps are made (pages populated) by a helper thread one table ahead of
  // the uploads: table t goes up while table t + 1 is being mapped
  std::atomic<uint32_t> mapped{0};
  std::atomic<int> map_failed{-1};
  std::thread mapper([&] {
    for (uint32_t t = 0; t < nt; t++) {
      const int fd = open(inputs[t].path.c_str(), O_RDONLY | O_CLOEXEC);
      struct stat st;
      const bool big_enough = fd >= 0 && fstat(fd, &st) == 0 && static_cast<uint64_t>(st.st_size) >= hi[t]; // no page past EOF
      void *p = big_enough ? mmap(r->host_ + r->table_base_[t], hi[t], PROT_READ,
                                  MAP_PRIVATE | MAP_FIXED | MAP_POPULATE, fd, 0)
                           : MAP_FAILED;
      if (fd >= 0) close(fd);
      if (p == MAP_FAILED) {
        map_failed.store(static_cast<int>(t), std::memory_order_release);
        return;
      }
      mapped.store(t + 1, std::memory_order_release);
    }
  });
  struct Join {
    std::thread &th;
    ~Join() { th.join(); }
  } join_mapper{mapper};
  const int dev = sstc__ctx_device(ctx);
  hipStream_t s = static_cast<hipStream_t>(sstc__ctx_stream(ctx));
  DeviceScope on(dev);
  r->device_ = dev;
  if (hipMalloc(reinterpret_cast<void **>(&r->dev_), total) != hipSuccess) {
    r->dev_ = nullptr;
    return fail("hipMalloc of the device copy");
  }
  double t_wait = 0;
  for (uint32_t t = 0; t < nt; t++) {
    const double w0 = now_ms();
    while (mapped.load(std::memory_order_acquire) <= t) {
      const int bad = map_failed.load(std::memory_order_acquire);
      if (bad >= 0) return fail("cannot map " + inputs[bad].path);
      std::this_thread::yield();
    }
    t_wait += now_ms() - w0;
    const uint64_t a = r->table_base_[t] + lo[t];
    if (hipMemcpyAsync(r->dev_ + a, r->host_ + a, hi[t] - lo[t], hipMemcpyHostToDevice, s) != hipSuccess)
      return fail("H2D of the inputs");
  }
  const double t1 = t0 + t_wait; // (trace: "map" = the time the uploads waited for maps)
  // block index (range offsets), table first blocks
  std::vector<uint64_t> idx(2 * nblocks), tfb(nt + 1, 0);
  for (uint32_t t = 0, b = 0; t < nt; t++) {
    for (size_t i = 0; i < inputs[t].off.size(); i++, b++) {
      idx[b] = r->table_base_[t] + inputs[t].off[i];
      idx[nblocks + b] = inputs[t].len[i];
    }
    tfb[t + 1] = tfb[t] + inputs[t].off.size();
  }
  RecStage &stage = g_rec_stage[dev];
  uint64_t *d_idx = nullptr;
  if (hipMalloc(reinterpret_cast<void **>(&d_idx), 16 * nblocks) != hipSuccess) return fail("hipMalloc");
  struct Free {
    void *p;
    ~Free() { (void)hipFree(p); }
  } free_idx{d_idx};
  if (hipMemcpyAsync(d_idx, idx.data(), 16 * nblocks, hipMemcpyHostToDevice, s) != hipSuccess)
    return fail("H2D of the block index");
  const double t2 = now_ms();
  sstc_merge_result mr{};
  int rc = SSTC_E_CAPACITY;
  for (int attempt = 0; attempt < 2 && rc == SSTC_E_CAPACITY; attempt++) {
    if (attempt) { // the first call said how many records there are
      if (stage.p) (void)hipFree(stage.p);
      stage.p = nullptr;
      stage.cap = 0;
      const uint64_t cap = mr.records + mr.records / 8 + 1024;
      if (hipMalloc(&stage.p, cap * sizeof(sstc_merged_record)) != hipSuccess) return fail("hipMalloc");
      stage.cap = cap;
    }
    rc = sstc_merge_records(ctx, r->dev_, d_idx, d_idx + nblocks, nblocks, tfb.data(), nt, txn_mode,
                            static_cast<sstc_merged_record *>(stage.p), stage.cap, &mr);
  }
  if (rc != SSTC_OK) return fail(std::string("device merge: ") + sstc_last_error_string());
  const double t3 = now_ms();
  r->n_ = mr.records;
  r->cross_ties_ = mr.cross_ties;
  r->tie_diffs_ = mr.tie_diffs;
  r->rec_.reset(new sstc_merged_record[r->n_ ? r->n_ : 1]);
  r->drec_ = stage.p; // lent to the download until r is destroyed
  r->drec_cap_ = stage.cap;
  stage.p = nullptr;
  stage.cap = 0;
  r->helper_ = std::thread([p = r.get()] { p->Download(); });
  const double t4 = now_ms();
  r->ms[0] = t1 - t0;
  r->ms[1] = t2 - t0;
  r->ms[2] = t3 - t2;
  r->ms[3] = t4 - t3;
  if (TraceHostOn()) {
    TraceHost("resident inputs: waits for the maps", t1 - t0);
    TraceHost("resident inputs: maps + H2D (overlapped)", t2 - t0);
    TraceHost("resident inputs: device decode + merge (incl. H2D)", t3 - t2);
    TraceHost("resident inputs: download thread started", t4 - t3);
  }
  return r;
}

} // namespace sstc
