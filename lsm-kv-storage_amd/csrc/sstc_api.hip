// sstc_api.hip — extern "C" implementation of include/sstcodec.h.
//
// Host side of the boundary: argument checks, the per-context workspace and
// the launch sequences.  No compute happens here and there is no CPU fallback:
// every entry point fails with SSTC_E_NO_DEVICE when no HIP device exists.
#include <hip/hip_runtime.h>
#include <cstdlib>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>

#include "../../include/sstcodec.h"
#include "sstc_launch.h"

struct sstc_ctx {
  int device = 0;
  uint32_t num_cus = 256;
  hipStream_t stream = nullptr;
  hipEvent_t switch_ev = nullptr;           // orders a new stream after the old one
  uint64_t cap_records = 0, cap_scan = 0, cap_jump = 0;
  uint32_t scan_epoch = 0;                  // tag of the last scan on scan_ws (0: ws all zero)
  void *counters = nullptr;                 // 64 B: error counter
  unsigned long long *err_count = nullptr;  // 1
  uint64_t *scan_ws = nullptr;              // cap_scan
  uint64_t *P = nullptr;                    // cap_records + 1
  uint32_t *jump = nullptr;                 // cap_jump
  sstc::Arena arena;                        // compaction workspace
  struct HostPipe *pipe = nullptr;          // sstc_roundtrip_host staging (lazy)
};

// sstc_roundtrip_host: one stream per copy engine beside the context's stream,
// a ring of device buffer pairs ordered by events, pinned staging for the
// per-block arrays
constexpr int kPipeBuf = 3;
struct HostPipe {
  hipStream_t up = nullptr, down = nullptr;
  hipEvent_t ev_up[kPipeBuf] = {}, ev_comp[kPipeBuf] = {}, ev_down[kPipeBuf] = {};
  uint8_t *d_buf = nullptr; // kPipeBuf x (in, out) spans
  uint64_t cap_span = 0;
  uint64_t *d_blk = nullptr; // rel offset, length, out length (3 x nblocks) + status words
  uint64_t cap_blocks = 0;
  uint64_t *h_stage = nullptr; // pinned: rel offsets + lengths, then the results
  uint64_t cap_stage = 0;
};

namespace {

thread_local std::string g_last_error;

int fail(int code, const char *what, hipError_t e = hipSuccess) {
  g_last_error = what;
  if (e != hipSuccess) {
    g_last_error += ": ";
    g_last_error += hipGetErrorString(e);
  }
  return code;
}

#define SSTC_HIP(call, what)                                                                       \
  do {                                                                                             \
    hipError_t e_ = (call);                                                                        \
    if (e_ != hipSuccess) return fail(SSTC_E_HIP, what, e_);                                       \
  } while (0)

int bind_device(sstc_ctx *c) {
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess) return fail(SSTC_E_NO_DEVICE, "no HIP device");
  if (cur != c->device) SSTC_HIP(hipSetDevice(c->device), "hipSetDevice");
  return SSTC_OK;
}

template <class T> int grow(sstc_ctx *c, T *&p, uint64_t &cap, uint64_t need, const char *what) {
  if (need <= cap && p) return SSTC_OK;
  SSTC_HIP(hipStreamSynchronize(c->stream), "hipStreamSynchronize before workspace growth");
  if (p) SSTC_HIP(hipFree(p), "hipFree");
  p = nullptr;
  cap = 0;
  uint64_t n = need < 1024 ? 1024 : need;
  n += n / 4; // headroom
  if (hipMalloc(reinterpret_cast<void **>(&p), n * sizeof(T)) != hipSuccess) {
    p = nullptr;
    return fail(SSTC_E_NOMEM, what);
  }
  cap = n;
  return SSTC_OK;
}

// scan_ws is zeroed when (re)allocated; every scan on it then takes a fresh
// epoch (sstc::launch_scan), so no memset precedes a scan.  When the 14-bit
// epoch would wrap, the words are cleared once and the count restarts.
int ensure_scan_words(sstc_ctx *c, uint64_t words) {
  const uint64_t old = c->cap_scan;
  const uint64_t *before = c->scan_ws;
  if (int r = grow(c, c->scan_ws, c->cap_scan, words, "scan workspace")) return r;
  if (c->scan_ws != before || c->cap_scan != old) {
    SSTC_HIP(hipMemsetAsync(c->scan_ws, 0, c->cap_scan * sizeof(uint64_t), c->stream), "scan workspace clear");
    c->scan_epoch = 0;
  }
  return SSTC_OK;
}

int ensure_scan(sstc_ctx *c, uint64_t n) { return ensure_scan_words(c, sstc::scan_workspace_elems(n)); }

int next_epoch(sstc_ctx *c, uint32_t &epoch) {
  if (c->scan_epoch + 1 >= sstc::kScanEpochs) {
    SSTC_HIP(hipMemsetAsync(c->scan_ws, 0, c->cap_scan * sizeof(uint64_t), c->stream), "scan workspace clear");
    c->scan_epoch = 0;
  }
  epoch = ++c->scan_epoch;
  return SSTC_OK;
}

// every per-block scan a call may run: the u64 block scans and the encode's
// one-kernel block offsets (a tile per 256 blocks, finer than the scans'), so
// that no call after sstc_ctx_reserve grows the workspace
int ensure_blocks(sstc_ctx *c, uint64_t nb) {
  return ensure_scan_words(c, std::max({sstc::scan_workspace_elems(nb + 1), sstc::enc_offsets_workspace(nb),
                                        sstc::count_scan_workspace(nb)}));
}

int ensure_records(sstc_ctx *c, uint64_t nr) {
  if (int r = grow(c, c->P, c->cap_records, nr + 1, "record workspace")) return r;
  return ensure_scan(c, nr + 1);
}


bool bad_records(const sstc_records &r) {
  return !r.type || !r.key_len || !r.val_len || !r.txn || !r.key_off || !r.val_off;
}

} // namespace

extern "C" {

uint32_t sstc_version(void) { return SSTC_ABI_VERSION; }

// internal: lets the host-only translation units (host/*.cpp) report errors
// through sstc_last_error_string
int sstc__fail(int code, const char *what) { return fail(code, what); }
int sstc__ctx_device(const sstc_ctx *c) { return c ? c->device : -1; }
void *sstc__ctx_stream(const sstc_ctx *c) { return c ? static_cast<void *>(c->stream) : nullptr; }

// test hook (not in the public header): the context's scan epoch, to run scans
// across the 14-bit wrap of next_epoch without 16 k calls first
int sstc__ctx_set_scan_epoch(sstc_ctx *c, uint32_t epoch) {
  if (!c || epoch >= sstc::kScanEpochs) return SSTC_E_INVALID_ARG;
  c->scan_epoch = epoch;
  return SSTC_OK;
}

// test hook (not in the public header): corrupt the next compaction jobs'
// filter output on the device (sstc::Arena::fault) so the job's consistency
// guard can be exercised; 0 turns it off
int sstc__ctx_set_fault(sstc_ctx *c, uint32_t fault) {
  if (!c) return SSTC_E_INVALID_ARG;
  c->arena.fault = fault;
  return SSTC_OK;
}
// test hook: the compaction block split's plan for the context's next job
// (0 both paths, 1 the arithmetic chain alone, 2 the general walk alone) and
// how many jobs had to run their tail twice (a chain-alone plan that failed)
int sstc__ctx_seg_stats(sstc_ctx *c, uint32_t *mode, uint64_t *redos) {
  if (!c || !mode || !redos) return SSTC_E_INVALID_ARG;
  *mode = static_cast<uint32_t>(c->arena.seg_mode);
  *redos = c->arena.seg_redo_count;
  return SSTC_OK;
}
int sstc__ctx_sync(sstc_ctx *c) {
  if (!c || bind_device(c)) return SSTC_E_NO_DEVICE;
  return hipStreamSynchronize(c->stream) == hipSuccess ? SSTC_OK : SSTC_E_HIP;
}

const char *sstc_last_error_string(void) { return g_last_error.c_str(); }

int sstc_ctx_create(int device, void *stream, sstc_ctx **out) {
  if (!out) return fail(SSTC_E_INVALID_ARG, "out is NULL");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(SSTC_E_NO_DEVICE, "no HIP device: libsstcodec has no CPU path");
  if (device < 0 || device >= ndev) return fail(SSTC_E_INVALID_ARG, "device index out of range");
  sstc_ctx *c = new sstc_ctx();
  c->device = device;
  c->stream = static_cast<hipStream_t>(stream);
  if (int r = bind_device(c)) {
    delete c;
    return r;
  }
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
    c->num_cus = static_cast<uint32_t>(cus);
  if (hipMalloc(&c->counters, 64) != hipSuccess) {
    delete c;
    return fail(SSTC_E_NOMEM, "context counters");
  }
  c->err_count = static_cast<unsigned long long *>(c->counters);
  if (hipMemset(c->counters, 0, 64) != hipSuccess) {
    (void)hipFree(c->counters);
    delete c;
    return fail(SSTC_E_HIP, "context counters");
  }
  *out = c;
  return SSTC_OK;
}

int sstc_ctx_destroy(sstc_ctx *c) {
  if (!c) return SSTC_OK;
  bind_device(c);
  (void)hipStreamSynchronize(c->stream);
  if (c->arena.host) (void)hipHostFree(c->arena.host);
  if (c->arena.up) (void)hipHostFree(c->arena.up);
  if (HostPipe *hp = c->pipe) {
    for (hipStream_t st : {hp->up, hp->down})
      if (st) {
        (void)hipStreamSynchronize(st);
        (void)hipStreamDestroy(st);
      }
    for (int k = 0; k < kPipeBuf; k++)
      for (hipEvent_t e : {hp->ev_up[k], hp->ev_comp[k], hp->ev_down[k]})
        if (e) (void)hipEventDestroy(e);
    if (hp->d_buf) (void)hipFree(hp->d_buf);
    if (hp->d_blk) (void)hipFree(hp->d_blk);
    if (hp->h_stage) (void)hipHostFree(hp->h_stage);
    delete hp;
  }
  if (c->switch_ev) (void)hipEventDestroy(c->switch_ev);
  for (void *p : {c->counters, c->arena.base, static_cast<void *>(c->arena.lb),
                  static_cast<void *>(c->scan_ws),
                  static_cast<void *>(c->P), static_cast<void *>(c->jump)})
    if (p) (void)hipFree(p);
  delete c;
  return SSTC_OK;
}

// A context's workspace (scan scratch, record arrays, compaction arena, mapped
// host words, error counter) is shared by every call, so a stream switch must
// not let work on the new stream overtake work still queued on the old one:
// the new stream waits on an event recorded on the old stream.
int sstc_ctx_set_stream(sstc_ctx *c, void *stream) {
  if (!c) return fail(SSTC_E_INVALID_ARG, "ctx is NULL");
  hipStream_t ns = static_cast<hipStream_t>(stream);
  if (ns == c->stream) return SSTC_OK;
  if (int r = bind_device(c)) return r;
  if (!c->switch_ev) SSTC_HIP(hipEventCreateWithFlags(&c->switch_ev, hipEventDisableTiming), "stream switch event");
  SSTC_HIP(hipEventRecord(c->switch_ev, c->stream), "stream switch: record on the old stream");
  SSTC_HIP(hipStreamWaitEvent(ns, c->switch_ev, 0), "stream switch: new stream waits");
  c->stream = ns;
  return SSTC_OK;
}

int sstc_ctx_drop_stream(sstc_ctx *c) {
  if (!c) return fail(SSTC_E_INVALID_ARG, "ctx is NULL");
  c->stream = nullptr; // the caller synchronized it: nothing is recorded on it
  return SSTC_OK;
}

int sstc_ctx_reserve(sstc_ctx *c, uint64_t max_blocks, uint64_t max_records) {
  if (!c) return fail(SSTC_E_INVALID_ARG, "ctx is NULL");
  if (int r = bind_device(c)) return r;
  if (int r = ensure_blocks(c, max_blocks)) return r;
  if (int r = ensure_records(c, max_records)) return r;
  if (int r = grow(c, c->jump, c->cap_jump, sstc::segment_workspace_u32(max_records), "segmentation workspace"))
    return r;
  return SSTC_OK;
}

int sstc_ctx_error_count(sstc_ctx *c, uint64_t *out) {
  if (!c || !out) return fail(SSTC_E_INVALID_ARG, "NULL argument");
  if (int r = bind_device(c)) return r;
  unsigned long long v = 0;
  SSTC_HIP(hipMemcpyAsync(&v, c->err_count, sizeof(v), hipMemcpyDeviceToHost, c->stream), "error count copy");
  SSTC_HIP(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
  *out = v;
  return SSTC_OK;
}

int sstc_ctx_reset_errors(sstc_ctx *c) {
  if (!c) return fail(SSTC_E_INVALID_ARG, "ctx is NULL");
  if (int r = bind_device(c)) return r;
  SSTC_HIP(hipMemsetAsync(c->err_count, 0, sizeof(unsigned long long), c->stream), "reset errors");
  return SSTC_OK;
}

int sstc_count_records(sstc_ctx *c, const uint8_t *d_src, const uint64_t *d_blk_off,
                       const uint64_t *d_blk_len, uint64_t nblocks, uint64_t *d_rec_base) {
  if (!c || !d_rec_base || (nblocks && (!d_src || !d_blk_off || !d_blk_len)))
    return fail(SSTC_E_INVALID_ARG, "sstc_count_records: NULL argument");
  if (int r = bind_device(c)) return r;
  if (int r = ensure_scan_words(c, sstc::count_scan_workspace(nblocks))) return r;
  uint32_t ep = 0;
  if (int r = next_epoch(c, ep)) return r;
  sstc::CountScanArgs a{};
  a.src = d_src;
  a.blk_off = d_blk_off;
  a.blk_len = d_blk_len;
  a.nblocks = nblocks;
  a.rec_base = d_rec_base;
  a.ws = c->scan_ws;
  a.epoch = ep;
  a.lb_fail = c->err_count; // a look-back that gave up counts as an error
  SSTC_HIP(sstc::launch_count_scan(a, false, c->stream), "count + scan kernel");
  return SSTC_OK;
}

int sstc_decode_blocks(sstc_ctx *c, const uint8_t *d_src, const uint64_t *d_blk_off,
                       const uint64_t *d_blk_len, uint64_t nblocks, const uint64_t *d_rec_base,
                       sstc_records out, uint32_t txn_mode, uint32_t *d_block_status) {
  if (!c || (nblocks && (!d_src || !d_blk_off || !d_blk_len || !d_rec_base || bad_records(out))))
    return fail(SSTC_E_INVALID_ARG, "sstc_decode_blocks: NULL argument");
  if (txn_mode > SSTC_TXN_CORRECT) return fail(SSTC_E_INVALID_ARG, "bad txn_mode");
  if (int r = bind_device(c)) return r;
  sstc::DecArgs a{d_src, d_blk_off, d_blk_len, nblocks, d_rec_base, out, txn_mode, d_block_status,
                  c->err_count};
  SSTC_HIP(sstc::launch_decode(a, c->stream), "decode kernel");
  return SSTC_OK;
}

int sstc_pack_records(sstc_ctx *c, sstc_records in, uint64_t nrec, sstc_record32 *d_out) {
  if (!c || (nrec && (!d_out || bad_records(in)))) return fail(SSTC_E_INVALID_ARG, "sstc_pack_records: NULL argument");
  if (int r = bind_device(c)) return r;
  SSTC_HIP(sstc::launch_pack_records(in, nrec, d_out, c->stream), "pack kernel");
  return SSTC_OK;
}

int sstc_segment_records(sstc_ctx *c, const uint32_t *d_key_len, const uint32_t *d_val_len,
                         uint64_t nrec, uint64_t block_threshold, uint64_t *d_blk_first,
                         uint64_t *d_nblocks) {
  if (!c || !d_blk_first || !d_nblocks || (nrec && (!d_key_len || !d_val_len)))
    return fail(SSTC_E_INVALID_ARG, "sstc_segment_records: NULL argument");
  if (nrec >= 0xFFFFFFFFull) return fail(SSTC_E_INVALID_ARG, "too many records for one call");
  if (int r = bind_device(c)) return r;
  if (int r = ensure_records(c, nrec)) return r;
  if (int r = grow(c, c->jump, c->cap_jump, sstc::segment_workspace_u32(nrec), "segmentation workspace")) return r;
  // weights = entry_size + 16 (block_builder.cc:33), Pw = exclusive scan
  uint32_t ep = 0;
  if (int r = next_epoch(c, ep)) return r;
  SSTC_HIP(sstc::launch_scan_entry_sizes(d_key_len, d_val_len, nrec, 16, c->P, c->scan_ws, c->stream, ep,
                                                 c->err_count), "scan");
  SSTC_HIP(sstc::launch_segment(c->P, nrec, block_threshold, c->jump, d_nblocks, d_blk_first, c->stream),
           "segment kernels");
  return SSTC_OK;
}

int sstc_encode_blocks(sstc_ctx *c, const uint8_t *d_key_src, const uint8_t *d_val_src,
                       sstc_records in, uint64_t nrec, const uint64_t *d_blk_first,
                       uint64_t nblocks, uint64_t out_base, uint8_t *d_dst,
                       uint64_t *d_out_blk_off, uint64_t *d_out_blk_len) {
  if (!c || !d_out_blk_off || (nblocks && (!d_blk_first || !d_dst || !d_out_blk_len)) ||
      (nrec && (!d_key_src || !d_val_src || bad_records(in))))
    return fail(SSTC_E_INVALID_ARG, "sstc_encode_blocks: NULL argument");
  if (int r = bind_device(c)) return r;
  if (nblocks >= 0xFFFFFFFFull) return fail(SSTC_E_INVALID_ARG, "too many blocks for one call");
  if (int r = ensure_records(c, nrec)) return r;
  if (int r = ensure_blocks(c, nblocks)) return r; // the block-offset scan's workspace
  // block lengths (entry sizes summed per block), their scan = block offsets,
  // P (entry-size prefix) per block, then the block images
  uint32_t ep = 0;
  if (int r = next_epoch(c, ep)) return r;
  // block lengths and offsets; the entry offsets are scanned inside each
  // block's wave (no P pass: config-2 encode leg 134.7 -> 127.7 us,
  // profiles/r02_ab/encode_ab.md); c->P is the workspace of the blocks past an
  // LDS slot, which their own wave encodes (Zipf 64 KiB set 329 -> 236 us)
  SSTC_HIP(sstc::launch_enc_offsets(in.key_len, in.val_len, d_blk_first, nblocks, out_base, d_out_blk_off,
                                    d_out_blk_len, c->scan_ws, c->stream, ep, c->err_count),
           "block offsets");
  sstc::EncArgs a{d_key_src, d_val_src, in, d_blk_first, nblocks, c->P, d_out_blk_off, d_out_blk_len, d_dst};
  SSTC_HIP(sstc::launch_enc_emit(a, c->stream), "emit kernel");
  return SSTC_OK;
}

int sstc_roundtrip_blocks(sstc_ctx *c, const uint8_t *d_src, uint8_t *d_dst,
                          const uint64_t *d_blk_off, const uint64_t *d_blk_len, uint64_t nblocks,
                          uint32_t txn_mode, uint64_t *d_out_blk_len, uint32_t *d_block_status) {
  if (!c || (nblocks && (!d_src || !d_dst || !d_blk_off || !d_blk_len)))
    return fail(SSTC_E_INVALID_ARG, "sstc_roundtrip_blocks: NULL argument");
  if (d_src == d_dst && nblocks) return fail(SSTC_E_INVALID_ARG, "d_dst must not alias d_src");
  if (txn_mode > SSTC_TXN_CORRECT) return fail(SSTC_E_INVALID_ARG, "bad txn_mode");
  if (nblocks >= 0xFFFFFFFFull) return fail(SSTC_E_INVALID_ARG, "too many blocks for one call");
  if (int r = bind_device(c)) return r;
  sstc::RtArgs a{d_src, d_dst, d_blk_off, d_blk_len, nblocks, txn_mode, d_out_blk_len, d_block_status,
                 c->err_count, c->num_cus};
  SSTC_HIP(sstc::launch_roundtrip(a, c->stream), "roundtrip kernels");
  return SSTC_OK;
}

int sstc_roundtrip_host(sstc_ctx *c, const uint8_t *h_src, uint8_t *h_dst, uint64_t nbytes,
                        const uint64_t *h_blk_off, const uint64_t *h_blk_len, uint64_t nblocks, uint32_t txn_mode,
                        uint64_t chunk_bytes, uint64_t *h_out_blk_len, uint32_t *h_block_status) {
  if (!c || (nblocks && (!h_src || !h_dst || !h_blk_off || !h_blk_len)))
    return fail(SSTC_E_INVALID_ARG, "sstc_roundtrip_host: NULL argument");
  if (h_src == h_dst && nblocks) return fail(SSTC_E_INVALID_ARG, "h_dst must not alias h_src");
  if (txn_mode > SSTC_TXN_CORRECT) return fail(SSTC_E_INVALID_ARG, "bad txn_mode");
  if (chunk_bytes < 4096) return fail(SSTC_E_INVALID_ARG, "chunk_bytes must be >= 4096");
  if (nblocks >= 0xFFFFFFFFull) return fail(SSTC_E_INVALID_ARG, "too many blocks for one call");
  uint64_t prev_end = 0;
  for (uint64_t b = 0; b < nblocks; b++) {
    if (h_blk_off[b] < prev_end || h_blk_off[b] > nbytes || h_blk_len[b] > nbytes - h_blk_off[b])
      return fail(SSTC_E_INVALID_ARG, "sstc_roundtrip_host: blocks must be ascending, disjoint and inside h_src");
    prev_end = h_blk_off[b] + h_blk_len[b];
  }
  if (!nblocks) return SSTC_OK;
  if (int r = bind_device(c)) return r;
  // chunks: runs of consecutive blocks whose byte span (from the first block's
  // offset rounded down to 16) fits chunk_bytes; a larger block is a chunk alone
  struct Chunk {
    uint64_t b0, b1, lo, hi;
  };
  std::vector<Chunk> ch;
  uint64_t span = 0;
  for (uint64_t b = 0; b < nblocks;) {
    Chunk k{b, b + 1, h_blk_off[b] & ~uint64_t(15), h_blk_off[b] + h_blk_len[b]};
    while (k.b1 < nblocks && h_blk_off[k.b1] + h_blk_len[k.b1] - k.lo <= chunk_bytes) {
      k.hi = h_blk_off[k.b1] + h_blk_len[k.b1];
      k.b1++;
    }
    span = std::max(span, k.hi - k.lo);
    ch.push_back(k);
    b = k.b1;
  }
  if (!c->pipe) c->pipe = new HostPipe();
  HostPipe &hp = *c->pipe;
  if (!hp.up) {
    SSTC_HIP(hipStreamCreateWithFlags(&hp.up, hipStreamNonBlocking), "upload stream");
    SSTC_HIP(hipStreamCreateWithFlags(&hp.down, hipStreamNonBlocking), "download stream");
    for (int k = 0; k < kPipeBuf; k++) {
      SSTC_HIP(hipEventCreateWithFlags(&hp.ev_up[k], hipEventDisableTiming), "pipeline events");
      SSTC_HIP(hipEventCreateWithFlags(&hp.ev_comp[k], hipEventDisableTiming), "pipeline events");
      SSTC_HIP(hipEventCreateWithFlags(&hp.ev_down[k], hipEventDisableTiming), "pipeline events");
    }
  }
  SSTC_HIP(hipStreamSynchronize(hp.up), "hipStreamSynchronize");
  SSTC_HIP(hipStreamSynchronize(hp.down), "hipStreamSynchronize");
  const uint64_t slot = (span + 16 + 255) & ~uint64_t(255);
  if (int r = grow(c, hp.d_buf, hp.cap_span, 2 * kPipeBuf * slot, "pipeline buffers")) return r;
  if (int r = grow(c, hp.d_blk, hp.cap_blocks, 4 * nblocks, "pipeline block arrays")) return r;
  if (hp.cap_stage < 4 * nblocks) {
    if (hp.h_stage) (void)hipHostFree(hp.h_stage);
    hp.h_stage = nullptr;
    hp.cap_stage = 0;
    SSTC_HIP(hipHostMalloc(reinterpret_cast<void **>(&hp.h_stage), 4 * nblocks * sizeof(uint64_t)),
             "pipeline pinned staging");
    hp.cap_stage = 4 * nblocks;
  }
  uint64_t *rel = hp.h_stage, *len = hp.h_stage + nblocks;
  for (const Chunk &k : ch)
    for (uint64_t b = k.b0; b < k.b1; b++) {
      rel[b] = h_blk_off[b] - k.lo;
      len[b] = h_blk_len[b];
    }
  uint64_t *d_rel = hp.d_blk, *d_len = hp.d_blk + nblocks, *d_olen = hp.d_blk + 2 * nblocks;
  uint32_t *d_st = reinterpret_cast<uint32_t *>(hp.d_blk + 3 * nblocks);
  hipStream_t work = c->stream;
  SSTC_HIP(hipMemcpyAsync(d_rel, rel, 2 * nblocks * sizeof(uint64_t), hipMemcpyHostToDevice, hp.up),
           "block arrays upload");
  for (size_t i = 0; i < ch.size(); i++) {
    const Chunk &k = ch[i];
    const int s = static_cast<int>(i % kPipeBuf);
    uint8_t *d_in = hp.d_buf + 2 * s * slot, *d_out = d_in + slot;
    const uint64_t n = k.hi - k.lo;
    if (i >= kPipeBuf) SSTC_HIP(hipStreamWaitEvent(hp.up, hp.ev_comp[s], 0), "wait");
    SSTC_HIP(hipMemcpyAsync(d_in, h_src + k.lo, n, hipMemcpyHostToDevice, hp.up), "chunk upload");
    SSTC_HIP(hipEventRecord(hp.ev_up[s], hp.up), "event");
    SSTC_HIP(hipStreamWaitEvent(work, hp.ev_up[s], 0), "wait");
    if (i >= kPipeBuf) SSTC_HIP(hipStreamWaitEvent(work, hp.ev_down[s], 0), "wait");
    // rejected blocks and gaps keep the source bytes
    SSTC_HIP(hipMemcpyAsync(d_out, d_in, n, hipMemcpyDeviceToDevice, work), "chunk copy");
    sstc::RtArgs a{d_in, d_out, d_rel + k.b0, d_len + k.b0, k.b1 - k.b0, txn_mode, d_olen + k.b0, d_st + k.b0,
                   c->err_count, c->num_cus};
    SSTC_HIP(sstc::launch_roundtrip(a, work), "roundtrip kernels");
    SSTC_HIP(hipEventRecord(hp.ev_comp[s], work), "event");
    SSTC_HIP(hipStreamWaitEvent(hp.down, hp.ev_comp[s], 0), "wait");
    const uint64_t first = h_blk_off[k.b0];
    SSTC_HIP(hipMemcpyAsync(h_dst + first, d_out + (first - k.lo), k.hi - first, hipMemcpyDeviceToHost, hp.down),
             "chunk download");
    SSTC_HIP(hipEventRecord(hp.ev_down[s], hp.down), "event");
  }
  SSTC_HIP(hipMemcpyAsync(hp.h_stage + 2 * nblocks, d_olen, nblocks * (sizeof(uint64_t) + sizeof(uint32_t)),
                          hipMemcpyDeviceToHost, work),
           "results download");
  SSTC_HIP(hipStreamSynchronize(work), "hipStreamSynchronize");
  SSTC_HIP(hipStreamSynchronize(hp.down), "hipStreamSynchronize");
  if (h_out_blk_len) std::memcpy(h_out_blk_len, hp.h_stage + 2 * nblocks, nblocks * sizeof(uint64_t));
  if (h_block_status) std::memcpy(h_block_status, hp.h_stage + 3 * nblocks, nblocks * sizeof(uint32_t));
  return SSTC_OK;
}

int sstc_compact(sstc_ctx *c, const uint8_t *d_src, const uint64_t *d_blk_off, const uint64_t *d_blk_len,
                 uint64_t nblocks, const uint64_t *h_table_first_block, uint32_t ntables,
                 const sstc_compact_params *params, uint8_t *d_dst, uint64_t dst_cap, uint64_t *d_table_off,
                 uint64_t *d_table_len, uint64_t max_tables, sstc_compact_result *result) {
  if (!c || !h_table_first_block || !params || !d_dst || !d_table_off || !d_table_len || !result ||
      (nblocks && (!d_src || !d_blk_off || !d_blk_len)))
    return fail(SSTC_E_INVALID_ARG, "sstc_compact: NULL argument");
  if (params->block_threshold == 0 || params->table_limit == 0 || params->txn_mode > SSTC_TXN_CORRECT)
    return fail(SSTC_E_INVALID_ARG, "sstc_compact: bad parameters");
  if (h_table_first_block[0] != 0 || h_table_first_block[ntables] != nblocks)
    return fail(SSTC_E_INVALID_ARG, "sstc_compact: table ranges must cover the block list");
  for (uint32_t t = 0; t < ntables; t++)
    if (h_table_first_block[t] > h_table_first_block[t + 1])
      return fail(SSTC_E_INVALID_ARG, "sstc_compact: table ranges must be ascending");
  if (int r = bind_device(c)) return r;
  uint64_t res[5] = {0, 0, 0, 0, 0};
  std::string err;
  const int rc = sstc::compact_impl(c->arena, c->stream, c->err_count, d_src, d_blk_off, d_blk_len, nblocks,
                                    h_table_first_block, ntables, params->block_threshold, params->table_limit,
                                    params->base_level, params->txn_mode, d_dst, dst_cap, d_table_off, d_table_len,
                                    max_tables, res, err);
  result->records_in = res[0];
  result->records_kept = res[1];
  result->blocks_out = res[2];
  result->tables_out = res[3];
  result->bytes_out = res[4];
  if (rc != SSTC_OK) {
    // an error return can follow a mid-job fetch, which waits on the pack
    // kernel's sequence word rather than the stream: drain it so the call
    // returns with the stream idle, as documented
    (void)hipStreamSynchronize(c->stream);
    return fail(rc, ("sstc_compact: " + err).c_str());
  }
  return SSTC_OK;
}

int sstc_merge_records(sstc_ctx *c, const uint8_t *d_src, const uint64_t *d_blk_off, const uint64_t *d_blk_len,
                       uint64_t nblocks, const uint64_t *h_table_first_block, uint32_t ntables, uint32_t txn_mode,
                       sstc_merged_record *d_out, uint64_t max_records, sstc_merge_result *result) {
  if (!c || !h_table_first_block || !result || (nblocks && (!d_src || !d_blk_off || !d_blk_len)) ||
      (max_records && !d_out))
    return fail(SSTC_E_INVALID_ARG, "sstc_merge_records: NULL argument");
  if (txn_mode > SSTC_TXN_CORRECT) return fail(SSTC_E_INVALID_ARG, "sstc_merge_records: bad txn mode");
  if (ntables == 0 || h_table_first_block[0] != 0 || h_table_first_block[ntables] != nblocks)
    return fail(SSTC_E_INVALID_ARG, "sstc_merge_records: table ranges must cover the block list");
  for (uint32_t t = 0; t < ntables; t++)
    if (h_table_first_block[t] > h_table_first_block[t + 1])
      return fail(SSTC_E_INVALID_ARG, "sstc_merge_records: table ranges must be ascending");
  if (int r = bind_device(c)) return r;
  uint64_t res[5] = {0, 0, 0, 0, 0};
  std::string err;
  sstc::MergeOut mo{d_out, max_records, {0, 0}};
  const int rc = sstc::compact_impl(c->arena, c->stream, c->err_count, d_src, d_blk_off, d_blk_len, nblocks,
                                    h_table_first_block, ntables, 1, 1, 1, txn_mode, nullptr, 0, nullptr, nullptr,
                                    0, res, err, &mo);
  result->records = res[0];
  result->cross_ties = mo.ties[0];
  result->tie_diffs = mo.ties[1];
  if (rc != SSTC_OK) {
    (void)hipStreamSynchronize(c->stream);
    return fail(rc, ("sstc_merge_records: " + err).c_str());
  }
  return SSTC_OK;
}

int sstc_copy_probe(sstc_ctx *c, const uint8_t *d_src, uint8_t *d_dst, uint64_t nbytes) {
  if (!c || (nbytes && (!d_src || !d_dst))) return fail(SSTC_E_INVALID_ARG, "sstc_copy_probe: NULL argument");
  if ((nbytes | reinterpret_cast<uintptr_t>(d_src) | reinterpret_cast<uintptr_t>(d_dst)) & 15u)
    return fail(SSTC_E_INVALID_ARG, "sstc_copy_probe: size and pointers must be 16 B aligned");
  if (int r = bind_device(c)) return r;
  SSTC_HIP(sstc::launch_copy_probe(d_src, d_dst, nbytes / 16, c->stream), "sstc_copy_probe launch");
  return SSTC_OK;
}

int sstc_open_tables(sstc_ctx *c, const uint8_t *d_src, uint64_t src_bytes, const uint64_t *h_tab_off,
                     const uint64_t *h_tab_bytes, uint32_t ntables, uint64_t max_blocks, uint64_t *d_blk_off,
                     uint64_t *d_blk_len, uint64_t *d_first_key_off, uint32_t *d_first_key_len,
                     uint64_t *d_last_key_off, uint32_t *d_last_key_len, uint64_t *d_table_first_block,
                     uint64_t *h_table_first_block, int32_t *h_table_status, uint64_t *h_footer) {
  if (!c || !h_table_first_block || (ntables && (!d_src || !h_tab_off || !h_tab_bytes || !h_table_status)))
    return fail(SSTC_E_INVALID_ARG, "sstc_open_tables: NULL argument");
  if (max_blocks && (!d_blk_off || !d_blk_len || !d_first_key_off || !d_first_key_len || !d_last_key_off ||
                     !d_last_key_len))
    return fail(SSTC_E_INVALID_ARG, "sstc_open_tables: NULL output array");
  for (uint32_t t = 0; t < ntables; t++)
    if (h_tab_off[t] > src_bytes || h_tab_bytes[t] > src_bytes - h_tab_off[t])
      return fail(SSTC_E_INVALID_ARG, "sstc_open_tables: table image outside d_src");
  if (int r = bind_device(c)) return r;
  const sstc::OpenOut o{d_blk_off, d_blk_len, d_first_key_off, d_last_key_off, d_table_first_block,
                        d_first_key_len, d_last_key_len};
  std::string err;
  const int rc = sstc::open_tables_impl(c->arena, c->stream, d_src, src_bytes, h_tab_off, h_tab_bytes, ntables,
                                        max_blocks, o, h_table_first_block, h_table_status, h_footer, err);
  if (rc != SSTC_OK) return fail(rc, ("sstc_open_tables: " + err).c_str());
  return SSTC_OK;
}

int sstc_get_batch(sstc_ctx *c, const uint8_t *d_src, const sstc_block_index *index, const uint32_t *d_q_table,
                   const uint8_t *d_q_keys, uint64_t q_keys_bytes, const uint64_t *d_q_key_off,
                   const uint32_t *d_q_key_len, uint64_t nq, uint32_t *d_out_type, uint64_t *d_out_val_off,
                   uint32_t *d_out_val_len, uint64_t *d_out_block) {
  if (!c || !index) return fail(SSTC_E_INVALID_ARG, "sstc_get_batch: NULL argument");
  if (nq && (!d_src || !index->blk_off || !index->blk_len || !index->last_key_off || !index->last_key_len ||
             !index->keys || !index->table_first_block || !d_q_table || !d_q_keys || !d_q_key_off ||
             !d_q_key_len || !d_out_type || !d_out_val_off || !d_out_val_len))
    return fail(SSTC_E_INVALID_ARG, "sstc_get_batch: NULL argument");
  if (int r = bind_device(c)) return r;
  const sstc::GetArgs a{d_src,        index->blk_off,  index->blk_len, index->last_key_off, index->last_key_len,
                        index->keys,  index->table_first_block, index->ntables, d_q_table, d_q_keys, d_q_key_off,
                        d_q_key_len,  nq, d_out_type, d_out_val_off, d_out_val_len, d_out_block, c->err_count,
                        index->src_bytes, index->keys_bytes, q_keys_bytes};
  SSTC_HIP(sstc::launch_get(a, c->stream), "sstc_get_batch launch");
  return SSTC_OK;
}

} // extern "C"
