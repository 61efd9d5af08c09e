// sstc_launch.h — kernel argument blocks and host-side launch wrappers.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/sstcodec.h"

namespace sstc {

constexpr uint32_t kRtSlotBytes = 4608; // LDS bytes per wave in rt_fast_kernel

struct RtArgs {
  const uint8_t *src;
  uint8_t *dst;
  const uint64_t *blk_off;
  const uint64_t *blk_len;
  uint64_t nblocks;
  uint32_t txn_mode;
  uint64_t *out_len;   // may be null
  uint32_t *status;    // may be null
  unsigned long long *err_count;
  uint32_t num_cus;
  uint32_t xcd = 0; // XCD-aware block order (set by the launcher)
};

// 32 B merge key of one record (compaction): 16 B big-endian key prefix (zero
// padded), merge txn, key length, record id.  The merge txn is the txn as read
// (compat or correct) run through a running minimum over the record's key
// group in its input run, so an input whose versions of a key are not in
// descending txn order as read (the compat empty-value quirk turns txn t into
// (t & 0xffffffff) << 32, block_reader.cc:109-111) merges the way the
// reference's MergeIterator heap pops it: a run's records leave in file order
// and each competes with the others' heads under the smallest txn before it.
// kSkRead in kl marks a record whose merge txn differs from its txn as read:
// the filter re-reads that one from the source.
constexpr uint32_t kSkRead = 1u << 31;
struct __attribute__((aligned(16))) SortKey {
  uint64_t p0, p1, tx;
  uint32_t kl, id; // kl: key length | kSkRead
};

// per-record fields of the compaction job beside its SortKey (key length and
// txn live there): one 16 B gather per record instead of one per SoA column
struct __attribute__((aligned(16))) RecX {
  uint64_t ko;   // key offset in the source bytes (value offset = ko + kl + 4)
  uint32_t vl;   // value length, kNoValue for a DELETE
  uint32_t type; // ValueType
};

struct DecArgs {
  const uint8_t *src;
  const uint64_t *blk_off;
  const uint64_t *blk_len;
  uint64_t nblocks;
  const uint64_t *rec_base;
  sstc_records out;
  uint32_t txn_mode;
  uint32_t *status; // may be null
  unsigned long long *err_count;
  SortKey *sk = nullptr; // optional merge keys (compaction)
  // optional: count of records that sort before their predecessor in the block
  unsigned long long *unsorted = nullptr;
  RecX *rx = nullptr; // compaction: written instead of the `out` columns
  uint32_t xcd = 0;
  // compaction: the guard word; kGuardInv is set when a record's merge txn
  // differs from its txn as read (SortKey, kSkRead)
  unsigned long long *inv = nullptr;
};

// consistency-guard bits of the compaction job (sstc_compact.hip)
constexpr unsigned long long kGuardMergeId = 1, kGuardEntry = 2, kGuardBlockRange = 4, kGuardMeta = 8,
                             kGuardFooter = 16, kGuardLayout = 32, kGuardLongGroup = 64,
                             kGuardInv = 128, kGuardTieCross = 256, kGuardTieDiff = 512;
// Equal (key, merge txn) neighbours in the merged order from different inputs
// (kGuardTieCross) and such neighbours whose records differ (kGuardTieDiff):
// with both, the reference's heap (merge_iterator.h:91-95) may order them
// otherwise than this job, so the job writes nothing and returns
// SSTC_E_TIE_ORDER (the writers stand down on both bits).
constexpr unsigned long long kGuardTieBoth = kGuardTieCross | kGuardTieDiff;
// The block split's arithmetic chain (seg_arith_*) failed: kGuardArithFail is
// a note (the general walk ran behind it); kGuardSplitRedo means the general
// walk was NOT enqueued (the context's last job took the chain, SegMode::
// kArithOnly), so the split is not the greedy one: every writer stands down
// and the host runs the job's tail again with the general walk.
constexpr unsigned long long kGuardArithFail = 1024, kGuardSplitRedo = 2048;
// A decoupled look-back of the job gave up waiting for a predecessor tile
// (kLbSpinLimit, sstc_device.h LbFail): its prefix sums are wrong, the writers
// stand down and the job returns SSTC_E_INTERNAL.
constexpr unsigned long long kGuardLookback = 4096;
// the job's writers (encode, meta, footer) write nothing
__host__ __device__ inline bool writers_stand_down(unsigned long long g) {
  return (g & (kGuardSplitRedo | kGuardLookback)) || (g & kGuardTieBoth) == kGuardTieBoth;
}
// block split launch plan (launch_segment): both paths (the general walk's
// kernels return at once when the chain holds), the chain alone, the walk alone
enum class SegMode : uint32_t { kBoth = 0, kArithOnly = 1, kGeneralOnly = 2 };

struct EncArgs {
  const uint8_t *key_src;
  const uint8_t *val_src;
  sstc_records in;
  const uint64_t *blk_first;
  uint64_t nblocks;
  // mode 1 (entries_in_src): exclusive scan of the entry sizes, nrec + 1;
  // mode 0: a workspace (nrec + 1) the wave of a block past its LDS slot fills
  // with the block-relative entry offsets (other blocks scan them in the wave)
  const uint64_t *P;
  const uint64_t *out_blk_off;
  const uint64_t *out_blk_len;
  uint8_t *dst;
  uint32_t entries_in_src = 0; // records decoded from blocks in key_src (== val_src)
  uint32_t xcd = 0; // block order: 0 dispatch, 1 XCD-grouped ranges (exact grid), 2 XCD chunks (bound grid)
  // mode 1: most blocks are past the LDS slot (the build with wider copies,
  // launch_enc_emit); 0: most fit it (the 8-waves-per-SIMD build)
  uint32_t large_blocks = 0;
  // optional (compaction, entries_in_src): per block 4 words -- min txn, max
  // txn (table footer, table_builder.cc:47-49), and the first / last entry's
  // key offset | key length << 40 (meta entries, AddIndexBlockEntry): one
  // 4-lane store per block
  uint64_t *bmeta = nullptr;
  // optional capacity guard (compaction): nothing is written when *need > cap
  const uint64_t *need = nullptr;
  uint64_t cap = 0;
  __device__ bool over() const { return (need && *need > cap) || (guard && writers_stand_down(*guard)); }
  // optional consistency guard (compaction, mode 1): every block's output range
  // must lie in [0, cap), every entry inside its block image (offset + size
  // <= data bytes, size >= its header + key) and its source inside
  // [5, *src_end); a block that fails is not written and sets *guard
  const uint64_t *src_end = nullptr;
  unsigned long long *guard = nullptr;
  // optional (compaction): the block count is on the device (nb_dev) and
  // nblocks is only its host-side upper bound (the grid); a count past the
  // bound means a corrupt layout: every wave stands down
  const uint64_t *nb_dev = nullptr;
};

// kGuardLongGroup / kGuardInv are notes, not faults: a key's versions continue
// over more than kGroupCarryBlocks blocks / some group is out of txn order as
// read.  Both together send the check kernel's last workgroup through the
// repair pass (long_carry_repair: the carries as one segmented min-scan).
// blocks a thread of ck_check_blocks_kernel walks back for a key group's carry
constexpr uint32_t kGroupCarryBlocks = 64;

// point lookups (sstc_get.hip)
struct GetArgs {
  const uint8_t *src;
  const uint64_t *blk_off, *blk_len, *lk_off;
  const uint32_t *lk_len;
  const uint8_t *keys;
  const uint64_t *tfb;
  uint32_t ntables;
  const uint32_t *q_table;
  const uint8_t *q_keys;
  const uint64_t *q_key_off;
  const uint32_t *q_key_len;
  uint64_t nq;
  uint32_t *out_type;
  uint64_t *out_val_off;
  uint32_t *out_val_len;
  uint64_t *out_block; // may be null
  unsigned long long *err_count;
  uint64_t src_bytes, keys_bytes, q_keys_bytes; // read bounds
};
hipError_t launch_get(const GetArgs &a, hipStream_t s);

hipError_t launch_roundtrip(const RtArgs &a, hipStream_t s);
hipError_t launch_copy_probe(const uint8_t *src, uint8_t *dst, uint64_t n16, hipStream_t s);
// record bases rec_base[0..nblocks] (exclusive scan of the blocks' entry
// counts) in one kernel; start: the compaction job's first host hand-off as
// well (count_scan_kernel<true>, sstc_kernels.hip)
struct CountScanArgs {
  const uint8_t *src;
  const uint64_t *blk_off, *blk_len;
  uint64_t nblocks;
  uint64_t *rec_base; // nblocks + 1
  // count_scan_workspace(nblocks) words: [0] ticket (start), status words at
  // + 32.  start: zero at entry, left zero (epoch 0); else epoch-tagged words
  // (a context's scan workspace, next_epoch)
  uint64_t *ws;
  uint32_t epoch;
  // start only
  uint64_t *part;                       // 2 x count_scan_tiles(nblocks)
  const uint64_t *tfb;                  // ntfb table first blocks (device-readable)
  uint64_t ntfb;
  uint64_t *run_start;                  // ntfb: rec_base[tfb[i]]
  const unsigned long long *err_count;  // snapshot into *errs
  uint64_t *errs;
  unsigned long long *bad, *guard;      // cleared (guard[1] = the source end)
  uint64_t *host;                       // pinned: [0] input bytes, [1..ntfb] run starts
  uint64_t seq, flag;                   // host[flag] = seq last
  // not start: counts a look-back that gave up (a context's error counter);
  // start: such a tile makes host[0] = ~0 and sets kGuardLookback instead
  unsigned long long *lb_fail = nullptr;
};
uint64_t count_scan_tiles(uint64_t nblocks);
uint64_t count_scan_workspace(uint64_t nblocks);
hipError_t launch_count_scan(const CountScanArgs &a, bool start, hipStream_t s);
hipError_t launch_decode(const DecArgs &a, hipStream_t s);
hipError_t launch_pack_records(const sstc_records &in, uint64_t nrec, sstc_record32 *out, hipStream_t s);
uint64_t scan_workspace_elems(uint64_t n);
// look-back status words a scan of n items needs cleared (0: single-workgroup scan)
uint64_t scan_status_words(uint64_t n);
// ws_zeroed: the caller cleared scan_status_words(n) words of ws in an earlier
// kernel on the same stream (seg_walk_kernel's zws, ...), no memset here.
// epoch (1..kScanEpochs-1): ws holds status words of earlier scans tagged with
// other epochs (a context's own workspace, see sstc_api.hip next_epoch): no
// memset either.  Neither: the status words are cleared with a memset.
constexpr uint32_t kScanEpochs = 1u << 14;
// guard: a look-back that gave up sets kGuardLookback there (may be null).
hipError_t launch_scan(const uint64_t *in, uint64_t n, uint64_t carry_in, uint64_t *out, uint64_t *ws,
                       hipStream_t s, bool ws_zeroed = false, uint32_t epoch = 0,
                       unsigned long long *guard = nullptr);
// out = exclusive scan of the entry sizes (+ add) of records (klen, vlen);
// err_count counts a look-back that gave up (may be null)
hipError_t launch_scan_entry_sizes(const uint32_t *klen, const uint32_t *vlen, uint64_t nrec, uint64_t add,
                                   uint64_t *out, uint64_t *ws, hipStream_t s, uint32_t epoch,
                                   unsigned long long *err_count = nullptr);
// block offsets (nblocks + 1) and lengths of a records -> blocks encode: block
// lengths by reduction over each block's records and their scan, one kernel
// (ws: enc_offsets_workspace(nblocks) words, epoch != 0) or, for one
// workgroup's worth of blocks / epoch 0, a sum kernel + a scan
uint64_t enc_offsets_workspace(uint64_t nblocks);
hipError_t launch_enc_offsets(const uint32_t *kl, const uint32_t *vl, const uint64_t *blk_first, uint64_t nblocks,
                              uint64_t out_base, uint64_t *blk_off, uint64_t *blk_len, uint64_t *ws, hipStream_t s,
                              uint32_t epoch, unsigned long long *err_count = nullptr);
hipError_t launch_enc_emit(const EncArgs &a, hipStream_t s);
// greedy segmentation; J = segment_workspace_u32(nrec) u32 of device workspace
uint64_t segment_workspace_u32(uint64_t nrec);
// ends: optional sorted segment-end list (a coarser segmentation's starts with
// its sentinel, e.g. the output tables'): no segment crosses one of them
hipError_t launch_segment(const uint64_t *Pw, uint64_t nrec, uint64_t threshold, uint32_t *J,
                          uint64_t *d_nblocks, uint64_t *blk_first, hipStream_t s,
                          const uint64_t *ends = nullptr, const uint64_t *d_nends = nullptr, uint64_t add = 0,
                          bool long_segments = false, const uint64_t *d_nrec = nullptr,
                          SegMode mode = SegMode::kBoth, unsigned long long *fail = nullptr);
// d_nrec: the record count on the device (nrec is then only its upper bound:
// grids and workspace are sized by nrec, the kernels segment *d_nrec records)

// persistent device workspace of one context (compaction)
struct Arena {
  void *base = nullptr;
  uint64_t cap = 0;
  uint64_t *host = nullptr;     // pinned host words: the job's few device -> host reads
  uint64_t *host_dev = nullptr; // the same words as mapped into the device
  uint64_t host_cap = 0;
  uint64_t seq = 0; // sequence word of the last host fetch (sstc_compact.hip fetch)
  // pinned, device-mapped bytes the host fills before a launch that copies
  // them to the device (the merge passes' group descriptors)
  uint8_t *up = nullptr;
  uint8_t *up_dev = nullptr;
  uint64_t up_cap = 0;
  // the first kernel's ticket + look-back status words (count_scan_kernel
  // <true>): zeroed when allocated, left zero by every launch
  uint64_t *lb = nullptr;
  uint64_t lb_cap = 0;
  // fault injection for tests (sstc__ctx_set_fault): corrupts the compaction
  // job's filter output on the device so its consistency guard can be tested
  // (1: survivor key offsets, 2: entry prefix sums); 0 in production
  uint32_t fault = 0;
  // the block split plan of this context's next compaction job: the chain
  // alone while the last job's chain held, the walk alone while it failed
  // (with a retry of both every kSegProbe jobs), both when unknown
  SegMode seg_mode = SegMode::kBoth;
  uint32_t seg_general_jobs = 0;
  uint64_t seg_redo_count = 0; // jobs whose tail ran twice (diagnostics / tests)
};
constexpr uint32_t kSegProbe = 8;

// sstc_merge_records: compact_impl stops after the merge and writes the merged
// order (out, up to cap records) instead of filtering and encoding
struct MergeOut {
  sstc_merged_record *out;
  uint64_t cap;
  uint64_t ties[2]; // result: cross-input (key, merge txn) ties, ties whose records differ
};

int compact_impl(Arena &arena, hipStream_t s, unsigned long long *err_count, const uint8_t *d_src,
                 const uint64_t *d_blk_off,
                 const uint64_t *d_blk_len, uint64_t nblocks, const uint64_t *h_tfb, uint32_t ntables,
                 uint64_t block_threshold, uint64_t table_limit, uint32_t base_level, uint32_t txn_mode,
                 uint8_t *d_dst, uint64_t dst_cap, uint64_t *d_table_off, uint64_t *d_table_len, uint64_t max_tables,
                 uint64_t *res, std::string &err, MergeOut *mo = nullptr);

// SST open on the device (sstc_open_tables): block index outputs
struct OpenOut {
  uint64_t *blk_off, *blk_len, *first_key_off, *last_key_off, *table_first_block;
  uint32_t *first_key_len, *last_key_len;
};

int open_tables_impl(Arena &arena, hipStream_t s, const uint8_t *d_src, uint64_t src_bytes, const uint64_t *h_off,
                     const uint64_t *h_bytes, uint32_t nt, uint64_t max_blocks, const OpenOut &out, uint64_t *h_tfb,
                     int32_t *h_status, uint64_t *h_footer, std::string &err);

} // namespace sstc
