// sstc_compact.hip — device-resident compaction job (reference db/compact.cc:
// 232-363 with MergeIterator, db/merge_iterator.{h,cc}).
//
//   decode every input block (sstc decode kernels, COMPAT txn = what the
//   reference iterator reads)
//   -> merge the per-table sorted runs: ceil(log8 k) k-way merge passes on a
//      16 B big-endian key prefix + length + txn (full key bytes compared only
//      when two prefixes tie and both keys are longer than 16 B); order = key
//      ascending, txn descending, then input table order
//   -> ShouldKeepEntry as flags (group head = key differs from the previous
//      merged record, group head txn by a scatter of group heads)
//   -> stream compaction of the survivors
//   -> output-table split (key+value bytes >= table_limit, compact.cc:290) and
//      block split (entry_size+16 >= block_threshold, table_builder.cc:57),
//      both greedy, both by the pointer-doubling segmentation, blocks clamped
//      at their table's end
//   -> layout scans, block encode (enc_emit_kernel), meta entries and footers
//      (table_builder.cc:101-211) written on the device.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <initializer_list>
#include <stdexcept>
#include <string>
#include <vector>

#include "sstc_device.h"
#include "sstc_launch.h"

namespace sstc {

namespace {

// ------------------------------------------------------------------ kernels
struct KeyView {
  const uint8_t *src;
  const RecX *rx; // by record id
};

using SK = SortKey;

// Device-side abort of the merge / filter kernels that run before the host
// sees the decode and sortedness verdicts: a failed block leaves its records
// (and their ids) unwritten, an unsorted run breaks the co-rank invariants the
// merge windows rely on; either would send those kernels out of bounds.
struct Abort {
  const unsigned long long *err;  // context decode-error counter
  const uint64_t *err0;           // its value before this job's decode
  const unsigned long long *bad;  // unsorted records (null: not checked)
  __device__ __forceinline__ bool operator()() const { return *err != *err0 || (bad && *bad); }
};

// three-way key compare: prefix, then (only when both are longer than 16 B and
// the prefixes tie) the remaining bytes, then the length (std::string_view <)
__device__ __forceinline__ int key_cmp(uint64_t a0, uint64_t a1, uint32_t al, uint32_t aid, uint64_t b0,
                                       uint64_t b1, uint32_t bl, uint32_t bid, const KeyView &kv) {
  al &= ~kSkRead; // SortKey::kl carries the read flag
  bl &= ~kSkRead;
  if (a0 != b0) return a0 < b0 ? -1 : 1;
  if (a1 != b1) return a1 < b1 ? -1 : 1;
  if (al > 16 && bl > 16) {
    const uint8_t *pa = kv.src + kv.rx[aid].ko;
    const uint8_t *pb = kv.src + kv.rx[bid].ko;
    const uint32_t m = al < bl ? al : bl;
    for (uint32_t j = 16; j < m; j++) {
      const uint32_t x = pa[j], y = pb[j];
      if (x != y) return x < y ? -1 : 1;
    }
  }
  return al < bl ? -1 : (al > bl ? 1 : 0);
}

// merge order: key asc, then txn desc (db/merge_iterator.h:91-95)
__device__ __forceinline__ bool sk_less(const SK &a, const SK &b, const KeyView &kv) {
  const int c = key_cmp(a.p0, a.p1, a.kl, a.id, b.p0, b.p1, b.kl, b.id, kv);
  return c < 0 || (c == 0 && a.tx > b.tx);
}

// k-way merge pass: every group of up to kKWay consecutive sorted runs is
// merged in ONE pass (ceil(log8 k) passes instead of log2 k pairwise rounds).
//  1. splitters: every S-th record of every run (S = kKWin / runs).  A wave
//     lane per (splitter, run) binary-searches the splitter's co-rank in that
//     run (records of the run that precede it in merge order); 8 lanes reduce
//     them to the splitter's rank among splitters (sum of ceil(c / S)) and
//     among records (sum of c), and write the co-rank row in sorted order.
//     Between two consecutive splitter rows a run contributes <= S records.
//  2. windows: window w holds the records between the first splitter rows at
//     or after output ranks w * kKWin and (w + 1) * kKWin (< 2 kKWin records);
//     a thread per window resolves its output position and sub-runs.
//  3. merge: a workgroup per window stages the <= kKWay sub-runs in LDS and
//     merges them by a pairwise merge-path tree (ck_mg_merge_kernel).  Order =
//     key asc, txn desc, then lower run first, i.e. the stable pairwise merge
//     of MergeIterator (merge_iterator.cc:34-46).
constexpr uint32_t kKWay = 8;
constexpr uint32_t kKWin = 512;
constexpr uint32_t kKRegion = 2 * kKWin;

struct KGroup {
  uint64_t start[kKWay + 1]; // absolute run starts; start[nruns] = group end
  uint32_t sbase[kKWay + 1]; // prefix of the runs' splitter counts
  uint32_t nruns, stride;    // runs, splitter stride S
  uint32_t base;             // first splitter id == first row (nsamp + 1 of each, the last a sentinel)
  uint32_t wg0;              // first merge workgroup
};


// Sortedness of every input run (TableBuilder requires sorted input,
// table_builder.h:77): decode_kernel checks each record against its
// predecessor in the same block; this kernel checks the first record of every
// non-empty block against the last record before it, unless it starts a run.
// (Until round 4 it also reduced the source-end bound with one same-address
// atomic per workgroup, which capped its grid; the count kernel reduces it now.)
constexpr uint32_t kRsLds = 1024; // run starts / table starts searched in LDS up to this many

// A key group continuing from block b - 1 into block b (r = its first record
// in b): the merge txns of block b's leading part take the running minimum of
// the group's part before it (the decode computed it per block).  That
// minimum is the smallest merge txn at the ends of the group's parts in the
// earlier blocks (each part's last merge txn is its own running minimum), so
// the walk goes back block end by block end, up to kGroupCarryBlocks blocks;
// a group reaching further back is left to long_carry_repair (kGuardLongGroup).
// Other threads may lower those ends meanwhile; the minimum is the same.
// Returns true when it lowered a merge txn.
__device__ bool carry_group(SK *s, const uint64_t *rec_base, uint64_t b, uint64_t r, uint64_t run0, const KeyView &kv,
                            unsigned long long *guard) {
  const SK k = s[r];
  uint64_t carry = s[r - 1].tx, end = r - 1, bb = b;
  for (uint32_t hop = 0;; hop++) {
    // the block holding `end`, then the first record of the group's part in it
    uint64_t q = bb - 1;
    while (rec_base[q] > end) q--;
    const uint64_t f = rec_base[q];
    const SK y = s[f];
    if (f == run0 || key_cmp(y.p0, y.p1, y.kl, y.id, k.p0, k.p1, k.kl, k.id, kv) != 0) break; // starts in q
    const SK z = s[f - 1];
    if (key_cmp(z.p0, z.p1, z.kl, z.id, k.p0, k.p1, k.kl, k.id, kv) != 0) break;
    if (hop + 1 >= kGroupCarryBlocks) { // a key's versions over many blocks: the repair pass carries it
      atomicOr(guard, kGuardLongGroup);
      return false;
    }
    end = f - 1;
    bb = q;
    carry = s[end].tx < carry ? s[end].tx : carry;
  }
  bool wrote = false;
  const uint64_t e = rec_base[b + 1];
  for (uint64_t i = r; i < e; i++) {
    SK x = s[i];
    if (key_cmp(x.p0, x.p1, x.kl, x.id, k.p0, k.p1, k.kl, k.id, kv) != 0) break;
    if (carry < x.tx) {
      x.tx = carry;
      x.kl |= kSkRead;
      s[i] = x;
      wrote = true;
    }
  }
  return wrote;
}

__device__ __forceinline__ bool is_run_start(const uint64_t *rs, uint64_t nruns, uint64_t r) {
  uint64_t lo = 0, hi = nruns; // last run_start <= r
  while (lo + 1 < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (rs[mid] <= r) lo = mid;
    else hi = mid;
  }
  return rs[lo] == r;
}

// The carries of EVERY block boundary as one segmented min-scan over the
// blocks, by one workgroup (the last of ck_check_blocks_kernel to finish, and
// only when some walk gave up at kGroupCarryBlocks AND some group is out of
// txn order, kGuardInv): block b contributes the merge txn at its end
// (its trailing group's running minimum) and starts a new segment unless the
// whole block continues the group of the block before it; the carry into a
// block whose first record continues that group is the scan up to the block
// before.  Values already lowered by carry_group are at least as low as the
// decode's and never below the group's true minimum, so the scan over them is
// the true one.  O(blocks), whatever a group's length: what MergeIterator's
// heap does for any number of versions (merge_iterator.cc:34-46 with the
// compat txn of block_reader.cc:109-111).
__device__ void long_carry_repair(SK *s, const uint64_t *rec_base, uint64_t nblocks, const uint64_t *rs,
                                  uint64_t nruns, const KeyView &kv) {
  __shared__ uint64_t s_v[256];
  __shared__ uint32_t s_r[256];
  __shared__ uint64_t s_carry; // scan value at the end of the previous chunk
  const uint32_t tid = threadIdx.x;
  if (tid == 0) s_carry = UINT64_MAX;
  __syncthreads();
  for (uint64_t c0 = 0; c0 < nblocks; c0 += 256) {
    const uint64_t b = c0 + tid;
    uint64_t v = UINT64_MAX, r0 = 0, r1 = 0;
    uint32_t rst = 0;
    bool cont = false;
    if (b < nblocks) {
      r0 = rec_base[b];
      r1 = rec_base[b + 1];
      if (r1 > r0) { // an empty block is transparent (identity element)
        const SK f = s[r0], l = s[r1 - 1];
        if (r0 > 0 && !is_run_start(rs, nruns, r0)) {
          const SK p = s[r0 - 1];
          cont = key_cmp(f.p0, f.p1, f.kl, f.id, p.p0, p.p1, p.kl, p.id, kv) == 0;
        }
        const bool full = cont && key_cmp(l.p0, l.p1, l.kl, l.id, f.p0, f.p1, f.kl, f.id, kv) == 0;
        v = l.tx;
        rst = !full;
      }
    }
    s_v[tid] = v;
    s_r[tid] = rst;
    __syncthreads();
    // inclusive segmented min-scan (Hillis-Steele): (a, b) -> b.reset ? b : (a.reset, min)
    for (uint32_t d = 1; d < 256; d <<= 1) {
      uint64_t nv = s_v[tid];
      uint32_t nr = s_r[tid];
      if (tid >= d && !nr) {
        nv = s_v[tid - d] < nv ? s_v[tid - d] : nv;
        nr = s_r[tid - d];
      }
      __syncthreads();
      s_v[tid] = nv;
      s_r[tid] = nr;
      __syncthreads();
    }
    const uint64_t cin = s_carry;
    // the scan value before block b (exclusive), the chunk's carry folded in
    uint64_t before = cin;
    if (tid > 0) before = s_r[tid - 1] ? s_v[tid - 1] : (s_v[tid - 1] < cin ? s_v[tid - 1] : cin);
    const uint64_t last = s_r[255] ? s_v[255] : (s_v[255] < cin ? s_v[255] : cin);
    __syncthreads();
    if (tid == 0) s_carry = last;
    if (cont) {
      const SK k = s[r0];
      for (uint64_t i = r0; i < r1; i++) {
        SK x = s[i];
        if (key_cmp(x.p0, x.p1, x.kl, x.id, k.p0, k.p1, k.kl, k.id, kv) != 0) break;
        if (before < x.tx) {
          x.tx = before;
          x.kl |= kSkRead;
          s[i] = x;
        }
      }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void ck_check_blocks_kernel(SK *s, const uint64_t *rec_base, uint64_t nblocks,
                                       const uint64_t *run_start, uint64_t nruns, KeyView kv,
                                       unsigned long long *bad, Abort stop, uint64_t *zws, uint64_t nz,
                                       unsigned long long *guard, const uint64_t *kg_host, uint64_t *kg,
                                       uint64_t kg_words, unsigned int *ticket) {
  // the merge passes' group descriptors, written by the host into pinned
  // mapped memory before the launch: copied here by workgroup 0 (a copy
  // command between the decode and the merge cost ~5 us)
  if (blockIdx.x == 0)
    for (uint64_t i = threadIdx.x; i < kg_words; i += blockDim.x) kg[i] = kg_host[i];
  // the run starts in LDS for the per-block binary search (log2 runs dependent
  // L2 round trips per block otherwise: config 4's 128 runs, 7 of them)
  __shared__ uint64_t s_rs[kRsLds];
  const bool rs_lds = nruns + 1 <= kRsLds;
  if (rs_lds)
    for (uint64_t i = threadIdx.x; i <= nruns; i += blockDim.x) s_rs[i] = run_start[i];
  __syncthreads();
  const uint64_t *rs = rs_lds ? s_rs : run_start;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (uint64_t z = t0; z < nz; z += stride) zws[z] = 0; // filter look-back
  const bool stopped = stop(); // uniform
  bool wrote = false;
  if (!stopped) {
    for (uint64_t b = t0; b < nblocks; b += stride) {
      const uint64_t r = rec_base[b];
      if (r == 0 || rec_base[b + 1] == r) continue;
      uint64_t lo = 0, hi = nruns; // run containing r: last run_start <= r
      while (lo + 1 < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (rs[mid] <= r) lo = mid;
        else hi = mid;
      }
      if (rs[lo] == r) continue; // first record of its run
      const SK cur = s[r], pv = s[r - 1];
      const int c = key_cmp(cur.p0, cur.p1, cur.kl, cur.id, pv.p0, pv.p1, pv.kl, pv.id, kv);
      if (c < 0) atomicAdd(bad, 1ull);
      // a key group continuing across the boundary takes its running minimum
      // from the blocks before it (a no-op unless some version of it is out of
      // txn order: the minimum of older versions is then >= every txn here)
      if (c == 0) {
        if (cur.tx > pv.tx) atomicOr(guard, kGuardInv); // a group out of txn order across the boundary
        wrote |= carry_group(s, rec_base, b, r, rs[lo], kv, guard);
      }
    }
  }
  // Long groups: the last workgroup to finish repairs them (an in-launch
  // hand-off: every workgroup that lowered a merge txn drains its stores and
  // releases them at agent scope before its ticket; the last arriver acquires
  // before it reads them).  No workgroup waits on another.  Two-level tickets:
  // a counter per dispatch group (workgroup i % 8, i.e. per XCD) and one over
  // the groups, so no address takes more than ~1/8 of the workgroups' atomics
  // (one same-address atomic per workgroup cost this kernel ~7 us at config 3)
  __shared__ uint32_t s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const bool any = __syncthreads_or(wrote);
  if (threadIdx.x == 0) {
    if (any) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    constexpr uint32_t kG = 8;
    const uint32_t g = blockIdx.x % kG, groups = gridDim.x < kG ? gridDim.x : kG;
    const uint32_t in_g = gridDim.x / kG + (g < gridDim.x % kG ? 1u : 0u);
    uint32_t last = 0;
    // counters 256 B apart: separate lines / channels
    if (__hip_atomic_fetch_add(ticket + 64 * g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_g - 1) {
      // the group's last: pass its group's writes on to the last group
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(ticket + 64 * g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(ticket + 64 * kG, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == groups - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned long long gw = __hip_atomic_load(guard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        constexpr unsigned long long kLongInv = kGuardLongGroup | kGuardInv;
        last = (gw & kLongInv) == kLongInv && !stop(); // the job's verdicts are final here
        __hip_atomic_store(ticket + 64 * kG, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    s_last = last;
  }
  __syncthreads();
  if (s_last) long_carry_repair(s, rec_base, nblocks, rs, nruns, kv);
}


// y precedes x in merge order, y from run ry, x from run rx != ry
__device__ __forceinline__ bool kw_before(const SK &y, uint32_t ry, const SK &x, uint32_t rx, const KeyView &kv) {
  return ry < rx ? !sk_less(x, y, kv) : sk_less(y, x, kv);
}

template <class T>
__device__ __forceinline__ uint32_t find_group(const KGroup *g, uint32_t ng, uint32_t v, T field) {
  uint32_t lo = 0, hi = ng; // last group with field <= v
  while (lo + 1 < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (field(g[mid]) <= v) lo = mid;
    else hi = mid;
  }
  return lo;
}

// kw_before(*yp, ry, x, rx) reading only y's 16 B key prefix unless it equals
// x's: a prefix that differs decides the order whatever the runs.  The
// splitter search is bound by its probe bytes, not by the probe chain (an
// 8-ary search was 2x slower): config 3 splitters 92 -> 89 us, config 4
// 259 -> 241 us (profiles/r02_ab/merge_ab.md)
__device__ __forceinline__ bool kw_before_at(const SK *yp, uint32_t ry, const SK &x, uint32_t rx, const KeyView &kv) {
  const u32x4 h = *reinterpret_cast<const u32x4 *>(yp);
  const uint64_t p0 = static_cast<uint64_t>(h.x) | (static_cast<uint64_t>(h.y) << 32);
  const uint64_t p1 = static_cast<uint64_t>(h.z) | (static_cast<uint64_t>(h.w) << 32);
  if (p0 != x.p0) return p0 < x.p0;
  if (p1 != x.p1) return p1 < x.p1;
  return kw_before(*yp, ry, x, rx, kv);
}

// the splitter records of a pass gathered by splitter id (run-major, sorted
// within each run): the co-rank searches first run over this compact array
// (a few MiB, cache resident) and only the last log2(S) probes touch the runs
__global__ void ck_kw_sample_kernel(const SK *in, const KGroup *groups, uint32_t ngroups, uint32_t nids, SK *smp,
                                    Abort stop) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nids || stop()) return;
  const KGroup &gr = groups[find_group(groups, ngroups, u, [](const KGroup &x) { return x.base; })];
  const uint32_t local = u - gr.base, nsamp = gr.sbase[gr.nruns];
  if (local == nsamp) return; // sentinel row
  uint32_t q = 0;
  while (gr.sbase[q + 1] <= local) q++;
  smp[u] = in[gr.start[q] + static_cast<uint64_t>(local - gr.sbase[q]) * gr.stride];
}

// Splitter slot v of a group -> its splitter id (run-major): the j-th splitters
// of all runs take adjacent slots (j = 0 of runs 0..k-1, then j = 1, ...; the
// runs' splitters past the shortest run's count follow run-major).  Adjacent
// slots share a wave, and the j-th splitters of runs with similar key
// distributions search the same region of every other run: its records are
// read once per wave instead of once per probing run (config 3: the run-major
// order fetched 485 MB, 1.9x the merge keys, for these probes).
__device__ __forceinline__ uint32_t kw_interleave(const KGroup &gr, uint32_t v) {
  const uint32_t k = gr.nruns, nsamp = gr.sbase[k];
  if (v >= nsamp) return v; // the sentinel row
  uint32_t m = ~0u;
  for (uint32_t q = 0; q < k; q++) m = min(m, gr.sbase[q + 1] - gr.sbase[q]);
  if (v < k * m) return gr.sbase[v % k] + v / k;
  uint32_t r = v - k * m;
  for (uint32_t q = 0; q < k; q++) {
    const uint32_t left = gr.sbase[q + 1] - gr.sbase[q] - m;
    if (r < left) return gr.sbase[q] + m + r;
    r -= left;
  }
  return v;
}

// kL lanes per splitter (one per run of its group): 8, or 4 for passes whose
// groups merge <= 4 runs (config 4's first two passes: half the waves)
template <uint32_t kL>
__global__ __launch_bounds__(256) void ck_kw_split_kernel(const SK *in, const SK *smp, const KGroup *groups,
                                                          uint32_t ngroups, uint32_t nids, KeyView kv, uint32_t *C,
                                                          uint64_t *G, Abort stop) {
  static_assert(kL == 4 || kL == 8, "lanes per splitter");
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t uu = t / kL, r = t % kL;
  if (uu >= nids || stop()) return; // whole lane groups leave together
  const KGroup &gr = groups[find_group(groups, ngroups, uu, [](const KGroup &x) { return x.base; })];
  const uint32_t local = kw_interleave(gr, uu - gr.base), nsamp = gr.sbase[gr.nruns], S = gr.stride;
  const uint32_t u = gr.base + local;
  uint64_t c = 0;
  if (r < gr.nruns) {
    const uint64_t rs = gr.start[r], len = gr.start[r + 1] - rs;
    if (local == nsamp) {
      c = len; // sentinel row
    } else {
      uint32_t q = 0;
      while (gr.sbase[q + 1] <= local) q++;
      const uint64_t p = static_cast<uint64_t>(local - gr.sbase[q]) * S;
      if (r == q) {
        c = p;
      } else {
        const SK x = smp[u];
        // samples of run r (records j * S) that precede x: cs; then the
        // co-rank lies in ((cs - 1) S, cs S]
        const SK *rsmp = smp + gr.base + gr.sbase[r];
        uint32_t slo = 0, shi = gr.sbase[r + 1] - gr.sbase[r];
        while (slo < shi) {
          const uint32_t mid = (slo + shi) >> 1;
          if (kw_before_at(rsmp + mid, r, x, q, kv)) slo = mid + 1;
          else shi = mid;
        }
        uint64_t lo = slo ? static_cast<uint64_t>(slo - 1) * S + 1 : 0;
        uint64_t hi = static_cast<uint64_t>(slo) * S < len ? static_cast<uint64_t>(slo) * S : len;
        while (lo < hi) {
          const uint64_t mid = (lo + hi) >> 1;
          if (kw_before_at(in + rs + mid, r, x, q, kv)) lo = mid + 1;
          else hi = mid;
        }
        c = lo;
      }
    }
  }
  uint64_t sr = (c + S - 1) / S, sc = c;
#pragma unroll
  for (uint32_t d = 1; d < kL; d <<= 1) {
    sr += __shfl_xor(sr, d, kL);
    sc += __shfl_xor(sc, d, kL);
  }
  const uint64_t row = gr.base + sr;
  C[row * kKWay + r] = static_cast<uint32_t>(c);
  if (r == 0) G[row] = sc;
}

// first splitter row of every merge window: window w starts at the first row
// whose record rank G is >= w * kKWin (rows are sorted, G increasing)
__global__ void ck_kw_bounds_kernel(const KGroup *groups, uint32_t ngroups, uint32_t nids, const uint64_t *G,
                                    uint32_t *J, Abort stop) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nids || stop()) return;
  const KGroup &gr = groups[find_group(groups, ngroups, u, [](const KGroup &x) { return x.base; })];
  const uint32_t j = u - gr.base, nsamp = gr.sbase[gr.nruns];
  const uint64_t N = gr.start[gr.nruns] - gr.start[0];
  const uint32_t nw = static_cast<uint32_t>((N + kKWin - 1) / kKWin);
  const uint64_t g = G[u];
  const uint64_t gp = j ? G[u - 1] : 0;
  // windows w with gp < w*kKWin <= g start at row j (row 0 also takes w = 0);
  // the sentinel row (G = N) also takes every window past the last record
  uint64_t w0 = j ? gp / kKWin + 1 : 0;
  uint64_t w1 = j == nsamp ? nw : g / kKWin; // inclusive
  for (uint64_t w = w0; w <= w1 && w <= nw; w++) J[gr.wg0 + gr.base + w] = j;
}

// one merge window, resolved once per window by a thread (not by the merge
// workgroup, whose dependent group -> J -> C -> record loads would each stall
// a whole LDS-holding workgroup): output position, the absolute start of every
// sub-run and the sub-runs' offsets in the window (off[q] for q > k = n)
struct __attribute__((aligned(16))) KWin {
  uint32_t out, n, k, pad;
  uint32_t src[kKWay];
  uint32_t off[kKWay + 1];
  uint32_t pad2[3];
};

__global__ void ck_kw_win_kernel(const KGroup *groups, uint32_t ngroups, uint32_t nwin, const uint32_t *C,
                                 const uint64_t *G, const uint32_t *J, KWin *win, Abort stop) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nwin) return;
  KWin d{};
  if (!stop()) { // an aborted job merges nothing (n = 0 in every window)
    const KGroup &gr = groups[find_group(groups, ngroups, u, [](const KGroup &x) { return x.wg0; })];
    const uint32_t at = gr.wg0 + gr.base + (u - gr.wg0), k = gr.nruns;
    const uint32_t j0 = J[at], j1 = J[at + 1];
    d.k = k;
    if (j0 != j1) {
      d.out = static_cast<uint32_t>(gr.start[0] + G[gr.base + j0]);
      uint32_t acc = 0;
#pragma unroll
      for (uint32_t q = 0; q < kKWay; q++) { // static indices: d stays in registers
        if (q < k) {
          const uint32_t lo = C[static_cast<uint64_t>(gr.base + j0) * kKWay + q];
          const uint32_t hi = C[static_cast<uint64_t>(gr.base + j1) * kKWay + q];
          d.src[q] = static_cast<uint32_t>(gr.start[q] + lo);
          d.off[q] = acc;
          acc += hi - lo;
        }
      }
      d.n = acc;
    }
#pragma unroll
    for (uint32_t q = 0; q <= kKWay; q++)
      if (q >= k) d.off[q] = d.n;
  }
  win[u] = d;
}


// Merge of one window by a pairwise tree in LDS: the staged key prefixes stay
// put; log2(k) levels each merge neighbouring sub-run groups into a
// permutation of 16-bit slot indices (ping-pong), the first straight from the
// staged order; the last permutation drives a coalesced copy to the output.
// Every thread produces ceil(n / threads) consecutive outputs of a level (all
// threads busy whatever the window size): one merge-path search for its first
// output, then a sequential two-head merge with the heads' prefixes in
// registers.  The left group always holds the lower runs, so taking B only
// when B sorts strictly first gives key asc, txn desc, lower run first
// (merge_iterator.cc:34-46).
constexpr uint32_t kMgThreads = 256;

struct MgPf { // a record's 16 B big-endian key prefix
  uint64_t p0, p1;
};

// Only the 16 B key-prefix plane is in LDS (20 KiB per workgroup: 8
// workgroups per CU; the round-2 tile of whole 32 B records held 37 KB, 4 per
// CU, and merged config 3 in 206 us vs 167 us, config 4 797 vs 677 us -- the
// merge is bound by its dependent LDS / load chains, so resident workgroups
// are what hides them; profiles/r03_ab/merge_pf.md).  The rest of a record (txn, key length, id) is read
// from the input -- L2-hot, the window staged it moments before -- only on a
// prefix tie and for the output copy.  The descriptor stays in scalar
// registers (no LDS copy): sub-run of a slot and its source index by selects.
struct MgDesc {
  // sub-run starts in the window (o8 = n; o_q = n for q >= k) and the source
  // index offsets (slot x of sub-run q is record x + b_q).  Every field read
  // goes through u() (readfirstlane: a no-op on these uniform values) -- a
  // select chain over plain field loads is folded into one load at a selected
  // offset, which pins the descriptor in scratch memory
  uint32_t o0, o1, o2, o3, o4, o5, o6, o7, o8;
  uint32_t b0, b1, b2, b3, b4, b5, b6, b7;
  static __device__ __forceinline__ uint32_t u(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
  __device__ __forceinline__ uint32_t run_of(uint32_t x) const {
    return (x >= o1) + (x >= o2) + (x >= o3) + (x >= o4) + (x >= o5) + (x >= o6) + (x >= o7);
  }
  __device__ __forceinline__ uint32_t gidx(uint32_t x) const {
    uint32_t b = u(b0);
    b = x >= o1 ? u(b1) : b;
    b = x >= o2 ? u(b2) : b;
    b = x >= o3 ? u(b3) : b;
    b = x >= o4 ? u(b4) : b;
    b = x >= o5 ? u(b5) : b;
    b = x >= o6 ? u(b6) : b;
    b = x >= o7 ? u(b7) : b;
    return x + b;
  }
  __device__ __forceinline__ uint32_t bound(uint32_t q) const { // o_min(q, 8)
    uint32_t r = u(o8); // ordered compares: equality selects become a table lookup
    r = q <= 7 ? u(o7) : r;
    r = q <= 6 ? u(o6) : r;
    r = q <= 5 ? u(o5) : r;
    r = q <= 4 ? u(o4) : r;
    r = q <= 3 ? u(o3) : r;
    r = q <= 2 ? u(o2) : r;
    r = q <= 1 ? u(o1) : r;
    r = q == 0 ? u(o0) : r;
    return r;
  }
};
static_assert(kKWay == 8, "MgDesc holds 8 sub-runs");

// (waves_per_eu(8): the p1-only instantiation took 102 SGPRs, 7 waves per
// SIMD; 8 spills 25 SGPRs to VGPR lanes)
__global__ __launch_bounds__(kMgThreads) __attribute__((amdgpu_waves_per_eu(8))) void ck_mg_merge_kernel(const SK *__restrict__ in, SK *__restrict__ out,
                                                                   const KWin *__restrict__ win, KeyView kv) {
  __shared__ u32x4 pf[kKRegion];
  __shared__ uint16_t ix[2][kKRegion];
  const KWin *w = win + blockIdx.x;
  const uint32_t total = __builtin_amdgcn_readfirstlane(w->n), k = __builtin_amdgcn_readfirstlane(w->k);
  if (total == 0) return;
  SK *o = out + __builtin_amdgcn_readfirstlane(w->out);
  MgDesc d;
#define SSTC_MG_LD(q) \
  d.o##q = __builtin_amdgcn_readfirstlane(w->off[q]);
  SSTC_MG_LD(0) SSTC_MG_LD(1) SSTC_MG_LD(2) SSTC_MG_LD(3) SSTC_MG_LD(4) SSTC_MG_LD(5) SSTC_MG_LD(6) SSTC_MG_LD(7)
  SSTC_MG_LD(8)
#undef SSTC_MG_LD
#define SSTC_MG_LD(q) \
  d.b##q = __builtin_amdgcn_readfirstlane(w->src[q]) - d.o##q;
  SSTC_MG_LD(0) SSTC_MG_LD(1) SSTC_MG_LD(2) SSTC_MG_LD(3) SSTC_MG_LD(4) SSTC_MG_LD(5) SSTC_MG_LD(6) SSTC_MG_LD(7)
#undef SSTC_MG_LD
  if (k == 1) {
    for (uint32_t i = threadIdx.x; i < total; i += kMgThreads) o[i] = in[d.b0 + i];
    return;
  }
  // slot i = tid + 256 j is staged by this thread: its prefix into LDS, its
  // second half (txn, key length, id) kept in registers for the output
  constexpr uint32_t kPer = kKRegion / kMgThreads;
  u32x4 rest[kPer];
  // the window's first 8 key bytes, when every record shares them (a window
  // is a narrow key range: keys with a common prefix of 8+ bytes, e.g. every
  // config-3 / 4 key, "k0000000..."), let the merge read only the second 8
  // bytes of each prefix from LDS: half the LDS bytes per probe
  const uint64_t c0 = reinterpret_cast<const uint64_t *>(in + d.gidx(0))[0];
  bool same = true;
#pragma unroll
  for (uint32_t j = 0; j < kPer; j++) {
    const uint32_t i = threadIdx.x + j * kMgThreads;
    if (i < total) {
      const u32x4 *r = reinterpret_cast<const u32x4 *>(in + d.gidx(i));
      pf[i] = r[0];
      rest[j] = r[1];
      same &= (static_cast<uint64_t>(r[0].x) | (static_cast<uint64_t>(r[0].y) << 32)) == c0;
    }
  }
  // the verdict through ix[0] (free until the second level writes it): one
  // word per wave, no extra LDS (__syncthreads_and took 256 B: 8 -> 7
  // workgroups per CU)
  const bool wall = __all(same);
  if (lane_id() == 0) ix[0][threadIdx.x / kWave] = wall ? 1 : 0;
  __syncthreads();
  bool p1only = true;
#pragma unroll
  for (uint32_t w = 0; w < kMgThreads / kWave; w++) p1only &= ix[0][w] != 0;
  const uint64_t *pf64 = reinterpret_cast<const uint64_t *>(pf);
  // slot sa (prefix a) before slot sb (prefix b); the whole records on a tie
  auto less = [&](uint32_t sa, const MgPf &a, uint32_t sb, const MgPf &b) __attribute__((always_inline)) {
    if (a.p0 != b.p0) return a.p0 < b.p0;
    if (a.p1 != b.p1) return a.p1 < b.p1;
    // the records' second halves (txn, key length, id) from the input
    const u32x4 ra = reinterpret_cast<const u32x4 *>(in + d.gidx(sa))[1];
    const u32x4 rb = reinterpret_cast<const u32x4 *>(in + d.gidx(sb))[1];
    const int c = key_cmp(a.p0, a.p1, ra.z, ra.w, b.p0, b.p1, rb.z, rb.w, kv);
    return c < 0 || (c == 0 && (static_cast<uint64_t>(ra.x) | (static_cast<uint64_t>(ra.y) << 32)) >
                                   (static_cast<uint64_t>(rb.x) | (static_cast<uint64_t>(rb.y) << 32)));
  };
  const uint32_t per = (total + kMgThreads - 1) / kMgThreads; // outputs per thread
  const uint32_t p0 = threadIdx.x * per;
  auto levels = [&](auto p1tag) __attribute__((always_inline)) -> uint32_t {
  constexpr bool kP1 = decltype(p1tag)::value;
  auto pfx = [&](uint32_t sl) __attribute__((always_inline)) -> MgPf {
    if constexpr (kP1) return {c0, pf64[2 * sl + 1]};
    const u32x4 h = pf[sl];
    return {static_cast<uint64_t>(h.x) | (static_cast<uint64_t>(h.y) << 32),
            static_cast<uint64_t>(h.z) | (static_cast<uint64_t>(h.w) << 32)};
  };
  uint32_t src = 0;
  for (uint32_t wd = 1; wd < k; wd <<= 1) {
    const bool first = wd == 1;
    const uint16_t *a_ix = ix[src];
    uint16_t *o_ix = ix[src ^ 1];
    auto slot = [&](uint32_t x) __attribute__((always_inline)) -> uint32_t { return first ? x : a_ix[x]; };
    if (p0 < total) {
      uint32_t m = d.run_of(p0) & ~(2 * wd - 1);
      uint32_t lo = d.bound(m), mid = d.bound(m + wd), hi = d.bound(m + 2 * wd);
      const uint32_t diag = p0 - lo;
      uint32_t i = diag > hi - mid ? diag - (hi - mid) : 0, ihi = diag < mid - lo ? diag : mid - lo;
      while (i < ihi) {
        const uint32_t im = (i + ihi) >> 1;
        const uint32_t sb = slot(mid + diag - 1 - im), sa = slot(lo + im);
        if (!less(sb, pfx(sb), sa, pfx(sa))) i = im + 1;
        else ihi = im;
      }
      uint32_t j = diag - i, ai = 0, bi = 0;
      MgPf a{0, 0}, b{0, 0};
      if (lo + i < mid) a = pfx(ai = slot(lo + i));
      if (mid + j < hi) b = pfx(bi = slot(mid + j));
      for (uint32_t e = 0; e < per; e++) {
        const uint32_t p = p0 + e;
        if (p >= total) break;
        while (p == hi) { // the next pair starts inside this thread's outputs
          m += 2 * wd;
          lo = hi;
          mid = d.bound(m + wd);
          hi = d.bound(m + 2 * wd);
          i = j = 0;
          if (lo < mid) a = pfx(ai = slot(lo));
          if (mid < hi) b = pfx(bi = slot(mid));
        }
        const bool take_b = lo + i >= mid || (mid + j < hi && less(bi, b, ai, a));
        o_ix[p] = static_cast<uint16_t>(take_b ? bi : ai);
        if (take_b) {
          j++;
          if (mid + j < hi) b = pfx(bi = slot(mid + j));
        } else {
          i++;
          if (lo + i < mid) a = pfx(ai = slot(lo + i));
        }
      }
    }
    __syncthreads();
    src ^= 1;
  }
  return src;
  };
  const uint32_t src = p1only ? levels(std::true_type{}) : levels(std::false_type{});
  // output: the inverse permutation, then every thread writes its own staged
  // records at their merged positions (prefix from LDS, second half from its
  // registers) -- reading the records again from the input after the merge
  // doubled the kernel's fetch (the window's lines had left L2)
  for (uint32_t p = threadIdx.x; p < total; p += kMgThreads) ix[src ^ 1][ix[src][p]] = static_cast<uint16_t>(p);
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < kPer; j++) {
    const uint32_t i = threadIdx.x + j * kMgThreads;
    if (i < total) {
      u32x4 *q = reinterpret_cast<u32x4 *>(o + ix[src ^ 1][i]);
      q[0] = pf[i];
      q[1] = rest[j];
    }
  }
}

struct Rec { // survivor columns (vl / vo null in the compaction job: unused by its encode)
  uint8_t *type;
  uint32_t *kl, *vl;
  uint64_t *tx, *ko, *vo;
};

// Keep / drop (ShouldKeepEntry, compact.cc:324-363) over the merged records,
// then stream compaction of the survivors with the prefix sums the splits
// need (ck_filter_kernel).  A row = kFtThreads lane-consecutive records, so
// loads and stores coalesce.
constexpr uint32_t kFtThreads = 256;

// data_size increment (table_builder.cc:55)
__device__ __forceinline__ uint64_t data_bytes(uint32_t kl, uint32_t vl) {
  return static_cast<uint64_t>(kl) + (vl != kNoValue ? vl : 0u);
}

// Keep / drop and survivor compaction in one pass (round 1 used three kernels:
// flags + tile sums, a scan of the tile sums, compaction): a tile of kFfRows
// rows keeps its survivors' fields in registers, publishes its three totals
// (kept records, key+value bytes, entry bytes) through decoupled look-back
// (one wave per total; ws = [unused, status[3][tiles]], cleared before the
// launch), then writes the survivors row by row at their global positions.
// The merged keys and the side records are read once.
constexpr uint32_t kFfRows = 8, kFfTile = kFtThreads * kFfRows;

// keep record i: the first merged record always; a group head (key differs
// from the previous record, compact.cc:266-268) if PUT, or if DELETED and not
// the base level; any other record iff its txn equals its group head's (drop
// if last_txn > txn).  Txns descend within a group, so a non-head whose txn
// differs from its predecessor's is dropped; an equal one (records duplicated
// across inputs) finds its group head by galloping back over equal keys and
// compares txns: O(log distance) per record, so a long run of equal
// (key, txn) records costs n log n, not the n^2 of a walk back record by record.
__device__ __forceinline__ bool ff_same_key(const SK &a, const SK &b, const KeyView &kv) {
  return key_cmp(a.p0, a.p1, a.kl, a.id, b.p0, b.p1, b.kl, b.id, kv) == 0;
}
// a record read back by the gallop / binary search carries an unchecked
// merged id: one out of range (a broken merge, rejected by the guard) is
// taken as "not the same key", so no key compare indexes past the inputs
__device__ __forceinline__ bool ff_same_key_at(const SK &a, const SK &b, const KeyView &kv, uint64_t n) {
  return a.id < n && ff_same_key(a, b, kv);
}
// ShouldKeepEntry keeps a non-head record iff its txn (as read) is not below
// its group head's (compact.cc:357-362, `!(last_txn > txn)`).  The head of a
// merged group is an input's first version of the key, whose merge txn is its
// txn as read; a record whose merge txn is its txn as read sits at or below
// the head (merge txns descend through the group), so it needs an equal txn
// all the way back (quick reject on its predecessor's merge txn).  Only a
// lowered record (kSkRead; tread = its txn as read) can lie above the head.
__device__ __forceinline__ uint32_t ff_keep(const SK *s, uint64_t i, const SK &x, const SK &pv, uint32_t ty,
                                            uint32_t base_level, const KeyView &kv, uint64_t n, uint64_t tread) {
  if (i == 0) return 1;
  if (!ff_same_key(pv, x, kv)) return ty == kTypePut ? 1u : (base_level ? 0u : 1u);
  const bool lowered = (x.kl & kSkRead) != 0;
  if (!lowered && x.tx != pv.tx) return 0;
  // group head = first record of x's key group: s[hi] has x's key, s[lo] not
  // (or lo = -1 past the start)
  uint64_t hi = i - 1;
  int64_t lo = -1;
  for (uint64_t step = 1;; step <<= 1) {
    if (hi == 0) break;
    const uint64_t p = hi > step ? hi - step : 0;
    if (ff_same_key_at(s[p], x, kv, n)) {
      hi = p;
    } else {
      lo = static_cast<int64_t>(p);
      break;
    }
  }
  while (lo + 1 < static_cast<int64_t>(hi)) {
    const uint64_t mid = static_cast<uint64_t>((lo + static_cast<int64_t>(hi)) >> 1);
    if (ff_same_key_at(s[mid], x, kv, n)) hi = mid;
    else lo = static_cast<int64_t>(mid);
  }
  return lowered ? (tread >= s[hi].tx ? 1u : 0u) : (s[hi].tx == x.tx ? 1u : 0u);
}

// the txn of record x as the reference's iterator reads it (parse_entry,
// block_reader.cc:109-111): for a record whose merge txn was lowered
// (kSkRead), re-read from its entry in the source
__device__ __forceinline__ uint64_t read_txn(const KeyView &kv, const RecX &rx, uint32_t kl, uint32_t txn_mode) {
  const bool after_value = rx.type != kTypeDeleted && !(txn_mode == 0u && rx.vl == 0u);
  return g_u64u(kv.src + rx.ko + kl + (after_value ? 4ull + rx.vl : 0ull));
}

__device__ __forceinline__ uint32_t run_of_record(const uint64_t *rs, uint32_t nruns, uint64_t id) {
  uint32_t lo = 0, hi = nruns; // last run start <= id
  while (lo + 1 < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (rs[mid] <= id) lo = mid;
    else hi = mid;
  }
  return lo;
}

// A run of merged records with equal key and merge txn: where the reference's
// heap decides the order by its history (merge_iterator.h:91-95 compares key
// and txn only).  Every order of the run gives the same records in the same
// order unless the run holds records of two or more inputs AND not all of
// them are alike (type, txn as read, value).  Called for merged neighbours
// i - 1, i with equal key and merge txn (rare: txns are unique per write); the
// run's first pair walks the run once.
//   ties != null (sstc_merge_records, the iterator's whole order is
//   observable): ties[0] counts runs spanning inputs, ties[1] those of them
//   whose records differ.
//   guard != null (the compaction filter): only the order of what
//   ShouldKeepEntry keeps can reach an output (compact.cc:324-363): the
//   run's records whose txn as read is not below the key group's first
//   record's (the group head: the run's own merge txn when the run starts
//   the group -- every input's first version in it has that txn -- else the
//   group's first record's, galloped to as ff_keep does).  A run whose kept
//   records span inputs and are not alike sets kGuardTieBoth: the job is
//   refused (SSTC_E_TIE_ORDER).
__device__ __forceinline__ uint64_t txn_as_read(const SK &x, const RecX &r, const KeyView &kv, uint32_t txn_mode) {
  return x.kl & kSkRead ? read_txn(kv, r, x.kl & ~kSkRead, txn_mode) : x.tx;
}

__device__ __forceinline__ void note_tie(const SK *s, uint64_t n, uint64_t i, const KeyView &kv, const uint64_t *rs,
                                         uint32_t nruns, uint32_t txn_mode, unsigned long long *ties,
                                         unsigned long long *guard) {
  const SK h = s[i - 1];
  if (h.id >= n) return;
  bool group_head = true; // the run starts its key group
  if (i >= 2) {
    const SK q = s[i - 2];
    if (q.id < n && ff_same_key(q, h, kv)) {
      if (q.tx == h.tx) return; // not the run's first pair: the pair that is walks it
      group_head = false;
    }
  }
  uint64_t head_txn = h.tx;
  if (guard && !group_head) { // the group's first record (s[hi] has the key, s[lo] not)
    uint64_t hi = i - 2;
    int64_t lo = -1;
    for (uint64_t step = 1;; step <<= 1) {
      if (hi == 0) break;
      const uint64_t p = hi > step ? hi - step : 0;
      if (ff_same_key_at(s[p], h, kv, n)) {
        hi = p;
      } else {
        lo = static_cast<int64_t>(p);
        break;
      }
    }
    while (lo + 1 < static_cast<int64_t>(hi)) {
      const uint64_t mid = static_cast<uint64_t>((lo + static_cast<int64_t>(hi)) >> 1);
      if (ff_same_key_at(s[mid], h, kv, n)) hi = mid;
      else lo = static_cast<int64_t>(mid);
    }
    head_txn = s[hi].tx;
  }
  const uint32_t kl = h.kl & ~kSkRead;
  bool have = false, cross = false, diff = false;
  uint32_t fin = 0;
  RecX fr{};
  uint64_t ftx = 0;
  for (uint64_t j = i - 1; j < n; j++) {
    const SK x = s[j];
    if (x.id >= n || x.tx != h.tx || !ff_same_key(h, x, kv)) break;
    const RecX r = kv.rx[x.id];
    const uint64_t tx = txn_as_read(x, r, kv, txn_mode);
    if (guard && tx < head_txn) continue; // dropped whatever the order (!(last_txn > txn), compact.cc:357-362)
    const uint32_t in = run_of_record(rs, nruns, x.id);
    if (!have) {
      have = true;
      fin = in;
      fr = r;
      ftx = tx;
      continue;
    }
    cross |= in != fin;
    if (diff) continue;
    diff = r.type != fr.type || r.vl != fr.vl || tx != ftx;
    if (!diff && r.vl != kNoValue) {
      const uint8_t *a = kv.src + r.ko + kl + 4, *b = kv.src + fr.ko + kl + 4;
      for (uint32_t k = 0; k < r.vl && !diff; k++) diff = a[k] != b[k];
    }
  }
  if (!cross) return;
  if (ties) atomicAdd(&ties[0], 1ull);
  if (!diff) return;
  if (ties) atomicAdd(&ties[1], 1ull);
  if (guard) atomicOr(guard, kGuardTieBoth);
}

__global__ __launch_bounds__(kFtThreads) void ck_filter_kernel(const SK *s, uint64_t n, KeyView kv,
                                                               uint32_t base_level, Rec out, uint64_t *Pd,
                                                               uint64_t *Pe, uint64_t *ws, uint64_t *totals,
                                                               Abort stop, unsigned long long *guard,
                                                               uint32_t txn_mode, const uint64_t *rs,
                                                               uint32_t nruns) {
  __shared__ uint64_t s_pre[3];
  if (stop()) { // uniform over the grid: no status published, the host rejects the job
    if (blockIdx.x == 0 && threadIdx.x == 0) { // no survivor: the layout below splits nothing, writes nothing
      totals[0] = totals[1] = totals[2] = 0;
      Pd[0] = Pe[0] = 0;
    }
    return;
  }
  const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid / kWave;
  // tile = workgroup id: workgroups are dispatched in id order (per XCD, in
  // order), so the lowest unfinished tile is always resident and its
  // look-back only waits on finished tiles; a drawn ticket cost 6-20 us
  // (one device-scope atomic per tile, profiles/r05/filter_ab.md)
  const uint64_t tile = blockIdx.x, t0 = tile * kFfTile;
  uint32_t km = 0, kl[kFfRows], vl[kFfRows], ty[kFfRows];
  uint64_t tx[kFfRows], ko[kFfRows];
  // every row's merged keys and side records in flight together; a record's
  // predecessor is the lane before it (shuffled), a wave's first lane takes
  // the last lane of the wave before it in merge order through LDS
  // (s_edge[4 j + w]; [0] = the record before the tile).  Round 4 loaded
  // every predecessor again and issued the rows in two dependent groups.
  __shared__ SK s_edge[kFfRows * (kFtThreads / kWave) + 1];
  {
    SK x[kFfRows];
    RecX rr[kFfRows];
#pragma unroll
    for (uint32_t j = 0; j < kFfRows; j++) {
      const uint64_t i = t0 + static_cast<uint64_t>(j) * kFtThreads + tid;
      x[j] = s[i < n ? i : n - 1]; // clamped, unconditional: the loads stay in flight together
    }
    if (tid == 0) s_edge[0] = s[t0 ? t0 - 1 : 0]; // (t0 < n: a tile starts below n)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (uint32_t j = 0; j < kFfRows; j++) {
      rr[j] = kv.rx[x[j].id < n ? x[j].id : 0u]; // unconditional (past n: the first record's)
      if (lane == kWave - 1) s_edge[1 + j * (kFtThreads / kWave) + w] = x[j];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kFfRows; j++) {
      const uint64_t i = t0 + static_cast<uint64_t>(j) * kFtThreads + tid;
      SK pv;
      pv.p0 = __shfl_up(x[j].p0, 1u, kWave);
      pv.p1 = __shfl_up(x[j].p1, 1u, kWave);
      pv.tx = __shfl_up(x[j].tx, 1u, kWave);
      pv.kl = __shfl_up(x[j].kl, 1u, kWave);
      pv.id = __shfl_up(x[j].id, 1u, kWave);
      if (lane == 0) pv = s_edge[j * (kFtThreads / kWave) + w];
      if (__any(x[j].id >= n || pv.id >= n)) { // no key compare may follow such an id: the job is rejected
        if (lane == 0) atomicOr(guard, kGuardMergeId);
        x[j].id = pv.id = 0;
        x[j].kl &= ~kSkRead; // and no source read for it
      }
      // the txn as read (a merge txn lowered by its group: re-read, rare)
      const uint64_t tread = x[j].kl & kSkRead ? read_txn(kv, rr[j], x[j].kl & ~kSkRead, txn_mode) : x[j].tx;
      const uint32_t k = i < n ? ff_keep(s, i, x[j], pv, rr[j].type, base_level, kv, n, tread) : 0u;
      if (i < n && i > 0 && pv.tx == x[j].tx && ff_same_key(pv, x[j], kv)) // (rare: txns are unique per write)
        note_tie(s, n, i, kv, rs, nruns, txn_mode, nullptr, guard);
      km |= k << j;
      kl[j] = x[j].kl & ~kSkRead;
      tx[j] = tread;
      vl[j] = rr[j].vl;
      ty[j] = rr[j].type;
      ko[j] = rr[j].ko;
    }
  }
  // per row and wave: kept count and the two byte sums, exchanged once
  // through LDS for the whole tile (one barrier instead of two per row of a
  // workgroup scan); the sums are the last lanes of the rows' inclusive DPP
  // scans, which the survivor writes below reuse (no separate LDS-swizzle
  // reductions)
  __shared__ uint64_t s_row[kFfRows][kFtThreads / kWave][3];
  uint64_t dinc[kFfRows], einc[kFfRows];
#pragma unroll
  for (uint32_t j = 0; j < kFfRows; j++) {
    const bool k = (km >> j) & 1u;
    const uint64_t c = static_cast<uint64_t>(__popcll(__ballot(k)));
    dinc[j] = wave_incl_scan_u64(k ? data_bytes(kl[j], vl[j]) : 0ull);
    einc[j] = wave_incl_scan_u64(k ? entry_size(kl[j], vl[j]) : 0ull);
    const uint64_t d = readlane_u64(dinc[j], kWave - 1), e = readlane_u64(einc[j], kWave - 1);
    if (lane == 0) {
      s_row[j][w][0] = c;
      s_row[j][w][1] = d;
      s_row[j][w][2] = e;
    }
  }
  __syncthreads();
  if (w < 3) { // wave c: decoupled look-back of total c
    uint64_t *status = ws + 1 + static_cast<uint64_t>(w) * gridDim.x;
    constexpr uint32_t kRW = kFfRows * (kFtThreads / kWave);
    const uint64_t total =
        wave_sum_u64(lane < kRW ? s_row[lane / (kFtThreads / kWave)][lane % (kFtThreads / kWave)][w] : 0ull);
    uint64_t prefix = 0;
    if (tile == 0) {
      if (lane == 0) __hip_atomic_store(&status[0], kLbInc | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(&status[tile], kLbAgg | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int64_t p = static_cast<int64_t>(tile) - 1; // window [p - 63, p]
      uint64_t spins = 0;
      for (;;) {
        const int64_t q = p - static_cast<int64_t>(lane);
        const uint64_t st = q >= 0 ? __hip_atomic_load(&status[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : kLbInc;
        const uint64_t inc = __ballot((st >> 62) == 2);
        const uint32_t need = inc ? static_cast<uint32_t>(__ffsll(static_cast<long long>(inc))) : kWave;
        const uint64_t zero = __ballot((st >> 62) == 0 && lane < need);
        if (zero) {
          if (++spins > kLbSpinLimit) { // a predecessor never published: give up (no hang), the job rejected
            if (lane == 0) atomicOr(guard, kGuardLookback);
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
        __hip_atomic_store(&status[tile], kLbInc | (prefix + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) s_pre[w] = prefix;
  }
  __syncthreads();
  uint64_t base[3] = {s_pre[0], s_pre[1], s_pre[2]};
#pragma unroll
  for (uint32_t j = 0; j < kFfRows; j++) { // row by row: survivors of a row are lane-consecutive
    const bool k = (km >> j) & 1u;
    uint64_t off[3] = {base[0], base[1], base[2]}, rt[3] = {0, 0, 0};
#pragma unroll
    for (uint32_t x = 0; x < kFtThreads / kWave; x++) { // waves before this one in the row
#pragma unroll
      for (int c = 0; c < 3; c++) {
        const uint64_t y = s_row[j][x][c];
        off[c] += x < w ? y : 0ull;
        rt[c] += y;
      }
    }
    const uint64_t bal = __ballot(k);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(bal >> 32),
                                                    __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(bal), 0u));
    const uint64_t dv = k ? data_bytes(kl[j], vl[j]) : 0ull, ev = k ? entry_size(kl[j], vl[j]) : 0ull;
    const uint64_t dincl = dinc[j], eincl = einc[j];
    const uint64_t q = off[0] + rank;
    if (k && q < n) { // (q < n holds by construction; the bound guards the stores)
      out.type[q] = static_cast<uint8_t>(ty[j]);
      out.kl[q] = kl[j];
      out.tx[q] = tx[j];
      out.ko[q] = ko[j];
      // no value length / offset columns: the entry is copied whole from its
      // input block (enc_lds_kernel<1>), which only reads type, key length,
      // txn and key offset (12 B per survivor fewer written)
      Pd[q] = off[1] + dincl - dv;
      Pe[q] = off[2] + eincl - ev;
    }
#pragma unroll
    for (int c = 0; c < 3; c++) base[c] += rt[c];
  }
  if (tid == 0 && t0 + kFfTile >= n) { // the last tile: grand totals and the closing prefix sums
    if (base[0] <= n) {
      Pd[base[0]] = base[1];
      Pe[base[0]] = base[2];
    }
    totals[0] = base[0];
    totals[1] = base[1];
    totals[2] = base[2];
  }
}

// The merged order itself (sstc_merge_records: MergeIterator's SeekToFirst +
// Next sequence, merge_iterator.cc:34-46,79-92, without the compaction's
// filter): a thread per merged position writes the record's key offset and
// its txn as the reference's iterator reads it (the merge txn unless the
// decode lowered it, kSkRead).  Equal (key, merge txn) neighbours are where
// the reference's std::priority_queue decides the order by heap history
// (merge_iterator.h:91-95 compares only key and txn), so their runs are
// counted (note_tie): ties[0] = runs spanning inputs, ties[1] = those of them
// whose records differ -- where the heap's order may give other bytes.
__global__ __launch_bounds__(256) void ck_merged_kernel(const SK *s, uint64_t n, KeyView kv, const uint64_t *rs,
                                                        uint32_t nruns, sstc_merged_record *out,
                                                        unsigned long long *ties, Abort stop,
                                                        unsigned long long *guard, uint32_t txn_mode) {
  if (stop()) return; // a rejected job: the host reads the verdicts, nothing here is used
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const SK x = s[i];
  if (x.id >= n) { // a broken merge: rejected by the guard, no source read
    atomicOr(guard, kGuardMergeId);
    return;
  }
  const RecX rr = kv.rx[x.id];
  const uint32_t kl = x.kl & ~kSkRead;
  const uint64_t tread = x.kl & kSkRead ? read_txn(kv, rr, kl, txn_mode) : x.tx;
  sstc_merged_record m;
  m.key_off = rr.ko;
  m.txn = tread;
  out[i] = m;
  if (i == 0) return;
  const SK pv = s[i - 1];
  if (pv.id >= n || pv.tx != x.tx || !ff_same_key(pv, x, kv)) return;
  note_tie(s, n, i, kv, rs, nruns, txn_mode, ties, nullptr); // equal (key, merge txn): the rare path
}

// The output table and block counts stay on the device (dn[0], dn[1]): the
// layout kernels run on host-side upper bounds (nt_max, nb_max: every table
// but the last holds >= table_limit key+value bytes, every block but a
// table's last >= block_threshold entry + offset bytes), so the job needs no
// host fetch between the split and the encode (it cost 12-36 us of idle GPU).
// Array slots past the real counts are zero (the scans over the bounds then
// end at the real totals); counts past the bounds (a corrupt split, or more
// tables than max_tables) make every layout / encode kernel stand down.
struct Lay {
  const uint64_t *dn;
  uint64_t nt_max, nb_max;
  __device__ __forceinline__ uint64_t nt() const { return dn[0]; }
  __device__ __forceinline__ uint64_t nb() const { return dn[1]; }
  __device__ __forceinline__ bool ok() const { return dn[0] <= nt_max && dn[1] <= nb_max; }
};

// Offset of block b in the concatenated data blocks: the blocks partition the
// survivors in order, so it is the entry bytes before its first record + 16 B
// per offset entry before it + 16 B per extra before it -- a closed form of
// the survivors' entry-size prefix sums (no scan of the block lengths)
struct BlkOff {
  const uint64_t *Pe, *bf;
  __device__ __forceinline__ uint64_t operator[](uint64_t b) const {
    const uint64_t f = bf[b];
    return Pe[f] + 16 * (f + b);
  }
};

// block b: length, meta entry size, table index
__global__ __launch_bounds__(256) void ck_block_info_kernel(const uint64_t *bf, Lay L, const uint64_t *Pe,
                                                            const uint32_t *kl, const uint64_t *tf, uint64_t *blen,
                                                            uint64_t *msz, uint32_t *btab, uint64_t *tbf,
                                                            uint64_t *zws, uint64_t nz, unsigned long long *guard) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b < nz) zws[b] = 0; // look-back status words of the two block scans that follow
  const bool ok = L.ok();
  const uint64_t nb = L.nb(), nt = L.nt();
  // the table starts in LDS for the binary search below
  __shared__ uint64_t s_tf[kRsLds];
  const bool tf_lds = ok && nt + 1 <= kRsLds;
  if (tf_lds)
    for (uint64_t i = threadIdx.x; i <= nt; i += blockDim.x) s_tf[i] = tf[i];
  __syncthreads();
  const uint64_t *T = tf_lds ? s_tf : tf;
  if (b >= L.nb_max) return;
  if (!ok || b >= nb) { // past the real blocks: zero (the scans over nb_max stay exact)
    blen[b] = 0;
    msz[b] = 0;
    btab[b] = 0;
    if (!ok && b == 0) atomicOr(guard, kGuardLayout);
    return;
  }
  const uint64_t f0 = bf[b], f1 = bf[b + 1];
  blen[b] = (Pe[f1] - Pe[f0]) + 16 * (f1 - f0) + 16;
  msz[b] = 24ull + kl[f0] + kl[f1 - 1]; // AddIndexBlockEntry, table_builder.cc:101-145
  uint64_t lo = 0, hi = nt;
  while (lo + 1 < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (T[mid] <= f0) lo = mid;
    else hi = mid;
  }
  btab[b] = static_cast<uint32_t>(lo);
  if (T[lo] == f0) tbf[lo] = b; // a table's first block (ck_table_info_kernel checks it)
}

// table t: first block index, data / meta bytes, total.  kScan: one
// workgroup holds every table slot (nt_max + 1 <= kTiThreads) and also writes
// the tables' offsets (the exclusive scan of the totals; one launch fewer)
constexpr uint32_t kTiThreads = 1024;
template <bool kScan>
__global__ __launch_bounds__(kTiThreads) void ck_table_info_kernel(const uint64_t *tf, Lay L, const uint64_t *bf,
                                                                   BlkOff BL, const uint64_t *MS, uint64_t *tbf,
                                                                   uint64_t *tdata, uint64_t *tmeta, uint64_t *tlen,
                                                                   uint64_t *toff) {
  const uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t nt = L.nt(), nb = L.nb();
  uint64_t len = 0; // this slot's total (0 past the real tables: the table scan over nt_max stays exact)
  if (t <= L.nt_max) {
    if (!L.ok() || t > nt) {
      if (t < L.nt_max) {
        tlen[t] = 0;
        tdata[t] = 0;
        tmeta[t] = 0;
      }
      tbf[t] = L.ok() ? nb : 0;
    } else {
      // block starting at record tf[t] (every table start is a block start):
      // block_info scattered it into tbf[t] for t < nt; checked, and searched
      // for when it does not hold (a corrupt split: the guards reject the job)
      const uint64_t r = tf[t];
      auto first_block = [&](uint64_t rr, uint64_t guess) {
        if (guess <= nb && bf[guess] == rr) return guess;
        uint64_t lo = 0, hi = nb + 1;
        while (lo + 1 < hi) {
          const uint64_t mid = (lo + hi) >> 1;
          if (bf[mid] <= rr) lo = mid;
          else hi = mid;
        }
        return lo;
      };
      const uint64_t lo = first_block(r, t < nt ? tbf[t] : nb), lo2g = t + 1 < nt ? tbf[t + 1] : nb;
      tbf[t] = lo;
      if (t == nt) { // the sentinel: a zero length when nt < nt_max
        if (t < L.nt_max) {
          tlen[t] = 0;
          tdata[t] = 0;
          tmeta[t] = 0;
        }
      } else {
        // tbf[t+1]: thread t + 1 writes it; found here the same way for the sizes
        const uint64_t lo2 = first_block(tf[t + 1], lo2g);
        const uint64_t d = BL[lo2] - BL[lo], m = MS[lo2] - MS[lo];
        tdata[t] = d;
        tmeta[t] = m;
        len = d + m + 40;
        tlen[t] = len;
      }
    }
  }
  if constexpr (kScan) {
    __shared__ uint64_t s_w[kTiThreads / kWave];
    const uint32_t w = threadIdx.x / kWave;
    const uint64_t inc = wave_incl_scan_u64(len);
    if (lane_id() == kWave - 1) s_w[w] = inc;
    __syncthreads();
    uint64_t before = 0;
    for (uint32_t x = 0; x < w; x++) before += s_w[x];
    if (t <= L.nt_max) toff[t] = before + inc - len; // toff[nt_max] = the total
  }
}

// per block: its output offset (bo, the encode's), its offset inside its
// table and the output offset of its meta entry (brel / mo, the meta
// kernel's: the dependent table lookups are taken here, off the meta
// kernel's chain of loads)
__global__ void ck_block_off_kernel(const uint32_t *btab, Lay L, BlkOff BL, const uint64_t *tbf,
                                    const uint64_t *toff, const uint64_t *tdata, const uint64_t *MS, uint64_t *bo,
                                    uint64_t *brel, uint64_t *mo) {
  const uint64_t b = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= L.nb_max || !L.ok() || b >= L.nb()) return;
  const uint32_t t = btab[b];
  const uint64_t f = tbf[t], rel = BL[b] - BL[f];
  bo[b] = toff[t] + rel;
  brel[b] = rel;
  mo[b] = toff[t] + tdata[t] + (MS[b] - MS[f]);
}

__device__ __forceinline__ void put_le(uint8_t *p, uint64_t v, int n) {
  for (int j = 0; j < n; j++) p[j] = static_cast<uint8_t>(v >> (8 * j));
}

// meta entry of block b (table_builder.cc:101-145): u32 first-key length,
// first key, u32 last-key length, last key, u64 block offset, u64 block size.
// Entries are assembled in LDS by a thread per block, then every table run of
// the workgroup's 256 blocks is written with aligned 16 B stores (byte stores
// straight to HBM from 256 threads at a 56 B stride cost ~10x more).
constexpr uint32_t kMetaLds = 24576; // 256 entries of keys up to 32 B (32 KiB: 4 workgroups per CU, 48 -> 45 us at 16 KiB)
// The block's first / last key come from the encode, which had both entries
// in hand: their source key offsets and key lengths (EncArgs::bmeta, 16 B per
// block), so a meta entry costs one dependent read of each key from the input
// (round 3 read them back from the block just encoded -- extra, then the last
// offset entry, then the key: three dependent lines per block, 247 MB fetched
// for 16 MB of meta at config 3).  MKeys: where the two keys are.
struct MKeys {
  const uint8_t *k0, *k1;
  uint32_t fk, lk;
};
// the keys inside the source bytes [0, send) and the entry size the layout
// used (MS); a failed check sets the guard
__device__ __forceinline__ bool meta_keys(uint64_t b, const uint64_t *bmeta, const uint64_t *MS, const uint8_t *src,
                                          uint64_t send, unsigned long long *guard, MKeys &m) {
  const uint64_t w0 = bmeta[4 * b + 2], w1 = bmeta[4 * b + 3];
  const uint64_t k0 = w0 & ((1ull << 40) - 1), k1 = w1 & ((1ull << 40) - 1);
  m.fk = static_cast<uint32_t>(w0 >> 40);
  m.lk = static_cast<uint32_t>(w1 >> 40);
  m.k0 = src + k0;
  m.k1 = src + k1;
  const bool ok = m.fk <= kMaxKey && m.lk <= kMaxKey && k0 <= send && m.fk <= send - k0 && k1 <= send &&
                  m.lk <= send - k1 && MS[b + 1] - MS[b] == 24ull + m.fk + m.lk;
  if (!ok) atomicOr(guard, kGuardMeta);
  return ok;
}
__device__ __forceinline__ void meta_entry(uint8_t *p, uint64_t rel, uint64_t len, const MKeys &m) {
  put_le(p, m.fk, 4);
  for (uint32_t j = 0; j < m.fk; j++) p[4 + j] = m.k0[j];
  put_le(p + 4 + m.fk, m.lk, 4);
  for (uint32_t j = 0; j < m.lk; j++) p[8 + m.fk + j] = m.k1[j];
  put_le(p + 8 + m.fk + m.lk, rel, 8);
  put_le(p + 16 + m.fk + m.lk, len, 8);
}

__global__ __launch_bounds__(256) void ck_meta_kernel(const uint64_t *bmeta, Lay L, const uint32_t *btab,
                                                      const uint64_t *brel, const uint64_t *mo, const uint64_t *MS,
                                                      const uint64_t *blen, const uint64_t *tbf, uint8_t *dst,
                                                      const uint64_t *need, uint64_t cap, unsigned long long *guard,
                                                      const uint8_t *src, const uint64_t *src_end) {
  __shared__ __attribute__((aligned(16))) uint8_t img[kMetaLds + 16];
  if (*need > cap || !L.ok() || writers_stand_down(*guard))
    return; // output capacity exceeded / corrupt layout / heap-order ties / a redone split: nothing is written
  const uint64_t nb = L.nb();
  const uint64_t b0 = static_cast<uint64_t>(blockIdx.x) * 256u;
  if (b0 >= nb) return;
  const uint64_t bend = b0 + 256u < nb ? b0 + 256u : nb;
  const uint64_t b = b0 + threadIdx.x;
  const uint64_t m0 = MS[b0];
  const uint64_t send = *src_end;
  // a table's meta section must end inside the output buffer (o = mo[...])
  auto in_cap = [&](uint64_t o, uint64_t len) {
    const bool ok = o <= cap && len <= cap - o;
    if (!ok) atomicOr(guard, kGuardMeta);
    return ok;
  };
  MKeys mk{};
  if (MS[bend] - m0 > kMetaLds) {  // long keys: direct per-thread writes
    if (b < bend && meta_keys(b, bmeta, MS, src, send, guard, mk)) {
      const uint64_t o = mo[b];
      if (in_cap(o, MS[b + 1] - MS[b])) meta_entry(dst + o, brel[b], blen[b], mk);
    }
    return;
  }
  const bool ok = b >= bend || meta_keys(b, bmeta, MS, src, send, guard, mk);
  if (b < bend && ok) meta_entry(img + (MS[b] - m0), brel[b], blen[b], mk);
  if (__syncthreads_or(!ok)) return; // a bad entry: the workgroup writes nothing
  for (uint64_t bs = b0; bs < bend;) {  // one run per output table touched
    const uint32_t t = btab[bs];
    const uint64_t be = tbf[t + 1] < bend ? tbf[t + 1] : bend;
    const uint32_t l0 = static_cast<uint32_t>(MS[bs] - m0);
    const int64_t len = static_cast<int64_t>(MS[be] - MS[bs]);
    const uint64_t o = mo[bs];
    if (!in_cap(o, static_cast<uint64_t>(len))) return; // uniform
    uint8_t *g = dst + o;
    const uint32_t pad = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(g) & 15u);
    const uint32_t nchunk = static_cast<uint32_t>((pad + len + 15) >> 4);
    for (uint32_t c = threadIdx.x; c < nchunk; c += 256u) {
      const int64_t lo = 16 * static_cast<int64_t>(c) - pad;
      if (lo >= 0 && lo + 16 <= len) {
        const uint32_t o2 = l0 + static_cast<uint32_t>(lo);
        u32x4 v;
        v.x = lds_u32u(img, o2);
        v.y = lds_u32u(img, o2 + 4);
        v.z = lds_u32u(img, o2 + 8);
        v.w = lds_u32u(img, o2 + 12);
        *reinterpret_cast<u32x4 *>(g + lo) = v;
      } else {
        const int64_t x1 = lo + 16 < len ? lo + 16 : len;
        for (int64_t x = lo < 0 ? 0 : lo; x < x1; x++) g[x] = img[l0 + x];
      }
    }
    bs = be;
  }
}

struct FootWords { // (ck_footer_kernel's copy of Words: declared before it)
  const uint64_t *p[8];
  uint32_t n;
};
struct FootDone {
  FootWords w;     // the device words the host reads after the job
  uint64_t *host;  // pinned, device-mapped host words
  unsigned int *ticket; // zeroed by count_scan_kernel<true>
};

// footer of table t (table_builder.cc:179-211), one workgroup per table: its
// min / max txn (table_builder.cc:47-49) reduced from the blocks' (the encode
// wrote every block's), then the 40 B footer.  (Round 4: folded the separate
// 16-workgroups-per-table reduction kernel in -- one launch fewer.)
constexpr uint32_t kFootThreads = 1024;
__global__ __launch_bounds__(kFootThreads) void ck_footer_kernel(Lay L, const uint64_t *tbf, const uint64_t *toff,
                                                                 const uint64_t *tdata, const uint64_t *tmeta,
                                                                 const uint64_t *bmeta, uint8_t *dst, uint64_t cap,
                                                                 unsigned long long *guard, FootDone done) {
  __shared__ uint64_t smn[kFootThreads / kWave], smx[kFootThreads / kWave];
  const uint64_t t = blockIdx.x;
  const uint64_t nt = L.ok() ? L.nt() : 0;
  if (L.ok() && t < nt && toff[nt] <= cap && !writers_stand_down(*guard)) { // uniform
    const uint64_t f = tbf[t], e = tbf[t + 1];
    const uint64_t o = toff[t], dbytes = tdata[t], mbytes = tmeta[t]; // in flight with the reduction's loads
    uint64_t mn = ~0ull, mx = 0;
#pragma unroll 4
    for (uint64_t b = f + threadIdx.x; b < e; b += kFootThreads) {
      const u32x4 v = *reinterpret_cast<const u32x4 *>(bmeta + 4 * b); // min, max
      const uint64_t x = static_cast<uint64_t>(v.x) | static_cast<uint64_t>(v.y) << 32;
      const uint64_t y = static_cast<uint64_t>(v.z) | static_cast<uint64_t>(v.w) << 32;
      mn = x < mn ? x : mn;
      mx = y > mx ? y : mx;
    }
    for (uint32_t d = kWave / 2; d > 0; d >>= 1) {
      const uint64_t x = __shfl_xor(mn, d, kWave), y = __shfl_xor(mx, d, kWave);
      mn = x < mn ? x : mn;
      mx = y > mx ? y : mx;
    }
    if (lane_id() == 0) {
      smn[threadIdx.x / kWave] = mn;
      smx[threadIdx.x / kWave] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (uint32_t w = 1; w < kFootThreads / kWave; w++) {
        mn = smn[w] < mn ? smn[w] : mn;
        mx = smx[w] > mx ? smx[w] : mx;
      }
      const uint64_t at = o + dbytes + mbytes;
      if (at < o || at > cap || cap - at < 40) { // the footer must end inside the output buffer
        atomicOr(guard, kGuardFooter);
      } else {
        uint8_t *p = dst + at;
        put_le(p, e - f, 8);
        put_le(p + 8, dbytes, 8);
        put_le(p + 16, mbytes, 8);
        put_le(p + 24, mn, 8);
        put_le(p + 32, mx, 8);
      }
    }
  }
  // the job's completion words to the pinned host words by the last footer
  // workgroup to finish (round 5: a one-workgroup pack kernel after this
  // one); a footer's guard bit is released before its ticket, the last
  // arriver acquires before it reads the words.  The host synchronises the
  // stream, then reads them.
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (__hip_atomic_fetch_add(done.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      for (uint32_t i = 0; i < done.w.n; i++)
        done.host[i] = __hip_atomic_load(done.w.p[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
    }
  }
}

// ------------------------------------------------------------------ host side
inline uint32_t grid(uint64_t n, uint32_t per = 256) { return static_cast<uint32_t>((n + per - 1) / per); }

// Bump allocator over the context's persistent compaction arena; requests
// beyond it fall back to hipMalloc and the arena is regrown to the high-water
// mark for the next call (a steady-state call then allocates nothing).
struct Pool {
  Arena &arena;
  uint64_t used = 0;
  std::vector<void *> extra;
  explicit Pool(Arena &a) : arena(a) {}
  ~Pool() {
    for (void *p : extra) (void)hipFree(p);
    if (used > arena.cap) {
      if (arena.base) (void)hipFree(arena.base);
      arena.base = nullptr;
      arena.cap = 0;
      const uint64_t want = used + used / 8;
      if (hipMalloc(&arena.base, want) == hipSuccess) arena.cap = want;
    }
  }
  template <class T> T *get(uint64_t n) {
    const uint64_t bytes = ((n ? n : 1) * sizeof(T) + 255) & ~uint64_t(255);
    const uint64_t at = used;
    used += bytes;
    if (arena.base && used <= arena.cap) return reinterpret_cast<T *>(static_cast<char *>(arena.base) + at);
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) throw std::runtime_error("compaction workspace");
    extra.push_back(p);
    return static_cast<T *>(p);
  }
};

#define CK(x)                                                                                                  \
  do {                                                                                                         \
    hipError_t e_ = (x);                                                                                       \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_));           \
  } while (0)



// greedy segmentation of [0, m) by weights whose prefix sums are
// Pw[i] + add * i (>= threshold closes), optionally clamped at ends[0..*nends];
// the count lands in *dn on the device.
// m: the device record count, n its host bound
void segment(Pool &pool, const uint64_t *Pw, uint64_t add, uint64_t n, const uint64_t *m, uint64_t threshold,
             const uint64_t *ends, const uint64_t *nends, uint64_t *first, uint64_t *dn, hipStream_t s,
             bool long_segments) {
  uint32_t *J = pool.get<uint32_t>(segment_workspace_u32(n));
  CK(launch_segment(Pw, n, threshold, J, dn, first, s, ends, nends, add, long_segments, m));
}

struct Words {
  const uint64_t *p[8];
  uint32_t n;
};

// words w, then arr[0..narr), to the pinned host words; then the sequence
// number at out[flag] once every word has landed (the host spins on it)
__global__ __launch_bounds__(256) void ck_pack_kernel(Words w, const uint64_t *arr, uint64_t narr, uint64_t *out,
                                                      uint64_t seq, uint64_t flag) {
  if (threadIdx.x < w.n) out[threadIdx.x] = *w.p[threadIdx.x];
  for (uint64_t i = threadIdx.x; i < narr; i += 256) out[w.n + i] = arr[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(out + flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the persistent region of count_scan_kernel<true> (Arena::lb): zero when
// (re)allocated, left zero by every launch (its last tile clears it)
void ensure_lb(Arena &arena, uint64_t words, hipStream_t s) {
  if (arena.lb && arena.lb_cap >= words) return;
  if (arena.lb) {
    CK(hipStreamSynchronize(s));
    (void)hipFree(arena.lb);
  }
  arena.lb = nullptr;
  arena.lb_cap = 0;
  const uint64_t cap = words < 1024 ? 1024 : words + words / 4;
  CK(hipMalloc(reinterpret_cast<void **>(&arena.lb), cap * sizeof(uint64_t)));
  arena.lb_cap = cap;
  CK(hipMemsetAsync(arena.lb, 0, cap * sizeof(uint64_t), s));
}

// pinned, device-mapped, coherent host words: kernels store the job's few
// host-bound values straight into them (no copy command per sync)
void ensure_host(Arena &arena, uint64_t words) {
  if (arena.host && arena.host_cap >= words) return;
  if (arena.host) (void)hipHostFree(arena.host);
  arena.host = nullptr;
  arena.host_dev = nullptr;
  arena.host_cap = 0;
  const uint64_t cap = words < 64 ? 64 : words;
  if (hipHostMalloc(reinterpret_cast<void **>(&arena.host), cap * sizeof(uint64_t),
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void **>(&arena.host_dev), arena.host, 0) != hipSuccess) {
    if (arena.host) (void)hipHostFree(arena.host);
    arena.host = nullptr;
    arena.host_dev = nullptr;
    throw std::runtime_error("pinned host words");
  }
  memset(arena.host, 0, cap * sizeof(uint64_t)); // no stale word can equal a sequence number
  arena.host_cap = cap;
}

// pinned, device-mapped upload bytes (Arena::up); the caller's last job is
// complete when it returns, so the bytes are free to overwrite
void ensure_up(Arena &arena, uint64_t bytes) {
  if (arena.up && arena.up_cap >= bytes) return;
  if (arena.up) (void)hipHostFree(arena.up);
  arena.up = nullptr;
  arena.up_dev = nullptr;
  arena.up_cap = 0;
  const uint64_t cap = bytes < 4096 ? 4096 : bytes;
  if (hipHostMalloc(reinterpret_cast<void **>(&arena.up), cap, hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void **>(&arena.up_dev), arena.up, 0) != hipSuccess) {
    if (arena.up) (void)hipHostFree(arena.up);
    arena.up = nullptr;
    arena.up_dev = nullptr;
    throw std::runtime_error("pinned upload bytes");
  }
  arena.up_cap = cap;
}

// device words (+ an optional array after them) -> pinned host words: one
// pack kernel, then the host spins on the sequence word the kernel stores
// last instead of a stream synchronize (each of the job's mid-job syncs cost
// ~20-35 us of idle GPU with hipStreamSynchronize); `complete` also waits for
// the stream to drain (the job's last fetch: the call returns with its work done)
// the host side of a hand-off: spin until the kernel's sequence word lands
void wait_seq(Arena &arena, hipStream_t s, uint64_t flag, uint64_t seq) {
  for (uint64_t it = 1;; it++) {
    if (__atomic_load_n(arena.host + flag, __ATOMIC_ACQUIRE) == seq) return;
    if ((it & 255) == 0) { // a failed stream never stores the word
      const hipError_t q = hipStreamQuery(s);
      if (q == hipSuccess) {
        if (__atomic_load_n(arena.host + flag, __ATOMIC_ACQUIRE) == seq) return;
        throw std::runtime_error("pack kernel finished without its sequence word");
      }
      if (q != hipErrorNotReady) throw std::runtime_error(hipGetErrorString(q));
    }
  }
}

void fetch(Arena &arena, hipStream_t s, std::initializer_list<const uint64_t *> src, const uint64_t *arr = nullptr,
           uint64_t narr = 0, bool complete = false) {
  ensure_host(arena, 8 + narr + 1);
  Words w{};
  for (const uint64_t *p : src) w.p[w.n++] = p;
  const uint64_t flag = arena.host_cap - 1, seq = ++arena.seq;
  ck_pack_kernel<<<1, 256, 0, s>>>(w, arr, narr, arena.host_dev, seq, flag);
  CK(hipGetLastError());
  if (complete) {
    CK(hipStreamSynchronize(s));
    return;
  }
  wait_seq(arena, s, flag, seq);
}

} // namespace

int compact_impl(Arena &arena, hipStream_t s, unsigned long long *err_count, const uint8_t *d_src,
                 const uint64_t *d_blk_off,
                 const uint64_t *d_blk_len, uint64_t nblocks, const uint64_t *h_tfb, uint32_t ntables,
                 uint64_t block_threshold, uint64_t table_limit, uint32_t base_level, uint32_t txn_mode,
                 uint8_t *d_dst, uint64_t dst_cap, uint64_t *d_table_off, uint64_t *d_table_len, uint64_t max_tables,
                 uint64_t *res, std::string &err, MergeOut *mo) {
  try {
    Pool pool(arena);
    // Host syncs: (1) the run starts and the input block bytes (they size
    // every array and bound the output counts), (2) completion with the
    // output size, the table / block counts and the error flags (the
    // capacity check is on the device: no writer touches d_dst when the
    // output exceeds dst_cap).  Everything else stays on the stream: the
    // kept count stays on the device (the segmentation reads it there), so
    // the host enqueues the whole tail while the merge runs.
    // 1. decode every block
    uint64_t *rb_all = pool.get<uint64_t>(nblocks + 1);
    uint64_t *errs = pool.get<uint64_t>(2);
    uint64_t *d_rs = pool.get<uint64_t>(ntables + 1);
    uint64_t *part = pool.get<uint64_t>(2 * count_scan_tiles(nblocks));
    ensure_lb(arena, count_scan_workspace(nblocks), s);
    unsigned long long *bad = reinterpret_cast<unsigned long long *>(pool.get<uint64_t>(1));
    // consistency guard: [0] bits set by any check of the job, [1] the end of
    // the source bytes its blocks span (both set by count_scan_kernel<true>)
    // guard[0] bits, guard[1] source end; guard + 32 the check kernel's 9
    // ticket counters, then the footer's, 256 B apart (u32 at guard + 32 + 32 g)
    unsigned long long *guard = reinterpret_cast<unsigned long long *>(pool.get<uint64_t>(32 + 10 * 32));
    const uint64_t *src_end = reinterpret_cast<const uint64_t *>(guard + 1);
    // record index of every input table's first record (its run start): the
    // table first blocks travel in the pinned upload words (no copy command),
    // the run starts and the input bytes come back in the pinned host words
    ensure_up(arena, (ntables + 1) * 8);
    memcpy(arena.up, h_tfb, (ntables + 1) * 8);
    ensure_host(arena, 8 + ntables + 2);
    {
      const uint64_t flag = arena.host_cap - 1, seq = ++arena.seq;
      CountScanArgs ca{};
      ca.src = d_src;
      ca.blk_off = d_blk_off;
      ca.blk_len = d_blk_len;
      ca.nblocks = nblocks;
      ca.rec_base = rb_all;
      ca.ws = arena.lb;
      ca.epoch = 0;
      ca.part = part;
      ca.tfb = reinterpret_cast<const uint64_t *>(arena.up_dev);
      ca.ntfb = ntables + 1;
      ca.run_start = d_rs;
      ca.err_count = err_count;
      ca.errs = errs;
      ca.bad = bad;
      ca.guard = guard;
      ca.host = arena.host_dev;
      ca.seq = seq;
      ca.flag = flag;
      CK(launch_count_scan(ca, true, s));
      wait_seq(arena, s, flag, seq);
    }
    const uint64_t in_bytes = arena.host[0]; // every survivor's entry lies in these bytes
    if (in_bytes == ~0ull) { // count_scan_kernel<true>: a look-back gave up (kGuardLookback)
      err = "device consistency check failed (a look-back of the record count scan gave up): nothing was written";
      return SSTC_E_INTERNAL;
    }
    std::vector<uint64_t> run_start(arena.host + 1, arena.host + 2 + ntables);
    const uint64_t n = run_start[ntables];
    res[0] = n;
    if (n >= 0xFFFFFFFFull) {
      err = "too many records";
      return SSTC_E_INVALID_ARG;
    }
    if (mo && n > mo->cap) { // (nothing else is enqueued yet)
      err = "more records than max_records";
      return SSTC_E_CAPACITY;
    }
    const uint64_t wsn = scan_workspace_elems(n + 1) + 64;
    uint64_t *ws2 = pool.get<uint64_t>(wsn);
    RecX *RX = pool.get<RecX>(n);
    uint32_t *status = pool.get<uint32_t>(nblocks);
    SK *A = pool.get<SK>(n ? n : 1), *B = pool.get<SK>(n ? n : 1);
    DecArgs da{d_src, d_blk_off, d_blk_len, nblocks, rb_all,
               sstc_records{}, txn_mode, status, err_count, A, bad};
    da.rx = RX;
    da.inv = guard;
    CK(launch_decode(da, s));
    if (n == 0) { // DoCompactJob still finishes its first (empty) output table
      fetch(arena, s, {reinterpret_cast<const uint64_t *>(err_count), errs});
      if (arena.host[0] != arena.host[1]) {
        err = "an input block failed to decode";
        return SSTC_E_INVALID_ARG;
      }
      if (mo) { // nothing to merge
        CK(hipStreamSynchronize(s));
        mo->ties[0] = mo->ties[1] = 0;
        return SSTC_OK;
      }
      if (max_tables < 1 || dst_cap < 40) {
        err = "output capacity";
        return SSTC_E_CAPACITY;
      }
      uint8_t foot[40] = {0};
      const uint64_t mn = ~0ull;
      memcpy(foot + 24, &mn, 8);
      const uint64_t offs[2] = {0, 40}, forty = 40;
      CK(hipMemcpyAsync(d_dst, foot, 40, hipMemcpyHostToDevice, s));
      CK(hipMemcpyAsync(d_table_off, offs, 16, hipMemcpyHostToDevice, s)); // nt + 1 entries
      CK(hipMemcpyAsync(d_table_len, &forty, 8, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      res[1] = 0; res[2] = 0; res[3] = 1; res[4] = 40;
      return SSTC_OK;
    }
    // 2. sort keys + merge
    const KeyView kv{d_src, RX};
    uint64_t nruns = ntables;
    const uint64_t *rb = d_rs; // run starts, nruns + 1
    const Abort dec_fail{err_count, errs, nullptr}, stop{err_count, errs, bad};
    const uint64_t fftiles = (n + kFfTile - 1) / kFfTile;
    uint64_t *ffws = nullptr; // look-back words of the filter
    // survivors of the keep / drop filter (sized by n: the kept count is known after it)
    uint64_t *totals = pool.get<uint64_t>(3);
    Rec KR{pool.get<uint8_t>(n), pool.get<uint32_t>(n), nullptr, pool.get<uint64_t>(n), pool.get<uint64_t>(n),
           nullptr}; // vl / vo: not needed by the whole-entry encode
    uint64_t *Pd = pool.get<uint64_t>(n + 1), *Pe = pool.get<uint64_t>(n + 1);
    // k-way merge passes; run boundaries of every pass are known on the host,
    // which builds every pass's group descriptors into pinned mapped memory;
    // the check kernel copies them to the device
    std::vector<KGroup> kg;
    std::vector<uint32_t> pass_groups, pass_ids, pass_wgs, pass_ways;
    {
      std::vector<uint64_t> cur = run_start;
      // passes: ceil(log8 runs), each pass as narrow as that allows (the
      // splitter search grows with k^2): 128 runs merge as 4, 4, 8 instead of
      // 8, 8, 2 (config 4 splitters 310 -> 257 us, merge unchanged)
      auto passes_for = [](size_t runs) {
        uint32_t p = 0;
        for (size_t c = 1; c < runs; c *= kKWay) p++;
        return p;
      };
      while (cur.size() > 2) {
        std::vector<uint64_t> next;
        uint32_t ids = 0, wgs = 0, ng = 0;
        size_t way = kKWay;
        {
          const size_t runs = cur.size() - 1;
          const uint32_t P = passes_for(runs);
          // the largest power of two <= runs^(1/P), doubled until the
          // remaining passes still suffice (128 runs: 4, 4, 8 instead of 8, 8, 2)
          size_t w = 2;
          while (w * 2 <= kKWay) {
            size_t pw = 1;
            for (uint32_t q = 0; q < P; q++) pw *= w * 2;
            if (pw > runs) break;
            w *= 2;
          }
          while (w < kKWay && passes_for((runs + w - 1) / w) + 1 > P) w *= 2;
          way = w;
        }
        for (size_t r0 = 0; r0 + 1 < cur.size(); r0 += way) {
          const uint32_t k = static_cast<uint32_t>(std::min<size_t>(way, cur.size() - 1 - r0));
          KGroup g{};
          g.nruns = k;
          g.stride = kKWin / k;
          g.base = ids;
          g.wg0 = wgs;
          g.sbase[0] = 0;
          for (uint32_t q = 0; q <= k; q++) g.start[q] = cur[r0 + q];
          for (uint32_t q = 0; q < k; q++)
            g.sbase[q + 1] = g.sbase[q] + static_cast<uint32_t>((g.start[q + 1] - g.start[q] + g.stride - 1) / g.stride);
          ids += g.sbase[k] + 1;
          wgs += static_cast<uint32_t>((g.start[k] - g.start[0] + kKWin - 1) / kKWin);
          kg.push_back(g);
          ng++;
          next.push_back(cur[r0]);
        }
        next.push_back(cur.back());
        pass_groups.push_back(ng);
        pass_ways.push_back(static_cast<uint32_t>(way));
        pass_ids.push_back(ids);
        pass_wgs.push_back(wgs);
        cur = std::move(next);
      }
      // the filter's look-back status words, cleared by the check kernel
      ffws = pool.get<uint64_t>(1 + 3 * fftiles);
      KGroup *d_kg = kg.empty() ? nullptr : pool.get<KGroup>(kg.size());
      const uint64_t kg_bytes = kg.size() * sizeof(KGroup);
      static_assert(sizeof(KGroup) % 8 == 0, "KGroup copied as words");
      ensure_up(arena, kg_bytes);
      if (kg_bytes) memcpy(arena.up, kg.data(), kg_bytes);
      // a thread per block boundary (the source-end bound, once a same-address
      // atomic per workgroup that capped this grid, comes from the count kernel)
      ck_check_blocks_kernel<<<std::max<uint32_t>(grid(std::max<uint64_t>(nblocks, 1ull + 3 * fftiles)), 1u), 256, 0,
                               s>>>(A, rb_all, nblocks, rb, nruns, kv, bad, dec_fail, ffws, 1 + 3 * fftiles, guard,
                                                           reinterpret_cast<const uint64_t *>(arena.up_dev),
                                                           reinterpret_cast<uint64_t *>(d_kg), kg_bytes / 8,
                                                           reinterpret_cast<unsigned int *>(guard + 32));
      if (!kg.empty()) {
        const uint32_t max_ids = *std::max_element(pass_ids.begin(), pass_ids.end());
        uint32_t *Cm = pool.get<uint32_t>(static_cast<uint64_t>(max_ids) * kKWay);
        uint64_t *Gm = pool.get<uint64_t>(max_ids);
        uint32_t max_j = 0;
        for (size_t p = 0; p < pass_groups.size(); p++) max_j = std::max(max_j, pass_ids[p] + pass_wgs[p] + pass_groups[p]);
        uint32_t *Jm = pool.get<uint32_t>(max_j);
        SK *Sm = pool.get<SK>(max_ids);
        KWin *Wm = pool.get<KWin>(*std::max_element(pass_wgs.begin(), pass_wgs.end()) + 1);
        size_t at = 0;
        for (size_t p = 0; p < pass_groups.size(); p++) {
          const uint32_t ng = pass_groups[p];
          ck_kw_sample_kernel<<<grid(pass_ids[p]), 256, 0, s>>>(A, d_kg + at, ng, pass_ids[p], Sm, stop);
          if (pass_ways[p] <= 4)
            ck_kw_split_kernel<4><<<grid(static_cast<uint64_t>(pass_ids[p]) * 4), 256, 0, s>>>(A, Sm, d_kg + at, ng,
                                                                                               pass_ids[p], kv, Cm, Gm, stop);
          else
            ck_kw_split_kernel<8><<<grid(static_cast<uint64_t>(pass_ids[p]) * 8), 256, 0, s>>>(A, Sm, d_kg + at, ng,
                                                                                               pass_ids[p], kv, Cm, Gm, stop);
          ck_kw_bounds_kernel<<<grid(pass_ids[p]), 256, 0, s>>>(d_kg + at, ng, pass_ids[p], Gm, Jm, stop);
          if (pass_wgs[p]) {
            ck_kw_win_kernel<<<grid(pass_wgs[p]), 256, 0, s>>>(d_kg + at, ng, pass_wgs[p], Cm, Gm, Jm, Wm, stop);
            ck_mg_merge_kernel<<<pass_wgs[p], kMgThreads, 0, s>>>(A, B, Wm, kv);
          }
          std::swap(A, B);
          at += ng;
        }
      }
    }
    // the job's error words (decode errors, unsorted inputs, guard bits) are
    // read after the last kernel: a rejected job writes nothing (the filter
    // of a stopped job reports no survivor)
    const std::initializer_list<const uint64_t *> err_words = {
        reinterpret_cast<const uint64_t *>(err_count), errs, reinterpret_cast<const uint64_t *>(bad),
        reinterpret_cast<const uint64_t *>(guard)};
    auto job_error = [&](const uint64_t *h) -> int { // h: the err_words as fetched
      if (h[0] != h[1]) {
        err = "an input block failed to decode";
        return SSTC_E_INVALID_ARG;
      }
      if (h[2]) {
        err = "input SST records are not sorted (key asc)";
        return SSTC_E_INVALID_ARG;
      }
      if (h[3] & kGuardLookback) {
        err = "device consistency check failed (a decoupled look-back gave up waiting for a predecessor "
              "workgroup): nothing was written";
        return SSTC_E_INTERNAL;
      }
      if (h[3] & kGuardMergeId) {
        err = "device consistency check failed after the merge (merged record ids out of range)";
        return SSTC_E_INTERNAL;
      }
      if (!mo && (h[3] & kGuardTieBoth) == kGuardTieBoth) {
        err = "inputs hold equal (key, txn) records with different contents in different tables: the "
              "reference's heap orders them by its history; nothing was written";
        return SSTC_E_TIE_ORDER;
      }
      return SSTC_OK;
    };
    if (mo) { // sstc_merge_records: the merged order, no filter
      unsigned long long *ties = reinterpret_cast<unsigned long long *>(pool.get<uint64_t>(2));
      CK(hipMemsetAsync(ties, 0, 2 * sizeof(uint64_t), s));
      ck_merged_kernel<<<grid(n), 256, 0, s>>>(A, n, kv, rb, static_cast<uint32_t>(nruns), mo->out, ties, stop, guard,
                                               txn_mode);
      CK(hipGetLastError());
      fetch(arena, s, {reinterpret_cast<const uint64_t *>(err_count), errs, reinterpret_cast<const uint64_t *>(bad),
                       reinterpret_cast<const uint64_t *>(guard), reinterpret_cast<const uint64_t *>(ties),
                       reinterpret_cast<const uint64_t *>(ties + 1)},
            nullptr, 0, true);
      if (const int r = job_error(arena.host)) return r;
      mo->ties[0] = arena.host[4];
      mo->ties[1] = arena.host[5];
      return SSTC_OK;
    }
    // 3. keep / drop and the survivors gathered in merge order with their
    // prefix sums (sized by n: the kept count is known after the pass)
    ck_filter_kernel<<<static_cast<uint32_t>(fftiles), kFtThreads, 0, s>>>(A, n, kv, base_level, KR, Pd, Pe, ffws,
                                                                        totals, stop, guard, txn_mode, rb,
                                                                        static_cast<uint32_t>(nruns));
    if (arena.fault == 1) CK(hipMemsetAsync(KR.ko, 0xFF, n * sizeof(uint64_t), s)); // test: bad key offsets
    if (arena.fault == 3) { // test: a look-back that gave up (kGuardLookback, byte 1 of the guard word)
      CK(hipMemsetAsync(reinterpret_cast<uint8_t *>(guard) + 1, static_cast<int>(kGuardLookback >> 8), 1, s));
    }
    if (arena.fault == 2) CK(hipMemsetAsync(Pe, 0x5A, (n + 1) * sizeof(uint64_t), s)); // test: bad prefix sums
    if (max_tables == 0) { // no room for the first table (m >= 1 unless the job is rejected)
      fetch(arena, s, err_words, nullptr, 0, true);
      if (const int r = job_error(arena.host)) return r;
      err = "more output tables than max_tables";
      return SSTC_E_CAPACITY;
    }
    // 4. the table split (key+value bytes, compact.cc:290) and the block split
    // (entry + offset-entry bytes, table_builder.cc:57-59) clamped at table
    // ends, over the device kept count (totals[0]; n bounds it)
    uint64_t *tf = pool.get<uint64_t>(n + 1), *dn = pool.get<uint64_t>(2);
    segment(pool, Pd, 0, n, totals, table_limit, nullptr, nullptr, tf, dn, s, true);
    uint64_t *bf = pool.get<uint64_t>(n + 1);
    uint32_t *Jb = pool.get<uint32_t>(segment_workspace_u32(n));
    // the block split's launch plan: this context's last job decides (kArithOnly
    // while the equal-size chain held: none of the general walk's nine
    // launches; kGeneralOnly while it failed, retrying both every kSegProbe jobs)
    SegMode mode = arena.seg_mode;
    if (mode == SegMode::kGeneralOnly && ++arena.seg_general_jobs >= kSegProbe) {
      mode = SegMode::kBoth;
      arena.seg_general_jobs = 0;
    }
    // 5. layout over count bounds (no host fetch: see Lay): the survivors'
    // key+value and entry + offset-entry bytes are at most the input block bytes
    const uint64_t tl = table_limit ? table_limit : 1, bt = block_threshold ? block_threshold : 1;
    const uint64_t nt_max = std::max<uint64_t>(1, std::min<uint64_t>({n, in_bytes / tl + 1, max_tables}));
    const uint64_t nb_max = std::max<uint64_t>(1, std::min<uint64_t>(n, in_bytes / bt + nt_max));
    const Lay L{dn, nt_max, nb_max};
    uint64_t *blen = pool.get<uint64_t>(nb_max), *msz = pool.get<uint64_t>(nb_max);
    uint32_t *btab = pool.get<uint32_t>(nb_max);
    const uint64_t nzb = scan_status_words(nb_max); // <= nb_max
    uint64_t *ws3 = pool.get<uint64_t>(2 * nzb);
    uint64_t *tbf = pool.get<uint64_t>(nt_max + 1);
    const BlkOff BL{Pe, bf}; // block offsets in closed form (Pe[0] = 0)
    uint64_t *MS = pool.get<uint64_t>(nb_max + 1);
    uint64_t *tdata = pool.get<uint64_t>(nt_max), *tmeta = pool.get<uint64_t>(nt_max);
    // the output size is checked on the device (every writer below stands down
    // when it exceeds dst_cap) and by the host after the last sync
    const uint64_t *need = d_table_off + nt_max; // = d_table_off[nt]: the lengths past nt are zero
    uint64_t *bo = pool.get<uint64_t>(nb_max);
    uint64_t *brel = pool.get<uint64_t>(nb_max), *mo = pool.get<uint64_t>(nb_max);
    uint64_t *bmeta = pool.get<uint64_t>(4 * nb_max); // per block: min / max txn, first / last key
    ensure_host(arena, 9);
    FootDone done{};
    {
      const std::initializer_list<const uint64_t *> words = {
          reinterpret_cast<const uint64_t *>(err_count), errs, reinterpret_cast<const uint64_t *>(bad),
          reinterpret_cast<const uint64_t *>(guard), need, dn, dn + 1, totals};
      for (const uint64_t *p : words) done.w.p[done.w.n++] = p;
    }
    done.host = arena.host_dev;
    done.ticket = reinterpret_cast<unsigned int *>(guard + 32 + 32 * 9);
    // the block split (entry + offset-entry bytes, table_builder.cc:57-59,
    // clamped at the table ends) and everything after it: enqueued once, and
    // once more with the general walk when a kArithOnly chain failed
    auto tail = [&](SegMode m) {
      CK(launch_segment(Pe, n, block_threshold, Jb, dn + 1, bf, s, tf, dn, 16, false, totals, m, guard));
      ck_block_info_kernel<<<grid(nb_max), 256, 0, s>>>(bf, L, Pe, KR.kl, tf, blen, msz, btab, tbf, ws3, 2 * nzb,
                                                        guard);
      CK(launch_scan(msz, nb_max, 0, MS, ws3 + nzb, s, true, 0, guard));
      if (nt_max + 1 <= kTiThreads) {
        ck_table_info_kernel<true><<<1, kTiThreads, 0, s>>>(tf, L, bf, BL, MS, tbf, tdata, tmeta, d_table_len,
                                                            d_table_off);
      } else {
        ck_table_info_kernel<false><<<grid(nt_max + 1), 256, 0, s>>>(tf, L, bf, BL, MS, tbf, tdata, tmeta,
                                                                     d_table_len, nullptr);
        CK(launch_scan(d_table_len, nt_max, 0, d_table_off, ws2, s, false, 0, guard)); // <= max_tables + 1 elements
      }
      ck_block_off_kernel<<<grid(nb_max), 256, 0, s>>>(btab, L, BL, tbf, d_table_off, tdata, MS, bo, brel, mo);
      // 6. encode blocks, meta entries, footers
      EncArgs ea{d_src, d_src, sstc_records{KR.type, KR.kl, KR.vl, KR.tx, KR.ko, KR.vo}, bf, nb_max, Pe, bo, blen,
                 d_dst, 1};
      ea.nb_dev = dn + 1;
      // blocks past an LDS slot are encoded by the wave that met them (config 5 319 -> 233 us)
      ea.need = need;
      ea.cap = dst_cap;
      ea.bmeta = bmeta; // block min / max txn (reduced by the encode kernels) and first / last key
      // output blocks are as large as the input's on average (an entry is copied
      // whole): past 8 KiB the job's blocks mostly exceed the encode's LDS slot
      ea.large_blocks = nblocks && in_bytes / nblocks > 8192 ? 1u : 0u;
      ea.src_end = src_end;
      ea.guard = guard;
      ea.xcd = 2; // XCD-chunked block order (the grid is the nb_max bound)
      CK(launch_enc_emit(ea, s));
      ck_meta_kernel<<<static_cast<uint32_t>((nb_max + 255) / 256), 256, 0, s>>>(bmeta, L, btab, brel, mo, MS, blen,
                                                                                tbf, d_dst, need, dst_cap, guard,
                                                                                d_src, src_end);
      ck_footer_kernel<<<static_cast<uint32_t>(nt_max), kFootThreads, 0, s>>>(L, tbf, d_table_off, tdata, tmeta,
                                                                             bmeta, d_dst, dst_cap, guard, done);
      CK(hipGetLastError());
      CK(hipStreamSynchronize(s));
    };
    tail(mode);
    if (const int r = job_error(arena.host)) return r;
    if (arena.host[3] & kGuardSplitRedo) { // the chain failed and nothing was written: the walk this time
      const uint64_t g = arena.host[3] & (kGuardLongGroup | kGuardInv | kGuardTieCross | kGuardTieDiff);
      CK(hipMemcpyAsync(guard, &g, sizeof g, hipMemcpyHostToDevice, s));
      CK(hipMemsetAsync(done.ticket, 0, sizeof(unsigned int), s));
      arena.seg_redo_count++;
      mode = SegMode::kGeneralOnly;
      tail(mode);
      if (const int r = job_error(arena.host)) return r;
    }
    // the next job's plan: the chain alone after a job whose chain held
    if (mode != SegMode::kGeneralOnly)
      arena.seg_mode = arena.host[3] & (kGuardArithFail | kGuardSplitRedo) ? SegMode::kGeneralOnly
                                                                            : SegMode::kArithOnly;
    else if (arena.seg_mode != SegMode::kGeneralOnly)
      arena.seg_mode = SegMode::kGeneralOnly;
    res[1] = arena.host[7];
    res[4] = arena.host[4];
    res[2] = arena.host[6];
    res[3] = arena.host[5];
    if (arena.host[5] > max_tables) {
      err = "more output tables than max_tables";
      return SSTC_E_CAPACITY;
    }
    if (arena.host[3] & ~(kGuardLongGroup | kGuardInv | kGuardTieCross | kGuardTieDiff | kGuardArithFail)) {
      err = "device consistency check failed (guard bits 0x" + [](uint64_t v) {
        char b[24];
        snprintf(b, sizeof b, "%llx", static_cast<unsigned long long>(v));
        return std::string(b);
      }(arena.host[3]) + "): d_dst and the table arrays are undefined";
      return SSTC_E_INTERNAL;
    }
    if (res[4] > dst_cap) {
      err = "output buffer too small";
      return SSTC_E_CAPACITY;
    }
    return SSTC_OK;
  } catch (const std::exception &e) {
    err = e.what();
    return SSTC_E_HIP;
  }
}

} // namespace sstc

// ------------------------------------------------------------------ SST open
// DecodeExtraInfo + FetchBlockIndexInfo (sstable/table_reader.cc:52-156) for
// many SST images at once.  The meta section is a length-prefixed stream
// (entry = u32 fkl | first key | u32 lkl | last key | u64 block offset | u64
// block size, table_builder.cc:101-145) with no offset table, so the entry
// starts are the chain 0 -> next(0) -> ... with next(p) = p + 24 + fkl + lkl.
// It is recovered in parallel, 16 KiB tiles of the section at a time:
//   ot_tile_kernel  next(p) for every byte position p of the tile; pointer
//                   doubling in LDS gives, for every p, the entries the chain
//                   from p holds inside the tile and the first chain position
//                   past the tile (its exit)
//   ot_hop_kernel   one wave per table follows the exits tile to tile
//                   (section bytes / 16 KiB dependent loads) and records where
//                   the chain enters each tile and with which entry index
//   ot_emit_kernel  every entered tile is staged in LDS, one lane walks the
//                   chain from the entry point (the tile kernel already proved
//                   where it starts), and the workgroup writes the block index
//                   entries in parallel
namespace sstc {
namespace {

constexpr uint32_t kOtTile = 16384, kOtThreads = 1024, kOtPer = kOtTile / kOtThreads;
constexpr uint32_t kOtRounds = 10; // 2^10 > 16384 / 24 chain positions per tile
static_assert((1u << kOtRounds) > kOtTile / 24 && kOtPer % 8 == 0, "doubling rounds must cover a tile's chain");
constexpr uint32_t kOtBad = 0xFFFFFFFFu;

struct OtTable {
  uint64_t meta;  // absolute offset of the meta section in d_src
  uint64_t data;  // absolute offset of the table image (block offsets are relative to it)
  uint64_t moff;  // data section length = meta section offset
  uint64_t nb;    // footer num_blocks (0 for a table whose footer is rejected)
  uint64_t fb;    // first output block
  uint32_t mlen;  // meta section length (< 2^32 - 1)
  uint32_t tile0; // first tile
};

__device__ __forceinline__ uint32_t ot_find(const OtTable *t, uint32_t nt, uint32_t g) {
  uint32_t lo = 0, hi = nt; // last table with tile0 <= g
  while (lo + 1 < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (t[mid].tile0 <= g) lo = mid;
    else hi = mid;
  }
  return lo;
}

// next(p) = p + 24 + fkl + lkl, or kOtBad when the entry at p runs past the
// section (the bounds FetchBlockIndexInfo leaves unchecked), for kOtBatch
// positions (each < mlen) of a thread: all first-length loads in flight
// together, then all second-length loads (one position at a time serializes
// 2 dependent global loads per position; the whole thread's set at once
// spills).  A load at p < mlen stays inside the image (the 40 B footer
// follows the section); the second load's address is clamped and its result
// dropped when invalid.
constexpr uint32_t kOtBatch = 8;
__device__ __forceinline__ void ot_next_group(const uint8_t *m, uint32_t mlen, const uint32_t *pos, uint32_t *e) {
  uint32_t k1[kOtBatch], q[kOtBatch];
#pragma unroll
  for (uint32_t k = 0; k < kOtBatch; k++) k1[k] = g_u32u(m + pos[k]);
#pragma unroll
  for (uint32_t k = 0; k < kOtBatch; k++) {
    const uint64_t qq = static_cast<uint64_t>(pos[k]) + 4 + k1[k];
    const bool ok = static_cast<uint64_t>(pos[k]) + 4 <= mlen && qq + 4 <= mlen;
    q[k] = ok ? static_cast<uint32_t>(qq) : kOtBad;
  }
#pragma unroll
  for (uint32_t k = 0; k < kOtBatch; k++) {
    const uint32_t k2 = g_u32u(m + (q[k] == kOtBad ? 0u : q[k]));
    const uint64_t ee = static_cast<uint64_t>(q[k]) + 20 + k2;
    e[k] = q[k] != kOtBad && ee <= mlen ? static_cast<uint32_t>(ee) : kOtBad;
  }
}

__global__ void ot_footer_kernel(const uint8_t *src, const uint64_t *foot_at, uint32_t nt, uint64_t *out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nt || foot_at[t] == ~uint64_t(0)) return;
  const uint8_t *f = src + foot_at[t];
#pragma unroll
  for (int k = 0; k < 5; k++) out[5 * static_cast<uint64_t>(t) + k] = g_u64u(f + 8 * k);
}

__global__ __launch_bounds__(kOtThreads) void ot_tile_kernel(const uint8_t *src, const OtTable *tabs, uint32_t nt,
                                                             uint64_t *EC, uint32_t *tstart) {
  __shared__ uint16_t sL[kOtTile]; // last in-tile position of the chain from p
  __shared__ uint16_t sC[kOtTile]; // hops from p to it
  const uint32_t g = blockIdx.x;
  const OtTable T = tabs[ot_find(tabs, nt, g)];
  const uint8_t *m = src + T.meta;
  const uint32_t t0 = (g - T.tile0) * kOtTile;
  const uint32_t n = min(kOtTile, T.mlen - t0);
  if (threadIdx.x == 0) tstart[g] = kOtBad;
#pragma unroll 1
  for (uint32_t g0 = 0; g0 < kOtPer; g0 += kOtBatch) {
    uint32_t pos[kOtBatch], nx[kOtBatch];
#pragma unroll
    for (uint32_t j = 0; j < kOtBatch; j++) {
      const uint32_t p = threadIdx.x + (g0 + j) * kOtThreads;
      pos[j] = t0 + (p < n ? p : 0u);
    }
    ot_next_group(m, T.mlen, pos, nx);
#pragma unroll
    for (uint32_t j = 0; j < kOtBatch; j++) {
      const uint32_t p = threadIdx.x + (g0 + j) * kOtThreads;
      if (p < n) {
        const bool in = nx[j] != kOtBad && nx[j] < t0 + n;
        sL[p] = static_cast<uint16_t>(in ? nx[j] - t0 : p);
        sC[p] = in ? 1 : 0;
      }
    }
  }
  __syncthreads();
  for (uint32_t r = 0; r < kOtRounds; r++) {
    uint16_t l[kOtPer], c[kOtPer];
#pragma unroll
    for (uint32_t k = 0; k < kOtPer; k++) {
      const uint32_t p = threadIdx.x + k * kOtThreads;
      if (p < n) {
        const uint32_t j = sL[p];
        l[k] = sL[j];
        c[k] = static_cast<uint16_t>(sC[p] + sC[j]);
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kOtPer; k++) {
      const uint32_t p = threadIdx.x + k * kOtThreads;
      if (p < n) {
        sL[p] = l[k];
        sC[p] = c[k];
      }
    }
    __syncthreads();
  }
  uint64_t *ec = EC + static_cast<uint64_t>(g) * kOtTile;
  // the chain's last in-tile position: its entry is valid iff its next is
#pragma unroll 1
  for (uint32_t g0 = 0; g0 < kOtPer; g0 += kOtBatch) {
    uint32_t pos[kOtBatch], nx[kOtBatch];
#pragma unroll
    for (uint32_t j = 0; j < kOtBatch; j++) {
      const uint32_t p = threadIdx.x + (g0 + j) * kOtThreads;
      pos[j] = t0 + (p < n ? sL[p] : 0u);
    }
    ot_next_group(m, T.mlen, pos, nx);
#pragma unroll
    for (uint32_t j = 0; j < kOtBatch; j++) {
      const uint32_t p = threadIdx.x + (g0 + j) * kOtThreads;
      if (p < n) {
        const uint64_t cnt = sC[p] + (nx[j] != kOtBad ? 1u : 0u);
        ec[p] = nx[j] | (cnt << 32);
      }
    }
  }
}

// One wave per table.  The chain enters a tile near its start (within one
// entry of the previous exit: 56 B at 16 B keys), so the exit words of the
// first kOtWinPos positions of kOtWinTiles tiles are fetched into LDS in one
// batch of coalesced loads and the hops inside that window resolve from LDS;
// an entry point further into a tile reads its word from HBM.
constexpr uint32_t kOtWinTiles = 64, kOtWinPos = kWave, kOtWinBatch = 16;
__global__ __launch_bounds__(kWave) void ot_hop_kernel(const OtTable *tabs, uint32_t nt, const uint64_t *EC,
                                                       uint32_t *tstart, uint64_t *tbase, int32_t *status) {
  __shared__ uint64_t sW[kOtWinTiles][kOtWinPos];
  const uint32_t t = blockIdx.x;
  const OtTable T = tabs[t];
  if (T.nb == 0) return; // uniform
  const uint32_t lane = threadIdx.x;
  const uint32_t ntiles = (T.mlen + kOtTile - 1) / kOtTile;
  uint64_t x = 0, idx = 0;
  uint32_t wb = ~0u; // first (table-relative) tile of the LDS window
  int32_t st = SSTC_TAB_OK;
  for (;;) {
    if (x >= T.mlen) { // the section ends before num_blocks entries
      st = SSTC_TAB_BAD_META;
      break;
    }
    const uint32_t gl = static_cast<uint32_t>(x / kOtTile), o = static_cast<uint32_t>(x % kOtTile);
    uint64_t v;
    if (o < kOtWinPos) {
      if (wb == ~0u || gl < wb || gl >= wb + kOtWinTiles) {
        wb = gl;
        const uint32_t rows = min(kOtWinTiles, ntiles - gl);
        for (uint32_t i0 = 0; i0 < rows; i0 += kOtWinBatch) {
          uint64_t w[kOtWinBatch];
#pragma unroll
          for (uint32_t j = 0; j < kOtWinBatch; j++) {
            const uint32_t row = min(i0 + j, rows - 1); // clamped: loads issue unconditionally
            w[j] = EC[static_cast<uint64_t>(T.tile0 + wb + row) * kOtTile + lane];
          }
#pragma unroll
          for (uint32_t j = 0; j < kOtWinBatch; j++)
            if (i0 + j < rows) sW[i0 + j][lane] = w[j];
        }
        __syncthreads();
      }
      v = sW[gl - wb][o];
    } else {
      v = EC[static_cast<uint64_t>(T.tile0 + gl) * kOtTile + o];
    }
    if (lane == 0) {
      tstart[T.tile0 + gl] = o;
      tbase[T.tile0 + gl] = idx;
    }
    idx += v >> 32;
    if (idx >= T.nb) break;
    const uint32_t e = static_cast<uint32_t>(v);
    if (e == kOtBad) {
      st = SSTC_TAB_BAD_META;
      break;
    }
    x = e;
  }
  if (lane == 0 && st != SSTC_TAB_OK) status[t] = st;
}

struct OtOut {
  uint64_t *blk_off, *blk_len, *fk_off, *lk_off;
  uint32_t *fk_len, *lk_len;
};

// the chain from the tile's entry point is walked by one lane over the tile
// staged in LDS (two dependent LDS reads per entry, <= 683 entries), then the
// workgroup parses the listed entries in parallel.  It replaced a marking pass
// by pointer doubling from the entry point (10 rounds of barriers over every
// byte position): config 3 162 -> 85 us.
constexpr uint32_t kOtEmitThreads = 256, kOtMaxEntries = kOtTile / 24 + 1;
__global__ __launch_bounds__(kOtEmitThreads) void ot_emit_kernel(const uint8_t *src, const OtTable *tabs, uint32_t nt,
                                                                 const uint32_t *tstart, const uint64_t *tbase,
                                                                 OtOut o, int32_t *status) {
  __shared__ uint32_t sImg[kOtTile / 4 + 4];
  __shared__ uint16_t sPos[kOtMaxEntries];
  __shared__ uint32_t sCnt;
  const uint32_t g = blockIdx.x;
  const uint32_t s = tstart[g];
  if (s == kOtBad) return; // uniform: the chain skips this tile
  const uint32_t ti = ot_find(tabs, nt, g);
  const OtTable T = tabs[ti];
  const uint8_t *m = src + T.meta;
  const uint32_t t0 = (g - T.tile0) * kOtTile;
  const uint32_t n = min(kOtTile, T.mlen - t0);
  // words covering tile bytes [0, n + 8); the reads past the section stay in
  // the image (the 40 B footer follows it)
  const uint32_t W = (n + 8 + 3) / 4;
  for (uint32_t i = threadIdx.x; i < W; i += kOtEmitThreads) sImg[i] = g_u32u(m + t0 + 4 * i);
  __syncthreads();
  const uint8_t *img = reinterpret_cast<const uint8_t *>(sImg);
  const uint64_t base = tbase[g];
  const uint64_t want = base < T.nb ? T.nb - base : 0;
  const uint64_t lim = T.mlen - t0; // section end, tile-relative
  if (threadIdx.x == 0) {
    uint64_t p = s;
    uint32_t j = 0;
    while (p < n && j < want && p + 4 <= lim) {
      const uint64_t q = p + 4 + lds_u32u(img, static_cast<uint32_t>(p));
      if (q + 4 > lim) break;
      const uint32_t k2 = q <= n ? lds_u32u(img, static_cast<uint32_t>(q)) : g_u32u(m + t0 + q);
      const uint64_t e = q + 20 + k2;
      if (e > lim) break;
      sPos[j++] = static_cast<uint16_t>(p);
      p = e;
    }
    sCnt = j;
  }
  __syncthreads();
  const uint32_t cnt = sCnt;
  for (uint32_t j = threadIdx.x; j < cnt; j += kOtEmitThreads) {
    const uint32_t p = sPos[j];
    const uint32_t fkl = lds_u32u(img, p);
    const uint64_t q = p + 4ull + fkl;
    const uint32_t lkl = q <= n ? lds_u32u(img, static_cast<uint32_t>(q)) : g_u32u(m + t0 + q);
    const uint64_t r = q + 4 + lkl;
    uint64_t bo, bl;
    if (r + 16 <= n) {
      bo = lds_u64u(img, static_cast<uint32_t>(r));
      bl = lds_u64u(img, static_cast<uint32_t>(r + 8));
    } else {
      bo = g_u64u(m + t0 + r);
      bl = g_u64u(m + t0 + r + 8);
    }
    const uint64_t b = T.fb + base + j;
    o.blk_off[b] = T.data + bo;
    o.blk_len[b] = bl;
    o.fk_off[b] = T.meta + t0 + p + 4;
    o.fk_len[b] = fkl;
    o.lk_off[b] = T.meta + t0 + q + 4;
    o.lk_len[b] = lkl;
    if (bo > T.moff || bl > T.moff - bo) atomicCAS(&status[ti], SSTC_TAB_OK, SSTC_TAB_BAD_BLOCK);
  }
}

} // namespace

int open_tables_impl(Arena &arena, hipStream_t s, const uint8_t *d_src, uint64_t src_bytes, const uint64_t *h_off,
                     const uint64_t *h_bytes, uint32_t nt, uint64_t max_blocks, const OpenOut &out, uint64_t *h_tfb,
                     int32_t *h_status, uint64_t *h_footer, std::string &err) {
  try {
    // pinned words: [0, nt) footer addresses, [nt, 6 nt) footers, then the
    // table descriptors, the first-block prefix and the statuses
    const uint64_t w_tab = 6 * static_cast<uint64_t>(nt), w_tfb = w_tab + 6 * static_cast<uint64_t>(nt);
    const uint64_t w_st = w_tfb + nt + 1, words = w_st + nt / 2 + 2;
    ensure_host(arena, words);
    uint64_t *H = arena.host;
    std::vector<int32_t> st(nt, SSTC_TAB_OK);
    for (uint32_t t = 0; t < nt; t++) {
      H[t] = h_bytes[t] >= 40 ? h_off[t] + h_bytes[t] - 40 : ~uint64_t(0);
      if (h_bytes[t] < 40) st[t] = SSTC_TAB_BAD_FOOTER;
    }
    if (nt) {
      ot_footer_kernel<<<grid(nt), 256, 0, s>>>(d_src, arena.host_dev, nt, arena.host_dev + nt);
      CK(hipGetLastError());
      CK(hipStreamSynchronize(s));
    }
    std::vector<OtTable> tabs(nt);
    uint64_t total = 0, tiles = 0;
    h_tfb[0] = 0;
    for (uint32_t t = 0; t < nt; t++) {
      const uint64_t *f = H + nt + 5 * static_cast<uint64_t>(t);
      uint64_t nb = 0, moff = 0, mlen = 0;
      if (st[t] == SSTC_TAB_OK) {
        nb = f[0];
        moff = f[1];
        mlen = f[2];
        if (moff > h_bytes[t] - 40 || mlen > h_bytes[t] - 40 - moff) st[t] = SSTC_TAB_BAD_FOOTER;
        else if (mlen >= kOtBad) st[t] = SSTC_TAB_TOO_LARGE;
        else if (nb > mlen / 24) st[t] = SSTC_TAB_BAD_META; // every entry takes >= 24 B
      }
      if (h_footer) {
        for (int k = 0; k < 5; k++) h_footer[5 * static_cast<uint64_t>(t) + k] = st[t] == SSTC_TAB_BAD_FOOTER ? 0 : f[k];
      }
      OtTable &T = tabs[t];
      T.data = h_off[t];
      T.meta = h_off[t] + moff;
      T.moff = moff;
      T.nb = st[t] == SSTC_TAB_OK ? nb : 0;
      T.fb = total;
      T.mlen = st[t] == SSTC_TAB_OK ? static_cast<uint32_t>(mlen) : 0;
      T.tile0 = static_cast<uint32_t>(tiles);
      total += T.nb;
      if (T.nb) tiles += (mlen + kOtTile - 1) / kOtTile;
      else T.mlen = 0; // no tiles: nothing to parse
      h_tfb[t + 1] = total;
    }
    for (uint32_t t = 0; t < nt; t++) h_status[t] = st[t];
    if (total > max_blocks) {
      err = "block index capacity too small (" + std::to_string(total) + " blocks)";
      return SSTC_E_CAPACITY;
    }
    if (tiles >= (uint64_t(1) << 31)) {
      err = "meta sections too large";
      return SSTC_E_INVALID_ARG;
    }
    (void)src_bytes;
    std::memcpy(H + w_tab, tabs.data(), nt * sizeof(OtTable));
    std::memcpy(H + w_tfb, h_tfb, (nt + 1) * sizeof(uint64_t));
    std::memcpy(H + w_st, st.data(), nt * sizeof(int32_t));
    Pool pool(arena);
    OtTable *d_tabs = pool.get<OtTable>(nt);
    int32_t *d_st = pool.get<int32_t>(nt);
    if (nt) {
      CK(hipMemcpyAsync(d_tabs, H + w_tab, nt * sizeof(OtTable), hipMemcpyHostToDevice, s));
      CK(hipMemcpyAsync(d_st, H + w_st, nt * sizeof(int32_t), hipMemcpyHostToDevice, s));
    }
    if (out.table_first_block)
      CK(hipMemcpyAsync(out.table_first_block, H + w_tfb, (nt + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    if (tiles) {
      uint64_t *EC = pool.get<uint64_t>(tiles * kOtTile);
      uint32_t *tstart = pool.get<uint32_t>(tiles);
      uint64_t *tbase = pool.get<uint64_t>(tiles);
      ot_tile_kernel<<<static_cast<uint32_t>(tiles), kOtThreads, 0, s>>>(d_src, d_tabs, nt, EC, tstart);
      ot_hop_kernel<<<nt, kWave, 0, s>>>(d_tabs, nt, EC, tstart, tbase, d_st);
      OtOut o{out.blk_off, out.blk_len, out.first_key_off, out.last_key_off, out.first_key_len, out.last_key_len};
      ot_emit_kernel<<<static_cast<uint32_t>(tiles), kOtEmitThreads, 0, s>>>(d_src, d_tabs, nt, tstart, tbase, o, d_st);
      CK(hipGetLastError());
    }
    if (nt) CK(hipMemcpyAsync(H + w_st, d_st, nt * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    std::memcpy(h_status, H + w_st, nt * sizeof(int32_t));
    return SSTC_OK;
  } catch (const std::exception &e) {
    err = e.what();
    return SSTC_E_HIP;
  }
}

} // namespace sstc
