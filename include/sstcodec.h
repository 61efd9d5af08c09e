/*
 * sstcodec.h — C-ABI of the MI355X SST block codec (libsstcodec.so).
 *
 * Drop-in boundary for the byte work of the reference's sstable layer
 * (NamHoaiNguyen/LSM-KV-Storage).  The reference has no FFI; its boundary is the
 * C++ class API of sstable/ (see INTEGRATION.md).  Each entry point below says
 * which reference interface it replaces.
 *
 * Conventions
 *   - Every pointer named d_* is DEVICE memory (hipMalloc / torch CUDA tensor)
 *     owned by the caller.  Nothing in this header takes ownership.
 *   - All work is enqueued on the context's stream; calls return after enqueue
 *     (asynchronous) unless documented otherwise.  A call whose workspace need
 *     exceeds what the context holds grows it (synchronising the stream); after
 *     sstc_ctx_reserve() for the largest batch no call allocates or
 *     synchronises, so a sequence of calls can be captured into a hipGraph.
 *   - Return value: 0 = SSTC_OK, negative = error; the thread-local message is
 *     in sstc_last_error_string().  Per-block data errors are NOT call errors:
 *     they are reported in d_block_status[] (SSTC_BLK_*) and counted in the
 *     context error counter (sstc_ctx_error_count).
 *   - Re-entrancy: no global mutable state.  A context is used by one host
 *     thread at a time; concurrent TableBuilders (reference db/db_impl.cc:
 *     354-362) each own a context.
 *
 * Block format (reference sstable/block_builder.h:14-57), all little-endian:
 *   block       = data entries | offset entries | extra
 *   PUT entry   = u8 type(0) | u32 key_len | key | u32 val_len | val | u64 txn
 *   DEL entry   = u8 type(1) | u32 key_len | key | u64 txn
 *   offset      = u64 entry_start | u64 entry_size            (16 B per entry)
 *   extra       = u64 num_entries | u64 offset_section_start   (16 B)
 *
 * Record model: value fields are encoded iff val_len != SSTC_NO_VALUE (the
 * reference's `value.data() != nullptr`, block_builder.cc:19-21,56).  Decode
 * gives DELETE records SSTC_NO_VALUE (block_reader.cc:84-88).
 */
#ifndef SSTCODEC_H
#define SSTCODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SSTC_ABI_VERSION 1u
#define SSTC_NO_VALUE 0xFFFFFFFFu
#define SSTC_TYPE_PUT 0u     /* db/status.h:13 ValueType::PUT     */
#define SSTC_TYPE_DELETED 1u /* db/status.h:15 ValueType::DELETED */
#define SSTC_MAX_KEY 4096u   /* common/macros.h:29 kMaxKeySize     */

/* call status */
#define SSTC_OK 0
#define SSTC_E_INVALID_ARG -1
#define SSTC_E_HIP -2
#define SSTC_E_NOMEM -3
#define SSTC_E_NO_DEVICE -4
#define SSTC_E_CAPACITY -5 /* workspace too small: call sstc_ctx_reserve */
#define SSTC_E_INTERNAL -6 /* a device-side consistency check of a job failed: no out-of-range access was made,
                              but d_dst and the output table arrays are undefined (partly written) */
#define SSTC_E_TIE_ORDER -7 /* sstc_compact / sstc_compact_files: the inputs hold records with equal key and txn
                               in different tables whose contents differ, so the reference's MergeIterator heap
                               orders them by its push / pop history (merge_iterator.h:91-95), which this job does
                               not reproduce: nothing was written (d_dst untouched, no output file created or
                               changed); the output table arrays are undefined.  The engine never writes such
                               inputs (its txn ids are unique per write); a caller that must handle them runs
                               the drop-in MergeIterator path, which takes the heap's order */

/* per-block status, d_block_status[b] */
#define SSTC_BLK_OK 0
#define SSTC_BLK_TOO_SMALL 1      /* block shorter than its 16 B extra            */
#define SSTC_BLK_EMPTY 2          /* num_entries == 0 (FlushBlock never writes it) */
#define SSTC_BLK_OFFSETS_RANGE 3  /* offset section outside [0, len-16)           */
#define SSTC_BLK_ENTRY_RANGE 4    /* an entry runs outside the data section        */
#define SSTC_BLK_BAD_TYPE 5       /* type byte not PUT/DELETED                     */
#define SSTC_BLK_KEY_TOO_LONG 6   /* key_len > 4096 (block_builder.cc:38 assert)   */
#define SSTC_BLK_TOO_LARGE 7      /* block >= 4 GiB                                */
#define SSTC_BLK_NO_ROOM 8        /* round trip: re-encoded block longer than the  */
                                  /* input block (overlapping offset entries)     */
#define SSTC_BLK_COUNT_MISMATCH 9 /* decode: num_entries != d_rec_base difference  */

/* txn read mode.  COMPAT reproduces BlockReader::GetTransactionIdFromDataEntry
 * (block_reader.cc:104-114): it tests value.empty() instead of the type, so an
 * empty-value PUT reads its txn as (txn & 0xffffffff) << 32 and a re-encode
 * writes that value.  CORRECT reads the field the encoder wrote. */
#define SSTC_TXN_COMPAT 0u
#define SSTC_TXN_CORRECT 1u

typedef struct sstc_ctx sstc_ctx;

/* Structure-of-arrays record table in device memory (one element per record).
 * key_off / val_off are byte offsets into the key / value source buffer given
 * alongside (for decode output: into d_src). */
typedef struct sstc_records {
  uint8_t *type;
  uint32_t *key_len;
  uint32_t *val_len; /* SSTC_NO_VALUE = no value fields */
  uint64_t *txn;
  uint64_t *key_off;
  uint64_t *val_off;
} sstc_records;

/* One decoded record packed in 32 B: what a host-side iterator serves per
 * entry (sstc_pack_records).  Offsets into the decoded bytes; the value starts
 * at key_off + val_rel. */
typedef struct sstc_record32 {
  uint64_t key_off;
  uint64_t txn;
  uint32_t key_len;
  uint32_t val_rel;  /* value offset - key offset; 0 without value fields */
  uint32_t val_len;  /* SSTC_NO_VALUE = no value fields (a DELETE) */
  uint8_t type;
  uint8_t pad[3];
} sstc_record32;

uint32_t sstc_version(void);
const char *sstc_last_error_string(void);

/* Context: device, stream and workspace.  stream is a hipStream_t (NULL = the
 * null stream); it may be changed between calls with sstc_ctx_set_stream,
 * which orders the new stream after all work already queued on the old one
 * (an event recorded on the old stream, waited on by the new one), because
 * every call of a context shares its workspace.  A context is not
 * thread-safe: one host thread at a time (SURVEY.md §8(b) threading). */
int sstc_ctx_create(int device, void *stream, sstc_ctx **out);
int sstc_ctx_destroy(sstc_ctx *ctx);
int sstc_ctx_set_stream(sstc_ctx *ctx, void *stream);
/* The current stream must still be alive when sstc_ctx_set_stream switches
 * away from it (an event is recorded on it).  A caller about to destroy the
 * context's stream synchronizes it and calls sstc_ctx_drop_stream first: the
 * context forgets it without recording anything on it and runs on the null
 * stream until the next sstc_ctx_set_stream. */
int sstc_ctx_drop_stream(sstc_ctx *ctx);
/* Pre-size the workspace for up to max_blocks blocks and max_records records. */
int sstc_ctx_reserve(sstc_ctx *ctx, uint64_t max_blocks, uint64_t max_records);
/* Synchronise the stream; return the number of blocks that failed since the
 * last reset (per-block codes are in the callers' d_block_status arrays).
 * The count also includes any prefix scan of sstc_count_records /
 * sstc_segment_records / sstc_encode_blocks whose decoupled look-back gave up
 * waiting for a predecessor workgroup (its sums are wrong; never seen unless
 * the GPU stalls a workgroup for seconds); the compaction calls reject such a
 * job with SSTC_E_INTERNAL instead. */
int sstc_ctx_error_count(sstc_ctx *ctx, uint64_t *out);
int sstc_ctx_reset_errors(sstc_ctx *ctx);

/* ---- decode (replaces TableReader::CreateAndSetupDataForBlockReader,
 *      sstable/table_reader.cc:212-241, and the BlockReader field accessors,
 *      sstable/block_reader.cc:59-114, for a batch of blocks) ---------------- */

/* Exclusive scan of per-block entry counts from the 16 B extras.
 * d_rec_base has nblocks+1 elements; d_rec_base[nblocks] = total records.  A
 * block whose extra is malformed counts 0 records. */
int sstc_count_records(sstc_ctx *ctx, const uint8_t *d_src, const uint64_t *d_blk_off,
                       const uint64_t *d_blk_len, uint64_t nblocks, uint64_t *d_rec_base);

/* Parse every entry of every block into the record table at d_rec_base[b] + i.
 * Key/value offsets are absolute offsets into d_src.  d_block_status may be
 * NULL. */
int sstc_decode_blocks(sstc_ctx *ctx, const uint8_t *d_src, const uint64_t *d_blk_off,
                       const uint64_t *d_blk_len, uint64_t nblocks, const uint64_t *d_rec_base,
                       sstc_records out, uint32_t txn_mode, uint32_t *d_block_status);

/* Pack records [0, nrec) of a device record table (sstc_decode_blocks output)
 * into d_out[0, nrec) (device, 32 B each), for one device-to-host copy of what
 * a table iterator serves (BlockReaderIterator's accessors,
 * sstable/block_reader_iterator.cc:30-71). */
int sstc_pack_records(sstc_ctx *ctx, sstc_records in, uint64_t nrec, sstc_record32 *d_out);

/* ---- encode (replaces BlockBuilder::AddEntry/EncodeExtraInfo and the block
 *      write of TableBuilder::FlushBlock, sstable/block_builder.cc:12-109,
 *      sstable/table_builder.cc:62-99) --------------------------------------- */

/* Greedy block segmentation of TableBuilder::AddEntry (table_builder.cc:57-59):
 * a block is closed right after the record that brings sum(entry_size + 16) to
 * >= block_threshold.  Writes record-index boundaries d_blk_first[0..nb] and the
 * block count to *d_nblocks (device). d_blk_first needs nrec+1 elements. */
int sstc_segment_records(sstc_ctx *ctx, const uint32_t *d_key_len, const uint32_t *d_val_len,
                         uint64_t nrec, uint64_t block_threshold, uint64_t *d_blk_first,
                         uint64_t *d_nblocks);

/* Encode records [d_blk_first[b], d_blk_first[b+1]) into block b, blocks laid
 * out back-to-back from byte out_base of d_dst.  The record table holds nrec
 * records and every d_blk_first[] value is <= nrec.  Writes d_out_blk_len[b]
 * (nblocks elements) and d_out_blk_off[0..nblocks] (nblocks+1 elements; the
 * last one is the end offset).  Keys are read at d_key_src + key_off[r], values
 * at d_val_src + val_off[r].  An empty range encodes a 16 B block with
 * num_entries = 0 (TableBuilder::FlushBlock never writes one, so callers skip
 * empty ranges). */
int sstc_encode_blocks(sstc_ctx *ctx, const uint8_t *d_key_src, const uint8_t *d_val_src,
                       sstc_records in, uint64_t nrec, const uint64_t *d_blk_first,
                       uint64_t nblocks, uint64_t out_base, uint8_t *d_dst,
                       uint64_t *d_out_blk_off, uint64_t *d_out_blk_len);

/* ---- fused device-resident decode -> re-encode (the compaction pass-through
 *      of db/compact.cc:254-302 for blocks whose records all survive) -------- */

/* Decode every block and re-encode its records; block b is written at
 * d_blk_off[b] of d_dst (d_dst must not alias d_src).  d_out_blk_len[b] gets
 * the re-encoded size (0 on error); d_block_status[b] the decode status.
 * Either output pointer may be NULL. */
int sstc_roundtrip_blocks(sstc_ctx *ctx, const uint8_t *d_src, uint8_t *d_dst,
                          const uint64_t *d_blk_off, const uint64_t *d_blk_len,
                          uint64_t nblocks, uint32_t txn_mode, uint64_t *d_out_blk_len,
                          uint32_t *d_block_status);

/* Host-resident round trip (the path starts and ends in host memory, as
 * compaction's SST files do): the blocks of h_src (ascending, disjoint,
 * inside nbytes; pinned memory for full PCIe rate) are streamed through the
 * device in chunks of <= chunk_bytes (>= 4096; a larger block travels alone):
 * H2D on an upload stream, sstc_roundtrip_blocks on the context's stream,
 * D2H on a download stream, a ring of 3 device buffer pairs ordered by
 * events, so both copy directions and the kernels overlap.  Results as
 * sstc_roundtrip_blocks, written to h_dst at the blocks' offsets; a rejected
 * block keeps its source bytes, bytes between blocks are unspecified.
 * h_out_blk_len / h_block_status may be NULL.  Synchronises. */
int sstc_roundtrip_host(sstc_ctx *ctx, const uint8_t *h_src, uint8_t *h_dst, uint64_t nbytes,
                        const uint64_t *h_blk_off, const uint64_t *h_blk_len, uint64_t nblocks, uint32_t txn_mode,
                        uint64_t chunk_bytes, uint64_t *h_out_blk_len, uint32_t *h_block_status);

/* Diagnostic: the copy ceiling the codec kernels are compared to — a plain
 * device copy of nbytes (multiple of 16, both pointers 16 B aligned), one
 * 16 B non-temporal load + store per lane.  Asynchronous on the context's
 * stream.  Not part of the reference interface. */
int sstc_copy_probe(sstc_ctx *ctx, const uint8_t *d_src, uint8_t *d_dst, uint64_t nbytes);

/* ---- compaction job (replaces Compact::DoCompactJob, db/compact.cc:232-363,
 *      with its MergeIterator, db/merge_iterator.cc) ------------------------ */

typedef struct sstc_compact_params {
  uint64_t block_threshold; /* Config::GetSSTBlockSize() (4096)                 */
  uint64_t table_limit;     /* Config::GetPerMemTableSizeLimit() (32 MiB): an   */
                            /* output SST is finished once its key+value bytes */
                            /* reach it (compact.cc:290)                       */
  uint32_t base_level;      /* 1: IsBaseLevelForKey() holds for every key, so a */
                            /* tombstone that starts a key group is dropped.   */
                            /* This is the only state the reference reaches    */
                            /* (only L0->L1 compactions exist, so levels >= 2  */
                            /* stay empty, compact.cc:365-380) and the only    */
                            /* mode that claims reference parity.  0: every    */
                            /* such tombstone is kept (the branch compact.cc:  */
                            /* 347-349 takes for a key equal to the smallest   */
                            /* key of a level->=2 SST) -- framework-defined    */
                            /* semantics for engines with deeper levels,       */
                            /* pinned by the restated driver oracle/           */
                            /* ref_compact.cc, not by a reachable reference run */
  uint32_t txn_mode;        /* SSTC_TXN_COMPAT = the reference iterator's txn   */
} sstc_compact_params;

typedef struct sstc_compact_result {
  uint64_t records_in, records_kept, blocks_out, tables_out, bytes_out;
} sstc_compact_result;

/* Host staging for the C++ mirror's TableBuilder (include/sstc_table.h
 * HostVec): `bytes` of page-locked memory when the HIP runtime can pin it
 * (*pinned = 1; a later H2D copy from it is a true async DMA), else ordinary
 * memory (*pinned = 0); NULL when neither is available.  Free it with
 * sstc_host_free and the same `pinned`.  (The builder keeps its arrays in a
 * per-thread pool, so a thread that builds SST after SST pins once.) */
void *sstc_host_alloc(uint64_t bytes, int *pinned);
void sstc_host_free(void *p, int pinned);

/* Compact `ntables` input SSTs given in iterator order (compact.cc:186-230).
 * Their data blocks are listed table by table in d_blk_off/d_blk_len (block
 * index order); table t owns blocks [h_table_first_block[t],
 * h_table_first_block[t+1]) (HOST array, ntables+1 elements).  Every input
 * table must hold its keys in ascending order (SSTC_E_INVALID_ARG otherwise).
 * The versions of a key may be in any txn order as read (the compat reader
 * turns an empty-value PUT's txn t into (t & 0xffffffff) << 32,
 * block_reader.cc:109-111): they merge as the reference's heap pops them, each
 * input in file order under the smallest txn before it, for groups of up to
 * 64 blocks (longer out-of-order groups: SSTC_E_INVALID_ARG).  Records merge
 * in MergeIterator order (key asc, txn desc; equal (key, txn): lower input
 * table first -- the reference's std::priority_queue orders such ties by heap
 * history: identical copies, the only kind the engine writes, give the same
 * bytes in any order; inputs holding the same (key, txn) with different
 * contents in different tables are refused with SSTC_E_TIE_ORDER and nothing
 * written), ShouldKeepEntry filters
 * them, and the survivors are written as complete SST images (blocks, meta
 * section, 40 B footer) back to back into d_dst: table t at d_table_off[t]
 * with d_table_len[t] bytes (TableBuilder::GetFileSize() = d_table_len[t] + 1).
 * d_table_off needs max_tables+1 elements; entries past tables_out may be
 * overwritten (d_table_len with 0, d_table_off with the total).  This call
 * allocates its own workspace and synchronises the stream (output sizes are
 * data dependent).  Output larger than dst_cap: SSTC_E_CAPACITY with
 * result->bytes_out = the exact size needed and not one byte of d_dst written
 * (every writer checks the size on the device); more tables than max_tables:
 * SSTC_E_CAPACITY (result->tables_out = the count) and not one byte of d_dst
 * written. */
int sstc_compact(sstc_ctx *ctx, const uint8_t *d_src, const uint64_t *d_blk_off, const uint64_t *d_blk_len,
                 uint64_t nblocks, const uint64_t *h_table_first_block, uint32_t ntables,
                 const sstc_compact_params *params, uint8_t *d_dst, uint64_t dst_cap, uint64_t *d_table_off,
                 uint64_t *d_table_len, uint64_t max_tables, sstc_compact_result *result);

/* ---- merge order (replaces db::MergeIterator's SeekToFirst + Next walk,
 *      db/merge_iterator.cc:34-46,79-92, over the TableReaderIterators that
 *      Compact::CreateMergeIterator makes, db/compact.cc:186-230) ----------- */

/* One record of the merged order: the key's offset in d_src (the entry's type
 * byte and u32 key length precede it, its u32 value length and value follow
 * it, block format above) and its txn as the reference's iterator reads it
 * (txn_mode). */
typedef struct sstc_merged_record {
  uint64_t key_off;
  uint64_t txn;
} sstc_merged_record;

typedef struct sstc_merge_result {
  uint64_t records;    /* records of all inputs = merged records                  */
  uint64_t cross_ties; /* runs of merged records with equal key and merge txn     */
                       /* that span two or more inputs                            */
  uint64_t tie_diffs;  /* those of them whose records are not all alike (type,    */
                       /* txn as read, value): the heap's order may differ        */
} sstc_merge_result;

/* Decode every block of the `ntables` inputs (given as for sstc_compact) and
 * write their records to d_out[0, records) in MergeIterator order: key
 * ascending, then txn descending, where an input's versions of a key compete
 * under the smallest txn before them in that input (the order the reference's
 * heap pops them when the compat reader returns them out of txn order), then
 * the lower input first.  The heap orders records with equal (key, txn) from
 * different inputs by heap history (merge_iterator.h:91-95); such runs are
 * counted, and when tie_diffs is non-zero this order may differ from the
 * reference's heap (the caller then takes the heap's order).  Inputs whose
 * keys are not ascending, or with a block that fails to decode:
 * SSTC_E_INVALID_ARG.  More records than max_records: SSTC_E_CAPACITY with
 * result->records set and nothing written.  Synchronises the stream. */
int sstc_merge_records(sstc_ctx *ctx, const uint8_t *d_src, const uint64_t *d_blk_off, const uint64_t *d_blk_len,
                       uint64_t nblocks, const uint64_t *h_table_first_block, uint32_t ntables, uint32_t txn_mode,
                       sstc_merged_record *d_out, uint64_t max_records, sstc_merge_result *result);

/* ---- point lookups (replaces TableReader::GetValue without a block cache,
 *      sstable/table_reader.cc:168-210, with BlockReader::GetValue,
 *      sstable/block_reader.cc:20-57, for a batch of keys) ------------------ */

#define SSTC_GET_PUT 0u       /* db::ValueType::PUT                          */
#define SSTC_GET_DELETED 1u   /* db::ValueType::DELETED                      */
#define SSTC_GET_NOT_FOUND 2u /* db::ValueType::NOT_FOUND                    */
#define SSTC_GET_BAD_BLOCK 4u /* a probed entry / trailer / index entry is out of range */

/* Block indexes of one or many SSTs (device arrays; what TableReader holds
 * after FetchBlockIndexInfo, table_reader.cc:86-156). */
typedef struct sstc_block_index {
  const uint64_t *blk_off;           /* block b = d_src[blk_off[b] .. + blk_len[b])     */
  const uint64_t *blk_len;
  const uint64_t *last_key_off;      /* GetLargestKey() of block b = keys[off .. + len) */
  const uint32_t *last_key_len;
  const uint8_t *keys;
  const uint64_t *table_first_block; /* table t owns blocks [tfb[t], tfb[t+1])          */
  uint32_t ntables;
  uint64_t src_bytes;                /* size of d_src: every read is bounds-checked    */
  uint64_t keys_bytes;               /* size of keys                                   */
} sstc_block_index;

/* Query q looks key d_q_keys[d_q_key_off[q] .. + d_q_key_len[q]) up in table
 * d_q_table[q]: the block is the first whose largest key >= key (the table's
 * last block when none is: GetBlockOffsetAndSize), then the block's entries
 * are binary-searched exactly as BlockReader::GetValue does (the first probed
 * equal key wins; the txn is not consulted).  Outputs per query: SSTC_GET_*
 * type, for PUT the value at d_src[d_out_val_off .. + d_out_val_len), and the
 * probed block (UINT64_MAX when the table has no block).  d_out_block may be
 * NULL.  A table without blocks answers NOT_FOUND (the reference reads
 * block_index_[-1] there). */
int sstc_get_batch(sstc_ctx *ctx, const uint8_t *d_src, const sstc_block_index *index,
                   const uint32_t *d_q_table, const uint8_t *d_q_keys, uint64_t q_keys_bytes,
                   const uint64_t *d_q_key_off, const uint32_t *d_q_key_len, uint64_t nq, uint32_t *d_out_type,
                   uint64_t *d_out_val_off, uint32_t *d_out_val_len, uint64_t *d_out_block);

/* ---- SST open on the device (replaces CreateAndSetupDataForTableReader's
 *      DecodeExtraInfo + FetchBlockIndexInfo, sstable/table_reader.cc:52-156,
 *      for many tables at once) --------------------------------------------- */

#define SSTC_TAB_OK 0
#define SSTC_TAB_BAD_FOOTER 1 /* image < 40 B, or the footer's meta section lies  */
                              /* outside the image                               */
#define SSTC_TAB_BAD_META 2   /* the meta section ends (or an entry runs past it)  */
                              /* before num_blocks entries                       */
#define SSTC_TAB_BAD_BLOCK 3  /* a block range lies outside the data section       */
#define SSTC_TAB_TOO_LARGE 4  /* meta section >= 4 GiB                             */

/* Table t is the SST image d_src[h_tab_off[t] .. + h_tab_bytes[t]) with
 * h_tab_bytes[t] = TableBuilder::GetFileSize() - 1 (the reference reads the
 * footer at file_size - 40 - 1).  The footers are read and the meta sections
 * parsed on the device (the length-prefixed entry chain is recovered by
 * pointer doubling over 16 KiB tiles, not walked): table t's blocks are
 * [h_table_first_block[t], h_table_first_block[t+1]) of the outputs, with
 * d_blk_off / d_first_key_off / d_last_key_off ABSOLUTE offsets into d_src,
 * so (d_blk_off, d_blk_len, d_last_key_off, d_last_key_len, keys = d_src,
 * d_table_first_block) is an sstc_block_index and (d_blk_off, d_blk_len,
 * h_table_first_block) is sstc_compact's input.  Per-table status in
 * h_table_status (SSTC_TAB_*): a table with a rejected footer gets no blocks;
 * for BAD_META its block entries are undefined; for BAD_BLOCK the entries are
 * the raw meta values.  h_footer (5 words per table: num_blocks, meta offset,
 * meta length, min txn, max txn; NULL to skip), d_table_first_block (NULL to
 * skip).  Returns SSTC_E_CAPACITY (with h_table_first_block filled) when
 * more than max_blocks blocks are listed.  Synchronises the stream. */
int sstc_open_tables(sstc_ctx *ctx, const uint8_t *d_src, uint64_t src_bytes, const uint64_t *h_tab_off,
                     const uint64_t *h_tab_bytes, uint32_t ntables, uint64_t max_blocks, uint64_t *d_blk_off,
                     uint64_t *d_blk_len, uint64_t *d_first_key_off, uint32_t *d_first_key_len,
                     uint64_t *d_last_key_off, uint32_t *d_last_key_len, uint64_t *d_table_first_block,
                     uint64_t *h_table_first_block, int32_t *h_table_status, uint64_t *h_footer);

/* ---- file-to-file compaction (Compact::DoCompactJob end to end: the input
 *      SST files are read, compacted on the device and the output SSTs written
 *      and fsync'ed, db/compact.cc:232-322 with io/linux_file.cc:138-195) --- */

typedef struct sstc_pipe sstc_pipe; /* pinned host + device staging, grow-only */

typedef struct sstc_file_out {
  uint64_t sst_id;           /* output file = out_prefix + sst_id + ".sst"      */
  uint64_t file_size;        /* TableBuilder::GetFileSize(): bytes + 1          */
  uint64_t smallest_key_off; /* GetSmallestKey() bytes in key_arena             */
  uint64_t largest_key_off;  /* GetLargestKey() bytes in key_arena              */
  uint32_t smallest_key_len, largest_key_len;
} sstc_file_out;

typedef struct sstc_files_timing {
  double index_s;   /* footer + meta section read and parse (host, per file) */
  double load_s;    /* data sections: pread into pinned memory + H2D, overlapped */
  double compact_s; /* sstc_compact on the device                               */
  double store_s;   /* D2H + pwrite + fsync of the outputs, overlapped          */
  double total_s;
} sstc_files_timing;

int sstc_pipe_create(sstc_ctx *ctx, uint32_t io_threads, sstc_pipe **out);
int sstc_pipe_destroy(sstc_pipe *pipe);

/* Compact the SST files in_paths[0..n_in) (iterator order, each with its
 * GetFileSize() value in in_file_sizes = bytes + 1) into out_prefix + id +
 * ".sst", ids first_sst_id, first_sst_id + 1, ... (Compact::DoCompactJob's
 * GetNextSSTId() sequence).  Output files are created, or -- when the path
 * exists -- opened without truncation as io/linux_file.cc:99-119 does (a longer
 * stale file keeps its tail); fsync when do_fsync (TableBuilder::Finish does).  Per output: id, GetFileSize() and the
 * smallest / largest key copied into key_arena (what VersionEdit::AddNewFiles
 * records).  timing may be NULL. */
int sstc_compact_files(sstc_pipe *pipe, const char *const *in_paths, const uint64_t *in_file_sizes,
                       uint32_t n_in, const char *out_prefix, uint64_t first_sst_id,
                       const sstc_compact_params *params, uint32_t do_fsync, sstc_file_out *outs,
                       uint32_t max_outs, uint32_t *n_out, uint8_t *key_arena, uint64_t key_arena_cap,
                       sstc_files_timing *timing);

/* In-process multi-device compaction (the engine's one
 * compaction job, db/db_impl.cc:548,553-598, spread over the node's GPUs
 * without a process per GPU): n_shards key-range-disjoint input groups, shard s
 * = in_paths[shard_first[s] .. shard_first[s + 1]) (shard_first has
 * n_shards + 1 entries, shard_first[0] = 0), each compacted independently
 * exactly as sstc_compact_files would, shard s by pipes[s % n_pipes] (create
 * one pipe per device, each on a context of its own device) on a host thread
 * of its own per pipe.  No data crosses devices.  Output ids continue from
 * shard to shard: shard 0 takes first_sst_id.., shard s the ids after shard
 * s - 1's last (the GetNextSSTId() sequence of the shards compacted one after
 * another).  The device work of the shards overlaps; their writes do not: a
 * shard writes only once the shard before it has written all of its
 * outputs, and only after max_outs and key_arena_cap hold for the outputs of
 * every shard up to it (checked before any of its files is touched).  outs /
 * key_arena receive the outputs in shard order; timing, when not NULL, has
 * n_shards entries.  A failing shard -- whatever fails: its inputs, its
 * device job, a check above or one of its writes -- fails the call with its
 * error; the shards after it write nothing; the ones before it complete and
 * their outputs are still reported in outs / n_out / key_arena.  The pipes
 * must be distinct (each is used by one thread). */
int sstc_compact_files_multi(sstc_pipe *const *pipes, uint32_t n_pipes, const char *const *in_paths,
                             const uint64_t *in_file_sizes, const uint32_t *shard_first, uint32_t n_shards,
                             const char *out_prefix, uint64_t first_sst_id, const sstc_compact_params *params,
                             uint32_t do_fsync, sstc_file_out *outs, uint32_t max_outs, uint32_t *n_out,
                             uint8_t *key_arena, uint64_t key_arena_cap, sstc_files_timing *timing);

#ifdef __cplusplus
}
#endif
#endif /* SSTCODEC_H */
