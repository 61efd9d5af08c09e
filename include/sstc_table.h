/*
 * sstc_table.h — host C++ mirror of the reference's SST table API over the
 * codec C-ABI (include/sstcodec.h), plus a C shim for other language bindings.
 *
 *   sstc::TableBuilder  mirrors kvs::sstable::TableBuilder
 *                       (reference sstable/table_builder.h:63-151): AddEntry
 *                       tracks the block boundaries exactly as the reference
 *                       (table_builder.cc:35-60); Finish encodes every data
 *                       block on the GPU (sstc_encode_blocks), appends the meta
 *                       section and the 40 B footer (table_builder.cc:101-211)
 *                       and writes the file with one pwrite + fsync instead of
 *                       three pwrite64 per block.
 *   sstc::TableReader   mirrors CreateAndSetupDataForTableReader /
 *                       DecodeExtraInfo / FetchBlockIndexInfo
 *                       (table_reader.cc:32-156) and replaces the per-block
 *                       CreateAndSetupDataForBlockReader (:212-241) by one
 *                       batched GPU decode of every block.
 *
 *   sstc::BlockReader / TableReader::CreateAndSetupDataForBlockReader(s)
 *                       the decoded records of one data block
 *                       (block_reader.h:24-45,104-119, table_reader.h:99-101);
 *                       the batched form decodes many blocks in one GPU call.
 *   sstc::TableReaderIterator
 *                       the record stream of table_reader_iterator.cc:46-149
 *                       (SeekToFirst / Next / Prev / Seek / accessors) over the
 *                       whole table decoded in one GPU call.
 *
 * Drop-in surface: TableBuilder(std::string&&, const Config*) takes any config
 * type with GetSSTBlockSize() (db/config.h) and uses the calling thread's
 * context (ThreadContext()), and AddEntry accepts the engine's own
 * db::ValueType (any enum with PUT = 0 / DELETED = 1), so db/compact.cc and
 * db/db_impl.cc compile unchanged against `namespace kvs::sstable { using
 * TableBuilder = ::sstc::TableBuilder; }`.
 *
 * Error behaviour follows the reference: Open() returns false, Finish() throws
 * std::runtime_error, CreateAndSetupDataForBlockReader returns nullptr on a
 * read failure; the C shim returns SSTC_* codes instead.
 */
#ifndef SSTC_TABLE_H
#define SSTC_TABLE_H

#include "sstcodec.h"

#ifdef __cplusplus
#include <atomic>
#include <cstdint>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <string_view>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

namespace sstc {

/* db/status.h:11-19, common/macros.h */
enum class ValueType : uint8_t { PUT = 0, DELETED = 1, NOT_FOUND = 2, kTooManyOpenFiles = 3 };
using TxnId = uint64_t;
using BlockOffset = uint64_t;
using BlockSize = uint64_t;

/* The calling host thread's context on the current HIP device, created on
 * first use and destroyed at thread exit (the reference builds / reads SSTs
 * from pool threads, one TableBuilder per thread: db/db_impl.cc:354-362). */
sstc_ctx *ThreadContext();

/* Page-locked buffers a HostVec outgrew: hipHostFree synchronises the whole
 * device, so a builder that grows its arrays during AddEntry hands the old
 * ones here and they are freed at the end of the thread's next Finish() (which
 * synchronises its own stream anyway) or at thread exit, never between two
 * AddEntry calls while other threads' builders run. */
void DeferHostFree(void *p, int pinned);
void FlushDeferredHostFrees();

/* SSTC_TRACE_HOST=1 in the environment: phase times of the host-side paths
 * on stderr (diagnostics; off by default) */
bool TraceHostOn();
double TraceNowMs();
void TraceHost(const char *what, double ms);

/* Growable host array for the builder's pending records: storage from
 * sstc_host_alloc (pinned, so Finish() copies it to the GPU without a pack
 * copy; pageable when pinning fails).  A TableBuilder takes its arrays from a
 * per-thread pool and returns them with their capacity, so a thread that
 * builds many SSTs appends into memory that is already pinned and faulted in. */
template <class T> class HostVec {
public:
  HostVec() = default;
  HostVec(const HostVec &) = delete;
  HostVec &operator=(const HostVec &) = delete;
  ~HostVec() {
    if (p_) sstc_host_free(p_, pinned_);
  }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  T *data() { return p_; }
  const T *data() const { return p_; }
  T &operator[](size_t i) { return p_[i]; }
  const T &operator[](size_t i) const { return p_[i]; }
  T &back() { return p_[n_ - 1]; }
  const T &back() const { return p_[n_ - 1]; }
  void clear() { n_ = 0; }
  void reserve(size_t c) {
    if (c > cap_) grow(c);
  }
  void push_back(T v) {
    if (n_ == cap_) grow(cap_ ? 2 * cap_ : 4096);
    p_[n_++] = v;
  }
  void append(const T *src, size_t k) {
    if (n_ + k > cap_) grow(n_ + k > 2 * cap_ ? n_ + k : 2 * cap_);
    if (k) std::memcpy(p_ + n_, src, k * sizeof(T));
    n_ += k;
  }

private:
  void grow(size_t c) {
    int pinned = 0;
    T *q = static_cast<T *>(sstc_host_alloc(c * sizeof(T), &pinned));
    if (!q) throw std::bad_alloc();
    if (n_) std::memcpy(q, p_, n_ * sizeof(T));
    if (p_) DeferHostFree(p_, pinned_);
    p_ = q;
    cap_ = c;
    pinned_ = pinned;
  }
  T *p_ = nullptr;
  size_t n_ = 0, cap_ = 0;
  int pinned_ = 0;
};

/* one TableBuilder's pending records (sst_table.cpp keeps a per-thread pool) */
struct BuilderArena;

/* The inputs of one merge (a compaction's input SSTs, db/compact.cc:186-230)
 * made resident for the drop-in MergeIterator (include/dropin/db/
 * merge_iterator.h): every input's data section is mapped read-only into ONE
 * host address range, uploaded once to the device at the same offsets, and
 * its records decoded and merged there (sstc_merge_records) into the order
 * the reference's MergeIterator walks them.  Host views (keys, values) point
 * into the mapping; offsets are the same on both sides, so a TableBuilder on
 * the same thread that is handed such views records (offset) instead of
 * copying bytes and encodes its blocks from the device copy (Activate). */
class ResidentInputs : public std::enable_shared_from_this<ResidentInputs> {
public:
  struct Input {                      // one input table, iterator order
    std::string path;                 // its SST file
    std::vector<uint64_t> off, len;   // its data blocks (BlockIndex order), file offsets
  };
  /* Map, upload, decode + merge (txn as the reference's iterator reads it).
   * nullptr when the merged order cannot be produced on the device (a file
   * that cannot be mapped, a table without blocks, a corrupt block, keys out
   * of order, no HIP device); *why says which. */
  static std::shared_ptr<ResidentInputs> Create(sstc_ctx *ctx, const std::vector<Input> &inputs, uint32_t txn_mode,
                                                std::string *why);
  ~ResidentInputs();
  ResidentInputs(const ResidentInputs &) = delete;
  ResidentInputs &operator=(const ResidentInputs &) = delete;

  uint64_t NumRecords() const { return n_; }
  /* the merged records, downloaded in chunks behind the caller's walk by a
   * helper thread: Records()[0, WaitRecords(k)) are in host memory, and
   * WaitRecords(k) returns >= min(k, NumRecords()) (throws std::runtime_error
   * when the download failed) */
  const sstc_merged_record *Records() const { return rec_.get(); }
  uint64_t WaitRecords(uint64_t k);
  const uint8_t *Host() const { return host_; }
  uint64_t Bytes() const { return bytes_; }
  const uint8_t *DeviceBytes() const { return dev_; }
  int Device() const { return device_; }
  /* runs of equal (key, merge txn) records spanning inputs / those whose
   * records differ (sstc_merge_result): TieDiffs() > 0 = the reference heap's
   * order may give other bytes */
  uint64_t CrossTies() const { return cross_ties_; }
  uint64_t TieDiffs() const { return tie_diffs_; }
  /* the input a record's key lies in */
  uint32_t InputOf(uint64_t key_off) const;
  /* host-side phase times of Create (ms): waits for the maps, maps + uploads,
   * device merge, download start */
  double ms[4] = {0, 0, 0, 0};

  /* TableBuilders on the calling thread may reference this region from now
   * until Deactivate (the drop-in MergeIterator activates it for its life) */
  void Activate();
  void Deactivate();
  static ResidentInputs *Active(); /* the calling thread's, or nullptr */

private:
  ResidentInputs() = default;
  uint8_t *host_ = nullptr;   // reserved range (PROT_NONE) with the files mapped in it
  uint64_t bytes_ = 0;
  uint8_t *dev_ = nullptr;    // device copy, same offsets
  int device_ = -1;
  uint64_t n_ = 0, cross_ties_ = 0, tie_diffs_ = 0;
  std::unique_ptr<sstc_merged_record[]> rec_;
  std::vector<uint64_t> table_base_; // offset of table t's file in the range
  // the download: device records (the creating thread's merge buffer, lent to
  // this object until the helper is done), records ready, failure flag
  void Download();
  void *drec_ = nullptr;
  uint64_t drec_cap_ = 0;
  std::atomic<uint64_t> ready_{0};
  std::atomic<int> failed_{0};
  std::thread helper_;
};

/* One meta entry (reference sstable/block_index.h:22-57). */
struct BlockIndex {
  std::string smallest_key;
  std::string largest_key;
  uint64_t offset = 0;
  uint64_t size = 0;
};

class TableBuilder {
public:
  /* block_threshold = Config::GetSSTBlockSize() (config/config.toml:11). */
  TableBuilder(std::string filename, uint64_t block_threshold, sstc_ctx *ctx);
  /* table_builder.h:65: TableBuilder(std::string &&, const db::Config *) */
  template <class Config, class = decltype(std::declval<const Config *>()->GetSSTBlockSize())>
  TableBuilder(std::string &&filename, const Config *config)
      : TableBuilder(std::move(filename), static_cast<uint64_t>(config->GetSSTBlockSize()), ThreadContext()) {}
  ~TableBuilder();
  TableBuilder(const TableBuilder &) = delete;
  TableBuilder &operator=(const TableBuilder &) = delete;

  bool Open();
  /* value.data() == nullptr -> no value fields (a DELETE), like the reference. */
  void AddEntry(std::string_view key, std::string_view value, uint64_t txn_id, uint8_t value_type);
  /* table_builder.h:81: AddEntry(string_view, string_view, TxnId, db::ValueType) */
  template <class VT, class = std::enable_if_t<std::is_enum_v<VT>>>
  void AddEntry(std::string_view key, std::string_view value, TxnId txn_id, VT value_type) {
    AddEntry(key, value, txn_id, static_cast<uint8_t>(value_type));
  }
  void FlushBlock();
  void Finish();
  /* n records from SoA arrays (val_len[i] == SSTC_NO_VALUE: no value fields),
   * the same as n AddEntry calls */
  void AddEntries(uint64_t n, const uint8_t *type, const uint32_t *key_len, const uint32_t *val_len,
                  const uint64_t *txn, const uint8_t *key_src, const uint64_t *key_off, const uint8_t *val_src,
                  const uint64_t *val_off);

  std::string_view GetSmallestKey() const { return table_smallest_key_; }
  /* the last key added (a view into the builder's key arena or the resident
   * inputs; no string copy per AddEntry, the reference's #1 host hotspot,
   * table_builder.cc:37-53) */
  std::string_view GetLargestKey() const {
    if (type_.empty()) return {};
    return {reinterpret_cast<const char *>(KeyPtr(type_.size() - 1)), key_len_.back()};
  }
  std::string_view GetFilename() const { return filename_; }
  uint64_t GetFileSize() const { return current_offset_ + 1; } /* table_builder.cc:228 */
  uint64_t GetDataSize() const { return data_size_; }
  uint64_t GetNumBlocks() const { return blk_first_.size() - 1; }

private:
  std::string filename_;
  uint64_t threshold_;
  sstc_ctx *ctx_;
  int fd_ = -1;
  // pending records (host SoA + arenas), borrowed from the thread's pool
  BuilderArena *arena_;
  HostVec<uint8_t> &type_;
  HostVec<uint32_t> &key_len_, &val_len_;
  HostVec<uint64_t> &txn_, &key_off_, &val_off_;
  HostVec<uint8_t> &keys_, &vals_;
  HostVec<uint64_t> &blk_first_;
  uint64_t block_size_ = 0; /* sum(entry_size + 16) of the open block */
  std::string table_smallest_key_;
  uint64_t min_txn_ = UINT64_MAX, max_txn_ = 0;
  uint64_t data_size_ = 0;
  uint64_t current_offset_ = 0;
  /* Resident inputs (ResidentInputs::Activate on this thread, same device as
   * ctx_): a record whose key and value views lie in them is kept as offsets
   * into them (no copy; Finish encodes from the device copy); one that does not
   * is copied into the arenas with kArenaRef in its offsets. */
  static constexpr uint64_t kArenaRef = 1ull << 63;
  std::shared_ptr<ResidentInputs> res_;
  const uint8_t *res_host_ = nullptr;
  uint64_t res_bytes_ = 0, arena_recs_ = 0;
  bool AdoptResident();
  const uint8_t *KeyPtr(size_t i) const {
    const uint64_t o = key_off_[i];
    return res_host_ && !(o & kArenaRef) ? res_host_ + o : keys_.data() + (o & ~kArenaRef);
  }
  const uint8_t *ValPtr(size_t i) const {
    const uint64_t o = val_off_[i];
    return res_host_ && !(o & kArenaRef) ? res_host_ + o : vals_.data() + (o & ~kArenaRef);
  }
};

/* The records of one data block, decoded on the GPU (BlockReaderData +
 * BlockReader accessors, block_reader.h:24-45,104-119, block_reader.cc:59-114).
 * Views point into the block bytes the reader owns.  GetValue of a DELETE is
 * a null view (value.data() == nullptr), of a PUT a non-null view even when
 * empty, so AddEntry(GetKey(i), GetValue(i), ...) re-encodes exactly. */
class BlockReader {
public:
  uint64_t NumEntries() const { return type_.size(); }
  ValueType GetType(uint64_t i) const { return static_cast<ValueType>(type_[i]); }
  std::string_view GetKey(uint64_t i) const {
    return {reinterpret_cast<const char *>(buf_.data()) + key_off_[i], key_len_[i]};
  }
  std::string_view GetValue(uint64_t i) const {
    if (val_len_[i] == SSTC_NO_VALUE) return {};
    return {reinterpret_cast<const char *>(buf_.data()) + val_off_[i], val_len_[i]};
  }
  TxnId GetTransactionId(uint64_t i) const { return txn_[i]; }
  int Status() const { return status_; } /* SSTC_BLK_* of this block */

private:
  friend class TableReader;
  std::vector<uint8_t> buf_; /* the block's bytes */
  std::vector<uint8_t> type_;
  std::vector<uint32_t> key_len_, val_len_;
  std::vector<uint64_t> txn_, key_off_, val_off_;
  int status_ = SSTC_BLK_OK;
};

class TableReader {
public:
  /* file_size as recorded by TableBuilder::GetFileSize() (bytes + 1). */
  static TableReader *Open(const std::string &filename, uint64_t file_size, sstc_ctx *ctx);
  /* CreateAndSetupDataForTableReader(std::string&&, SSTId, uint64_t) on the
   * calling thread's context (table_reader.h:134-136); nullptr on failure. */
  static std::unique_ptr<TableReader> Create(std::string &&filename, uint64_t table_id, uint64_t file_size) {
    (void)table_id;
    return std::unique_ptr<TableReader>(Open(filename, file_size, ThreadContext()));
  }
  ~TableReader();

  /* table_reader.h:99-101: pread one block and decode it (one GPU call). */
  std::unique_ptr<BlockReader> CreateAndSetupDataForBlockReader(BlockOffset offset, uint64_t block_size,
                                                               uint32_t txn_mode = SSTC_TXN_COMPAT) const;
  /* The same for many blocks with ONE decode call (what compaction and scans
   * want: every block of a table at once).  Entries are nullptr for blocks
   * that could not be read. */
  std::vector<std::unique_ptr<BlockReader>> CreateAndSetupDataForBlockReaders(
      const std::vector<std::pair<BlockOffset, uint64_t>> &blocks, uint32_t txn_mode = SSTC_TXN_COMPAT) const;
  uint64_t GetFileSize() const { return bytes_ + 1; }

  const std::vector<BlockIndex> &GetBlockIndex() const { return index_; }
  uint64_t GetMinTxn() const { return min_txn_; }
  uint64_t GetMaxTxn() const { return max_txn_; }
  /* Read the data section and decode every block on the GPU into a host
   * record table (offsets into the returned data bytes).  Returns the block
   * status of the first failing block, or SSTC_BLK_OK. */
  int DecodeAll(uint32_t txn_mode, std::vector<uint8_t> &data, std::vector<uint8_t> &type,
                std::vector<uint32_t> &key_len, std::vector<uint32_t> &val_len, std::vector<uint64_t> &txn,
                std::vector<uint64_t> &key_off, std::vector<uint64_t> &val_off);

private:
  TableReader() = default;
  int fd_ = -1;
  sstc_ctx *ctx_ = nullptr;
  uint64_t bytes_ = 0, meta_off_ = 0;
  uint64_t min_txn_ = 0, max_txn_ = 0;
  std::vector<BlockIndex> index_;
};

/* The records of many blocks decoded in ONE GPU call (sstc_count_records +
 * sstc_decode_blocks through `ctx`): block b's records are
 * [base[b], base[b+1]), offsets point into the host bytes that were decoded,
 * val_len == SSTC_NO_VALUE marks a record without value fields (a DELETE),
 * status[b] is the block's SSTC_BLK_* code. */
struct DecodedBlocks {
  std::vector<uint64_t> base;
  std::vector<uint32_t> status;
  std::vector<uint8_t> type;
  std::vector<uint32_t> key_len, val_len;
  std::vector<uint64_t> txn, key_off, val_off;
};
/* blocks (off[b], len[b]) inside data[0, bytes); SSTC_OK or a negative
 * SSTC_E_* code (bad arguments, HIP failure) */
int DecodeBlocks(sstc_ctx *ctx, const uint8_t *data, uint64_t bytes, const uint64_t *off, const uint64_t *len,
                 uint64_t nb, uint32_t txn_mode, DecodedBlocks &out);

/* The same decode with the records packed on the GPU (sstc_pack_records) and
 * copied back in one piece: 32 B per record instead of six columns, no host
 * repacking.  What the drop-in kvs::sstable::TableReaderIterator serves its
 * entries from. */
struct DecodedTable {
  std::vector<uint64_t> base;            // nb + 1: block b's records are [base[b], base[b + 1])
  std::vector<uint32_t> status;          // SSTC_BLK_* per block
  std::unique_ptr<sstc_record32[]> rec;  // n records
  uint64_t n = 0;
};
int DecodeTable(sstc_ctx *ctx, const uint8_t *data, uint64_t bytes, const uint64_t *off, const uint64_t *len,
                uint64_t nb, uint32_t txn_mode, DecodedTable &out);

/* table_reader_iterator.cc:46-149 over a table decoded whole on the GPU at the
 * first Seek (one sstc_count_records + sstc_decode_blocks call instead of a
 * pread and a BlockReader per block). */
class TableReaderIterator {
public:
  explicit TableReaderIterator(TableReader *table, uint32_t txn_mode = SSTC_TXN_COMPAT)
      : table_(table), txn_mode_(txn_mode) {}
  bool IsValid() const { return pos_ < n_; }
  void SeekToFirst() {
    Load();
    pos_ = 0;
  }
  void SeekToLast() {
    Load();
    pos_ = n_ ? n_ - 1 : n_;
  }
  /* first entry whose key is >= key (block_reader_iterator.cc:84-119) */
  void Seek(std::string_view key);
  void Next() {
    if (pos_ < n_) pos_++;
  }
  void Prev() { pos_ = pos_ == 0 || pos_ >= n_ ? n_ : pos_ - 1; }
  std::string_view GetKey() const {
    return {reinterpret_cast<const char *>(data_.data()) + key_off_[pos_], key_len_[pos_]};
  }
  std::string_view GetValue() const {
    if (val_len_[pos_] == SSTC_NO_VALUE) return {};
    return {reinterpret_cast<const char *>(data_.data()) + val_off_[pos_], val_len_[pos_]};
  }
  ValueType GetType() const { return static_cast<ValueType>(type_[pos_]); }
  TxnId GetTransactionId() const { return txn_[pos_]; }
  int Status() const { return status_; } /* first failing block's SSTC_BLK_* code */

private:
  void Load();
  TableReader *table_;
  uint32_t txn_mode_;
  bool loaded_ = false;
  int status_ = SSTC_BLK_OK;
  uint64_t pos_ = 0, n_ = 0;
  std::vector<uint8_t> data_, type_;
  std::vector<uint32_t> key_len_, val_len_;
  std::vector<uint64_t> txn_, key_off_, val_off_;
};

} // namespace sstc
#endif /* __cplusplus */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sstc_table_builder sstc_table_builder;
typedef struct sstc_table_reader sstc_table_reader;

int sstc_tb_create(const char *path, uint64_t block_threshold, sstc_ctx *ctx, sstc_table_builder **out);
int sstc_tb_open(sstc_table_builder *tb);
/* val == NULL -> no value fields (DELETE). */
int sstc_tb_add(sstc_table_builder *tb, const uint8_t *key, uint32_t key_len, const uint8_t *val,
                uint32_t val_len, uint64_t txn, uint8_t type);
/* n records from host arrays (val_len[i] == SSTC_NO_VALUE -> no value fields). */
int sstc_tb_add_batch(sstc_table_builder *tb, uint64_t n, const uint8_t *type, const uint32_t *key_len,
                      const uint32_t *val_len, const uint64_t *txn, const uint8_t *key_src,
                      const uint64_t *key_off, const uint8_t *val_src, const uint64_t *val_off);
int sstc_tb_finish(sstc_table_builder *tb);
uint64_t sstc_tb_file_size(const sstc_table_builder *tb);
uint64_t sstc_tb_num_blocks(const sstc_table_builder *tb);
int sstc_tb_destroy(sstc_table_builder *tb);

int sstc_tr_open(const char *path, uint64_t file_size, sstc_ctx *ctx, sstc_table_reader **out);
uint64_t sstc_tr_num_blocks(const sstc_table_reader *tr);
int sstc_tr_block_index(const sstc_table_reader *tr, uint64_t *blk_off, uint64_t *blk_len);
uint64_t sstc_tr_num_records(sstc_table_reader *tr, uint32_t txn_mode);
/* Outputs sized by sstc_tr_num_records; offsets point into the file. */
int sstc_tr_decode_all(sstc_table_reader *tr, uint32_t txn_mode, uint8_t *type, uint32_t *key_len,
                       uint32_t *val_len, uint64_t *txn, uint64_t *key_off, uint64_t *val_off);
int sstc_tr_destroy(sstc_table_reader *tr);

#ifdef __cplusplus
}
#endif
#endif /* SSTC_TABLE_H */
