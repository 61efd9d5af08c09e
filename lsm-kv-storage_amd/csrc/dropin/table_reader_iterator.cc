// table_reader_iterator.cc — the drop-in kvs::sstable::TableReaderIterator
// (include/dropin/sstable/table_reader_iterator.h), compiled by the ENGINE's
// build in place of /root/reference/sstable/table_reader_iterator.cc, with
// include/dropin/ first and the reference's own headers after it on the
// include path (oracle/Makefile target `dropin`).  It is not part of
// libsstcodec.so, which never sees a reference type: this TU is the thin
// adapter between the engine's TableReader (friend access, table_reader.h:105)
// and the codec's host API (sstc::DecodeBlocks, include/sstc_table.h).
//
// Cursor semantics follow the reference line by line:
//   table_reader_iterator.cc:41-44   IsValid = block cursor in range
//   table_reader_iterator.cc:46-67   Next (entry++, else next block's first)
//   table_reader_iterator.cc:69-90   Prev (entry--, else previous block's last)
//   table_reader_iterator.cc:92-95   Seek (block by largest key, entry 0, the
//                                    block cursor is NOT moved)
//   table_reader_iterator.cc:97-109  SeekToFirst / SeekToLast
//   block_reader_iterator.cc:20-81   entry cursor (uint64_t, wraps) and the
//                                    out-of-range accessor values
// The block caches (table_reader_iterator.cc:125-134) are not consulted:
// compaction never inserts into them (:144-146) and a cached block holds the
// file's bytes, which this iterator decodes whole.
#include "sstable/table_reader_iterator.h"

#include "io/linux_file.h"
#include "sstable/block_index.h"
#include "sstable/lru_table_item.h"
#include "sstable/table_reader.h"
#include "sstc_table.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <span>
#include <stdexcept>
#include <string>

namespace kvs {

namespace sstable {

TableReaderIterator::TableReaderIterator(
    const std::vector<std::unique_ptr<BlockReaderCache>> &block_reader_cache,
    std::shared_ptr<LRUTableItem> lru_table_item)
    : current_block_offset_index_(0), block_reader_cache_(block_reader_cache), lru_table_item_(lru_table_item) {
  table_reader_ = lru_table_item_->GetTableReader();
  assert(table_reader_);
}

// table_reader_iterator.cc:23
TableReaderIterator::~TableReaderIterator() {
  if (map_) munmap(map_, map_len_);
  lru_table_item_->Unref();
}

void TableReaderIterator::Load() {
  if (loaded_) return;
  const bool tr = sstc::TraceHostOn();
  const double t0 = tr ? sstc::TraceNowMs() : 0;
  const std::vector<BlockIndex> &index = table_reader_->block_index_;
  const uint64_t nb = index.size();
  // the data section: every block the meta section lists (table_reader.cc:
  // 220-221 reads them one by one).  Mapped read-only, pages populated in the
  // one call: a read into fresh memory paid a page fault (and the kernel's
  // zeroing) per 4 KiB of the destination, ~180 ms of config 5's 1 GB.  An SST
  // is immutable once written (db_impl.cc:430-436), so the map is its bytes.
  // Fallback: the TableReader's own file object into a pageable buffer
  // (page-locking a fresh buffer per table cost more than the staged copy:
  // config 4's 128 tables, 6.2 s vs 4.6 s per PickCompact).
  uint64_t lo = UINT64_MAX, hi = 0;
  for (const BlockIndex &bi : index) {
    lo = std::min<uint64_t>(lo, bi.GetBlockStartOffset());
    hi = std::max<uint64_t>(hi, bi.GetBlockStartOffset() + bi.GetBlockSize());
  }
  if (nb == 0) lo = hi = 0;
  data_size_ = hi - lo;
  static const bool no_map = std::getenv("SSTC_DROPIN_NO_MAP") != nullptr; // (tests: the read path)
  if (data_size_ && !no_map) {
    const int fd = open(table_reader_->filename_.c_str(), O_RDONLY | O_CLOEXEC);
    struct stat st;
    if (fd >= 0 && fstat(fd, &st) == 0 && static_cast<uint64_t>(st.st_size) >= hi) { // (no page past EOF)
      void *p = mmap(nullptr, hi, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
      if (p != MAP_FAILED) {
        map_ = p;
        map_len_ = hi;
        data_ = static_cast<const uint8_t *>(p) + lo;
      }
    }
    if (fd >= 0) close(fd);
  }
  if (!map_) {
    buf_.reset(new uint8_t[data_size_ ? data_size_ : 1]);
    for (uint64_t done = 0; done < data_size_;) {
      const uint64_t chunk = std::min<uint64_t>(data_size_ - done, 1ull << 30);
      const ssize_t r =
          table_reader_->read_file_object_->RandomRead(std::span<Byte>(buf_.get() + done, chunk), lo + done);
      if (r <= 0)
        throw std::runtime_error("TableReaderIterator: cannot read the data section of " + table_reader_->filename_);
      done += static_cast<uint64_t>(r);
    }
    data_ = buf_.get();
  }
  const double t1 = tr ? sstc::TraceNowMs() : 0;
  std::vector<uint64_t> off(nb), len(nb);
  for (uint64_t b = 0; b < nb; b++) {
    off[b] = index[b].GetBlockStartOffset() - lo;
    len[b] = index[b].GetBlockSize();
  }
  // every block of the table in ONE GPU decode, txn as the reference reads
  // it, the records packed on the GPU into what the accessors read
  sstc::DecodedTable d;
  const int rc = sstc::DecodeTable(sstc::ThreadContext(), data_, data_size_, off.data(), len.data(), nb,
                                   SSTC_TXN_COMPAT, d);
  if (rc != SSTC_OK)
    throw std::runtime_error("TableReaderIterator: GPU decode of " + table_reader_->filename_ +
                             " failed: " + sstc_last_error_string());
  for (uint64_t b = 0; b < nb; b++)
    if (d.status[b] != SSTC_BLK_OK)
      throw std::runtime_error("TableReaderIterator: corrupt block " + std::to_string(b) + " in " +
                               table_reader_->filename_ + " (SSTC_BLK code " + std::to_string(d.status[b]) + ")");
  const double t2 = tr ? sstc::TraceNowMs() : 0;
  rec_ = std::move(d.rec);
  base_ = std::move(d.base);
  loaded_ = true;
  if (tr) {
    sstc::TraceHost(map_ ? "iterator map data section" : "iterator read data section", t1 - t0);
    sstc::TraceHost("iterator GPU decode (H2D, count, decode, pack, D2H)", t2 - t1);
  }
}

void TableReaderIterator::Describe(std::string *path, std::vector<uint64_t> *off, std::vector<uint64_t> *len) const {
  *path = table_reader_->filename_;
  const std::vector<BlockIndex> &index = table_reader_->block_index_;
  off->resize(index.size());
  len->resize(index.size());
  for (size_t b = 0; b < index.size(); b++) {
    (*off)[b] = index[b].GetBlockStartOffset();
    (*len)[b] = index[b].GetBlockSize();
  }
}

void TableReaderIterator::ShowBlock(uint64_t block) {
  has_block_ = true;
  shown_block_ = block;
  shown_first_ = base_[block];
  shown_n_ = base_[block + 1] - base_[block];
}

// block_reader_iterator.cc:30-40
std::string_view TableReaderIterator::GetKey() {
  if (!EntryValid()) return std::string_view{};
  const sstc_record32 &r = rec_[shown_first_ + entry_];
  return {reinterpret_cast<const char *>(data_) + r.key_off, r.key_len};
}

// block_reader_iterator.cc:42-52 + block_reader.cc:84-102: a DELETE has no
// value (null view), a PUT a view into the block even when empty
std::string_view TableReaderIterator::GetValue() {
  if (!EntryValid()) return std::string_view{};
  const sstc_record32 &r = rec_[shown_first_ + entry_];
  if (r.type == static_cast<uint8_t>(db::ValueType::DELETED) || r.val_len == SSTC_NO_VALUE)
    return std::string_view{};
  return {reinterpret_cast<const char *>(data_) + r.key_off + r.val_rel, r.val_len};
}

// block_reader_iterator.cc:54-61
db::ValueType TableReaderIterator::GetType() {
  if (!EntryValid()) return db::ValueType::NOT_FOUND;
  return static_cast<db::ValueType>(rec_[shown_first_ + entry_].type);
}

// block_reader_iterator.cc:63-71 (compat txn: block_reader.cc:104-114)
TxnId TableReaderIterator::GetTransactionId() {
  if (!EntryValid()) return INVALID_TXN_ID;
  return rec_[shown_first_ + entry_].txn;
}

// table_reader_iterator.cc:41-44
bool TableReaderIterator::IsValid() {
  return current_block_offset_index_ < table_reader_->block_index_.size();
}

// table_reader_iterator.cc:46-67
void TableReaderIterator::Next() {
  if (!has_block_) return;
  entry_++;
  if (EntryValid()) return;
  current_block_offset_index_++;
  if (!IsValid()) return;
  ShowBlock(current_block_offset_index_);
  entry_ = 0;
}

// table_reader_iterator.cc:69-90
void TableReaderIterator::Prev() {
  if (!has_block_) return;
  entry_--;
  if (EntryValid()) return;
  current_block_offset_index_--;
  if (!IsValid()) return;
  ShowBlock(current_block_offset_index_);
  entry_ = shown_n_ - 1;
}

// table_reader_iterator.cc:92-95 with TableReader::GetBlockOffsetAndSize
// (table_reader.cc:191-210): the block with the smallest largest key >= key
// (the last block when none is), entry cursor at 0; the block cursor stays
void TableReaderIterator::Seek(std::string_view key) {
  Load();
  const std::vector<BlockIndex> &index = table_reader_->block_index_;
  int64_t left = 0;
  int64_t right = static_cast<int64_t>(index.size()) - 1;
  while (left < right) {
    const int64_t mid = left + (right - left) / 2;
    if (index[mid].GetLargestKey() >= key) right = mid;
    else left = mid + 1;
  }
  if (right < 0) return; // no block (the reference indexes block_index_[-1])
  ShowBlock(static_cast<uint64_t>(right));
  entry_ = 0;
}

// table_reader_iterator.cc:97-102
void TableReaderIterator::SeekToFirst() {
  Load();
  current_block_offset_index_ = 0;
  if (!IsValid()) return; // empty table (the reference indexes block_index_[0])
  ShowBlock(current_block_offset_index_);
  entry_ = 0;
}

// table_reader_iterator.cc:104-109
void TableReaderIterator::SeekToLast() {
  Load();
  current_block_offset_index_ = table_reader_->block_index_.size() - 1;
  if (!IsValid()) return;
  ShowBlock(current_block_offset_index_);
  entry_ = shown_n_ - 1;
}

} // namespace sstable

} // namespace kvs
