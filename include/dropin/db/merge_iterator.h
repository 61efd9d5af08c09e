/*
 * include/dropin/db/merge_iterator.h — the drop-in for the reference's
 * db/merge_iterator.h (/root/reference/db/merge_iterator.h:22-118).
 *
 * With include/dropin/ first on the include path and
 * lsm-kv-storage_amd/csrc/dropin/merge_iterator.cc compiled in place of the
 * reference's db/merge_iterator.cc, db/compact.cc builds UNCHANGED:
 * Compact::CreateMergeIterator (compact.cc:186-230) hands its
 * TableReaderIterators to this class and DoCompactJob walks it
 * (compact.cc:254-302).  Same class, base, constructor, include guard.
 *
 * SeekToFirst (the walk compaction makes) runs on the GPU: the inputs' data
 * sections are mapped into one host range, uploaded once, decoded and merged
 * on the device (sstc::ResidentInputs, sstc_merge_records), and the merged
 * order -- 16 B per record, key offset + txn as read -- comes back in one
 * copy.  Next / IsValid / the accessors then walk that array: no heap, no
 * per-record virtual hop into a table iterator.  Views point into the mapped
 * inputs and stay valid for this iterator's life (and for any TableBuilder
 * holding records of it), so compact.cc:250's last_current_key never
 * dangles.  While it lives, the region is this thread's active resident
 * inputs: a TableBuilder handed these views keeps offsets instead of copying
 * the bytes and encodes its blocks from the device copy.
 *
 * The reference's own semantics, kept exactly (merge_iterator.cc:14-108):
 *   - order: key ascending, txn descending (LessCompare, merge_iterator.h:
 *     91-95); a table's versions of a key as its iterator returns them (the
 *     compat txn of block_reader.cc:109-111 can put them out of txn order)
 *     pop exactly as the heap pops them;
 *   - equal (key, txn) from different tables: the heap orders them by its
 *     history.  When the device finds such a tie whose records differ (never
 *     in what the engine writes: identical copies give the same bytes in any
 *     order), and whenever the inputs are not something the device path takes
 *     (a table without blocks -- the reference pushes its invalid iterator --,
 *     a corrupt block, keys out of order), the iterator runs the reference's
 *     two heaps over the TableReaderIterators instead (heap mode): same
 *     std::priority_queue, same comparators, same push / pop sequence;
 *   - IsValid() is the MIN heap's non-emptiness, also after SeekToLast; Prev
 *     pops the MAX heap filled by SeekToLast; accessors read the min heap's
 *     top.  Any call other than SeekToFirst / Next / IsValid / the accessors
 *     after a device walk first replays the walk on the heaps (SeekToFirst +
 *     the same number of Next calls), so mixed sequences see the reference's
 *     state -- compaction never makes one.
 *   - past the end of a device walk the accessors return what an exhausted
 *     table iterator returns (empty view, NOT_FOUND, INVALID_TXN_ID) where the
 *     reference reads the top of an empty heap.
 *
 * Errors: the iterator throws std::runtime_error where the drop-in
 * TableReaderIterator does (a table that cannot be read, a corrupt block).
 */
#ifndef DB_MERGE_ITERATOR_H
#define DB_MERGE_ITERATOR_H

#include "common/base_iterator.h"
#include "common/macros.h"
#include "sstc_table.h"

// libC++
#include <cassert>
#include <cstring>
#include <memory>
#include <queue>
#include <string>
#include <vector>

namespace kvs {

namespace sstable {
class TableReaderIterator;
}

namespace db {

class MergeIterator final : public kvs::BaseIterator {
public:
  MergeIterator(std::vector<std::unique_ptr<sstable::TableReaderIterator>>
                    table_reader_iterators);

  ~MergeIterator();

  // No copy allowed
  MergeIterator(const MergeIterator &) = delete;
  MergeIterator &operator=(MergeIterator &) = delete;

  // Move constructor/assignment
  MergeIterator(MergeIterator &&) = default;
  MergeIterator &operator=(MergeIterator &&) = default;

  // Return the smallest key(which is the top of min heap)
  std::string_view GetKey() override {
    if (OnDevice()) return {Key(), KeyLen()};
    return HeapGetKey();
  }

  // Return value of smallest key
  std::string_view GetValue() override {
    if (OnDevice()) {
      const uint32_t kl = KeyLen();
      if (Key()[-5] == static_cast<char>(db::ValueType::DELETED)) return std::string_view{};
      uint32_t vl;
      std::memcpy(&vl, Key() + kl, 4);
      return {Key() + kl + 4, vl};
    }
    return HeapGetValue();
  }

  // Return type of smallest key
  db::ValueType GetType() override {
    if (OnDevice()) return static_cast<db::ValueType>(Key()[-5]);
    return HeapGetType();
  }

  // Return transaction id of smallest key
  TxnId GetTransactionId() override {
    if (OnDevice()) return rec_[pos_].txn;
    return HeapGetTransactionId();
  }

  bool IsValid() override { return device_ ? pos_ < n_ : !min_heap_.empty(); }

  // Get table iterator that have, currently, the smallest key then move it
  // forward
  void Next() override {
    if (device_) {
      if (pos_ + ahead_ < avail_) { // the entry ahead_ records on: its header + key lines, ahead of the loop
        const char *e = reinterpret_cast<const char *>(base_) + rec_[pos_ + ahead_].key_off;
        __builtin_prefetch(e - 5);
        __builtin_prefetch(e + 24);
      }
      if (++pos_ >= avail_) WaitRecords();
      return;
    }
    HeapNext();
  }

  // Get table iterator that have, currently, the smallest key then move it
  // backward
  void Prev() override;

  // Jump  to and load first block in table
  void Seek(std::string_view key) override;

  void SeekToFirst() override;

  void SeekToLast() override;

private:
  struct HeapItem {
    HeapItem(std::string_view key_item, TxnId txn_id_item,
             sstable::TableReaderIterator *iterator_item)
        : key(key_item), txn_id(txn_id_item), iterator(iterator_item) {}

    std::string_view key;

    TxnId txn_id;

    sstable::TableReaderIterator *iterator;
  };

  // min heap: smallest key first, for equal keys the largest txn
  struct LessCompare {
    bool operator()(const HeapItem &a, const HeapItem &b) {
      return a.key > b.key || (a.key == b.key && a.txn_id < b.txn_id);
    }
  };

  // max heap: largest key first, for equal keys the smallest txn
  struct GreaterCompare {
    bool operator()(const HeapItem &a, const HeapItem &b) {
      return a.key < b.key || (a.key == b.key && a.txn_id > b.txn_id);
    }
  };

  // the device walk: record pos_ of the merged order.  The merged records
  // arrive in chunks (ResidentInputs downloads them behind the walk): records
  // [0, avail_) are in host memory.  The merged order interleaves the tables'
  // entries (128 tables in BASELINE config 4), so the walk prefetches the
  // entry ahead_ records ahead instead of waiting on one cache miss per record.
  uint64_t ahead_ = 24;
  bool OnDevice() const { return device_ && pos_ < n_; }
  // pos_ past the records that have arrived: wait for more (pos_ <= n_)
  void WaitRecords();
  const char *Key() const { return reinterpret_cast<const char *>(base_) + rec_[pos_].key_off; }
  uint32_t KeyLen() const {
    uint32_t kl;
    std::memcpy(&kl, Key() - 4, 4);
    return kl;
  }
  // leave the device walk for the heaps (replays it; see the header comment)
  void LeaveDevice();
  // merge_iterator.cc:14-108 on the heaps
  std::string_view HeapGetKey();
  std::string_view HeapGetValue();
  db::ValueType HeapGetType();
  TxnId HeapGetTransactionId();
  void HeapNext();
  void HeapSeekToFirst();

  std::vector<std::unique_ptr<sstable::TableReaderIterator>>
      table_reader_iterators_;

  size_t num_iterators_;

  // Min heap for forward traverse
  std::priority_queue<HeapItem, std::vector<HeapItem>, LessCompare> min_heap_;

  // Max heap for backward traverse
  std::priority_queue<HeapItem, std::vector<HeapItem>, GreaterCompare>
      max_heap_;

  // device walk state
  bool device_tried_ = false; // (the merged order is made once: the inputs are immutable)
  bool device_ = false;
  uint64_t pos_ = 0, n_ = 0, avail_ = 0;
  const uint8_t *base_ = nullptr;
  const sstc_merged_record *rec_ = nullptr;
  std::shared_ptr<sstc::ResidentInputs> resident_;
  double t_first_ = 0; // (SSTC_TRACE_HOST: when the device walk began)
};

} // namespace db

} // namespace kvs

#endif // DB_MERGE_ITERATOR_H
