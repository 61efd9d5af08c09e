// merge_iterator.cc — the drop-in kvs::db::MergeIterator
// (include/dropin/db/merge_iterator.h), compiled by the ENGINE's build in
// place of /root/reference/db/merge_iterator.cc (oracle/Makefile target
// `dropin`).  Like table_reader_iterator.cc it is a thin adapter: the device
// merge lives in libsstcodec (sstc::ResidentInputs, sstc_merge_records).
//
// Heap mode restates merge_iterator.cc:14-108: the same two
// std::priority_queue<HeapItem> with the same comparators, pushed and popped
// in the same sequence, over the same (drop-in) TableReaderIterators.
#include "db/merge_iterator.h"

#include "sstable/table_reader_iterator.h"
#include "sstc_table.h"

#include <cstdio>
#include <cstdlib>
#include <string>
#include <utility>

namespace kvs {

namespace db {

MergeIterator::MergeIterator(
    std::vector<std::unique_ptr<sstable::TableReaderIterator>>
        table_reader_iterators)
    : table_reader_iterators_(std::move(table_reader_iterators)),
      num_iterators_(table_reader_iterators_.size()) {}

MergeIterator::~MergeIterator() {
  if (resident_) resident_->Deactivate();
  if (t_first_ > 0)
    sstc::TraceHost("MergeIterator life after the device merge (the caller's loop incl. its Finish calls)",
                    sstc::TraceNowMs() - t_first_);
}

// SeekToFirst (merge_iterator.cc:79-92): the merged order of every record of
// every table, made on the device once per iterator
void MergeIterator::SeekToFirst() {
  static const bool heap_only = std::getenv("SSTC_DROPIN_HEAP_MERGE") != nullptr; // (tests: the heap mode)
  if (!resident_ && !device_tried_ && !heap_only) {
    device_tried_ = true;
    std::vector<sstc::ResidentInputs::Input> in(num_iterators_);
    for (size_t t = 0; t < num_iterators_; t++)
      table_reader_iterators_[t]->Describe(&in[t].path, &in[t].off, &in[t].len);
    std::string why;
    std::shared_ptr<sstc::ResidentInputs> r =
        num_iterators_ ? sstc::ResidentInputs::Create(sstc::ThreadContext(), in, SSTC_TXN_COMPAT, &why) : nullptr;
    if (r && r->TieDiffs()) {
      why = "equal (key, txn) records with different contents in different tables: the heap's own order";
      r.reset();
    }
    if (r) {
      resident_ = std::move(r);
      resident_->Activate();
    }
    if (sstc::TraceHostOn())
      std::fprintf(stderr, "[sstc] MergeIterator over %zu tables: %s%s\n", num_iterators_,
                   resident_ ? "device merge" : "heap mode: ", resident_ ? "" : why.c_str());
  }
  if (resident_) {
    if (sstc::TraceHostOn() && t_first_ == 0) t_first_ = sstc::TraceNowMs();
    static const char *pf = std::getenv("SSTC_DROPIN_PF"); // (diagnostics: the prefetch distance)
    if (pf) ahead_ = std::strtoull(pf, nullptr, 10);
    if (!ahead_) ahead_ = ~0ull >> 1;
    device_ = true;
    pos_ = 0;
    avail_ = 0;
    n_ = resident_->NumRecords();
    base_ = resident_->Host();
    rec_ = resident_->Records();
    WaitRecords();
    return;
  }
  HeapSeekToFirst();
}

void MergeIterator::WaitRecords() {
  if (pos_ > n_) pos_ = n_;
  if (pos_ >= n_) return;
  try {
    avail_ = resident_->WaitRecords(pos_ + 1);
  } catch (const std::exception &e) { // the records' download failed: the heaps from here on (the views
                                      // handed out so far stay valid: resident_ lives on)
    std::fprintf(stderr, "[sstc] MergeIterator: %s; heap mode from record %llu\n", e.what(),
                 static_cast<unsigned long long>(pos_));
    LeaveDevice();
  }
}

// ---------------------------------------------------------------- heap mode

void MergeIterator::LeaveDevice() {
  if (!device_) return;
  const uint64_t walked = pos_;
  device_ = false;
  HeapSeekToFirst();
  for (uint64_t i = 0; i < walked && !min_heap_.empty(); i++) HeapNext();
}

void MergeIterator::HeapSeekToFirst() {
  min_heap_ = {};
  for (auto &iterator : table_reader_iterators_) {
    iterator->SeekToFirst();
    // pushed whether or not the table iterator is valid (merge_iterator.cc:86-90)
    min_heap_.push(HeapItem(iterator->GetKey(), iterator->GetTransactionId(), iterator.get()));
  }
}

// merge_iterator.cc:16-30 (past the end: an exhausted table iterator's values
// where the reference reads the top of an empty heap)
std::string_view MergeIterator::HeapGetKey() {
  return device_ || min_heap_.empty() ? std::string_view{} : min_heap_.top().iterator->GetKey();
}

std::string_view MergeIterator::HeapGetValue() {
  return device_ || min_heap_.empty() ? std::string_view{} : min_heap_.top().iterator->GetValue();
}

db::ValueType MergeIterator::HeapGetType() {
  return device_ || min_heap_.empty() ? db::ValueType::NOT_FOUND : min_heap_.top().iterator->GetType();
}

TxnId MergeIterator::HeapGetTransactionId() {
  return device_ || min_heap_.empty() ? INVALID_TXN_ID : min_heap_.top().iterator->GetTransactionId();
}

// merge_iterator.cc:34-46
void MergeIterator::HeapNext() {
  if (min_heap_.empty()) return;
  HeapItem item = min_heap_.top();
  min_heap_.pop();
  item.iterator->Next();
  if (item.iterator->IsValid())
    min_heap_.push(HeapItem(item.iterator->GetKey(), item.iterator->GetTransactionId(), item.iterator));
}

// merge_iterator.cc:48-60
void MergeIterator::Prev() {
  LeaveDevice();
  if (max_heap_.empty()) return;
  HeapItem item = max_heap_.top();
  max_heap_.pop();
  item.iterator->Prev();
  if (item.iterator->IsValid())
    max_heap_.push(HeapItem(item.iterator->GetKey(), item.iterator->GetTransactionId(), item.iterator));
}

// merge_iterator.cc:63-77
void MergeIterator::Seek(std::string_view key) {
  LeaveDevice();
  min_heap_ = {};
  for (auto &iterator : table_reader_iterators_) {
    iterator->Seek(key);
    min_heap_.push(HeapItem(iterator->GetKey(), iterator->GetTransactionId(), iterator.get()));
  }
}

// merge_iterator.cc:94-107
void MergeIterator::SeekToLast() {
  LeaveDevice();
  max_heap_ = {};
  for (auto &iterator : table_reader_iterators_) {
    iterator->SeekToLast();
    max_heap_.push(HeapItem(iterator->GetKey(), iterator->GetTransactionId(), iterator.get()));
  }
}

} // namespace db

} // namespace kvs
