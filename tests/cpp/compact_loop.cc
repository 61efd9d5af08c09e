// compact_loop.cc — a C++ caller compiled against include/sstc_table.h (test TU).
//
// It runs the compaction loop of the reference's Compact::DoCompactJob
// (/root/reference/db/compact.cc:232-322, ShouldKeepEntry :324-363) and its
// MergeIterator (db/merge_iterator.cc:37-46, merge_iterator.h:91-95: a
// std::priority_queue with the same comparator, so ties between equal
// (key, txn) records pop in the reference's order) over this framework's
// types, with the reference's own spellings: kvs::sstable::TableBuilder is an
// alias of sstc::TableBuilder, constructed from (std::string&&, const
// db::Config*) and fed db::ValueType -- the lines a maintainer keeps unchanged
// in db/compact.cc.  Inputs are read through sstc::TableReaderIterator (each
// table decoded in one GPU call), outputs encoded on the GPU at Finish().
//
//   sstc_compact_loop out_dir block_size table_limit base_level [file size]...
//
// prints "path smallest_key_hex largest_key_hex GetFileSize()" per output.
//
//   sstc_compact_loop --readers dump_path [file size]...
//
// checks TableReader::CreateAndSetupDataForBlockReader (one block per call)
// and CreateAndSetupDataForBlockReaders (all blocks, one call) against the
// TableReaderIterator stream, record by record, and Seek(); writes the
// records to dump_path (per record: u8 type, u64 txn, u32 key length, key,
// u8 value-non-null, u32 value length, value) for comparison with the
// reference's own BlockReaderIterator (tests/readers_util.py); prints
// "readers ok <records>".
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <queue>
#include <string>
#include <vector>

#include "sstc_table.h"

namespace kvs {
using TxnId = uint64_t;
constexpr TxnId INVALID_TXN_ID = 0;
namespace db {
enum class ValueType : uint8_t { PUT = 0, DELETED = 1, NOT_FOUND = 2, kTooManyOpenFiles = 3 }; // db/status.h:11-19
struct Config { // the two knobs of db/config.h this path reads
  uint64_t block_size, table_limit;
  uint64_t GetSSTBlockSize() const { return block_size; }
  uint64_t GetPerMemTableSizeLimit() const { return table_limit; }
};
} // namespace db
namespace sstable {
using TableBuilder = ::sstc::TableBuilder; // the drop-in
using TableReaderIterator = ::sstc::TableReaderIterator;
} // namespace sstable

namespace db {
// merge_iterator.h/.cc (min-heap part)
class MergeIterator {
public:
  explicit MergeIterator(std::vector<std::unique_ptr<sstable::TableReaderIterator>> its) : its_(std::move(its)) {}
  void SeekToFirst() {
    std::priority_queue<HeapItem, std::vector<HeapItem>, LessCompare> pq;
    min_heap_.swap(pq);
    for (auto &it : its_) {
      it->SeekToFirst();
      if (it->IsValid()) min_heap_.push(HeapItem{it->GetKey(), it->GetTransactionId(), it.get()});
    }
  }
  bool IsValid() const { return !min_heap_.empty(); }
  void Next() {
    HeapItem h = min_heap_.top();
    min_heap_.pop();
    h.iterator->Next();
    if (h.iterator->IsValid()) min_heap_.push(HeapItem{h.iterator->GetKey(), h.iterator->GetTransactionId(), h.iterator});
  }
  std::string_view GetKey() const { return min_heap_.top().iterator->GetKey(); }
  std::string_view GetValue() const { return min_heap_.top().iterator->GetValue(); }
  ValueType GetType() const { return static_cast<ValueType>(min_heap_.top().iterator->GetType()); }
  TxnId GetTransactionId() const { return min_heap_.top().iterator->GetTransactionId(); }

private:
  struct HeapItem {
    std::string_view key;
    TxnId txn_id;
    sstable::TableReaderIterator *iterator;
  };
  struct LessCompare {
    bool operator()(const HeapItem &a, const HeapItem &b) {
      return a.key > b.key || (a.key == b.key && a.txn_id < b.txn_id);
    }
  };
  std::vector<std::unique_ptr<sstable::TableReaderIterator>> its_;
  std::priority_queue<HeapItem, std::vector<HeapItem>, LessCompare> min_heap_;
};
} // namespace db
} // namespace kvs

using namespace kvs;

static int check_readers(int argc, char **argv) {
  uint64_t total = 0;
  std::FILE *dump = std::fopen(argv[2], "wb");
  if (!dump) return 4;
  std::unique_ptr<std::FILE, int (*)(std::FILE *)> closer(dump, std::fclose);
  auto put = [&](const void *p, size_t n) { std::fwrite(p, 1, n, dump); };
  for (int i = 3; i + 1 < argc; i += 2) {
    auto tr = sstc::TableReader::Create(std::string(argv[i]), 1, std::strtoull(argv[i + 1], nullptr, 10));
    if (!tr) return 4;
    std::vector<std::pair<sstc::BlockOffset, uint64_t>> blocks;
    for (const auto &bi : tr->GetBlockIndex()) blocks.emplace_back(bi.offset, bi.size);
    auto batched = tr->CreateAndSetupDataForBlockReaders(blocks);
    sstable::TableReaderIterator it(tr.get());
    it.SeekToFirst();
    for (size_t b = 0; b < blocks.size(); b++) {
      auto one = tr->CreateAndSetupDataForBlockReader(blocks[b].first, blocks[b].second);
      if (!one || !batched[b] || one->Status() != SSTC_BLK_OK || one->NumEntries() != batched[b]->NumEntries())
        return 6;
      for (uint64_t e = 0; e < one->NumEntries(); e++, it.Next()) {
        for (const sstc::BlockReader *r : {one.get(), batched[b].get()}) {
          if (!it.IsValid() || r->GetKey(e) != it.GetKey() || r->GetType(e) != it.GetType() ||
              r->GetTransactionId(e) != it.GetTransactionId() || r->GetValue(e) != it.GetValue() ||
              (r->GetValue(e).data() == nullptr) != (it.GetValue().data() == nullptr))
            return 7;
        }
        const uint8_t ty = static_cast<uint8_t>(it.GetType());
        const uint64_t tx = it.GetTransactionId();
        const std::string_view k = it.GetKey(), v = it.GetValue();
        const uint32_t kl = static_cast<uint32_t>(k.size()), vl = static_cast<uint32_t>(v.size());
        const uint8_t has = v.data() != nullptr;
        put(&ty, 1), put(&tx, 8), put(&kl, 4), put(k.data(), kl), put(&has, 1), put(&vl, 4);
        if (vl) put(v.data(), vl);
        total++;
      }
    }
    if (it.IsValid()) return 8;
    // Seek: every block's first key is found at a position holding it
    for (const auto &bi : tr->GetBlockIndex()) {
      it.Seek(bi.smallest_key);
      if (!it.IsValid() || it.GetKey() != bi.smallest_key) return 9;
    }
  }
  std::printf("readers ok %llu\n", static_cast<unsigned long long>(total));
  return 0;
}

int main(int argc, char **argv) {
  if (argc >= 2 && std::string(argv[1]) == "--readers") {
    try {
      return check_readers(argc, argv);
    } catch (const std::exception &e) {
      std::fprintf(stderr, "sstc_compact_loop: %s\n", e.what());
      return 3;
    }
  }
  if (argc < 5 || (argc - 5) % 2) {
    std::fprintf(stderr, "usage: %s out_dir block_size table_limit base_level [file size]...\n", argv[0]);
    return 2;
  }
  const std::string out_dir = argv[1];
  const db::Config config{std::strtoull(argv[2], nullptr, 10), std::strtoull(argv[3], nullptr, 10)};
  const bool base_level = std::atoi(argv[4]) != 0;
  try {
    std::vector<std::unique_ptr<sstc::TableReader>> readers;
    std::vector<std::unique_ptr<sstable::TableReaderIterator>> its;
    for (int i = 5; i < argc; i += 2) {
      readers.push_back(sstc::TableReader::Create(std::string(argv[i]), readers.size() + 1,
                                                  std::strtoull(argv[i + 1], nullptr, 10)));
      if (!readers.back()) {
        std::fprintf(stderr, "cannot open %s\n", argv[i]);
        return 4;
      }
      its.push_back(std::make_unique<sstable::TableReaderIterator>(readers.back().get()));
    }
    auto iterator = std::make_unique<db::MergeIterator>(std::move(its));

    uint64_t next_id = 0;
    auto new_name = [&] { return out_dir + "/" + std::to_string(next_id++) + ".sst"; };
    auto hex = [](std::string_view k) {
      std::string h;
      for (unsigned char c : k) {
        char b[3];
        std::snprintf(b, sizeof b, "%02x", c);
        h += b;
      }
      return h.empty() ? std::string("-") : h;
    };
    auto report = [&](sstable::TableBuilder &t) { // what VersionEdit::AddNewFiles records (compact.cc:292-297)
      std::printf("%s %s %s %llu\n", std::string(t.GetFilename()).c_str(), hex(t.GetSmallestKey()).c_str(),
                  hex(t.GetLargestKey()).c_str(), static_cast<unsigned long long>(t.GetFileSize()));
    };
    // ---- db/compact.cc:232-322, the loop body as the reference writes it
    std::string filename = new_name();
    auto new_sst = std::make_unique<sstable::TableBuilder>(std::move(filename), &config);
    if (!new_sst->Open()) return 5;
    std::string last_current_key; // owned copy: the intended semantics of :250 (no dangling view)
    bool have_last = false;
    TxnId last_txn_id = INVALID_TXN_ID;
    for (iterator->SeekToFirst(); iterator->IsValid(); iterator->Next()) {
      std::string_view key = iterator->GetKey();
      std::string_view value = iterator->GetValue();
      db::ValueType type = iterator->GetType();
      TxnId txn_id = iterator->GetTransactionId();
      // ShouldKeepEntry (:324-363) with IsBaseLevelForKey() == base_level
      bool should_keep_entry;
      if (!have_last) should_keep_entry = true;
      else if (last_current_key != key)
        should_keep_entry = type == db::ValueType::PUT ? true : !base_level;
      else should_keep_entry = !(last_txn_id > txn_id);
      if (!have_last || last_current_key != key) {
        last_current_key.assign(key.data(), key.size());
        last_txn_id = txn_id;
        have_last = true;
      }
      if (!should_keep_entry) continue;
      if (!new_sst) {
        filename = new_name();
        new_sst = std::make_unique<sstable::TableBuilder>(std::move(filename), &config);
        if (!new_sst->Open()) return 5;
      }
      new_sst->AddEntry(key, value, txn_id, type);
      if (new_sst->GetDataSize() >= config.GetPerMemTableSizeLimit()) {
        new_sst->Finish();
        report(*new_sst);
        new_sst.reset();
      }
    }
    if (new_sst) {
      new_sst->Finish();
      report(*new_sst);
    }
  } catch (const std::exception &e) {
    std::fprintf(stderr, "sstc_compact_loop: %s\n", e.what());
    return 3;
  }
  return 0;
}
