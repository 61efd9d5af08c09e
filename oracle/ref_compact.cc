// ref_compact.cc — compaction driver over the REFERENCE's own merge and table
// code (TEST INFRASTRUCTURE ONLY; golden fixtures).
//
// db/compact.cc itself cannot be built here: Compact needs DBImpl, whose
// db_impl.cc requires the empty third_party/rapidjson submodule.  This driver
// therefore runs the reference's MergeIterator (db/merge_iterator.cc) over the
// reference's TableReaderIterators (sstable/table_reader_iterator.cc) and writes
// with the reference's TableBuilder; the loop between them restates
// Compact::DoCompactJob / ShouldKeepEntry (db/compact.cc:232-363) with one
// deliberate difference: the previous key is held in a std::string instead of a
// std::string_view into a block buffer that the iterator frees (the dangling
// view of compact.cc:250,266-268).
//
// The binary is linked with --unresolved-symbols=ignore-all: the only missing
// symbol, TableReaderCache::AddVictim (sstable/table_reader_cache.cc needs
// DBImpl), is reachable only through a non-null cache pointer, and this driver
// passes nullptr (lru_table_item.cc:24-27).
//
// usage: ref_compact <out_dir> <block_size> <table_limit> <base_level 0|1> <file> <file_size> ...
//   prints one line per output table: "<path> <GetFileSize()>"
#include "db/config.h"
#include "db/merge_iterator.h"
#include "db/status.h"
#include "sstable/block_builder.h"
#include "sstable/block_reader.h"
#include "sstable/block_reader_cache.h"
#include "sstable/lru_table_item.h"
#include "sstable/table_builder.h"
#include "sstable/table_reader.h"
#include "sstable/table_reader_iterator.h"

#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <memory>
#include <string>
#include <vector>

namespace fs = std::filesystem;

static std::unique_ptr<kvs::db::Config> MakeConfig(uint64_t block_size) {
  // db/config.cc:37-53 reads <cwd>/../tests/test_config.toml
  char tmpl[] = "/tmp/sstref_cfgXXXXXX";
  if (!mkdtemp(tmpl)) return nullptr;
  fs::path root(tmpl);
  fs::create_directories(root / "tests");
  fs::create_directories(root / "run");
  {
    std::ofstream t(root / "tests" / "test_config.toml");
    t << "[lsm]\nLSM_PER_MEM_SIZE_LIMIT = 33554432\nMAX_IMMUTABLE_MEMTABLES_IN_MEMORY = 4\n"
      << "SST_BLOCK_SIZE = " << block_size << "\nLSM_SST_NUM_LEVELS = 7\n"
      << "LVL0_COMPACTION_TRIGGER = 6\n[cache]\nTOTAL_BG_THREADS = 12\n"
      << "TOTAL_TABLES_CACHE = 1000\nTOTAL_BLOCKS_EACH_CACHE = 20000\nTOTAL_BLOCKS_CACHE = 5\n";
  }
  fs::path old = fs::current_path();
  fs::current_path(root / "run");
  auto cfg = std::make_unique<kvs::db::Config>(true);
  fs::current_path(old);
  fs::remove_all(root);
  return cfg;
}

int main(int argc, char **argv) {
  if (argc < 5 || (argc - 5) % 2) {
    std::fprintf(stderr, "usage: %s out_dir block_size table_limit base_level [file size]...\n", argv[0]);
    return 2;
  }
  const std::string out_dir = argv[1];
  const uint64_t block_size = std::strtoull(argv[2], nullptr, 10);
  const uint64_t table_limit = std::strtoull(argv[3], nullptr, 10);
  const bool base_level = std::atoi(argv[4]) != 0;
  auto cfg = MakeConfig(block_size);
  if (!cfg) return 3;

  std::vector<std::unique_ptr<kvs::sstable::BlockReaderCache>> no_block_cache;
  std::vector<std::unique_ptr<kvs::sstable::TableReaderIterator>> iters;
  for (int i = 5; i < argc; i += 2) {
    const uint64_t size = std::strtoull(argv[i + 1], nullptr, 10);
    const kvs::SSTId id = static_cast<kvs::SSTId>(iters.size() + 1);
    auto reader = kvs::sstable::CreateAndSetupDataForTableReader(std::string(argv[i]), id, size);
    if (!reader) return 4;
    auto item = std::make_shared<kvs::sstable::LRUTableItem>(id, std::move(reader), nullptr);
    iters.emplace_back(std::make_unique<kvs::sstable::TableReaderIterator>(no_block_cache, item));
  }
  kvs::db::MergeIterator it(std::move(iters));

  int next_id = 0;
  auto new_table = [&]() {
    auto tb = std::make_unique<kvs::sstable::TableBuilder>(out_dir + "/" + std::to_string(next_id++) + ".sst",
                                                           cfg.get());
    if (!tb->Open()) std::exit(5);
    return tb;
  };
  auto finish = [&](std::unique_ptr<kvs::sstable::TableBuilder> &tb) {
    tb->Finish();
    std::printf("%s %llu\n", std::string(tb->GetFilename()).c_str(),
                static_cast<unsigned long long>(tb->GetFileSize()));
    tb.reset();
  };

  std::unique_ptr<kvs::sstable::TableBuilder> sst = new_table(); // compact.cc:236-240
  std::string last_key;
  bool have_last = false;
  kvs::TxnId last_txn = kvs::INVALID_TXN_ID;
  for (it.SeekToFirst(); it.IsValid(); it.Next()) {
    std::string_view key = it.GetKey();
    std::string_view value = it.GetValue();
    kvs::db::ValueType type = it.GetType();
    kvs::TxnId txn = it.GetTransactionId();
    // ShouldKeepEntry, compact.cc:324-363 (IsBaseLevelForKey -> base_level)
    bool keep;
    const bool new_key = !have_last || last_key != key;
    if (!have_last) keep = true;
    else if (new_key) keep = type == kvs::db::ValueType::PUT ? true : !base_level;
    else keep = !(last_txn > txn);
    if (new_key) {
      last_key.assign(key.data(), key.size());
      last_txn = txn;
      have_last = true;
    }
    if (!keep) continue;
    if (!sst) sst = new_table();
    sst->AddEntry(key, value, txn, type);
    if (sst->GetDataSize() >= table_limit) finish(sst); // compact.cc:289-301
  }
  if (sst) finish(sst);
  return 0;
}
