// ref_pick_compact.cc — runs the REFERENCE's own Compact::PickCompact
// (/root/reference/db/compact.cc, compiled unchanged) over given L0 SSTs
// (TEST INFRASTRUCTURE ONLY).
//
// db/db_impl.cc cannot be compiled here (it includes the empty
// third_party/rapidjson submodule), and compact.cc / version*.cc /
// table_reader_cache.cc reach DBImpl only through seven accessors, so this TU
// defines exactly those plus the constructor/destructor,
// mirroring db/db_impl.cc:54-83,240-245,600-624 minus the memtable, the
// transaction manager and the trash-file thread, which compaction never
// touches.
//
// The same TU is linked twice by oracle/Makefile:
//   _ref/ref_pick_compact  against the reference's own sstable/table_builder.cc:
//                          the as-written compaction, INCLUDING the dangling
//                          `std::string_view last_current_key` of
//                          compact.cc:250,266-268;
//   _ref/compact_dropin    with include/dropin/ first on the include path, so
//                          db/compact.cc (unchanged) builds its outputs with
//                          sstc::TableBuilder (GPU encode, libsstcodec.so):
//                          the drop-in of INTEGRATION.md, demonstrated.
//
// usage: <exe> <db_dir> <block_size> <table_limit> [<file> <file_size> <smallest_hex> <largest_hex>]...
//   The inputs become L0 tables 1..k (table 1 = oldest), db_dir receives the
//   outputs "<id>.sst" (ids k+1, ...).  Prints one line per input the job
//   picked ("in <table_id>") and one per output ("out <path> <GetFileSize()>
//   <smallest_hex> <largest_hex>"), in VersionEdit order.
//
// usage: <exe> --loop <db_dir> <block_size> <table_limit> <base_level> [<file> <file_size>]...
//   The DoCompactJob loop (compact.cc:232-322) with the output split at ANY
//   table_limit (db::Config refuses limits below 4 MiB, db/config.cc:66-70)
//   and IsBaseLevelForKey() == base_level, over the REAL readers and merge:
//   TableReaderIterators made as Compact::CreateMergeIterator makes them
//   (compact.cc:207-225, through the TableReaderCache) and the reference's own
//   db::MergeIterator.  Prints the "out" lines.  Only the ~40-line loop body
//   is restated (ShouldKeepEntry is a private member of Compact).
//
// usage: <exe> --iter <dump> [<file> <file_size>]...
//   A scripted walk of every table through sstable::TableReaderIterator
//   (SeekToFirst + Next to the end and past it, SeekToLast + Prev to the
//   start and past it, Seek to every block's first / last key and to keys
//   outside the table, each followed by Nexts), every step's IsValid / key /
//   value / type / txn written to <dump>: linked against the reference's
//   table_reader_iterator.cc this is the reference's trace, linked as the
//   drop-in it is the GPU-decoding iterator's, and the two must be equal.
#include "common/base_iterator.h"
#include "common/thread_pool.h"
#include "db/merge_iterator.h"
#include "sstable/block_builder.h"
#include "sstable/block_index.h"
#include "sstable/lru_table_item.h"
#include "sstable/table_builder.h"
#include "sstable/table_reader.h"
#include "sstable/table_reader_iterator.h"
#include "db/base_memtable.h"
#include "db/compact.h"
#include "db/config.h"
#include "db/db_impl.h"
#include "db/version.h"
#include "db/version_edit.h"
#include "db/version_manager.h"
#include "io/base_file.h"
#include "mvcc/transaction.h"
#include "mvcc/transaction_manager.h"
#include "sstable/block_reader_cache.h"
#include "sstable/table_reader_cache.h"

#include <chrono>
#ifdef SSTC_DROPIN
#include "sstc_table.h" // sstc::ThreadContext
#endif
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <string>
#include <unistd.h>

namespace fs = std::filesystem;

namespace {
std::string g_db_path;
uint64_t g_block_size = 4096, g_table_limit = 32ull << 20, g_first_id = 1;

// db/config.cc:37-53 reads <cwd>/../tests/test_config.toml
std::unique_ptr<kvs::db::Config> MakeConfig() {
  char tmpl[] = "/tmp/sstref_pickXXXXXX";
  if (!mkdtemp(tmpl)) std::exit(3);
  fs::path root(tmpl);
  fs::create_directories(root / "tests");
  fs::create_directories(root / "run");
  {
    std::ofstream t(root / "tests" / "test_config.toml");
    t << "[lsm]\nLSM_PER_MEM_SIZE_LIMIT = " << g_table_limit << "\nMAX_IMMUTABLE_MEMTABLES_IN_MEMORY = 4\n"
      << "SST_BLOCK_SIZE = " << g_block_size << "\nLSM_SST_NUM_LEVELS = 7\n"
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

std::string Unhex(const char *h) {
  std::string s;
  if (h[0] == '-') return s;
  for (size_t i = 0; h[i] && h[i + 1]; i += 2) s.push_back(static_cast<char>(std::stoi(std::string(h + i, 2), nullptr, 16)));
  return s;
}

std::string Hex(std::string_view k) {
  std::string h;
  char b[3];
  for (unsigned char c : k) {
    std::snprintf(b, sizeof b, "%02x", c);
    h += b;
  }
  return h.empty() ? std::string("-") : h;
}
} // namespace

namespace kvs {
namespace db {

// db/db_impl.cc:54-75 (memtable, transaction manager and trash thread omitted)
DBImpl::DBImpl(bool is_testing)
    : db_path_(g_db_path), next_sstable_id_(g_first_id), memtable_version_(1), sequence_number_(0),
      config_(MakeConfig()), background_compaction_scheduled_(false),
      thread_pool_(std::make_unique<kvs::ThreadPool>(config_->GetTotalBackGroundThreads())),
      table_reader_cache_(std::make_unique<sstable::TableReaderCache>(this, thread_pool_.get())),
      block_cache_thread_pool_(std::make_unique<kvs::ThreadPool>(config_->GetTotalBlocksCache())),
      version_manager_(std::make_unique<VersionManager>(this, thread_pool_.get())) {
  (void)is_testing;
  for (int i = 0; i < config_->GetTotalBlocksCache(); i++) {
    block_reader_cache_.emplace_back(std::make_unique<sstable::BlockReaderCache>(
        config_->GetTotalBlocksCache(), block_cache_thread_pool_.get()));
  }
}

// db/db_impl.cc:77-83
DBImpl::~DBImpl() {
  block_reader_cache_.clear();
  table_reader_cache_.reset();
  shutdown_ = true;
  trash_files_cv_.notify_one();
}

// db/db_impl.cc:240-245
void DBImpl::WakeupBgThreadToCleanupFiles(std::string_view filename) const {
  std::scoped_lock rwlock(trash_files_mutex_);
  trash_files_.push(std::string(filename));
  trash_files_cv_.notify_one();
}

// db/db_impl.cc:600-624
uint64_t DBImpl::GetNextSSTId() { return next_sstable_id_.fetch_add(1); }
const Config *DBImpl::GetConfig() const { return config_.get(); }
const VersionManager *DBImpl::GetVersionManager() const { return version_manager_.get(); }
std::string DBImpl::GetDBPath() const { return db_path_; }
const std::vector<std::unique_ptr<sstable::BlockReaderCache>> &DBImpl::GetBlockReaderCache() const {
  return block_reader_cache_;
}
const sstable::TableReaderCache *DBImpl::GetTableReaderCache() const { return table_reader_cache_.get(); }

} // namespace db
} // namespace kvs

namespace {
using namespace kvs;

// compact.cc:207-225: a TableReader opened and inserted into the table cache,
// then an iterator over the cached item
std::unique_ptr<sstable::TableReaderIterator> OpenIterator(db::DBImpl *db, SSTId id, const char *path,
                                                           uint64_t file_size) {
  auto reader = sstable::CreateAndSetupDataForTableReader(std::string(path), id, file_size);
  if (!reader) return nullptr;
  auto item = std::make_shared<sstable::LRUTableItem>(id, std::move(reader), db->GetTableReaderCache());
  auto inserted = db->GetTableReaderCache()->AddNewTableReaderThenGet(id, item, true /*add_then_get*/);
  return std::make_unique<sstable::TableReaderIterator>(db->GetBlockReaderCache(), inserted);
}

int RunLoop(int argc, char **argv) {
  // argv: --loop db_dir block_size table_limit base_level [file size]...
  g_db_path = std::string(argv[2]);
  if (g_db_path.back() != '/') g_db_path += '/';
  g_block_size = std::strtoull(argv[3], nullptr, 10);
  const uint64_t table_limit = std::strtoull(argv[4], nullptr, 10);
  const bool base_level = std::atoi(argv[5]) != 0;
  const int k = (argc - 6) / 2;
  g_first_id = static_cast<uint64_t>(k) + 1;
  g_table_limit = 32ull << 20; // what db::Config accepts; the loop splits at table_limit
  auto *db = new db::DBImpl(true);
  std::vector<std::unique_ptr<sstable::TableReaderIterator>> its;
  for (int i = 0; i < k; i++) {
    its.push_back(OpenIterator(db, static_cast<SSTId>(i + 1), argv[6 + 2 * i],
                               std::strtoull(argv[7 + 2 * i], nullptr, 10)));
    if (!its.back()) return 4;
  }
  auto iterator = std::make_unique<db::MergeIterator>(std::move(its));
  auto report = [](uint64_t id, sstable::TableBuilder &t) {
    std::printf("out %s%llu.sst %llu %s %s\n", g_db_path.c_str(), (unsigned long long)id,
                (unsigned long long)t.GetFileSize(), Hex(t.GetSmallestKey()).c_str(), Hex(t.GetLargestKey()).c_str());
  };
  // ---- compact.cc:235-311 (the loop as written, minus the version edits)
  uint64_t new_sst_id = db->GetNextSSTId();
  std::string filename = db->GetDBPath() + std::to_string(new_sst_id) + ".sst";
  auto new_sst = std::make_unique<sstable::TableBuilder>(std::move(filename), db->GetConfig());
  if (!new_sst->Open()) return 5;
  std::string last_current_key; // an owned copy: the intended semantics of compact.cc:250
  bool have_last = false;
  TxnId last_txn_id = INVALID_TXN_ID;
  for (iterator->SeekToFirst(); iterator->IsValid(); iterator->Next()) {
    std::string_view key = iterator->GetKey();
    std::string_view value = iterator->GetValue();
    db::ValueType type = iterator->GetType();
    TxnId txn_id = iterator->GetTransactionId();
    // ShouldKeepEntry (compact.cc:324-363) with IsBaseLevelForKey() == base_level
    bool should_keep_entry;
    if (!have_last) should_keep_entry = true;
    else if (last_current_key != key) should_keep_entry = type == db::ValueType::PUT ? true : !base_level;
    else should_keep_entry = !(last_txn_id > txn_id);
    if (!have_last || last_current_key != key) {
      last_current_key.assign(key.data(), key.size());
      last_txn_id = txn_id;
      have_last = true;
    }
    if (!should_keep_entry) continue;
    if (!new_sst) {
      new_sst_id = db->GetNextSSTId();
      filename = db->GetDBPath() + std::to_string(new_sst_id) + ".sst";
      new_sst = std::make_unique<sstable::TableBuilder>(std::move(filename), db->GetConfig());
      if (!new_sst->Open()) return 5;
    }
    new_sst->AddEntry(key, value, txn_id, type);
    if (new_sst->GetDataSize() >= table_limit) {
      new_sst->Finish();
      report(new_sst_id, *new_sst);
      new_sst.reset();
    }
  }
  if (new_sst) {
    new_sst->Finish();
    report(new_sst_id, *new_sst);
  }
  std::fflush(stdout);
  _exit(0);
}

int RunIter(int argc, char **argv) {
  // argv: --iter dump [file size]...
  std::FILE *dump = std::fopen(argv[2], "wb");
  if (!dump) return 4;
  char tmpl[] = "/tmp/sstref_iterXXXXXX";
  if (!mkdtemp(tmpl)) return 3;
  g_db_path = std::string(tmpl) + "/";
  auto *db = new db::DBImpl(true);
  auto put = [&](const void *p, size_t n) { std::fwrite(p, 1, n, dump); };
  auto view = [&](std::string_view v) {
    const uint8_t has = v.data() != nullptr;
    const uint32_t n = static_cast<uint32_t>(v.size());
    put(&has, 1), put(&n, 4);
    if (n) put(v.data(), n);
  };
  uint64_t steps = 0;
  for (int i = 3; i + 1 < argc; i += 2) {
    const uint64_t fs = std::strtoull(argv[i + 1], nullptr, 10);
    auto it = OpenIterator(db, static_cast<SSTId>(i), argv[i], fs);
    if (!it) return 4;
    auto step = [&](char op) {
      const uint8_t valid = it->IsValid();
      const uint8_t type = static_cast<uint8_t>(it->GetType());
      const TxnId txn = it->GetTransactionId();
      put(&op, 1), put(&valid, 1), put(&type, 1), put(&txn, 8);
      view(it->GetKey());
      view(it->GetValue());
      steps++;
    };
    // the block index, through a second reader (the iterator's is private)
    auto reader = sstable::CreateAndSetupDataForTableReader(std::string(argv[i]), 0, fs);
    if (!reader) return 4;
    std::vector<std::string> keys;
    for (const auto &bi : reader->GetBlockIndex()) {
      keys.emplace_back(bi.GetSmallestKey());
      keys.emplace_back(bi.GetLargestKey());
    }
    it->SeekToFirst();
    for (step('F'); it->IsValid(); step('N')) it->Next();
    it->Next(), step('N');
    it->SeekToLast();
    for (step('L'); it->IsValid(); step('P')) it->Prev();
    it->Next(), step('N'); // the entry cursor wraps back to entry 0 of the shown block
    keys.emplace_back("");
    keys.emplace_back(std::string(1, '\0'));
    keys.emplace_back(std::string(64, '\xff'));
    for (const std::string &k : keys) {
      it->Seek(k), step('S');
      for (int j = 0; j < 3; j++) it->Next(), step('N');
      it->Prev(), step('P');
    }
  }
  std::fclose(dump);
  std::printf("iter ok %llu\n", (unsigned long long)steps);
  std::fflush(stdout);
  _exit(0);
}
} // namespace

// usage: <exe> --merge <dump> <mid_key_hex> [<file> <file_size>]...
//   db::MergeIterator over TableReaderIterators of every file (as
//   CreateMergeIterator makes them), every step's IsValid / key / value /
//   type / txn written to <dump>: (1) SeekToFirst + Next to the end (the whole
//   merged order), then SeekToLast + Prev while IsValid, as the reference's
//   tests/test_mergeIterator.cc:154-182 walks it; (2) a second iterator
//   walked half way, then SeekToLast, Prev x 3 (IsValid is the min heap's,
//   the accessors read the min heap's top), Seek(mid key) + Next x 3,
//   SeekToFirst + Next x 2 (only steps whose outcome the reference defines:
//   no min-heap pop after SeekToLast, whose table iterators then hold new
//   blocks while the min heap's keys still view the freed ones).  Linked against the reference's merge_iterator.cc
//   this is the reference's trace; linked as the drop-in it is the device
//   merge's, and the two must be equal.
int RunMerge(int argc, char **argv) {
  using namespace kvs;
  std::FILE *dump = std::fopen(argv[2], "wb");
  if (!dump) return 4;
  const std::string mid = Unhex(argv[3]);
  char tmpl[] = "/tmp/sstref_mergeXXXXXX";
  if (!mkdtemp(tmpl)) return 3;
  g_db_path = std::string(tmpl) + "/";
  auto *db = new db::DBImpl(true);
  auto put = [&](const void *p, size_t n) { std::fwrite(p, 1, n, dump); };
  auto view = [&](std::string_view v) {
    const uint8_t has = v.data() != nullptr;
    const uint32_t n = static_cast<uint32_t>(v.size());
    put(&has, 1), put(&n, 4);
    if (n) put(v.data(), n);
  };
  auto make = [&](int pass) {
    std::vector<std::unique_ptr<sstable::TableReaderIterator>> its;
    for (int i = 4; i + 1 < argc; i += 2) {
      its.push_back(OpenIterator(db, static_cast<SSTId>(100 * pass + i), argv[i],
                                 std::strtoull(argv[i + 1], nullptr, 10)));
      if (!its.back()) std::exit(4);
    }
    return std::make_unique<db::MergeIterator>(std::move(its));
  };
  uint64_t steps = 0, walked = 0;
  auto step = [&](db::MergeIterator &it, char op, bool read = true) {
    const uint8_t valid = it.IsValid();
    put(&op, 1), put(&valid, 1);
    if (read) {
      const uint8_t type = static_cast<uint8_t>(it.GetType());
      const TxnId txn = it.GetTransactionId();
      put(&type, 1), put(&txn, 8);
      view(it.GetKey());
      view(it.GetValue());
    }
    steps++;
  };
  {
    auto it = make(1);
    for (it->SeekToFirst(); it->IsValid(); it->Next(), walked++) step(*it, 'N');
    step(*it, 'E', false);
    for (it->SeekToLast(); it->IsValid(); it->Prev()) step(*it, 'P');
    step(*it, 'L', false);
  }
  if (walked >= 8) {
    auto it = make(2);
    it->SeekToFirst();
    for (uint64_t i = 0; i < walked / 2; i++) it->Next();
    step(*it, 'H');
    it->SeekToLast(), step(*it, 'L');
    for (int j = 0; j < 3; j++) it->Prev(), step(*it, 'P');
    // (a Next here would pop the min heap, whose keys SeekToLast left
    // dangling in the reference: its table iterators freed those blocks)
    it->Seek(mid), step(*it, 'S');
    for (int j = 0; j < 3; j++) it->Next(), step(*it, 'N');
    it->SeekToFirst(), step(*it, 'F');
    for (int j = 0; j < 2; j++) it->Next(), step(*it, 'N');
  }
  std::fclose(dump);
  std::printf("merge ok %llu %llu\n", (unsigned long long)walked, (unsigned long long)steps);
  std::fflush(stdout);
  _exit(0);
}

// usage: <exe> --walk <level> [<file> <file_size>]...
//   Diagnostic: the time of DoCompactJob's loop parts over db::MergeIterator
//   (level 0: SeekToFirst + Next + the four accessors; 1: + the key compare of
//   ShouldKeepEntry; 2: + TableBuilder::AddEntry into builders split at 32 MiB
//   that are never finished -- no encode, no file written).
int RunWalk(int argc, char **argv) {
  using namespace kvs;
  const int level = std::atoi(argv[2]);
  char tmpl[] = "/tmp/sstref_walkXXXXXX";
  if (!mkdtemp(tmpl)) return 3;
  g_db_path = std::string(tmpl) + "/";
  auto *db = new db::DBImpl(true);
  std::vector<std::unique_ptr<sstable::TableReaderIterator>> its;
  for (int i = 3; i + 1 < argc; i += 2) {
    its.push_back(OpenIterator(db, static_cast<SSTId>(i), argv[i], std::strtoull(argv[i + 1], nullptr, 10)));
    if (!its.back()) return 4;
  }
#ifdef SSTC_DROPIN
  sstc::ThreadContext();
#endif
  auto it = std::make_unique<db::MergeIterator>(std::move(its));
  const auto t0 = std::chrono::steady_clock::now();
  it->SeekToFirst();
  const auto t1 = std::chrono::steady_clock::now();
  uint64_t n = 0, sum = 0, kept = 0;
  std::string_view last;
  std::unique_ptr<sstable::TableBuilder> b;
  for (; it->IsValid(); it->Next(), n++) {
    std::string_view key = it->GetKey(), value = it->GetValue();
    const db::ValueType type = it->GetType();
    const TxnId txn = it->GetTransactionId();
    sum += key.size() + value.size() + static_cast<int>(type) + txn;
    if (level >= 1) {
      kept += last != key;
      last = key;
    }
    if (level >= 2) {
      if (!b) b = std::make_unique<sstable::TableBuilder>(g_db_path + "walk.sst", db->GetConfig());
      b->AddEntry(key, value, txn, type);
      if (b->GetDataSize() >= (32ull << 20)) b.reset();
    }
  }
  const auto t2 = std::chrono::steady_clock::now();
  std::printf("walk level %d: %llu records (%llu keys, sum %llu): SeekToFirst %.6f s, loop %.6f s = %.1f ns/record\n",
              level, (unsigned long long)n, (unsigned long long)kept, (unsigned long long)sum,
              std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t2 - t1).count(),
              1e9 * std::chrono::duration<double>(t2 - t1).count() / (n ? n : 1));
  std::fflush(stdout);
  _exit(0);
}

int main(int argc, char **argv) {
  if (argc >= 3 && std::string(argv[1]) == "--walk" && (argc - 3) % 2 == 0) return RunWalk(argc, argv);
  if (argc >= 4 && std::string(argv[1]) == "--merge" && (argc - 4) % 2 == 0) return RunMerge(argc, argv);
  if (argc >= 6 && std::string(argv[1]) == "--loop" && (argc - 6) % 2 == 0) return RunLoop(argc, argv);
  if (argc >= 3 && std::string(argv[1]) == "--iter" && (argc - 3) % 2 == 0) return RunIter(argc, argv);
  if (argc < 4 || (argc - 4) % 4) {
    std::fprintf(stderr, "usage: %s db_dir block_size table_limit [file size smallest_hex largest_hex]...\n",
                 argv[0]);
    return 2;
  }
  g_db_path = std::string(argv[1]);
  if (g_db_path.back() != '/') g_db_path += '/';
  g_block_size = std::strtoull(argv[2], nullptr, 10);
  g_table_limit = std::strtoull(argv[3], nullptr, 10);
  const int k = (argc - 4) / 4;
  g_first_id = static_cast<uint64_t>(k) + 1;

  // a DBImpl that is never destroyed: the reference tears its caches down
  // while their pool threads may still run (db_impl.cc:77-83); the process
  // exits through _exit once the outputs are on disk.
  auto *db = new kvs::db::DBImpl(true);
  auto *vm = const_cast<kvs::db::VersionManager *>(db->GetVersionManager());
  const int levels = db->GetConfig()->GetSSTNumLvels();

  // the first edit only creates the initial version (whose
  // scores would pick the last level); the second one adds the L0 inputs and
  // gives level 0 the score |L0| / trigger (version_manager.cc:200-203).
  vm->ApplyNewChanges(std::make_unique<kvs::db::VersionEdit>(levels));
  auto add = std::make_unique<kvs::db::VersionEdit>(levels);
  for (int i = 0; i < k; i++) {
    char **a = argv + 4 + 4 * i;
    add->AddNewFiles(static_cast<kvs::SSTId>(i + 1), 0, std::strtoull(a[1], nullptr, 10), Unhex(a[2]), Unhex(a[3]),
                     std::string(a[0]));
  }
  vm->ApplyNewChanges(std::move(add));

  const kvs::db::Version *version = vm->GetLatestVersion();
  kvs::db::VersionEdit out_edit(levels);
  kvs::db::Compact compact(db->GetBlockReaderCache(), db->GetTableReaderCache(), version, &out_edit, db);
#ifdef SSTC_DROPIN
  { // the drop-in build: open this thread's codec context (HIP runtime, code
    // objects, stream) before the timer, as an engine does once at DB open --
    // the reference's caches above are built outside the timer too
    const auto ti = std::chrono::steady_clock::now();
    sstc::ThreadContext();
    std::printf("init %.6f\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - ti).count());
  }
#endif
  const auto t0 = std::chrono::steady_clock::now();
  const bool ok = compact.PickCompact(); // db/compact.cc:35-52 -> DoL0L1Compact -> DoCompactJob
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  for (const auto &del : out_edit.GetImmutableDeletedFiles()) std::printf("in %llu\n", (unsigned long long)del.first);
  for (const auto &level_files : out_edit.GetImmutableNewFiles())
    for (const auto &m : level_files)
      std::printf("out %s %llu %s %s\n", m->filename.c_str(), (unsigned long long)m->file_size,
                  Hex(m->smallest_key).c_str(), Hex(m->largest_key).c_str());
  std::printf("time %.6f\n", secs); // PickCompact wall time (inputs opened, merged, outputs written + fsync'd)
  std::fflush(stdout);
  _exit(ok ? 0 : 1);
}
