// ref_harness.cc — extern "C" driver over the REFERENCE's own sstable classes.
//
// TEST INFRASTRUCTURE ONLY.  oracle/Makefile compiles this file together with
// the reference sources where they lie under /root/reference (nothing is copied)
// into oracle/_ref/libsstref.so.  It is used (a) by tests/golden/make_golden.py
// to dump golden fixtures, (b) by CPU tests to pin oracle/sst_oracle.c, and
// (c) as bench.py's cpu_baseline ("kind": "reference").
//
// Entry points mirror the reference call sequences:
//   encode    : BlockBuilder::AddEntry... EncodeExtraInfo      (block_builder.cc)
//   decode    : BlockReaderData parse as in TableReader::
//               CreateAndSetupDataForBlockReader (table_reader.cc:212-241) +
//               BlockReaderIterator accessors (block_reader_iterator.cc:20-119)
//   roundtrip : decode then re-encode with a BlockBuilder, i.e. the per-record
//               work db/compact.cc:254-302 does when every record survives
//   table     : TableBuilder Open/AddEntry/Finish (table_builder.cc) and
//               CreateAndSetupDataForTableReader / GetBlockIndex (table_reader.cc)

#include "db/config.h"
#include "db/status.h"
#include "sstable/block_builder.h"
#include "sstable/block_index.h"
#include "sstable/block_reader.h"
#include "sstable/block_reader_iterator.h"
#include "sstable/lru_block_item.h"
#include "sstable/table_builder.h"
#include "sstable/table_reader.h"

#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <memory>
#include <string>

namespace {

constexpr uint32_t kNoValue = 0xFFFFFFFFu;

// Same parse as TableReader::CreateAndSetupDataForBlockReader, from memory
// instead of pread (table_reader.cc:226-237).
std::unique_ptr<kvs::sstable::BlockReader> MakeBlockReader(const uint8_t *blk, uint64_t len) {
  auto d = std::make_unique<kvs::sstable::BlockReaderData>(len);
  std::memcpy(d->buffer.data(), blk, len);
  const int64_t last = static_cast<int64_t>(d->buffer.size()) - 1;
  d->total_data_entries = *reinterpret_cast<uint64_t *>(&d->buffer[last - 15]);
  d->offset_section = *reinterpret_cast<uint64_t *>(&d->buffer[last - 7]);
  for (uint64_t i = 0; i < d->total_data_entries; i++) {
    uint64_t e = d->offset_section + i * 16;
    d->data_entries_offset_info.emplace_back(*reinterpret_cast<const uint64_t *>(&d->buffer[e]));
  }
  return std::make_unique<kvs::sstable::BlockReader>(std::move(d));
}

// TableReaderIterator::CreateNewBlockReaderIterator builds the item this way on a
// cache miss (table_reader_iterator.cc:144-149).
std::unique_ptr<kvs::sstable::BlockReaderIterator> MakeIter(const uint8_t *blk, uint64_t len) {
  auto item = std::make_shared<kvs::sstable::LRUBlockItem>(std::make_pair(0ull, 0ull),
                                                           MakeBlockReader(blk, len), nullptr);
  return std::make_unique<kvs::sstable::BlockReaderIterator>(item);
}

std::string_view ValueView(const uint8_t *src, const uint64_t *off, const uint32_t *len,
                           uint64_t i) {
  if (len[i] == kNoValue) return std::string_view{};
  return std::string_view(reinterpret_cast<const char *>(src + off[i]), len[i]);
}

} // namespace

extern "C" {

uint64_t ref_block_encode(uint64_t n, const uint8_t *type, const uint32_t *key_len,
                          const uint32_t *val_len, const uint64_t *txn, const uint8_t *key_src,
                          const uint64_t *key_off, const uint8_t *val_src, const uint64_t *val_off,
                          uint8_t *out) {
  kvs::sstable::BlockBuilder b;
  for (uint64_t i = 0; i < n; i++) {
    std::string_view k(reinterpret_cast<const char *>(key_src + key_off[i]), key_len[i]);
    b.AddEntry(k, ValueView(val_src, val_off, val_len, i), txn[i],
               static_cast<kvs::db::ValueType>(type[i]));
  }
  b.EncodeExtraInfo();
  uint64_t p = 0;
  for (auto v : {b.GetDataView(), b.GetOffsetView(), b.GetExtraView()}) {
    std::memcpy(out + p, v.data(), v.size());
    p += v.size();
  }
  return p;
}

// Decode one block through the reference's reader. Offsets are relative to the
// block start.  Returns the record count.
uint64_t ref_block_decode(const uint8_t *blk, uint64_t len, uint8_t *type, uint32_t *key_len,
                          uint32_t *val_len, uint64_t *txn, uint64_t *key_off,
                          uint64_t *val_off) {
  auto it = MakeIter(blk, len);
  // MakeIter copied the block: views point into the copy and are rebased below.
  uint64_t i = 0;
  for (it->SeekToFirst(); it->IsValid(); it->Next(), i++) {
    auto k = it->GetKey();
    auto v = it->GetValue();
    type[i] = static_cast<uint8_t>(it->GetType());
    key_len[i] = static_cast<uint32_t>(k.size());
    val_len[i] = v.data() ? static_cast<uint32_t>(v.size()) : kNoValue;
    txn[i] = it->GetTransactionId();
    key_off[i] = reinterpret_cast<uintptr_t>(k.data());
    val_off[i] = v.data() ? reinterpret_cast<uintptr_t>(v.data()) : 0;
  }
  // Convert raw pointers to block-relative offsets: the first entry's start is
  // the stored start offset of entry 0.
  if (i) {
    const uint64_t s0 = *reinterpret_cast<const uint64_t *>(
        blk + *reinterpret_cast<const uint64_t *>(blk + len - 8));
    const uint64_t base = key_off[0] - 5 - s0;
    for (uint64_t j = 0; j < i; j++) {
      key_off[j] -= base;
      if (val_len[j] != kNoValue) val_off[j] -= base;
    }
  }
  return i;
}

// Decode every block with the reference reader and re-encode its records with
// a BlockBuilder (same sequence as compaction for surviving records); output at
// the same offset. out_len may be NULL.  Returns total records processed.
uint64_t ref_roundtrip_blocks(const uint8_t *src, const uint64_t *blk_off, const uint64_t *blk_len,
                              uint64_t nblocks, uint8_t *dst, uint64_t *out_len) {
  uint64_t total = 0;
  kvs::sstable::BlockBuilder b;
  for (uint64_t bi = 0; bi < nblocks; bi++) {
    auto it = MakeIter(src + blk_off[bi], blk_len[bi]);
    b.Reset();
    for (it->SeekToFirst(); it->IsValid(); it->Next()) {
      b.AddEntry(it->GetKey(), it->GetValue(), it->GetTransactionId(), it->GetType());
      total++;
    }
    b.EncodeExtraInfo();
    uint64_t p = blk_off[bi];
    for (auto v : {b.GetDataView(), b.GetOffsetView(), b.GetExtraView()}) {
      std::memcpy(dst + p, v.data(), v.size());
      p += v.size();
    }
    if (out_len) out_len[bi] = p - blk_off[bi];
  }
  return total;
}

// Write an SST with the reference TableBuilder. The Config is loaded the way the
// reference's tests load it (db/config.cc:37-53: <cwd>/../tests/test_config.toml);
// the harness writes that TOML into a scratch directory with the requested block
// size, chdirs there for the constructor and back.  Returns GetFileSize()
// (bytes on disk + 1, table_builder.cc:228) or 0 on failure.
uint64_t ref_table_build(const char *path, uint64_t block_size, uint64_t n, const uint8_t *type,
                         const uint32_t *key_len, const uint32_t *val_len, const uint64_t *txn,
                         const uint8_t *key_src, const uint64_t *key_off, const uint8_t *val_src,
                         const uint64_t *val_off) {
  namespace fs = std::filesystem;
  char tmpl[] = "/tmp/sstref_cfgXXXXXX";
  if (!mkdtemp(tmpl)) return 0;
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
  uint64_t fsize = 0;
  {
    kvs::sstable::TableBuilder tb(std::string(path), cfg.get());
    if (!tb.Open()) return 0;
    for (uint64_t i = 0; i < n; i++) {
      std::string_view k(reinterpret_cast<const char *>(key_src + key_off[i]), key_len[i]);
      tb.AddEntry(k, ValueView(val_src, val_off, val_len, i), txn[i],
                  static_cast<kvs::db::ValueType>(type[i]));
    }
    tb.Finish();
    fsize = tb.GetFileSize();
  }
  return fsize;
}

// Open an SST with the reference reader and list its block index
// (CreateAndSetupDataForTableReader, table_reader.cc:32-156).  Returns the
// number of blocks (fills up to cap), or UINT64_MAX on open failure.
uint64_t ref_table_index(const char *path, uint64_t file_size, uint64_t cap, uint64_t *blk_off,
                         uint64_t *blk_len, uint32_t *first_key_len, uint32_t *last_key_len,
                         uint8_t *first_key0, uint8_t *last_key_last) {
  auto tr = kvs::sstable::CreateAndSetupDataForTableReader(std::string(path), 1, file_size);
  if (!tr) return UINT64_MAX;
  const auto &idx = tr->GetBlockIndex();
  for (uint64_t i = 0; i < idx.size() && i < cap; i++) {
    blk_off[i] = idx[i].GetBlockStartOffset();
    blk_len[i] = idx[i].GetBlockSize();
    first_key_len[i] = static_cast<uint32_t>(idx[i].GetSmallestKey().size());
    last_key_len[i] = static_cast<uint32_t>(idx[i].GetLargestKey().size());
  }
  if (!idx.empty() && first_key0)
    std::memcpy(first_key0, idx.front().GetSmallestKey().data(), idx.front().GetSmallestKey().size());
  if (!idx.empty() && last_key_last)
    std::memcpy(last_key_last, idx.back().GetLargestKey().data(), idx.back().GetLargestKey().size());
  return idx.size();
}


// TableReader::GetValue without a block cache (table_reader.cc:168-189 ->
// BlockReader::GetValue, block_reader.cc:20-57), on the SST file itself.
// Per query: type (db::ValueType) and, for PUT, the value bytes appended to
// val_out (val_off / val_len).  Returns the bytes used in val_out, or
// UINT64_MAX on open failure / capacity.
uint64_t ref_table_get(const char *path, uint64_t file_size, uint64_t nq, const uint8_t *keys,
                       const uint64_t *key_off, const uint32_t *key_len, uint32_t *out_type,
                       uint64_t *val_off, uint32_t *val_len, uint8_t *val_out, uint64_t val_cap) {
  auto tr = kvs::sstable::CreateAndSetupDataForTableReader(std::string(path), 1, file_size);
  if (!tr) return UINT64_MAX;
  uint64_t used = 0;
  for (uint64_t q = 0; q < nq; q++) {
    const std::string_view key(reinterpret_cast<const char *>(keys + key_off[q]), key_len[q]);
    const kvs::db::GetStatus st = tr->GetValue(key, 1, nullptr, tr.get());
    out_type[q] = static_cast<uint32_t>(st.type);
    val_off[q] = used;
    val_len[q] = 0;
    if (st.value) {
      if (used + st.value->size() > val_cap) return UINT64_MAX;
      std::memcpy(val_out + used, st.value->data(), st.value->size());
      val_len[q] = static_cast<uint32_t>(st.value->size());
      used += st.value->size();
    }
  }
  return used;
}

} // extern "C"
