// readers_check.cc — a C++ caller compiled against include/sstc_table.h (test TU).
//
// The codec's own C++ reader surface, checked block by block:
// sstc::TableReader::CreateAndSetupDataForBlockReader (one block per call,
// table_reader.cc:212-241) and CreateAndSetupDataForBlockReaders (all blocks,
// one GPU call) against the sstc::TableReaderIterator stream, record by
// record, and Seek(); the records are written to dump_path (per record: u8
// type, u64 txn, u32 key length, key, u8 value-non-null, u32 value length,
// value) for comparison with the reference's own BlockReaderIterator
// (tests/readers_util.py).  Prints "readers ok <records>".
//
//   sstc_readers_check --readers dump_path [file size]...
//
// (The compaction loop over the reference's MergeIterator lives in the
// drop-in harness, oracle/ref_pick_compact.cc --loop, linked with the drop-in
// readers and builders: tests/test_gpu_dropin.py.)
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "sstc_table.h"

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
    sstc::TableReaderIterator it(tr.get());
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
  if (argc < 3 || std::string(argv[1]) != "--readers" || (argc - 3) % 2) {
    std::fprintf(stderr, "usage: %s --readers dump_path [file size]...\n", argv[0]);
    return 2;
  }
  try {
    return check_readers(argc, argv);
  } catch (const std::exception &e) {
    std::fprintf(stderr, "sstc_readers_check: %s\n", e.what());
    return 3;
  }
}
