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
 * Error behaviour follows the reference: Open() returns false, Finish() throws
 * std::runtime_error; the C shim returns SSTC_* codes instead.
 */
#ifndef SSTC_TABLE_H
#define SSTC_TABLE_H

#include "sstcodec.h"

#ifdef __cplusplus
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace sstc {

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
  ~TableBuilder();
  TableBuilder(const TableBuilder &) = delete;
  TableBuilder &operator=(const TableBuilder &) = delete;

  bool Open();
  /* value.data() == nullptr -> no value fields (a DELETE), like the reference. */
  void AddEntry(std::string_view key, std::string_view value, uint64_t txn_id, uint8_t value_type);
  void FlushBlock();
  void Finish();

  std::string_view GetSmallestKey() const { return table_smallest_key_; }
  std::string_view GetLargestKey() const { return table_largest_key_; }
  std::string_view GetFilename() const { return filename_; }
  uint64_t GetFileSize() const { return current_offset_ + 1; } /* table_builder.cc:228 */
  uint64_t GetDataSize() const { return data_size_; }
  uint64_t GetNumBlocks() const { return blk_first_.size() - 1; }

private:
  std::string filename_;
  uint64_t threshold_;
  sstc_ctx *ctx_;
  int fd_ = -1;
  // pending records (host SoA + arenas)
  std::vector<uint8_t> type_;
  std::vector<uint32_t> key_len_, val_len_;
  std::vector<uint64_t> txn_, key_off_, val_off_;
  std::vector<uint8_t> keys_, vals_;
  std::vector<uint64_t> blk_first_{0};
  uint64_t block_size_ = 0; /* sum(entry_size + 16) of the open block */
  std::string table_smallest_key_, table_largest_key_;
  uint64_t min_txn_ = UINT64_MAX, max_txn_ = 0;
  uint64_t data_size_ = 0;
  uint64_t current_offset_ = 0;
};

class TableReader {
public:
  /* file_size as recorded by TableBuilder::GetFileSize() (bytes + 1). */
  static TableReader *Open(const std::string &filename, uint64_t file_size, sstc_ctx *ctx);
  ~TableReader();

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
