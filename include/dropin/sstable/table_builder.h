/*
 * include/dropin/sstable/table_builder.h — the drop-in for the reference's
 * sstable/table_builder.h (/root/reference/sstable/table_builder.h:63-151).
 *
 * Put this directory first on the include path of the engine's build and
 * db/compact.cc / db/db_impl.cc compile UNCHANGED: every
 * `sstable::TableBuilder` they construct (compact.cc:238-239,280-281,
 * db_impl.cc:410) is this framework's GPU-encoding builder.  It is a class
 * (not an alias) because db/db_impl.h:41-45 forward-declares
 * `class TableBuilder;` in kvs::sstable.  The include guard is the
 * reference's, so the reference header is never seen twice.
 *
 * Surface used by the engine (table_builder.h:65-117): the constructor
 * (std::string&&, const db::Config*) — reads Config::GetSSTBlockSize(); Open;
 * AddEntry(string_view, string_view, TxnId, db::ValueType) — a null
 * value.data() means no value fields, as block_builder.cc:19-21,56; FlushBlock;
 * Finish (throws std::runtime_error on failure, like table_builder.cc:155-170);
 * GetSmallestKey / GetLargestKey / GetFilename / GetFileSize (bytes + 1,
 * table_builder.cc:228) / GetDataSize.  Blocks are encoded on the GPU at
 * Finish() (sstc_encode_blocks through the calling thread's context) and
 * written with one pwrite + fsync.
 */
#ifndef SSTABLE_TABLE_BUILDER_H
#define SSTABLE_TABLE_BUILDER_H

#include "common/macros.h"
#include "db/status.h"
#include "sstc_table.h"

namespace kvs {

/* the forward declarations the reference header provides to its includers
 * (table_builder.h:14-27,57-58; db/version.h:113 relies on db::Config) */
namespace db {
class AccessFile;
class BaseIterator;
class Compact;
class Config;
} // namespace db
namespace io {
class ReadOnlyFile;
class WriteOnlyFile;
} // namespace io

namespace sstable {

class BlockBuilder;
class BlockIndex;

class TableBuilder : public ::sstc::TableBuilder {
public:
  using ::sstc::TableBuilder::TableBuilder;
};

} // namespace sstable
} // namespace kvs

#endif // SSTABLE_TABLE_BUILDER_H
