// minibase.hpp -- C++ mirror of the reference's scan/index operator surface,
// executed by the MI355X kernels behind include/mbx.h.
//
// Class and method names, argument meaning and error behaviour follow the
// Java reference (R/ = minijava/src): a caller of
//   iterator::ColumnarFileScan   (R/iterator/ColumnarFileScan.java:51-188)
//   iterator::ColumnarColumnScan (R/iterator/ColumnarColumnScan.java:39-211)
//   index::ColumnIndexScan       (R/index/ColumnIndexScan.java:76-741, Bitmap branch)
//   index::ColumnarIndexScan     (R/index/ColumnarIndexScan.java:79-370)
// builds the same CondExpr[] / FldSpec[] and drives get_next() / close() /
// restart() exactly as with the Java classes.  Rows are never evaluated here:
// every predicate, BitSet operation and projection is a kernel launch.
//
// The storage layer below the scans (DB file, BufMgr, heap files) is out of
// scope for the GPU build: columnar::Columnarfile holds the decoded columns
// of a file in a process-wide registry (the stand-in for SystemDefs'
// JavabaseDB) and stages them to HBM once.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mbx.h"
#include "../../include/mbx_db.h"

// Everything lives in `minibase::` (the Java packages become nested
// namespaces; `index` would otherwise collide with POSIX index(3)).
namespace minibase {

namespace chainexception {
// R/chainexception/ChainException.java:11 -- every checked exception's root.
class ChainException : public std::runtime_error {
 public:
  explicit ChainException(const std::string& msg, int code = 0) : std::runtime_error(msg), code(code) {}
  int code;  // MBX_E_* when raised from the device layer
};
}  // namespace chainexception

namespace global {
struct AttrType {  // R/global/AttrType.java:45-49
  enum { attrString = 0, attrInteger = 1, attrReal = 2, attrSymbol = 3, attrNull = 4 };
  int attrType;
  AttrType(int t = attrNull) : attrType(t) {}
};
struct AttrOperator {  // R/global/AttrOperator.java:98-106
  enum { aopEQ = 0, aopLT = 1, aopGT = 2, aopNE = 3, aopLE = 4, aopGE = 5, aopNOT = 6, aopNOP = 7, opRANGE = 8 };
  int attrOperator;
  AttrOperator(int o = aopEQ) : attrOperator(o) {}
  static AttrOperator findOperator(const std::string& op);  // :154-172
  std::string toString() const;
};
struct IndexType {  // R/global/IndexType.java:10-13
  enum { None = 0, B_Index = 1, Hash = 2, Bitmap = 3 };
  int indexType;
  IndexType(int t = None) : indexType(t) {}
  std::string toString() const;
};
struct TID {  // R/global/TID.java: numRIDs + position
  int numRIDs = 0;
  int64_t position = -1;
};
// SystemDefs (R/global/SystemDefs.java:6-9): the process-wide engine state;
// here the GPU context every operator launches on.
// SystemDefs(dbname, num_pgs, ...) (R/global/SystemDefs.java:19-80): the
// open Minibase DB file (JavabaseDB) and the GPU context.  open() creates the
// file with num_pgs pages when it does not exist (BatchInsert passes
// 1024*1024), else opens it; files stay open until shutdown().
class SystemDefs {
 public:
  static mbx_ctx* ctx();
  static mbx_db* open(const std::string& dbname, int num_pgs);
  static mbx_db* db();  // the DB opened last (JavabaseDB)
  static bool exists(const std::string& dbname);
  static void shutdown();
};

// The GPUs a sharded scan runs on: one context per
// shard -- shard g on device g % (visible devices) -- and, when every shard
// has a device of its own, one RCCL clique over them (mbx_comm_init_all),
// owned here and shared by every sharded scan of the process (a context
// holds at most one communicator).  Cached per shard count.
class GpuSet {
 public:
  static GpuSet& get(int nshards);
  const std::vector<mbx_ctx*>& ctxs() const { return ctxs_; }
  const std::vector<mbx_comm*>& comms() const { return comms_; }  // empty: devices repeat
  ~GpuSet();

 private:
  std::vector<mbx_ctx*> ctxs_;
  std::vector<mbx_comm*> comms_;
};
}  // namespace global

namespace heap {
// The projected output tuple (iterator's Jtuple).  Field accessors mirror
// R/heap/Tuple.java:194-343 (1-based field numbers).
class Tuple {
 public:
  void setHdr(const std::vector<global::AttrType>& types, const std::vector<short>& str_sizes);
  // the accessors run once per field per delivered row: inline, with the
  // reference's field-number / type checks (FieldNumberOutOfBoundException,
  // UnknowAttrType) thrown out of line
  int getIntFld(int fldNo) const {
    check(fldNo, global::AttrType::attrInteger);
    return ints_[(size_t)fldNo - 1];
  }
  float getFloFld(int fldNo) const {
    check(fldNo, global::AttrType::attrReal);
    return reals_[(size_t)fldNo - 1];
  }
  std::string getStrFld(int fldNo) const;
  void setIntFld(int fldNo, int v) {
    check(fldNo, global::AttrType::attrInteger);
    ints_[(size_t)fldNo - 1] = v;
  }
  void setFloFld(int fldNo, float v) {
    check(fldNo, global::AttrType::attrReal);
    reals_[(size_t)fldNo - 1] = v;
  }
  void setStrFld(int fldNo, const std::string& v);
  void setStrFld(int fldNo, const char* p, size_t n);  // no temporary std::string
  // fields 1..n from row i of n int columns (Projection.Project's copy of an
  // all-int projection): one range check against the header's leading int
  // fields instead of one per field
  void setIntFlds(const int32_t* const* cols, int64_t i, int n) {
    if (__builtin_expect(n > int_prefix_, 0)) bad_field(int_prefix_ + 1, global::AttrType::attrInteger);
    int32_t* d = ints_.data();
    for (int j = 0; j < n; j++) d[j] = cols[j][i];
  }
  short noOfFlds() const { return (short)kinds_.size(); }
  int size() const;  // header + fields, as Tuple.size() with setHdr's layout
 private:
  void check(int fldNo, int type) const {
    if (__builtin_expect(fldNo < 1 || fldNo > (int)kinds_.size() || kinds_[(size_t)fldNo - 1] != type, 0))
      bad_field(fldNo, type);
  }
  [[noreturn]] void bad_field(int fldNo, int type) const;
  std::vector<int> kinds_;  // types_[i].attrType
  int int_prefix_ = 0;      // leading attrInteger fields
  std::vector<global::AttrType> types_;
  std::vector<short> str_sizes_;
  std::vector<int32_t> ints_;
  std::vector<float> reals_;
  std::vector<std::string> strs_;
};
}  // namespace heap

namespace iterator {
using global::AttrOperator;
using global::AttrType;
using global::IndexType;

class FileScanException : public chainexception::ChainException {
  using ChainException::ChainException;
};
class PredEvalException : public chainexception::ChainException {
  using ChainException::ChainException;
};
class UnknowAttrType : public chainexception::ChainException {
  using ChainException::ChainException;
};
class FieldNumberOutOfBoundException : public chainexception::ChainException {
  using ChainException::ChainException;
};
class InvalidRelation : public chainexception::ChainException {
  using ChainException::ChainException;
};
// java.lang.ArrayIndexOutOfBoundsException (unchecked, not a ChainException)
class ArrayIndexOutOfBoundsException : public std::out_of_range {
  using std::out_of_range::out_of_range;
};
// a plain java.lang.Exception (e.g. Heapfile.findPosition's "Invalid RID")
class JavaException : public std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct RelSpec {  // R/iterator/RelSpec.java
  enum { outer = 0, innerRel = 1 };
  int key;
  RelSpec(int k = outer) : key(k) {}
};
struct FldSpec {  // R/iterator/FldSpec.java
  RelSpec relation;
  int offset;  // 1-based
  FldSpec(RelSpec r = RelSpec(), int off = 1) : relation(r), offset(off) {}
};
struct Operand {  // R/iterator/Operand.java
  FldSpec symbol;
  std::string string;  // modified UTF-8 bytes (ASCII text is its own encoding)
  int integer = 0;
  float real = 0.0f;
};
// R/iterator/CondExpr.java:12-57: one OR-linked disjunct list element.
struct CondExpr {
  AttrOperator op;
  AttrType type1, type2;
  Operand operand1, operand2;
  IndexType indexType;
  CondExpr* next = nullptr;
};

// CondExpr[] (null-terminated array of OR-chains) -> the C-ABI's flat CNF.
struct CnfImage {
  std::vector<mbx_condexpr> conds;
  std::vector<int32_t> offsets;
  mbx_cnf view() const;
};
CnfImage flatten(CondExpr* const* filter, int fld_remap_from = 0, int fld_remap_to = 0);

// R/iterator/Iterator.java:12-141
class Iterator {
 public:
  virtual ~Iterator() = default;
  virtual heap::Tuple* get_next() = 0;
  virtual void close() = 0;
  virtual void restart() = 0;
  virtual int getTupleSize() = 0;

 protected:
  bool closeFlag = false;
};
}  // namespace iterator

namespace columnar {
using global::AttrType;

// A device BitSet handle (java.util.BitSet on the GPU).
class DeviceBitSet {
 public:
  DeviceBitSet() = default;
  explicit DeviceBitSet(mbx_bitmap* b) : b_(b) {}
  ~DeviceBitSet();
  DeviceBitSet(const DeviceBitSet&) = delete;
  DeviceBitSet& operator=(const DeviceBitSet&) = delete;
  mbx_bitmap* get() const { return b_; }
  int64_t cardinality() const;
  std::vector<uint64_t> toLongArray() const;  // BitSet.toLongArray()
  std::vector<int64_t> positions(int64_t row_offset = 0) const;

 private:
  mbx_bitmap* b_ = nullptr;
};
using BitSetPtr = std::shared_ptr<DeviceBitSet>;

// R/columnar/Columnarfile.java: the file's schema + its HBM image.
// A Columnarfile of a Minibase DB file (include/mbx_db.h); its rows are
// staged to HBM by the GPU page decoder on first use after a change.
class Columnarfile {
 public:
  // open an existing file (:194-300)
  Columnarfile(mbx_db* db, const std::string& name);
  // create (:60-192), or open it when it exists with the same arity
  Columnarfile(mbx_db* db, const std::string& name, int numColumns, const std::vector<std::string>& colNames,
               const std::vector<AttrType>& types, const std::vector<short>& sizes);

  void insertColumns(const std::vector<std::vector<int32_t>>& ints, const std::vector<std::vector<float>>& reals,
                     const std::vector<std::vector<std::string>>& strs, int64_t nrows);
  int64_t getTupleCnt() const;  // live tuples
  int64_t positions() const;     // highest position + 1 (bits of every BitSet)
  int getFieldCount() const;
  std::vector<AttrType> getAttributeTypes() const;
  std::vector<short> getStringSizes() const;  // sizes of the string columns, in order
  std::vector<short> getAttrSizes() const;
  int colNameToIndex(const std::string& name) const;
  std::string indexToColName(int idx) const;
  const std::string& get_fileName() const { return name_; }
  mbx_table* table() const;  // staged on first use
  mbx_db* db() const;        // the DB file (shards stage their row ranges from it)

  // bitmap index registry (createBitMapIndex :698-753, getBitmapIndex :1103-1127,
  // getBitmapValues :1138)
  void createBitMapIndex(int colNo);
  bool bitmapIndexExists(int colNo) const;
  std::vector<std::string> getBitmapValues(int colNo) const;  // registered value keys
  BitSetPtr getBitmapIndex(int colNo, const std::string& key) const;  // empty BitSet if absent
  BitSetPtr getMarkedDeleted() const;  // may be null (nothing deleted)
  void markTupleDeleted(int64_t position);
  void invalidate();  // the DB file changed under this object: re-stage on next use

  struct Impl;

 private:
  std::string name_;
  std::shared_ptr<Impl> impl_;
};

std::string int_key(int v);
}  // namespace columnar

namespace iterator {

// get_next() over an mbx_cursor (Iterator.get_next, R/iterator/Iterator.java:12-141):
// batches of kRows positions + projected rows come out of the cursor's
// double-buffered delivery; fill() writes the current row into Jtuple.
class CursorBatches {
 public:
  // rows per batch: one packed device -> pinned copy each; 256 Ki rows copy
  // at 42 GB/s vs 24 GB/s for 64 Ki (bench_delivery, profiles/r04/b)
  static constexpr int64_t kRows = 262144;
  CursorBatches() = default;
  ~CursorBatches() { close(); }
  CursorBatches(const CursorBatches&) = delete;
  CursorBatches& operator=(const CursorBatches&) = delete;
  // takes ownership of c; cols = the projected file columns
  void reset(mbx_cursor* c, const std::vector<AttrType>& types, const std::vector<short>& sizes,
             const std::vector<int32_t>& cols);
  bool open() const { return cur_ != nullptr; }
  int64_t count() const;
  // the next row; false at the end of the stream (a new batch every kRows rows)
  bool next() {
    if (i_ < n_) {
      i_++;
      return true;
    }
    return next_batch();
  }
  int64_t position() const { return vids_[i_ - 1]; }
  // the current row into J's fields 1..n (Projection.Project's copy)
  void fill(heap::Tuple& J) const {
    const int64_t i = i_ - 1;
    if (all_int_) {
      J.setIntFlds(reinterpret_cast<const int32_t* const*>(vcols_.data()), i, (int)vcols_.size());
      return;
    }
    for (size_t j = 0; j < kind_.size(); j++) {
      const uint8_t* p = (const uint8_t*)vcols_[j] + i * width_[j];
      switch (kind_[j]) {
        case AttrType::attrInteger: {
          int32_t v;
          memcpy(&v, p, 4);
          J.setIntFld((int)j + 1, v);
          break;
        }
        case AttrType::attrReal: {
          float v;
          memcpy(&v, p, 4);
          J.setFloFld((int)j + 1, v);
          break;
        }
        default:
          J.setStrFld((int)j + 1, (const char*)p, strnlen((const char*)p, (size_t)width_[j]));
      }
    }
  }
  void restart();
  void close();

 private:
  bool next_batch();
  mbx_cursor* cur_ = nullptr;
  std::vector<AttrType> types_;
  std::vector<short> sizes_;
  std::vector<int32_t> cols_;
  std::vector<int> kind_;    // per projected column: its AttrType code
  std::vector<int64_t> width_;  // per projected column: bytes per row in the batch
  bool all_int_ = false;        // every projected column is attrInteger (fill's bulk copy)
  // the current batch in the cursor's pinned buffer (mbx_cursor_next_view:
  // rows are read in place, valid until the next batch)
  const int64_t* vids_ = nullptr;
  std::vector<const void*> vcols_;
  int64_t n_ = 0, i_ = 0;
};

// R/iterator/ColumnarFileScan.java:51-99 (+ get_next :156-172, get_next_tid :174-188)
class ColumnarFileScan : public Iterator {
 public:
  ColumnarFileScan(const std::string& file_name, const std::vector<AttrType>& in1,
                   const std::vector<short>& s1_sizes, short len_in1, int n_out_flds,
                   const std::vector<FldSpec>& proj_list, CondExpr* const* outFilter);
  // per delivered row: inline, and final so a caller holding the concrete
  // class calls it directly
  heap::Tuple* get_next() final {
    if (__builtin_expect(!rows_.open(), 0)) open_rows();
    if (!rows_.next()) return nullptr;
    rows_.fill(Jtuple_);
    return &Jtuple_;
  }
  global::TID get_next_tid();
  void close() override;
  void restart() override;
  int getTupleSize() override;
  int64_t resultCount() const;  // COUNT of the whole selection (one kernel)
  columnar::BitSetPtr selection() const { return sel_; }

 private:
  void open_rows();
  columnar::Columnarfile f_;
  std::vector<AttrType> in1_;
  std::vector<FldSpec> perm_mat_;
  heap::Tuple Jtuple_;
  mbx_plan* plan_ = nullptr;
  columnar::BitSetPtr sel_;
  std::vector<int32_t> proj_cols_;
  std::vector<AttrType> types_;  // the file's schema, read once (get_next runs per row)
  std::vector<short> sizes_;
  CursorBatches rows_;           // opened at the first get_next / get_next_tid
};

// R/iterator/ColumnarColumnsScan.java:39-257: a CNF over the tuple of the
// columns colNos (CondExpr field i = colNos[i-1]), one ColumnScan per column
// in lockstep (deleted positions skipped), late-materialised out_indexes.
// Reference behaviour kept (drop-in):
//  * the constructor's dest_s_sizes loop indexes an array sized by the number
//    of string columns with the column's position (:77-82): a string column
//    at position >= that count throws ArrayIndexOutOfBoundsException, i.e.
//    only colNos whose string columns come first construct (NljQuery's
//    TreeSet order over a schema with its strings first, R/input/NljQuery.java:245-268);
//  * get_next_tid (:205-224) asks the heapfile of colNos[0] for the position
//    of the RID the LAST column's scan returned: for colNos[0] != colNos[last]
//    that page is not in the file and findPosition throws "Invalid RID"
//    (R/heap/Heapfile.java:262-273) at the first selected row;
//  * Jtuple's types come from proj_list, its values from out_indexes (:57-60,
//    :191-199).
// Predicate, deleted skip and projection run on the GPU like ColumnarFileScan.
class ColumnarColumnsScan : public Iterator {
 public:
  ColumnarColumnsScan(columnar::Columnarfile* cf, const std::vector<int>& colNos, int n_out_flds,
                      const std::vector<int>& out_indexes, const std::vector<FldSpec>& proj_list,
                      CondExpr* const* outFilter);
  // the delete-query form (:103-154): no projection, get_next_tid only
  ColumnarColumnsScan(columnar::Columnarfile* cf, const std::vector<int>& colNos, CondExpr* const* outFilter);
  heap::Tuple* get_next() override;
  global::TID get_next_tid();
  void close() override;
  void restart() override;
  int getTupleSize() override;
  columnar::BitSetPtr selection() const { return inner_->selection(); }

 private:
  void init(columnar::Columnarfile* cf, const std::vector<int>& colNos, int n_out_flds,
            const std::vector<int>& out_indexes, CondExpr* const* outFilter);
  std::vector<int> colNos_;
  std::unique_ptr<ColumnarFileScan> inner_;
  heap::Tuple Jtuple_;  // typed by proj_list (getTupleSize)
  bool has_proj_ = false;
};

// R/iterator/ColumnarColumnScan.java:39-88: predicate on one column (field 1
// of the CondExpr refers to column colNo), late-materialised out_indexes.
class ColumnarColumnScan : public Iterator {
 public:
  ColumnarColumnScan(columnar::Columnarfile* cf, int colNo, int n_out_flds, const std::vector<int>& out_indexes,
                     const std::vector<FldSpec>& proj_list, CondExpr* const* outFilter);
  heap::Tuple* get_next() override;
  global::TID get_next_tid();
  void close() override;
  void restart() override;
  int getTupleSize() override;

 private:
  std::unique_ptr<ColumnarFileScan> inner_;
};
}  // namespace iterator

namespace index {
using global::AttrType;
using global::IndexType;
using iterator::CondExpr;
using iterator::FldSpec;

class IndexException : public chainexception::ChainException {
  using ChainException::ChainException;
};
class UnknownIndexTypeException : public chainexception::ChainException {
  using ChainException::ChainException;
};

// R/index/ColumnIndexScan.java:76-272 (Bitmap branch): `col op literal`
// over the bitmap indexes; positions skip deleted rows.
class ColumnIndexScan : public iterator::Iterator {
 public:
  ColumnIndexScan(IndexType index, columnar::Columnarfile* cf, const std::string& indName,
                  const std::vector<AttrType>& types, const std::vector<short>& str_sizes, int noInFlds, int noOutFlds,
                  const std::vector<int>& outIndexes, const std::vector<FldSpec>& outFlds, CondExpr* const* selects,
                  int fldNum, bool indexOnly);
  // the short form ColumnarIndexScan uses (:185-272): positions only
  ColumnIndexScan(IndexType index, columnar::Columnarfile* cf, const std::string& indName,
                  const std::vector<AttrType>& types, const std::vector<short>& str_sizes, int noInFlds,
                  CondExpr* const* selects, int fldNum);
  heap::Tuple* get_next() override;
  global::TID get_next_tid();
  columnar::BitSetPtr getPositionsOfIndexScan();  // :647-654
  void close() override;
  void restart() override;
  int getTupleSize() override;

  // getBitSet's value selection (:656-740): the bitmaps whose value v
  // satisfies `v op literal`
  static std::vector<columnar::BitSetPtr> valueBitmaps(const columnar::Columnarfile& cf, int colNo,
                                                       const CondExpr& e);
  // the same selection as value keys (BitMapFile cf.bm.<col>.<key>)
  static std::vector<std::string> valueKeys(const columnar::Columnarfile& cf, int colNo, const CondExpr& e);

 private:
  void open_cursor();
  columnar::Columnarfile* f_;
  int colNo_;
  std::vector<int> outIndexes_;
  std::vector<AttrType> types_;
  bool index_only_ = false;
  CondExpr sel_{};
  std::vector<columnar::BitSetPtr> values_;  // the value bitmaps OR-ed by getBitSet
  columnar::BitSetPtr positions_;            // their OR minus deleted, built on first use
  heap::Tuple Jtuple_;
  iterator::CursorBatches rows_;             // get_next: one k_cnf_select launch
};

// R/index/ColumnarIndexScan.java:79-182 (+ getOutputPositions :270, get_next :287-308)
class ColumnarIndexScan : public iterator::Iterator {
 public:
  ColumnarIndexScan(columnar::Columnarfile* cf, const std::vector<int>& fldNums,
                    const std::vector<IndexType>& indexTypes, const std::vector<std::string>& indNames,
                    const std::vector<AttrType>& types, const std::vector<short>& str_sizes, int noInFlds,
                    int noOutFlds, const std::vector<int>& out_indexes, const std::vector<FldSpec>& outFlds,
                    CondExpr* const* selects, bool indexOnly);
  // the CNF's BitSet (on the one-launch path it is formed on first request)
  columnar::BitSetPtr getOutputPositions();
  heap::Tuple* get_next() final {  // per delivered row: inline (ColumnarFileScan::get_next)
    if (__builtin_expect(!rows_.open(), 0)) open_cursor();
    if (!rows_.next()) return nullptr;
    rows_.fill(Jtuple_);
    return &Jtuple_;
  }
  global::TID get_next_tid();
  void close() override;
  void restart() override;
  int getTupleSize() override;
  // true: no repeated constraint -- CNF, positions and projection in ONE
  // kernel launch (mbx_cnf_cursor_open / k_cnf_select); false: the
  // reference's step-wise BitSet objects (its duplicate-constraint cache)
  bool usedFusedCnf() const { return fused_; }

 private:
  void open_cursor();
  columnar::Columnarfile* f_;
  std::vector<int> outIndexes_;
  std::vector<AttrType> types_;
  std::vector<std::vector<columnar::BitSetPtr>> lists_;  // fused: bitmaps per conjunct
  columnar::BitSetPtr output_;
  heap::Tuple Jtuple_;
  iterator::CursorBatches rows_;
  bool fused_ = false;
};
// ColumnarIndexScan over row-range shards of one Columnarfile, one shard per
// GPU: shard g holds positions
// [s_g, s_{g+1}) (mbx_shard_bounds: multiples of 64), staged straight from
// the DB file by range (mbx_db_stage_range) with its slice of every BitMapFile
// the CNF names and of cf.md (mbx_db_bitmap_stage_range).  Every shard runs
// the one-launch CNF + projection (mbx_cnf_cursor_launch) -- all GPUs in
// flight together -- then ONE grouped RCCL all-gather of the per-shard counts
// (mbx_comm_allgather_count_all) gives every shard its offset in the output;
// get_next() walks the shards in order, which is the reference's ascending
// nextSetBit order (R/index/ColumnarIndexScan.java:130-181, 270, 287-308).
// Without a clique (shards sharing a device) the counts are read per shard.
// Terms: Bitmap (value-set OR, ColumnIndexScan.getBitSet) or B_Index (the
// term's scan on the shard); a repeated constraint (the reference's mutable
// cache, :147-172) throws -- use ColumnarIndexScan.
class ShardedColumnarIndexScan : public iterator::Iterator {
 public:
  ShardedColumnarIndexScan(columnar::Columnarfile* cf, global::GpuSet& gpus, int noOutFlds,
                           const std::vector<int>& out_indexes, const std::vector<FldSpec>& outFlds,
                           CondExpr* const* selects);
  ~ShardedColumnarIndexScan();
  heap::Tuple* get_next() override;
  global::TID get_next_tid();
  void close() override;
  void restart() override;
  int getTupleSize() override;
  int64_t count() const { return total_; }
  const std::vector<int64_t>& shardOffsets() const { return offsets_; }  // nshards + 1
  bool exchangedOverRccl() const { return rccl_; }

 private:
  bool advance();
  columnar::Columnarfile* f_;
  std::vector<int> outIndexes_;
  heap::Tuple Jtuple_;
  std::vector<mbx_table*> tables_;
  std::vector<std::vector<mbx_bitmap*>> bitmaps_;  // per shard, all staged slices
  std::vector<std::unique_ptr<iterator::CursorBatches>> rows_;
  std::vector<int64_t> offsets_;
  int64_t total_ = 0;
  size_t shard_ = 0;
  bool rccl_ = false;
};
}  // namespace index

}  // namespace minibase
