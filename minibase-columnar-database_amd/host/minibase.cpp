// minibase.cpp -- implementation of the C++ operator mirror (minibase.hpp).
// Every row-level computation is a libmbx kernel; this file only translates
// the reference's objects (CondExpr chains, FldSpec lists, Columnarfile
// metadata) into C-ABI calls and walks result batches for get_next().
#include "minibase.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <sstream>

namespace minibase {

namespace {

template <class E>
void chk(int rc, const std::string& what) {
  if (rc < 0) throw E(what + ": " + mbx_last_error(), rc);
}

// Java String.compareTo over modified UTF-8 payloads: decode to UTF-16 code
// units and compare (used only for value-dictionary decisions, never rows).
std::vector<uint16_t> utf16_of(const std::string& s) {
  std::vector<uint16_t> u;
  const unsigned char* p = (const unsigned char*)s.data();
  size_t i = 0, n = s.size();
  while (i < n) {
    unsigned c = p[i];
    if (c < 0x80) {
      u.push_back((uint16_t)c);
      i += 1;
    } else if ((c & 0xE0) == 0xC0 && i + 1 < n) {
      u.push_back((uint16_t)(((c & 0x1F) << 6) | (p[i + 1] & 0x3F)));
      i += 2;
    } else if (i + 2 < n) {
      u.push_back((uint16_t)(((c & 0x0F) << 12) | ((p[i + 1] & 0x3F) << 6) | (p[i + 2] & 0x3F)));
      i += 3;
    } else {
      break;
    }
  }
  return u;
}

int java_compare(const std::string& a, const std::string& b) {
  const auto x = utf16_of(a), y = utf16_of(b);
  const size_t lim = std::min(x.size(), y.size());
  for (size_t k = 0; k < lim; k++)
    if (x[k] != y[k]) return x[k] < y[k] ? -1 : 1;
  return x.size() == y.size() ? 0 : (x.size() < y.size() ? -1 : 1);
}

mbx_ctx* g_ctx = nullptr;

}  // namespace

// ------------------------------------------------------------------ global

namespace global {

mbx_ctx* SystemDefs::ctx() {
  if (!g_ctx) {
    const char* d = getenv("MBX_DEVICE");
    chk<chainexception::ChainException>(mbx_init(d ? atoi(d) : 0, &g_ctx), "SystemDefs: GPU context");
  }
  return g_ctx;
}

static std::map<int, std::unique_ptr<GpuSet>>& gpu_sets() {
  static std::map<int, std::unique_ptr<GpuSet>>* sets = new std::map<int, std::unique_ptr<GpuSet>>();
  return *sets;  // released by SystemDefs::shutdown, never at static destruction
}

GpuSet& GpuSet::get(int nshards) {
  auto& sets = gpu_sets();
  if (nshards < 1) throw chainexception::ChainException("GpuSet: " + std::to_string(nshards) + " shards");
  auto it = sets.find(nshards);
  if (it != sets.end()) return *it->second;
  std::unique_ptr<GpuSet> g(new GpuSet());
  int32_t nd = 0;
  chk<chainexception::ChainException>(mbx_device_count(&nd), "GpuSet: device count");
  if (nd < 1) throw chainexception::ChainException("GpuSet: no GPU visible");
  for (int i = 0; i < nshards; i++) {
    mbx_ctx* c = nullptr;
    chk<chainexception::ChainException>(mbx_init(i % nd, &c), "GpuSet: context for shard " + std::to_string(i));
    g->ctxs_.push_back(c);
  }
  if (nshards <= nd) {  // a device per shard: one RCCL clique
    g->comms_.assign((size_t)nshards, nullptr);
    chk<chainexception::ChainException>(mbx_comm_init_all(g->ctxs_.data(), nshards, g->comms_.data()),
                                        "GpuSet: RCCL clique");
  }
  GpuSet& ref = *g;
  sets[nshards] = std::move(g);
  return ref;
}

GpuSet::~GpuSet() {
  for (mbx_comm* m : comms_) mbx_comm_free(m);
  for (mbx_ctx* c : ctxs_) mbx_free(c);
}

}  // namespace global
namespace columnar {
void close_all_files();
}
namespace global {

static std::map<std::string, mbx_db*>& open_dbs() {
  static std::map<std::string, mbx_db*> m;
  return m;
}
static mbx_db* g_db = nullptr;

bool SystemDefs::exists(const std::string& dbname) {
  FILE* f = fopen(dbname.c_str(), "rb");
  if (f) fclose(f);
  return f != nullptr;
}

mbx_db* SystemDefs::open(const std::string& dbname, int num_pgs) {
  auto& m = open_dbs();
  auto it = m.find(dbname);
  if (it != m.end()) return g_db = it->second;
  mbx_db* db = nullptr;
  if (exists(dbname))
    chk<chainexception::ChainException>(mbx_db_open(dbname.c_str(), &db), "DB.openDB " + dbname);
  else
    chk<chainexception::ChainException>(mbx_db_create(dbname.c_str(), num_pgs, &db), "DB.openDB " + dbname);
  m[dbname] = db;
  return g_db = db;
}

mbx_db* SystemDefs::db() { return g_db; }

// flushAllPages + close: every device object goes before the context
static std::map<int, std::unique_ptr<GpuSet>>& gpu_sets();

void SystemDefs::shutdown() {
  columnar::close_all_files();
  for (auto& kv : open_dbs()) mbx_db_close(kv.second);
  open_dbs().clear();
  g_db = nullptr;
  gpu_sets().clear();
  if (g_ctx) mbx_free(g_ctx);
  g_ctx = nullptr;
}

AttrOperator AttrOperator::findOperator(const std::string& op) {
  if (op == "=") return AttrOperator(aopEQ);
  if (op == "<") return AttrOperator(aopLT);
  if (op == ">") return AttrOperator(aopGT);
  if (op == "!=") return AttrOperator(aopNE);
  if (op == ">=") return AttrOperator(aopGE);
  if (op == "<=") return AttrOperator(aopLE);
  throw chainexception::ChainException("unsupported or invalid operator");
}

std::string AttrOperator::toString() const {
  static const char* n[] = {"aopEQ", "aopLT", "aopGT", "aopNE", "aopLE", "aopGE", "aopNOT", "aopNOP", "opRANGE"};
  if (attrOperator >= 0 && attrOperator <= 8) return n[attrOperator];
  return "Unexpected AttrOperator " + std::to_string(attrOperator);
}

std::string IndexType::toString() const {
  switch (indexType) {
    case None: return "None";
    case B_Index: return "B_Index";
    case Hash: return "Hash";
    case Bitmap: return "Bitmap";
  }
  return "Unexpected IndexType " + std::to_string(indexType);
}

}  // namespace global

// ------------------------------------------------------------------- heap

namespace heap {

void Tuple::setHdr(const std::vector<global::AttrType>& types, const std::vector<short>& str_sizes) {
  types_ = types;
  kinds_.clear();
  for (const auto& t : types) kinds_.push_back(t.attrType);
  int_prefix_ = 0;
  while (int_prefix_ < (int)kinds_.size() && kinds_[(size_t)int_prefix_] == global::AttrType::attrInteger) int_prefix_++;
  str_sizes_ = str_sizes;
  ints_.assign(types.size(), 0);
  reals_.assign(types.size(), 0.0f);
  strs_.assign(types.size(), std::string());
}

void Tuple::bad_field(int fldNo, int type) const {
  if (fldNo < 1 || fldNo > (int)types_.size())
    throw iterator::FieldNumberOutOfBoundException("Tuple: field number " + std::to_string(fldNo) + " out of bound");
  throw iterator::UnknowAttrType("Tuple: field " + std::to_string(fldNo) + " has another type (" +
                                 std::to_string(type) + " asked)");
}
std::string Tuple::getStrFld(int f) const {
  check(f, global::AttrType::attrString);
  return strs_[(size_t)f - 1];
}
void Tuple::setStrFld(int f, const std::string& v) {
  check(f, global::AttrType::attrString);
  strs_[(size_t)f - 1] = v;
}
void Tuple::setStrFld(int f, const char* p, size_t n) {
  check(f, global::AttrType::attrString);
  strs_[(size_t)f - 1].assign(p, n);
}

int Tuple::size() const {
  // Tuple.setHdr layout (R/heap/Tuple.java:369-411): 2 + 2*(n+1) header bytes
  int sz = 2 + 2 * ((int)types_.size() + 1);
  size_t k = 0;
  for (const auto& t : types_) {
    if (t.attrType == global::AttrType::attrString) sz += str_sizes_.size() > k ? str_sizes_[k++] + 2 : 2;
    else sz += 4;
  }
  return sz;
}

}  // namespace heap

// --------------------------------------------------------------- columnar

namespace columnar {

std::string int_key(int v) { return std::to_string(v); }

struct Columnarfile::Impl {
  mbx_db* db = nullptr;
  std::string name;
  std::vector<std::string> names;
  std::vector<AttrType> types;
  std::vector<short> sizes;  // attrSizes: 4 or char(n)
  mbx_table* table = nullptr;
  bool dirty = true;  // the DB file changed since the table was staged
  std::map<int, std::map<std::string, BitSetPtr>> bitmaps;  // staged BitMapFiles: col -> value key
  BitSetPtr deleted_bm;
  bool deleted_loaded = false;
  void invalidate() {
    bitmaps.clear();
    deleted_bm.reset();
    deleted_loaded = false;
    dirty = true;
  }
  ~Impl() {
    bitmaps.clear();
    deleted_bm.reset();
    if (table) mbx_table_free(table);
  }
};

// one Impl per (DB, Columnarfile) so every iterator of a session shares the
// staged table and the staged index BitSets
static std::map<std::pair<mbx_db*, std::string>, std::shared_ptr<Columnarfile::Impl>>& registry() {
  static std::map<std::pair<mbx_db*, std::string>, std::shared_ptr<Columnarfile::Impl>> r;
  return r;
}

void close_all_files() { registry().clear(); }

DeviceBitSet::~DeviceBitSet() {
  if (b_) mbx_bitmap_free(b_);
}
int64_t DeviceBitSet::cardinality() const {
  int64_t c = 0;
  mbx_bitmap_info(b_, nullptr, nullptr, &c);
  if (c < 0) {
    std::vector<int64_t> p = positions();
    c = (int64_t)p.size();
  }
  return c;
}

std::vector<uint64_t> DeviceBitSet::toLongArray() const {
  int64_t nw = 0;
  mbx_bitmap_info(b_, nullptr, &nw, nullptr);
  std::vector<uint64_t> w((size_t)nw);
  if (nw) chk<chainexception::ChainException>(mbx_bitmap_download(global::SystemDefs::ctx(), b_, w.data(), nw),
                                              "BitSet download");
  return w;
}

std::vector<int64_t> DeviceBitSet::positions(int64_t row_offset) const {
  int64_t nbits = 0;
  mbx_bitmap_info(b_, &nbits, nullptr, nullptr);
  std::vector<int64_t> ids((size_t)(nbits > 0 ? nbits : 1));
  int64_t n = 0;
  chk<chainexception::ChainException>(
      mbx_bitmap_select(global::SystemDefs::ctx(), b_, row_offset, ids.data(), (int64_t)ids.size(), &n),
      "BitSet nextSetBit");
  ids.resize((size_t)n);
  return ids;
}

static void load_schema(Columnarfile::Impl& I) {
  int32_t n = 0;
  chk<chainexception::ChainException>(mbx_db_columnar_info(I.db, I.name.c_str(), 0, &n, nullptr, nullptr, nullptr,
                                                           nullptr),
                                      "Columnar File does not exist.");
  std::vector<mbx_col_desc> d((size_t)n);
  std::vector<char> names((size_t)n * (MBX_DB_MAX_ATTR_NAME + 1));
  chk<chainexception::ChainException>(mbx_db_columnar_info(I.db, I.name.c_str(), n, &n, d.data(), names.data(),
                                                           nullptr, nullptr),
                                      "Columnarfile " + I.name);
  I.names.clear();
  I.types.clear();
  I.sizes.clear();
  for (int32_t j = 0; j < n; j++) {
    I.names.emplace_back(names.data() + (size_t)j * (MBX_DB_MAX_ATTR_NAME + 1));
    I.types.emplace_back(d[(size_t)j].attr_type);
    I.sizes.push_back((short)d[(size_t)j].size);
  }
}

static std::shared_ptr<Columnarfile::Impl> find_or_open(mbx_db* db, const std::string& name) {
  if (!db) throw chainexception::ChainException("Database does not exist.");
  auto& reg = registry();
  auto it = reg.find({db, name});
  if (it != reg.end()) return it->second;
  auto I = std::make_shared<Columnarfile::Impl>();
  I->db = db;
  I->name = name;
  load_schema(*I);
  reg[{db, name}] = I;
  return I;
}

Columnarfile::Columnarfile(mbx_db* db, const std::string& name) : name_(name) { impl_ = find_or_open(db, name); }

Columnarfile::Columnarfile(mbx_db* db, const std::string& name, int numColumns,
                           const std::vector<std::string>& colNames, const std::vector<AttrType>& types,
                           const std::vector<short>& sizes)
    : name_(name) {
  if ((int)colNames.size() != numColumns || (int)types.size() != numColumns || (int)sizes.size() != numColumns)
    throw chainexception::ChainException("Columns Meta Info lengths are not equal to num columns.");
  int32_t first = -1;
  chk<chainexception::ChainException>(mbx_db_file_entry(db, (name + ".hdr").c_str(), &first), "get_file_entry");
  if (first < 0) {
    std::vector<mbx_col_desc> d((size_t)numColumns);
    std::vector<const char*> nm((size_t)numColumns);
    for (int j = 0; j < numColumns; j++) {
      d[(size_t)j].attr_type = types[(size_t)j].attrType;
      d[(size_t)j].size = sizes[(size_t)j];
      nm[(size_t)j] = colNames[(size_t)j].c_str();
    }
    chk<chainexception::ChainException>(mbx_db_columnar_create(db, name.c_str(), numColumns, d.data(), nm.data()),
                                        "Columnarfile " + name);
  }
  impl_ = find_or_open(db, name);
  if ((int)impl_->types.size() != numColumns) throw chainexception::ChainException("Existing file has diff num of cols");
  for (int j = 0; j < numColumns; j++) {
    if (impl_->types[(size_t)j].attrType != types[(size_t)j].attrType)
      throw chainexception::ChainException("Unmatched Type");
    if (impl_->sizes[(size_t)j] != sizes[(size_t)j]) throw chainexception::ChainException("Unmatched Size");
    if (impl_->names[(size_t)j] != colNames[(size_t)j]) throw chainexception::ChainException("Unmatched Name");
  }
}

void Columnarfile::insertColumns(const std::vector<std::vector<int32_t>>& ints,
                                 const std::vector<std::vector<float>>& reals,
                                 const std::vector<std::vector<std::string>>& strs, int64_t nrows) {
  Impl& I = *impl_;
  std::vector<std::vector<uint8_t>> host(I.types.size());
  std::vector<const void*> p(I.types.size());
  size_t ki = 0, kr = 0, ks = 0;
  for (size_t j = 0; j < I.types.size(); j++) {
    std::vector<uint8_t>& h = host[j];
    if (I.types[j].attrType == AttrType::attrInteger) {
      const auto& v = ints.at(ki++);
      h.resize((size_t)nrows * 4);
      memcpy(h.data(), v.data(), (size_t)nrows * 4);
    } else if (I.types[j].attrType == AttrType::attrReal) {
      const auto& v = reals.at(kr++);
      h.resize((size_t)nrows * 4);
      memcpy(h.data(), v.data(), (size_t)nrows * 4);
    } else {
      const auto& v = strs.at(ks++);
      const size_t sz = (size_t)I.sizes[j];
      h.assign((size_t)nrows * sz, 0);
      for (int64_t r = 0; r < nrows; r++) {
        if (v[(size_t)r].size() > sz) throw chainexception::ChainException("column value exceeds size limit");
        memcpy(h.data() + (size_t)r * sz, v[(size_t)r].data(), v[(size_t)r].size());
      }
    }
    p[j] = h.data();
  }
  chk<chainexception::ChainException>(mbx_db_columnar_insert(I.db, I.name.c_str(), nrows, p.data()),
                                      "Columnarfile.insertTuple");
  I.invalidate();
}

int64_t Columnarfile::getTupleCnt() const {
  int64_t live = 0;
  chk<chainexception::ChainException>(mbx_db_columnar_info(impl_->db, impl_->name.c_str(), 0, nullptr, nullptr,
                                                           nullptr, nullptr, &live),
                                      "getTupleCnt");
  return live;
}

int64_t Columnarfile::positions() const {
  int64_t n = 0;
  mbx_table_info(table(), &n, nullptr, nullptr);
  return n;
}

int Columnarfile::getFieldCount() const { return (int)impl_->types.size(); }
std::vector<AttrType> Columnarfile::getAttributeTypes() const { return impl_->types; }
std::vector<short> Columnarfile::getAttrSizes() const { return impl_->sizes; }

std::vector<short> Columnarfile::getStringSizes() const {
  std::vector<short> s;
  for (size_t j = 0; j < impl_->types.size(); j++)
    if (impl_->types[j].attrType == AttrType::attrString) s.push_back(impl_->sizes[j]);
  return s;
}

int Columnarfile::colNameToIndex(const std::string& name) const {
  for (size_t j = 0; j < impl_->names.size(); j++)
    if (impl_->names[j] == name) return (int)j;
  throw chainexception::ChainException("Column " + name + " does not exist");
}

std::string Columnarfile::indexToColName(int idx) const { return impl_->names.at((size_t)idx); }

// the DB file's pages -> HBM, records decoded by the GPU (mbx_db_stage)
mbx_db* Columnarfile::db() const { return impl_->db; }

mbx_table* Columnarfile::table() const {
  Impl& I = *impl_;
  if (I.table && !I.dirty) return I.table;
  if (I.table) {
    mbx_table_free(I.table);
    I.table = nullptr;
  }
  chk<chainexception::ChainException>(mbx_db_stage(global::SystemDefs::ctx(), I.db, I.name.c_str(), &I.table),
                                      "Columnarfile " + name_ + ": staging to HBM");
  I.dirty = false;
  return I.table;
}

void Columnarfile::createBitMapIndex(int colNo) {
  Impl& I = *impl_;
  if (colNo < 0 || colNo >= (int)I.types.size()) throw chainexception::ChainException("createBitMapIndex: column");
  int32_t n = 0;
  chk<chainexception::ChainException>(
      mbx_db_create_bitmap_index(global::SystemDefs::ctx(), I.db, I.name.c_str(), table(), colNo, &n),
      "createBitMapIndex");
  I.bitmaps.erase(colNo);
}

std::vector<std::string> Columnarfile::getBitmapValues(int colNo) const {
  int32_t cnt = 0;
  int64_t bytes = 0;
  chk<chainexception::ChainException>(
      mbx_db_bitmap_values(impl_->db, impl_->name.c_str(), colNo, nullptr, 0, &cnt, &bytes), "getBitmapValues");
  std::vector<char> buf((size_t)bytes + 1, 0);
  chk<chainexception::ChainException>(
      mbx_db_bitmap_values(impl_->db, impl_->name.c_str(), colNo, buf.data(), bytes, &cnt, &bytes),
      "getBitmapValues");
  std::vector<std::string> v;
  for (size_t k = 0; k < (size_t)bytes;) {
    v.emplace_back(buf.data() + k);
    k += v.back().size() + 1;
  }
  return v;
}

bool Columnarfile::bitmapIndexExists(int colNo) const { return !getBitmapValues(colNo).empty(); }

// getBitmapIndex (Columnarfile.java:1103-1127): the BitMapFile of the value,
// staged to HBM once; a value without one reads as an empty BitSet (:1124)
BitSetPtr Columnarfile::getBitmapIndex(int colNo, const std::string& key) const {
  Impl& I = *impl_;
  table();  // staging first: a changed DB file drops every staged BitSet
  auto& staged = I.bitmaps[colNo];
  auto jt = staged.find(key);
  if (jt != staged.end()) return jt->second;
  const int64_t nbits = positions();
  const std::string file = I.name + ".bm." + std::to_string(colNo) + "." + key;
  int32_t head = -1;
  chk<chainexception::ChainException>(mbx_db_file_entry(I.db, file.c_str(), &head), "get_file_entry");
  mbx_bitmap* z = nullptr;
  if (head >= 0) {
    chk<chainexception::ChainException>(
        mbx_db_bitmap_stage(global::SystemDefs::ctx(), I.db, file.c_str(), nbits, &z), "BitMapFile " + file);
  } else {
    // a CNF with one empty OR-conjunct: the empty BitSet, made on the device
    int64_t cnt = 0;
    int32_t offs[2] = {0, 0};
    chk<chainexception::ChainException>(
        mbx_bitmap_cnf(global::SystemDefs::ctx(), nbits, nullptr, offs, 1, nullptr, &z, &cnt), "empty BitSet");
  }
  auto b = std::make_shared<DeviceBitSet>(z);
  staged[key] = b;
  return b;
}

BitSetPtr Columnarfile::getMarkedDeleted() const {
  Impl& I = *impl_;
  table();
  if (!I.deleted_loaded) {
    mbx_bitmap* b = nullptr;
    chk<chainexception::ChainException>(
        mbx_db_bitmap_stage(global::SystemDefs::ctx(), I.db, (I.name + ".md").c_str(), positions(), &b),
        "markedDeleted");
    auto bs = std::make_shared<DeviceBitSet>(b);
    I.deleted_bm = bs->cardinality() > 0 ? bs : nullptr;
    I.deleted_loaded = true;
  }
  return I.deleted_bm;
}

void Columnarfile::invalidate() { impl_->invalidate(); }

void Columnarfile::markTupleDeleted(int64_t position) {
  Impl& I = *impl_;
  chk<chainexception::ChainException>(mbx_db_mark_deleted(I.db, I.name.c_str(), position), "markTupleDeleted");
  I.invalidate();
}

}  // namespace columnar

// --------------------------------------------------------------- iterator

namespace iterator {

mbx_cnf CnfImage::view() const {
  mbx_cnf c;
  c.conds = conds.data();
  c.conj_offsets = offsets.data();
  c.nconj = (int32_t)offsets.size() - 1;
  return c;
}

static mbx_operand operand_of(const AttrType& t, const Operand& o, int remap_from, int remap_to) {
  mbx_operand m;
  memset(&m, 0, sizeof(m));
  m.type = t.attrType;
  if (t.attrType == AttrType::attrSymbol) {
    if (o.symbol.relation.key != RelSpec::outer) throw InvalidRelation("Invalid relation -innerRel");
    m.fld = (remap_from && o.symbol.offset == remap_from) ? remap_to : o.symbol.offset;
  } else if (t.attrType == AttrType::attrInteger) {
    m.integer = o.integer;
  } else if (t.attrType == AttrType::attrReal) {
    m.real = o.real;
  } else if (t.attrType == AttrType::attrString) {
    m.string = o.string.data();
    m.string_len = (int32_t)o.string.size();
  }
  return m;
}

CnfImage flatten(CondExpr* const* filter, int remap_from, int remap_to) {
  CnfImage img;
  img.offsets.push_back(0);
  if (!filter) {
    img.offsets.clear();
    img.offsets.push_back(0);
    return img;  // nconj = 0: p == null
  }
  for (int i = 0; filter[i] != nullptr; i++) {
    for (const CondExpr* e = filter[i]; e; e = e->next) {
      mbx_condexpr c;
      memset(&c, 0, sizeof(c));
      c.op = e->op.attrOperator;
      c.operand1 = operand_of(e->type1, e->operand1, remap_from, remap_to);
      c.operand2 = operand_of(e->type2, e->operand2, remap_from, remap_to);
      c.index_type = e->indexType.indexType;
      img.conds.push_back(c);
    }
    img.offsets.push_back((int32_t)img.conds.size());
  }
  return img;
}

// ---- result batches shared by the scans: project `proj` columns of the
// selection on the GPU, hand them out row by row

static void setup_jtuple(heap::Tuple& J, const std::vector<AttrType>& in1, const std::vector<short>& s_sizes,
                         const std::vector<FldSpec>& proj) {
  // TupleUtils.setup_op_tuple (R/iterator/TupleUtils.java:295-341)
  std::vector<short> sizesT1(in1.size(), 0);
  size_t k = 0;
  for (size_t i = 0; i < in1.size(); i++)
    if (in1[i].attrType == AttrType::attrString) sizesT1[i] = k < s_sizes.size() ? s_sizes[k++] : 0;
  std::vector<AttrType> res;
  std::vector<short> res_sizes;
  for (const auto& f : proj) {
    if (f.relation.key != RelSpec::outer) throw InvalidRelation("Invalid relation -innerRel");
    if (f.offset < 1 || f.offset > (int)in1.size())
      throw FieldNumberOutOfBoundException("projection offset " + std::to_string(f.offset));
    res.push_back(in1[(size_t)f.offset - 1]);
    if (in1[(size_t)f.offset - 1].attrType == AttrType::attrString) res_sizes.push_back(sizesT1[(size_t)f.offset - 1]);
  }
  J.setHdr(res, res_sizes);
}

static int64_t col_width(const std::vector<AttrType>& types, const std::vector<short>& sizes, int col) {
  return types[(size_t)col].attrType == AttrType::attrString ? sizes[(size_t)col] : 4;
}

void CursorBatches::reset(mbx_cursor* c, const std::vector<AttrType>& types, const std::vector<short>& sizes,
                          const std::vector<int32_t>& cols) {
  close();
  cur_ = c;
  types_ = types;
  sizes_ = sizes;
  cols_ = cols;
  kind_.assign(cols.size(), 0);
  width_.assign(cols.size(), 0);
  for (size_t j = 0; j < cols.size(); j++) {
    kind_[j] = types[(size_t)cols[j]].attrType;
    width_[j] = col_width(types, sizes, cols[j]);
  }
  all_int_ = !cols.empty();
  for (int k : kind_) all_int_ = all_int_ && k == AttrType::attrInteger;
  vcols_.assign(cols.size(), nullptr);
  vids_ = nullptr;
  n_ = i_ = 0;
}

int64_t CursorBatches::count() const {
  int64_t n = 0;
  if (cur_) chk<FileScanException>(mbx_cursor_count(cur_, &n), "cursor count");
  return n;
}

bool CursorBatches::next_batch() {
  if (!cur_) return false;
  chk<FileScanException>(mbx_cursor_next_view(cur_, kRows, &vids_, vcols_.data(), &n_), "get_next");
  i_ = 0;
  if (n_ == 0) return false;
  i_++;
  return true;
}

void CursorBatches::restart() {
  if (cur_) chk<FileScanException>(mbx_cursor_restart(cur_), "restart");
  n_ = i_ = 0;
}

void CursorBatches::close() {
  if (cur_) mbx_cursor_close(cur_);
  cur_ = nullptr;
  n_ = i_ = 0;
}

ColumnarFileScan::ColumnarFileScan(const std::string& file_name, const std::vector<AttrType>& in1,
                                   const std::vector<short>& s1_sizes, short len_in1, int n_out_flds,
                                   const std::vector<FldSpec>& proj_list, CondExpr* const* outFilter)
    : f_(global::SystemDefs::db(), file_name), in1_(in1), perm_mat_(proj_list) {
  if ((int)in1.size() != len_in1 || len_in1 != f_.getFieldCount())
    throw FileScanException("ColumnarFileScan: in1/len_in1 do not match " + file_name);
  if ((int)proj_list.size() != n_out_flds) throw FileScanException("ColumnarFileScan: n_out_flds");
  setup_jtuple(Jtuple_, in1, s1_sizes, proj_list);
  for (const auto& p : proj_list) proj_cols_.push_back(p.offset - 1);
  types_ = f_.getAttributeTypes();
  sizes_ = f_.getAttrSizes();
  CnfImage img = flatten(outFilter);
  mbx_cnf cnf = img.view();
  mbx_ctx* c = global::SystemDefs::ctx();
  chk<PredEvalException>(mbx_plan_compile(c, f_.table(), &cnf, &plan_), "ColumnarFileScan: predicate");
  mbx_bitmap* b = nullptr;
  int64_t n = 0;
  chk<FileScanException>(mbx_scan_bitmap(c, plan_, &b, &n), "ColumnarFileScan: scan");
  sel_ = std::make_shared<columnar::DeviceBitSet>(b);
}

int64_t ColumnarFileScan::resultCount() const {
  int64_t n = 0;
  chk<FileScanException>(mbx_scan_count(global::SystemDefs::ctx(), plan_, &n), "ColumnarFileScan: count");
  return n;
}

void ColumnarFileScan::open_rows() {
  mbx_cursor* cur = nullptr;
  chk<FileScanException>(mbx_cursor_open(global::SystemDefs::ctx(), f_.table(), sel_->get(), proj_cols_.data(),
                                         (int32_t)proj_cols_.size(), &cur),
                         "ColumnarFileScan: materialise");
  rows_.reset(cur, types_, sizes_, proj_cols_);
}

global::TID ColumnarFileScan::get_next_tid() {
  global::TID tid;
  tid.numRIDs = f_.getFieldCount();
  if (!rows_.open()) open_rows();
  if (!rows_.next()) return tid;  // position -1: end of scan (null in Java)
  tid.position = rows_.position();
  return tid;
}

void ColumnarFileScan::close() {
  if (!closeFlag) {
    rows_.close();
    sel_.reset();
    if (plan_) mbx_plan_free(plan_);
    plan_ = nullptr;
    closeFlag = true;
  }
}

void ColumnarFileScan::restart() { rows_.restart(); }

int ColumnarFileScan::getTupleSize() { return Jtuple_.size(); }

ColumnarColumnScan::ColumnarColumnScan(columnar::Columnarfile* cf, int colNo, int n_out_flds,
                                       const std::vector<int>& out_indexes, const std::vector<FldSpec>& proj_list,
                                       CondExpr* const* outFilter) {
  (void)proj_list;
  // the CondExpr refers to the scanned column as field 1
  // (Query.buildQueryCondExprColscan, R/input/Query.java:337-360)
  std::vector<FldSpec> proj;
  for (int i = 0; i < n_out_flds; i++) proj.push_back(FldSpec(RelSpec(RelSpec::outer), out_indexes.at((size_t)i) + 1));
  // remap field 1 -> colNo + 1 by rewriting a copy of the chain
  std::vector<std::vector<CondExpr>> copies;
  std::vector<CondExpr*> heads;
  for (int i = 0; outFilter && outFilter[i]; i++) {
    std::vector<CondExpr> chain;
    for (const CondExpr* e = outFilter[i]; e; e = e->next) chain.push_back(*e);
    copies.push_back(chain);
  }
  for (auto& chain : copies) {
    for (size_t k = 0; k < chain.size(); k++) {
      if (chain[k].type1.attrType == AttrType::attrSymbol && chain[k].operand1.symbol.offset == 1)
        chain[k].operand1.symbol.offset = colNo + 1;
      if (chain[k].type2.attrType == AttrType::attrSymbol && chain[k].operand2.symbol.offset == 1)
        chain[k].operand2.symbol.offset = colNo + 1;
      chain[k].next = k + 1 < chain.size() ? &chain[k + 1] : nullptr;
    }
    heads.push_back(chain.empty() ? nullptr : &chain[0]);
  }
  heads.push_back(nullptr);
  inner_.reset(new ColumnarFileScan(cf->get_fileName(), cf->getAttributeTypes(), cf->getStringSizes(),
                                    (short)cf->getFieldCount(), n_out_flds, proj,
                                    outFilter ? heads.data() : nullptr));
}

ColumnarColumnsScan::ColumnarColumnsScan(columnar::Columnarfile* cf, const std::vector<int>& colNos, int n_out_flds,
                                         const std::vector<int>& out_indexes, const std::vector<FldSpec>& proj_list,
                                         CondExpr* const* outFilter) {
  // TupleUtils.setup_op_tuple over the file's schema and proj_list (:57-60)
  setup_jtuple(Jtuple_, cf->getAttributeTypes(), cf->getStringSizes(), proj_list);
  has_proj_ = true;
  init(cf, colNos, n_out_flds, out_indexes, outFilter);
}

ColumnarColumnsScan::ColumnarColumnsScan(columnar::Columnarfile* cf, const std::vector<int>& colNos,
                                         CondExpr* const* outFilter) {
  init(cf, colNos, 0, {}, outFilter);
}

void ColumnarColumnsScan::init(columnar::Columnarfile* cf, const std::vector<int>& colNos, int n_out_flds,
                               const std::vector<int>& out_indexes, CondExpr* const* outFilter) {
  const auto types = cf->getAttributeTypes();
  const int ncols = cf->getFieldCount();
  colNos_ = colNos;
  // destType / dest_s_sizes (:68-82), including its index quirk
  size_t nstr = 0;
  for (int c : colNos) {
    if (c < 0 || c >= ncols) throw ArrayIndexOutOfBoundsException(std::to_string(c));
    if (types[(size_t)c].attrType == AttrType::attrString) nstr++;
  }
  for (size_t i = 0; i < colNos.size(); i++)
    if (types[(size_t)colNos[i]].attrType == AttrType::attrString && i >= nstr)
      throw ArrayIndexOutOfBoundsException("Index " + std::to_string(i) + " out of bounds for length " +
                                           std::to_string(nstr));
  if ((int)out_indexes.size() < n_out_flds) throw FileScanException("ColumnarColumnsScan: out_indexes");
  for (int i = 0; i < n_out_flds; i++)
    if (out_indexes[(size_t)i] < 0 || out_indexes[(size_t)i] >= ncols)
      throw ArrayIndexOutOfBoundsException(std::to_string(out_indexes[(size_t)i]));
  // CondExpr fields address the colNos tuple (tuple1, :86): field k -> file
  // column colNos[k-1]; a field outside it is Tuple's FieldNumberOutOfBound
  std::vector<std::vector<CondExpr>> copies;
  for (int i = 0; outFilter && outFilter[i]; i++) {
    std::vector<CondExpr> chain;
    for (const CondExpr* e = outFilter[i]; e; e = e->next) chain.push_back(*e);
    copies.push_back(chain);
  }
  auto remap = [&](const AttrType& t, Operand& o) {
    if (t.attrType != AttrType::attrSymbol) return;
    if (o.symbol.offset < 1 || o.symbol.offset > (int)colNos.size())
      throw FieldNumberOutOfBoundException("ColumnarColumnsScan: field " + std::to_string(o.symbol.offset));
    o.symbol.offset = colNos[(size_t)o.symbol.offset - 1] + 1;
  };
  std::vector<CondExpr*> heads;
  for (auto& chain : copies) {
    for (size_t k = 0; k < chain.size(); k++) {
      remap(chain[k].type1, chain[k].operand1);
      remap(chain[k].type2, chain[k].operand2);
      chain[k].next = k + 1 < chain.size() ? &chain[k + 1] : nullptr;
    }
    heads.push_back(chain.empty() ? nullptr : &chain[0]);
  }
  heads.push_back(nullptr);
  std::vector<FldSpec> proj;
  for (int i = 0; i < n_out_flds; i++) proj.push_back(FldSpec(RelSpec(RelSpec::outer), out_indexes[(size_t)i] + 1));
  inner_.reset(new ColumnarFileScan(cf->get_fileName(), types, cf->getStringSizes(), (short)ncols, n_out_flds, proj,
                                    outFilter ? heads.data() : nullptr));
}

heap::Tuple* ColumnarColumnsScan::get_next() {
  if (!has_proj_) throw FileScanException("ColumnarColumnsScan: get_next without a projection (delete-query form)");
  return inner_->get_next();
}

global::TID ColumnarColumnsScan::get_next_tid() {
  global::TID tid = inner_->get_next_tid();
  // findPosition on colNos[0]'s heapfile with the last column's RID (:219)
  if (tid.position >= 0 && colNos_.size() > 1 && colNos_.front() != colNos_.back())
    throw JavaException("Invalid RID");
  return tid;
}

void ColumnarColumnsScan::close() {
  if (!closeFlag) {
    inner_->close();
    closeFlag = true;
  }
}
void ColumnarColumnsScan::restart() { inner_->restart(); }
int ColumnarColumnsScan::getTupleSize() { return has_proj_ ? Jtuple_.size() : inner_->getTupleSize(); }

heap::Tuple* ColumnarColumnScan::get_next() { return inner_->get_next(); }
global::TID ColumnarColumnScan::get_next_tid() { return inner_->get_next_tid(); }
void ColumnarColumnScan::close() {
  if (!closeFlag) {
    inner_->close();
    closeFlag = true;
  }
}
// ColumnarColumnScan does not override Iterator.restart() / getTupleSize()
// (R/iterator/Iterator.java:134-140): a no-op and -1
void ColumnarColumnScan::restart() {}
int ColumnarColumnScan::getTupleSize() { return -1; }

}  // namespace iterator

// ------------------------------------------------------------------ index

namespace index {

using columnar::BitSetPtr;

std::vector<BitSetPtr> ColumnIndexScan::valueBitmaps(const columnar::Columnarfile& cf, int colNo, const CondExpr& e) {
  std::vector<BitSetPtr> out;
  for (const std::string& k : valueKeys(cf, colNo, e)) out.push_back(cf.getBitmapIndex(colNo, k));
  return out;
}

std::vector<std::string> ColumnIndexScan::valueKeys(const columnar::Columnarfile& cf, int colNo, const CondExpr& e) {
  const auto types = cf.getAttributeTypes();
  const bool str = types.at((size_t)colNo).attrType == AttrType::attrString;
  const std::string lit = str ? e.operand2.string : columnar::int_key(e.operand2.integer);
  const int op = e.op.attrOperator;
  std::vector<std::string> out;
  using O = global::AttrOperator;
  // symbol = value (R/index/ColumnIndexScan.java:660-668)
  if (op == O::aopEQ || op == O::aopLE || op == O::aopGE) out.push_back(lit);
  if (op == O::aopLT || op == O::aopLE || op == O::aopGT || op == O::aopGE || op == O::aopNE) {
    for (const std::string& other : cf.getBitmapValues(colNo)) {
      int c;  // sign(value.compareTo(other))
      if (str) c = java_compare(lit, other);
      else {
        const int a = e.operand2.integer, b = atoi(other.c_str());
        c = a == b ? 0 : (a < b ? -1 : 1);
      }
      bool take = false;
      if ((op == O::aopLT || op == O::aopLE) && c > 0) take = true;   // :671-688
      if ((op == O::aopGT || op == O::aopGE) && c < 0) take = true;   // :691-709
      if (op == O::aopNE && c != 0) take = true;                      // :712-730
      if (take) out.push_back(other);
    }
  }
  return out;  // aopNOT / aopNOP / opRANGE: no value, an empty BitSet
}

// OR of value bitmaps AND NOT deleted, as one device CNF launch
static BitSetPtr or_bitmaps(const columnar::Columnarfile& cf, const std::vector<std::vector<BitSetPtr>>& conjuncts) {
  std::vector<mbx_bitmap*> bms;
  std::vector<int32_t> offs{0};
  for (const auto& conj : conjuncts) {
    for (const auto& b : conj) bms.push_back(b->get());
    offs.push_back((int32_t)bms.size());
  }
  mbx_bitmap* out = nullptr;
  int64_t n = 0;
  BitSetPtr del = cf.getMarkedDeleted();
  chk<IndexException>(mbx_bitmap_cnf(global::SystemDefs::ctx(), cf.positions(), bms.data(), offs.data(),
                                     (int32_t)conjuncts.size(), del ? del->get() : nullptr, &out, &n),
                      "index BitSet CNF");
  return std::make_shared<columnar::DeviceBitSet>(out);
}

static bool trace_on() {
  static const bool on = getenv("MBX_TRACE") && atoi(getenv("MBX_TRACE")) != 0;
  return on;
}

// ColumnarIndexScan / ColumnIndexScan get_next() in ONE kernel launch: the
// CNF over the conjuncts' bitmaps (minus cf.md), the positions and the
// projected rows straight into a cursor (mbx_cnf_cursor_open, k_cnf_select)
static mbx_cursor* cnf_cursor(const columnar::Columnarfile& cf, const std::vector<std::vector<BitSetPtr>>& conjuncts,
                              const std::vector<int>& cols, const char* who) {
  std::vector<mbx_bitmap*> bms;
  std::vector<int32_t> offs{0};
  for (const auto& conj : conjuncts) {
    for (const auto& b : conj) bms.push_back(b->get());
    offs.push_back((int32_t)bms.size());
  }
  std::vector<int32_t> pc(cols.begin(), cols.end());
  BitSetPtr del = cf.getMarkedDeleted();
  mbx_cursor* c = nullptr;
  chk<IndexException>(mbx_cnf_cursor_open(global::SystemDefs::ctx(), cf.table(), bms.data(), offs.data(),
                                          (int32_t)conjuncts.size(), del ? del->get() : nullptr, pc.data(),
                                          (int32_t)pc.size(), &c),
                      std::string(who) + ": one-launch CNF + projection");
  if (trace_on()) {
    int64_t n = 0;
    mbx_cursor_count(c, &n);
    fprintf(stderr, "trace: %s: one launch (k_cnf_select), %zu conjuncts, %zu bitmaps, %lld rows\n", who,
            conjuncts.size(), bms.size(), (long long)n);
  }
  return c;
}

// a cursor over a BitSet the reference's step-wise objects produced
static mbx_cursor* bitset_cursor(const columnar::Columnarfile& cf, const BitSetPtr& sel, const std::vector<int>& cols,
                                 const char* who) {
  std::vector<int32_t> pc(cols.begin(), cols.end());
  mbx_cursor* c = nullptr;
  chk<IndexException>(mbx_cursor_open(global::SystemDefs::ctx(), cf.table(), sel->get(), pc.data(), (int32_t)pc.size(),
                                      &c),
                      std::string(who) + ": late materialisation");
  if (trace_on()) fprintf(stderr, "trace: %s: step-wise BitSets + materialise\n", who);
  return c;
}

ColumnIndexScan::ColumnIndexScan(IndexType index, columnar::Columnarfile* cf, const std::string& indName,
                                 const std::vector<AttrType>& types, const std::vector<short>& str_sizes,
                                 int noInFlds, int noOutFlds, const std::vector<int>& outIndexes,
                                 const std::vector<FldSpec>& outFlds, CondExpr* const* selects, int fldNum,
                                 bool indexOnly)
    : f_(cf), colNo_(fldNum - 1), outIndexes_(outIndexes), types_(types), index_only_(indexOnly) {
  (void)indName;
  (void)noInFlds;
  if (index.indexType != IndexType::Bitmap)
    throw UnknownIndexTypeException("only the Bitmap branch of ColumnIndexScan runs on the GPU (B-tree: out of scope)");
  if (!selects || !selects[0]) throw IndexException("ColumnIndexScan: no selection");
  if ((int)outFlds.size() != noOutFlds) throw IndexException("ColumnIndexScan: noOutFlds");
  sel_ = *selects[0];
  sel_.next = nullptr;
  std::vector<AttrType> otypes;
  std::vector<short> osizes;
  const auto sizes = cf->getAttrSizes();
  for (int c : outIndexes) {
    otypes.push_back(types.at((size_t)c));
    if (types[(size_t)c].attrType == AttrType::attrString) osizes.push_back(sizes[(size_t)c]);
  }
  (void)str_sizes;
  Jtuple_.setHdr(otypes, osizes);
  values_ = valueBitmaps(*cf, colNo_, sel_);
}

ColumnIndexScan::ColumnIndexScan(IndexType index, columnar::Columnarfile* cf, const std::string& indName,
                                 const std::vector<AttrType>& types, const std::vector<short>& str_sizes, int noInFlds,
                                 CondExpr* const* selects, int fldNum)
    : ColumnIndexScan(index, cf, indName, types, str_sizes, noInFlds, 0, {}, {}, selects, fldNum, false) {}

BitSetPtr ColumnIndexScan::getPositionsOfIndexScan() {
  if (!positions_) positions_ = or_bitmaps(*f_, {values_});
  return positions_;
}

void ColumnIndexScan::open_cursor() {
  if (rows_.open()) return;
  const std::vector<int> cols = index_only_ ? std::vector<int>{} : outIndexes_;
  std::vector<int32_t> pc(cols.begin(), cols.end());
  rows_.reset(cnf_cursor(*f_, {values_}, cols, "ColumnIndexScan"), f_->getAttributeTypes(), f_->getAttrSizes(), pc);
}

heap::Tuple* ColumnIndexScan::get_next() {
  open_cursor();
  if (!rows_.next()) return nullptr;
  if (index_only_) {
    // only the key is returned (R/index/ColumnIndexScan.java:512-565)
    std::vector<AttrType> t{types_.at((size_t)colNo_)};
    std::vector<short> s;
    if (t[0].attrType == AttrType::attrString) s.push_back(f_->getAttrSizes()[(size_t)colNo_]);
    Jtuple_.setHdr(t, s);
    if (t[0].attrType == AttrType::attrString) Jtuple_.setStrFld(1, sel_.operand2.string);
    else Jtuple_.setIntFld(1, sel_.operand2.integer);
    return &Jtuple_;
  }
  rows_.fill(Jtuple_);
  return &Jtuple_;
}

global::TID ColumnIndexScan::get_next_tid() {
  open_cursor();
  global::TID tid;
  tid.numRIDs = f_->getFieldCount();
  if (rows_.next()) tid.position = rows_.position();
  return tid;
}

void ColumnIndexScan::close() {
  rows_.close();
  closeFlag = true;
}
// nor does ColumnIndexScan (R/index/ColumnIndexScan.java:28-740): Iterator's no-op and -1
void ColumnIndexScan::restart() {}
int ColumnIndexScan::getTupleSize() { return -1; }

ColumnarIndexScan::ColumnarIndexScan(columnar::Columnarfile* cf, const std::vector<int>& fldNums,
                                     const std::vector<IndexType>& indexTypes,
                                     const std::vector<std::string>& indNames, const std::vector<AttrType>& types,
                                     const std::vector<short>& str_sizes, int noInFlds, int noOutFlds,
                                     const std::vector<int>& out_indexes, const std::vector<FldSpec>& outFlds,
                                     CondExpr* const* selects, bool indexOnly)
    : f_(cf), outIndexes_(out_indexes), types_(types) {
  (void)fldNums;
  (void)indexTypes;
  (void)indNames;
  (void)str_sizes;
  (void)noInFlds;
  (void)indexOnly;
  if ((int)outFlds.size() != noOutFlds) throw IndexException("ColumnarIndexScan: noOutFlds");
  if (!selects || !selects[0]) throw IndexException("ColumnarIndexScan: no selection");
  std::vector<AttrType> otypes;
  std::vector<short> osizes;
  const auto sizes = cf->getAttrSizes();
  for (int c : out_indexes) {
    otypes.push_back(types.at((size_t)c));
    if (types[(size_t)c].attrType == AttrType::attrString) osizes.push_back(sizes[(size_t)c]);
  }
  Jtuple_.setHdr(otypes, osizes);

  // constraint keys (column + op + literal + index type), as the reference's
  // duplicate-constraint string (:137-141)
  struct Term {
    const CondExpr* e;
    int col;
    std::string key;
  };
  std::vector<std::vector<Term>> conj;
  std::map<std::string, int> occurrences;
  for (int i = 0; selects[i]; i++) {
    std::vector<Term> ts;
    for (const CondExpr* e = selects[i]; e; e = e->next) {
      int col;
      if (e->type1.attrType == AttrType::attrSymbol && e->type2.attrType != AttrType::attrSymbol)
        col = e->operand1.symbol.offset - 1;
      else if (e->type2.attrType == AttrType::attrSymbol && e->type1.attrType != AttrType::attrSymbol)
        col = e->operand2.symbol.offset - 1;
      else
        throw IndexException("IndexScan.java: invalid constraint");
      const std::string lit = e->type2.attrType == AttrType::attrInteger ? std::to_string(e->operand2.integer)
                                                                          : e->operand2.string;
      Term t{e, col, cf->indexToColName(col) + e->op.toString() + lit + e->indexType.toString()};
      occurrences[t.key]++;
      ts.push_back(t);
    }
    conj.push_back(ts);
  }
  auto term_bitmaps = [&](const Term& t) -> std::vector<BitSetPtr> {
    if (t.e->indexType.indexType == IndexType::B_Index) {
      // B-tree branch: same positions as the predicate itself; evaluated by
      // the scan kernel (the B-tree access path is out of scope)
      CondExpr one = *t.e;
      one.next = nullptr;
      CondExpr* arr[2] = {&one, nullptr};
      iterator::CnfImage img = iterator::flatten(arr);
      mbx_cnf cnf = img.view();
      mbx_plan* p = nullptr;
      chk<IndexException>(mbx_plan_compile(global::SystemDefs::ctx(), cf->table(), &cnf, &p), "B_Index term");
      mbx_bitmap* b = nullptr;
      int64_t n = 0;
      const int rc = mbx_scan_bitmap(global::SystemDefs::ctx(), p, &b, &n);
      mbx_plan_free(p);
      chk<IndexException>(rc, "B_Index term scan");
      return {std::make_shared<columnar::DeviceBitSet>(b)};
    }
    if (!cf->bitmapIndexExists(t.col))
      throw IndexException("Bitmap index does not exist on column " + cf->indexToColName(t.col));
    return ColumnIndexScan::valueBitmaps(*cf, t.col, *t.e);
  };

  bool dup = false;
  for (const auto& kv : occurrences) dup = dup || kv.second > 1;
  size_t total = 0;
  std::vector<std::vector<BitSetPtr>> lists;
  if (!dup) {
    for (const auto& ts : conj) {
      std::vector<BitSetPtr> l;
      for (const auto& t : ts) {
        auto v = term_bitmaps(t);
        l.insert(l.end(), v.begin(), v.end());
      }
      total += l.size();
      lists.push_back(l);
    }
  }
  if (!dup && total <= 64) {
    // one k_cnf_select launch at the first get_next: AND_c OR_k bitmaps AND
    // NOT deleted, the positions and the projected rows; the BitSet itself is
    // formed only if getOutputPositions() asks for it
    lists_ = lists;
    fused_ = true;
    return;
  }
  // Step-wise form, keeping the reference's object semantics (:130-181):
  // one positions BitSet per conjunct (conjunct 0's is outputPositions and
  // is AND-ed in place); a repeated constraint ORs in the cached *object*.
  std::vector<BitSetPtr> objs;
  std::map<std::string, size_t> cache;
  mbx_ctx* c = global::SystemDefs::ctx();
  auto combine = [&](int op, const BitSetPtr& a, const BitSetPtr& b) {
    mbx_bitmap* r = nullptr;
    int64_t n = 0;
    chk<IndexException>(mbx_bitmap_combine(c, op, a->get(), b->get(), &r, &n), "BitSet combine");
    return std::make_shared<columnar::DeviceBitSet>(r);
  };
  for (size_t i = 0; i < conj.size(); i++) {
    BitSetPtr positions = cf->getBitmapIndex(-1, "");  // empty BitSet
    objs.push_back(positions);
    for (const auto& t : conj[i]) {
      const bool in_cache = cache.count(t.key) > 0;
      const bool dflag = in_cache ? true : occurrences[t.key] > 1;
      if (!dflag || !in_cache) {
        BitSetPtr term = or_bitmaps(*cf, {term_bitmaps(t)});  // getPositionsOfIndexScan
        objs[i] = combine(MBX_BM_OR, objs[i], term);
        if (dflag) cache[t.key] = i;
      } else {
        objs[i] = combine(MBX_BM_OR, objs[i], objs[cache[t.key]]);
      }
    }
    if (i > 0) objs[0] = combine(MBX_BM_AND, objs[0], objs[i]);
  }
  output_ = objs[0];
}

BitSetPtr ColumnarIndexScan::getOutputPositions() {
  if (!output_) output_ = or_bitmaps(*f_, lists_);
  return output_;
}

void ColumnarIndexScan::open_cursor() {
  if (rows_.open()) return;
  std::vector<int32_t> pc(outIndexes_.begin(), outIndexes_.end());
  mbx_cursor* c = fused_ ? cnf_cursor(*f_, lists_, outIndexes_, "ColumnarIndexScan")
                         : bitset_cursor(*f_, output_, outIndexes_, "ColumnarIndexScan");
  rows_.reset(c, f_->getAttributeTypes(), f_->getAttrSizes(), pc);
}

global::TID ColumnarIndexScan::get_next_tid() {
  open_cursor();
  global::TID tid;
  tid.numRIDs = f_->getFieldCount();
  if (rows_.next()) tid.position = rows_.position();
  return tid;
}

void ColumnarIndexScan::close() {
  rows_.close();
  closeFlag = true;
}
void ColumnarIndexScan::restart() { rows_.restart(); }
int ColumnarIndexScan::getTupleSize() { return Jtuple_.size(); }

ShardedColumnarIndexScan::ShardedColumnarIndexScan(columnar::Columnarfile* cf, global::GpuSet& gpus, int noOutFlds,
                                                   const std::vector<int>& out_indexes,
                                                   const std::vector<FldSpec>& outFlds, CondExpr* const* selects)
    : f_(cf), outIndexes_(out_indexes) {
  if ((int)outFlds.size() != noOutFlds) throw IndexException("ShardedColumnarIndexScan: noOutFlds");
  if (!selects || !selects[0]) throw IndexException("ShardedColumnarIndexScan: no selection");
  const auto types = cf->getAttributeTypes();
  const auto sizes = cf->getAttrSizes();
  std::vector<AttrType> otypes;
  std::vector<short> osizes;
  for (int c : out_indexes) {
    otypes.push_back(types.at((size_t)c));
    if (types[(size_t)c].attrType == AttrType::attrString) osizes.push_back(sizes[(size_t)c]);
  }
  Jtuple_.setHdr(otypes, osizes);
  // the conjuncts' terms and their constraint keys (:137-146)
  struct Term {
    const CondExpr* e;
    int col;
  };
  std::vector<std::vector<Term>> conj;
  std::set<std::string> keys;
  for (int i = 0; selects[i]; i++) {
    std::vector<Term> ts;
    for (const CondExpr* e = selects[i]; e; e = e->next) {
      if (e->type1.attrType != AttrType::attrSymbol || e->type2.attrType == AttrType::attrSymbol)
        throw IndexException("IndexScan.java: invalid constraint");
      const int col = e->operand1.symbol.offset - 1;
      const std::string lit = e->type2.attrType == AttrType::attrInteger ? std::to_string(e->operand2.integer)
                                                                          : e->operand2.string;
      if (!keys.insert(cf->indexToColName(col) + e->op.toString() + lit + e->indexType.toString()).second)
        throw IndexException("ShardedColumnarIndexScan: a repeated constraint (use ColumnarIndexScan)");
      if (e->indexType.indexType != IndexType::B_Index && !cf->bitmapIndexExists(col))
        throw IndexException("Bitmap index does not exist on column " + cf->indexToColName(col));
      ts.push_back({e, col});
    }
    conj.push_back(ts);
  }
  mbx_db* db = cf->db();
  const std::string& name = cf->get_fileName();
  int64_t N = 0;
  chk<IndexException>(mbx_db_columnar_info(db, name.c_str(), 0, nullptr, nullptr, nullptr, &N, nullptr),
                      "ShardedColumnarIndexScan: positions");
  const auto& ctxs = gpus.ctxs();
  const int n = (int)ctxs.size();
  std::vector<int32_t> proj(out_indexes.begin(), out_indexes.end());
  std::vector<int64_t*> dcounts((size_t)n, nullptr);
  tables_.assign((size_t)n, nullptr);
  bitmaps_.assign((size_t)n, {});
  for (int g = 0; g < n; g++) {
    mbx_ctx* c = ctxs[(size_t)g];
    int64_t b = 0, e = 0;
    chk<IndexException>(mbx_shard_bounds(N, n, g, &b, &e), "shard bounds");
    chk<IndexException>(mbx_db_stage_range(c, db, name.c_str(), b, e, &tables_[(size_t)g]),
                        "shard " + std::to_string(g) + ": staging rows [" + std::to_string(b) + ", " +
                            std::to_string(e) + ")");
    int64_t nb = 0;
    mbx_table_info(tables_[(size_t)g], &nb, nullptr, nullptr);
    auto& owned = bitmaps_[(size_t)g];
    auto slice = [&](const std::string& file) -> mbx_bitmap* {
      int32_t head = -1;
      chk<IndexException>(mbx_db_file_entry(db, file.c_str(), &head), "get_file_entry");
      mbx_bitmap* z = nullptr;
      if (head >= 0) {
        chk<IndexException>(mbx_db_bitmap_stage_range(c, db, file.c_str(), b, nb, &z), "BitMapFile " + file);
      } else {  // no BitMapFile for the value: the empty BitSet (Columnarfile.java:1124)
        int64_t cnt = 0;
        int32_t offs[2] = {0, 0};
        chk<IndexException>(mbx_bitmap_cnf(c, nb, nullptr, offs, 1, nullptr, &z, &cnt), "empty BitSet");
      }
      owned.push_back(z);
      return z;
    };
    mbx_bitmap* del = slice(name + ".md");
    int64_t ndel = 0;
    mbx_bitmap_info(del, nullptr, nullptr, &ndel);
    std::vector<mbx_bitmap*> bms;
    std::vector<int32_t> offs{0};
    for (const auto& ts : conj) {
      for (const Term& t : ts) {
        if (t.e->indexType.indexType == IndexType::B_Index) {
          // the B-tree branch selects the term's own rows: the scan on the shard
          CondExpr one = *t.e;
          one.next = nullptr;
          CondExpr* arr[2] = {&one, nullptr};
          iterator::CnfImage img = iterator::flatten(arr);
          mbx_cnf cnf = img.view();
          mbx_plan* p = nullptr;
          chk<IndexException>(mbx_plan_compile(c, tables_[(size_t)g], &cnf, &p), "B_Index term");
          mbx_bitmap* z = nullptr;
          int64_t cnt = 0;
          const int rc = mbx_scan_bitmap(c, p, &z, &cnt);
          mbx_plan_free(p);
          chk<IndexException>(rc, "B_Index term scan");
          owned.push_back(z);
          bms.push_back(z);
        } else {
          for (const std::string& k : ColumnIndexScan::valueKeys(*cf, t.col, *t.e))
            bms.push_back(slice(name + ".bm." + std::to_string(t.col) + "." + k));
        }
      }
      offs.push_back((int32_t)bms.size());
    }
    mbx_cursor* cur = nullptr;
    chk<IndexException>(mbx_cnf_cursor_launch(c, tables_[(size_t)g], bms.data(), offs.data(), (int32_t)conj.size(),
                                              ndel > 0 ? del : nullptr, proj.data(), (int32_t)proj.size(), &cur,
                                              &dcounts[(size_t)g]),
                        "shard " + std::to_string(g) + ": one-launch CNF + projection");
    rows_.emplace_back(new iterator::CursorBatches());
    rows_.back()->reset(cur, types, sizes, proj);
  }
  // the exchange: every shard's count to every GPU (the concatenation offsets)
  std::vector<int64_t> counts((size_t)n, 0);
  const auto& comms = gpus.comms();
  if (!comms.empty()) {
    std::vector<int64_t*> alls((size_t)n, nullptr);
    for (int g = 0; g < n; g++)
      chk<IndexException>(mbx_dev_alloc(ctxs[(size_t)g], (int64_t)sizeof(int64_t) * n, (void**)&alls[(size_t)g]),
                          "device slots");
    std::vector<const int64_t*> src(dcounts.begin(), dcounts.end());
    int rc = mbx_comm_allgather_count_all(comms.data(), n, src.data(), alls.data());
    if (rc == MBX_OK) rc = mbx_comm_wait(comms[0]);
    if (rc == MBX_OK) rc = mbx_dev_download(ctxs[0], alls[0], counts.data(), (int64_t)sizeof(int64_t) * n);
    for (int g = 0; g < n; g++) mbx_dev_free(ctxs[(size_t)g], alls[(size_t)g]);
    chk<IndexException>(rc, "shard counts all-gather (RCCL)");
    rccl_ = true;
    for (int g = 0; g < n; g++)
      if (rows_[(size_t)g]->count() != counts[(size_t)g])
        throw IndexException("ShardedColumnarIndexScan: exchanged count differs from shard " + std::to_string(g));
  } else {
    for (int g = 0; g < n; g++) counts[(size_t)g] = rows_[(size_t)g]->count();
  }
  offsets_.assign((size_t)n + 1, 0);
  for (int g = 0; g < n; g++) offsets_[(size_t)g + 1] = offsets_[(size_t)g] + counts[(size_t)g];
  total_ = offsets_[(size_t)n];
  if (trace_on()) {
    fprintf(stderr, "trace: ShardedColumnarIndexScan: %d shards, exchange %s, counts", n, rccl_ ? "rccl" : "host");
    for (int64_t k : counts) fprintf(stderr, " %lld", (long long)k);
    fprintf(stderr, ", %lld rows\n", (long long)total_);
  }
}

ShardedColumnarIndexScan::~ShardedColumnarIndexScan() { close(); }

bool ShardedColumnarIndexScan::advance() {
  while (shard_ < rows_.size()) {
    if (rows_[shard_]->next()) return true;
    shard_++;
  }
  return false;
}

heap::Tuple* ShardedColumnarIndexScan::get_next() {
  if (!advance()) return nullptr;
  rows_[shard_]->fill(Jtuple_);
  return &Jtuple_;
}

global::TID ShardedColumnarIndexScan::get_next_tid() {
  global::TID tid;
  tid.numRIDs = f_->getFieldCount();
  if (advance()) tid.position = rows_[shard_]->position();
  return tid;
}

void ShardedColumnarIndexScan::close() {
  if (closeFlag) return;
  rows_.clear();
  for (auto& v : bitmaps_)
    for (mbx_bitmap* b : v) mbx_bitmap_free(b);
  bitmaps_.clear();
  for (mbx_table* t : tables_) mbx_table_free(t);
  tables_.clear();
  closeFlag = true;
}

void ShardedColumnarIndexScan::restart() {
  for (auto& r : rows_) r->restart();
  shard_ = 0;
}

int ShardedColumnarIndexScan::getTupleSize() { return Jtuple_.size(); }

}  // namespace index

}  // namespace minibase
