// columnar_main.cpp -- the reference's command driver (R/input/ColumnarMain.java:8-80)
// for the scan/index commands, executed on the MI355X through the C++
// operator mirror (minibase.hpp):
//
//   batchinsert DATAFILE DBNAME COLUMNARFILENAME NUMCOLUMNS   (R/input/BatchInsert.java:17-137)
//     (DBNAME is a Minibase DB file in the working directory, created with
//      1024*1024 pages when absent -- include/mbx_db.h; the other commands
//      open it and stage the Columnarfile to HBM with the GPU page decoder)
//   index DBNAME COLUMNARFILENAME COLUMNNAME bitmap            (R/input/Index.java:16-67)
//   query DBNAME COLUMNARFILENAME [TARGETCOLS] {C,OP,V} NUMBUF FILESCAN|COLUMNSCAN|BITMAP
//                                                              (R/input/Query.java:35-361)
//   indexes_query DBNAME COLUMNARFILENAME [TARGETCOLS] {(C,OP,V,BM|BT)|..}^{..} NUMBUF
//                                                              (R/input/MultiIndexQuery.java:30-252)
//   nlj DBNAME OUTERFILE INNERFILE OUTERCONST INNERCONST JOINCONST OUTERACCESS INNERACCESS
//       [TARGETCOLUMNS] NUMBUF AMT_OF_MEMORY                   (R/input/NljQuery.java:30-230)
//   bmj DBNAME OUTERFILE INNERFILE OUTERCONST INNERCONST EQUICONST [TARGETCOLUMNS] NUMBUF
//                                                              (R/input/BitMapQuery.java:48-300)
//   delete_query DBNAME COLUMNARFILENAME {C,OP,V} NUMBUF ACCESS md|pd
//                                                              (R/input/DeleteQuery.java:28-215)
//   exit
//
// Output lines (column header, rows, "Total Results Count By Query: n")
// match the reference's, so a transcript can be diffed line by line.
// Page-I/O counters (PCounter) do not exist here -- there is no buffer pool
// on the GPU path; the driver prints the device time instead (stderr).
#include <algorithm>
#include <chrono>
#include <cstring>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <set>
#include <sstream>

#include "../../include/mbx_join.h"
#include "minibase.hpp"

namespace minibase {

using global::AttrOperator;
using global::AttrType;
using global::IndexType;
using iterator::CondExpr;
using iterator::FldSpec;
using iterator::RelSpec;

namespace {

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char ch : s) {
    if (ch == sep) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(ch);
    }
  }
  out.push_back(cur);
  return out;
}

std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && isspace((unsigned char)s[a])) a++;
  while (b > a && isspace((unsigned char)s[b - 1])) b--;
  return s.substr(a, b - a);
}

void print_results_footer(int64_t n) {
  std::cout << "\n************************************************************************\n"
            << "Total Results Count By Query: " << n << "\n"
            << "************************************************************************\n\n";
}

void batchinsert(const std::vector<std::string>& a) {
  if (a.size() < 5) throw std::runtime_error("Invalid number of attributes.");
  const std::string& datafile = a[1];
  const std::string db = a[2], cfname = a[3];
  const int numcolumns = std::stoi(a[4]);
  std::ifstream in(datafile);
  if (!in) throw std::runtime_error("data file " + datafile + " not found");
  std::string header;
  std::getline(in, header);
  auto heads = split(header, '\t');
  if ((int)heads.size() > numcolumns || numcolumns == 0)
    throw std::runtime_error("Number of columns specified does not match the number of columns in data file");
  std::vector<std::string> names;
  std::vector<AttrType> types;
  std::vector<short> sizes;
  for (int i = 0; i < numcolumns; i++) {
    auto nt = split(trim(heads[(size_t)i]), ':');
    names.push_back(nt[0]);
    if (nt[1] == "int") {
      types.emplace_back(AttrType::attrInteger);
      sizes.push_back(4);
    } else if (nt[1].rfind("char", 0) == 0) {
      types.emplace_back(AttrType::attrString);
      sizes.push_back((short)std::stoi(nt[1].substr(5, nt[1].size() - 6)));
    } else {
      throw std::runtime_error("column attr type is not supported.");
    }
  }
  // SystemDefs(db, exists ? 0 : 1024*1024, ...) (R/input/BatchInsert.java:52-57)
  mbx_db* dbh = global::SystemDefs::open(db, 1024 * 1024);
  columnar::Columnarfile cf(dbh, cfname, numcolumns, names, types, sizes);
  std::vector<std::vector<int32_t>> ints;
  std::vector<std::vector<float>> reals;
  std::vector<std::vector<std::string>> strs;
  std::vector<int> slot(numcolumns);
  for (int i = 0; i < numcolumns; i++) {
    if (types[(size_t)i].attrType == AttrType::attrInteger) {
      slot[(size_t)i] = (int)ints.size();
      ints.emplace_back();
    } else {
      slot[(size_t)i] = (int)strs.size();
      strs.emplace_back();
    }
  }
  std::string line;
  int64_t n = 0;
  while (std::getline(in, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.empty()) continue;
    auto v = split(line, '\t');
    for (int i = 0; i < numcolumns; i++) {
      if (types[(size_t)i].attrType == AttrType::attrInteger) {
        ints[(size_t)slot[(size_t)i]].push_back(std::stoi(v.at((size_t)i)));
      } else {
        if ((int)v.at((size_t)i).size() > sizes[(size_t)i]) throw std::runtime_error("column value exceeds size limit");
        strs[(size_t)slot[(size_t)i]].push_back(v[(size_t)i]);
      }
    }
    n++;
  }
  cf.insertColumns(ints, reals, strs, n);  // pages written to the DB file
  std::cout << "Record count: " << cf.getTupleCnt() << "\n";
}

columnar::Columnarfile open_cf(const std::string& db, const std::string& cf) {
  if (!global::SystemDefs::exists(db)) throw std::runtime_error("Database does not exist.");
  return columnar::Columnarfile(global::SystemDefs::open(db, 0), cf);
}

void index_cmd(const std::vector<std::string>& a) {
  if (a.size() < 5) throw std::runtime_error("Invalid number of attributes.");
  columnar::Columnarfile cf = open_cf(a[1], a[2]);
  const int col = cf.colNameToIndex(a[3]);
  if (a[4] == "bitmap" || a[4] == "BITMAP") {
    cf.createBitMapIndex(col);
  } else {
    throw std::runtime_error("BTREE indexes are not built by the GPU executor (B-tree access path out of scope)");
  }
}

struct Target {
  std::vector<std::string> names;
  std::vector<int> out_indexes;
  std::vector<FldSpec> proj;
};

Target targets(const columnar::Columnarfile& cf, const std::string& s) {
  if (s.size() < 2 || s.front() != '[' || s.back() != ']') throw std::runtime_error("[TARGETCOLUMNNAMES] format invalid.");
  Target t;
  for (auto& n : split(s.substr(1, s.size() - 2), ',')) {
    t.names.push_back(trim(n));
    const int c = cf.colNameToIndex(trim(n));
    t.out_indexes.push_back(c);
    t.proj.emplace_back(RelSpec(RelSpec::outer), c + 1);
  }
  return t;
}

// literal typed from the column (Query.buildQueryCondExpr, R/input/Query.java:299-323)
void set_literal(const columnar::Columnarfile& cf, int col, const std::string& val, CondExpr& e) {
  e.type1 = AttrType(AttrType::attrSymbol);
  const auto at = cf.getAttributeTypes()[(size_t)col].attrType;
  if (at == AttrType::attrInteger) {
    e.type2 = AttrType(AttrType::attrInteger);
    e.operand2.integer = std::stoi(val);
  } else if (at == AttrType::attrReal) {
    e.type2 = AttrType(AttrType::attrReal);
    e.operand2.real = std::stof(val);
  } else {
    e.type2 = AttrType(AttrType::attrString);
    e.operand2.string = val;
  }
}

void print_rows(iterator::Iterator& it, const columnar::Columnarfile& cf, const Target& t) {
  for (size_t i = 0; i < t.names.size(); i++) std::cout << (i ? ", " : "") << t.names[i];
  std::cout << "\n";
  int64_t n = 0;
  const auto types = cf.getAttributeTypes();
  heap::Tuple* tup;
  std::string buf;
  while ((tup = it.get_next()) != nullptr) {
    buf.clear();
    for (size_t i = 0; i < t.out_indexes.size(); i++) {
      if (i) buf += ", ";
      switch (types[(size_t)t.out_indexes[i]].attrType) {
        case AttrType::attrInteger: buf += std::to_string(tup->getIntFld((int)i + 1)); break;
        case AttrType::attrReal: buf += std::to_string(tup->getFloFld((int)i + 1)); break;
        default: buf += tup->getStrFld((int)i + 1);
      }
    }
    std::cout << buf << "\n";
    n++;
  }
  it.close();
  print_results_footer(n);
}

void query(const std::vector<std::string>& a) {
  if (a.size() < 7) throw std::runtime_error("Invalid number of attributes.");
  columnar::Columnarfile cf = open_cf(a[1], a[2]);
  Target t = targets(cf, a[3]);
  const std::string& cons = a[4];
  if (cons.size() < 2 || cons.front() != '{' || cons.back() != '}') throw std::runtime_error("VALUECONSTRAINT format invalid.");
  auto parts = split(trim(cons.substr(1, cons.size() - 2)), ',');
  if (parts.size() != 3) throw std::runtime_error("Invalid VALUECONSTRAINT elements");
  if (std::stoi(a[5]) < 1) throw std::runtime_error("NUMBUF is not more than 1.");
  const std::string access = a[6];
  const int col = cf.colNameToIndex(parts[0]);
  CondExpr e;
  e.op = AttrOperator::findOperator(parts[1]);
  set_literal(cf, col, parts[2], e);
  CondExpr* filter[2] = {&e, nullptr};
  if (access == "FILESCAN") {
    e.operand1.symbol = FldSpec(RelSpec(RelSpec::outer), col + 1);
    iterator::ColumnarFileScan fs(cf.get_fileName(), cf.getAttributeTypes(), cf.getStringSizes(),
                                  (short)cf.getFieldCount(), (int)t.proj.size(), t.proj, filter);
    print_rows(fs, cf, t);
  } else if (access == "COLUMNSCAN") {
    e.operand1.symbol = FldSpec(RelSpec(RelSpec::outer), 1);  // the scanned column is field 1
    iterator::ColumnarColumnScan cs(&cf, col, (int)t.proj.size(), t.out_indexes, t.proj, filter);
    print_rows(cs, cf, t);
  } else if (access == "BITMAP") {
    if (!cf.bitmapIndexExists(col)) throw std::runtime_error("Bitmap index does not exist on column " + parts[0]);
    e.operand1.symbol = FldSpec(RelSpec(RelSpec::outer), 1);
    e.indexType = IndexType(IndexType::Bitmap);
    index::ColumnIndexScan is(IndexType(IndexType::Bitmap), &cf, cf.get_fileName() + ".bm." + std::to_string(col),
                              cf.getAttributeTypes(), cf.getStringSizes(), cf.getFieldCount(), (int)t.proj.size(),
                              t.out_indexes, t.proj, filter, col + 1, false);
    print_rows(is, cf, t);
  } else if (access == "BTREE") {
    throw std::runtime_error("BTREE access is not part of the GPU path (out of scope)");
  } else {
    throw std::runtime_error("access type invalid.");
  }
}

struct IndexCnf {
  std::vector<std::unique_ptr<CondExpr>> pool;
  std::vector<CondExpr*> heads;
  std::vector<IndexType> itypes;
  std::vector<std::string> inames;
};
IndexCnf index_cnf(columnar::Columnarfile& cf, const std::string& spec);

void indexes_query(const std::vector<std::string>& a) {
  if (a.size() < 6) throw std::runtime_error("Invalid number of attributes.");
  columnar::Columnarfile cf = open_cf(a[1], a[2]);
  Target t = targets(cf, a[3]);
  if (std::stoi(a[5]) < 1) throw std::runtime_error("NUMBUF is not more than 1.");
  IndexCnf q = index_cnf(cf, a[4]);
  if (a[0] == "indexes_query_sharded") {
    // test / bench hook (no reference command): the same query over row-range
    // shards, one per GPU (index::ShardedColumnarIndexScan)
    if (a.size() < 7) throw std::runtime_error("indexes_query_sharded: SHARDS missing");
    global::GpuSet& gpus = global::GpuSet::get(std::stoi(a[6]));
    index::ShardedColumnarIndexScan scan(&cf, gpus, (int)t.proj.size(), t.out_indexes, t.proj, q.heads.data());
    print_rows(scan, cf, t);
    return;
  }
  index::ColumnarIndexScan scan(&cf, {}, q.itypes, q.inames, cf.getAttributeTypes(), cf.getStringSizes(),
                                cf.getFieldCount(), (int)t.proj.size(), t.out_indexes, t.proj, q.heads.data(), true);
  print_rows(scan, cf, t);
}

// MultiIndexQuery.buildCNFQueryCondExpr (R/input/MultiIndexQuery.java:159-230)
IndexCnf index_cnf(columnar::Columnarfile& cf, const std::string& spec) {
  IndexCnf q;
  auto& pool = q.pool;
  auto& heads = q.heads;
  auto& itypes = q.itypes;
  auto& inames = q.inames;
  for (const std::string& conj : split(spec, '^')) {
    if (conj.size() < 2 || conj.front() != '{' || conj.back() != '}') throw std::runtime_error("Invalid query format");
    CondExpr* head = nullptr;
    CondExpr* tail = nullptr;
    for (const std::string& dis : split(conj.substr(1, conj.size() - 2), '|')) {
      if (dis.size() < 2 || dis.front() != '(' || dis.back() != ')') throw std::runtime_error("Invalid query format");
      auto c = split(trim(dis.substr(1, dis.size() - 2)), ',');
      for (auto& x : c) x = trim(x);
      if (c.size() != 4) throw std::runtime_error("Invalid VALUECONSTRAINT elements");
      if (c[3] != "BT" && c[3] != "BM" && c[3] != "bt" && c[3] != "bm") throw std::runtime_error("Index type invalid");
      pool.emplace_back(new CondExpr());
      CondExpr* e = pool.back().get();
      const int col = cf.colNameToIndex(c[0]);
      e->op = AttrOperator::findOperator(c[1]);
      set_literal(cf, col, c[2], *e);
      e->operand1.symbol = FldSpec(RelSpec(RelSpec::outer), col + 1);
      if (c[3] == "BT" || c[3] == "bt") {
        e->indexType = IndexType(IndexType::B_Index);
        inames.push_back(cf.get_fileName() + ".btree." + std::to_string(col));
      } else {
        if (!cf.bitmapIndexExists(col)) throw std::runtime_error("Bitmap index does not exist on column " + c[0]);
        e->indexType = IndexType(IndexType::Bitmap);
        inames.push_back(cf.get_fileName() + ".bm." + std::to_string(col) + "." + c[2]);
      }
      itypes.push_back(e->indexType);
      if (!head) head = e;
      else tail->next = e;
      tail = e;
    }
    heads.push_back(head);
  }
  heads.push_back(nullptr);
  return q;
}

// ------------------------------------------------------------------ joins

using Cnf = std::vector<std::vector<std::vector<std::string>>>;  // conjunct -> term -> (a, op, b)

void ok(int rc, const std::string& what) {
  if (rc < 0) throw std::runtime_error(what + ": " + mbx_last_error());
}

Cnf parse_cnf(const std::string& s) {
  Cnf out;
  for (const std::string& conj : split(s, '^')) {
    if (conj.size() < 2 || conj.front() != '{' || conj.back() != '}') throw std::runtime_error("Invalid query format");
    std::vector<std::vector<std::string>> terms;
    for (const std::string& dis : split(conj.substr(1, conj.size() - 2), '|')) {
      if (dis.size() < 2 || dis.front() != '(' || dis.back() != ')') throw std::runtime_error("Invalid query format");
      auto c = split(trim(dis.substr(1, dis.size() - 2)), ',');
      for (auto& x : c) x = trim(x);
      if (c.size() != 3) throw std::runtime_error("Invalid VALUECONSTRAINT elements");
      terms.push_back(c);
    }
    out.push_back(terms);
  }
  return out;
}

// CondExpr[] of `column OP literal` terms over conjuncts [from, to) (literals
// typed from the column; index type per term)
struct CondArray {
  std::vector<std::unique_ptr<CondExpr>> pool;
  std::vector<CondExpr*> heads;
  std::vector<IndexType> itypes;
  std::vector<std::string> inames;
};

CondArray conds(const columnar::Columnarfile& cf, const Cnf& cnf, size_t from, size_t to, int index_type) {
  CondArray a;
  for (size_t k = from; k < to; k++) {
    CondExpr* head = nullptr;
    CondExpr* tail = nullptr;
    for (const auto& t : cnf[k]) {
      a.pool.emplace_back(new CondExpr());
      CondExpr* e = a.pool.back().get();
      const int col = cf.colNameToIndex(t[0]);
      e->op = AttrOperator::findOperator(t[1]);
      set_literal(cf, col, t[2], *e);
      e->operand1.symbol = FldSpec(RelSpec(RelSpec::outer), col + 1);
      e->indexType = IndexType(index_type);
      a.itypes.push_back(e->indexType);
      a.inames.push_back(" ");
      if (!head) head = e;
      else tail->next = e;
      tail = e;
    }
    a.heads.push_back(head);
  }
  a.heads.push_back(nullptr);
  return a;
}

// the BitSet a PredEval scan of conjuncts [from, to) selects (ColumnarFileScan)
columnar::BitSetPtr scan_sel(columnar::Columnarfile& cf, const Cnf& cnf, size_t from, size_t to) {
  CondArray a = conds(cf, cnf, from, to, IndexType::None);
  std::vector<FldSpec> proj{FldSpec(RelSpec(RelSpec::outer), 1)};
  iterator::ColumnarFileScan fs(cf.get_fileName(), cf.getAttributeTypes(), cf.getStringSizes(),
                                (short)cf.getFieldCount(), 1, proj, a.heads.data());
  return fs.selection();
}

// NljQuery.getIterator's COLUMNSCAN branch (R/input/NljQuery.java:245-270):
// the columns of conjunct 0 as a TreeSet (colNums), its fields renumbered
// into that tuple (findFieldOffset), out_indexes = the target columns; the
// BitSet the ColumnarColumnsScan selects
columnar::BitSetPtr columns_sel(columnar::Columnarfile& cf, const Cnf& cnf, const std::set<int>& target_cols) {
  CondArray a = conds(cf, cnf, 0, 1, IndexType::None);
  std::set<int> colset;
  for (CondExpr* e = a.heads[0]; e; e = e->next) colset.insert(e->operand1.symbol.offset - 1);
  const std::vector<int> colNums(colset.begin(), colset.end());
  for (CondExpr* e = a.heads[0]; e; e = e->next) {
    const int c = e->operand1.symbol.offset - 1;
    e->operand1.symbol.offset = (int)(std::find(colNums.begin(), colNums.end(), c) - colNums.begin()) + 1;
  }
  std::vector<int> out_indexes(target_cols.begin(), target_cols.end());
  std::vector<FldSpec> proj;
  for (int c : out_indexes) proj.emplace_back(RelSpec(RelSpec::outer), c + 1);
  iterator::ColumnarColumnsScan cs(&cf, colNums, (int)out_indexes.size(), out_indexes, proj, a.heads.data());
  return cs.selection();
}

// the BitSet a ColumnarIndexScan over conjuncts [from, to) returns
columnar::BitSetPtr index_sel(columnar::Columnarfile& cf, const Cnf& cnf, size_t from, size_t to, int index_type) {
  CondArray a = conds(cf, cnf, from, to, index_type);
  index::ColumnarIndexScan is(&cf, {}, a.itypes, a.inames, cf.getAttributeTypes(), cf.getStringSizes(),
                              cf.getFieldCount(), 0, {}, {}, a.heads.data(), true);
  return is.getOutputPositions();
}

columnar::BitSetPtr and_sel(const columnar::BitSetPtr& x, const columnar::BitSetPtr& y) {
  mbx_bitmap* b = nullptr;
  int64_t n = 0;
  ok(mbx_bitmap_combine(global::SystemDefs::ctx(), MBX_BM_AND, x->get(), y->get(), &b, &n),
                                      "BitSet.and");
  return std::make_shared<columnar::DeviceBitSet>(b);
}

std::string java_bitset(const std::vector<int64_t>& pos) {
  std::string s = "{";
  for (size_t k = 0; k < pos.size(); k++) s += (k ? ", " : "") + std::to_string(pos[k]);
  return s + "}";
}

struct JoinTargets {
  std::vector<std::string> names;
  std::vector<std::pair<int, int>> cols;  // (0 outer / 1 inner, column)
  std::set<int> outer, inner;             // TreeSet<Integer> of target columns per side
};

JoinTargets join_targets(const std::string& s, const std::string& outer_name, const columnar::Columnarfile& O,
                         const columnar::Columnarfile& I) {
  if (s.size() < 2 || s.front() != '[' || s.back() != ']') throw std::runtime_error("[TARGETCOLUMNNAMES] format invalid.");
  JoinTargets t;
  for (auto& n : split(s.substr(1, s.size() - 2), ',')) {
    const std::string name = trim(n);
    auto rc = split(name, '.');
    if (rc.size() != 2) throw std::runtime_error("Column " + name + " does not exist");
    const bool outer = rc[0] == outer_name;
    const int col = (outer ? O : I).colNameToIndex(rc[1]);
    t.names.push_back(name);
    t.cols.emplace_back(outer ? 0 : 1, col);
    (outer ? t.outer : t.inner).insert(col);
  }
  return t;
}

std::vector<mbx_join_term> join_terms(const Cnf& jc, const columnar::Columnarfile& O, const columnar::Columnarfile& I,
                                      std::vector<int32_t>& offs) {
  std::vector<mbx_join_term> terms;
  offs.assign(1, 0);
  for (const auto& conj : jc) {
    for (const auto& t : conj) {
      mbx_join_term jt;
      jt.op = AttrOperator::findOperator(t[1]).attrOperator;
      jt.outer_col = O.colNameToIndex(t[0]);
      jt.inner_col = I.colNameToIndex(t[2]);
      jt.pad_ = 0;
      if (O.getAttributeTypes()[(size_t)jt.outer_col].attrType != I.getAttributeTypes()[(size_t)jt.inner_col].attrType)
        throw std::runtime_error("Invalid JOIN COLUMN ATTR TYPE NOT MATCH.");
      terms.push_back(jt);
    }
    offs.push_back((int32_t)terms.size());
  }
  return terms;
}

// run the GPU join and print its rows (per pass for NLJ)
int64_t join_and_print(columnar::Columnarfile& O, columnar::Columnarfile& I, const columnar::BitSetPtr& osel,
                       const columnar::BitSetPtr& isel, const Cnf& jc, int32_t order, int64_t block,
                       const JoinTargets& tg) {
  std::vector<int32_t> offs;
  std::vector<mbx_join_term> terms = join_terms(jc, O, I, offs);
  mbx_join_cnf cnf{terms.data(), offs.data(), (int32_t)jc.size()};
  mbx_ctx* c = global::SystemDefs::ctx();
  mbx_join_result* r = nullptr;
  ok(mbx_join(c, O.table(), osel->get(), I.table(), isel->get(), &cnf, order, block, &r),
                                      "join");
  int64_t n = 0, passes = 1;
  mbx_join_info(r, &n, &passes);
  std::vector<int64_t> op((size_t)n), ip((size_t)n);
  std::vector<int32_t> ps((size_t)n);
  const int rc = mbx_join_fetch(c, r, 0, n, op.data(), ip.data(), ps.data());
  mbx_join_free(r);
  ok(rc, "join fetch");
  // late materialisation of every target column by position (GPU gather)
  std::vector<std::vector<std::string>> text(tg.cols.size());
  for (size_t j = 0; j < tg.cols.size(); j++) {
    columnar::Columnarfile& F = tg.cols[j].first == 0 ? O : I;
    const std::vector<int64_t>& pos = tg.cols[j].first == 0 ? op : ip;
    const int col = tg.cols[j].second;
    const auto at = F.getAttributeTypes()[(size_t)col].attrType;
    const int w = at == AttrType::attrString ? F.getAttrSizes()[(size_t)col] : 4;
    std::vector<uint8_t> buf((size_t)std::max<int64_t>(n, 1) * (size_t)w);
    void* outp = buf.data();
    int32_t pc = col;
    ok(mbx_gather(c, F.table(), pos.data(), n, &pc, 1, &outp), "gather");
    text[j].resize((size_t)n);
    for (int64_t k = 0; k < n; k++) {
      const uint8_t* v = buf.data() + (size_t)k * (size_t)w;
      if (at == AttrType::attrInteger) {
        int32_t x;
        memcpy(&x, v, 4);
        text[j][(size_t)k] = std::to_string(x);
      } else if (at == AttrType::attrReal) {
        float x;
        memcpy(&x, v, 4);
        text[j][(size_t)k] = std::to_string(x);
      } else {
        text[j][(size_t)k] = std::string((const char*)v, strnlen((const char*)v, (size_t)w));
      }
    }
  }
  auto pass_header = [](int64_t p) {
    std::cout << "\n************************************************************************\n"
              << "Next Pass Over Inner Table: " << p << "\n"
              << "************************************************************************\n\n";
  };
  int64_t k = 0;
  for (int64_t p = 0; p < passes; p++) {
    if (order == MBX_JOIN_NLJ && p > 0) pass_header(p);
    if (p == 0) {
      for (size_t j = 0; j < tg.names.size(); j++) std::cout << (j ? ", " : "") << tg.names[j];
      std::cout << "\n";
    }
    for (; k < n && (order != MBX_JOIN_NLJ || ps[(size_t)k] == p); k++) {
      std::string line;
      for (size_t j = 0; j < text.size(); j++) line += (j ? ", " : "") + text[j][(size_t)k];
      std::cout << line << "\n";
    }
  }
  return n;
}

// delete_query DB CF {C,OP,V} NUMBUF FILESCAN|COLUMNSCAN|BITMAP md|pd
// (R/input/DeleteQuery.java:28-215): the scan picks the live positions on the
// GPU, each one is marked deleted (cf.md + cf.dtid); `pd` then purges.
void delete_query(const std::vector<std::string>& a) {
  if (a.size() < 7) throw std::runtime_error("Invalid number of attributes.");
  if (!global::SystemDefs::exists(a[1])) throw std::runtime_error("Database does not exist.");
  const std::string& cons = a[3];
  if (cons.size() < 2 || cons.front() != '{' || cons.back() != '}') throw std::runtime_error("VALUECONSTRAINT format invalid.");
  int numbuf = 0;
  try {
    numbuf = std::stoi(a[4]);
  } catch (...) {
    throw std::runtime_error("NUMBUF is not integer.");
  }
  if (numbuf < 1) throw std::runtime_error("NUMBUF is not integer.");
  std::string acc = a[5], kind = a[6];
  for (auto& ch : acc) ch = (char)toupper((unsigned char)ch);
  for (auto& ch : kind) ch = (char)tolower((unsigned char)ch);
  if (acc != "FILESCAN" && acc != "COLUMNSCAN" && acc != "BTREE" && acc != "BITMAP")
    throw std::runtime_error("access type invalid.");
  if (kind != "md" && kind != "pd") throw std::runtime_error("delete type invalid.");
  mbx_db* db = global::SystemDefs::open(a[1], 0);
  columnar::Columnarfile cf(db, a[2]);
  auto parts = split(trim(cons.substr(1, cons.size() - 2)), ',');
  for (auto& x : parts) x = trim(x);
  if (parts.size() != 3) throw std::runtime_error("Invalid VALUECONSTRAINT elements");
  const int col = cf.colNameToIndex(parts[0]);
  Cnf cnf{{parts}};
  columnar::BitSetPtr sel;
  if (acc == "BTREE") {
    throw std::runtime_error("BTREE index does not exist on column " + parts[0]);
  } else if (acc == "BITMAP") {
    if (!cf.bitmapIndexExists(col)) throw std::runtime_error("Bitmap index does not exist on column " + parts[0]);
    sel = index_sel(cf, cnf, 0, 1, IndexType::Bitmap);
  } else {
    sel = scan_sel(cf, cnf, 0, 1);  // FILESCAN and COLUMNSCAN: the same PredEval, live rows only
  }
  const std::vector<int64_t> pos = sel->positions();
  ok(mbx_db_mark_deleted_many(db, cf.get_fileName().c_str(), pos.data(), (int64_t)pos.size()), "markTupleDeleted");
  if (kind == "pd") ok(mbx_db_purge(db, cf.get_fileName().c_str()), "purgeAllDeletedTuples");
  cf.invalidate();
  std::cout << "=======================EXTRA METAINFO===============================\n" << cf.getTupleCnt() << "\n";
  columnar::BitSetPtr md = cf.getMarkedDeleted();
  std::cout << java_bitset(md ? md->positions() : std::vector<int64_t>()) << "\n";
}

void nlj_cmd(const std::vector<std::string>& a) {
  if (a.size() < 12) throw std::runtime_error("Invalid number of attributes.");
  if (!global::SystemDefs::exists(a[1])) throw std::runtime_error("Database does not exist.");
  int numbuf = 0, amt = 0;
  try {
    numbuf = std::stoi(a[10]);
  } catch (...) {
    throw std::runtime_error("NUMBUF is not integer.");
  }
  if (numbuf < 1) throw std::runtime_error("NUMBUF is not integer.");
  try {
    amt = std::stoi(a[11]);
  } catch (...) {
    throw std::runtime_error("amt_of_memory is not integer.");
  }
  if (amt < 2) throw std::runtime_error("amt_of_memory is not integer.");
  mbx_db* db = global::SystemDefs::open(a[1], 0);
  columnar::Columnarfile O(db, a[2]), I(db, a[3]);
  const std::string oacc = a[7], iacc = a[8];
  auto valid = [](std::string x) {
    for (auto& ch : x) ch = (char)toupper((unsigned char)ch);
    return x == "FILESCAN" || x == "COLUMNSCAN" || x == "BTREE" || x == "BITMAP" ? x : std::string();
  };
  const std::string OA = valid(oacc), IA = valid(iacc);
  if (OA.empty()) throw std::runtime_error("outerAccessType invalid.");
  if (IA.empty()) throw std::runtime_error("innerAccessType invalid.");
  JoinTargets tg = join_targets(a[9], a[2], O, I);
  const Cnf oc = parse_cnf(a[4]), ic = parse_cnf(a[5]), jc = parse_cnf(a[6]);
  // findConsTargetCols / findJoinTargetCols (NljQuery.java:406-470)
  if (OA != "FILESCAN")
    for (size_t k = 1; k < oc.size(); k++)
      for (const auto& t : oc[k]) tg.outer.insert(O.colNameToIndex(t[0]));
  if (IA != "FILESCAN")
    for (size_t k = 1; k < ic.size(); k++)
      for (const auto& t : ic[k]) tg.inner.insert(I.colNameToIndex(t[0]));
  for (const auto& conj : jc)
    for (const auto& t : conj) {
      tg.outer.insert(O.colNameToIndex(t[0]));
      tg.inner.insert(I.colNameToIndex(t[2]));
    }
  // access path selection + pending filter (getIterator, NljQuery.java:232-300;
  // fillOuterBuffer / fillInnerBuffer, ColumnarNestedLoopJoins.java:120-158)
  auto select = [](columnar::Columnarfile& F, const Cnf& cnf, const std::string& acc, const std::set<int>& targets,
                   columnar::BitSetPtr* it) {
    if (acc == "FILESCAN") {
      *it = scan_sel(F, cnf, 0, cnf.size());
      return *it;
    }
    *it = acc == "COLUMNSCAN" ? columns_sel(F, cnf, targets)
                              : index_sel(F, cnf, 0, 1, acc == "BTREE" ? IndexType::B_Index : IndexType::Bitmap);
    return cnf.size() > 1 ? and_sel(*it, scan_sel(F, cnf, 1, cnf.size())) : *it;
  };
  columnar::BitSetPtr o_iter, i_iter;
  columnar::BitSetPtr osel = select(O, oc, OA, tg.outer, &o_iter);
  columnar::BitSetPtr isel = select(I, ic, IA, tg.inner, &i_iter);
  // the outer iterator's tuple (Tuple.setHdr over the TreeSet of outer
  // target columns) sizes the outer block (ColumnarNestedLoopJoins.java:122)
  int tsize = ((int)tg.outer.size() + 2) * 2;
  for (int col : tg.outer)
    tsize += O.getAttributeTypes()[(size_t)col].attrType == AttrType::attrString ? O.getAttrSizes()[(size_t)col] + 2 : 4;
  const int64_t block = (int64_t)(amt - 1) * (1024 / tsize);
  std::cout << "\n************************************************************************\n"
            << "Next Pass Over Inner Table: 0\n"
            << "************************************************************************\n\n";
  const int64_t n = join_and_print(O, I, osel, isel, jc, MBX_JOIN_NLJ, block, tg);
  std::cout << "\n************************************************************************\n"
            << "Tuple Size: " << tsize << "\n"
            << "Number of Tuples Buffer Can Hold: " << block << "\n"
            << "Total Outer Tuples By Full Constraint: " << osel->cardinality() << "\n"
            << "Total Outer Tuples By Iterator: " << o_iter->cardinality() << "\n"
            << "************************************************************************\n\n";
  print_results_footer(n);
}

// Test hook (no reference command): drives iterator::ColumnarColumnsScan
// directly, as NljQuery does (R/input/NljQuery.java:269).
//   columnsscan DB CF [COLNOS] CNF [OUTCOLS] [tid]
// COLNOS (column names, in the given order) make the scan's tuple; CNF terms
// name columns of it ({(C,=,6)|(A,>=,M)}^{...}); get_next prints OUTCOLS rows,
// `tid` prints get_next_tid positions instead.
void columnsscan_cmd(const std::vector<std::string>& a) {
  if (a.size() < 6) throw std::runtime_error("Invalid number of attributes.");
  columnar::Columnarfile cf = open_cf(a[1], a[2]);
  Target cols = targets(cf, a[3]);
  Target out = targets(cf, a[5]);
  const Cnf cnf = parse_cnf(a[4]);
  CondArray c = conds(cf, cnf, 0, cnf.size(), IndexType::None);
  for (size_t k = 0; k + 1 < c.heads.size(); k++)
    for (CondExpr* e = c.heads[k]; e; e = e->next) {
      const int col = e->operand1.symbol.offset - 1;
      const auto it = std::find(cols.out_indexes.begin(), cols.out_indexes.end(), col);
      e->operand1.symbol.offset = it == cols.out_indexes.end() ? 0 : (int)(it - cols.out_indexes.begin()) + 1;
    }
  iterator::ColumnarColumnsScan cs(&cf, cols.out_indexes, (int)out.out_indexes.size(), out.out_indexes, out.proj,
                                   c.heads.data());
  if (a.size() > 6 && a[6] == "tid") {
    int64_t n = 0;
    std::cout << "positions\n";
    for (global::TID t = cs.get_next_tid(); t.position >= 0; t = cs.get_next_tid()) {
      std::cout << t.position << "\n";
      n++;
    }
    cs.close();
    print_results_footer(n);
    return;
  }
  print_rows(cs, cf, out);
}

void bmj_cmd(const std::vector<std::string>& a) {
  if (a.size() < 9) throw std::runtime_error("Invalid number of attributes.");
  if (!global::SystemDefs::exists(a[1])) throw std::runtime_error("Database does not exist.");
  (void)std::stoi(a[8]);  // bufferSize
  mbx_db* db = global::SystemDefs::open(a[1], 0);
  columnar::Columnarfile O(db, a[2]), I(db, a[3]);
  // getConstraintBitset: ColumnarIndexScan over bitmap indexes (BitMapQuery.java:300-330)
  const Cnf oc = parse_cnf(a[4]), ic = parse_cnf(a[5]), jc = parse_cnf(a[6]);
  columnar::BitSetPtr osel = index_sel(O, oc, 0, oc.size(), IndexType::Bitmap);
  std::cout << "OuterConstraint Bitset After performing AND and ORs\n" << java_bitset(osel->positions()) << "\n";
  columnar::BitSetPtr isel = index_sel(I, ic, 0, ic.size(), IndexType::Bitmap);
  std::cout << "InnerConstraint Bitset After performing AND and ORs\n" << java_bitset(isel->positions()) << "\n";
  JoinTargets tg = join_targets(a[7], a[2], O, I);
  const int64_t n = join_and_print(O, I, osel, isel, jc, MBX_JOIN_BMJ, 0, tg);
  print_results_footer(n);
}

}  // namespace

int run() {
  std::cout << "Enter your command to the Minibase ColumnarDB:\n";
  std::string line;
  while (true) {
    std::cout << "> " << std::flush;
    if (!std::getline(std::cin, line)) break;
    line = trim(line);
    if (line.empty()) continue;
    std::vector<std::string> a;
    for (auto& w : split(line, ' '))
      if (!w.empty()) a.push_back(w);
    const auto t0 = std::chrono::steady_clock::now();
    try {
      if (a[0] == "batchinsert") batchinsert(a);
      else if (a[0] == "index") index_cmd(a);
      else if (a[0] == "query") query(a);
      else if (a[0] == "indexes_query" || a[0] == "indexes_query_sharded") indexes_query(a);
      else if (a[0] == "nlj") nlj_cmd(a);
      else if (a[0] == "delete_query") delete_query(a);
      else if (a[0] == "bmj") bmj_cmd(a);
      else if (a[0] == "columnsscan") columnsscan_cmd(a);
      else if (a[0] == "exit") break;
      else std::cout << "Command not supported by the GPU executor: " << a[0] << "\n";
    } catch (const std::exception& e) {
      std::cout << "java.lang.Exception: " << e.what() << "\n";
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    std::cerr << "[mbx] " << a[0] << ": " << ms << " ms\n";
  }
  global::SystemDefs::shutdown();
  return 0;
}

}  // namespace minibase

int main() { return minibase::run(); }
