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
//   exit
//
// Output lines (column header, rows, "Total Results Count By Query: n")
// match the reference's, so a transcript can be diffed line by line.
// Page-I/O counters (PCounter) do not exist here -- there is no buffer pool
// on the GPU path; the driver prints the device time instead (stderr).
#include <chrono>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <set>
#include <sstream>

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

void indexes_query(const std::vector<std::string>& a) {
  if (a.size() < 6) throw std::runtime_error("Invalid number of attributes.");
  columnar::Columnarfile cf = open_cf(a[1], a[2]);
  Target t = targets(cf, a[3]);
  if (std::stoi(a[5]) < 1) throw std::runtime_error("NUMBUF is not more than 1.");
  // MultiIndexQuery.buildCNFQueryCondExpr (R/input/MultiIndexQuery.java:159-230)
  std::vector<std::unique_ptr<CondExpr>> pool;
  std::vector<CondExpr*> heads;
  std::vector<IndexType> itypes;
  std::vector<std::string> inames;
  for (const std::string& conj : split(a[4], '^')) {
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
  index::ColumnarIndexScan scan(&cf, {}, itypes, inames, cf.getAttributeTypes(), cf.getStringSizes(),
                                cf.getFieldCount(), (int)t.proj.size(), t.out_indexes, t.proj, heads.data(), true);
  print_rows(scan, cf, t);
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
      else if (a[0] == "indexes_query") indexes_query(a);
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
