// mbx_db.cpp -- Minibase DB files (include/mbx_db.h): the page formats of
// the reference's disk manager, heap files, Columnarfile and BitMapFile,
// restated in C++ over an mmap of the DB file, plus the GPU staging path.
//
// The writer replays the reference's page-allocation order (first fit over
// the space map, DB.allocate_page, R/diskmgr/DB.java:212-290) for the same
// sequence of calls: Heapfile(name) (Heapfile.java:349-390), insertRecord
// (Heapfile.java:420-520), HFPage.insertRecord (HFPage.java:337-396),
// Columnarfile(...) (Columnarfile.java:60-192), insertTuple
// (Columnarfile.java:400-470), BitMapFile(name, true) / BM.insertBitSet
// (BitMapFile.java:60-120, BM.java:60-120).  Only page bytes the reference
// defines are written; nothing about the JVM's buffer pool is modelled.
//
// The reader feeds mbx_db_stage: host code only walks directories (page ids
// per column, schema records, the .md BitSet); every record is decoded on
// the GPU (mbx_pages.hip).
#include "../../include/mbx_db.h"

#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "mbx_internal.hpp"
#include "mbx_objects.hpp"

using namespace mbx;

namespace {

constexpr int kPage = kDbPage;
constexpr int kMaxSpace = 1024;                    // GlobalConst.MAX_SPACE
constexpr int kBitsPerMapPage = kMaxSpace * 8;     // DB.bits_per_page
constexpr int32_t kInvalidPage = -1;               // GlobalConst.INVALID_PAGE
constexpr int kMaxName = MBX_DB_MAX_NAME;
constexpr int kFileEntry = 4 + kMaxName + 2;       // DBHeaderPage.SIZE_OF_FILE_ENTRY
constexpr int kStartEntries = 8;                   // DBHeaderPage.START_FILE_ENTRIES
constexpr int kFirstPageUsed = 8 + 8 + 4;          // PageUsedBytes.FIRST_PAGE_USED_BYTES
constexpr int kDirPageUsed = 8 + 8;                // PageUsedBytes.DIR_PAGE_USED_BYTES
// HFPage header fields (HFPage.java:31-40)
constexpr int kSlotCnt = 0, kUsedPtr = 2, kFreeSpace = 4, kType = 6, kPrev = 8, kNext = 12, kCur = 16;
constexpr int kDpFixed = kDbSlotBase;
constexpr int kSlotSize = 4;
constexpr int kDpInfoSize = 8;                      // DataPageInfo.size
constexpr int kRecsPerDirPage = (kPage - kDpFixed) / (kSlotSize + kDpInfoSize);  // 83
constexpr int kBmRecord = kMaxSpace - kDpFixed - kSlotSize;                      // 1000
constexpr int16_t kBmHead = 13;                     // NodeType.BMHEAD
constexpr int kAttrNameCell = MBX_DB_MAX_ATTR_NAME + 2;

inline int32_t get32(const uint8_t* p) {
  return (int32_t)(((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3]);
}
inline void put32(uint8_t* p, int32_t v) {
  p[0] = (uint8_t)((uint32_t)v >> 24);
  p[1] = (uint8_t)((uint32_t)v >> 16);
  p[2] = (uint8_t)((uint32_t)v >> 8);
  p[3] = (uint8_t)v;
}
inline int16_t get16(const uint8_t* p) { return (int16_t)(((uint32_t)p[0] << 8) | (uint32_t)p[1]); }
inline void put16(uint8_t* p, int32_t v) {
  p[0] = (uint8_t)((uint32_t)v >> 8);
  p[1] = (uint8_t)v;
}

// DataOutputStream.writeUTF of a byte string that is already modified UTF-8
// (file and attribute names here are ASCII)
inline void put_utf(uint8_t* p, const std::string& s) {
  put16(p, (int32_t)s.size());
  memcpy(p + 2, s.data(), s.size());
}
inline std::string get_utf(const uint8_t* p, int32_t cap) {
  int32_t n = (uint16_t)get16(p);
  if (n > cap - 2) n = cap - 2;
  return std::string((const char*)p + 2, (size_t)(n > 0 ? n : 0));
}

int32_t recs_per_data_page(int32_t rec_len) { return (kPage - kDpFixed) / (kSlotSize + rec_len); }

int32_t record_len(const mbx_col_desc& d) { return d.attr_type == MBX_ATTR_STRING ? d.size + 2 : 4; }

struct HeapHint {
  int32_t reclen = 0;     // valid for records at least this long
  int32_t dir_pid = kInvalidPage;
  int32_t dir_slot = 0;   // first directory slot worth checking
};

}  // namespace

struct mbx_db {
  std::string path;
  int fd = -1;
  uint8_t* base = nullptr;
  size_t bytes = 0;
  int32_t num_pages = 0;
  int32_t num_map_pages = 0;
  int64_t alloc_hint = 0;  // every page below is allocated
  std::unordered_map<int32_t, HeapHint> hints;  // per heap file (first dir page)

  uint8_t* page(int32_t pid) { return base + (size_t)pid * kPage; }
};

namespace {

// -------------------------------------------------------------- space map

bool page_bit(mbx_db* db, int64_t pid) {
  const uint8_t* map = db->page(1);  // map pages are contiguous from page 1
  return (map[pid >> 3] >> (pid & 7)) & 1;
}

void set_page_bit(mbx_db* db, int64_t pid, bool on) {
  uint8_t* map = db->page(1);
  if (on)
    map[pid >> 3] |= (uint8_t)(1u << (pid & 7));
  else
    map[pid >> 3] &= (uint8_t)~(1u << (pid & 7));
}

// DB.allocate_page(start, run): first run of `run` zero bits
int alloc_run(mbx_db* db, int32_t run, int32_t* start) {
  int64_t len = 0;
  for (int64_t p = db->alloc_hint; p < db->num_pages; ++p) {
    len = page_bit(db, p) ? 0 : len + 1;
    if (len == run) {
      const int64_t s = p - run + 1;
      for (int64_t q = s; q <= p; ++q) set_page_bit(db, q, true);
      while (db->alloc_hint < db->num_pages && page_bit(db, db->alloc_hint)) ++db->alloc_hint;
      *start = (int32_t)s;
      return MBX_OK;
    }
  }
  return fail(MBX_E_NOMEM, "OutOfSpaceException: DB %s has no run of %d free pages", db->path.c_str(), run);
}

// DB.allocate_page(start, 1): first zero bit of the space map
int alloc_page(mbx_db* db, int32_t* pid) {
  for (int64_t p = db->alloc_hint; p < db->num_pages; ++p) {
    if (!page_bit(db, p)) {
      set_page_bit(db, p, true);
      db->alloc_hint = p + 1;
      *pid = (int32_t)p;
      return MBX_OK;
    }
  }
  db->alloc_hint = db->num_pages;
  return fail(MBX_E_NOMEM, "OutOfSpaceException: DB %s has no free page (%d pages)", db->path.c_str(),
              db->num_pages);
}

// ----------------------------------------------------------- file entries

// DBHeaderPage(page, usedBytes): next = -1, entry count, every entry pid -1
void init_header_page(uint8_t* pg, int used) {
  put32(pg, kInvalidPage);
  const int n = (kMaxSpace - used) / kFileEntry;
  put32(pg + 4, n);
  for (int i = 0; i < n; ++i) put32(pg + kStartEntries + i * kFileEntry, kInvalidPage);
}

int32_t get_file_entry(mbx_db* db, const std::string& name) {
  int32_t hp = 0;
  int guard = 0;
  while (hp != kInvalidPage && hp >= 0 && hp < db->num_pages && guard++ < db->num_pages) {
    uint8_t* pg = db->page(hp);
    const int32_t n = get32(pg + 4);
    for (int32_t e = 0; e < n && kStartEntries + (e + 1) * kFileEntry <= kPage; ++e) {
      const uint8_t* ent = pg + kStartEntries + e * kFileEntry;
      const int32_t pid = get32(ent);
      if (pid != kInvalidPage && get_utf(ent + 4, kMaxName + 2) == name) return pid;
    }
    hp = get32(pg);
  }
  return kInvalidPage;
}

// DB.add_file_entry (DB.java:420-500)
int add_file_entry(mbx_db* db, const std::string& name, int32_t start) {
  if ((int)name.size() >= kMaxName) return fail(MBX_E_INVALID, "FileNameTooLongException: %s", name.c_str());
  if (get_file_entry(db, name) != kInvalidPage) return fail(MBX_E_INVALID, "DuplicateEntryException: %s", name.c_str());
  int32_t hp = 0;
  for (;;) {
    uint8_t* pg = db->page(hp);
    const int32_t n = get32(pg + 4);
    for (int32_t e = 0; e < n; ++e) {
      uint8_t* ent = pg + kStartEntries + e * kFileEntry;
      if (get32(ent) == kInvalidPage) {
        put32(ent, start);
        put_utf(ent + 4, name);
        return MBX_OK;
      }
    }
    const int32_t next = get32(pg);
    if (next != kInvalidPage) {
      hp = next;
      continue;
    }
    int32_t np;
    int rc = alloc_page(db, &np);
    if (rc) return rc;
    put32(pg, np);
    init_header_page(db->page(np), kDirPageUsed);
    hp = np;
  }
}

// ----------------------------------------------------------------- HFPage

void hf_init(uint8_t* pg, int32_t pid) {
  put16(pg + kSlotCnt, 0);
  put32(pg + kCur, pid);
  put32(pg + kPrev, kInvalidPage);
  put32(pg + kNext, kInvalidPage);
  put16(pg + kUsedPtr, kMaxSpace);
  put16(pg + kFreeSpace, kMaxSpace - kDpFixed);
}

int32_t hf_available(const uint8_t* pg) { return get16(pg + kFreeSpace) - kSlotSize; }
int32_t hf_slot_len(const uint8_t* pg, int32_t s) { return get16(pg + kDpFixed + s * kSlotSize); }
int32_t hf_slot_off(const uint8_t* pg, int32_t s) { return (uint16_t)get16(pg + kDpFixed + s * kSlotSize + 2); }

// HFPage.insertRecord: -1 when it does not fit
int32_t hf_insert(uint8_t* pg, const uint8_t* rec, int32_t len) {
  int32_t free_space = get16(pg + kFreeSpace);
  if (len + kSlotSize > free_space) return -1;
  const int32_t cnt = get16(pg + kSlotCnt);
  int32_t i = 0;
  while (i < cnt && hf_slot_len(pg, i) != -1) ++i;
  if (i == cnt) {
    free_space -= len + kSlotSize;
    put16(pg + kSlotCnt, cnt + 1);
  } else {
    free_space -= len;
  }
  put16(pg + kFreeSpace, free_space);
  const int32_t used = get16(pg + kUsedPtr) - len;
  put16(pg + kUsedPtr, used);
  put16(pg + kDpFixed + i * kSlotSize, len);
  put16(pg + kDpFixed + i * kSlotSize + 2, used);
  memcpy(pg + used, rec, (size_t)len);
  return i;
}

// ---------------------------------------------------------------- Heapfile

// Heapfile(name): existing first directory page, or a new one (newPage,
// add_file_entry, init -- in that order)
int heap_open(mbx_db* db, const std::string& name, bool create, int32_t* first_dir) {
  *first_dir = get_file_entry(db, name);
  if (*first_dir != kInvalidPage || !create) return MBX_OK;
  int32_t pid;
  int rc = alloc_page(db, &pid);
  if (rc) return rc;
  if ((rc = add_file_entry(db, name, pid))) return rc;
  hf_init(db->page(pid), pid);
  *first_dir = pid;
  return MBX_OK;
}

// Heapfile.insertRecord: the first data page (directory order) whose
// availspace fits the record, else a new data page registered in the first
// directory page with room for a DataPageInfo, else a new directory page.
int heap_insert(mbx_db* db, int32_t first_dir, const uint8_t* rec, int32_t len, int32_t* rid_pid,
                int32_t* rid_slot) {
  HeapHint& h = db->hints[first_dir];
  int32_t dir = first_dir;
  int32_t s0 = 0;
  if (h.dir_pid != kInvalidPage && len >= h.reclen) {
    dir = h.dir_pid;
    s0 = h.dir_slot;
  }
  int32_t found_dir = kInvalidPage, found_slot = -1;
  for (;;) {
    uint8_t* dp = db->page(dir);
    const int32_t cnt = get16(dp + kSlotCnt);
    for (int32_t s = s0; s < cnt; ++s) {
      if (hf_slot_len(dp, s) == -1) continue;
      const uint8_t* info = dp + hf_slot_off(dp, s);
      if (len <= get16(info)) {
        found_dir = dir;
        found_slot = s;
        break;
      }
    }
    if (found_slot >= 0) break;
    if (hf_available(dp) >= kDpInfoSize) {
      int32_t np;
      int rc = alloc_page(db, &np);
      if (rc) return rc;
      uint8_t* pg = db->page(np);
      hf_init(pg, np);
      uint8_t info[kDpInfoSize];
      put16(info, hf_available(pg));
      put16(info + 2, 0);
      put32(info + 4, np);
      found_slot = hf_insert(dp, info, kDpInfoSize);
      if (found_slot < 0) return fail(MBX_E_INVALID, "HFException: no space to insert rec.");
      found_dir = dir;
      break;
    }
    int32_t next = get32(dp + kNext);
    if (next == kInvalidPage) {
      int rc = alloc_page(db, &next);
      if (rc) return rc;
      uint8_t* ndp = db->page(next);
      hf_init(ndp, next);
      put32(ndp + kNext, kInvalidPage);
      put32(ndp + kPrev, dir);
      put32(dp + kNext, next);
    }
    dir = next;
    s0 = 0;
  }
  uint8_t* dp = db->page(found_dir);
  uint8_t* info = dp + hf_slot_off(dp, found_slot);
  const int32_t data_pid = get32(info + 4);
  uint8_t* pg = db->page(data_pid);
  const int32_t slot = hf_insert(pg, rec, len);
  if (slot < 0) return fail(MBX_E_INVALID, "SpaceNotAvailableException: no available space");
  put16(info + 2, get16(info + 2) + 1);
  put16(info, hf_available(pg));
  h.reclen = len;
  h.dir_pid = found_dir;
  h.dir_slot = found_slot;
  *rid_pid = data_pid;
  *rid_slot = slot;
  return MBX_OK;
}

// one entry per DataPageInfo in directory order: page index (the position
// formula's dirPageIndex * 83 + dirSlot, Heapfile.loadPositionBuffer) + pid
struct DataPage {
  int64_t index;
  int32_t pid;
  int32_t recct;
};

int heap_pages(mbx_db* db, int32_t first_dir, std::vector<DataPage>* out) {
  out->clear();
  int32_t dir = first_dir;
  int64_t dir_index = 0;
  while (dir != kInvalidPage) {
    if (dir < 0 || dir >= db->num_pages || dir_index > db->num_pages)
      return fail(MBX_E_INVALID, "heapfile directory chain leaves the DB at page %d", dir);
    const uint8_t* dp = db->page(dir);
    const int32_t cnt = get16(dp + kSlotCnt);
    for (int32_t s = 0; s < cnt && s < kRecsPerDirPage + 1; ++s) {
      if (hf_slot_len(dp, s) == -1) continue;
      const uint8_t* info = dp + hf_slot_off(dp, s);
      DataPage d;
      d.index = dir_index * kRecsPerDirPage + s;
      d.pid = get32(info + 4);
      d.recct = get16(info + 2);
      if (d.pid < 0 || d.pid >= db->num_pages) return fail(MBX_E_INVALID, "DataPageInfo names page %d", d.pid);
      out->push_back(d);
    }
    dir = get32(dp + kNext);
    ++dir_index;
  }
  return MBX_OK;
}

// heap.Scan order: directory order, then slot order within a data page
template <typename F>
int heap_scan(mbx_db* db, int32_t first_dir, F&& fn) {
  std::vector<DataPage> pages;
  int rc = heap_pages(db, first_dir, &pages);
  if (rc) return rc;
  for (const DataPage& d : pages) {
    const uint8_t* pg = db->page(d.pid);
    const int32_t cnt = get16(pg + kSlotCnt);
    for (int32_t s = 0; s < cnt; ++s) {
      const int32_t len = hf_slot_len(pg, s);
      if (len == -1) continue;
      const int32_t off = hf_slot_off(pg, s);
      if (len < 0 || off + len > kPage) return fail(MBX_E_INVALID, "corrupt slot %d on page %d", s, d.pid);
      if (!fn(d, s, pg + off, len)) return MBX_OK;
    }
  }
  return MBX_OK;
}

// ---------------------------------------------------------------- BitMapFile

// BitMapFile header page: new BMIndexPage (newPage + HFPage.init), type
// BMHEAD (initBitMapHeaderPage), then add_file_entry
int bm_create_header(mbx_db* db, const std::string& name, int32_t* head) {
  int rc = alloc_page(db, head);
  if (rc) return rc;
  uint8_t* pg = db->page(*head);
  hf_init(pg, *head);
  put16(pg + kType, kBmHead);
  return add_file_entry(db, name, *head);
}

// BM.readBitSet: the first record of every page of the chain, concatenated
int bm_read_bytes(mbx_db* db, int32_t head, std::vector<uint8_t>* bytes) {
  bytes->clear();
  int32_t p = head;
  int guard = 0;
  while (p != kInvalidPage) {
    if (p < 0 || p >= db->num_pages || guard++ > db->num_pages)
      return fail(MBX_E_INVALID, "BitMapFile chain leaves the DB at page %d", p);
    const uint8_t* pg = db->page(p);
    const int32_t cnt = get16(pg + kSlotCnt);
    int32_t s = 0;
    while (s < cnt && hf_slot_len(pg, s) == -1) ++s;
    if (s == cnt) return fail(MBX_E_INVALID, "InvalidSlotNumberException: BitMapFile page %d holds no record", p);
    const int32_t len = hf_slot_len(pg, s), off = hf_slot_off(pg, s);
    if (len < 0 || off + len > kPage) return fail(MBX_E_INVALID, "corrupt BitMapFile page %d", p);
    bytes->insert(bytes->end(), pg + off, pg + off + len);
    p = get32(pg + kNext);
  }
  return MBX_OK;
}

// BitSet.toByteArray(): little-endian bytes up to the last non-zero one
std::vector<uint8_t> bitset_bytes(const uint64_t* words, int64_t nwords) {
  int64_t nb = nwords * 8;
  const uint8_t* b = reinterpret_cast<const uint8_t*>(words);
  while (nb > 0 && b[nb - 1] == 0) --nb;
  return std::vector<uint8_t>(b, b + nb);
}

// BM.insertBitSet into a header page with no record yet: 1000-byte chunks,
// header page first, then new pages chained by next / prev
int bm_insert_bitset(mbx_db* db, int32_t head, const std::vector<uint8_t>& bytes) {
  const int64_t nchunks = ((int64_t)bytes.size() + kBmRecord - 1) / kBmRecord;
  if (nchunks == 0) return fail(MBX_E_INVALID, "BM.insertBitSet: empty BitSet (no chunk to store)");
  int32_t prev = kInvalidPage;
  int32_t cur = head;
  std::vector<uint8_t> rec(kBmRecord);
  for (int64_t i = 0; i < nchunks; ++i) {
    if (i > 0) {
      int rc = alloc_page(db, &cur);
      if (rc) return rc;
      hf_init(db->page(cur), cur);
    }
    std::fill(rec.begin(), rec.end(), 0);
    const int64_t start = i * kBmRecord;
    const int64_t n = std::min<int64_t>(kBmRecord, (int64_t)bytes.size() - start);
    memcpy(rec.data(), bytes.data() + start, (size_t)n);
    uint8_t* pg = db->page(cur);
    if (hf_insert(pg, rec.data(), kBmRecord) < 0) return fail(MBX_E_INVALID, "BitMapFile page %d is full", cur);
    put32(pg + kNext, kInvalidPage);
    put32(pg + kPrev, prev);
    if (prev != kInvalidPage) put32(db->page(prev) + kNext, cur);
    prev = cur;
  }
  return MBX_OK;
}

// BitMapFile.insert(position) on an existing file (the .md BitSet): set the
// bit inside its 1000-byte chunk, creating chunk pages up to it
int bm_set_bit(mbx_db* db, int32_t head, int64_t position) {
  const int64_t chunk = position / (kBmRecord * 8);
  int32_t p = head;
  for (int64_t i = 0;; ++i) {
    uint8_t* pg = db->page(p);
    if (i == chunk) {
      const int32_t cnt = get16(pg + kSlotCnt);
      int32_t s = 0;
      while (s < cnt && hf_slot_len(pg, s) == -1) ++s;
      if (s == cnt) return fail(MBX_E_INVALID, "BitMapFile page %d holds no record", p);
      uint8_t* rec = pg + hf_slot_off(pg, s);
      const int64_t bit = position - chunk * kBmRecord * 8;
      rec[bit >> 3] |= (uint8_t)(1u << (bit & 7));
      return MBX_OK;
    }
    int32_t next = get32(pg + kNext);
    if (next == kInvalidPage) {
      int rc = alloc_page(db, &next);
      if (rc) return rc;
      uint8_t* npg = db->page(next);
      hf_init(npg, next);
      std::vector<uint8_t> zero(kBmRecord, 0);
      hf_insert(npg, zero.data(), kBmRecord);
      put32(npg + kNext, kInvalidPage);
      put32(npg + kPrev, p);
      put32(pg + kNext, next);
    }
    p = next;
  }
}

// ----------------------------------------------------------- Columnarfile

struct Schema {
  int32_t ncols = 0;
  std::vector<mbx_col_desc> cols;
  std::vector<std::string> names;
  std::vector<uint8_t> btree_exist, bitmap_exist;
  std::vector<std::string> bm_values;  // "col.value" records
};

int read_schema(mbx_db* db, const std::string& name, Schema* sc) {
  const int32_t hdr = get_file_entry(db, name + ".hdr");
  if (hdr == kInvalidPage) return fail(MBX_E_INVALID, "Columnar File does not exist: %s", name.c_str());
  std::vector<std::vector<uint8_t>> recs;
  int rc = heap_scan(db, hdr, [&](const DataPage&, int32_t, const uint8_t* r, int32_t len) {
    recs.emplace_back(r, r + len);
    return true;
  });
  if (rc) return rc;
  if (recs.size() < 6 || recs[0].size() < 4) return fail(MBX_E_INVALID, "Columnar File does not exist: %s", name.c_str());
  sc->ncols = get32(recs[0].data());
  const int32_t n = sc->ncols;
  if (n <= 0 || (int64_t)recs[1].size() < 4LL * n || (int64_t)recs[2].size() < 4LL * n ||
      (int64_t)recs[3].size() < (int64_t)kAttrNameCell * n)
    return fail(MBX_E_INVALID, "%s.hdr: malformed header records", name.c_str());
  sc->cols.resize((size_t)n);
  sc->names.resize((size_t)n);
  for (int32_t i = 0; i < n; ++i) {
    sc->cols[(size_t)i].attr_type = get32(recs[1].data() + 4 * i);
    sc->cols[(size_t)i].size = get32(recs[2].data() + 4 * i);
    sc->names[(size_t)i] = get_utf(recs[3].data() + kAttrNameCell * i, kAttrNameCell);
  }
  sc->btree_exist = recs[4];
  sc->bitmap_exist = recs[5];
  for (size_t k = 6; k < recs.size(); ++k) sc->bm_values.push_back(get_utf(recs[k].data(), (int32_t)recs[k].size()));
  return MBX_OK;
}

int open_db_file(const char* path, bool create, int32_t num_pages, mbx_db** out) {
  *out = nullptr;
  if (!path) return fail(MBX_E_INVALID, "DB: null path");
  const int fd = create ? ::open(path, O_RDWR | O_CREAT | O_TRUNC, 0644) : ::open(path, O_RDWR);
  if (fd < 0) return fail(MBX_E_INVALID, "FileIOException: cannot open %s", path);
  if (create) {
    if (num_pages < 2) num_pages = 2;
    if (ftruncate(fd, (off_t)num_pages * kPage) != 0) {
      ::close(fd);
      return fail(MBX_E_NOMEM, "FileIOException: cannot size %s to %d pages", path, num_pages);
    }
  } else {
    struct stat st;
    uint8_t first[kPage];
    if (fstat(fd, &st) != 0 || st.st_size < kPage || pread(fd, first, kPage, 0) != kPage) {
      ::close(fd);
      return fail(MBX_E_INVALID, "InvalidPageNumberException: %s is not a Minibase DB", path);
    }
    num_pages = get32(first + kPage - 4);
    if (num_pages < 2 || (int64_t)num_pages * kPage > (int64_t)st.st_size) {
      ::close(fd);
      return fail(MBX_E_INVALID, "%s: numDBPages %d does not match the file size", path, num_pages);
    }
  }
  mbx_db* db = new (std::nothrow) mbx_db();
  if (!db) {
    ::close(fd);
    return fail(MBX_E_NOMEM, "DB: host allocation");
  }
  db->path = path;
  db->fd = fd;
  db->num_pages = num_pages;
  db->num_map_pages = (num_pages + kBitsPerMapPage - 1) / kBitsPerMapPage;
  db->bytes = (size_t)num_pages * kPage;
  void* m = mmap(nullptr, db->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (m == MAP_FAILED) {
    ::close(fd);
    delete db;
    return fail(MBX_E_NOMEM, "DB: mmap of %s failed", path);
  }
  db->base = (uint8_t*)m;
  if (create) {
    // DBFirstPage(page): header entries, numDBPages; space map: pages
    // 0 .. num_map_pages are in use (DB.openDB(name, num_pgs))
    init_header_page(db->page(0), kFirstPageUsed);
    put32(db->page(0) + kPage - 4, num_pages);
    for (int64_t p = 0; p <= db->num_map_pages; ++p) set_page_bit(db, p, true);
  }
  db->alloc_hint = 0;
  while (db->alloc_hint < db->num_pages && page_bit(db, db->alloc_hint)) ++db->alloc_hint;
  *out = db;
  return MBX_OK;
}

}  // namespace

// ================================================================== C-ABI

extern "C" int mbx_db_create(const char* path, int32_t num_pages, mbx_db** out) {
  NOTNULL(out);
  return open_db_file(path, true, num_pages, out);
}

extern "C" int mbx_db_open(const char* path, mbx_db** out) {
  NOTNULL(out);
  return open_db_file(path, false, 0, out);
}

extern "C" int mbx_db_close(mbx_db* db) {
  if (!db) return MBX_OK;
  int rc = MBX_OK;
  if (db->base) {
    if (msync(db->base, db->bytes, MS_SYNC) != 0) rc = fail(MBX_E_INVALID, "FileIOException: msync %s", db->path.c_str());
    munmap(db->base, db->bytes);
  }
  if (db->fd >= 0) ::close(db->fd);
  delete db;
  return rc;
}

extern "C" int mbx_db_info(const mbx_db* cdb, int32_t* num_pages, int32_t* allocated_pages) {
  NOTNULL(cdb);
  mbx_db* db = const_cast<mbx_db*>(cdb);
  if (num_pages) *num_pages = db->num_pages;
  if (allocated_pages) {
    int32_t n = 0;
    for (int64_t p = 0; p < db->num_pages; ++p) n += page_bit(db, p) ? 1 : 0;
    *allocated_pages = n;
  }
  return MBX_OK;
}

extern "C" int mbx_db_allocate_pages(mbx_db* db, int32_t run_size, int32_t* start) {
  NOTNULL(db);
  NOTNULL(start);
  if (run_size < 1) return fail(MBX_E_INVALID, "InvalidRunSizeException: %d", run_size);
  return alloc_run(db, run_size, start);
}

extern "C" int mbx_db_add_file_entry(mbx_db* db, const char* name, int32_t start) {
  NOTNULL(db);
  NOTNULL(name);
  if (start < 0 || start >= db->num_pages) return fail(MBX_E_INVALID, "InvalidPageNumberException: %d", start);
  return add_file_entry(db, name, start);
}

extern "C" int mbx_db_file_entry(mbx_db* db, const char* name, int32_t* first_page) {
  NOTNULL(db);
  NOTNULL(name);
  NOTNULL(first_page);
  *first_page = get_file_entry(db, name);
  return MBX_OK;
}

extern "C" int mbx_db_columnar_create(mbx_db* db, const char* name, int32_t ncols, const mbx_col_desc* cols,
                                      const char* const* attr_names) {
  NOTNULL(db);
  NOTNULL(name);
  NOTNULL(cols);
  NOTNULL(attr_names);
  const std::string cf = name;
  if ((int)cf.size() > MBX_DB_MAX_CF_NAME) return fail(MBX_E_INVALID, "File name too long: %s", name);
  if (ncols <= 0 || ncols > 4096) return fail(MBX_E_INVALID, "Columnarfile: %d columns", ncols);
  for (int32_t i = 0; i < ncols; ++i) {
    if (!attr_names[i]) return fail(MBX_E_INVALID, "Columnarfile: attr_names[%d] is null", i);
    if ((int)strlen(attr_names[i]) > MBX_DB_MAX_ATTR_NAME) return fail(MBX_E_INVALID, "Attribute name too long.");
    const int32_t t = cols[i].attr_type;
    if (t != MBX_ATTR_INTEGER && t != MBX_ATTR_REAL && t != MBX_ATTR_STRING)
      return fail(MBX_E_TYPE, "Columnarfile: column %d has AttrType %d", i, t);
    if (t == MBX_ATTR_STRING && (cols[i].size <= 0 || cols[i].size + 2 > kMaxSpace - kDpFixed - kSlotSize))
      return fail(MBX_E_INVALID, "Columnarfile: char(%d) does not fit a page", cols[i].size);
  }
  if (get_file_entry(db, cf + ".hdr") != kInvalidPage)
    return fail(MBX_E_INVALID, "Columnarfile %s already exists", name);
  int32_t hdr;
  int rc = heap_open(db, cf + ".hdr", true, &hdr);
  if (rc) return rc;
  // header records (Columnarfile.java:72-118)
  std::vector<uint8_t> r_n(4), r_t(4 * (size_t)ncols), r_s(4 * (size_t)ncols), r_names((size_t)kAttrNameCell * ncols, 0),
      r_bt((size_t)ncols, 0), r_bm((size_t)ncols, 0);
  put32(r_n.data(), ncols);
  for (int32_t i = 0; i < ncols; ++i) {
    put32(r_t.data() + 4 * i, cols[i].attr_type);
    put32(r_s.data() + 4 * i, cols[i].attr_type == MBX_ATTR_STRING ? cols[i].size : 4);
    put_utf(r_names.data() + kAttrNameCell * i, attr_names[i]);
  }
  int32_t pid, slot;
  for (const std::vector<uint8_t>* r : {&r_n, &r_t, &r_s, &r_names, &r_bt, &r_bm})
    if ((rc = heap_insert(db, hdr, r->data(), (int32_t)r->size(), &pid, &slot))) return rc;
  for (int32_t i = 0; i < ncols; ++i) {
    int32_t first;
    if ((rc = heap_open(db, cf + "." + std::to_string(i), true, &first))) return rc;
  }
  // markedDeleted = new BitMapFile(name + ".md", true): header page + one
  // 1000-byte zero record
  int32_t md;
  if ((rc = bm_create_header(db, cf + ".md", &md))) return rc;
  std::vector<uint8_t> zero(kBmRecord, 0);
  if (hf_insert(db->page(md), zero.data(), kBmRecord) < 0) return fail(MBX_E_INVALID, ".md header page is full");
  int32_t dtid;
  return heap_open(db, cf + ".dtid", true, &dtid);
}

extern "C" int mbx_db_columnar_insert(mbx_db* db, const char* name, int64_t nrows, const void* const* host_cols) {
  NOTNULL(db);
  NOTNULL(name);
  if (nrows < 0) return fail(MBX_E_INVALID, "insert: nrows %lld", (long long)nrows);
  if (nrows == 0) return MBX_OK;
  NOTNULL(host_cols);
  Schema sc;
  int rc = read_schema(db, name, &sc);
  if (rc) return rc;
  for (uint8_t b : sc.bitmap_exist)
    if (b == 1) return fail(MBX_E_UNSUPPORTED, "insert into %s: bitmap indexes are maintained on the GPU path, "
                            "rebuild them after the insert", name);
  for (uint8_t b : sc.btree_exist)
    if (b == 1) return fail(MBX_E_UNSUPPORTED, "insert into %s: B-tree indexes are out of scope", name);
  const int32_t n = sc.ncols;
  std::vector<int32_t> heap((size_t)n), rl((size_t)n);
  for (int32_t i = 0; i < n; ++i) {
    if (!host_cols[i]) return fail(MBX_E_INVALID, "insert: host_cols[%d] is null", i);
    heap[(size_t)i] = get_file_entry(db, std::string(name) + "." + std::to_string(i));
    if (heap[(size_t)i] == kInvalidPage) return fail(MBX_E_INVALID, "%s.%d is missing", name, i);
    rl[(size_t)i] = record_len(sc.cols[(size_t)i]);
  }
  std::vector<uint8_t> rec(kPage);
  for (int64_t r = 0; r < nrows; ++r) {
    for (int32_t i = 0; i < n; ++i) {
      const mbx_col_desc& d = sc.cols[(size_t)i];
      if (d.attr_type == MBX_ATTR_STRING) {
        const uint8_t* src = (const uint8_t*)host_cols[i] + (size_t)r * (size_t)d.size;
        const int32_t len = (int32_t)strnlen((const char*)src, (size_t)d.size);
        std::fill(rec.begin(), rec.begin() + rl[(size_t)i], 0);
        put16(rec.data(), len);
        memcpy(rec.data() + 2, src, (size_t)len);
      } else {
        uint32_t v;
        memcpy(&v, (const uint8_t*)host_cols[i] + (size_t)r * 4, 4);
        put32(rec.data(), (int32_t)v);
      }
      int32_t pid, slot;
      if ((rc = heap_insert(db, heap[(size_t)i], rec.data(), rl[(size_t)i], &pid, &slot))) return rc;
    }
  }
  return MBX_OK;
}

namespace {

// positions of a column heapfile: page table + nrows (max position + 1)
struct ColumnPages {
  std::vector<DataPage> pages;
  std::vector<int32_t> page_of;  // page index -> pid
  int64_t nrows = 0;
  int64_t records = 0;
  int32_t rec_len = 0;
  int32_t recs_per_page = 0;
  int32_t max_pid = -1;
};

int column_pages_lazy(mbx_db* db, const std::string& file, int32_t rec_len, ColumnPages* cp);

int column_pages(mbx_db* db, const std::string& file, int32_t rec_len, ColumnPages* cp) {
  const int32_t first = get_file_entry(db, file);
  if (first == kInvalidPage) return fail(MBX_E_INVALID, "heapfile %s is missing", file.c_str());
  int rc = heap_pages(db, first, &cp->pages);
  if (rc) return rc;
  cp->rec_len = rec_len;
  cp->recs_per_page = recs_per_data_page(rec_len);
  int64_t npi = 0;
  for (const DataPage& d : cp->pages) npi = std::max(npi, d.index + 1);
  cp->page_of.assign((size_t)npi, kInvalidPage);
  for (const DataPage& d : cp->pages) {
    cp->page_of[(size_t)d.index] = d.pid;
    cp->max_pid = std::max(cp->max_pid, d.pid);
    const int32_t cnt = get16(db->page(d.pid) + kSlotCnt);
    if (cnt < 0 || cnt > cp->recs_per_page)
      return fail(MBX_E_INVALID, "%s: data page %d holds %d slots (max %d)", file.c_str(), d.pid, cnt,
                  cp->recs_per_page);
    if (cnt > 0) cp->nrows = std::max(cp->nrows, d.index * cp->recs_per_page + cnt);
    cp->records += d.recct;
  }
  return MBX_OK;
}

}  // namespace

extern "C" int mbx_db_columnar_info(mbx_db* db, const char* name, int32_t max_cols, int32_t* ncols,
                                    mbx_col_desc* cols, char* attr_names, int64_t* nrows, int64_t* live) {
  NOTNULL(db);
  NOTNULL(name);
  Schema sc;
  int rc = read_schema(db, name, &sc);
  if (rc) return rc;
  if (ncols) *ncols = sc.ncols;
  for (int32_t i = 0; i < sc.ncols && i < max_cols; ++i) {
    if (cols) cols[i] = sc.cols[(size_t)i];
    if (attr_names) {
      char* cell = attr_names + (size_t)i * (MBX_DB_MAX_ATTR_NAME + 1);
      memset(cell, 0, MBX_DB_MAX_ATTR_NAME + 1);
      memcpy(cell, sc.names[(size_t)i].data(), std::min<size_t>(sc.names[(size_t)i].size(), MBX_DB_MAX_ATTR_NAME));
    }
  }
  if (nrows || live) {
    // the directory + the last data pages' headers (not every data page)
    ColumnPages cp;
    if ((rc = column_pages_lazy(db, std::string(name) + ".0", record_len(sc.cols[0]), &cp))) return rc;
    if (nrows) *nrows = cp.nrows;
    if (live) {
      int64_t del = 0;
      const int32_t md = get_file_entry(db, std::string(name) + ".md");
      if (md != kInvalidPage) {
        std::vector<uint8_t> bytes;
        if ((rc = bm_read_bytes(db, md, &bytes))) return rc;
        for (uint8_t b : bytes) del += __builtin_popcount(b);
      }
      *live = cp.records - del;
    }
  }
  return MBX_OK;
}

extern "C" int mbx_db_mark_deleted(mbx_db* db, const char* name, int64_t position) {
  NOTNULL(db);
  NOTNULL(name);
  if (position < 0) return fail(MBX_E_INVALID, "Invalid position");
  Schema sc;
  int rc = read_schema(db, name, &sc);
  if (rc) return rc;
  // RIDs of the position in every column (Heapfile.findRID)
  std::vector<uint8_t> tid((size_t)sc.ncols * 8);
  for (int32_t i = 0; i < sc.ncols; ++i) {
    ColumnPages cp;
    if ((rc = column_pages(db, std::string(name) + "." + std::to_string(i), record_len(sc.cols[(size_t)i]), &cp)))
      return rc;
    const int64_t pi = position / cp.recs_per_page;
    if (pi >= (int64_t)cp.page_of.size() || cp.page_of[(size_t)pi] == kInvalidPage)
      return fail(MBX_E_INVALID, "Invalid Position %lld", (long long)position);
    put32(tid.data() + 8 * i, (int32_t)(position - pi * cp.recs_per_page));  // RID.writeToByteArray: slotNo
    put32(tid.data() + 8 * i + 4, cp.page_of[(size_t)pi]);                  // then pageNo
  }
  const int32_t md = get_file_entry(db, std::string(name) + ".md");
  if (md == kInvalidPage) return fail(MBX_E_INVALID, "%s.md is missing", name);
  if ((rc = bm_set_bit(db, md, position))) return rc;
  int32_t dtid;
  if ((rc = heap_open(db, std::string(name) + ".dtid", true, &dtid))) return rc;
  int32_t pid, slot;
  return heap_insert(db, dtid, tid.data(), (int32_t)tid.size(), &pid, &slot);
}

extern "C" int mbx_db_bitmap_write(mbx_db* db, const char* filename, const uint64_t* words, int64_t nwords) {
  NOTNULL(db);
  NOTNULL(filename);
  if (nwords < 0 || (nwords > 0 && !words)) return fail(MBX_E_INVALID, "bitmap_write: %lld words", (long long)nwords);
  if (get_file_entry(db, filename) != kInvalidPage)
    return fail(MBX_E_INVALID, "The BitMapFile %s is already created.", filename);
  const std::vector<uint8_t> bytes = bitset_bytes(words, nwords);
  if (bytes.empty()) return fail(MBX_E_INVALID, "BM.insertBitSet: %s would be an empty BitSet", filename);
  int32_t head;
  int rc = bm_create_header(db, filename, &head);
  if (rc) return rc;
  return bm_insert_bitset(db, head, bytes);
}

extern "C" int mbx_db_bitmap_read(mbx_db* db, const char* filename, uint64_t* words, int64_t nwords_cap,
                                  int64_t* nwords_out) {
  NOTNULL(db);
  NOTNULL(filename);
  const int32_t head = get_file_entry(db, filename);
  if (head == kInvalidPage) return fail(MBX_E_INVALID, "The file %s does not exist.", filename);
  std::vector<uint8_t> bytes;
  int rc = bm_read_bytes(db, head, &bytes);
  if (rc) return rc;
  const int64_t nw = ((int64_t)bytes.size() + 7) / 8;
  if (nwords_out) *nwords_out = nw;
  if (words && nwords_cap > 0) {
    const int64_t n = std::min(nw, nwords_cap);
    memset(words, 0, (size_t)nwords_cap * 8);
    memcpy(words, bytes.data(), (size_t)std::min<int64_t>((int64_t)bytes.size(), n * 8));
  }
  return MBX_OK;
}

// ------------------------------------------------------------ GPU staging

extern "C" int mbx_db_stage(mbx_ctx* c, mbx_db* db, const char* name, mbx_table** out) {
  NOTNULL(c);
  NOTNULL(db);
  NOTNULL(name);
  NOTNULL(out);
  *out = nullptr;
  Schema sc;
  int rc = read_schema(db, name, &sc);
  if (rc) return rc;
  const int32_t n = sc.ncols;
  std::vector<ColumnPages> cps((size_t)n);
  int64_t nrows = 0;
  int32_t max_pid = 0;
  for (int32_t i = 0; i < n; ++i) {
    if ((rc = column_pages(db, std::string(name) + "." + std::to_string(i), record_len(sc.cols[(size_t)i]),
                           &cps[(size_t)i])))
      return rc;
    nrows = std::max(nrows, cps[(size_t)i].nrows);
    max_pid = std::max(max_pid, cps[(size_t)i].max_pid);
  }
  std::vector<uint8_t> md_bytes;
  const int32_t md = get_file_entry(db, std::string(name) + ".md");
  if (md != kInvalidPage && (rc = bm_read_bytes(db, md, &md_bytes))) return rc;
  const int64_t nwords = words_for(nrows);
  const int64_t md_words = std::min<int64_t>(((int64_t)md_bytes.size() + 7) / 8, nwords);

  mbx_table* t = nullptr;
  if ((rc = table_alloc(c, sc.cols.data(), n, nrows, 0, true, &t))) return rc;
  // device scratch: page image, page tables, present sets, .md words, flags
  const int64_t image_pages = (int64_t)max_pid + 1;
  uint8_t* dimg = nullptr;
  int32_t* dpage_of = nullptr;
  uint64_t* dpresent = nullptr;
  uint64_t* dmd = nullptr;
  int32_t* dflags = nullptr;
  int64_t npi_total = 0;
  for (const ColumnPages& cp : cps) npi_total += (int64_t)cp.page_of.size();
  const int64_t pw = nwords > 0 ? nwords : 1;
  void* pinned = nullptr;
  const size_t chunk = (size_t)32 << 20;
  hipStream_t s = c->stream;
  hipError_t e = hipMalloc(&dimg, (size_t)image_pages * kPage);
  if (e == hipSuccess) e = hipMalloc(&dpage_of, sizeof(int32_t) * (size_t)(npi_total > 0 ? npi_total : 1));
  if (e == hipSuccess) e = hipMalloc(&dpresent, sizeof(uint64_t) * (size_t)pw * (size_t)n);
  if (e == hipSuccess) e = hipMalloc(&dmd, sizeof(uint64_t) * (size_t)(md_words > 0 ? md_words : 1));
  if (e == hipSuccess) e = hipMalloc(&dflags, sizeof(int32_t) * 2);
  if (e == hipSuccess) e = hipHostMalloc(&pinned, 2 * chunk, hipHostMallocDefault);
  if (e == hipSuccess) e = hipMemsetAsync(dpresent, 0, sizeof(uint64_t) * (size_t)pw * (size_t)n, s);
  if (e == hipSuccess) e = hipMemsetAsync(dflags, 0, sizeof(int32_t) * 2, s);
  for (int32_t i = 0; i < n && e == hipSuccess; ++i) {
    const TCol& tc = t->cols[(size_t)i];
    e = hipMemsetAsync(tc.dev, 0, (size_t)(nrows > 0 ? nrows : 1) * (size_t)tc.stride_w * 4, s);
  }
  // the used part of the DB file, as it lies on disk, through two pinned
  // chunks (the copy of one overlaps the memcpy into the other)
  {
    const size_t total = (size_t)image_pages * kPage;
    hipEvent_t done[2] = {nullptr, nullptr};
    if (e == hipSuccess) e = hipEventCreateWithFlags(&done[0], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&done[1], hipEventDisableTiming);
    int k = 0;
    for (size_t off = 0; off < total && e == hipSuccess; off += chunk, k ^= 1) {
      const size_t len = std::min(chunk, total - off);
      e = hipEventSynchronize(done[k]);
      uint8_t* buf = (uint8_t*)pinned + (size_t)k * chunk;
      if (e == hipSuccess) {
        memcpy(buf, db->base + off, len);
        e = hipMemcpyAsync(dimg + off, buf, len, hipMemcpyHostToDevice, s);
      }
      if (e == hipSuccess) e = hipEventRecord(done[k], s);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (done[0]) hipEventDestroy(done[0]);
    if (done[1]) hipEventDestroy(done[1]);
  }
  std::vector<int32_t> page_of;
  page_of.reserve((size_t)npi_total);
  for (const ColumnPages& cp : cps) page_of.insert(page_of.end(), cp.page_of.begin(), cp.page_of.end());
  if (e == hipSuccess && npi_total > 0)
    e = hipMemcpy(dpage_of, page_of.data(), sizeof(int32_t) * page_of.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess && md_words > 0) {
    std::vector<uint64_t> mdw((size_t)md_words, 0);
    memcpy(mdw.data(), md_bytes.data(), std::min<size_t>(md_bytes.size(), (size_t)md_words * 8));
    e = hipMemcpy(dmd, mdw.data(), sizeof(uint64_t) * (size_t)md_words, hipMemcpyHostToDevice);
  }
  int64_t pofs = 0;
  for (int32_t i = 0; i < n && e == hipSuccess; ++i) {
    const ColumnPages& cp = cps[(size_t)i];
    const TCol& tc = t->cols[(size_t)i];
    PageDecodeArgs A{};
    A.image = dimg;
    A.image_pages = image_pages;
    A.page_of = dpage_of + pofs;
    A.npages = (int64_t)cp.page_of.size();
    A.rec_len = cp.rec_len;
    A.recs_per_page = cp.recs_per_page;
    A.kind = tc.attr_type == MBX_ATTR_STRING ? kStr : (tc.attr_type == MBX_ATTR_REAL ? kReal : kInt);
    A.size = tc.size;
    A.stride = tc.stride_w * 4;
    A.pad_ = 0;
    A.out = (uint8_t*)tc.dev;
    A.present = dpresent + (size_t)pw * (size_t)i;
    A.nrows = nrows;
    A.err = dflags;
    e = launch_page_decode(A, s);
    pofs += A.npages;
  }
  if (e == hipSuccess)
    e = launch_present_merge(dpresent, dpresent + pw, n - 1, pw, dmd, md_words, nrows, t->deleted, dflags + 1, s);
  int32_t flags[2] = {0, 0};
  if (e == hipSuccess) e = hipMemcpyAsync(flags, dflags, sizeof(flags), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  hipFree(dimg);
  hipFree(dpage_of);
  hipFree(dpresent);
  hipFree(dmd);
  hipFree(dflags);
  if (pinned) hipHostFree(pinned);
  if (e != hipSuccess) {
    mbx_table_free(t);
    return fail(MBX_E_DEVICE, "db_stage %s: %s", name, hipGetErrorString(e));
  }
  if (flags[0]) {
    mbx_table_free(t);
    return fail(MBX_E_INVALID, "db_stage %s: malformed data pages (flags 0x%x)", name, flags[0]);
  }
  if (flags[1] & 1) {
    mbx_table_free(t);
    return fail(MBX_E_INVALID, "Invalid position calculations: the column heapfiles of %s disagree", name);
  }
  if (!(flags[1] & 2) && t->deleted) {
    // every position holds a live record: scan without a deleted mask
    hipFree(t->deleted);
    t->deleted = nullptr;
    t->owns_deleted = false;
  }
  *out = t;
  return MBX_OK;
}

// ------------------------------------------------- row-range staging (shards)

namespace {

// the column's highest position + 1 from its directory and the slot counts
// of its last non-empty data pages only (column_pages reads every data
// page's header; a shard must not touch the other shards' pages)
int column_pages_lazy(mbx_db* db, const std::string& file, int32_t rec_len, ColumnPages* cp) {
  const int32_t first = get_file_entry(db, file);
  if (first == kInvalidPage) return fail(MBX_E_INVALID, "heapfile %s is missing", file.c_str());
  int rc = heap_pages(db, first, &cp->pages);
  if (rc) return rc;
  cp->rec_len = rec_len;
  cp->recs_per_page = recs_per_data_page(rec_len);
  int64_t npi = 0;
  for (const DataPage& d : cp->pages) npi = std::max(npi, d.index + 1);
  cp->page_of.assign((size_t)npi, kInvalidPage);
  for (const DataPage& d : cp->pages) {
    cp->page_of[(size_t)d.index] = d.pid;
    cp->records += d.recct;
  }
  for (int64_t pi = npi - 1; pi >= 0; --pi) {
    const int32_t pid = cp->page_of[(size_t)pi];
    if (pid == kInvalidPage) continue;
    const int32_t cnt = get16(db->page(pid) + kSlotCnt);
    if (cnt < 0 || cnt > cp->recs_per_page)
      return fail(MBX_E_INVALID, "%s: data page %d holds %d slots (max %d)", file.c_str(), pid, cnt,
                  cp->recs_per_page);
    if (cnt > 0) {
      cp->nrows = pi * cp->recs_per_page + cnt;
      break;
    }
  }
  return MBX_OK;
}

}  // namespace

extern "C" int mbx_db_stage_range(mbx_ctx* c, mbx_db* db, const char* name, int64_t row_begin, int64_t row_end,
                                  mbx_table** out) {
  NOTNULL(c);
  NOTNULL(db);
  NOTNULL(name);
  NOTNULL(out);
  *out = nullptr;
  if (row_begin < 0 || (row_begin & 63) || row_end < row_begin)
    return fail(MBX_E_INVALID, "db_stage_range: rows [%lld, %lld) (begin must be a multiple of 64)",
                (long long)row_begin, (long long)row_end);
  Schema sc;
  int rc = read_schema(db, name, &sc);
  if (rc) return rc;
  const int32_t n = sc.ncols;
  std::vector<ColumnPages> cps((size_t)n);
  int64_t total = 0;
  for (int32_t i = 0; i < n; ++i) {
    if ((rc = column_pages_lazy(db, std::string(name) + "." + std::to_string(i), record_len(sc.cols[(size_t)i]),
                                &cps[(size_t)i])))
      return rc;
    total = std::max(total, cps[(size_t)i].nrows);
  }
  const int64_t r0 = std::min(row_begin, total), r1 = std::min(row_end, total);
  const int64_t nrows = r1 - r0;
  const int64_t nwords = words_for(nrows);
  // per column: the page indices covering [r0, r1) and their pages, packed
  // into one compact image in page-index order (runs of consecutive pids
  // copied together)
  std::vector<int64_t> pi0((size_t)n, 0);
  std::vector<std::vector<int32_t>> local_of((size_t)n);  // page index - pi0 -> image page (-1: none)
  std::vector<int32_t> image_pids;
  for (int32_t i = 0; i < n && nrows > 0; ++i) {
    const ColumnPages& cp = cps[(size_t)i];
    const int64_t a = r0 / cp.recs_per_page, b = (r1 - 1) / cp.recs_per_page;
    pi0[(size_t)i] = a;
    local_of[(size_t)i].assign((size_t)(b - a + 1), -1);
    for (int64_t pi = a; pi <= b && pi < (int64_t)cp.page_of.size(); ++pi) {
      const int32_t pid = cp.page_of[(size_t)pi];
      if (pid == kInvalidPage) continue;
      local_of[(size_t)i][(size_t)(pi - a)] = (int32_t)image_pids.size();
      image_pids.push_back(pid);
    }
  }
  // cf.md bits [r0, r1) (r0 is a multiple of 64: whole words)
  std::vector<uint8_t> md_bytes;
  const int32_t md = get_file_entry(db, std::string(name) + ".md");
  if (md != kInvalidPage && (rc = bm_read_bytes(db, md, &md_bytes))) return rc;
  std::vector<uint64_t> mdw;
  {
    const int64_t have = ((int64_t)md_bytes.size() + 7) / 8;
    const int64_t w0 = r0 / 64, nw = std::max<int64_t>(0, std::min(have - w0, nwords));
    mdw.assign((size_t)(nw > 0 ? nw : 0), 0ull);
    for (int64_t w = 0; w < nw; ++w) {
      const size_t byte0 = (size_t)(w0 + w) * 8;
      const size_t len = std::min<size_t>(8, md_bytes.size() - byte0);
      memcpy(&mdw[(size_t)w], md_bytes.data() + byte0, len);
    }
  }
  const int64_t md_words = (int64_t)mdw.size();

  mbx_table* t = nullptr;
  if ((rc = table_alloc(c, sc.cols.data(), n, nrows, r0, true, &t))) return rc;
  const int64_t image_pages = (int64_t)image_pids.size();
  uint8_t* dimg = nullptr;
  int32_t* dpage_of = nullptr;
  uint64_t* dpresent = nullptr;
  uint64_t* dmd = nullptr;
  int32_t* dflags = nullptr;
  int64_t npi_total = 0;
  for (const auto& l : local_of) npi_total += (int64_t)l.size();
  const int64_t pw = nwords > 0 ? nwords : 1;
  void* pinned = nullptr;
  const size_t chunk = (size_t)32 << 20;
  hipStream_t s = c->stream;
  hipError_t e = hipMalloc(&dimg, (size_t)(image_pages > 0 ? image_pages : 1) * kPage);
  if (e == hipSuccess) e = hipMalloc(&dpage_of, sizeof(int32_t) * (size_t)(npi_total > 0 ? npi_total : 1));
  if (e == hipSuccess) e = hipMalloc(&dpresent, sizeof(uint64_t) * (size_t)pw * (size_t)n);
  if (e == hipSuccess) e = hipMalloc(&dmd, sizeof(uint64_t) * (size_t)(md_words > 0 ? md_words : 1));
  if (e == hipSuccess) e = hipMalloc(&dflags, sizeof(int32_t) * 2);
  if (e == hipSuccess) e = hipHostMalloc(&pinned, 2 * chunk, hipHostMallocDefault);
  if (e == hipSuccess) e = hipMemsetAsync(dpresent, 0, sizeof(uint64_t) * (size_t)pw * (size_t)n, s);
  if (e == hipSuccess) e = hipMemsetAsync(dflags, 0, sizeof(int32_t) * 2, s);
  for (int32_t i = 0; i < n && e == hipSuccess; ++i) {
    const TCol& tc = t->cols[(size_t)i];
    e = hipMemsetAsync(tc.dev, 0, (size_t)(nrows > 0 ? nrows : 1) * (size_t)tc.stride_w * 4, s);
  }
  // this shard's pages only, through two pinned chunks
  {
    hipEvent_t done[2] = {nullptr, nullptr};
    if (e == hipSuccess) e = hipEventCreateWithFlags(&done[0], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&done[1], hipEventDisableTiming);
    const int64_t per_chunk = (int64_t)(chunk / kPage);
    int k = 0;
    for (int64_t p0 = 0; p0 < image_pages && e == hipSuccess; p0 += per_chunk, k ^= 1) {
      const int64_t np = std::min(per_chunk, image_pages - p0);
      e = hipEventSynchronize(done[k]);
      uint8_t* buf = (uint8_t*)pinned + (size_t)k * chunk;
      for (int64_t j = 0; j < np && e == hipSuccess;) {
        int64_t run = 1;
        while (j + run < np && image_pids[(size_t)(p0 + j + run)] == image_pids[(size_t)(p0 + j)] + run) ++run;
        memcpy(buf + (size_t)j * kPage, db->page(image_pids[(size_t)(p0 + j)]), (size_t)run * kPage);
        j += run;
      }
      if (e == hipSuccess)
        e = hipMemcpyAsync(dimg + (size_t)p0 * kPage, buf, (size_t)np * kPage, hipMemcpyHostToDevice, s);
      if (e == hipSuccess) e = hipEventRecord(done[k], s);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (done[0]) hipEventDestroy(done[0]);
    if (done[1]) hipEventDestroy(done[1]);
  }
  std::vector<int32_t> page_of;
  page_of.reserve((size_t)npi_total);
  for (const auto& l : local_of) page_of.insert(page_of.end(), l.begin(), l.end());
  if (e == hipSuccess && npi_total > 0)
    e = hipMemcpy(dpage_of, page_of.data(), sizeof(int32_t) * page_of.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess && md_words > 0)
    e = hipMemcpy(dmd, mdw.data(), sizeof(uint64_t) * (size_t)md_words, hipMemcpyHostToDevice);
  int64_t pofs = 0;
  for (int32_t i = 0; i < n && e == hipSuccess && nrows > 0; ++i) {
    const ColumnPages& cp = cps[(size_t)i];
    const TCol& tc = t->cols[(size_t)i];
    PageDecodeArgs A{};
    A.image = dimg;
    A.image_pages = image_pages;
    A.page_of = dpage_of + pofs;
    A.npages = (int64_t)local_of[(size_t)i].size();
    A.rec_len = cp.rec_len;
    A.recs_per_page = cp.recs_per_page;
    A.kind = tc.attr_type == MBX_ATTR_STRING ? kStr : (tc.attr_type == MBX_ATTR_REAL ? kReal : kInt);
    A.size = tc.size;
    A.stride = tc.stride_w * 4;
    A.out = (uint8_t*)tc.dev;
    A.present = dpresent + (size_t)pw * (size_t)i;
    A.nrows = nrows;
    A.err = dflags;
    A.page_index0 = pi0[(size_t)i];
    A.pos_begin = r0;
    A.range = 1;
    e = launch_page_decode(A, s);
    pofs += A.npages;
  }
  if (e == hipSuccess && nrows > 0)
    e = launch_present_merge(dpresent, dpresent + pw, n - 1, pw, dmd, md_words, nrows, t->deleted, dflags + 1, s);
  int32_t flags[2] = {0, 0};
  if (e == hipSuccess) e = hipMemcpyAsync(flags, dflags, sizeof(flags), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  hipFree(dimg);
  hipFree(dpage_of);
  hipFree(dpresent);
  hipFree(dmd);
  hipFree(dflags);
  if (pinned) hipHostFree(pinned);
  if (e != hipSuccess) {
    mbx_table_free(t);
    return fail(MBX_E_DEVICE, "db_stage_range %s: %s", name, hipGetErrorString(e));
  }
  if (flags[0]) {
    mbx_table_free(t);
    return fail(MBX_E_INVALID, "db_stage_range %s: malformed data pages (flags 0x%x)", name, flags[0]);
  }
  if (flags[1] & 1) {
    mbx_table_free(t);
    return fail(MBX_E_INVALID, "Invalid position calculations: the column heapfiles of %s disagree", name);
  }
  if (!(flags[1] & 2) && t->deleted) {
    hipFree(t->deleted);
    t->deleted = nullptr;
    t->owns_deleted = false;
  }
  *out = t;
  return MBX_OK;
}

extern "C" int mbx_db_bitmap_stage_range(mbx_ctx* c, mbx_db* db, const char* filename, int64_t bit_begin,
                                         int64_t nbits, mbx_bitmap** out) {
  NOTNULL(c);
  NOTNULL(db);
  NOTNULL(filename);
  NOTNULL(out);
  *out = nullptr;
  if (nbits < 0 || bit_begin < 0 || (bit_begin & 63))
    return fail(MBX_E_INVALID, "bitmap_stage_range: bits [%lld, +%lld) (begin must be a multiple of 64)",
                (long long)bit_begin, (long long)nbits);
  const int32_t head = get_file_entry(db, filename);
  if (head == kInvalidPage) return fail(MBX_E_INVALID, "The file %s does not exist.", filename);
  const int64_t nw = words_for(nbits);
  std::vector<uint64_t> words((size_t)(nw > 0 ? nw : 1), 0ull);
  uint8_t* wb = reinterpret_cast<uint8_t*>(words.data());
  // BM.readBitSet's concatenation of the chain's records, keeping only the
  // bytes of [bit_begin / 8, bit_begin / 8 + 8 * nw)
  const int64_t b0 = bit_begin / 8, b1 = b0 + nw * 8;
  int64_t at = 0;  // byte offset of the current record in the concatenation
  int32_t p = head;
  int guard = 0;
  while (p != kInvalidPage && at < b1) {
    if (p < 0 || p >= db->num_pages || guard++ > db->num_pages)
      return fail(MBX_E_INVALID, "BitMapFile chain leaves the DB at page %d", p);
    const uint8_t* pg = db->page(p);
    const int32_t cnt = get16(pg + kSlotCnt);
    int32_t sl = 0;
    while (sl < cnt && hf_slot_len(pg, sl) == -1) ++sl;
    if (sl == cnt) return fail(MBX_E_INVALID, "InvalidSlotNumberException: BitMapFile page %d holds no record", p);
    const int32_t len = hf_slot_len(pg, sl), off = hf_slot_off(pg, sl);
    if (len < 0 || off + len > kPage) return fail(MBX_E_INVALID, "corrupt BitMapFile page %d", p);
    const int64_t lo = std::max(at, b0), hi = std::min(at + len, b1);
    if (lo < hi) memcpy(wb + (lo - b0), pg + off + (lo - at), (size_t)(hi - lo));
    at += len;
    p = get32(pg + kNext);
  }
  if (nbits & 63) words[(size_t)nw - 1] &= (1ull << (nbits & 63)) - 1ull;
  return mbx_bitmap_upload(c, nbits, words.data(), out);
}

// ------------------------------------------------- bitmap-index persistence

namespace {

// modified UTF-8 -> UTF-16 code units (DataInputStream.readUTF)
std::vector<uint16_t> mutf8_units(const std::string& s) {
  std::vector<uint16_t> u;
  for (size_t i = 0; i < s.size();) {
    const uint8_t b = (uint8_t)s[i];
    if (b < 0x80) {
      u.push_back(b);
      i += 1;
    } else if ((b & 0xE0) == 0xC0 && i + 1 < s.size()) {
      u.push_back((uint16_t)(((b & 0x1F) << 6) | ((uint8_t)s[i + 1] & 0x3F)));
      i += 2;
    } else if (i + 2 < s.size()) {
      u.push_back((uint16_t)(((b & 0x0F) << 12) | (((uint8_t)s[i + 1] & 0x3F) << 6) | ((uint8_t)s[i + 2] & 0x3F)));
      i += 3;
    } else {
      u.push_back(b);
      i += 1;
    }
  }
  return u;
}

int32_t java_string_hash(const std::string& mutf8) {
  uint32_t h = 0;
  for (uint16_t c : mutf8_units(mutf8)) h = 31u * h + c;
  return (int32_t)h;
}

// java.util.HashMap iteration order of keys put in the given order (JDK 8+:
// table of 16 at the first put, doubled when size exceeds 0.75 * capacity or
// when a bin reaches 8 nodes while the table is smaller than 64; buckets
// visited in index order, each bin in insertion order -- bins that would
// become trees keep list order here, a documented approximation)
std::vector<size_t> hashmap_order(const std::vector<int32_t>& hashes) {
  auto spread = [](int32_t h) { return (uint32_t)h ^ ((uint32_t)h >> 16); };
  uint32_t cap = 16;
  std::unordered_map<uint32_t, int> bins;
  auto rebuild = [&](size_t upto) {
    bins.clear();
    for (size_t j = 0; j < upto; ++j) bins[spread(hashes[j]) & (cap - 1)]++;
  };
  for (size_t i = 0; i < hashes.size(); ++i) {
    const uint32_t b = spread(hashes[i]) & (cap - 1);
    const int before = bins[b]++;
    if (before >= 8 && cap < 64) {  // treeifyBin -> resize()
      cap *= 2;
      rebuild(i + 1);
    }
    if (i + 1 > (size_t)(cap * 3 / 4)) {
      cap *= 2;
      rebuild(i + 1);
    }
  }
  std::vector<size_t> order(hashes.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
    return (spread(hashes[a]) & (cap - 1)) < (spread(hashes[b]) & (cap - 1));
  });
  return order;
}

constexpr int64_t kMaxDistinct = 65536;

int find_hdr_record(mbx_db* db, int32_t hdr, int32_t index, uint8_t** rec, int32_t* len) {
  int32_t k = 0;
  *rec = nullptr;
  int rc = heap_scan(db, hdr, [&](const DataPage& d, int32_t s, const uint8_t*, int32_t l) {
    if (k++ == index) {
      uint8_t* pg = db->page(d.pid);
      *rec = pg + hf_slot_off(pg, s);
      *len = l;
      return false;
    }
    return true;
  });
  if (rc) return rc;
  if (!*rec) return fail(MBX_E_INVALID, "hdr record %d is missing", index);
  return MBX_OK;
}

}  // namespace

extern "C" int mbx_db_create_bitmap_index(mbx_ctx* c, mbx_db* db, const char* name, const mbx_table* t, int32_t col,
                                          int32_t* nvalues) {
  NOTNULL(c);
  NOTNULL(db);
  NOTNULL(name);
  NOTNULL(t);
  if (nvalues) *nvalues = 0;
  Schema sc;
  int rc = read_schema(db, name, &sc);
  if (rc) return rc;
  if (col < 0 || col >= sc.ncols) return fail(MBX_E_RANGE, "createBitMapIndex: column %d of %d", col, sc.ncols);
  if ((int32_t)t->cols.size() != sc.ncols) return fail(MBX_E_INVALID, "createBitMapIndex: table is not %s", name);
  const int32_t type = sc.cols[(size_t)col].attr_type;
  if (type != MBX_ATTR_INTEGER && type != MBX_ATTR_STRING)
    return fail(MBX_E_UNSUPPORTED, "createBitMapIndex: AttrType %d columns have no bitmap index in the reference",
                type);
  if ((size_t)col < sc.bitmap_exist.size() && sc.bitmap_exist[(size_t)col] == 1) return MBX_OK;
  if ((rc = set_device(c))) return rc;
  const TCol& tc = t->cols[(size_t)col];
  const int64_t nrows = t->nrows;
  hipStream_t s = c->stream;

  // 1. distinct live values and their first positions (k_distinct)
  int64_t cap = 64;
  while (cap < 2 * std::min<int64_t>(nrows, kMaxDistinct)) cap *= 2;
  unsigned long long *keys = nullptr, *minpos = nullptr;
  int32_t* dflag = nullptr;
  HIPCHK(hipMalloc(&keys, sizeof(unsigned long long) * (size_t)cap));
  hipError_t e = hipMalloc(&minpos, sizeof(unsigned long long) * (size_t)cap);
  if (e == hipSuccess) e = hipMalloc(&dflag, sizeof(int32_t));
  if (e == hipSuccess) e = hipMemsetAsync(keys, 0xFF, sizeof(unsigned long long) * (size_t)cap, s);
  if (e == hipSuccess) e = hipMemsetAsync(minpos, 0xFF, sizeof(unsigned long long) * (size_t)cap, s);
  if (e == hipSuccess) e = hipMemsetAsync(dflag, 0, sizeof(int32_t), s);
  KCol kc;
  kc.base = tc.dev;
  kc.kind = type == MBX_ATTR_STRING ? kStr : kInt;
  kc.stride_w = tc.stride_w;
  if (e == hipSuccess) {
    DistinctArgs A;
    A.col = kc;
    A.nrows = nrows;
    A.del = t->deleted;
    A.keys = keys;
    A.minpos = minpos;
    A.cap = cap;
    A.overflow = dflag;
    // test knob (mbx_set_tuning "distinct_lds_probes"): 0 sends every row to the global table
    A.lds_probes = c->tune.distinct_lds_probes >= 0 ? c->tune.distinct_lds_probes : kLdsProbes;
    e = launch_distinct(A, s);
  }
  std::vector<unsigned long long> hmin((size_t)cap);
  int32_t overflow = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(hmin.data(), minpos, sizeof(unsigned long long) * (size_t)cap,
                                          hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(&overflow, dflag, sizeof(int32_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  hipFree(keys);
  hipFree(minpos);
  hipFree(dflag);
  if (e != hipSuccess) return fail(MBX_E_DEVICE, "createBitMapIndex: %s", hipGetErrorString(e));
  std::vector<int64_t> first;
  for (unsigned long long p : hmin)
    if (p != kEmptySlot) first.push_back((int64_t)p);
  if (overflow || (int64_t)first.size() > kMaxDistinct)
    return fail(MBX_E_UNSUPPORTED, "createBitMapIndex: more than %lld distinct values", (long long)kMaxDistinct);
  std::sort(first.begin(), first.end());
  const int32_t nv = (int32_t)first.size();
  if (nv == 0) {
    // no live row: the reference registers nothing and only sets the flag
    uint8_t* rec;
    int32_t len;
    if ((rc = find_hdr_record(db, get_file_entry(db, std::string(name) + ".hdr"), 5, &rec, &len))) return rc;
    if (col < len) rec[col] = 1;
    return MBX_OK;
  }

  // 2. the values themselves (device image of the first-occurrence rows)
  const int32_t vw = kc.kind == kStr ? tc.stride_w : 1;
  std::vector<uint32_t> vals((size_t)nv * (size_t)vw);
  {
    int64_t* drows = nullptr;
    uint32_t* dvals = nullptr;
    HIPCHK(hipMalloc(&drows, sizeof(int64_t) * (size_t)nv));
    e = hipMalloc(&dvals, sizeof(uint32_t) * vals.size());
    if (e == hipSuccess) e = hipMemcpyAsync(drows, first.data(), sizeof(int64_t) * (size_t)nv, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = launch_rows_fetch(kc, drows, nv, dvals, s);
    if (e == hipSuccess) e = hipMemcpyAsync(vals.data(), dvals, sizeof(uint32_t) * vals.size(), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    hipFree(drows);
    hipFree(dvals);
    if (e != hipSuccess) return fail(MBX_E_DEVICE, "createBitMapIndex: %s", hipGetErrorString(e));
  }
  std::vector<std::string> text((size_t)nv);
  std::vector<int32_t> hashes((size_t)nv);
  for (int32_t v = 0; v < nv; ++v) {
    if (kc.kind == kStr) {
      std::vector<uint8_t> buf((size_t)tc.size + 1, 0);
      decode_device_string((const uint8_t*)&vals[(size_t)v * vw], vw * 4, buf.data(), tc.size);
      text[(size_t)v] = std::string((const char*)buf.data(), strnlen((const char*)buf.data(), (size_t)tc.size));
      hashes[(size_t)v] = java_string_hash(text[(size_t)v]);
    } else {
      const int32_t x = (int32_t)vals[(size_t)v];
      text[(size_t)v] = std::to_string(x);
      hashes[(size_t)v] = x;  // Integer.hashCode
    }
  }

  // 3. one BitSet per value on the GPU
  std::vector<mbx_bitmap*> bms((size_t)nv, nullptr);
  if ((rc = index_build_encoded(c, t, col, vals.data(), nv, bms.data()))) return rc;
  auto free_all = [&]() {
    for (mbx_bitmap* b : bms) mbx_bitmap_free(b);
  };

  // 4. files, in the reference's order: per value (scan order) the header
  // page + file entry, then the hdr registry record; then the BitSet chunks
  // in HashMap order; then bitmapExist
  const std::string cf = name;
  const int32_t hdr = get_file_entry(db, cf + ".hdr");
  std::vector<int32_t> heads((size_t)nv);
  for (int32_t v = 0; v < nv && !rc; ++v) {
    const std::string key = std::to_string(col) + "." + text[(size_t)v];
    rc = bm_create_header(db, cf + ".bm." + key, &heads[(size_t)v]);
    std::vector<uint8_t> rec(key.size() + 2, 0);
    put_utf(rec.data(), key);
    int32_t pid, slot;
    if (!rc) rc = heap_insert(db, hdr, rec.data(), (int32_t)rec.size(), &pid, &slot);
  }
  std::vector<uint64_t> words;
  for (size_t k : hashmap_order(hashes)) {
    if (rc) break;
    mbx_bitmap* b = bms[k];
    words.assign((size_t)(b->nwords > 0 ? b->nwords : 1), 0ull);
    if (b->nwords > 0 && (rc = mbx_bitmap_download(c, b, words.data(), b->nwords))) break;
    rc = bm_insert_bitset(db, heads[k], bitset_bytes(words.data(), b->nwords));
  }
  free_all();
  if (rc) return rc;
  uint8_t* rec;
  int32_t len;
  if ((rc = find_hdr_record(db, hdr, 5, &rec, &len))) return rc;
  if (col < len) rec[col] = 1;
  if (nvalues) *nvalues = nv;
  return MBX_OK;
}

extern "C" int mbx_db_bitmap_values(mbx_db* db, const char* name, int32_t col, char* buf, int64_t cap,
                                    int32_t* count, int64_t* bytes) {
  NOTNULL(db);
  NOTNULL(name);
  Schema sc;
  int rc = read_schema(db, name, &sc);
  if (rc) return rc;
  const std::string prefix = std::to_string(col) + ".";
  std::string out;
  int32_t n = 0;
  for (const std::string& r : sc.bm_values) {
    if (r.compare(0, prefix.size(), prefix) != 0) continue;
    out += r.substr(prefix.size());
    out.push_back('\0');
    ++n;
  }
  if (count) *count = n;
  if (bytes) *bytes = (int64_t)out.size();
  if (buf && cap >= (int64_t)out.size()) memcpy(buf, out.data(), out.size());
  return MBX_OK;
}

extern "C" int mbx_db_bitmap_stage(mbx_ctx* c, mbx_db* db, const char* filename, int64_t nbits, mbx_bitmap** out) {
  NOTNULL(c);
  NOTNULL(db);
  NOTNULL(filename);
  NOTNULL(out);
  *out = nullptr;
  if (nbits < 0) return fail(MBX_E_INVALID, "bitmap_stage: nbits %lld", (long long)nbits);
  const int32_t head = get_file_entry(db, filename);
  if (head == kInvalidPage) return fail(MBX_E_INVALID, "The file %s does not exist.", filename);
  std::vector<uint8_t> bytes;
  int rc = bm_read_bytes(db, head, &bytes);
  if (rc) return rc;
  const int64_t nw = words_for(nbits);
  std::vector<uint64_t> words((size_t)(nw > 0 ? nw : 1), 0ull);
  memcpy(words.data(), bytes.data(), std::min<size_t>(bytes.size(), (size_t)nw * 8));
  if (nbits & 63) words[(size_t)nw - 1] &= (1ull << (nbits & 63)) - 1ull;
  return mbx_bitmap_upload(c, nbits, words.data(), out);
}

// ------------------------------------------------------ delete lifecycle

namespace {

void free_page(mbx_db* db, int32_t pid) {
  set_page_bit(db, pid, false);
  if (pid < db->alloc_hint) db->alloc_hint = pid;
}

// HFPage.deleteRecord (R/heap/HFPage.java:398-450): close the hole by
// shifting the records below it up, fix their offsets, empty the slot
int hf_delete(uint8_t* pg, int32_t slot) {
  const int32_t cnt = get16(pg + kSlotCnt);
  const int32_t len = slot >= 0 && slot < cnt ? hf_slot_len(pg, slot) : -1;
  if (len <= 0) return fail(MBX_E_INVALID, "InvalidSlotNumberException: HEAPFILE: INVALID_SLOTNO");
  const int32_t off = hf_slot_off(pg, slot);
  const int32_t used = get16(pg + kUsedPtr);
  memmove(pg + used + len, pg + used, (size_t)(off - used));
  for (int32_t i = 0; i < cnt; ++i) {
    if (hf_slot_len(pg, i) >= 0) {
      const int32_t o = hf_slot_off(pg, i);
      if (o < off) put16(pg + kDpFixed + i * kSlotSize + 2, o + len);
    }
  }
  put16(pg + kUsedPtr, used + len);
  put16(pg + kFreeSpace, get16(pg + kFreeSpace) + len);
  put16(pg + kDpFixed + slot * kSlotSize, -1);
  put16(pg + kDpFixed + slot * kSlotSize + 2, 0);
  return MBX_OK;
}

bool hf_empty(const uint8_t* pg) {
  const int32_t cnt = get16(pg + kSlotCnt);
  for (int32_t i = 0; i < cnt; ++i)
    if (hf_slot_len(pg, i) != -1) return false;
  return true;
}

// directory page -> its index in the chain (Heapfile.loadPositionBuffer's dirPageOffset)
std::unordered_map<int32_t, int32_t> dir_offsets(mbx_db* db, int32_t first_dir) {
  std::unordered_map<int32_t, int32_t> m;
  int32_t d = first_dir, k = 0;
  while (d != kInvalidPage && k <= db->num_pages) {
    m[d] = k++;
    d = get32(db->page(d) + kNext);
  }
  return m;
}

// Heapfile.deleteRecord (R/heap/Heapfile.java:523-600)
int heap_delete(mbx_db* db, int32_t first_dir, int32_t pid, int32_t slot,
                const std::unordered_map<int32_t, int32_t>& offsets, std::vector<int32_t>* freed_dir) {
  int32_t dir = first_dir, dslot = -1;
  for (int guard = 0; dir != kInvalidPage && guard <= db->num_pages; ++guard) {
    const uint8_t* dp = db->page(dir);
    const int32_t cnt = get16(dp + kSlotCnt);
    for (int32_t s = 0; s < cnt && dslot < 0; ++s)
      if (hf_slot_len(dp, s) != -1 && get32(dp + hf_slot_off(dp, s) + 4) == pid) dslot = s;
    if (dslot >= 0) break;
    dir = get32(dp + kNext);
  }
  if (dslot < 0) return fail(MBX_E_INVALID, "Heapfile.deleteRecord: record (%d, %d) not found", pid, slot);
  uint8_t* dp = db->page(dir);
  uint8_t* info = dp + hf_slot_off(dp, dslot);
  uint8_t* pg = db->page(pid);
  int rc = hf_delete(pg, slot);
  if (rc) return rc;
  const int32_t recct = get16(info + 2) - 1;
  put16(info + 2, recct);
  db->hints.erase(first_dir);
  if (recct >= 1) {
    put16(info, hf_available(pg));
    return MBX_OK;
  }
  free_page(db, pid);
  if ((rc = hf_delete(dp, dslot))) return rc;
  const int32_t prev = get32(dp + kPrev);
  if (hf_empty(dp) && prev != kInvalidPage) {
    const int32_t next = get32(dp + kNext);
    put32(db->page(prev) + kNext, next);
    if (next != kInvalidPage) put32(db->page(next) + kPrev, prev);
    auto it = offsets.find(dir);
    if (it != offsets.end()) freed_dir->push_back(it->second);
    free_page(db, dir);
  }
  return MBX_OK;
}

// a BitMapFile in memory: the BitSet bytes + the chain of its pages
struct BmFile {
  int32_t head = kInvalidPage;
  std::vector<int32_t> pages;  // offsetToPage
  std::vector<uint8_t> bytes;
};

int bm_load(mbx_db* db, const std::string& name, BmFile* f) {
  f->head = get_file_entry(db, name);
  if (f->head == kInvalidPage) return fail(MBX_E_INVALID, "The file %s does not exist.", name.c_str());
  int rc = bm_read_bytes(db, f->head, &f->bytes);
  if (rc) return rc;
  f->pages.clear();
  for (int32_t p = f->head; p != kInvalidPage; p = get32(db->page(p) + kNext)) f->pages.push_back(p);
  return MBX_OK;
}

bool bm_get(const BmFile& f, int64_t pos) {
  return (size_t)(pos >> 3) < f.bytes.size() && ((f.bytes[(size_t)(pos >> 3)] >> (pos & 7)) & 1);
}

int64_t bm_next_set(const BmFile& f, int64_t from) {
  for (int64_t p = from; p < (int64_t)f.bytes.size() * 8; ++p)
    if (bm_get(f, p)) return p;
  return -1;
}

// rewrite chunk `k` (1000 bytes) of the in-memory BitSet into its page's record
void bm_write_chunk(mbx_db* db, const BmFile& f, int64_t k) {
  uint8_t* pg = db->page(f.pages[(size_t)k]);
  const int32_t cnt = get16(pg + kSlotCnt);
  int32_t s = 0;
  while (s < cnt && hf_slot_len(pg, s) == -1) ++s;
  if (s == cnt) return;
  uint8_t* rec = pg + hf_slot_off(pg, s);
  const int32_t len = hf_slot_len(pg, s);
  // BitSet.toByteArray() stops at the last non-zero byte
  int64_t nb = (int64_t)f.bytes.size();
  while (nb > 0 && f.bytes[(size_t)nb - 1] == 0) --nb;
  memset(rec, 0, (size_t)len);
  const int64_t start = k * kBmRecord;
  if (start < nb) memcpy(rec, f.bytes.data() + start, (size_t)std::min<int64_t>(len, nb - start));
}

// BitMapFile.delete(position) (R/bitmap/BitMapFile.java:245-290)
void bm_delete(mbx_db* db, BmFile& f, int64_t pos) {
  if (!bm_get(f, pos)) return;
  f.bytes[(size_t)(pos >> 3)] &= (uint8_t)~(1u << (pos & 7));
  const int64_t chunk = (int64_t)kBmRecord * 8;
  const int64_t offset = pos / chunk;
  if (bm_next_set(f, offset * chunk) == -1 && offset != 0) {
    int64_t cur = offset;
    while (bm_next_set(f, cur * chunk) == -1 && cur != 0) {
      if ((size_t)cur < f.pages.size()) {
        free_page(db, f.pages[(size_t)cur]);
        f.pages.resize((size_t)cur);
      }
      --cur;
    }
    put32(db->page(f.pages[(size_t)cur]) + kNext, kInvalidPage);
    return;
  }
  if ((size_t)offset < f.pages.size()) bm_write_chunk(db, f, offset);
}

// BitMapFile.purgeDelete (R/bitmap/BitMapFile.java:320-365) + BM.updateBitSet (R/bitmap/BM.java:216-290)
void bm_purge(mbx_db* db, BmFile& f, const std::vector<int64_t>& list, const std::vector<int64_t>& ranges) {
  if (ranges.empty()) {
    for (int64_t p : list) bm_delete(db, f, p);
    return;
  }
  for (int64_t p : list)
    if (bm_get(f, p)) f.bytes[(size_t)(p >> 3)] &= (uint8_t)~(1u << (p & 7));
  int64_t length = 0;  // BitSet.length(): highest set bit + 1
  for (int64_t b = (int64_t)f.bytes.size() - 1; b >= 0 && !length; --b)
    if (f.bytes[(size_t)b]) length = b * 8 + (32 - __builtin_clz((unsigned)f.bytes[(size_t)b]));
  std::vector<uint8_t> out(f.bytes.size(), 0);
  int64_t position = 0, start = 0;
  auto copy = [&](int64_t from, int64_t to) {
    for (int64_t j = from; j < to; ++j, ++position)
      if (bm_get(f, j)) out[(size_t)(position >> 3)] |= (uint8_t)(1u << (position & 7));
  };
  for (size_t i = 0; i + 1 < ranges.size(); i += 2) {
    copy(start, ranges[i]);
    start = ranges[i + 1];
  }
  copy(start, length);
  int64_t nb = (int64_t)out.size();
  while (nb > 0 && out[(size_t)nb - 1] == 0) --nb;
  if (nb == 0) return;  // BM.updateBitSet throws on an empty BitSet: the file keeps its old image
  f.bytes.assign(out.begin(), out.begin() + nb);
  const int64_t nchunks = (nb + kBmRecord - 1) / kBmRecord;
  for (int64_t k = 0; k < nchunks && (size_t)k < f.pages.size(); ++k) bm_write_chunk(db, f, k);
  for (size_t k = (size_t)nchunks; k < f.pages.size(); ++k) free_page(db, f.pages[k]);
  if ((size_t)nchunks < f.pages.size()) f.pages.resize((size_t)nchunks);
  put32(db->page(f.pages.back()) + kNext, kInvalidPage);
}

// DB.delete_file_entry (R/diskmgr/DB.java:510-560): pid -1, name "\0"
void delete_file_entry(mbx_db* db, const std::string& name) {
  for (int32_t hp = 0; hp != kInvalidPage;) {
    uint8_t* pg = db->page(hp);
    const int32_t n = get32(pg + 4);
    for (int32_t e = 0; e < n; ++e) {
      uint8_t* ent = pg + kStartEntries + e * kFileEntry;
      if (get32(ent) != kInvalidPage && get_utf(ent + 4, kMaxName + 2) == name) {
        put32(ent, kInvalidPage);
        put_utf(ent + 4, std::string("\xC0\x80", 2));  // writeUTF("\0")
        return;
      }
    }
    hp = get32(pg);
  }
}

// Heapfile.deleteFile (R/heap/Heapfile.java:1148-1204)
void heap_delete_file(mbx_db* db, const std::string& name) {
  const int32_t first = get_file_entry(db, name);
  if (first == kInvalidPage) return;
  for (int32_t d = first; d != kInvalidPage;) {
    const uint8_t* dp = db->page(d);
    const int32_t cnt = get16(dp + kSlotCnt);
    for (int32_t s = 0; s < cnt; ++s)
      if (hf_slot_len(dp, s) != -1) free_page(db, get32(dp + hf_slot_off(dp, s) + 4));
    const int32_t next = get32(dp + kNext);
    free_page(db, d);
    d = next;
  }
  db->hints.erase(first);
  delete_file_entry(db, name);
}

}  // namespace

extern "C" int mbx_db_mark_deleted_many(mbx_db* db, const char* name, const int64_t* positions, int64_t n) {
  NOTNULL(db);
  NOTNULL(name);
  if (n < 0) return fail(MBX_E_INVALID, "mark_deleted: n %lld", (long long)n);
  if (n == 0) return MBX_OK;
  NOTNULL(positions);
  Schema sc;
  int rc = read_schema(db, name, &sc);
  if (rc) return rc;
  std::vector<ColumnPages> cps((size_t)sc.ncols);
  for (int32_t i = 0; i < sc.ncols; ++i)
    if ((rc = column_pages(db, std::string(name) + "." + std::to_string(i), record_len(sc.cols[(size_t)i]),
                           &cps[(size_t)i])))
      return rc;
  const int32_t md = get_file_entry(db, std::string(name) + ".md");
  if (md == kInvalidPage) return fail(MBX_E_INVALID, "%s.md is missing", name);
  int32_t dtid;
  if ((rc = heap_open(db, std::string(name) + ".dtid", true, &dtid))) return rc;
  std::vector<uint8_t> tid((size_t)sc.ncols * 8);
  for (int64_t k = 0; k < n; ++k) {
    const int64_t position = positions[k];
    if (position < 0) return fail(MBX_E_INVALID, "Invalid position");
    for (int32_t i = 0; i < sc.ncols; ++i) {
      const ColumnPages& cp = cps[(size_t)i];
      const int64_t pi = position / cp.recs_per_page;
      if (pi >= (int64_t)cp.page_of.size() || cp.page_of[(size_t)pi] == kInvalidPage)
        return fail(MBX_E_INVALID, "Invalid Position %lld", (long long)position);
      put32(tid.data() + 8 * i, (int32_t)(position - pi * cp.recs_per_page));  // RID.writeToByteArray: slotNo
      put32(tid.data() + 8 * i + 4, cp.page_of[(size_t)pi]);                  // then pageNo
    }
    if ((rc = bm_set_bit(db, md, position))) return rc;
    int32_t pid, slot;
    if ((rc = heap_insert(db, dtid, tid.data(), (int32_t)tid.size(), &pid, &slot))) return rc;
  }
  return MBX_OK;
}

extern "C" int mbx_db_purge(mbx_db* db, const char* name) {
  NOTNULL(db);
  NOTNULL(name);
  Schema sc;
  int rc = read_schema(db, name, &sc);
  if (rc) return rc;
  const std::string cf = name;
  for (uint8_t b : sc.btree_exist)
    if (b == 1) return fail(MBX_E_UNSUPPORTED, "purge of %s: B-tree indexes are out of scope", name);
  std::vector<int32_t> heaps((size_t)sc.ncols);
  std::vector<std::unordered_map<int32_t, int32_t>> offsets((size_t)sc.ncols);
  std::vector<std::vector<int32_t>> freed((size_t)sc.ncols);
  for (int32_t i = 0; i < sc.ncols; ++i) {
    heaps[(size_t)i] = get_file_entry(db, cf + "." + std::to_string(i));
    if (heaps[(size_t)i] == kInvalidPage) return fail(MBX_E_INVALID, "%s.%d is missing", name, i);
    offsets[(size_t)i] = dir_offsets(db, heaps[(size_t)i]);
  }
  // 1. every TID of cf.dtid: delete its record from every column heapfile
  const int32_t dtid = get_file_entry(db, cf + ".dtid");
  std::vector<std::vector<uint8_t>> tids;
  if (dtid != kInvalidPage && (rc = heap_scan(db, dtid, [&](const DataPage&, int32_t, const uint8_t* r, int32_t len) {
        tids.emplace_back(r, r + len);
        return true;
      })))
    return rc;
  for (const auto& t : tids) {
    if ((int64_t)t.size() < 8LL * sc.ncols) return fail(MBX_E_INVALID, "%s.dtid: short TID record", name);
    for (int32_t i = 0; i < sc.ncols; ++i)
      if ((rc = heap_delete(db, heaps[(size_t)i], get32(t.data() + 8 * i + 4), get32(t.data() + 8 * i),
                            offsets[(size_t)i], &freed[(size_t)i])))
        return rc;
  }
  // 2. the deleted positions (markedDeleted, ascending)
  BmFile md;
  if ((rc = bm_load(db, cf + ".md", &md))) return rc;
  std::vector<int64_t> list;
  for (int64_t p = bm_next_set(md, 0); p != -1; p = bm_next_set(md, p + 1)) list.push_back(p);
  // 3. every bitmap index: clear them, drop the position ranges of removed
  //    directory pages (values in HashSet iteration order)
  for (int32_t i = 0; i < sc.ncols; ++i) {
    std::vector<int32_t> offs = freed[(size_t)i];
    std::sort(offs.begin(), offs.end());
    const int64_t per_dir = (int64_t)kRecsPerDirPage * recs_per_data_page(record_len(sc.cols[(size_t)i]));
    std::vector<int64_t> ranges;
    for (int32_t o : offs) {
      ranges.push_back((int64_t)o * per_dir);
      ranges.push_back((int64_t)(o + 1) * per_dir);
    }
    const std::string prefix = std::to_string(i) + ".";
    std::vector<std::string> vals;
    std::vector<int32_t> hashes;
    for (const std::string& r : sc.bm_values) {
      if (r.compare(0, prefix.size(), prefix) != 0) continue;
      vals.push_back(r.substr(prefix.size()));
      hashes.push_back(sc.cols[(size_t)i].attr_type == MBX_ATTR_STRING ? java_string_hash(vals.back())
                                                                      : (int32_t)atoi(vals.back().c_str()));
    }
    for (size_t k : hashmap_order(hashes)) {
      BmFile f;
      if (bm_load(db, cf + ".bm." + prefix + vals[k], &f)) continue;  // registered without a file
      bm_purge(db, f, list, ranges);
    }
  }
  // 4. markedDeleted.delete(position) for each; 5. a fresh cf.dtid
  for (int64_t p : list) bm_delete(db, md, p);
  heap_delete_file(db, cf + ".dtid");
  int32_t fresh;
  return heap_open(db, cf + ".dtid", true, &fresh);
}
