// CPU unit test of the C++ mirror's Jtuple (heap::Tuple, R/heap/Tuple.java:194-343):
// the per-field accessors and the all-int bulk copy (setIntFlds) accept and
// reject exactly the same fields.  Prints one line per check; exit 0 = pass.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../minibase-columnar-database_amd/host/minibase.hpp"

using namespace minibase;
using global::AttrType;

static int fails = 0;
#define EXPECT(c)                                     \
  do {                                                \
    if (!(c)) {                                       \
      printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      fails++;                                        \
    }                                                 \
  } while (0)

template <class E, class F>
static bool throws(F f) {
  try {
    f();
  } catch (const E&) {
    return true;
  } catch (...) {
    return false;
  }
  return false;
}

int main() {
  heap::Tuple J;
  J.setHdr({AttrType(AttrType::attrInteger), AttrType(AttrType::attrInteger), AttrType(AttrType::attrString),
            AttrType(AttrType::attrInteger)},
           {8});
  const int32_t a[3] = {10, 11, 12}, b[3] = {20, 21, 22}, c[3] = {30, 31, 32};
  const int32_t* cols[3] = {a, b, c};
  J.setIntFlds(cols, 2, 2);  // fields 1, 2 = row 2
  EXPECT(J.getIntFld(1) == 12 && J.getIntFld(2) == 22);
  // field 3 is a string: the bulk copy of 3 fields fails as setIntFld(3) does
  EXPECT(throws<iterator::UnknowAttrType>([&] { J.setIntFlds(cols, 0, 3); }));
  EXPECT(throws<iterator::UnknowAttrType>([&] { J.setIntFld(3, 1); }));
  EXPECT(J.getIntFld(1) == 12);  // nothing written by the failed call
  heap::Tuple K;
  K.setHdr({AttrType(AttrType::attrInteger), AttrType(AttrType::attrInteger)}, {});
  K.setIntFlds(cols, 1, 2);
  EXPECT(K.getIntFld(1) == 11 && K.getIntFld(2) == 21);
  // more fields than the tuple has: FieldNumberOutOfBoundException, as setIntFld(3)
  EXPECT(throws<iterator::FieldNumberOutOfBoundException>([&] { K.setIntFlds(cols, 0, 3); }));
  EXPECT(throws<iterator::FieldNumberOutOfBoundException>([&] { K.setIntFld(3, 1); }));
  EXPECT(throws<iterator::FieldNumberOutOfBoundException>([&] { K.getIntFld(0); }));
  // a header change re-derives the int prefix
  K.setHdr({AttrType(AttrType::attrReal), AttrType(AttrType::attrInteger)}, {});
  EXPECT(throws<iterator::UnknowAttrType>([&] { K.setIntFlds(cols, 0, 1); }));
  K.setFloFld(1, 2.5f);
  EXPECT(K.getFloFld(1) == 2.5f);
  printf("%s\n", fails ? "TUPLE_TEST_FAIL" : "TUPLE_TEST_OK");
  return fails ? 1 : 0;
}
