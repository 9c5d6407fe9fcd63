/*
 * mbx_jni.c -- JNI glue between the Java engine (R/ = minijava/src of
 * Neehaarika/MiniBase-Columnar-Database) and the MI355X executor's C-ABI
 * (include/mbx.h, include/mbx_db.h).  Every native method of
 * java/global/Native.java is a thin wrapper: Java objects in, the C-ABI's
 * plain structs out, MBX_E_* codes rethrown as the reference's exceptions.
 *
 * NOT COMPILED IN THIS IMAGE: there is no JDK here or on the GPU box (no
 * jni.h, no javac).  jni/Makefile builds libmbx_jni.so only where
 * $JAVA_HOME/include/jni.h exists:
 *   make -C jni JAVA_HOME=/usr/lib/jvm/...   ->  jni/libmbx_jni.so
 * The same C-ABI calls, argument for argument, are exercised by the C++
 * mirror (minibase-columnar-database_amd/host/) and the ctypes binding in
 * the test suite.
 *
 * Exception mapping: MBX_E_TYPE -> PredEvalException
 * (a plan) or UnknowAttrType, MBX_E_RANGE -> heap.FieldNumberOutOfBoundException,
 * MBX_E_INVALID -> the caller's FileScanException / IndexException,
 * MBX_E_DEVICE / MBX_E_NOMEM / MBX_E_UNSUPPORTED -> chainexception.ChainException.
 * Every reference exception class has the (Exception prev, String msg)
 * constructor (R/chainexception/ChainException.java:20), which is what
 * throw_chain calls.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mbx.h"
#include "../include/mbx_db.h"
#include "../include/mbx_join.h"

#define H(p) ((jlong)(intptr_t)(p))
#define P(T, j) ((T *)(intptr_t)(j))

static const char *kChain = "chainexception/ChainException";
static const char *kFileScan = "iterator/FileScanException";
static const char *kPredEval = "iterator/PredEvalException";
static const char *kIndex = "index/IndexException";
static const char *kFieldRange = "heap/FieldNumberOutOfBoundException";

/* throws cls(null, mbx_last_error()) */
static void throw_chain(JNIEnv *env, const char *cls, const char *msg) {
  jclass c = (*env)->FindClass(env, cls);
  if (!c) return; /* NoClassDefFoundError pending */
  jmethodID ctor = (*env)->GetMethodID(env, c, "<init>", "(Ljava/lang/Exception;Ljava/lang/String;)V");
  if (!ctor) {
    (*env)->ExceptionClear(env);
    (*env)->ThrowNew(env, c, msg);
    return;
  }
  jstring s = (*env)->NewStringUTF(env, msg);
  jobject e = (*env)->NewObject(env, c, ctor, (jobject)NULL, s);
  if (e) (*env)->Throw(env, (jthrowable)e);
}

/* rc != MBX_OK: throw the class for rc (op_cls for MBX_E_INVALID / _TYPE); returns 1 */
static int check(JNIEnv *env, int rc, const char *op_cls) {
  if (rc == MBX_OK) return 0;
  const char *cls = kChain;
  switch (rc) {
    case MBX_E_TYPE: cls = op_cls == kFileScan ? kPredEval : op_cls; break;
    case MBX_E_RANGE: cls = kFieldRange; break;
    case MBX_E_INVALID: cls = op_cls; break;
    default: cls = kChain;
  }
  throw_chain(env, cls, mbx_last_error());
  return 1;
}

/* ---- Java field access (classes of the reference) ----------------------- */

typedef struct {
  jfieldID ce_op, ce_t1, ce_t2, ce_o1, ce_o2, ce_it, ce_next;
  jfieldID op_val, at_val, it_val;
  jfieldID od_sym, od_str, od_int, od_real;
  jfieldID fs_off;
} Fields;

static int fields_of(JNIEnv *env, Fields *f) {
  jclass ce = (*env)->FindClass(env, "iterator/CondExpr");
  jclass ao = (*env)->FindClass(env, "global/AttrOperator");
  jclass at = (*env)->FindClass(env, "global/AttrType");
  jclass it = (*env)->FindClass(env, "global/IndexType");
  jclass od = (*env)->FindClass(env, "iterator/Operand");
  jclass fs = (*env)->FindClass(env, "iterator/FldSpec");
  if (!ce || !ao || !at || !it || !od || !fs) return -1;
  f->ce_op = (*env)->GetFieldID(env, ce, "op", "Lglobal/AttrOperator;");
  f->ce_t1 = (*env)->GetFieldID(env, ce, "type1", "Lglobal/AttrType;");
  f->ce_t2 = (*env)->GetFieldID(env, ce, "type2", "Lglobal/AttrType;");
  f->ce_o1 = (*env)->GetFieldID(env, ce, "operand1", "Literator/Operand;");
  f->ce_o2 = (*env)->GetFieldID(env, ce, "operand2", "Literator/Operand;");
  f->ce_it = (*env)->GetFieldID(env, ce, "indexType", "Lglobal/IndexType;");
  f->ce_next = (*env)->GetFieldID(env, ce, "next", "Literator/CondExpr;");
  f->op_val = (*env)->GetFieldID(env, ao, "attrOperator", "I");
  f->at_val = (*env)->GetFieldID(env, at, "attrType", "I");
  f->it_val = (*env)->GetFieldID(env, it, "indexType", "I");
  f->od_sym = (*env)->GetFieldID(env, od, "symbol", "Literator/FldSpec;");
  f->od_str = (*env)->GetFieldID(env, od, "string", "Ljava/lang/String;");
  f->od_int = (*env)->GetFieldID(env, od, "integer", "I");
  f->od_real = (*env)->GetFieldID(env, od, "real", "F");
  f->fs_off = (*env)->GetFieldID(env, fs, "offset", "I");
  return (*env)->ExceptionCheck(env) ? -1 : 0;
}

/* Strings borrowed from the JVM for the duration of one C-ABI call:
 * GetStringUTFChars returns modified UTF-8 -- exactly the bytes
 * DataOutputStream.writeUTF stores (R/global/Convert.java:254-275), which is
 * what mbx_operand.string expects. */
typedef struct {
  jstring js[2 * MBX_MAX_TERMS];
  const char *cs[2 * MBX_MAX_TERMS];
  int n;
} Strings;

static void strings_release(JNIEnv *env, Strings *s) {
  for (int i = 0; i < s->n; i++) (*env)->ReleaseStringUTFChars(env, s->js[i], s->cs[i]);
  s->n = 0;
}

/* CondExpr.typeN + Operand -> mbx_operand (R/iterator/CondExpr.java:12-57, Operand.java) */
static int operand_of(JNIEnv *env, const Fields *f, jobject type, jobject od, Strings *ss, mbx_operand *m) {
  memset(m, 0, sizeof(*m));
  m->type = type ? (*env)->GetIntField(env, type, f->at_val) : MBX_ATTR_NULL;
  if (!od) return 0;
  m->integer = (*env)->GetIntField(env, od, f->od_int);
  m->real = (*env)->GetFloatField(env, od, f->od_real);
  if (m->type == MBX_ATTR_SYMBOL) {
    jobject sym = (*env)->GetObjectField(env, od, f->od_sym);
    m->fld = sym ? (*env)->GetIntField(env, sym, f->fs_off) : 0;
  } else if (m->type == MBX_ATTR_STRING) {
    jstring js = (jstring)(*env)->GetObjectField(env, od, f->od_str);
    if (js) {
      if (ss->n >= 2 * MBX_MAX_TERMS) return -1;
      const char *cs = (*env)->GetStringUTFChars(env, js, NULL);
      if (!cs) return -1;
      ss->js[ss->n] = js;
      ss->cs[ss->n] = cs;
      ss->n++;
      m->string = cs;
      m->string_len = (int32_t)(*env)->GetStringUTFLength(env, js);
    }
  }
  return 0;
}

/* CondExpr[] (null-terminated array of .next chains: conjuncts of OR-lists,
 * R/iterator/PredEval.java:25-183) -> mbx_cnf.  filter == null is `p == null`. */
static int cnf_of(JNIEnv *env, jobjectArray filter, mbx_condexpr *conds, int32_t *offs, mbx_cnf *cnf, Strings *ss) {
  Fields f;
  if (fields_of(env, &f)) return -1;
  int32_t k = 0, c = 0;
  offs[0] = 0;
  const jsize len = filter ? (*env)->GetArrayLength(env, filter) : 0;
  for (; c < len; c++) {
    jobject e = (*env)->GetObjectArrayElement(env, filter, c);
    if (!e) break; /* the null terminator */
    if (c >= MBX_MAX_CONJ) {
      throw_chain(env, kPredEval, "CondExpr[]: more conjuncts than MBX_MAX_CONJ");
      return -1;
    }
    for (; e; e = (*env)->GetObjectField(env, e, f.ce_next)) {
      if (k >= MBX_MAX_TERMS) {
        throw_chain(env, kPredEval, "CondExpr[]: more terms than MBX_MAX_TERMS");
        return -1;
      }
      mbx_condexpr *m = &conds[k++];
      memset(m, 0, sizeof(*m));
      jobject op = (*env)->GetObjectField(env, e, f.ce_op);
      jobject it = (*env)->GetObjectField(env, e, f.ce_it);
      m->op = op ? (*env)->GetIntField(env, op, f.op_val) : MBX_OP_NOP;
      m->index_type = it ? (*env)->GetIntField(env, it, f.it_val) : MBX_INDEX_NONE;
      if (operand_of(env, &f, (*env)->GetObjectField(env, e, f.ce_t1), (*env)->GetObjectField(env, e, f.ce_o1), ss,
                     &m->operand1) ||
          operand_of(env, &f, (*env)->GetObjectField(env, e, f.ce_t2), (*env)->GetObjectField(env, e, f.ce_o2), ss,
                     &m->operand2)) {
        if (!(*env)->ExceptionCheck(env)) throw_chain(env, kPredEval, "CondExpr operand");
        return -1;
      }
    }
    offs[c + 1] = k;
  }
  cnf->conds = conds;
  cnf->conj_offsets = offs;
  cnf->nconj = c;
  return 0;
}

/* ---- context ------------------------------------------------------------- */

JNIEXPORT jint JNICALL Java_global_Native_deviceCount(JNIEnv *env, jclass cls) {
  int32_t n = 0;
  (void)env, (void)cls;
  if (mbx_device_count(&n)) return 0;
  return n;
}

JNIEXPORT jlong JNICALL Java_global_Native_init(JNIEnv *env, jclass cls, jint device) {
  mbx_ctx *c = NULL;
  (void)cls;
  if (check(env, mbx_init(device, &c), kChain)) return 0;
  return H(c);
}

JNIEXPORT void JNICALL Java_global_Native_free(JNIEnv *env, jclass cls, jlong ctx) {
  (void)env, (void)cls;
  mbx_free(P(mbx_ctx, ctx));
}

/* waits for the context stream: a NaN an async scan reached raises here */
JNIEXPORT void JNICALL Java_global_Native_sync(JNIEnv *env, jclass cls, jlong ctx) {
  (void)cls;
  check(env, mbx_sync(P(mbx_ctx, ctx)), kPredEval);
}

/* ---- tables -------------------------------------------------------------- */

/* cols: direct ByteBuffers in host order, one per column (char(n): n bytes
 * of zero-padded modified UTF-8 per row); deleted: BitSet.toLongArray() of
 * cf.md or null */
JNIEXPORT jlong JNICALL Java_global_Native_tableStage(JNIEnv *env, jclass cls, jlong ctx, jintArray types,
                                                      jshortArray sizes, jlong nrows, jobjectArray cols,
                                                      jlongArray deleted, jlong row_offset) {
  (void)cls;
  const jsize nc = (*env)->GetArrayLength(env, types);
  if (nc <= 0 || nc > 4096 || (*env)->GetArrayLength(env, sizes) != nc || (*env)->GetArrayLength(env, cols) != nc) {
    throw_chain(env, kFileScan, "tableStage: column arrays disagree");
    return 0;
  }
  mbx_col_desc *d = (mbx_col_desc *)calloc((size_t)nc, sizeof(mbx_col_desc));
  const void **host = (const void **)calloc((size_t)nc, sizeof(void *));
  jint *t = (*env)->GetIntArrayElements(env, types, NULL);
  jshort *s = (*env)->GetShortArrayElements(env, sizes, NULL);
  int bad = !d || !host || !t || !s;
  for (jsize j = 0; !bad && j < nc; j++) {
    d[j].attr_type = t[j];
    d[j].size = t[j] == MBX_ATTR_STRING ? s[j] : 4;
    jobject buf = (*env)->GetObjectArrayElement(env, cols, j);
    host[j] = buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL;
    const jlong cap = buf ? (*env)->GetDirectBufferCapacity(env, buf) : -1;
    bad = !host[j] || cap < nrows * (jlong)d[j].size;
  }
  if (t) (*env)->ReleaseIntArrayElements(env, types, t, JNI_ABORT);
  if (s) (*env)->ReleaseShortArrayElements(env, sizes, s, JNI_ABORT);
  mbx_table *out = NULL;
  if (bad) {
    throw_chain(env, kFileScan, "tableStage: every column needs a direct ByteBuffer of nrows values");
  } else {
    jlong *del = deleted ? (*env)->GetLongArrayElements(env, deleted, NULL) : NULL;
    const jsize dw = deleted ? (*env)->GetArrayLength(env, deleted) : 0;
    uint64_t *words = NULL;
    if (del) { /* cf.md's BitSet may be shorter than the table (toLongArray drops zero tail words) */
      const int64_t need = (nrows + 63) / 64;
      words = (uint64_t *)calloc((size_t)(need > 0 ? need : 1), sizeof(uint64_t));
      if (words) memcpy(words, del, sizeof(uint64_t) * (size_t)(dw < need ? dw : need));
      (*env)->ReleaseLongArrayElements(env, deleted, del, JNI_ABORT);
    }
    check(env, mbx_table_stage(P(mbx_ctx, ctx), d, (int32_t)nc, nrows, host, words, row_offset, &out), kFileScan);
    free(words);
  }
  free(d);
  free(host);
  return H(out);
}

JNIEXPORT void JNICALL Java_global_Native_tableFree(JNIEnv *env, jclass cls, jlong t) {
  (void)env, (void)cls;
  mbx_table_free(P(mbx_table, t));
}

JNIEXPORT jlong JNICALL Java_global_Native_tableRows(JNIEnv *env, jclass cls, jlong t) {
  (void)cls;
  int64_t nrows = 0, row_offset = 0;
  int32_t ncols = 0;
  check(env, mbx_table_info(P(mbx_table, t), &nrows, &row_offset, &ncols), kFileScan);
  return nrows;
}

JNIEXPORT jlong JNICALL Java_global_Native_dbOpen(JNIEnv *env, jclass cls, jstring path) {
  (void)cls;
  const char *p = (*env)->GetStringUTFChars(env, path, NULL);
  mbx_db *db = NULL;
  const int rc = p ? mbx_db_open(p, &db) : MBX_E_INVALID;
  if (p) (*env)->ReleaseStringUTFChars(env, path, p);
  check(env, rc, kFileScan);
  return H(db);
}

JNIEXPORT void JNICALL Java_global_Native_dbClose(JNIEnv *env, jclass cls, jlong db) {
  (void)env, (void)cls;
  mbx_db_close(P(mbx_db, db));
}

/* a Columnarfile straight from the DB file (pages -> HBM -> k_page_decode) */
JNIEXPORT jlong JNICALL Java_global_Native_dbStage(JNIEnv *env, jclass cls, jlong ctx, jlong db, jstring name) {
  (void)cls;
  const char *n = (*env)->GetStringUTFChars(env, name, NULL);
  mbx_table *t = NULL;
  const int rc = n ? mbx_db_stage(P(mbx_ctx, ctx), P(mbx_db, db), n, &t) : MBX_E_INVALID;
  if (n) (*env)->ReleaseStringUTFChars(env, name, n);
  check(env, rc, kFileScan);
  return H(t);
}

/* a BitMapFile's page chain -> device BitSet (BitMapFile.getBitSet) */
JNIEXPORT jlong JNICALL Java_global_Native_dbBitmapStage(JNIEnv *env, jclass cls, jlong ctx, jlong db, jstring file,
                                                         jlong nbits) {
  (void)cls;
  const char *n = (*env)->GetStringUTFChars(env, file, NULL);
  mbx_bitmap *b = NULL;
  const int rc = n ? mbx_db_bitmap_stage(P(mbx_ctx, ctx), P(mbx_db, db), n, nbits, &b) : MBX_E_INVALID;
  if (n) (*env)->ReleaseStringUTFChars(env, file, n);
  check(env, rc, kIndex);
  return H(b);
}

/* one shard of a Columnarfile: positions [row_begin, row_end), only its pages read */
JNIEXPORT jlong JNICALL Java_global_Native_dbStageRange(JNIEnv *env, jclass cls, jlong ctx, jlong db, jstring name,
                                                        jlong row_begin, jlong row_end) {
  (void)cls;
  const char *n = (*env)->GetStringUTFChars(env, name, NULL);
  mbx_table *t = NULL;
  const int rc = n ? mbx_db_stage_range(P(mbx_ctx, ctx), P(mbx_db, db), n, row_begin, row_end, &t) : MBX_E_INVALID;
  if (n) (*env)->ReleaseStringUTFChars(env, name, n);
  check(env, rc, kFileScan);
  return H(t);
}

/* a shard's slice of a BitMapFile */
JNIEXPORT jlong JNICALL Java_global_Native_dbBitmapStageRange(JNIEnv *env, jclass cls, jlong ctx, jlong db,
                                                              jstring file, jlong bit_begin, jlong nbits) {
  (void)cls;
  const char *n = (*env)->GetStringUTFChars(env, file, NULL);
  mbx_bitmap *b = NULL;
  const int rc =
      n ? mbx_db_bitmap_stage_range(P(mbx_ctx, ctx), P(mbx_db, db), n, bit_begin, nbits, &b) : MBX_E_INVALID;
  if (n) (*env)->ReleaseStringUTFChars(env, file, n);
  check(env, rc, kIndex);
  return H(b);
}

JNIEXPORT jlong JNICALL Java_global_Native_dbColumnarRows(JNIEnv *env, jclass cls, jlong db, jstring name) {
  (void)cls;
  const char *n = (*env)->GetStringUTFChars(env, name, NULL);
  int64_t nrows = 0;
  const int rc = n ? mbx_db_columnar_info(P(mbx_db, db), n, 0, NULL, NULL, NULL, &nrows, NULL) : MBX_E_INVALID;
  if (n) (*env)->ReleaseStringUTFChars(env, name, n);
  check(env, rc, kFileScan);
  return nrows;
}

JNIEXPORT jlong JNICALL Java_global_Native_tableRowOffset(JNIEnv *env, jclass cls, jlong t) {
  (void)cls;
  int64_t nrows = 0, row_offset = 0;
  int32_t ncols = 0;
  check(env, mbx_table_info(P(mbx_table, t), &nrows, &row_offset, &ncols), kFileScan);
  return row_offset;
}

/* column group: a row-interleaved copy of 2..4 four-byte columns (mbx_table_group) */
JNIEXPORT void JNICALL Java_global_Native_tableGroup(JNIEnv *env, jclass cls, jlong ctx, jlong t, jintArray cols) {
  (void)cls;
  const jsize n = cols ? (*env)->GetArrayLength(env, cols) : 0;
  jint *c = n > 0 ? (*env)->GetIntArrayElements(env, cols, NULL) : NULL;
  const int rc = (n > 0 && !c) ? MBX_E_NOMEM
                               : mbx_table_group(P(mbx_ctx, ctx), P(mbx_table, t), (const int32_t *)c, (int32_t)n);
  if (c) (*env)->ReleaseIntArrayElements(env, cols, c, JNI_ABORT);
  check(env, rc, kFileScan);
}

/* ---- plans and scans ----------------------------------------------------- */

JNIEXPORT jlong JNICALL Java_global_Native_planCompile(JNIEnv *env, jclass cls, jlong ctx, jlong table,
                                                       jobjectArray filter) {
  (void)cls;
  mbx_condexpr conds[MBX_MAX_TERMS];
  int32_t offs[MBX_MAX_CONJ + 1];
  mbx_cnf cnf;
  Strings ss;
  ss.n = 0;
  mbx_plan *p = NULL;
  if (cnf_of(env, filter, conds, offs, &cnf, &ss) == 0)
    check(env, mbx_plan_compile(P(mbx_ctx, ctx), P(mbx_table, table), &cnf, &p), kPredEval);
  strings_release(env, &ss);
  return H(p);
}

JNIEXPORT void JNICALL Java_global_Native_planFree(JNIEnv *env, jclass cls, jlong plan) {
  (void)env, (void)cls;
  mbx_plan_free(P(mbx_plan, plan));
}

/* Query.executeFileScan's resultCount (R/input/Query.java:121-155) */
JNIEXPORT jlong JNICALL Java_global_Native_scanCount(JNIEnv *env, jclass cls, jlong ctx, jlong plan) {
  (void)cls;
  int64_t n = 0;
  check(env, mbx_scan_count(P(mbx_ctx, ctx), P(mbx_plan, plan), &n), kFileScan);
  return n;
}

/* the get_next / get_next_tid selection as a device BitSet */
JNIEXPORT jlong JNICALL Java_global_Native_scanBitmap(JNIEnv *env, jclass cls, jlong ctx, jlong plan) {
  (void)cls;
  mbx_bitmap *b = NULL;
  int64_t n = 0;
  check(env, mbx_scan_bitmap(P(mbx_ctx, ctx), P(mbx_plan, plan), &b, &n), kFileScan);
  return H(b);
}

/* the get_next_tid stream as positions (DeleteQuery; R/iterator/ColumnarFileScan.java:174-188) */
JNIEXPORT jlongArray JNICALL Java_global_Native_scanSelect(JNIEnv *env, jclass cls, jlong ctx, jlong plan, jlong cap) {
  (void)cls;
  /* a Java long[] holds at most Integer.MAX_VALUE - 8 elements: a larger
   * selection raises (mbx_scan_select's capacity check) instead of wrapping */
  const jlong max_java = 0x7ffffff7;
  if (cap > max_java) cap = max_java;
  int64_t *ids = (int64_t *)malloc(sizeof(int64_t) * (size_t)(cap > 0 ? cap : 1));
  if (!ids) {
    throw_chain(env, kChain, "scanSelect: host allocation");
    return NULL;
  }
  int64_t n = 0;
  jlongArray out = NULL;
  if (!check(env, mbx_scan_select(P(mbx_ctx, ctx), P(mbx_plan, plan), ids, cap, &n), kFileScan)) {
    out = (*env)->NewLongArray(env, (jsize)n);
    if (out) (*env)->SetLongArrayRegion(env, out, 0, (jsize)n, (const jlong *)ids);
  }
  free(ids);
  return out;
}

/* mbx_agg -> {count, agg_type, isum, imin, imax, fsum (raw double bits), fmin, fmax (raw float bits)} */
static jlongArray agg_array(JNIEnv *env, const mbx_agg *a) {
  jlong v[8];
  int64_t fs;
  int32_t fmin, fmax;
  memcpy(&fs, &a->fsum, sizeof(fs));
  memcpy(&fmin, &a->fmin, sizeof(fmin));
  memcpy(&fmax, &a->fmax, sizeof(fmax));
  v[0] = a->count, v[1] = a->agg_type, v[2] = a->isum, v[3] = a->imin, v[4] = a->imax;
  v[5] = fs, v[6] = fmin, v[7] = fmax;
  jlongArray out = (*env)->NewLongArray(env, 8);
  if (out) (*env)->SetLongArrayRegion(env, out, 0, 8, v);
  return out;
}

JNIEXPORT jlongArray JNICALL Java_global_Native_scanAggregate(JNIEnv *env, jclass cls, jlong ctx, jlong plan,
                                                              jint col) {
  (void)cls;
  mbx_agg a;
  if (check(env, mbx_scan_aggregate(P(mbx_ctx, ctx), P(mbx_plan, plan), col, &a), kFileScan)) return NULL;
  return agg_array(env, &a);
}

JNIEXPORT void JNICALL Java_global_Native_scanCountAsync(JNIEnv *env, jclass cls, jlong ctx, jlong plan,
                                                         jlong dev_count) {
  (void)cls;
  check(env, mbx_scan_count_async(P(mbx_ctx, ctx), P(mbx_plan, plan), P(int64_t, dev_count)), kFileScan);
}

JNIEXPORT void JNICALL Java_global_Native_scanAggregateAsync(JNIEnv *env, jclass cls, jlong ctx, jlong plan,
                                                             jint col, jlong dev_rec) {
  (void)cls;
  check(env, mbx_scan_aggregate_async(P(mbx_ctx, ctx), P(mbx_plan, plan), col, P(mbx_agg, dev_rec)), kFileScan);
}

/* ---- BitSets (java.util.BitSet images: bit p%64 of word p/64) ----------- */

JNIEXPORT jlong JNICALL Java_global_Native_bitmapUpload(JNIEnv *env, jclass cls, jlong ctx, jlong nbits,
                                                        jlongArray words) {
  (void)cls;
  const int64_t need = (nbits + 63) / 64;
  const jsize have = words ? (*env)->GetArrayLength(env, words) : 0;
  uint64_t *w = (uint64_t *)calloc((size_t)(need > 0 ? need : 1), sizeof(uint64_t));
  if (!w) {
    throw_chain(env, kChain, "bitmapUpload: host allocation");
    return 0;
  }
  if (have > 0) (*env)->GetLongArrayRegion(env, words, 0, (jsize)(have < need ? have : need), (jlong *)w);
  mbx_bitmap *b = NULL;
  check(env, mbx_bitmap_upload(P(mbx_ctx, ctx), nbits, w, &b), kIndex);
  free(w);
  return H(b);
}

/* BitSet.valueOf(Native.bitmapDownload(...)) */
JNIEXPORT jlongArray JNICALL Java_global_Native_bitmapDownload(JNIEnv *env, jclass cls, jlong ctx, jlong bm) {
  (void)cls;
  int64_t nbits = 0, nwords = 0, count = 0;
  if (check(env, mbx_bitmap_info(P(mbx_bitmap, bm), &nbits, &nwords, &count), kIndex)) return NULL;
  jlongArray out = (*env)->NewLongArray(env, (jsize)nwords);
  if (!out || nwords == 0) return out;
  jlong *w = (*env)->GetLongArrayElements(env, out, NULL);
  const int rc = mbx_bitmap_download(P(mbx_ctx, ctx), P(mbx_bitmap, bm), (uint64_t *)w, nwords);
  (*env)->ReleaseLongArrayElements(env, out, w, 0);
  check(env, rc, kIndex);
  return out;
}

/* BitSet.cardinality() (-1 after an async producer until something counts it) */
JNIEXPORT jlong JNICALL Java_global_Native_bitmapCardinality(JNIEnv *env, jclass cls, jlong bm) {
  (void)cls;
  int64_t nbits = 0, nwords = 0, count = -1;
  check(env, mbx_bitmap_info(P(mbx_bitmap, bm), &nbits, &nwords, &count), kIndex);
  return count;
}

/* ColumnarIndexScan's OR/AND over index BitSets (R/index/ColumnarIndexScan.java:130-181)
 * and ColumnIndexScan.getBitSet's value-set OR (R/index/ColumnIndexScan.java:656-740),
 * AND NOT deleted (0 = none), in one pass */
JNIEXPORT jlong JNICALL Java_global_Native_bitmapCnf(JNIEnv *env, jclass cls, jlong ctx, jlong nbits, jlongArray bms,
                                                     jintArray conj_offsets, jlong deleted) {
  (void)cls;
  const jsize nb = (*env)->GetArrayLength(env, bms);
  const jsize no = (*env)->GetArrayLength(env, conj_offsets);
  if (no < 1) {
    throw_chain(env, kIndex, "bitmapCnf: conj_offsets needs nconj + 1 entries");
    return 0;
  }
  const mbx_bitmap **v = (const mbx_bitmap **)calloc((size_t)(nb > 0 ? nb : 1), sizeof(void *));
  jlong *h = nb > 0 ? (*env)->GetLongArrayElements(env, bms, NULL) : NULL;
  jint *o = (*env)->GetIntArrayElements(env, conj_offsets, NULL);
  mbx_bitmap *out = NULL;
  int64_t count = 0;
  if (v && o && (nb == 0 || h)) {
    for (jsize i = 0; i < nb; i++) v[i] = P(const mbx_bitmap, h[i]);
    check(env, mbx_bitmap_cnf(P(mbx_ctx, ctx), nbits, v, (const int32_t *)o, (int32_t)(no - 1),
                              P(const mbx_bitmap, deleted), &out, &count),
          kIndex);
  } else {
    throw_chain(env, kChain, "bitmapCnf: host allocation");
  }
  if (h) (*env)->ReleaseLongArrayElements(env, bms, h, JNI_ABORT);
  if (o) (*env)->ReleaseIntArrayElements(env, conj_offsets, o, JNI_ABORT);
  free(v);
  return H(out);
}

/* ColumnarIndexScan in one launch: the CNF of index BitSets + positions (devIds 0: none) + the projected
 * columns' rows into device slots (devAlloc); waits, returns the selected row count */
JNIEXPORT jlong JNICALL Java_global_Native_cnfMaterialize(JNIEnv *env, jclass cls, jlong ctx, jlong table,
                                                          jlongArray bms, jintArray conj_offsets, jlong deleted,
                                                          jintArray proj, jlong dev_ids, jlongArray dev_out,
                                                          jlong dev_count) {
  (void)cls;
  const jsize nb = (*env)->GetArrayLength(env, bms);
  const jsize no = (*env)->GetArrayLength(env, conj_offsets);
  const jsize np = (*env)->GetArrayLength(env, proj);
  if (no < 1 || (*env)->GetArrayLength(env, dev_out) != np) {
    throw_chain(env, kIndex, "cnfMaterialize: conj_offsets needs nconj + 1 entries, devOut one per column");
    return 0;
  }
  const mbx_bitmap **v = (const mbx_bitmap **)calloc((size_t)(nb > 0 ? nb : 1), sizeof(void *));
  void **outs = (void **)calloc((size_t)(np > 0 ? np : 1), sizeof(void *));
  jlong *h = nb > 0 ? (*env)->GetLongArrayElements(env, bms, NULL) : NULL;
  jint *o = (*env)->GetIntArrayElements(env, conj_offsets, NULL);
  jint *pj = np > 0 ? (*env)->GetIntArrayElements(env, proj, NULL) : NULL;
  jlong *d = np > 0 ? (*env)->GetLongArrayElements(env, dev_out, NULL) : NULL;
  int64_t count = 0;
  if (v && outs && o && (nb == 0 || h) && (np == 0 || (pj && d))) {
    for (jsize i = 0; i < nb; i++) v[i] = P(const mbx_bitmap, h[i]);
    for (jsize j = 0; j < np; j++) outs[j] = P(void, d[j]);
    /* the download waits for this launch on the context stream; it does not
     * consume the sticky NaN word an earlier async scan may have left (that
     * one is raised by the next Native.sync, where it belongs) */
    if (!check(env, mbx_cnf_materialize_async(P(mbx_ctx, ctx), P(const mbx_table, table), v, (const int32_t *)o,
                                              (int32_t)(no - 1), P(const mbx_bitmap, deleted),
                                              (const int32_t *)pj, (int32_t)np, P(int64_t, dev_ids), outs,
                                              P(int64_t, dev_count)),
               kIndex))
      check(env, mbx_dev_download(P(mbx_ctx, ctx), P(void, dev_count), &count, sizeof(count)), kChain);
  } else {
    throw_chain(env, kChain, "cnfMaterialize: host allocation");
  }
  if (h) (*env)->ReleaseLongArrayElements(env, bms, h, JNI_ABORT);
  if (o) (*env)->ReleaseIntArrayElements(env, conj_offsets, o, JNI_ABORT);
  if (pj) (*env)->ReleaseIntArrayElements(env, proj, pj, JNI_ABORT);
  if (d) (*env)->ReleaseLongArrayElements(env, dev_out, d, JNI_ABORT);
  free(v);
  free(outs);
  return count;
}

/* BitSet.and / or / andNot (MBX_BM_AND / _OR / _ANDNOT) */
JNIEXPORT jlong JNICALL Java_global_Native_bitmapCombine(JNIEnv *env, jclass cls, jlong ctx, jint op, jlong a,
                                                         jlong b) {
  (void)cls;
  mbx_bitmap *out = NULL;
  int64_t count = 0;
  check(env, mbx_bitmap_combine(P(mbx_ctx, ctx), op, P(mbx_bitmap, a), P(mbx_bitmap, b), &out, &count), kIndex);
  return H(out);
}

JNIEXPORT void JNICALL Java_global_Native_bitmapFree(JNIEnv *env, jclass cls, jlong bm) {
  (void)env, (void)cls;
  mbx_bitmap_free(P(mbx_bitmap, bm));
}

/* ---- cursors: Iterator.get_next batches (R/iterator/Iterator.java:12-141) - */

JNIEXPORT jlong JNICALL Java_global_Native_cursorOpen(JNIEnv *env, jclass cls, jlong ctx, jlong table, jlong sel,
                                                      jintArray proj) {
  (void)cls;
  const jsize np = proj ? (*env)->GetArrayLength(env, proj) : 0;
  jint *pj = np > 0 ? (*env)->GetIntArrayElements(env, proj, NULL) : NULL;
  mbx_cursor *c = NULL;
  check(env, mbx_cursor_open(P(mbx_ctx, ctx), P(mbx_table, table), P(mbx_bitmap, sel), (const int32_t *)pj,
                             (int32_t)np, &c),
        kFileScan);
  if (pj) (*env)->ReleaseIntArrayElements(env, proj, pj, JNI_ABORT);
  return H(c);
}

/* bitmap handles + conjunct offsets of a CNF, borrowed for one call */
typedef struct {
  const mbx_bitmap **v;
  jlong *h;
  jint *o;
  jint *pj;
  jsize nb, no, np;
} CnfArgs;

static int cnf_args_get(JNIEnv *env, jlongArray bms, jintArray conj_offsets, jintArray proj, CnfArgs *a) {
  memset(a, 0, sizeof(*a));
  a->nb = (*env)->GetArrayLength(env, bms);
  a->no = (*env)->GetArrayLength(env, conj_offsets);
  a->np = proj ? (*env)->GetArrayLength(env, proj) : 0;
  if (a->no < 1) {
    throw_chain(env, kIndex, "CNF: conj_offsets needs nconj + 1 entries");
    return -1;
  }
  a->v = (const mbx_bitmap **)calloc((size_t)(a->nb > 0 ? a->nb : 1), sizeof(void *));
  a->h = a->nb > 0 ? (*env)->GetLongArrayElements(env, bms, NULL) : NULL;
  a->o = (*env)->GetIntArrayElements(env, conj_offsets, NULL);
  a->pj = a->np > 0 ? (*env)->GetIntArrayElements(env, proj, NULL) : NULL;
  if (!a->v || !a->o || (a->nb > 0 && !a->h) || (a->np > 0 && !a->pj)) {
    throw_chain(env, kChain, "CNF: host allocation");
    return -1;
  }
  for (jsize i = 0; i < a->nb; i++) a->v[i] = P(const mbx_bitmap, a->h[i]);
  return 0;
}

static void cnf_args_release(JNIEnv *env, jlongArray bms, jintArray conj_offsets, jintArray proj, CnfArgs *a) {
  if (a->h) (*env)->ReleaseLongArrayElements(env, bms, a->h, JNI_ABORT);
  if (a->o) (*env)->ReleaseIntArrayElements(env, conj_offsets, a->o, JNI_ABORT);
  if (a->pj) (*env)->ReleaseIntArrayElements(env, proj, a->pj, JNI_ABORT);
  free(a->v);
}

/* ColumnarIndexScan (R/index/ColumnarIndexScan.java:79-182, get_next :287-308) in one launch, as a cursor */
JNIEXPORT jlong JNICALL Java_global_Native_cnfCursorOpen(JNIEnv *env, jclass cls, jlong ctx, jlong table,
                                                         jlongArray bms, jintArray conj_offsets, jlong deleted,
                                                         jintArray proj) {
  (void)cls;
  CnfArgs a;
  mbx_cursor *c = NULL;
  if (cnf_args_get(env, bms, conj_offsets, proj, &a) == 0)
    check(env,
          mbx_cnf_cursor_open(P(mbx_ctx, ctx), P(const mbx_table, table), a.v, (const int32_t *)a.o,
                              (int32_t)(a.no - 1), P(const mbx_bitmap, deleted), (const int32_t *)a.pj,
                              (int32_t)a.np, &c),
          kIndex);
  cnf_args_release(env, bms, conj_offsets, proj, &a);
  return H(c);
}

/* launch only: {cursor, device pointer of its count} (the count feeds the shards' exchange) */
JNIEXPORT jlongArray JNICALL Java_global_Native_cnfCursorLaunch(JNIEnv *env, jclass cls, jlong ctx, jlong table,
                                                               jlongArray bms, jintArray conj_offsets, jlong deleted,
                                                               jintArray proj) {
  (void)cls;
  CnfArgs a;
  mbx_cursor *c = NULL;
  int64_t *dcount = NULL;
  jlongArray out = NULL;
  if (cnf_args_get(env, bms, conj_offsets, proj, &a) == 0 &&
      !check(env,
             mbx_cnf_cursor_launch(P(mbx_ctx, ctx), P(const mbx_table, table), a.v, (const int32_t *)a.o,
                                   (int32_t)(a.no - 1), P(const mbx_bitmap, deleted), (const int32_t *)a.pj,
                                   (int32_t)a.np, &c, &dcount),
             kIndex)) {
    jlong v[2] = {H(c), H(dcount)};
    out = (*env)->NewLongArray(env, 2);
    if (out) (*env)->SetLongArrayRegion(env, out, 0, 2, v);
    else mbx_cursor_close(c);
  }
  cnf_args_release(env, bms, conj_offsets, proj, &a);
  return out;
}

JNIEXPORT jlong JNICALL Java_global_Native_cursorCount(JNIEnv *env, jclass cls, jlong cur) {
  (void)cls;
  int64_t n = 0;
  check(env, mbx_cursor_count(P(mbx_cursor, cur), &n), kFileScan);
  return n;
}

/* n values of one projected column in the mbx_materialize host layout ->
 * int[] / float[] / String[] (char(n): zero-padded modified UTF-8,
 * NUL-terminated for NewStringUTF) */
static jobject column_array(JNIEnv *env, jint type, jshort size, const void *buf, int64_t n, jclass strc) {
  jobject col = NULL;
  if (type == MBX_ATTR_INTEGER) {
    col = (*env)->NewIntArray(env, (jsize)n);
    if (col) (*env)->SetIntArrayRegion(env, (jintArray)col, 0, (jsize)n, (const jint *)buf);
  } else if (type == MBX_ATTR_REAL) {
    col = (*env)->NewFloatArray(env, (jsize)n);
    if (col) (*env)->SetFloatArrayRegion(env, (jfloatArray)col, 0, (jsize)n, (const jfloat *)buf);
  } else {
    jobjectArray sa = (*env)->NewObjectArray(env, (jsize)n, strc, NULL);
    char *tmp = (char *)malloc((size_t)size + 1);
    for (int64_t r = 0; sa && tmp && r < n; r++) {
      memcpy(tmp, (const char *)buf + r * size, (size_t)size);
      tmp[size] = 0;
      jstring js = (*env)->NewStringUTF(env, tmp);
      if (!js) break; /* OutOfMemoryError pending */
      (*env)->SetObjectArrayElement(env, sa, (jsize)r, js);
      (*env)->DeleteLocalRef(env, js);
    }
    const int have_tmp = tmp != NULL; /* read before free: a freed pointer's value is indeterminate */
    free(tmp);
    col = sa && have_tmp && !(*env)->ExceptionCheck(env) ? sa : NULL;
    if (sa && sa != col) (*env)->DeleteLocalRef(env, sa);
    if (!col && !(*env)->ExceptionCheck(env)) throw_chain(env, kChain, "cursor rows: host allocation");
  }
  return col;
}

/* The next <= max_rows rows: {long[] positions, Object[] columns}, a column
 * per projected field as int[] / float[] / String[] (types / sizes: the
 * projected columns' AttrType and char(n) size); null at the end of the
 * stream (get_next() returning null).  The batch is read in place from the
 * cursor's pinned buffer (mbx_cursor_next_view): one copy into the Java
 * arrays, none in between. */
JNIEXPORT jobjectArray JNICALL Java_global_Native_cursorNext(JNIEnv *env, jclass cls, jlong cur, jint max_rows,
                                                            jintArray types, jshortArray sizes) {
  (void)cls;
  const jsize np = types ? (*env)->GetArrayLength(env, types) : 0;
  if (max_rows <= 0 || (sizes && (*env)->GetArrayLength(env, sizes) != np)) {
    throw_chain(env, kFileScan, "cursorNext: bad arguments");
    return NULL;
  }
  jint *t = np > 0 ? (*env)->GetIntArrayElements(env, types, NULL) : NULL;
  jshort *s = np > 0 ? (*env)->GetShortArrayElements(env, sizes, NULL) : NULL;
  const void **bufs = (const void **)calloc((size_t)(np > 0 ? np : 1), sizeof(void *));
  const int64_t *ids = NULL;
  jobjectArray res = NULL;
  int64_t n = 0;
  if (!bufs || (np > 0 && (!t || !s))) {
    throw_chain(env, kChain, "cursorNext: host allocation");
  } else if (!check(env, mbx_cursor_next_view(P(mbx_cursor, cur), max_rows, &ids, bufs, &n), kFileScan) && n > 0) {
    jclass objc = (*env)->FindClass(env, "java/lang/Object");
    jclass strc = objc ? (*env)->FindClass(env, "java/lang/String") : NULL;
    jobjectArray cols = strc ? (*env)->NewObjectArray(env, np, objc, NULL) : NULL;
    jlongArray jids = cols ? (*env)->NewLongArray(env, (jsize)n) : NULL;
    if (jids) (*env)->SetLongArrayRegion(env, jids, 0, (jsize)n, (const jlong *)ids);
    for (jsize j = 0; jids && j < np; j++) {
      jobject col = column_array(env, t[j], s[j], bufs[j], n, strc);
      if (!col) break;
      (*env)->SetObjectArrayElement(env, cols, j, col);
      (*env)->DeleteLocalRef(env, col);
    }
    if (jids && !(*env)->ExceptionCheck(env)) {
      res = (*env)->NewObjectArray(env, 2, objc, NULL);
      if (res) {
        (*env)->SetObjectArrayElement(env, res, 0, jids);
        (*env)->SetObjectArrayElement(env, res, 1, cols);
      }
    }
  }
  free(bufs);
  if (t) (*env)->ReleaseIntArrayElements(env, types, t, JNI_ABORT);
  if (s) (*env)->ReleaseShortArrayElements(env, sizes, s, JNI_ABORT);
  return res;
}

JNIEXPORT void JNICALL Java_global_Native_cursorRestart(JNIEnv *env, jclass cls, jlong cur) {
  (void)cls;
  check(env, mbx_cursor_restart(P(mbx_cursor, cur)), kFileScan);
}

JNIEXPORT void JNICALL Java_global_Native_cursorClose(JNIEnv *env, jclass cls, jlong cur) {
  (void)env, (void)cls;
  mbx_cursor_close(P(mbx_cursor, cur));
}

/* ---- device result slots + multi-GPU (one JVM drives every GPU) --------- */

JNIEXPORT jlong JNICALL Java_global_Native_devAlloc(JNIEnv *env, jclass cls, jlong ctx, jlong bytes) {
  (void)cls;
  void *d = NULL;
  check(env, mbx_dev_alloc(P(mbx_ctx, ctx), bytes, &d), kChain);
  return H(d);
}

JNIEXPORT void JNICALL Java_global_Native_devFree(JNIEnv *env, jclass cls, jlong ctx, jlong dev) {
  (void)env, (void)cls;
  mbx_dev_free(P(mbx_ctx, ctx), P(void, dev));
}

JNIEXPORT jlong JNICALL Java_global_Native_countDownload(JNIEnv *env, jclass cls, jlong ctx, jlong dev_count) {
  (void)cls;
  int64_t v = 0;
  check(env, mbx_dev_download(P(mbx_ctx, ctx), P(void, dev_count), &v, sizeof(v)), kChain);
  return v;
}

JNIEXPORT jlongArray JNICALL Java_global_Native_aggDownload(JNIEnv *env, jclass cls, jlong ctx, jlong dev_rec) {
  (void)cls;
  mbx_agg a;
  if (check(env, mbx_dev_download(P(mbx_ctx, ctx), P(void, dev_rec), &a, sizeof(a)), kChain)) return NULL;
  return agg_array(env, &a);
}

JNIEXPORT jlongArray JNICALL Java_global_Native_shardBounds(JNIEnv *env, jclass cls, jlong nrows, jint nshards,
                                                            jint shard) {
  (void)cls;
  int64_t b = 0, e = 0;
  if (check(env, mbx_shard_bounds(nrows, nshards, shard, &b, &e), kFileScan)) return NULL;
  jlong v[2] = {b, e};
  jlongArray out = (*env)->NewLongArray(env, 2);
  if (out) (*env)->SetLongArrayRegion(env, out, 0, 2, v);
  return out;
}

JNIEXPORT jbyteArray JNICALL Java_global_Native_commUniqueId(JNIEnv *env, jclass cls) {
  (void)cls;
  jbyte id[MBX_COMM_ID_BYTES];
  if (check(env, mbx_comm_unique_id(id), kChain)) return NULL;
  jbyteArray out = (*env)->NewByteArray(env, MBX_COMM_ID_BYTES);
  if (out) (*env)->SetByteArrayRegion(env, out, 0, MBX_COMM_ID_BYTES, id);
  return out;
}

/* one process per GPU: the id travels through the launcher (any byte channel) */
JNIEXPORT jlong JNICALL Java_global_Native_commInitRank(JNIEnv *env, jclass cls, jlong ctx, jint nranks, jint rank,
                                                        jbyteArray id) {
  (void)cls;
  jbyte raw[MBX_COMM_ID_BYTES];
  if (!id || (*env)->GetArrayLength(env, id) != MBX_COMM_ID_BYTES) {
    throw_chain(env, kChain, "commInitRank: id must be MBX_COMM_ID_BYTES bytes");
    return 0;
  }
  (*env)->GetByteArrayRegion(env, id, 0, MBX_COMM_ID_BYTES, raw);
  mbx_comm *c = NULL;
  check(env, mbx_comm_init_rank(P(mbx_ctx, ctx), nranks, rank, raw, &c), kChain);
  return H(c);
}

/* one JVM, every GPU: ctxs[i] becomes rank i of one RCCL clique */
JNIEXPORT jlongArray JNICALL Java_global_Native_commInitAll(JNIEnv *env, jclass cls, jlongArray ctxs) {
  (void)cls;
  const jsize n = (*env)->GetArrayLength(env, ctxs);
  mbx_ctx **cv = (mbx_ctx **)calloc((size_t)(n > 0 ? n : 1), sizeof(void *));
  mbx_comm **out = (mbx_comm **)calloc((size_t)(n > 0 ? n : 1), sizeof(void *));
  jlong *h = n > 0 ? (*env)->GetLongArrayElements(env, ctxs, NULL) : NULL;
  jlongArray res = NULL;
  if (cv && out && h) {
    for (jsize i = 0; i < n; i++) cv[i] = P(mbx_ctx, h[i]);
    if (!check(env, mbx_comm_init_all(cv, (int32_t)n, out), kChain)) {
      res = (*env)->NewLongArray(env, n);
      for (jsize i = 0; res && i < n; i++) {
        const jlong v = H(out[i]);
        (*env)->SetLongArrayRegion(env, res, i, 1, &v);
      }
    }
  } else {
    throw_chain(env, kChain, "commInitAll: bad arguments");
  }
  if (h) (*env)->ReleaseLongArrayElements(env, ctxs, h, JNI_ABORT);
  free(cv);
  free(out);
  return res;
}

JNIEXPORT void JNICALL Java_global_Native_commFree(JNIEnv *env, jclass cls, jlong comm) {
  (void)env, (void)cls;
  mbx_comm_free(P(mbx_comm, comm));
}

JNIEXPORT void JNICALL Java_global_Native_commAllreduceCount(JNIEnv *env, jclass cls, jlong comm, jlong dev_count) {
  (void)cls;
  check(env, mbx_comm_allreduce_count_async(P(mbx_comm, comm), P(int64_t, dev_count), 1), kChain);
}

JNIEXPORT void JNICALL Java_global_Native_commAllreduceAgg(JNIEnv *env, jclass cls, jlong comm, jlong dev_rec) {
  (void)cls;
  check(env, mbx_comm_allreduce_agg_async(P(mbx_comm, comm), P(mbx_agg, dev_rec)), kChain);
}

/* ptrs[i]: a device pointer on comms[i]'s GPU (devAlloc) */
static int ptrs_of(JNIEnv *env, jlongArray comms, jlongArray ptrs, mbx_comm ***cv, void ***pv, jsize *n) {
  *n = (*env)->GetArrayLength(env, comms);
  if (*n <= 0 || (*env)->GetArrayLength(env, ptrs) != *n) return -1;
  *cv = (mbx_comm **)calloc((size_t)*n, sizeof(void *));
  *pv = (void **)calloc((size_t)*n, sizeof(void *));
  jlong *c = (*env)->GetLongArrayElements(env, comms, NULL);
  jlong *p = (*env)->GetLongArrayElements(env, ptrs, NULL);
  const int ok = *cv && *pv && c && p;
  for (jsize i = 0; ok && i < *n; i++) {
    (*cv)[i] = P(mbx_comm, c[i]);
    (*pv)[i] = P(void, p[i]);
  }
  if (c) (*env)->ReleaseLongArrayElements(env, comms, c, JNI_ABORT);
  if (p) (*env)->ReleaseLongArrayElements(env, ptrs, p, JNI_ABORT);
  return ok ? 0 : -1;
}

JNIEXPORT void JNICALL Java_global_Native_commAllreduceCountAll(JNIEnv *env, jclass cls, jlongArray comms,
                                                                jlongArray dev_counts) {
  (void)cls;
  mbx_comm **cv = NULL;
  void **pv = NULL;
  jsize n = 0;
  if (ptrs_of(env, comms, dev_counts, &cv, &pv, &n))
    throw_chain(env, kChain, "commAllreduceCountAll: one device count per communicator");
  else
    check(env, mbx_comm_allreduce_count_all(cv, (int32_t)n, (int64_t *const *)pv, 1), kChain);
  free(cv);
  free(pv);
}

JNIEXPORT void JNICALL Java_global_Native_commAllreduceAggAll(JNIEnv *env, jclass cls, jlongArray comms,
                                                              jlongArray dev_recs) {
  (void)cls;
  mbx_comm **cv = NULL;
  void **pv = NULL;
  jsize n = 0;
  if (ptrs_of(env, comms, dev_recs, &cv, &pv, &n))
    throw_chain(env, kChain, "commAllreduceAggAll: one device record per communicator");
  else
    check(env, mbx_comm_allreduce_agg_all(cv, (int32_t)n, (mbx_agg *const *)pv), kChain);
  free(cv);
  free(pv);
}

JNIEXPORT void JNICALL Java_global_Native_commAllgatherCountAll(JNIEnv *env, jclass cls, jlongArray comms,
                                                                jlongArray dev_counts, jlongArray dev_alls) {
  (void)cls;
  mbx_comm **cv = NULL, **cv2 = NULL;
  void **pv = NULL, **av = NULL;
  jsize n = 0, n2 = 0;
  if (ptrs_of(env, comms, dev_counts, &cv, &pv, &n) || ptrs_of(env, comms, dev_alls, &cv2, &av, &n2))
    throw_chain(env, kChain, "commAllgatherCountAll: one device count and one result slot per communicator");
  else
    check(env, mbx_comm_allgather_count_all(cv, (int32_t)n, (const int64_t *const *)pv, (int64_t *const *)av),
          kChain);
  free(cv);
  free(pv);
  free(cv2);
  free(av);
}

/* the context stream waits (on the device) for the collectives enqueued so far */
JNIEXPORT void JNICALL Java_global_Native_commWait(JNIEnv *env, jclass cls, jlong comm) {
  (void)cls;
  check(env, mbx_comm_wait(P(mbx_comm, comm)), kChain);
}

JNIEXPORT jlongArray JNICALL Java_global_Native_longsDownload(JNIEnv *env, jclass cls, jlong ctx, jlong dev, jint n) {
  (void)cls;
  if (n < 0) {
    throw_chain(env, kChain, "longsDownload: n < 0");
    return NULL;
  }
  jlong *v = (jlong *)calloc((size_t)(n > 0 ? n : 1), sizeof(jlong));
  jlongArray out = NULL;
  if (!v) {
    throw_chain(env, kChain, "longsDownload: host allocation");
    return NULL;
  }
  if (!check(env, mbx_dev_download(P(mbx_ctx, ctx), P(void, dev), v, (int64_t)n * (int64_t)sizeof(jlong)), kChain)) {
    out = (*env)->NewLongArray(env, n);
    if (out) (*env)->SetLongArrayRegion(env, out, 0, n, v);
  }
  free(v);
  return out;
}

/* ---- joins (include/mbx_join.h): ColumnarNestedLoopJoins / BitMapQuery pairs -- */

JNIEXPORT jlong JNICALL Java_global_Native_join(JNIEnv *env, jclass cls, jlong ctx, jlong outer, jlong outer_sel,
                                                jlong inner, jlong inner_sel, jintArray terms, jintArray conj_offsets,
                                                jint order, jlong outer_block) {
  (void)cls;
  const jsize nt3 = (*env)->GetArrayLength(env, terms);
  const jsize no = (*env)->GetArrayLength(env, conj_offsets);
  if (nt3 % 3 != 0 || no < 1 || nt3 / 3 > MBX_MAX_JOIN_TERMS) {
    throw_chain(env, kChain, "join: terms are {op, outerCol, innerCol} triples, conj_offsets nconj + 1 entries");
    return 0;
  }
  mbx_join_term jt[MBX_MAX_JOIN_TERMS];
  jint *t = nt3 > 0 ? (*env)->GetIntArrayElements(env, terms, NULL) : NULL;
  jint *o = (*env)->GetIntArrayElements(env, conj_offsets, NULL);
  mbx_join_result *r = NULL;
  if ((nt3 > 0 && !t) || !o) {
    throw_chain(env, kChain, "join: host allocation");
  } else {
    for (jsize k = 0; k < nt3 / 3; k++) {
      jt[k].op = t[3 * k];
      jt[k].outer_col = t[3 * k + 1];
      jt[k].inner_col = t[3 * k + 2];
      jt[k].pad_ = 0;
    }
    mbx_join_cnf cnf;
    cnf.terms = jt;
    cnf.conj_offsets = (const int32_t *)o;
    cnf.nconj = (int32_t)(no - 1);
    check(env,
          mbx_join(P(mbx_ctx, ctx), P(const mbx_table, outer), P(const mbx_bitmap, outer_sel),
                   P(const mbx_table, inner), P(const mbx_bitmap, inner_sel), &cnf, order, outer_block, &r),
          kChain);
  }
  if (t) (*env)->ReleaseIntArrayElements(env, terms, t, JNI_ABORT);
  if (o) (*env)->ReleaseIntArrayElements(env, conj_offsets, o, JNI_ABORT);
  return H(r);
}

JNIEXPORT jlongArray JNICALL Java_global_Native_joinInfo(JNIEnv *env, jclass cls, jlong res) {
  (void)cls;
  int64_t count = 0, passes = 0;
  if (check(env, mbx_join_info(P(const mbx_join_result, res), &count, &passes), kChain)) return NULL;
  jlong v[2] = {count, passes};
  jlongArray out = (*env)->NewLongArray(env, 2);
  if (out) (*env)->SetLongArrayRegion(env, out, 0, 2, v);
  return out;
}

/* pairs [start, start + n): {long[] outer positions, long[] inner positions, int[] pass} */
JNIEXPORT jobjectArray JNICALL Java_global_Native_joinFetch(JNIEnv *env, jclass cls, jlong ctx, jlong res, jlong start,
                                                            jint n) {
  (void)cls;
  if (n < 0 || start < 0) {
    throw_chain(env, kChain, "joinFetch: bad range");
    return NULL;
  }
  int64_t *op = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  int64_t *ip = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  int32_t *ps = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
  jobjectArray out = NULL;
  if (!op || !ip || !ps) {
    throw_chain(env, kChain, "joinFetch: host allocation");
  } else if (!check(env, mbx_join_fetch(P(mbx_ctx, ctx), P(const mbx_join_result, res), start, n, op, ip, ps),
                    kChain)) {
    jclass objc = (*env)->FindClass(env, "java/lang/Object");
    jlongArray jo = (*env)->NewLongArray(env, n);
    jlongArray ji = (*env)->NewLongArray(env, n);
    jintArray jp = (*env)->NewIntArray(env, n);
    if (jo) (*env)->SetLongArrayRegion(env, jo, 0, n, (const jlong *)op);
    if (ji) (*env)->SetLongArrayRegion(env, ji, 0, n, (const jlong *)ip);
    if (jp) (*env)->SetIntArrayRegion(env, jp, 0, n, (const jint *)ps);
    out = objc ? (*env)->NewObjectArray(env, 3, objc, NULL) : NULL;
    if (out) {
      (*env)->SetObjectArrayElement(env, out, 0, jo);
      (*env)->SetObjectArrayElement(env, out, 1, ji);
      (*env)->SetObjectArrayElement(env, out, 2, jp);
    }
  }
  free(op);
  free(ip);
  free(ps);
  return out;
}

JNIEXPORT void JNICALL Java_global_Native_joinFree(JNIEnv *env, jclass cls, jlong res) {
  (void)env, (void)cls;
  mbx_join_free(P(mbx_join_result, res));
}

/* late materialisation by explicit positions (Heapfile.findRID + getRecord per value) */
JNIEXPORT jobjectArray JNICALL Java_global_Native_gather(JNIEnv *env, jclass cls, jlong ctx, jlong table,
                                                         jlongArray positions, jintArray proj, jintArray types,
                                                         jshortArray sizes) {
  (void)cls;
  const jsize n = (*env)->GetArrayLength(env, positions);
  const jsize np = (*env)->GetArrayLength(env, proj);
  if ((*env)->GetArrayLength(env, types) != np || (*env)->GetArrayLength(env, sizes) != np) {
    throw_chain(env, kChain, "gather: proj / types / sizes disagree");
    return NULL;
  }
  jlong *pos = n > 0 ? (*env)->GetLongArrayElements(env, positions, NULL) : NULL;
  jint *pj = np > 0 ? (*env)->GetIntArrayElements(env, proj, NULL) : NULL;
  jint *t = np > 0 ? (*env)->GetIntArrayElements(env, types, NULL) : NULL;
  jshort *s = np > 0 ? (*env)->GetShortArrayElements(env, sizes, NULL) : NULL;
  void **bufs = (void **)calloc((size_t)(np > 0 ? np : 1), sizeof(void *));
  int bad = !bufs || (n > 0 && !pos) || (np > 0 && (!pj || !t || !s));
  for (jsize j = 0; !bad && j < np; j++) {
    bufs[j] = malloc((t[j] == MBX_ATTR_STRING ? (size_t)s[j] : 4) * (size_t)(n > 0 ? n : 1));
    bad = !bufs[j];
  }
  jobjectArray out = NULL;
  if (bad) {
    throw_chain(env, kChain, "gather: host allocation");
  } else if (!check(env, mbx_gather(P(mbx_ctx, ctx), P(const mbx_table, table), (const int64_t *)pos, n,
                                    (const int32_t *)pj, (int32_t)np, bufs),
                    kFileScan)) {
    jclass objc = (*env)->FindClass(env, "java/lang/Object");
    jclass strc = (*env)->FindClass(env, "java/lang/String");
    out = objc ? (*env)->NewObjectArray(env, np, objc, NULL) : NULL;
    for (jsize j = 0; out && j < np; j++) {
      jobject col = column_array(env, t[j], s[j], bufs[j], n, strc);
      if (!col) {
        out = NULL;
        break;
      }
      (*env)->SetObjectArrayElement(env, out, j, col);
      (*env)->DeleteLocalRef(env, col);
    }
  }
  for (jsize j = 0; bufs && j < np; j++) free(bufs[j]);
  free(bufs);
  if (pos) (*env)->ReleaseLongArrayElements(env, positions, pos, JNI_ABORT);
  if (pj) (*env)->ReleaseIntArrayElements(env, proj, pj, JNI_ABORT);
  if (t) (*env)->ReleaseIntArrayElements(env, types, t, JNI_ABORT);
  if (s) (*env)->ReleaseShortArrayElements(env, sizes, s, JNI_ABORT);
  return out;
}
