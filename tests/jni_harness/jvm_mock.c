/*
 * jvm_mock.c -- a minimal JVM stand-in that lets jni/mbx_jni.c run for real
 * with no JDK (test infrastructure only: tests/test_jni_harness.py).
 *
 * It implements exactly the JNIEnv function table of jni/jni_min/jni.h over
 * a small object model:
 *   - classes are known by name; the reference classes the glue reads are
 *     declared with their public fields and JNI signatures as the reference
 *     lays them out (R/iterator/CondExpr.java:12-41, R/iterator/Operand.java:5-9,
 *     R/iterator/FldSpec.java:4-6, R/iterator/RelSpec.java:3-4,
 *     R/global/AttrType.java:16, R/global/AttrOperator.java:20,
 *     R/global/IndexType.java:15); GetFieldID of anything else fails with a
 *     pending NoSuchFieldError, FindClass of an unknown class with
 *     NoClassDefFoundError, as a JVM would;
 *   - the reference's exception classes (ChainException and the subclasses
 *     the glue throws) have the (Exception, String) constructor of
 *     R/chainexception/ChainException.java:20;
 *   - strings hold modified UTF-8 (NewStringUTF validates it);
 *   - primitive arrays, object arrays and direct ByteBuffers.
 * Borrowed elements (Get<T>ArrayElements, GetStringUTFChars) are copies that
 * must be released; the harness counts what is outstanding.  Calls the JNI
 * specification forbids while an exception is pending, element-type
 * mismatches and out-of-range regions are recorded as violations (what
 * -Xcheck:jni reports).  The jh_* functions build objects for the test and
 * inspect results.
 */
#include <jni.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { K_PLAIN = 1, K_CLASS, K_STRING, K_ARRAY, K_BUFFER };
#define MAGIC 0x4a564d4f
#define MAXF 8

typedef struct {
  const char *name, *sig;
} FieldDecl;

typedef struct {
  const char *name;
  FieldDecl fields[MAXF];
  int is_exception;
} ClassDecl;

static const ClassDecl kClasses[] = {
    {"iterator/CondExpr",
     {{"op", "Lglobal/AttrOperator;"},
      {"type1", "Lglobal/AttrType;"},
      {"type2", "Lglobal/AttrType;"},
      {"operand1", "Literator/Operand;"},
      {"operand2", "Literator/Operand;"},
      {"indexType", "Lglobal/IndexType;"},
      {"next", "Literator/CondExpr;"}},
     0},
    {"iterator/Operand", {{"symbol", "Literator/FldSpec;"}, {"string", "Ljava/lang/String;"}, {"integer", "I"}, {"real", "F"}}, 0},
    {"iterator/FldSpec", {{"relation", "Literator/RelSpec;"}, {"offset", "I"}}, 0},
    {"iterator/RelSpec", {{"key", "I"}}, 0},
    {"global/AttrType", {{"attrType", "I"}}, 0},
    {"global/AttrOperator", {{"attrOperator", "I"}}, 0},
    {"global/IndexType", {{"indexType", "I"}}, 0},
    {"java/lang/Object", {{0, 0}}, 0},
    {"java/lang/String", {{0, 0}}, 0},
    {"chainexception/ChainException", {{0, 0}}, 1},
    {"iterator/FileScanException", {{0, 0}}, 1},
    {"iterator/PredEvalException", {{0, 0}}, 1},
    {"index/IndexException", {{0, 0}}, 1},
    {"heap/FieldNumberOutOfBoundException", {{0, 0}}, 1},
    {"java/lang/NoClassDefFoundError", {{0, 0}}, 2},
    {"java/lang/NoSuchFieldError", {{0, 0}}, 2},
    {"java/lang/NoSuchMethodError", {{0, 0}}, 2},
    {"java/lang/ArrayIndexOutOfBoundsException", {{0, 0}}, 2},
    {"java/lang/ArrayStoreException", {{0, 0}}, 2},
};
#define NCLASSES ((int)(sizeof(kClasses) / sizeof(kClasses[0])))
static const char *kExceptionCtorSig = "(Ljava/lang/Exception;Ljava/lang/String;)V";

struct _jobject {
  int magic, kind;
  const ClassDecl *cls; /* K_PLAIN / K_CLASS: the class; K_ARRAY of objects: element class (may be NULL) */
  /* K_PLAIN fields, in the class declaration's order */
  jint ival[MAXF];
  jfloat fval[MAXF];
  jobject oval[MAXF];
  /* exceptions */
  jobject cause, message;
  /* K_STRING */
  char *utf;
  jsize utflen;
  /* K_ARRAY: etype 'I','J','S','B','F' or 'L' */
  char etype;
  jsize len;
  void *data;
  /* K_BUFFER */
  void *addr;
  jlong cap;
  struct _jobject *all_next;
};

struct _jfieldID {
  const ClassDecl *cls;
  int slot;
  char sig[64];
};
struct _jmethodID {
  const ClassDecl *cls;
};

static struct _jobject *g_all;
static jthrowable g_pending;
static int g_outstanding, g_violations;
static char g_last_violation[512];
static struct _jfieldID g_fids[NCLASSES][MAXF];
static struct _jmethodID g_ctors[NCLASSES];

static void violation(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_violation, sizeof(g_last_violation), fmt, ap);
  va_end(ap);
  g_violations++;
}

static int valid(jobject o) { return o && o->magic == MAGIC; }

static jobject alloc_obj(int kind, const ClassDecl *cls) {
  jobject o = (jobject)calloc(1, sizeof(struct _jobject));
  if (!o) return NULL;
  o->magic = MAGIC;
  o->kind = kind;
  o->cls = cls;
  o->all_next = g_all;
  g_all = o;
  return o;
}

static const ClassDecl *class_decl(const char *name) {
  for (int i = 0; i < NCLASSES; i++)
    if (strcmp(kClasses[i].name, name) == 0) return &kClasses[i];
  return NULL;
}

static jobject new_string(const char *utf, jsize len) {
  jobject s = alloc_obj(K_STRING, class_decl("java/lang/String"));
  if (!s) return NULL;
  s->utf = (char *)malloc((size_t)len + 1);
  memcpy(s->utf, utf, (size_t)len);
  s->utf[len] = 0;
  s->utflen = len;
  return s;
}

static jobject new_exception(const ClassDecl *c, const char *msg) {
  jobject e = alloc_obj(K_PLAIN, c);
  if (e && msg) e->message = new_string(msg, (jsize)strlen(msg));
  return e;
}

static void raise(const char *cls, const char *msg) {
  g_pending = new_exception(class_decl(cls), msg);
}

/* JNI functions a native may call with an exception pending (JNI spec,
 * "Exceptions"): the rest are violations */
static void pending_check(const char *fn) {
  if (g_pending) violation("%s called with an exception pending", fn);
}

/* modified UTF-8: 1-, 2- and 3-byte forms only, no raw NUL, U+0000 as C0 80 */
static int valid_mutf8(const unsigned char *s, size_t n) {
  for (size_t i = 0; i < n;) {
    const unsigned c = s[i];
    if (c == 0) return 0;
    if (c < 0x80) {
      i += 1;
    } else if ((c & 0xE0) == 0xC0) {
      if (i + 1 >= n || (s[i + 1] & 0xC0) != 0x80) return 0;
      if (c < 0xC2 && !(c == 0xC0 && s[i + 1] == 0x80)) return 0;
      i += 2;
    } else if ((c & 0xF0) == 0xE0) {
      if (i + 2 >= n || (s[i + 1] & 0xC0) != 0x80 || (s[i + 2] & 0xC0) != 0x80) return 0;
      i += 3;
    } else {
      return 0;
    }
  }
  return 1;
}

/* ---- the JNIEnv table ---------------------------------------------------- */

static jclass J_FindClass(JNIEnv *env, const char *name) {
  (void)env;
  pending_check("FindClass");
  const ClassDecl *c = class_decl(name);
  if (!c) {
    raise("java/lang/NoClassDefFoundError", name);
    return NULL;
  }
  return alloc_obj(K_CLASS, c);
}

static jint J_Throw(JNIEnv *env, jthrowable obj) {
  (void)env;
  if (!valid(obj) || obj->kind != K_PLAIN || !obj->cls->is_exception) {
    violation("Throw of a non-throwable");
    return -1;
  }
  g_pending = obj;
  return 0;
}

static jint J_ThrowNew(JNIEnv *env, jclass clazz, const char *msg) {
  (void)env;
  if (!valid(clazz) || clazz->kind != K_CLASS || !clazz->cls->is_exception) {
    violation("ThrowNew on a non-throwable class");
    return -1;
  }
  g_pending = new_exception(clazz->cls, msg);
  return 0;
}

static void J_ExceptionClear(JNIEnv *env) {
  (void)env;
  g_pending = NULL;
}

static jboolean J_ExceptionCheck(JNIEnv *env) {
  (void)env;
  return g_pending ? JNI_TRUE : JNI_FALSE;
}

static void J_DeleteLocalRef(JNIEnv *env, jobject obj) {
  (void)env;
  if (obj && !valid(obj)) violation("DeleteLocalRef of a non-reference");
}

static jmethodID J_GetMethodID(JNIEnv *env, jclass clazz, const char *name, const char *sig) {
  (void)env;
  pending_check("GetMethodID");
  if (!valid(clazz) || clazz->kind != K_CLASS) {
    violation("GetMethodID on a non-class");
    return NULL;
  }
  if (clazz->cls->is_exception == 1 && strcmp(name, "<init>") == 0 && strcmp(sig, kExceptionCtorSig) == 0)
    return &g_ctors[clazz->cls - kClasses];
  raise("java/lang/NoSuchMethodError", name);
  return NULL;
}

static jobject J_NewObject(JNIEnv *env, jclass clazz, jmethodID m, ...) {
  (void)env;
  pending_check("NewObject");
  if (!valid(clazz) || clazz->kind != K_CLASS || m != &g_ctors[clazz->cls - kClasses]) {
    violation("NewObject with a method of another class");
    return NULL;
  }
  va_list ap;
  va_start(ap, m);
  jobject cause = va_arg(ap, jobject);
  jobject msg = va_arg(ap, jobject);
  va_end(ap);
  if ((cause && !valid(cause)) || (msg && (!valid(msg) || msg->kind != K_STRING))) {
    violation("NewObject: constructor arguments do not match %s", kExceptionCtorSig);
    return NULL;
  }
  jobject e = alloc_obj(K_PLAIN, clazz->cls);
  if (e) {
    e->cause = cause;
    e->message = msg;
  }
  return e;
}

static jfieldID J_GetFieldID(JNIEnv *env, jclass clazz, const char *name, const char *sig) {
  (void)env;
  pending_check("GetFieldID");
  if (!valid(clazz) || clazz->kind != K_CLASS) {
    violation("GetFieldID on a non-class");
    return NULL;
  }
  const ClassDecl *c = clazz->cls;
  for (int k = 0; k < MAXF && c->fields[k].name; k++)
    if (strcmp(c->fields[k].name, name) == 0 && strcmp(c->fields[k].sig, sig) == 0) {
      struct _jfieldID *f = &g_fids[c - kClasses][k];
      f->cls = c;
      f->slot = k;
      snprintf(f->sig, sizeof(f->sig), "%s", sig);
      return f;
    }
  raise("java/lang/NoSuchFieldError", name);
  return NULL;
}

static int field_ok(jobject obj, jfieldID f, char want, const char *fn) {
  pending_check(fn);
  if (!f) {
    violation("%s with a null field ID", fn);
    return 0;
  }
  if (!valid(obj) || obj->kind != K_PLAIN || obj->cls != f->cls) {
    violation("%s: object is not a %s", fn, f->cls->name);
    return 0;
  }
  if ((want == 'L' && f->sig[0] != 'L') || (want != 'L' && f->sig[0] != want)) {
    violation("%s on field %s of signature %s", fn, f->cls->fields[f->slot].name, f->sig);
    return 0;
  }
  return 1;
}

static jobject J_GetObjectField(JNIEnv *env, jobject obj, jfieldID f) {
  (void)env;
  return field_ok(obj, f, 'L', "GetObjectField") ? obj->oval[f->slot] : NULL;
}

static jint J_GetIntField(JNIEnv *env, jobject obj, jfieldID f) {
  (void)env;
  return field_ok(obj, f, 'I', "GetIntField") ? obj->ival[f->slot] : 0;
}

static jfloat J_GetFloatField(JNIEnv *env, jobject obj, jfieldID f) {
  (void)env;
  return field_ok(obj, f, 'F', "GetFloatField") ? obj->fval[f->slot] : 0.0f;
}

static jstring J_NewStringUTF(JNIEnv *env, const char *utf) {
  (void)env;
  pending_check("NewStringUTF");
  if (!utf) return NULL;
  const size_t n = strlen(utf);
  if (!valid_mutf8((const unsigned char *)utf, n)) violation("NewStringUTF: not modified UTF-8");
  return new_string(utf, (jsize)n);
}

static int string_ok(jstring s, const char *fn) {
  if (!valid(s) || s->kind != K_STRING) {
    violation("%s on a non-string", fn);
    return 0;
  }
  return 1;
}

static jsize J_GetStringUTFLength(JNIEnv *env, jstring str) {
  (void)env;
  pending_check("GetStringUTFLength");
  return string_ok(str, "GetStringUTFLength") ? str->utflen : 0;
}

static const char *J_GetStringUTFChars(JNIEnv *env, jstring str, jboolean *isCopy) {
  (void)env;
  pending_check("GetStringUTFChars");
  if (!string_ok(str, "GetStringUTFChars")) return NULL;
  char *c = (char *)malloc((size_t)str->utflen + 1);
  memcpy(c, str->utf, (size_t)str->utflen + 1);
  if (isCopy) *isCopy = JNI_TRUE;
  g_outstanding++;
  return c;
}

static void J_ReleaseStringUTFChars(JNIEnv *env, jstring str, const char *chars) {
  (void)env;
  if (!string_ok(str, "ReleaseStringUTFChars")) return;
  if (!chars) {
    violation("ReleaseStringUTFChars(NULL)");
    return;
  }
  free((void *)chars);
  g_outstanding--;
}

static int array_ok(jarray a, char et, const char *fn) {
  if (!valid(a) || a->kind != K_ARRAY) {
    violation("%s on a non-array", fn);
    return 0;
  }
  if (et && a->etype != et) {
    violation("%s on an array of element type %c", fn, a->etype);
    return 0;
  }
  return 1;
}

static size_t esize(char et) {
  switch (et) {
    case 'J': return 8;
    case 'I': case 'F': return 4;
    case 'S': return 2;
    case 'B': return 1;
    default: return sizeof(jobject);
  }
}

static jsize J_GetArrayLength(JNIEnv *env, jarray array) {
  (void)env;
  pending_check("GetArrayLength");
  return array_ok(array, 0, "GetArrayLength") ? array->len : 0;
}

static jobject new_array(char et, jsize len, const ClassDecl *ecls) {
  if (len < 0) return NULL;
  jobject a = alloc_obj(K_ARRAY, ecls);
  if (!a) return NULL;
  a->etype = et;
  a->len = len;
  a->data = calloc((size_t)(len > 0 ? len : 1), esize(et));
  return a;
}

static jobjectArray J_NewObjectArray(JNIEnv *env, jsize len, jclass clazz, jobject init) {
  (void)env;
  pending_check("NewObjectArray");
  if (!valid(clazz) || clazz->kind != K_CLASS) {
    violation("NewObjectArray with a non-class");
    return NULL;
  }
  jobject a = new_array('L', len, clazz->cls);
  for (jsize i = 0; a && i < len; i++) ((jobject *)a->data)[i] = init;
  return a;
}

static int index_ok(jarray a, jsize i, const char *fn) {
  if (i < 0 || i >= a->len) {
    raise("java/lang/ArrayIndexOutOfBoundsException", fn);
    return 0;
  }
  return 1;
}

static jobject J_GetObjectArrayElement(JNIEnv *env, jobjectArray array, jsize index) {
  (void)env;
  pending_check("GetObjectArrayElement");
  if (!array_ok(array, 'L', "GetObjectArrayElement") || !index_ok(array, index, "GetObjectArrayElement"))
    return NULL;
  return ((jobject *)array->data)[index];
}

static void J_SetObjectArrayElement(JNIEnv *env, jobjectArray array, jsize index, jobject val) {
  (void)env;
  pending_check("SetObjectArrayElement");
  if (!array_ok(array, 'L', "SetObjectArrayElement") || !index_ok(array, index, "SetObjectArrayElement")) return;
  if (val && !valid(val)) {
    violation("SetObjectArrayElement of a non-reference");
    return;
  }
  if (val && array->cls && strcmp(array->cls->name, "java/lang/String") == 0 && val->kind != K_STRING) {
    raise("java/lang/ArrayStoreException", "String[] element");
    return;
  }
  ((jobject *)array->data)[index] = val;
}

#define NEW_ARRAY(Name, T, ET)                                \
  static T##Array J_New##Name##Array(JNIEnv *env, jsize len) { \
    (void)env;                                                \
    pending_check("New" #Name "Array");                       \
    return new_array(ET, len, NULL);                          \
  }
NEW_ARRAY(Byte, jbyte, 'B')
NEW_ARRAY(Int, jint, 'I')
NEW_ARRAY(Long, jlong, 'J')
NEW_ARRAY(Float, jfloat, 'F')

static void *borrow(jarray a, char et, const char *fn, jboolean *isCopy) {
  pending_check(fn);
  if (!array_ok(a, et, fn)) return NULL;
  void *c = malloc(esize(et) * (size_t)(a->len > 0 ? a->len : 1));
  memcpy(c, a->data, esize(et) * (size_t)a->len);
  if (isCopy) *isCopy = JNI_TRUE;
  g_outstanding++;
  return c;
}

static void give_back(jarray a, char et, void *elems, jint mode, const char *fn) {
  if (!array_ok(a, et, fn)) return;
  if (!elems) {
    violation("%s(NULL)", fn);
    return;
  }
  if (mode == 0 || mode == JNI_COMMIT) memcpy(a->data, elems, esize(et) * (size_t)a->len);
  if (mode == 0 || mode == JNI_ABORT) {
    free(elems);
    g_outstanding--;
  } else if (mode != JNI_COMMIT) {
    violation("%s: bad mode %d", fn, mode);
  }
}

static jshort *J_GetShortArrayElements(JNIEnv *env, jshortArray a, jboolean *c) {
  (void)env;
  return (jshort *)borrow(a, 'S', "GetShortArrayElements", c);
}
static jint *J_GetIntArrayElements(JNIEnv *env, jintArray a, jboolean *c) {
  (void)env;
  return (jint *)borrow(a, 'I', "GetIntArrayElements", c);
}
static jlong *J_GetLongArrayElements(JNIEnv *env, jlongArray a, jboolean *c) {
  (void)env;
  return (jlong *)borrow(a, 'J', "GetLongArrayElements", c);
}
static void J_ReleaseShortArrayElements(JNIEnv *env, jshortArray a, jshort *e, jint mode) {
  (void)env;
  give_back(a, 'S', e, mode, "ReleaseShortArrayElements");
}
static void J_ReleaseIntArrayElements(JNIEnv *env, jintArray a, jint *e, jint mode) {
  (void)env;
  give_back(a, 'I', e, mode, "ReleaseIntArrayElements");
}
static void J_ReleaseLongArrayElements(JNIEnv *env, jlongArray a, jlong *e, jint mode) {
  (void)env;
  give_back(a, 'J', e, mode, "ReleaseLongArrayElements");
}

static int region_ok(jarray a, char et, jsize start, jsize len, const char *fn) {
  pending_check(fn);
  if (!array_ok(a, et, fn)) return 0;
  if (start < 0 || len < 0 || start + len > a->len) {
    raise("java/lang/ArrayIndexOutOfBoundsException", fn);
    return 0;
  }
  return 1;
}

#define REGION(Name, T, ET)                                                                              \
  __attribute__((unused)) static void J_Get##Name##ArrayRegion(JNIEnv *env, T##Array a, jsize s, jsize n, T *buf) { \
    (void)env;                                                                                           \
    if (region_ok(a, ET, s, n, "Get" #Name "ArrayRegion")) memcpy(buf, (T *)a->data + s, sizeof(T) * n); \
  }                                                                                                      \
  __attribute__((unused)) static void J_Set##Name##ArrayRegion(JNIEnv *env, T##Array a, jsize s, jsize n,    \
                                                               const T *buf) {                              \
    (void)env;                                                                                           \
    if (region_ok(a, ET, s, n, "Set" #Name "ArrayRegion")) memcpy((T *)a->data + s, buf, sizeof(T) * n); \
  }
REGION(Byte, jbyte, 'B')
REGION(Long, jlong, 'J')
REGION(Int, jint, 'I')
REGION(Float, jfloat, 'F')

static void *J_GetDirectBufferAddress(JNIEnv *env, jobject buf) {
  (void)env;
  pending_check("GetDirectBufferAddress");
  return valid(buf) && buf->kind == K_BUFFER ? buf->addr : NULL;
}

static jlong J_GetDirectBufferCapacity(JNIEnv *env, jobject buf) {
  (void)env;
  pending_check("GetDirectBufferCapacity");
  return valid(buf) && buf->kind == K_BUFFER ? buf->cap : -1;
}

static const struct JNINativeInterface_ kTable = {
    .FindClass = J_FindClass,
    .Throw = J_Throw,
    .ThrowNew = J_ThrowNew,
    .ExceptionClear = J_ExceptionClear,
    .ExceptionCheck = J_ExceptionCheck,
    .DeleteLocalRef = J_DeleteLocalRef,
    .GetMethodID = J_GetMethodID,
    .NewObject = J_NewObject,
    .GetFieldID = J_GetFieldID,
    .GetObjectField = J_GetObjectField,
    .GetIntField = J_GetIntField,
    .GetFloatField = J_GetFloatField,
    .NewStringUTF = J_NewStringUTF,
    .GetStringUTFLength = J_GetStringUTFLength,
    .GetStringUTFChars = J_GetStringUTFChars,
    .ReleaseStringUTFChars = J_ReleaseStringUTFChars,
    .GetArrayLength = J_GetArrayLength,
    .NewObjectArray = J_NewObjectArray,
    .GetObjectArrayElement = J_GetObjectArrayElement,
    .SetObjectArrayElement = J_SetObjectArrayElement,
    .NewByteArray = J_NewByteArray,
    .NewIntArray = J_NewIntArray,
    .NewLongArray = J_NewLongArray,
    .NewFloatArray = J_NewFloatArray,
    .GetShortArrayElements = J_GetShortArrayElements,
    .GetIntArrayElements = J_GetIntArrayElements,
    .GetLongArrayElements = J_GetLongArrayElements,
    .ReleaseShortArrayElements = J_ReleaseShortArrayElements,
    .ReleaseIntArrayElements = J_ReleaseIntArrayElements,
    .ReleaseLongArrayElements = J_ReleaseLongArrayElements,
    .GetByteArrayRegion = J_GetByteArrayRegion,
    .GetLongArrayRegion = J_GetLongArrayRegion,
    .SetByteArrayRegion = J_SetByteArrayRegion,
    .SetIntArrayRegion = J_SetIntArrayRegion,
    .SetLongArrayRegion = J_SetLongArrayRegion,
    .SetFloatArrayRegion = J_SetFloatArrayRegion,
    .GetDirectBufferAddress = J_GetDirectBufferAddress,
    .GetDirectBufferCapacity = J_GetDirectBufferCapacity,
};
static JNIEnv g_env = &kTable;

/* ---- the test's side (ctypes) ------------------------------------------------ */

#define EXPORT __attribute__((visibility("default")))

EXPORT JNIEnv *jh_env(void) { return &g_env; }

/* a new instance of a declared reference class: int / float fields 0, references null */
EXPORT jobject jh_new(const char *cls) {
  const ClassDecl *c = class_decl(cls);
  return c ? alloc_obj(K_PLAIN, c) : NULL;
}

static int slot_of(jobject o, const char *name, char kind) {
  if (!valid(o) || o->kind != K_PLAIN) return -1;
  for (int k = 0; k < MAXF && o->cls->fields[k].name; k++)
    if (strcmp(o->cls->fields[k].name, name) == 0) {
      const char s = o->cls->fields[k].sig[0];
      return (kind == 'L' ? s == 'L' : s == kind) ? k : -1;
    }
  return -1;
}

EXPORT int jh_set_int(jobject o, const char *name, jint v) {
  const int k = slot_of(o, name, 'I');
  if (k < 0) return -1;
  o->ival[k] = v;
  return 0;
}

EXPORT int jh_set_float(jobject o, const char *name, jfloat v) {
  const int k = slot_of(o, name, 'F');
  if (k < 0) return -1;
  o->fval[k] = v;
  return 0;
}

EXPORT int jh_set_obj(jobject o, const char *name, jobject v) {
  const int k = slot_of(o, name, 'L');
  if (k < 0 || (v && !valid(v))) return -1;
  o->oval[k] = v;
  return 0;
}

EXPORT jobject jh_string(const char *utf, jsize len) { return new_string(utf, len); }
EXPORT const char *jh_string_utf(jobject s) { return valid(s) && s->kind == K_STRING ? s->utf : NULL; }
EXPORT jsize jh_string_len(jobject s) { return valid(s) && s->kind == K_STRING ? s->utflen : -1; }

/* a primitive array ('I','J','S','B','F') initialised from data (may be NULL), or an object array of cls */
EXPORT jobject jh_array(char et, jsize len, const void *data, const char *cls) {
  jobject a = new_array(et, len, cls ? class_decl(cls) : NULL);
  if (a && data && et != 'L') memcpy(a->data, data, esize(et) * (size_t)len);
  return a;
}
EXPORT int jh_array_set(jobject a, jsize i, jobject v) {
  if (!valid(a) || a->kind != K_ARRAY || a->etype != 'L' || i < 0 || i >= a->len) return -1;
  ((jobject *)a->data)[i] = v;
  return 0;
}
EXPORT jobject jh_array_get(jobject a, jsize i) {
  if (!valid(a) || a->kind != K_ARRAY || a->etype != 'L' || i < 0 || i >= a->len) return NULL;
  return ((jobject *)a->data)[i];
}
EXPORT char jh_array_type(jobject a) { return valid(a) && a->kind == K_ARRAY ? a->etype : 0; }
EXPORT jsize jh_array_len(jobject a) { return valid(a) && a->kind == K_ARRAY ? a->len : -1; }
EXPORT void *jh_array_data(jobject a) { return valid(a) && a->kind == K_ARRAY ? a->data : NULL; }

/* a direct ByteBuffer over caller memory (ByteBuffer.allocateDirect) */
EXPORT jobject jh_direct_buffer(void *addr, jlong cap) {
  jobject b = alloc_obj(K_BUFFER, NULL);
  if (b) {
    b->addr = addr;
    b->cap = cap;
  }
  return b;
}

EXPORT jobject jh_pending(void) { return g_pending; }
EXPORT void jh_clear(void) { g_pending = NULL; }
EXPORT const char *jh_class_name(jobject o) { return valid(o) && o->cls ? o->cls->name : NULL; }
EXPORT jobject jh_exception_message(jobject e) { return valid(e) ? e->message : NULL; }
EXPORT jobject jh_exception_cause(jobject e) { return valid(e) ? e->cause : NULL; }
EXPORT int jh_outstanding(void) { return g_outstanding; }
EXPORT int jh_violations(void) { return g_violations; }
EXPORT const char *jh_last_violation(void) { return g_last_violation; }

/* drop every object (the test's objects and the glue's results) */
EXPORT void jh_reset(void) {
  while (g_all) {
    jobject o = g_all;
    g_all = o->all_next;
    free(o->utf);
    free(o->data);
    free(o);
  }
  g_pending = NULL;
  g_violations = 0;
  g_last_violation[0] = 0;
}
