/*
 * oracle.c -- CPU restatement of the Minibase-Columnar scan/filter/index path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Plain C, one row at a time, in
 * the reference's own order, deliberately unoptimised: it is the checker,
 * never the thing measured as the product.
 *
 * R/ = /root/reference/minijava/src.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- strings */

/* DataInputStream.readUTF: modified UTF-8 -> UTF-16 code units.
 * Returns the number of code units, or ORC_E_TYPE on malformed input
 * (UTFDataFormatException in Java). */
static int utf8m_to_utf16(const unsigned char *s, int32_t n, uint16_t *out) {
  int32_t i = 0, k = 0;
  while (i < n) {
    unsigned c = s[i];
    if (c < 0x80) {
      out[k++] = (uint16_t)c;
      i += 1;
    } else if ((c & 0xE0) == 0xC0) {
      if (i + 1 >= n || (s[i + 1] & 0xC0) != 0x80) return ORC_E_TYPE;
      out[k++] = (uint16_t)(((c & 0x1F) << 6) | (s[i + 1] & 0x3F));
      i += 2;
    } else if ((c & 0xF0) == 0xE0) {
      if (i + 2 >= n || (s[i + 1] & 0xC0) != 0x80 || (s[i + 2] & 0xC0) != 0x80) return ORC_E_TYPE;
      out[k++] = (uint16_t)(((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F));
      i += 3;
    } else {
      return ORC_E_TYPE;
    }
  }
  return k;
}

/* String.compareTo (lexicographic over UTF-16 code units, then length),
 * reduced to {-1,0,1} as TupleUtils.CompareTupleWithTuple does
 * (R/iterator/TupleUtils.java:79-82).  Returns -1/0/1, or 2 on malformed input. */
int orc_string_compare(const char *a, int32_t alen, const char *b, int32_t blen) {
  uint16_t ua[1024], ub[1024];
  if (alen > 1024 || blen > 1024) return 2;
  int na = utf8m_to_utf16((const unsigned char *)a, alen, ua);
  int nb = utf8m_to_utf16((const unsigned char *)b, blen, ub);
  if (na < 0 || nb < 0) return 2;
  int lim = na < nb ? na : nb;
  for (int k = 0; k < lim; k++) {
    if (ua[k] != ub[k]) return ua[k] < ub[k] ? -1 : 1;
  }
  if (na == nb) return 0;
  return na < nb ? -1 : 1;
}

/* payload length of a zero-padded string slot (Convert.getStrValue reads
 * exactly the writeUTF length; our payload is padded with 0x00, which never
 * occurs inside modified UTF-8) */
static int32_t slot_len(const char *p, int32_t size) {
  int32_t n = 0;
  while (n < size && p[n] != 0) n++;
  return n;
}

/* ------------------------------------------------------------- field reads */

typedef struct {
  int32_t type;
  int32_t i;
  float r;
  const char *s;
  int32_t slen;
} fieldval;

static int read_column(const orc_column *cols, int32_t ncols, int32_t fld, int64_t row, fieldval *v) {
  if (fld < 1 || fld > ncols) return ORC_E_RANGE; /* FieldNumberOutOfBoundException */
  const orc_column *c = &cols[fld - 1];
  v->type = c->attr_type;
  switch (c->attr_type) {
    case ORC_INTEGER: v->i = ((const int32_t *)c->data)[row]; return ORC_OK;
    case ORC_REAL: v->r = ((const float *)c->data)[row]; return ORC_OK;
    case ORC_STRING:
      v->s = (const char *)c->data + (size_t)row * (size_t)c->size;
      v->slen = slot_len(v->s, c->size);
      return ORC_OK;
    default: return ORC_E_TYPE;
  }
}

static int read_literal(const orc_operand *o, fieldval *v) {
  v->type = o->type;
  switch (o->type) {
    case ORC_INTEGER: v->i = o->integer; return ORC_OK;
    case ORC_REAL: v->r = o->real; return ORC_OK;
    case ORC_STRING: v->s = o->string; v->slen = o->string_len; return ORC_OK;
    default: return ORC_E_TYPE;
  }
}

/* TupleUtils.CompareTupleWithTuple (R/iterator/TupleUtils.java:35-87).
 * Both fields are read as `fldType`; a field of another type is what the
 * reference would misread (garbage or an exception) -> ORC_E_TYPE.
 * Float NaN falls through the float case into the string case in the
 * reference and raises there -> ORC_E_TYPE. */
static int compare_fields(int32_t fldType, const fieldval *a, const fieldval *b, int *res) {
  if (a->type != fldType || b->type != fldType) return ORC_E_TYPE;
  switch (fldType) {
    case ORC_INTEGER:
      *res = a->i == b->i ? 0 : (a->i < b->i ? -1 : 1);
      return ORC_OK;
    case ORC_REAL:
      if (a->r == b->r) { *res = 0; return ORC_OK; }
      if (a->r < b->r) { *res = -1; return ORC_OK; }
      if (a->r > b->r) { *res = 1; return ORC_OK; }
      return ORC_E_TYPE;
    case ORC_STRING: {
      int c = orc_string_compare(a->s, a->slen, b->s, b->slen);
      if (c == 2) return ORC_E_TYPE;
      *res = c;
      return ORC_OK;
    }
    default: return ORC_E_TYPE;
  }
}

/* the op switch of PredEval.Eval (R/iterator/PredEval.java:137-162) */
static int op_result(int32_t op, int comp_res) {
  switch (op) {
    case ORC_EQ: return comp_res == 0;
    case ORC_LT: return comp_res < 0;
    case ORC_GT: return comp_res > 0;
    case ORC_NE: return comp_res != 0;
    case ORC_LE: return comp_res <= 0;
    case ORC_GE: return comp_res >= 0;
    case ORC_NOT: return comp_res != 0;
    default: return 0; /* aopNOP, opRANGE */
  }
}

/* one CondExpr of PredEval.Eval (R/iterator/PredEval.java:54-135) */
static int eval_term(const orc_condexpr *t, const orc_column *cols, int32_t ncols, int64_t row) {
  fieldval v1, v2;
  int32_t comparison_type;
  int rc;
  /* operand 1 (:54-91): a literal goes into the shared `value` tuple and
   * fixes the comparison type; a symbol takes its column's type */
  if (t->operand1.type == ORC_SYMBOL) {
    rc = read_column(cols, ncols, t->operand1.fld, row, &v1);
    if (rc) return rc;
    comparison_type = v1.type;
  } else {
    rc = read_literal(&t->operand1, &v1);
    if (rc) return rc;
    comparison_type = t->operand1.type;
  }
  /* operand 2 (:93-128) */
  if (t->operand2.type == ORC_SYMBOL) {
    rc = read_column(cols, ncols, t->operand2.fld, row, &v2);
    if (rc) return rc;
  } else {
    rc = read_literal(&t->operand2, &v2);
    if (rc) return rc;
    /* both operands literal: `value` is one Tuple object, re-filled by
     * operand 2, so tuple1 == tuple2 and the reference compares operand 2
     * with itself */
    if (t->operand1.type != ORC_SYMBOL) v1 = v2;
  }
  int comp_res = 0;
  rc = compare_fields(comparison_type, &v1, &v2, &comp_res);
  if (rc) return rc;
  return op_result(t->op, comp_res);
}

int orc_pred_eval(const orc_cnf *cnf, const orc_column *cols, int32_t ncols, int64_t row) {
  if (cnf == NULL || cnf->nconj == 0) return 1; /* p == null */
  int col_res = 1;
  for (int32_t i = 0; i < cnf->nconj; i++) {     /* while (p[i] != null) */
    int row_res = 0;
    for (int32_t k = cnf->conj_offsets[i]; k < cnf->conj_offsets[i + 1]; k++) {
      int op_res = eval_term(&cnf->conds[k], cols, ncols, row);
      if (op_res < 0) return op_res;
      row_res = row_res || op_res;
      if (row_res) break;                            /* OR predicates satisfied */
    }
    col_res = col_res && row_res;
    if (!col_res) return 0;
  }
  return 1;
}

/* --------------------------------------------------------------- scanning */

static int deleted(const uint64_t *w, int64_t pos) {
  return w != NULL && ((w[pos >> 6] >> (pos & 63)) & 1ULL);
}

int64_t orc_filescan(const orc_column *cols, int32_t ncols, int64_t nrows,
                     const uint64_t *deleted_words, const orc_cnf *cnf,
                     uint64_t *out_words, int64_t *out_ids) {
  if (out_words) memset(out_words, 0, (size_t)((nrows + 63) / 64) * sizeof(uint64_t));
  int64_t count = 0;
  for (int64_t pos = 0; pos < nrows; pos++) {   /* TupleScan.getNext: position order */
    if (deleted(deleted_words, pos)) continue;  /* markedDeleted.get(pos) */
    int r = orc_pred_eval(cnf, cols, ncols, pos);
    if (r < 0) return r;
    if (!r) continue;
    if (out_words) out_words[pos >> 6] |= 1ULL << (pos & 63);
    if (out_ids) out_ids[count] = pos;
    count++;
  }
  return count;
}

/* The same COUNT with the rows split into `nthreads` contiguous ranges, each
 * evaluated by one OpenMP thread exactly like orc_filescan (the CPU baseline
 * bench.py reports: SURVEY 8(d)(ii), "the C++ CPU restatement across host
 * cores").  Row order inside a range is the reference's. */
int64_t orc_filescan_count_mt(const orc_column *cols, int32_t ncols, int64_t nrows,
                              const uint64_t *deleted_words, const orc_cnf *cnf, int32_t nthreads) {
  int64_t count = 0;
  int err = 0;
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel for num_threads(nthreads) reduction(+ : count) reduction(| : err) schedule(static)
  for (int32_t t = 0; t < nthreads; t++) {
    const int64_t a = nrows * t / nthreads, b = nrows * (t + 1) / nthreads;
    for (int64_t pos = a; pos < b; pos++) {
      if (deleted(deleted_words, pos)) continue;
      int r = orc_pred_eval(cnf, cols, ncols, pos);
      if (r < 0) {
        err |= 1;
        break;
      }
      count += r;
    }
  }
  return err ? ORC_E_TYPE : count;
}

int orc_aggregate(const orc_column *cols, int32_t ncols, int64_t nrows,
                  const uint64_t *deleted_words, const orc_cnf *cnf,
                  int32_t agg_col, orc_agg *out) {
  if (agg_col < 0 || agg_col >= ncols) return ORC_E_RANGE;
  const orc_column *a = &cols[agg_col];
  if (a->attr_type != ORC_INTEGER && a->attr_type != ORC_REAL) return ORC_E_TYPE;
  memset(out, 0, sizeof(*out));
  out->agg_type = a->attr_type;
  out->imin = INT32_MAX;
  out->imax = INT32_MIN;
  out->fmin = INFINITY;
  out->fmax = -INFINITY;
  for (int64_t pos = 0; pos < nrows; pos++) {
    if (deleted(deleted_words, pos)) continue;
    int r = orc_pred_eval(cnf, cols, ncols, pos);
    if (r < 0) return r;
    if (!r) continue;
    out->count++;
    if (a->attr_type == ORC_INTEGER) {
      int32_t v = ((const int32_t *)a->data)[pos];
      out->isum += v;
      if (v < out->imin) out->imin = v;
      if (v > out->imax) out->imax = v;
    } else {
      float v = ((const float *)a->data)[pos];
      out->fsum += (double)v;
      if (v < out->fmin) out->fmin = v;
      if (v > out->fmax) out->fmax = v;
    }
  }
  return ORC_OK;
}

/* ------------------------------------------------------------ bitmap index */

static int equal_value(const orc_column *col, int64_t row, const orc_operand *value, int *eq) {
  fieldval a, b;
  int rc = read_column(col, 1, 1, row, &a);
  if (rc) return rc;
  rc = read_literal(value, &b);
  if (rc) return rc;
  int c = 0;
  rc = compare_fields(col->attr_type, &a, &b, &c);
  if (rc) return rc;
  *eq = (c == 0);
  return ORC_OK;
}

int64_t orc_bitmap_eq(const orc_column *col, int64_t nrows, const uint64_t *deleted_words,
                      const orc_operand *value, uint64_t *out_words) {
  memset(out_words, 0, (size_t)((nrows + 63) / 64) * sizeof(uint64_t));
  int64_t n = 0;
  for (int64_t pos = 0; pos < nrows; pos++) {
    if (deleted(deleted_words, pos)) continue; /* ColumnScan.getNext skips it */
    int eq = 0;
    int rc = equal_value(col, pos, value, &eq);
    if (rc) return rc;
    if (eq) {
      out_words[pos >> 6] |= 1ULL << (pos & 63);
      n++;
    }
  }
  return n;
}

/* getBitmapValues: the distinct values the index registered while scanning
 * the live rows (Columnarfile.java:698-753, :1138).  Returned as row indices
 * of first occurrences. */
static int64_t distinct_rows(const orc_column *col, int64_t nrows, const uint64_t *deleted_words, int64_t **out) {
  int64_t *first = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nrows > 0 ? nrows : 1));
  int64_t nd = 0;
  if (col->attr_type == ORC_INTEGER) {
    /* sort-free O(n * distinct) -- fine for an oracle on low-cardinality columns */
    const int32_t *d = (const int32_t *)col->data;
    for (int64_t r = 0; r < nrows; r++) {
      if (deleted(deleted_words, r)) continue;
      int seen = 0;
      for (int64_t k = 0; k < nd && !seen; k++) seen = d[first[k]] == d[r];
      if (!seen) first[nd++] = r;
    }
  } else {
    const char *d = (const char *)col->data;
    for (int64_t r = 0; r < nrows; r++) {
      if (deleted(deleted_words, r)) continue;
      int seen = 0;
      for (int64_t k = 0; k < nd && !seen; k++)
        seen = memcmp(d + (size_t)first[k] * col->size, d + (size_t)r * col->size, (size_t)col->size) == 0;
      if (!seen) first[nd++] = r;
    }
  }
  *out = first;
  return nd;
}

int64_t orc_column_index_scan(const orc_column *col, int64_t nrows, const uint64_t *deleted_words,
                              int32_t op, const orc_operand *value, uint64_t *out_words) {
  int64_t nw = (nrows + 63) / 64;
  memset(out_words, 0, (size_t)nw * sizeof(uint64_t));
  if (col->attr_type != ORC_INTEGER && col->attr_type != ORC_STRING) return ORC_E_TYPE;
  if (value->type != col->attr_type) return ORC_E_TYPE;
  uint64_t *tmp = (uint64_t *)malloc((size_t)(nw > 0 ? nw : 1) * sizeof(uint64_t));
  int64_t rc = 0;
  /* symbol = value (EQ, LE, GE include the literal itself; :660-668).  A
   * literal with no bitmap file yields an empty BitSet (Columnarfile.java:1124). */
  if (op == ORC_EQ || op == ORC_LE || op == ORC_GE) {
    rc = orc_bitmap_eq(col, nrows, deleted_words, value, tmp);
    if (rc < 0) goto done;
    for (int64_t w = 0; w < nw; w++) out_words[w] |= tmp[w];
  }
  if (op == ORC_LT || op == ORC_LE || op == ORC_GT || op == ORC_GE || op == ORC_NE) {
    int64_t *first = NULL;
    int64_t nd = distinct_rows(col, nrows, deleted_words, &first);
    for (int64_t k = 0; k < nd; k++) {
      fieldval other, lit;
      read_column(col, 1, 1, first[k], &other);
      read_literal(value, &lit);
      int c = 0; /* c = sign(value.compareTo(other)) or int compare */
      rc = compare_fields(col->attr_type, &lit, &other, &c);
      if (rc < 0) { free(first); goto done; }
      int take = 0;
      if (op == ORC_LT || op == ORC_LE) take = take || c > 0;   /* value > other (:671-688) */
      if (op == ORC_GT || op == ORC_GE) take = take || c < 0;   /* value < other (:691-709) */
      if (op == ORC_NE) take = c != 0;                           /* (:712-730) */
      if (!take) continue;
      orc_operand ov;
      memset(&ov, 0, sizeof(ov));
      ov.type = col->attr_type;
      if (col->attr_type == ORC_INTEGER) ov.integer = other.i;
      else { ov.string = other.s; ov.string_len = other.slen; }
      rc = orc_bitmap_eq(col, nrows, deleted_words, &ov, tmp);
      if (rc < 0) { free(first); goto done; }
      for (int64_t w = 0; w < nw; w++) out_words[w] |= tmp[w];
    }
    free(first);
  }
  /* aopNOT / aopNOP / opRANGE select no value: the BitSet stays empty */
  /* getPositionsOfIndexScan: nextSetBit loop skipping markedDeleted */
  rc = 0;
  for (int64_t w = 0; w < nw; w++) {
    if (deleted_words) out_words[w] &= ~deleted_words[w];
    rc += __builtin_popcountll(out_words[w]);
  }
done:
  free(tmp);
  return rc;
}

int64_t orc_columnar_index_scan(const orc_column *cols, int32_t ncols, int64_t nrows,
                                const uint64_t *deleted_words, const orc_cnf *cnf,
                                uint64_t *out_words) {
  int64_t nw = (nrows + 63) / 64;
  if (cnf == NULL || cnf->nconj == 0) return ORC_E_INVALID;
  int32_t nc = cnf->nconj;
  int32_t nt = cnf->conj_offsets[nc];
  /* one BitSet object per conjunct; object 0 is also `outputPositions` */
  uint64_t *obj = (uint64_t *)calloc((size_t)nc * (size_t)(nw > 0 ? nw : 1), sizeof(uint64_t));
  uint64_t *term = (uint64_t *)malloc((size_t)(nw > 0 ? nw : 1) * sizeof(uint64_t));
  /* duplicateConstraints: constraint -> conjunct BitSet object (reference
   * semantics: the cached value is the *mutable* conjunct BitSet, :147-172) */
  int32_t *cache = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nt > 0 ? nt : 1));
  for (int32_t k = 0; k < nt; k++) cache[k] = -1;
  int64_t rc = 0;
  for (int32_t i = 0; i < nc; i++) {
    uint64_t *positions = obj + (size_t)i * (size_t)nw;
    for (int32_t k = cnf->conj_offsets[i]; k < cnf->conj_offsets[i + 1]; k++) {
      const orc_condexpr *t = &cnf->conds[k];
      if (t->operand1.type != ORC_SYMBOL || t->operand2.type == ORC_SYMBOL) { rc = ORC_E_INVALID; goto out; }
      if (t->operand1.fld < 1 || t->operand1.fld > ncols) { rc = ORC_E_RANGE; goto out; }
      /* the constraint key is column + op + literal (+ index type, always
       * Bitmap here); find the first earlier identical term */
      int32_t key = k;
      int32_t occurrences = 0;
      for (int32_t j = 0; j < nt; j++) {
        const orc_condexpr *u = &cnf->conds[j];
        int same = u->operand1.fld == t->operand1.fld && u->op == t->op &&
                   u->index_type == t->index_type &&
                   u->operand2.type == t->operand2.type &&
                   (t->operand2.type == ORC_STRING
                        ? (u->operand2.string_len == t->operand2.string_len &&
                           memcmp(u->operand2.string, t->operand2.string, (size_t)t->operand2.string_len) == 0)
                        : u->operand2.integer == t->operand2.integer);
        if (same) {
          occurrences++;
          if (j < key) key = j;
        }
      }
      int in_cache = cache[key] >= 0;
      int dup = in_cache ? 1 : occurrences > 1;
      if (!dup || !in_cache) {
        if (t->index_type == ORC_IDX_BTREE) {
          orc_cnf one;
          int32_t offs[2] = {0, 1};
          one.conds = t;
          one.conj_offsets = offs;
          one.nconj = 1;
          rc = orc_filescan(cols, ncols, nrows, deleted_words, &one, term, NULL);
        } else {
          rc = orc_column_index_scan(&cols[t->operand1.fld - 1], nrows, deleted_words, t->op,
                                     &t->operand2, term);
        }
        if (rc < 0) goto out;
        for (int64_t w = 0; w < nw; w++) positions[w] |= term[w];
        if (dup) cache[key] = i;
      } else {
        const uint64_t *src = obj + (size_t)cache[key] * (size_t)nw;
        for (int64_t w = 0; w < nw; w++) positions[w] |= src[w];
      }
    }
    if (i > 0) {
      for (int64_t w = 0; w < nw; w++) obj[w] &= positions[w]; /* outputPositions.and */
    }
  }
  rc = 0;
  for (int64_t w = 0; w < nw; w++) {
    out_words[w] = obj[w];
    rc += __builtin_popcountll(obj[w]);
  }
out:
  free(obj);
  free(term);
  free(cache);
  return rc;
}

int orc_gather(const orc_column *cols, int32_t ncols, const int64_t *ids, int64_t nids,
               const int32_t *proj, int32_t nproj, void *const *out) {
  for (int32_t j = 0; j < nproj; j++) {
    if (proj[j] < 0 || proj[j] >= ncols) return ORC_E_RANGE;
    const orc_column *c = &cols[proj[j]];
    size_t w = c->attr_type == ORC_STRING ? (size_t)c->size : 4;
    for (int64_t i = 0; i < nids; i++)
      memcpy((char *)out[j] + (size_t)i * w, (const char *)c->data + (size_t)ids[i] * w, w);
  }
  return ORC_OK;
}

int orc_decode_str_record(const uint8_t *rec, int32_t size, char *out_payload) {
  int32_t len = ((int32_t)rec[0] << 8) | rec[1];
  if (len > size) return ORC_E_RANGE;
  memset(out_payload, 0, (size_t)size);
  memcpy(out_payload, rec + 2, (size_t)len);
  return len;
}
