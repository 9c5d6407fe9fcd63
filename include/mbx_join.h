/*
 * mbx_join.h -- the join operators above the scan:
 * ColumnarNestedLoopJoins (`nlj`) and the bitmap join of BitMapQuery
 * (`bmj`), as one GPU primitive that evaluates a join CNF over every
 * (outer, inner) pair of two selections and emits the matching pairs in the
 * reference's order.  R/ = minijava/src of the reference.
 *
 * Both reference joins reduce to the same pair predicate: a CNF whose terms
 * compare an outer column with an inner column, `outer.a OP inner.b`
 * (NljQuery.buildCNFJoinCondExpr, PredEval.Eval with the outer tuple as
 * operand 1: R/input/NljQuery.java:372-404, R/iterator/PredEval.java:56-162);
 * BitMapQuery states the same term from the inner side with the mirrored
 * operator (AttrOperator.getOppositeOperator, BitMapQuery.java:438-460) and
 * evaluates it through bitmap indexes -- on live rows that selects exactly
 * the rows the predicate selects.  They differ only in the output order:
 *
 *   MBX_JOIN_BMJ  outer positions ascending, then inner ascending
 *                 (BitMapQuery.executeJoin, R/input/BitMapQuery.java:187-300);
 *   MBX_JOIN_NLJ  block nested loops (ColumnarNestedLoopJoins.get_next,
 *                 R/iterator/ColumnarNestedLoopJoins.java:160-200): the outer
 *                 selection in blocks of `outer_block` tuples (one pass over
 *                 the inner relation per block); within a pass inner
 *                 ascending, then outer ascending within the block.
 *
 * The pair matrix is computed by k_join_matrix (one wave per 64 pairs, the
 * wave ballot is one word of the matrix row), then compacted with the scan's
 * nextSetBit kernels; results stay in HBM until fetched.
 */
#ifndef MBX_JOIN_H
#define MBX_JOIN_H

#include <stdint.h>

#include "mbx.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MBX_JOIN_BMJ 0
#define MBX_JOIN_NLJ 1
#define MBX_MAX_JOIN_TERMS 16

typedef struct mbx_join_result mbx_join_result;

/* `outer_col OP inner_col` (0-based table columns; AttrOperator codes; both
 * columns of one AttrType -- "Invalid JOIN COLUMN ATTR TYPE NOT MATCH"
 * otherwise).  aopNOT compares as != (PredEval); aopNOP / opRANGE are never
 * true. */
typedef struct mbx_join_term {
  int32_t op;
  int32_t outer_col;
  int32_t inner_col;
  int32_t pad_;
} mbx_join_term;

/* CNF: conjunct k = terms[conj_offsets[k] .. conj_offsets[k+1]) OR-ed. */
typedef struct mbx_join_cnf {
  const mbx_join_term* terms;
  const int32_t* conj_offsets; /* nconj + 1 entries */
  int32_t nconj;
} mbx_join_cnf;

/* Join the rows of `outer` selected by `outer_sel` with the rows of `inner`
 * selected by `inner_sel` (BitSets of the tables' sizes).  order =
 * MBX_JOIN_BMJ or MBX_JOIN_NLJ (outer_block > 0 tuples per pass, i.e.
 * (amt_of_memory - 1) * (1024 / outer tuple size)).  *out owns the pairs. */
int mbx_join(mbx_ctx* ctx, const mbx_table* outer, const mbx_bitmap* outer_sel, const mbx_table* inner,
             const mbx_bitmap* inner_sel, const mbx_join_cnf* cnf, int32_t order, int64_t outer_block,
             mbx_join_result** out);

/* number of result pairs; number of passes over the inner relation (NLJ:
 * ceil(outer selected / outer_block), at least 1; BMJ: 1) */
int mbx_join_info(const mbx_join_result* r, int64_t* count, int64_t* passes);

/* copy pairs [start, start + n) to the host: global outer / inner positions
 * (row_offset added) and, for NLJ, the pass each pair belongs to.  Any output
 * pointer may be null. */
int mbx_join_fetch(mbx_ctx* ctx, const mbx_join_result* r, int64_t start, int64_t n, int64_t* outer_pos,
                   int64_t* inner_pos, int32_t* pass);

int mbx_join_free(mbx_join_result* r);

/* Late materialisation by explicit positions (Heapfile.findRID + getRecord
 * per value, R/input/BitMapQuery.java:215-262): out[j][k] = column proj[j]
 * at global position positions[k], in the mbx_materialize host layout. */
int mbx_gather(mbx_ctx* ctx, const mbx_table* t, const int64_t* positions, int64_t n, const int32_t* proj,
               int32_t nproj, void* const* host_out);

#ifdef __cplusplus
}
#endif

#endif /* MBX_JOIN_H */
