/* Host-side Hungarian matching of the DVC training step (C ABI, no device code).
 *
 * Reference: models/matcher.py:86-94 (HungarianMatcher.forward) runs
 * scipy.optimize.linear_sum_assignment on every clip's (queries x targets) block of the cost matrix,
 * and utils/preds_postprocess.py get_src_permutation_idx turns the matches into (clip, prediction)
 * index lists.  The DVC step does this for every decoder level between its two HIP graphs
 * (dvc_core.StagedDVCLoss.host): 48 scipy calls plus numpy index building, ~0.7-1 ms of host time
 * during which the GPU waits.  mfl_lsa_levels does all of it in one call with scipy's algorithm
 * (Crouse's shortest augmenting path, the same row order, dual updates and tie rules), so the
 * assignments are the ones scipy returns.
 */
#ifndef MFL_HOST_LSA_H
#define MFL_HOST_LSA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MFL_LSA_OK 0
#define MFL_LSA_BAD_ARGS 1
#define MFL_LSA_INVALID 2    /* a NaN or -inf cost (scipy: ValueError "contains invalid numeric entries") */
#define MFL_LSA_INFEASIBLE 3 /* scipy: ValueError "cost matrix is infeasible" */

/* scipy.optimize.linear_sum_assignment(cost) for one (nr x nc) row-major float64 matrix.  Writes
 * min(nr, nc) pairs: rows[k] ascending, cols[k] the matched column. */
int mfl_lsa(const double* cost, int64_t nr, int64_t nc, int64_t* rows, int64_t* cols);

/* Every level's matching of the staged DVC loss.  cost: L blocks of (B, Q, n_tgt) float64 (the
 * copied request, as HungarianMatcher.level_costs concatenates it); clip b's targets are columns
 * [bounds[b], bounds[b+1]).  Per level and clip the
 * assignment of cost[l, b, :, bounds[b]:bounds[b+1]] is written as
 *   src[l * n_tgt + bounds[b] + k], tgt[...]: prediction and target (rows ascending, scipy's order);
 *   idx[(l * 2 + 0) * n_tgt + o], idx[(l * 2 + 1) * n_tgt + o]: clip b and the prediction matched
 *   to the clip's targets in target order (get_src_permutation_idx), o = bounds[b] + t.
 * Requires Q >= the clip's target count (every target matched, as the DVC loss assumes). */
int mfl_lsa_levels(const double* cost, int64_t L, int64_t B, int64_t Q, int64_t n_tgt, const int64_t* bounds,
                   int64_t* src, int64_t* tgt, int64_t* idx);

#ifdef __cplusplus
}
#endif

#endif /* MFL_HOST_LSA_H */
