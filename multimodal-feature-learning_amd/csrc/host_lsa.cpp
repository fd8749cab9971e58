// Host-side Hungarian matching of the DVC step (include/host_lsa.h).
//
// The assignment is the one scipy.optimize.linear_sum_assignment returns (scipy's
// rectangular_lsap: Crouse, "On implementing 2D rectangular assignment algorithms", 2016): a wide
// matrix (rows <= cols; a tall one is transposed first) is solved row by row, each row adding one
// shortest augmenting path found by a Dijkstra-like scan over the remaining columns with reduced
// costs c[i][j] - u[i] - v[j].  The results depend on the scan order and the tie rule, so both follow
// scipy: the remaining-column list starts in descending column order and a removed column is
// replaced by the list's last one; among equal path costs a free column (no row yet) wins, else the
// first one met.  Costs are compared in double, as scipy converts them.
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <numeric>
#include <vector>

#include "host_lsa.h"

namespace {

struct Solver {
  int64_t nr = 0, nc = 0;
  std::vector<double> u, v, dist;
  std::vector<int64_t> path, col_of_row, row_of_col, remaining;
  std::vector<char> row_seen, col_seen;

  void reset(int64_t r, int64_t c) {
    nr = r;
    nc = c;
    u.assign(r, 0.0);
    v.assign(c, 0.0);
    dist.assign(c, INFINITY);
    path.assign(c, -1);
    col_of_row.assign(r, -1);
    row_of_col.assign(c, -1);
    remaining.assign(c, 0);
    row_seen.assign(r, 0);
    col_seen.assign(c, 0);
  }

  // one shortest augmenting path from free row `start`; returns the sink column (-1: infeasible)
  int64_t augment(const double* cost, int64_t start, double* min_out) {
    int64_t left = nc;
    for (int64_t k = 0; k < nc; ++k) remaining[k] = nc - 1 - k;
    std::fill(row_seen.begin(), row_seen.end(), 0);
    std::fill(col_seen.begin(), col_seen.end(), 0);
    std::fill(dist.begin(), dist.end(), INFINITY);
    double reach = 0.0;
    int64_t i = start;
    for (;;) {
      row_seen[i] = 1;
      int64_t best = -1;
      double lowest = INFINITY;
      const double* ci = cost + i * nc;
      for (int64_t k = 0; k < left; ++k) {
        const int64_t j = remaining[k];
        const double r = reach + ci[j] - u[i] - v[j];
        if (r < dist[j]) {
          path[j] = i;
          dist[j] = r;
        }
        if (dist[j] < lowest || (dist[j] == lowest && row_of_col[j] == -1)) {
          lowest = dist[j];
          best = k;
        }
      }
      reach = lowest;
      if (reach == INFINITY) return -1;
      const int64_t j = remaining[best];
      col_seen[j] = 1;
      remaining[best] = remaining[--left];
      if (row_of_col[j] == -1) {
        *min_out = reach;
        return j;
      }
      i = row_of_col[j];
    }
  }

  // cost: nr x nc, nr <= nc; fills col_of_row
  int solve(const double* cost) {
    for (int64_t row = 0; row < nr; ++row) {
      double m = 0.0;
      const int64_t sink = augment(cost, row, &m);
      if (sink < 0) return MFL_LSA_INFEASIBLE;
      u[row] += m;
      for (int64_t i = 0; i < nr; ++i)
        if (row_seen[i] && i != row) u[i] += m - dist[col_of_row[i]];
      for (int64_t j = 0; j < nc; ++j)
        if (col_seen[j]) v[j] -= m - dist[j];
      for (int64_t j = sink;;) {  // flip the path
        const int64_t i = path[j];
        row_of_col[j] = i;
        std::swap(col_of_row[i], j);
        if (i == row) break;
      }
    }
    return MFL_LSA_OK;
  }
};

// scipy's linear_sum_assignment on a row-major nr x nc matrix given through an accessor
template <class At>
int assign(Solver& s, std::vector<double>& buf, int64_t nr, int64_t nc, At at, int64_t* rows, int64_t* cols) {
  if (nr == 0 || nc == 0) return MFL_LSA_OK;
  const bool tall = nc < nr;
  const int64_t r = tall ? nc : nr, c = tall ? nr : nc;
  buf.resize((size_t)(r * c));
  for (int64_t i = 0; i < nr; ++i)
    for (int64_t j = 0; j < nc; ++j) {
      const double x = at(i, j);
      if (x != x || x == -INFINITY) return MFL_LSA_INVALID;
      if (tall)
        buf[j * nr + i] = x;
      else
        buf[i * nc + j] = x;
    }
  s.reset(r, c);
  const int rc = s.solve(buf.data());
  if (rc != MFL_LSA_OK) return rc;
  if (tall) {  // pairs by ascending original row (= solved column)
    std::vector<int64_t> order(r);
    std::iota(order.begin(), order.end(), 0);
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return s.col_of_row[a] < s.col_of_row[b]; });
    for (int64_t k = 0; k < r; ++k) {
      rows[k] = s.col_of_row[order[k]];
      cols[k] = order[k];
    }
  } else {
    for (int64_t k = 0; k < r; ++k) {
      rows[k] = k;
      cols[k] = s.col_of_row[k];
    }
  }
  return MFL_LSA_OK;
}

}  // namespace

extern "C" int mfl_lsa(const double* cost, int64_t nr, int64_t nc, int64_t* rows, int64_t* cols) {
  if (nr < 0 || nc < 0 || ((nr > 0 && nc > 0) && (cost == nullptr || rows == nullptr || cols == nullptr)))
    return MFL_LSA_BAD_ARGS;
  Solver s;
  std::vector<double> buf;
  return assign(s, buf, nr, nc, [&](int64_t i, int64_t j) { return cost[i * nc + j]; }, rows, cols);
}

extern "C" int mfl_lsa_levels(const double* cost, int64_t L, int64_t B, int64_t Q, int64_t n_tgt,
                              const int64_t* bounds, int64_t* src, int64_t* tgt, int64_t* idx) {
  if (L < 0 || B < 0 || Q <= 0 || n_tgt < 0 || cost == nullptr || bounds == nullptr || src == nullptr ||
      tgt == nullptr || idx == nullptr || bounds[0] != 0 || bounds[B] != n_tgt)
    return MFL_LSA_BAD_ARGS;
  for (int64_t b = 0; b < B; ++b)
    if (bounds[b + 1] < bounds[b] || bounds[b + 1] - bounds[b] > Q) return MFL_LSA_BAD_ARGS;
  Solver s;
  std::vector<double> buf;
  for (int64_t l = 0; l < L; ++l) {
    for (int64_t b = 0; b < B; ++b) {
      const int64_t t0 = bounds[b], nt = bounds[b + 1] - t0;
      if (nt == 0) continue;
      const double* blk = cost + ((l * B + b) * Q) * n_tgt + t0;  // (Q, nt) with row stride n_tgt
      int64_t* rs = src + l * n_tgt + t0;
      int64_t* cs = tgt + l * n_tgt + t0;
      const int rc = assign(s, buf, Q, nt, [&](int64_t i, int64_t j) { return blk[i * n_tgt + j]; }, rs, cs);
      if (rc != MFL_LSA_OK) return rc;
      // get_src_permutation_idx: the clip's matched predictions in target order
      int64_t* ib = idx + (l * 2) * n_tgt + t0;
      int64_t* ip = idx + (l * 2 + 1) * n_tgt + t0;
      for (int64_t k = 0; k < nt; ++k) {
        ib[cs[k]] = b;
        ip[cs[k]] = rs[k];
      }
    }
  }
  return MFL_LSA_OK;
}
