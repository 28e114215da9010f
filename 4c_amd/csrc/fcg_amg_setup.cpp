// fcg_amg_setup.cpp -- the graph half of the smoothed-aggregation AMG setup (SURVEY §8f row 2 on
// meshes without a box hierarchy).  4C solves the structural tangent with Belos + MueLu
// (4C_linear_solver_preconditioner_muelu.cpp, parameters from the input file's SOLVER block; MueLu
// itself -- Trilinos sha 06db4c85, not vendored -- defaults to smoothed aggregation with uncoupled
// aggregation, drop tolerance 0 and the rigid-body-mode near-null space of elasticity).  What is
// restated here is that published algorithm (Vanek, Mandel, Brezina, Computing 56 (1996)):
//
//  * fcg_amg_aggregate: uncoupled aggregation of the block (node) graph.  Phase 1: a node whose
//    neighbours are all unaggregated becomes a root, its aggregate the root plus its neighbours.
//    Phase 2 (twice): an unaggregated node joins the neighbouring aggregate it has the most
//    connections to (lowest id on ties).  Phase 3: what remains forms aggregates with its
//    unaggregated neighbours (a singleton if none).  Nodes marked `skip` (all DOFs Dirichlet)
//    are never aggregated: their prolongator rows stay empty.
//  * fcg_amg_tentative: the tentative prolongator block of every node and the coarse near-null
//    space: per aggregate the stacked near-null-space rows M (bs rows per node, 6 columns) are
//    factored M = Q R (modified Gram-Schmidt, two passes); Q's rows are the nodes' blocks, R the
//    coarse node's 6 x 6 near-null-space block.  A column that vanishes (an aggregate too small to
//    carry all six rigid-body modes) gives a zero column of Q and a zero coarse row: that coarse
//    DOF is decoupled by the device setup (unit diagonal, fcg_bsr_block_jacobi_setup).
//  * fcg_bsr_symbolic / fcg_bsr_transpose_pattern: block patterns of C = A B (each row's columns
//    sorted ascending -- the device product binary-searches them) and of P^T.
// The numeric half (products, smoothing, block inverses, the cycle's operators) is fcg_amg.hip.
#include <algorithm>
#include <thread>
#include <atomic>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "fourc_gpu.h"

extern "C" {

int64_t fcg_amg_aggregate(int64_t n, const int64_t* ptr, const int32_t* adj, const uint8_t* skip,
    int32_t* agg)
{
  if (n < 0 || (n > 0 && (!ptr || !adj || !agg))) return -1;
  if (n > 0 && ptr[0] != 0) return -1;
  for (int64_t i = 0; i < n; ++i)
  {
    if (ptr[i + 1] < ptr[i]) return -1;
    for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k)
      if (adj[k] < 0 || adj[k] >= n) return -1;
  }
  for (int64_t i = 0; i < n; ++i) agg[i] = -1;
  auto skipped = [&](int64_t i) { return skip && skip[i]; };
  int32_t n_agg = 0;
  // phase 1: roots whose whole neighbourhood is free
  for (int64_t i = 0; i < n; ++i)
  {
    if (skipped(i) || agg[i] >= 0) continue;
    bool free = true;
    for (int64_t k = ptr[i]; k < ptr[i + 1] && free; ++k)
    {
      const int32_t j = adj[k];
      if (j != i && !skipped(j) && agg[j] >= 0) free = false;
    }
    if (!free) continue;
    agg[i] = n_agg;
    for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k)
    {
      const int32_t j = adj[k];
      if (!skipped(j)) agg[j] = n_agg;
    }
    ++n_agg;
  }
  // phase 2 (two sweeps): join the neighbouring aggregate with the most connections
  std::vector<int32_t> cand, cnt;
  for (int sweep = 0; sweep < 2; ++sweep)
  {
    std::vector<int32_t> next(agg, agg + n);
    for (int64_t i = 0; i < n; ++i)
    {
      if (skipped(i) || agg[i] >= 0) continue;
      cand.clear();
      for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k)
      {
        const int32_t j = adj[k];
        if (j != i && !skipped(j) && agg[j] >= 0) cand.push_back(agg[j]);
      }
      if (cand.empty()) continue;
      std::sort(cand.begin(), cand.end());
      int32_t best = cand[0], best_n = 0;
      for (size_t s = 0; s < cand.size();)
      {
        size_t e = s;
        while (e < cand.size() && cand[e] == cand[s]) ++e;
        if (int32_t(e - s) > best_n)
        {
          best_n = int32_t(e - s);
          best = cand[s];
        }
        s = e;
      }
      next[i] = best;
    }
    std::memcpy(agg, next.data(), sizeof(int32_t) * size_t(n));
  }
  // phase 3: leftovers with their free neighbours (singletons if isolated)
  for (int64_t i = 0; i < n; ++i)
  {
    if (skipped(i) || agg[i] >= 0) continue;
    agg[i] = n_agg;
    for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k)
    {
      const int32_t j = adj[k];
      if (!skipped(j) && agg[j] < 0) agg[j] = n_agg;
    }
    ++n_agg;
  }
  return n_agg;
}

// ns: [n][bs][6] near-null space of the fine nodes (rows of Dirichlet DOFs zeroed by the caller);
// agg: aggregate of every node (-1 = none); p_vals: [n][bs][6] tentative blocks (zero for
// unaggregated nodes); ns_coarse: [n_agg][6][6].  *n_deficient: coarse DOFs with a zero column.
int fcg_amg_tentative(int64_t n, int bs, const double* ns, const int32_t* agg, int64_t n_agg,
    double* p_vals, double* ns_coarse, int64_t* n_deficient)
{
  constexpr int NM = 6;
  if (n < 0 || bs < 1 || bs > 6 || n_agg < 0 || (n > 0 && (!ns || !agg || !p_vals)) ||
      (n_agg > 0 && !ns_coarse))
    return FCG_ERR_ARG;
  // nodes of every aggregate in ascending order (counting sort)
  std::vector<int64_t> aptr(size_t(n_agg) + 1, 0);
  for (int64_t i = 0; i < n; ++i)
  {
    if (agg[i] >= n_agg) return FCG_ERR_ARG;
    if (agg[i] >= 0) ++aptr[size_t(agg[i]) + 1];
  }
  for (int64_t a = 0; a < n_agg; ++a) aptr[size_t(a) + 1] += aptr[size_t(a)];
  std::vector<int64_t> fill(aptr.begin(), aptr.end() - 1), nodes(size_t(aptr.back()));
  for (int64_t i = 0; i < n; ++i)
    if (agg[i] >= 0) nodes[size_t(fill[size_t(agg[i])]++)] = i;
  std::memset(p_vals, 0, sizeof(double) * size_t(n) * bs * NM);
  int64_t deficient = 0;
  std::vector<double> Q;
  for (int64_t a = 0; a < n_agg; ++a)
  {
    const int64_t b0 = aptr[size_t(a)], nn = aptr[size_t(a) + 1] - b0;
    const int64_t m = nn * bs;
    Q.assign(size_t(m) * NM, 0.0);  // [row][col]
    for (int64_t t = 0; t < nn; ++t)
      for (int d = 0; d < bs; ++d)
        for (int j = 0; j < NM; ++j)
          Q[size_t((t * bs + d) * NM + j)] = ns[size_t((nodes[size_t(b0 + t)] * bs + d) * NM + j)];
    double R[NM][NM] = {};
    for (int j = 0; j < NM; ++j)
    {
      double n0 = 0.0;
      for (int64_t r = 0; r < m; ++r) n0 += Q[size_t(r * NM + j)] * Q[size_t(r * NM + j)];
      n0 = std::sqrt(n0);
      for (int pass = 0; pass < 2; ++pass)
        for (int k = 0; k < j; ++k)
        {
          double s = 0.0;
          for (int64_t r = 0; r < m; ++r) s += Q[size_t(r * NM + k)] * Q[size_t(r * NM + j)];
          R[k][j] += s;
          for (int64_t r = 0; r < m; ++r) Q[size_t(r * NM + j)] -= s * Q[size_t(r * NM + k)];
        }
      double nr = 0.0;
      for (int64_t r = 0; r < m; ++r) nr += Q[size_t(r * NM + j)] * Q[size_t(r * NM + j)];
      nr = std::sqrt(nr);
      if (!(nr > 1e-10 * n0) || nr == 0.0)
      {
        // the column lies in the span of the earlier ones: R[k][j] (k < j) keeps its projections
        for (int64_t r = 0; r < m; ++r) Q[size_t(r * NM + j)] = 0.0;
        R[j][j] = 0.0;
        ++deficient;
        continue;
      }
      R[j][j] = nr;
      for (int64_t r = 0; r < m; ++r) Q[size_t(r * NM + j)] /= nr;
    }
    for (int64_t t = 0; t < nn; ++t)
      for (int d = 0; d < bs; ++d)
        for (int j = 0; j < NM; ++j)
          p_vals[size_t((nodes[size_t(b0 + t)] * bs + d) * NM + j)] = Q[size_t((t * bs + d) * NM + j)];
    for (int j = 0; j < NM; ++j)
      for (int k = 0; k < NM; ++k) ns_coarse[size_t(a * NM * NM + j * NM + k)] = R[j][k];
  }
  if (n_deficient) *n_deficient = deficient;
  return FCG_OK;
}

// Block pattern of C = A B.  c_col == NULL: count pass, fills c_ptr[0..n_rows] and returns the
// number of blocks; otherwise fills c_col (c_ptr from the count pass).  Returns -1 on bad input.
int64_t fcg_bsr_symbolic(int64_t n_rows, const int64_t* a_ptr, const int32_t* a_col,
    const int64_t* b_ptr, const int32_t* b_col, int64_t n_cols, int64_t* c_ptr, int32_t* c_col)
{
  if (n_rows < 0 || n_cols < 0 || !c_ptr || (n_rows > 0 && (!a_ptr || !a_col || !b_ptr || !b_col)))
    return -1;
  std::vector<int64_t> mark(size_t(n_cols), -1);
  std::vector<int32_t> row;
  if (!c_col) c_ptr[0] = 0;
  for (int64_t i = 0; i < n_rows; ++i)
  {
    row.clear();
    for (int64_t k = a_ptr[i]; k < a_ptr[i + 1]; ++k)
    {
      const int32_t a = a_col[k];
      for (int64_t q = b_ptr[a]; q < b_ptr[a + 1]; ++q)
      {
        const int32_t c = b_col[q];
        if (c < 0 || c >= n_cols) return -1;
        if (mark[size_t(c)] != i)
        {
          mark[size_t(c)] = i;
          row.push_back(c);
        }
      }
    }
    if (!c_col)
    {
      c_ptr[i + 1] = c_ptr[i] + int64_t(row.size());
      continue;
    }
    if (c_ptr[i + 1] - c_ptr[i] != int64_t(row.size())) return -1;
    std::sort(row.begin(), row.end());
    std::copy(row.begin(), row.end(), c_col + c_ptr[i]);
  }
  return c_ptr[n_rows];
}

// Product plan of C = A B on C's pattern: for every block of C, the pairs (A block, B block) whose
// product lands there, in A's row order -- what the searching SpGEMM kernel finds per call, listed
// once.  Count pass (pair_a = NULL): pair_ptr[0..nnzb_c]; fill pass: pair_a / pair_b.  Returns the
// pair count, -1 on bad input (block indices past int32).
int64_t fcg_bsr_product_plan(int64_t n_rows, const int64_t* a_ptr, const int32_t* a_col,
    const int64_t* b_ptr, const int32_t* b_col, const int64_t* c_ptr, const int32_t* c_col,
    int64_t n_cols, int64_t* pair_ptr, int32_t* pair_a, int32_t* pair_b)
{
  if (n_rows < 0 || n_cols < 0 || !pair_ptr || (n_rows > 0 && (!a_ptr || !a_col || !b_ptr || !b_col || !c_ptr)))
    return -1;
  if ((pair_a == nullptr) != (pair_b == nullptr)) return -1;
  const int64_t nnzb_c = n_rows ? c_ptr[n_rows] : 0;
  if ((n_rows && a_ptr[n_rows] > INT32_MAX) || nnzb_c < 0) return -1;
  const bool fill = pair_a != nullptr;
  if (!fill) std::fill(pair_ptr, pair_ptr + nnzb_c + 1, int64_t(0));
  // rows are independent (each C block belongs to one row): threads over row ranges, each with its
  // own column -> C block map
  std::atomic<bool> bad{false};
  auto rows = [&](int64_t r0, int64_t r1) {
    std::vector<int64_t> pos(size_t(n_cols), -1);  // C's block index of column c in the current row
    std::vector<int64_t> cursor;
    for (int64_t i = r0; i < r1 && !bad.load(std::memory_order_relaxed); ++i)
    {
      for (int64_t ci = c_ptr[i]; ci < c_ptr[i + 1]; ++ci)
      {
        if (c_col[ci] < 0 || c_col[ci] >= n_cols)
        {
          bad = true;
          return;
        }
        pos[size_t(c_col[ci])] = ci;
      }
      // (fill pass: a cursor per C block of the row; the count pass checked the indices)
      std::vector<int64_t>& cur = cursor;
      if (fill)
      {
        cur.clear();
        for (int64_t ci = c_ptr[i]; ci < c_ptr[i + 1]; ++ci) cur.push_back(pair_ptr[ci]);
      }
      for (int64_t ak = a_ptr[i]; ak < a_ptr[i + 1]; ++ak)
      {
        const int32_t k = a_col[ak];
        for (int64_t bk = b_ptr[k]; bk < b_ptr[k + 1]; ++bk)
        {
          const int32_t c = b_col[bk];
          if (!fill && (c < 0 || c >= n_cols || bk > INT32_MAX))
          {
            bad = true;
            return;
          }
          const int64_t ci = pos[size_t(c)];
          if (ci < 0) continue;  // a product outside C's pattern is not formed (as the search kernel)
          if (fill)
          {
            const int64_t t = cur[size_t(ci - c_ptr[i])]++;
            pair_a[t] = int32_t(ak);
            pair_b[t] = int32_t(bk);
          }
          else
            ++pair_ptr[ci + 1];
        }
      }
      for (int64_t ci = c_ptr[i]; ci < c_ptr[i + 1]; ++ci) pos[size_t(c_col[ci])] = -1;
    }
  };
  const int64_t nt = std::max<int64_t>(1, std::min<int64_t>({16, int64_t(std::thread::hardware_concurrency()), n_rows / 4096}));
  if (nt == 1)
    rows(0, n_rows);
  else
  {
    std::vector<std::thread> th;
    for (int64_t t = 0; t < nt; ++t) th.emplace_back(rows, n_rows * t / nt, n_rows * (t + 1) / nt);
    for (auto& x : th) x.join();
  }
  if (bad) return -1;
  if (!fill)
    for (int64_t ci = 0; ci < nnzb_c; ++ci) pair_ptr[ci + 1] += pair_ptr[ci];
  return pair_ptr[nnzb_c];
}

// Pattern of A^T (n_cols block rows): t_col ascending per row, perm[t] = A's block index.
int fcg_bsr_transpose_pattern(int64_t n_rows, int64_t n_cols, const int64_t* ptr,
    const int32_t* col, int64_t* t_ptr, int32_t* t_col, int64_t* perm)
{
  if (n_rows < 0 || n_cols < 0 || !t_ptr || (n_rows > 0 && (!ptr || !col)) ||
      (n_rows > 0 && ptr[n_rows] > 0 && (!t_col || !perm)))
    return FCG_ERR_ARG;
  std::fill(t_ptr, t_ptr + n_cols + 1, int64_t(0));
  const int64_t nnz = n_rows ? ptr[n_rows] : 0;
  for (int64_t k = 0; k < nnz; ++k)
  {
    if (col[k] < 0 || col[k] >= n_cols) return FCG_ERR_ARG;
    ++t_ptr[col[k] + 1];
  }
  for (int64_t c = 0; c < n_cols; ++c) t_ptr[c + 1] += t_ptr[c];
  std::vector<int64_t> fill(t_ptr, t_ptr + n_cols);
  for (int64_t i = 0; i < n_rows; ++i)
    for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k)
    {
      const int64_t t = fill[size_t(col[k])]++;
      t_col[t] = int32_t(i);
      perm[t] = k;
    }
  return FCG_OK;
}

}  // extern "C"
