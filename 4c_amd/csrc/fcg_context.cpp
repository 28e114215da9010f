// fcg_context.cpp -- C ABI entry points: context creation (the assembly plan, i.e. this path's
// FillComplete), device-resident and host-pointer evaluate, timing and info.
//
// Plan built here once per pattern (the reference rebuilds nothing either: the stiffness keeps
// its graph, `savegraph=true`, 4C_structure_new_timint_basedataglobalstate.cpp:650-652):
//   * incidences = (column element e, local node a) with node a owned by this rank, grouped by
//     the owned node (ascending row LID) and ordered by element index inside a node -- the order
//     in which the assembly kernel sums, hence bitwise-reproducible results;
//   * for every incidence and every local node b of the element, the position of b's first DOF
//     column inside the row of a -- the stride-3 fast path of SparseMatrix::assemble
//     (4C_linalg_sparsematrix.cpp:497-543) resolved once on the host instead of by a
//     lower_bound per element and row at every Newton iteration.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <array>
#include <climits>
#include <cstdlib>
#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fcg_internal.hpp"
#include "fcg_status.hpp"
#include "fcg_shape.hpp"

namespace {

std::mutex g_err_mutex;
std::string g_create_error;

void set_create_error(const std::string& s)
{
  std::lock_guard<std::mutex> lk(g_err_mutex);
  g_create_error = s;
}

template <class F>
void parallel_for(int64_t n, F f)
{
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (n < 4096) nt = 1;
  std::vector<std::thread> th;
  std::atomic<int64_t> next{0};
  const int64_t chunk = 1024;
  auto body = [&]() {
    for (;;)
    {
      const int64_t s = next.fetch_add(chunk);
      if (s >= n) break;
      const int64_t e = std::min(n, s + chunk);
      for (int64_t i = s; i < e; ++i) f(i);
    }
  };
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(body);
  body();
  for (auto& t : th) t.join();
}

template <class T>
hipError_t upload(T** dst, const T* src, int64_t n, int64_t& bytes)
{
  *dst = nullptr;
  if (n == 0) return hipSuccess;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(dst), sizeof(T) * n);
  if (e != hipSuccess) return e;
  bytes += sizeof(T) * n;
  if (src) return hipMemcpy(*dst, src, sizeof(T) * n, hipMemcpyHostToDevice);
  return hipSuccess;
}

// Structured plan (hex8 row-block sweep kernel).  Verifies the lattice hint against the connectivity:
// every element node must sit at lattice position ijk(e) + offset(a) consistently across
// elements, no two elements/nodes may share a position, and every owned node row must hold
// exactly the DOF triples of its existing lattice neighbours.
struct StructHost {
  int32_t lo[3] = {0, 0, 0}, n[3] = {0, 0, 0};    // owned-node box
  int32_t elo[3] = {0, 0, 0}, en[3] = {0, 0, 0};  // column-element box
  int32_t tiles_x = 0, tiles_y = 0, tiles_z = 0, seg = 0;
  std::vector<int32_t> elem_at, rownode_at;
  std::vector<uint16_t> nbr_pos;
  std::vector<double> lat_x;        // node coordinates on the column-node lattice
  std::vector<int32_t> lat_dof;     // column LID of the node's first DOF, -1 = none
  std::vector<uint32_t> plane_rec;  // [tiles_y][tiles_x][NK][PLANE_REC_WORDS]
  int64_t rows_unordered = 0;       // rows whose lower-plane neighbours are not their first columns
};

const int kOff8[8][3] = {{0, 0, 0}, {1, 0, 0}, {1, 1, 0}, {0, 1, 0}, {0, 0, 1}, {1, 0, 1}, {1, 1, 1},
    {0, 1, 1}};  // hex8 4C node order (4C_io_gridgenerator.cpp:371-379)

// Morton (Z-order) key of a point of the box [lo, hi]: 21 bits per axis, interleaved.  Sorting by
// it puts points that are close in space close in the order (gather plan).
uint64_t morton_key(const double* x, const double* lo, const double* hi)
{
  uint64_t key = 0;
  uint32_t q[3];
  for (int k = 0; k < 3; ++k)
  {
    const double ext = hi[k] - lo[k];
    const double t = ext > 0 ? (x[k] - lo[k]) / ext : 0.0;
    q[k] = uint32_t(std::min(2097151.0, std::max(0.0, t * 2097151.0)));
  }
  for (int b = 20; b >= 0; --b)
    for (int k = 0; k < 3; ++k) key = (key << 1) | ((q[k] >> b) & 1u);
  return key;
}

// Permutation sorting items by their Morton keys (ties by index: deterministic)
std::vector<int64_t> morton_order(const std::vector<uint64_t>& key)
{
  std::vector<int64_t> ord(key.size());
  for (size_t i = 0; i < ord.size(); ++i) ord[i] = int64_t(i);
  std::sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) {
    return key[a] != key[b] ? key[a] < key[b] : a < b;
  });
  return ord;
}

// Lattice positions (ex, ey, ez) of a hex8 mesh whose elements stack like a GridGenerator box,
// found from the connectivity alone (an input-file mesh without the fcg_desc.ele_ijk hint), with
// every element's own local numbering allowed to be any proper rotation of 4C's (mesh generators
// rotate element frames): element 0's local frame fixes the lattice axes; across every shared face
// (matched by sorting the sorted node quadruples) the neighbour's other four nodes sit one step
// along the face normal from their edge partners on the face; then every element must occupy one
// unit cell, with a right-handed local frame.  Returns the cells and the connectivity in 4C's
// local order for those cells (canon, what the row-block sweep reads); false (and why) otherwise
// -- build_structured_plan verifies the result like a given hint.
bool detect_lattice_hex8(const fcg_desc* d, std::vector<int32_t>& ijk, std::vector<int32_t>& canon,
    std::string& why)
{
  const int64_t n = d->n_ele;
  if (d->celltype != FCG_HEX8 || n == 0 || n >= (int64_t(1) << 31) / 6)
  {
    why = "not a hex8 mesh";
    return false;
  }
  // local faces (4C hex8 order) and, per local node, its three edge partners
  static const int kFace[6][4] = {{0, 1, 2, 3}, {4, 5, 6, 7}, {0, 1, 5, 4}, {3, 2, 6, 7},
      {0, 3, 7, 4}, {1, 2, 6, 5}};
  int partner[8][3];
  for (int u = 0; u < 8; ++u)
  {
    int c = 0;
    for (int v = 0; v < 8; ++v)
    {
      int diff = 0;
      for (int k = 0; k < 3; ++k) diff += kOff8[u][k] != kOff8[v][k];
      if (diff == 1) partner[u][c++] = v;
    }
  }
  // faces as sorted node quadruples, bucketed by their smallest node (a counting sort: at most 12
  // faces of a hex8 mesh start at one node), matched inside each bucket
  std::vector<std::array<int32_t, 4>> fv(6 * n);
  parallel_for(n, [&](int64_t e) {
    const int32_t* en = d->ele_nodes + 8 * e;
    for (int f = 0; f < 6; ++f)
    {
      std::array<int32_t, 4>& F = fv[6 * e + f];
      for (int k = 0; k < 4; ++k) F[k] = en[kFace[f][k]];
      std::sort(F.begin(), F.end());
    }
  });
  std::vector<int64_t> boff(d->n_node + 1, 0);
  for (int64_t i = 0; i < 6 * n; ++i) ++boff[fv[i][0] + 1];
  for (int64_t nd = 0; nd < d->n_node; ++nd) boff[nd + 1] += boff[nd];
  std::vector<int32_t> bface(6 * n);
  {
    std::vector<int64_t> fill(boff.begin(), boff.end() - 1);
    for (int64_t i = 0; i < 6 * n; ++i) bface[fill[fv[i][0]]++] = int32_t(i);
  }
  std::vector<int32_t> nbr(6 * n, -1);  // element across local face f of e
  std::atomic<int> shared3{0};
  parallel_for(d->n_node, [&](int64_t nd) {
    for (int64_t i = boff[nd]; i < boff[nd + 1]; ++i)
    {
      const int32_t fi = bface[i];
      int matches = 0;
      for (int64_t j = boff[nd]; j < boff[nd + 1]; ++j)
      {
        const int32_t fj = bface[j];
        if (fj != fi && fv[fj] == fv[fi])
        {
          ++matches;
          nbr[fi] = fj / 6;
        }
      }
      if (matches > 1) shared3 = 1;
    }
  });
  if (shared3)
  {
    why = "a face is shared by more than two elements";
    return false;
  }
  std::vector<std::array<int32_t, 4>>().swap(fv);

  // node positions spread from element 0 (its local frame = the lattice axes)
  const int64_t unset = INT64_MIN;
  std::vector<int64_t> pos(3 * int64_t(d->n_node), unset);
  auto set_pos = [&](int32_t node, const int64_t* p) -> bool {
    int64_t* q = &pos[3 * int64_t(node)];
    if (q[0] == unset)
    {
      q[0] = p[0];
      q[1] = p[1];
      q[2] = p[2];
      return true;
    }
    return q[0] == p[0] && q[1] == p[1] && q[2] == p[2];
  };
  std::vector<uint8_t> done(n, 0);
  {
    const int32_t* en = d->ele_nodes;
    for (int a = 0; a < 8; ++a)
    {
      const int64_t p[3] = {kOff8[a][0], kOff8[a][1], kOff8[a][2]};
      if (!set_pos(en[a], p))
      {
        why = "an element repeats a node";
        return false;
      }
    }
  }
  std::vector<int32_t> stack{0};
  done[0] = 1;
  int64_t seen = 1;
  while (!stack.empty())
  {
    const int32_t e = stack.back();
    stack.pop_back();
    const int32_t* en = d->ele_nodes + 8 * int64_t(e);
    for (int f = 0; f < 6; ++f)
    {
      const int32_t g = nbr[6 * int64_t(e) + f];
      if (g < 0) continue;
      // the face normal (out of e, into g): the coordinate the face's nodes share, away from
      // e's other nodes
      const int32_t* fn = en;
      int axis = -1;
      int64_t sgn = 0;
      const int64_t* p0 = &pos[3 * int64_t(fn[kFace[f][0]])];
      for (int k = 0; k < 3 && axis < 0; ++k)
      {
        bool same = true;
        for (int q = 1; q < 4; ++q) same = same && pos[3 * int64_t(fn[kFace[f][q]]) + k] == p0[k];
        if (same) axis = k;
      }
      if (axis < 0)
      {
        why = "an element is not a lattice cell";
        return false;
      }
      for (int a = 0; a < 8; ++a)
      {
        const int64_t c = pos[3 * int64_t(en[a]) + axis];
        if (c != p0[axis]) sgn = p0[axis] > c ? 1 : -1;
      }
      // g's nodes off the face: one step along the normal from their edge partner on the face
      const int32_t* gn = d->ele_nodes + 8 * int64_t(g);
      const int32_t sh[4] = {en[kFace[f][0]], en[kFace[f][1]], en[kFace[f][2]], en[kFace[f][3]]};
      auto on_face = [&](int32_t node) { return node == sh[0] || node == sh[1] || node == sh[2] || node == sh[3]; };
      int placed = 0;
      for (int u = 0; u < 8; ++u)
      {
        if (!on_face(gn[u])) continue;
        for (int j = 0; j < 3; ++j)
        {
          const int32_t m = gn[partner[u][j]];
          if (on_face(m)) continue;
          int64_t p[3] = {pos[3 * int64_t(gn[u])], pos[3 * int64_t(gn[u]) + 1], pos[3 * int64_t(gn[u]) + 2]};
          p[axis] += sgn;
          if (!set_pos(m, p))
          {
            why = "face neighbours give inconsistent lattice positions";
            return false;
          }
          ++placed;
        }
      }
      if (placed != 4)
      {
        why = "an element is not a lattice cell";
        return false;
      }
      if (!done[g])
      {
        done[g] = 1;
        stack.push_back(g);
        ++seen;
      }
    }
  }
  if (seen != n)
  {
    why = "the elements are not one face-connected block";
    return false;
  }
  // every element one unit cell with a right-handed local frame; cells and 4C-order connectivity
  int64_t mn[3] = {INT64_MAX, INT64_MAX, INT64_MAX};
  for (int64_t nd = 0; nd < d->n_node; ++nd)
    if (pos[3 * nd] != unset)
      for (int k = 0; k < 3; ++k) mn[k] = std::min(mn[k], pos[3 * nd + k]);
  ijk.assign(3 * n, 0);
  canon.assign(8 * n, -1);
  std::atomic<int> bad{0};
  parallel_for(n, [&](int64_t e) {
    const int32_t* en = d->ele_nodes + 8 * e;
    int64_t c[3] = {INT64_MAX, INT64_MAX, INT64_MAX};
    for (int a = 0; a < 8; ++a)
      for (int k = 0; k < 3; ++k) c[k] = std::min(c[k], pos[3 * int64_t(en[a]) + k]);
    int32_t* out = &canon[8 * e];
    for (int a = 0; a < 8; ++a)
    {
      int off[3], slot = -1;
      for (int k = 0; k < 3; ++k) off[k] = int(pos[3 * int64_t(en[a]) + k] - c[k]);
      for (int b = 0; b < 8; ++b)
        if (off[0] == kOff8[b][0] && off[1] == kOff8[b][1] && off[2] == kOff8[b][2]) slot = b;
      if (slot < 0 || out[slot] != -1)
      {
        bad = 1;
        return;
      }
      out[slot] = en[a];
    }
    // handedness of the local frame: local x, y, z axes (nodes 1, 3, 4 from node 0)
    int64_t ax[3][3];
    const int idx[3] = {1, 3, 4};
    for (int q = 0; q < 3; ++q)
      for (int k = 0; k < 3; ++k) ax[q][k] = pos[3 * int64_t(en[idx[q]]) + k] - pos[3 * int64_t(en[0]) + k];
    const int64_t det = ax[0][0] * (ax[1][1] * ax[2][2] - ax[1][2] * ax[2][1]) -
                        ax[0][1] * (ax[1][0] * ax[2][2] - ax[1][2] * ax[2][0]) +
                        ax[0][2] * (ax[1][0] * ax[2][1] - ax[1][1] * ax[2][0]);
    if (det != 1)
    {
      bad = 2;
      return;
    }
    for (int k = 0; k < 3; ++k)
    {
      const int64_t v = c[k] - mn[k];
      if (v >= INT32_MAX)
      {
        bad = 1;
        return;
      }
      ijk[3 * e + k] = int32_t(v);
    }
  });
  if (bad != 0)
  {
    why = bad == 2 ? "an element's local frame is mirrored against the lattice"
                   : "an element is not a lattice cell";
    return false;
  }
  return true;  // uniqueness of positions and nodes: build_structured_plan's checks
}

bool build_structured_plan(const fcg_desc* d, const std::vector<int32_t>& rownodes,
    const std::vector<int32_t>& row0, const int32_t* kcol, int cus, StructHost& P, std::string& why)
{
  if (d->celltype != FCG_HEX8 || !d->ele_ijk)
  {
    why = "no lattice hint, or not hex8";
    return false;
  }
  if (d->n_ele == 0 || rownodes.empty())
  {
    why = "nothing to evaluate";
    return false;
  }
  int64_t mn[3], mx[3];
  for (int k = 0; k < 3; ++k)
  {
    mn[k] = INT32_MAX;
    mx[k] = INT32_MIN;
  }
  for (int64_t e = 0; e < d->n_ele; ++e)
    for (int k = 0; k < 3; ++k)
    {
      mn[k] = std::min<int64_t>(mn[k], d->ele_ijk[3 * e + k]);
      mx[k] = std::max<int64_t>(mx[k], d->ele_ijk[3 * e + k]);
    }
  const int64_t EX = mx[0] - mn[0] + 1, EY = mx[1] - mn[1] + 1, EZ = mx[2] - mn[2] + 1;
  if ((EX + 1) * (EY + 1) * (EZ + 1) > 8 * d->n_ele + 4096)
  {
    why = "element lattice box far larger than the element set";
    return false;
  }
  P.elo[0] = int32_t(mn[0]); P.elo[1] = int32_t(mn[1]); P.elo[2] = int32_t(mn[2]);
  P.en[0] = int32_t(EX); P.en[1] = int32_t(EY); P.en[2] = int32_t(EZ);
  P.elem_at.assign(EX * EY * EZ, -1);
  for (int64_t e = 0; e < d->n_ele; ++e)
  {
    const int64_t idx = ((d->ele_ijk[3 * e + 2] - mn[2]) * EY + (d->ele_ijk[3 * e + 1] - mn[1])) * EX +
                        (d->ele_ijk[3 * e] - mn[0]);
    if (P.elem_at[idx] != -1)
    {
      why = "two elements at one lattice position";
      return false;
    }
    P.elem_at[idx] = int32_t(e);
  }
  // node lattice positions, relative to the element box origin, in [0, E+1)
  const int64_t NXn = EX + 1, NYn = EY + 1, NZn = EZ + 1;
  std::vector<int64_t> npos(d->n_node, -1);
  for (int64_t e = 0; e < d->n_ele; ++e)
  {
    const int64_t ex = d->ele_ijk[3 * e] - mn[0], ey = d->ele_ijk[3 * e + 1] - mn[1],
                  ez = d->ele_ijk[3 * e + 2] - mn[2];
    for (int a = 0; a < 8; ++a)
    {
      const int64_t p = ((ez + kOff8[a][2]) * NYn + ey + kOff8[a][1]) * NXn + ex + kOff8[a][0];
      const int32_t node = d->ele_nodes[8 * e + a];
      if (npos[node] == -1)
        npos[node] = p;
      else if (npos[node] != p)
      {
        why = "connectivity does not match the lattice hint";
        return false;
      }
    }
  }
  std::vector<int32_t> node_at(NXn * NYn * NZn, -1);
  for (int64_t nd = 0; nd < d->n_node; ++nd)
  {
    if (npos[nd] < 0) continue;
    if (node_at[npos[nd]] != -1)
    {
      why = "two nodes at one lattice position";
      return false;
    }
    node_at[npos[nd]] = int32_t(nd);
  }
  // owned-node box
  int64_t lo[3] = {INT64_MAX, INT64_MAX, INT64_MAX}, hi[3] = {-1, -1, -1};
  for (int32_t nd : rownodes)
  {
    if (npos[nd] < 0)
    {
      why = "owned node outside every column element";
      return false;
    }
    const int64_t q[3] = {npos[nd] % NXn, (npos[nd] / NXn) % NYn, npos[nd] / (NXn * NYn)};
    for (int k = 0; k < 3; ++k)
    {
      lo[k] = std::min(lo[k], q[k]);
      hi[k] = std::max(hi[k], q[k]);
    }
  }
  for (int k = 0; k < 3; ++k)
  {
    P.lo[k] = int32_t(lo[k] + mn[k]);  // in the hint's lattice coordinates
    P.n[k] = int32_t(hi[k] - lo[k] + 1);
  }
  P.rownode_at.assign(int64_t(P.n[0]) * P.n[1] * P.n[2], -1);
  for (size_t r = 0; r < rownodes.size(); ++r)
  {
    const int64_t p = npos[rownodes[r]];
    const int64_t q[3] = {p % NXn - lo[0], (p / NXn) % NYn - lo[1], p / (NXn * NYn) - lo[2]};
    P.rownode_at[(q[2] * P.n[1] + q[1]) * P.n[0] + q[0]] = int32_t(r);
  }
  // neighbour column positions per owned node row
  const int64_t nrn = int64_t(rownodes.size());
  P.nbr_pos.assign(nrn * 27, 0xFFFF);
  std::string err;
  std::mutex err_m;
  std::atomic<int64_t> unordered{0};
  parallel_for(nrn, [&](int64_t r) {
    const int64_t p = npos[rownodes[r]];
    const int64_t i = p % NXn, jj = (p / NXn) % NYn, k = p / (NXn * NYn);
    const int64_t s = d->rowptr[row0[r]];
    const int64_t len = d->rowptr[row0[r] + 1] - s;
    const int32_t* cols = d->col_lid + s;
    int count = 0;
    for (int t = 0; t < 27; ++t)
    {
      const int64_t x = i + t % 3 - 1, y = jj + (t / 3) % 3 - 1, z = k + t / 9 - 1;
      if (x < 0 || x >= NXn || y < 0 || y >= NYn || z < 0 || z >= NZn) continue;
      const int32_t m = node_at[(z * NYn + y) * NXn + x];
      if (m < 0) continue;
      // coupled only through an element holding both nodes (meshes with holes: a lattice
      // neighbour across a missing element is no column of the row, and its position stays absent)
      bool coupled = false;
      for (int64_t ez = std::max(k, z) - 1; ez <= std::min(k, z) && !coupled; ++ez)
        for (int64_t ey = std::max(jj, y) - 1; ey <= std::min(jj, y) && !coupled; ++ey)
          for (int64_t ex = std::max(i, x) - 1; ex <= std::min(i, x) && !coupled; ++ex)
            if (ex >= 0 && ey >= 0 && ez >= 0 && ex < EX && ey < EY && ez < EZ &&
                P.elem_at[(ez * EY + ey) * EX + ex] >= 0)
              coupled = true;
      if (!coupled) continue;
      const int32_t c = kcol[m];
      const int32_t* it = std::lower_bound(cols, cols + len, c);
      const int64_t pos = it - cols;
      if (it == cols + len || *it != c || pos + 3 > len || cols[pos + 1] != c + 1 ||
          cols[pos + 2] != c + 2)
      {
        std::lock_guard<std::mutex> lk(err_m);
        err = "row lacks a lattice neighbour's DOF triple";
        return;
      }
      P.nbr_pos[r * 27 + t] = uint16_t(pos);
      ++count;
    }
    if (3 * count != len)
    {
      std::lock_guard<std::mutex> lk(err_m);
      err = "row holds columns beyond the lattice neighbours";
    }
    // lattice order (GridGenerator numbering): the lower plane's triples open the row
    int lo_max = -1, hi_min = 1 << 30;
    for (int t = 0; t < 27; ++t)
    {
      const int q = P.nbr_pos[r * 27 + t];
      if (q == 0xFFFF) continue;
      if (t < 9)
        lo_max = std::max(lo_max, q);
      else
        hi_min = std::min(hi_min, q);
    }
    if (lo_max > hi_min) unordered.fetch_add(1, std::memory_order_relaxed);
  });
  P.rows_unordered = unordered.load();
  if (!err.empty())
  {
    why = err;
    return false;
  }
  // tiles: 4 x 4 node columns, z split into segments.  The workgroups are alike, so the sweep
  // runs in rounds of `slots` resident workgroups (CUs x workgroups per CU: 2 for the linear /
  // TSI sweep, 1 for TotLag, LDS-bound); a segment of s planes costs s + 1 element layers (it
  // starts one layer early).  Pick the segment count with the least rounds x layers -- e.g. 100^3
  // linear on 256 CUs: 3 segments of 34 planes, 2,028 workgroups in 4 full rounds, where a fixed
  // ">= 2,048 workgroups" rule gave 4 segments, 2,704 workgroups and a 28 %-full sixth round.
  P.tiles_x = (P.n[0] + 3) / 4;
  P.tiles_y = (P.n[1] + 3) / 4;
  const int64_t txy = int64_t(P.tiles_x) * P.tiles_y;
  // FCG_SWEEP_WGS_PER_CU: occupancy probes (tools/exp_lib.sh builds with another launch bound)
  const char* wenv = std::getenv("FCG_SWEEP_WGS_PER_CU");
  const int wpc = wenv ? std::max(1, std::atoi(wenv)) : 2;
  const char* tenv = std::getenv("FCG_SWEEP_TOTLAG_WGS_PER_CU");  // the same, TotLag
  const int tpc = tenv ? std::max(1, std::atoi(tenv)) : 1;
  const int64_t slots = int64_t(std::max(1, cus)) * (d->kinematics == FCG_TOTLAG ? tpc : wpc);
  int64_t nseg = 1;
  double best = 0.0;
  for (int64_t k = 1; k <= std::min<int64_t>(P.n[2], 64); ++k)
  {
    const int64_t segk = (P.n[2] + k - 1) / k;
    const int64_t wgs = txy * ((P.n[2] + segk - 1) / segk);
    const double cost = double((wgs + slots - 1) / slots) * double(segk + 1);
    if (k == 1 || cost < best)
    {
      best = cost;
      nseg = k;
    }
  }
  P.seg = int32_t((P.n[2] + nseg - 1) / nseg);
  P.tiles_z = (P.n[2] + P.seg - 1) / P.seg;
  // lattice node tables (coordinates and DOF column LIDs, by lattice position)
  P.lat_x.assign(3 * NXn * NYn * NZn, 0.0);
  P.lat_dof.assign(NXn * NYn * NZn, -1);
  for (int64_t nd = 0; nd < d->n_node; ++nd)
  {
    if (npos[nd] < 0) continue;
    for (int k = 0; k < 3; ++k) P.lat_x[3 * npos[nd] + k] = d->node_x[3 * nd + k];
    P.lat_dof[npos[nd]] = d->node_dof_col[nd];
  }
  // plane records: row bookkeeping of the 16 node columns of every tile, per node plane
  const int64_t W = fcg::PLANE_REC_WORDS;
  P.plane_rec.assign(int64_t(P.tiles_y) * P.tiles_x * P.n[2] * W, 0u);
  parallel_for(int64_t(P.tiles_y) * P.tiles_x * P.n[2], [&](int64_t idx) {
    const int64_t k = idx % P.n[2];
    const int64_t t = idx / P.n[2];
    const int64_t tx = t % P.tiles_x, ty = t / P.tiles_x;
    uint32_t* rec = P.plane_rec.data() + idx * W;
    uint16_t* np = reinterpret_cast<uint16_t*>(rec + 64);
    for (int c = 0; c < 16; ++c)
    {
      const int64_t i = 4 * tx + c % 4, jj = 4 * ty + c / 4;
      int32_t r = -1;
      if (i < P.n[0] && jj < P.n[1]) r = P.rownode_at[(k * P.n[1] + jj) * P.n[0] + i];
      if (r < 0)
      {
        rec[c] = 0xFFFFFFFFu;
        for (int q = 0; q < 27; ++q) np[27 * c + q] = 0xFFFF;
        continue;
      }
      const int64_t base = d->rowptr[row0[r]];
      rec[c] = uint32_t(row0[r]);
      rec[16 + c] = uint32_t(d->rowptr[row0[r] + 1] - base);
      rec[32 + 2 * c] = uint32_t(uint64_t(base) & 0xFFFFFFFFu);
      rec[32 + 2 * c + 1] = uint32_t(uint64_t(base) >> 32);
      for (int q = 0; q < 27; ++q) np[27 * c + q] = P.nbr_pos[r * 27 + q];
    }
  });
  return true;
}

// Colour-ordered direct assembly plan (hex27 on a verified lattice).  Element e at lattice
// position (ex, ey, ez) gets colour (ex & 1) + 2 (ey & 1) + 4 (ez & 1); two elements of one colour
// share no node, so the eight colour launches write disjoint rows.  The elements holding both
// nodes a, b of e form the product over the axes of {e} or {e, e -+ 1} (the latter when a and b
// both lie on e's lower / upper face along that axis); the first of them in colour order is the
// even one along every such axis, or e itself when the odd/even partner does not exist.  Bits of
// ft[e]: 2d = e comes first along axis d for pairs on its lower face, 2d+1 = on its upper face.
// The hint must place every element node at 2 ijk(e) + position(a) consistently (unique nodes
// and positions), which makes lattice neighbours share exactly their face nodes.
struct ColorHost {
  std::vector<int32_t> col_ele;
  std::vector<uint8_t> ft;
  int64_t color_ptr[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  // pencil order (hex27 StVK, fcg_hex27.hip): colour (ey & 1) + 2 (ez & 1); inside a colour the
  // maximal runs of lattice-consecutive elements along x ("pencils"), each walked in x order by
  // one workgroup.  pen_ele: elements by colour, pencil, ex; pen_ptr: pencil ranges in pen_ele;
  // pen_color: pencil range of colour c.  nb[e]: bit (dx+1) + 3 (dy+1) + 9 (dz+1) = lattice
  // neighbour e + (dx, dy, dz) exists; bits 27, 28 = ey & 1, ez & 1.
  std::vector<int32_t> pen_ele;
  std::vector<int64_t> pen_ptr;
  int64_t pen_color[5] = {0, 0, 0, 0, 0};
  std::vector<uint32_t> nb;
};

bool build_colored_plan(const fcg_desc* d, ColorHost& P, std::string& why)
{
  if (d->celltype != FCG_HEX27 || !d->ele_ijk)
  {
    why = "no lattice hint, or not hex27";
    return false;
  }
  if (d->n_ele == 0)
  {
    why = "nothing to evaluate";
    return false;
  }
  int64_t mn[3], mx[3];
  for (int k = 0; k < 3; ++k)
  {
    mn[k] = INT32_MAX;
    mx[k] = INT32_MIN;
  }
  for (int64_t e = 0; e < d->n_ele; ++e)
    for (int k = 0; k < 3; ++k)
    {
      mn[k] = std::min<int64_t>(mn[k], d->ele_ijk[3 * e + k]);
      mx[k] = std::max<int64_t>(mx[k], d->ele_ijk[3 * e + k]);
    }
  const int64_t EX = mx[0] - mn[0] + 1, EY = mx[1] - mn[1] + 1, EZ = mx[2] - mn[2] + 1;
  if (EX * EY * EZ > 8 * d->n_ele + 4096)
  {
    why = "element lattice box far larger than the element set";
    return false;
  }
  std::vector<int32_t> elem_at(EX * EY * EZ, -1);
  for (int64_t e = 0; e < d->n_ele; ++e)
  {
    const int64_t idx = ((d->ele_ijk[3 * e + 2] - mn[2]) * EY + (d->ele_ijk[3 * e + 1] - mn[1])) * EX +
                        (d->ele_ijk[3 * e] - mn[0]);
    if (elem_at[idx] != -1)
    {
      why = "two elements at one lattice position";
      return false;
    }
    elem_at[idx] = int32_t(e);
  }
  // node positions on the (2E+1)^3 lattice of the element box
  const int64_t NXn = 2 * EX + 1, NYn = 2 * EY + 1;
  std::vector<int64_t> npos(d->n_node, -1);
  for (int64_t e = 0; e < d->n_ele; ++e)
  {
    const int64_t ex = d->ele_ijk[3 * e] - mn[0], ey = d->ele_ijk[3 * e + 1] - mn[1],
                  ez = d->ele_ijk[3 * e + 2] - mn[2];
    for (int a = 0; a < 27; ++a)
    {
      const int64_t p = ((2 * ez + fcg::kHex27NodePos[a][2]) * NYn + 2 * ey + fcg::kHex27NodePos[a][1]) *
                            NXn + 2 * ex + fcg::kHex27NodePos[a][0];
      const int32_t node = d->ele_nodes[27 * e + a];
      if (npos[node] == -1)
        npos[node] = p;
      else if (npos[node] != p)
      {
        why = "connectivity does not match the lattice hint";
        return false;
      }
    }
  }
  {
    std::vector<int64_t> sorted;
    sorted.reserve(d->n_node);
    for (int64_t nd = 0; nd < d->n_node; ++nd)
      if (npos[nd] >= 0) sorted.push_back(npos[nd]);
    std::sort(sorted.begin(), sorted.end());
    if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end())
    {
      why = "two nodes at one lattice position";
      return false;
    }
  }
  P.ft.assign(d->n_ele, 0);
  std::vector<int64_t> cnt(8, 0);
  std::vector<uint8_t> color(d->n_ele);
  for (int64_t e = 0; e < d->n_ele; ++e)
  {
    const int64_t c[3] = {d->ele_ijk[3 * e] - mn[0], d->ele_ijk[3 * e + 1] - mn[1],
        d->ele_ijk[3 * e + 2] - mn[2]};
    uint8_t bits = 0, col = 0;
    for (int k = 0; k < 3; ++k)
    {
      const bool even = (d->ele_ijk[3 * e + k] & 1) == 0;
      int64_t lo[3] = {c[0], c[1], c[2]}, hi[3] = {c[0], c[1], c[2]};
      lo[k] -= 1;
      hi[k] += 1;
      auto exists = [&](const int64_t* q) {
        if (q[0] < 0 || q[1] < 0 || q[2] < 0 || q[0] >= EX || q[1] >= EY || q[2] >= EZ) return false;
        return elem_at[(q[2] * EY + q[1]) * EX + q[0]] >= 0;
      };
      if (even || !exists(lo)) bits |= uint8_t(1u << (2 * k));
      if (even || !exists(hi)) bits |= uint8_t(1u << (2 * k + 1));
      if (!even) col |= uint8_t(1u << k);
    }
    P.ft[e] = bits;
    color[e] = col;
    cnt[col]++;
  }
  P.color_ptr[0] = 0;
  for (int c = 0; c < 8; ++c) P.color_ptr[c + 1] = P.color_ptr[c] + cnt[c];
  P.col_ele.resize(d->n_ele);
  std::vector<int64_t> fill(P.color_ptr, P.color_ptr + 8);
  for (int64_t e = 0; e < d->n_ele; ++e) P.col_ele[fill[color[e]]++] = int32_t(e);

  // pencil order: walk the lattice box colour by colour, (ez, ey) rows, x runs
  P.nb.assign(d->n_ele, 0u);
  P.pen_ele.clear();
  P.pen_ele.reserve(d->n_ele);
  P.pen_ptr.assign(1, 0);
  auto at = [&](int64_t x, int64_t y, int64_t z) -> int32_t {
    if (x < 0 || y < 0 || z < 0 || x >= EX || y >= EY || z >= EZ) return -1;
    return elem_at[(z * EY + y) * EX + x];
  };
  for (int c = 0; c < 4; ++c)
  {
    P.pen_color[c] = int64_t(P.pen_ptr.size()) - 1;
    // parity of the absolute lattice index (the same colours on every rank of a box split)
    for (int64_t z = 0; z < EZ; ++z)
    {
      if (((z + mn[2]) & 1) != (c >> 1)) continue;
      for (int64_t y = 0; y < EY; ++y)
      {
        if (((y + mn[1]) & 1) != (c & 1)) continue;
        for (int64_t x = 0; x < EX; ++x)
        {
          const int32_t e = at(x, y, z);
          if (e < 0) continue;
          if (at(x - 1, y, z) < 0 && !P.pen_ele.empty() && int64_t(P.pen_ele.size()) != P.pen_ptr.back())
            P.pen_ptr.push_back(int64_t(P.pen_ele.size()));  // a new run starts
          P.pen_ele.push_back(e);
          uint32_t bits = 0;
          for (int dz = -1; dz <= 1; ++dz)
            for (int dy = -1; dy <= 1; ++dy)
              for (int dx = -1; dx <= 1; ++dx)
                if (at(x + dx, y + dy, z + dz) >= 0) bits |= 1u << ((dx + 1) + 3 * (dy + 1) + 9 * (dz + 1));
          bits |= uint32_t((y + mn[1]) & 1) << 27;
          bits |= uint32_t((z + mn[2]) & 1) << 28;
          P.nb[e] = bits;
        }
      }
    }
    if (int64_t(P.pen_ele.size()) != P.pen_ptr.back()) P.pen_ptr.push_back(int64_t(P.pen_ele.size()));
  }
  P.pen_color[4] = int64_t(P.pen_ptr.size()) - 1;
  return true;
}

// hex27 slab schedule (DeviceMesh::h27_*): elements in slabs of S consecutive elements; a row
// node is assembled after the slab of its last incident element (its completing slab c), and its
// records occupy consecutive ring slots from the moment its first element is evaluated (slab smin)
// until that assembly.  Rows are laid out in the ring in assembly order (by c, then Morton order),
// so a slot is reused by a later row; the smallest ring is the one in which every row's slots were
// last held by rows assembled at least 1 + lag slabs before the row's first writer slab (element
// and assembly launches alternate on one stream: lag 0).
struct H27Ring {
  int64_t nslab = 0, ring = 0;
  std::vector<int64_t> asm_ptr;
  std::vector<int32_t> rows, rslot0, slot;
};

void build_h27_ring(int64_t n_ele, int64_t S, int lag, const std::vector<int64_t>& inc_ptr,
    const std::vector<int32_t>& inc_ele, const std::vector<uint8_t>& inc_a,
    const std::vector<int64_t>& morton, H27Ring& R)
{
  const int64_t nrn = int64_t(inc_ptr.size()) - 1;
  R.nslab = (n_ele + S - 1) / S;
  std::vector<int32_t> smin(nrn, 0), cmax(nrn, 0);
  parallel_for(nrn, [&](int64_t r) {
    int64_t lo = INT64_MAX, hi = 0;
    for (int64_t k = inc_ptr[r]; k < inc_ptr[r + 1]; ++k)
    {
      const int64_t sl = int64_t(inc_ele[k]) / S;
      lo = std::min(lo, sl);
      hi = std::max(hi, sl);
    }
    smin[r] = int32_t(lo == INT64_MAX ? 0 : lo);
    cmax[r] = int32_t(hi);
  });
  // rows by completing slab, Morton order inside a slab (a stable counting sort of the Morton list)
  R.asm_ptr.assign(R.nslab + 1, 0);
  for (int64_t r = 0; r < nrn; ++r) R.asm_ptr[cmax[r] + 1]++;
  for (int64_t c = 0; c < R.nslab; ++c) R.asm_ptr[c + 1] += R.asm_ptr[c];
  R.rows.assign(nrn, 0);
  {
    std::vector<int64_t> fill(R.asm_ptr.begin(), R.asm_ptr.end() - 1);
    for (int64_t i = 0; i < nrn; ++i)
    {
      const int64_t r = morton[i];
      R.rows[fill[cmax[r]]++] = int32_t(r);
    }
  }
  std::vector<int64_t> P(nrn + 1, 0);  // first ring position (unwrapped) of the j-th row
  int64_t maxn = 1;
  for (int64_t j = 0; j < nrn; ++j)
  {
    const int64_t n = inc_ptr[R.rows[j] + 1] - inc_ptr[R.rows[j]];
    P[j + 1] = P[j] + n;
    maxn = std::max(maxn, n);
  }
  const int64_t n_inc = P[nrn];
  // does a ring of `ring` slots keep every row's slots free until its first writer slab?
  auto fits = [&](int64_t ring) {
    int64_t jp = 0;  // the row holding position P[j] + n - 1 - ring, found by a forward scan
    for (int64_t j = 0; j < nrn; ++j)
    {
      const int64_t last = P[j + 1] - 1 - ring;
      if (last < 0) continue;
      while (P[jp + 1] <= last) ++jp;
      if (cmax[R.rows[jp]] > smin[R.rows[j]] - 1 - lag) return false;
    }
    return true;
  };
  int64_t lo = maxn, hi = std::max<int64_t>(maxn, n_inc);
  while (lo < hi)
  {
    const int64_t mid = lo + (hi - lo) / 2;
    if (fits(mid))
      hi = mid;
    else
      lo = mid + 1;
  }
  R.ring = lo;
  R.rslot0.assign(nrn, 0);
  R.slot.assign(size_t(n_ele) * 27, -1);
  for (int64_t j = 0; j < nrn; ++j)
  {
    const int64_t r = R.rows[j];
    R.rslot0[r] = int32_t(P[j] % R.ring);
    for (int64_t k = inc_ptr[r]; k < inc_ptr[r + 1]; ++k)
      R.slot[size_t(inc_ele[k]) * 27 + inc_a[k]] = int32_t((P[j] + (k - inc_ptr[r])) % R.ring);
  }
}

// hex27 overlapped schedule (DeviceMesh::ovl_*, h27_element_kernel<KIN, 3>): the elements in chunks
// of C consecutive elements, the chunks in bands of G; a row node can be assembled once every band
// holding one of its incident elements is complete.  Rows are ordered by their last band (Morton
// order inside a band, as the slab schedule), cut into row items of R rows, and the queue lists
// band b's element chunks followed by the row items of band b - lag: a workgroup that claims a row
// item then rarely finds a band of it still running (the resident workgroups hold about
// `resident` chunks at a time, so lag ~ resident / G + 1 bands).
struct H27Overlap {
  int64_t nchunks = 0, nbands = 0;
  std::vector<int32_t> queue, ritem, rows;
};

void build_h27_overlap(int64_t n_ele, int64_t C, int64_t G, int64_t R, int64_t lag,
    const std::vector<int64_t>& inc_ptr, const std::vector<int32_t>& inc_ele,
    const std::vector<int64_t>& morton, H27Overlap& O)
{
  const int64_t nrn = int64_t(inc_ptr.size()) - 1;
  O.nchunks = (n_ele + C - 1) / C;
  O.nbands = (O.nchunks + G - 1) / G;
  const int64_t B = C * G;  // elements per band
  std::vector<int32_t> blo(nrn, 0), bhi(nrn, 0);
  parallel_for(nrn, [&](int64_t r) {
    int64_t lo = INT64_MAX, hi = 0;
    for (int64_t k = inc_ptr[r]; k < inc_ptr[r + 1]; ++k)
    {
      lo = std::min(lo, int64_t(inc_ele[k]) / B);
      hi = std::max(hi, int64_t(inc_ele[k]) / B);
    }
    blo[r] = int32_t(lo == INT64_MAX ? 0 : lo);
    bhi[r] = int32_t(hi);
  });
  std::vector<int64_t> ptr(O.nbands + 1, 0);
  for (int64_t r = 0; r < nrn; ++r) ptr[bhi[r] + 1]++;
  for (int64_t b = 0; b < O.nbands; ++b) ptr[b + 1] += ptr[b];
  O.rows.assign(nrn, 0);
  {
    std::vector<int64_t> fill(ptr.begin(), ptr.end() - 1);
    for (int64_t i = 0; i < nrn; ++i)
    {
      const int64_t r = morton[i];
      O.rows[fill[bhi[r]]++] = int32_t(r);
    }
  }
  // row items per band
  std::vector<std::vector<int32_t>> items(O.nbands);  // item indices of band b
  for (int64_t b = 0; b < O.nbands; ++b)
    for (int64_t j = ptr[b]; j < ptr[b + 1]; j += R)
    {
      const int64_t j1 = std::min(ptr[b + 1], j + R);
      int32_t lo = int32_t(b);
      for (int64_t jj = j; jj < j1; ++jj) lo = std::min(lo, blo[O.rows[jj]]);
      items[b].push_back(int32_t(O.ritem.size() / 4));
      O.ritem.insert(O.ritem.end(), {int32_t(j), int32_t(j1), lo, int32_t(b)});
    }
  O.queue.reserve(size_t(O.nchunks + O.ritem.size() / 4));
  auto rows_of = [&](int64_t b) {
    for (const int32_t q : items[b]) O.queue.push_back(~q);
  };
  for (int64_t b = 0; b < O.nbands; ++b)
  {
    for (int64_t c = b * G; c < std::min(O.nchunks, (b + 1) * G); ++c) O.queue.push_back(int32_t(c));
    if (b - lag >= 0) rows_of(b - lag);
  }
  for (int64_t b = std::max<int64_t>(0, O.nbands - lag); b < O.nbands; ++b) rows_of(b);
}

void free_mesh(fcg::DeviceMesh& m)
{
  void* ptrs[] = {m.apply_ye, m.apply_dof, m.gather_dummy, m.multi_ptr, m.rec_row0, m.rec_meta, m.rec_base, m.rec_ele, m.rec_a, m.rec_tmap, m.ele_orig, m.inc_ele, m.inc_a, m.asm_order, m.ele_x,
      m.ele_dof, m.ele_nodes, m.ele_gid, m.node_x, m.node_dof_col, m.inc_of, m.inc_ptr,
      m.rownode_row0, m.inc_pos, m.rowptr, m.scratch, m.err, m.elem_at, m.lat_x, m.lat_dof,
      m.plane_rec,
      m.tables, m.stamps, m.col_lid, m.diag_pos, m.pcg_work, m.col_ele, m.ele_ft, m.inc_row0, m.ele_gp,
      m.pen_ptr, m.ele_nb, m.h27_rows, m.h27_rslot0, m.h27_slot, m.ovl_queue, m.ovl_ritem,
      m.ovl_rows, m.ovl_rmeta, m.ovl_sync};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (m.err_host) (void)hipHostFree(m.err_host);
  m = fcg::DeviceMesh{};
}

// The CSR graph of the owned rows from the column elements, built by fcg_graph_build_device (the
// sorted-row graph Epetra_CrsMatrix::FillComplete gives 4C after the first assembly through the
// unfilled path, 4C_linalg_sparsematrix.cpp:578-611, 843-865), columns in the matrix column map
// (kcol), brought back to the host for the plan builders below.
int graph_on_device(const fcg_desc* d, const int32_t* kcol, std::vector<int64_t>& rowptr,
    std::vector<int32_t>& col, std::string& why)
{
  const int npe = d->celltype == FCG_HEX27 ? 27 : 8;
  if (d->n_rows % 3 != 0)
  {
    why = "n_rows must be 3 x owned nodes";
    return FCG_ERR_ARG;
  }
  for (int64_t n = 0; n < d->n_node; ++n)
    if (kcol[n] < 0 || (d->node_dof_row[n] >= 0 && d->node_dof_row[n] % 3 != 0))
    {
      why = "node DOF LIDs must be non-negative and owned rows start at multiples of 3";
      return FCG_ERR_ARG;
    }
  if (!fcg_use_device(d->device))
  {
    why = "hipSetDevice failed";
    return fcg_device_error();
  }
  int32_t *en = nullptr, *dc = nullptr, *dr = nullptr, *cl = nullptr;
  int64_t* rp = nullptr;
  int64_t bytes = 0, nnz = 0;
  hipError_t he = hipSuccess;
  auto chk = [&](hipError_t x) {
    if (he == hipSuccess) he = x;
  };
  chk(upload(&en, d->ele_nodes, d->n_ele * npe, bytes));
  chk(upload(&dc, kcol, d->n_node, bytes));
  chk(upload(&dr, d->node_dof_row, d->n_node, bytes));
  chk(upload<int64_t>(&rp, nullptr, d->n_rows + 1, bytes));
  int rc = FCG_OK;
  if (he == hipSuccess)
    rc = fcg_graph_build_device(d->device, d->celltype, d->n_ele, en, d->n_node, dc, dr, d->n_rows, rp,
        nullptr, 0, &nnz, nullptr);
  if (he == hipSuccess && rc == FCG_OK)
  {
    chk(upload<int32_t>(&cl, nullptr, std::max<int64_t>(nnz, 1), bytes));
    if (he == hipSuccess)
      rc = fcg_graph_build_device(d->device, d->celltype, d->n_ele, en, d->n_node, dc, dr, d->n_rows,
          rp, cl, nnz, &nnz, nullptr);
  }
  if (he == hipSuccess && rc == FCG_OK)
  {
    rowptr.resize(d->n_rows + 1);
    col.resize(nnz);
    chk(hipMemcpy(rowptr.data(), rp, sizeof(int64_t) * rowptr.size(), hipMemcpyDeviceToHost));
    if (nnz > 0) chk(hipMemcpy(col.data(), cl, sizeof(int32_t) * size_t(nnz), hipMemcpyDeviceToHost));
  }
  for (void* p : {static_cast<void*>(en), static_cast<void*>(dc), static_cast<void*>(dr),
           static_cast<void*>(rp), static_cast<void*>(cl)})
    if (p) (void)hipFree(p);
  if (he != hipSuccess)
  {
    why = hipGetErrorString(he);
    return fcg_device_error();
  }
  if (rc != FCG_OK) why = rc == FCG_ERR_ARG ? "row LIDs inconsistent or more than 16 elements at a node"
                                            : "device error";
  return rc;
}

}  // namespace

extern "C" {

const char* fcg_last_error(const fcg_ctx* ctx)
{
  if (ctx) return ctx->last_error.c_str();
  std::lock_guard<std::mutex> lk(g_err_mutex);
  return g_create_error.c_str();
}

int fcg_create(const fcg_desc* d, fcg_ctx** out)
{
  // phase clock (fcg_get_create_phases)
  double ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const auto t_start = std::chrono::steady_clock::now();
  auto t_last = t_start;
  auto phase = [&](int i) {
    const auto now = std::chrono::steady_clock::now();
    ph[i] += std::chrono::duration<double>(now - t_last).count();
    t_last = now;
  };
  if (!d || !out) return FCG_ERR_ARG;
  *out = nullptr;
  if (d->abi_version != FCG_ABI_VERSION)
  {
    set_create_error("abi_version mismatch");
    return FCG_ERR_ARG;
  }
  if ((d->celltype != FCG_HEX8 && d->celltype != FCG_HEX27) ||
      (d->kinematics != FCG_LINEAR && d->kinematics != FCG_TOTLAG))
  {
    set_create_error("unsupported celltype/kinematics");
    return FCG_ERR_ARG;
  }
  // Mat::PAR::StVenantKirchhoff parameter checks (4C_mat_stvenantkirchhoff.cpp:26-28)
  if (!(d->youngs > 0.0) || d->poisson >= 0.5 || d->poisson < -1.0)
  {
    set_create_error("Young's modulus must be > 0 and Poisson's ratio in [-1;0.5)");
    return FCG_ERR_ARG;
  }
  if (d->material != FCG_MAT_STVK && d->material != FCG_MAT_ELASTHYPER_COUPNEOHOOKE)
  {
    set_create_error("unsupported material");
    return FCG_ERR_ARG;
  }
  if (d->material == FCG_MAT_ELASTHYPER_COUPNEOHOOKE && d->kinematics != FCG_TOTLAG)
  {
    set_create_error("ElastHyper is supported with KINEM nonlinear (TotLag) only");
    return FCG_ERR_ARG;
  }
  if (d->material != FCG_MAT_STVK && d->path == FCG_PATH_STRUCTURED && d->celltype == FCG_HEX8)
  {
    set_create_error("the structured sweep implements StVenantKirchhoff only");
    return FCG_ERR_ARG;
  }
  // rowptr = col_lid = NULL: the graph is built here, on the device (FillComplete of the first
  // assembly, see graph_on_device); one of the two alone is an error
  const bool build_graph = d->n_rows > 0 && !d->rowptr && !d->col_lid;
  if (d->n_ele < 0 || d->n_node < 0 || d->n_rows < 0 || d->n_cols < 0 ||
      (d->n_ele > 0 && (!d->ele_nodes || !d->node_x || !d->node_dof_col || !d->node_dof_row)) ||
      (d->n_rows > 0 && !build_graph && (!d->rowptr || !d->col_lid)) || d->n_ele >= (int64_t(1) << 31))
  {
    set_create_error("invalid descriptor arrays/sizes");
    return FCG_ERR_ARG;
  }
  const int npe = d->celltype == FCG_HEX27 ? 27 : 8;
  const int maxrow = npe == 8 ? 81 : 375;
  const int32_t* kcol = d->node_dof_kcol ? d->node_dof_kcol : d->node_dof_col;

  // --- validate connectivity
  for (int64_t i = 0; i < d->n_ele * npe; ++i)
    if (d->ele_nodes[i] < 0 || d->ele_nodes[i] >= d->n_node)
    {
      set_create_error("element references a node outside [0, n_node)");
      return FCG_ERR_ARG;
    }
  for (int64_t n = 0; n < d->n_node; ++n)
  {
    if (d->node_dof_col[n] < 0 || d->node_dof_col[n] + 3 > d->n_cols)
    {
      set_create_error("node_dof_col out of range");
      return FCG_ERR_ARG;
    }
    if (d->node_dof_row[n] >= 0 && d->node_dof_row[n] + 3 > d->n_rows)
    {
      set_create_error("node_dof_row out of range");
      return FCG_ERR_ARG;
    }
  }
  phase(0);
  fcg_desc dg;
  std::vector<int64_t> g_rowptr;
  std::vector<int32_t> g_col;
  if (build_graph)
  {
    std::string why;
    const int rc = graph_on_device(d, kcol, g_rowptr, g_col, why);
    if (rc != FCG_OK)
    {
      set_create_error("graph on the device: " + why);
      return rc;
    }
    dg = *d;
    dg.rowptr = g_rowptr.data();
    dg.col_lid = g_col.data();
    d = &dg;
  }

  phase(1);
  // --- owned row nodes, ascending by row LID
  std::vector<int32_t> rownodes;
  for (int64_t n = 0; n < d->n_node; ++n)
    if (d->node_dof_row[n] >= 0) rownodes.push_back(int32_t(n));
  std::sort(rownodes.begin(), rownodes.end(),
      [&](int32_t a, int32_t b) { return d->node_dof_row[a] < d->node_dof_row[b]; });
  std::vector<int32_t> rn_of_node(d->n_node, -1);
  for (size_t i = 0; i < rownodes.size(); ++i) rn_of_node[rownodes[i]] = int32_t(i);
  const int64_t nrn = int64_t(rownodes.size());

  // --- CSR structure of node rows: 3 consecutive rows with identical column lists
  std::string err;
  std::mutex err_m;
  std::vector<int32_t> row0(nrn);
  int32_t max_rowlen = 0;
  for (int64_t r = 0; r < nrn; ++r)
  {
    row0[r] = d->node_dof_row[rownodes[r]];
    const int64_t s = d->rowptr[row0[r]];
    const int64_t len = d->rowptr[row0[r] + 1] - s;
    max_rowlen = std::max<int32_t>(max_rowlen, int32_t(len));
    if (len > maxrow || d->rowptr[row0[r] + 2] - d->rowptr[row0[r] + 1] != len ||
        d->rowptr[row0[r] + 3] - d->rowptr[row0[r] + 2] != len)
    {
      set_create_error("node rows must have 3 equal-length rows of <= 3*neighbours columns");
      return FCG_ERR_ARG;
    }
  }
  parallel_for(nrn, [&](int64_t r) {
    const int64_t s = d->rowptr[row0[r]];
    const int64_t len = d->rowptr[row0[r] + 1] - s;
    for (int i = 1; i < 3; ++i)
      if (std::memcmp(d->col_lid + s, d->col_lid + s + i * len, sizeof(int32_t) * len) != 0)
      {
        std::lock_guard<std::mutex> lk(err_m);
        err = "the 3 rows of a node must share one column pattern";
      }
  });
  if (!err.empty())
  {
    set_create_error(err);
    return FCG_ERR_ARG;
  }

  phase(2);
  // --- structured (row-block sweep) plan when a verified lattice hint is present
  StructHost sp;
  std::string why;
  bool structured = false;
  if (d->path != FCG_PATH_GENERAL && d->path != FCG_PATH_GATHER && d->material == FCG_MAT_STVK)
  {
    // compute units of the target device (the segment count depends on it; 256 when the device
    // cannot be queried, e.g. plan checks on a host without GPU)
    int cus = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d->device) == hipSuccess && prop.multiProcessorCount > 0)
      cus = prop.multiProcessorCount;
    else
      (void)hipGetLastError();
    // an input-file hex8 mesh without the hint: look for the lattice in the connectivity
    // (FCG_DETECT_LATTICE=0 turns this off)
    static const bool detect = [] {
      const char* e = std::getenv("FCG_DETECT_LATTICE");
      return !(e && e[0] == '0');
    }();
    std::vector<int32_t> found_ijk, found_nodes;
    fcg_desc dl;
    if (!d->ele_ijk && d->celltype == FCG_HEX8 && detect &&
        detect_lattice_hex8(d, found_ijk, found_nodes, why))
    {
      // the sweep reads the cells and the nodes in 4C's local order for them (element frames of
      // an input file may be any rotation of it; K and f do not depend on the local numbering)
      dl = *d;
      dl.ele_ijk = found_ijk.data();
      dl.ele_nodes = found_nodes.data();
      structured = build_structured_plan(&dl, rownodes, row0, kcol, cus, sp, why);
    }
    else if (d->ele_ijk)
      structured = build_structured_plan(d, rownodes, row0, kcol, cus, sp, why);
    else if (why.empty())
      why = "no lattice hint";
    if (!structured && d->path == FCG_PATH_STRUCTURED && d->celltype == FCG_HEX8)
    {
      set_create_error("structured path requested but the lattice hint does not verify: " + why);
      return FCG_ERR_ARG;
    }
  }
  // --- colour-ordered direct assembly (hex27 on a verified lattice, any material)
  ColorHost cp;
  bool colored = false;
  // AUTO keeps hex27 on the general path: it measured faster (hex27 40^3 on one MI355X: 4.2 vs
  // 5.2 ms linear, 4.8 vs 6.6 ms TotLag -- the colour launches write K in 72-byte runs that share
  // cache lines with other colours' runs); the colour-ordered path needs no scratch (1M hex27:
  // 53 GB less device memory) and is taken when requested.
  if ((d->path == FCG_PATH_STRUCTURED || d->path == FCG_PATH_COLORED) && d->celltype == FCG_HEX27)
  {
    colored = build_colored_plan(d, cp, why);
    if (!colored)
    {
      set_create_error("lattice path requested but the lattice hint does not verify: " + why);
      return FCG_ERR_ARG;
    }
  }
  if (d->path == FCG_PATH_COLORED && d->celltype != FCG_HEX27)
  {
    set_create_error("the colour-ordered path is implemented for hex27");
    return FCG_ERR_ARG;
  }
  // --- node-row gather: hex8 StVK meshes without a verified lattice (AUTO), or on request
  if (d->path == FCG_PATH_GATHER && (d->celltype != FCG_HEX8 || d->material != FCG_MAT_STVK))
  {
    set_create_error("the gather path is implemented for hex8 with StVenantKirchhoff");
    return FCG_ERR_ARG;
  }
  bool gather = !structured && d->celltype == FCG_HEX8 && d->material == FCG_MAT_STVK &&
                (d->path == FCG_PATH_GATHER || d->path == FCG_PATH_AUTO);

  phase(3);
  // --- incidences grouped by owned node (general path)
  std::vector<int64_t> inc_ptr(nrn + 1, 0);
  for (int64_t i = 0; i < (structured ? 0 : d->n_ele * npe); ++i)
  {
    const int32_t rn = rn_of_node[d->ele_nodes[i]];
    if (rn >= 0) inc_ptr[rn + 1]++;
  }
  for (int64_t r = 0; r < nrn; ++r) inc_ptr[r + 1] += inc_ptr[r];
  const int64_t n_inc = inc_ptr[nrn];
  if (n_inc >= (int64_t(1) << 31))
  {
    set_create_error("too many incidences for one context (> 2^31)");
    return FCG_ERR_ARG;
  }
  std::vector<int32_t> inc_of(structured ? 0 : d->n_ele * npe, -1);
  std::vector<int32_t> inc_ele(n_inc);
  std::vector<uint8_t> inc_a(n_inc);
  std::vector<int32_t> inc_row0(colored ? n_inc : 0);
  if (!structured)
  {
    std::vector<int64_t> fill(inc_ptr.begin(), inc_ptr.end() - 1);
    for (int64_t e = 0; e < d->n_ele; ++e)
      for (int a = 0; a < npe; ++a)
      {
        const int32_t rn = rn_of_node[d->ele_nodes[e * npe + a]];
        if (rn < 0) continue;
        const int64_t k = fill[rn]++;
        inc_of[e * npe + a] = int32_t(k);
        inc_ele[k] = int32_t(e);
        inc_a[k] = uint8_t(a);
        if (colored) inc_row0[k] = row0[rn];
      }
  }
  phase(4);
  // --- positions of every element node's DOF triple inside the row (stride fast path)
  std::vector<uint16_t> inc_pos(n_inc * npe);
  parallel_for(structured ? 0 : nrn, [&](int64_t r) {
    const int64_t s = d->rowptr[row0[r]];
    const int64_t len = d->rowptr[row0[r] + 1] - s;
    const int32_t* cols = d->col_lid + s;
    for (int64_t k = inc_ptr[r]; k < inc_ptr[r + 1]; ++k)
    {
      const int32_t* en = d->ele_nodes + int64_t(inc_ele[k]) * npe;
      for (int b = 0; b < npe; ++b)
      {
        const int32_t c = kcol[en[b]];
        const int32_t* it = std::lower_bound(cols, cols + len, c);
        const int64_t pos = it - cols;
        if (it == cols + len || *it != c || pos + 3 > len || cols[pos + 1] != c + 1 ||
            cols[pos + 2] != c + 2)
        {
          std::lock_guard<std::mutex> lk(err_m);
          err = "matrix graph lacks an element coupling or a node's DOF columns are not "
                "contiguous (SparseMatrix::assemble stride fast path)";
          return;
        }
        inc_pos[k * npe + b] = uint16_t(pos);
      }
    }
  });
  if (!err.empty())
  {
    set_create_error(err);
    return FCG_ERR_ARG;
  }
  // the gather path addresses a row by node triples (one byte each): every element node's columns
  // must start a triple of the row, which holds when the row is made of node DOF triples only
  if (gather)
    for (int64_t i = 0; i < n_inc * npe && gather; ++i)
      if (inc_pos[i] % 3 != 0) gather = false;
  if (!gather && d->path == FCG_PATH_GATHER)
  {
    set_create_error("gather path: a row holds columns that are not node DOF triples");
    return FCG_ERR_ARG;
  }

  phase(5);
  // --- device
  fcg_ctx* ctx = new fcg_ctx();
  ctx->device = d->device;
  hipError_t he = hipSetDevice(d->device);
  if (he == hipSuccess) he = hipStreamCreateWithFlags(&ctx->stream, hipStreamDefault);  // ordered with the null stream (torch's default)
  if (he != hipSuccess)
  {
    set_create_error(std::string("HIP: ") + hipGetErrorString(he));
    delete ctx;
    return fcg_device_error();
  }
  fcg::upload_constant_tables(d->celltype);
  fcg::DeviceMesh& m = ctx->mesh;
  m.celltype = d->celltype;
  m.kinem = d->kinematics;
  m.npe = npe;
  m.n_ele = d->n_ele;
  m.n_node = d->n_node;
  m.n_rows = d->n_rows;
  m.n_cols = d->n_cols;
  m.nnz = d->n_rows ? d->rowptr[d->n_rows] : 0;
  m.n_rownodes = nrn;
  m.n_inc = n_inc;
  m.max_rowlen = max_rowlen;
  // StVK constants, fill_cmat (4C_mat_stvenantkirchhoff.cpp:123-144)
  const double nu = d->poisson;
  const double mfac = d->youngs / ((1.0 + nu) * (1.0 - 2.0 * nu));
  m.cdiag = mfac * (1.0 - nu);
  m.lambda = mfac * nu;
  m.mu = mfac * 0.5 * (1.0 - 2.0 * nu);
  // Mat::Elastic::PAR::CoupNeoHooke (4C_mat_elast_coupneohooke.cpp): c, beta
  m.material = d->material;
  m.nh_c = d->youngs / (4.0 * (1.0 + nu));
  m.nh_beta = nu / (1.0 - 2.0 * nu);
  std::vector<int32_t> eg;
  if (!d->ele_gid)
  {
    eg.resize(d->n_ele);
    for (int64_t e = 0; e < d->n_ele; ++e) eg[e] = int32_t(e);
  }
  int64_t& bytes = ctx->device_bytes;
  he = hipSuccess;
  auto chk = [&](hipError_t x) {
    if (he == hipSuccess) he = x;
  };
  // arrays of 256 MB and more go through the context's pinned staging chunks (threaded host copy
  // overlapped with the DMA) instead of a pageable hipMemcpy: 1M hex27 moves 18.5 GB of column
  // indices and 1.5 GB of incidence positions here
  auto upload_big = [&](auto** dst, const auto* src, int64_t n) -> hipError_t {
    const int64_t nbytes = n * int64_t(sizeof(**dst));
    if (nbytes < (int64_t(256) << 20)) return upload(dst, src, n, bytes);
    hipError_t e = upload(dst, decltype(src)(nullptr), n, bytes);
    if (e == hipSuccess) e = fcg::staged_copy(ctx->staging, d->device, *dst, src, nbytes, true);
    return e;
  };
  chk(upload_big(&m.ele_nodes, d->ele_nodes, d->n_ele * npe));
  chk(upload(&m.ele_gid, d->ele_gid ? d->ele_gid : eg.data(), d->n_ele, bytes));
  chk(upload(&m.node_x, d->node_x, d->n_node * 3, bytes));
  chk(upload(&m.node_dof_col, d->node_dof_col, d->n_node, bytes));
  chk(upload(&m.rownode_row0, row0.data(), nrn, bytes));
  chk(upload_big(&m.rowptr, d->rowptr, d->n_rows + 1));
  // operator support: column LIDs, diagonal positions (the Dirichlet rows and the Jacobi
  // preconditioner need them) and whether the matrix column map is the row map (single rank)
  {
    std::vector<int64_t> diag(d->n_rows, -1);
    std::atomic<bool> rowcol_ok{3 * int64_t(rownodes.size()) == d->n_rows};  // owned column triple == row triple
    parallel_for(nrn, [&](int64_t r) {
      const int32_t nd = rownodes[r];
      if (kcol[nd] != row0[r]) rowcol_ok.store(false, std::memory_order_relaxed);
      for (int dd = 0; dd < 3; ++dd)
      {
        const int64_t row = row0[r] + dd;
        const int32_t* b = d->col_lid + d->rowptr[row];
        const int32_t* e = d->col_lid + d->rowptr[row + 1];
        const int32_t* it = std::lower_bound(b, e, kcol[nd] + dd);
        if (it != e && *it == kcol[nd] + dd) diag[row] = d->rowptr[row] + (it - b);
      }
    });
    const bool rowcol = rowcol_ok.load();
    m.square_local = rowcol && d->n_rows == d->n_cols;
    m.owned_cols_first = rowcol;
    chk(upload_big(&m.col_lid, d->col_lid, m.nnz));
    chk(upload(&m.diag_pos, diag.data(), d->n_rows, bytes));
  }
  chk(upload<int32_t>(&m.err, nullptr, 3, bytes));
  if (he == hipSuccess) he = hipHostMalloc(reinterpret_cast<void**>(&m.err_host), 2 * sizeof(int32_t),
      hipHostMallocDefault);
  if (structured)
  {
    m.path = FCG_PATH_STRUCTURED;
    m.tiles_x = sp.tiles_x;
    m.tiles_y = sp.tiles_y;
    m.tiles_z = sp.tiles_z;
    m.seg_planes = sp.seg;
    m.I0 = sp.lo[0]; m.J0 = sp.lo[1]; m.K0 = sp.lo[2];
    m.NI = sp.n[0]; m.NJ = sp.n[1]; m.NK = sp.n[2];
    m.EX0 = sp.elo[0]; m.EY0 = sp.elo[1]; m.EZ0 = sp.elo[2];
    m.EX = sp.en[0]; m.EY = sp.en[1]; m.EZ = sp.en[2];
    // rows not in lattice order (input-file numbering): the linear sweep defers each row's
    // lower-plane blocks by one layer (MODE 3; renumbered 1M box: 3.41 -> 2.23 GB written,
    // 1.45 -> 1.30-1.35 ms, profiles/r03/defer/).  TotLag keeps MODE 0: its sweep is bound by the
    // arithmetic at one workgroup per CU, and the extra LDS round trip cost 4-6 % there.
    // FCG_SWEEP_DEFER=0/1 forces the choice (A/B runs, tests)
    {
      const char* de = std::getenv("FCG_SWEEP_DEFER");
      m.sweep_defer = de && de[0] ? de[0] == '1'
                                  : d->kinematics == FCG_LINEAR &&
                                        8 * sp.rows_unordered > int64_t(rownodes.size());
    }
    chk(upload(&m.elem_at, sp.elem_at.data(), int64_t(sp.elem_at.size()), bytes));
    chk(upload(&m.lat_x, sp.lat_x.data(), int64_t(sp.lat_x.size()), bytes));
    chk(upload(&m.lat_dof, sp.lat_dof.data(), int64_t(sp.lat_dof.size()), bytes));
    chk(upload(&m.plane_rec, sp.plane_rec.data(), int64_t(sp.plane_rec.size()), bytes));
    // dN at the GPs [192] | dN at the nodes [192] | weights [8] | GP coordinates [24]
    std::vector<double> tab(8 * 8 * 3 * 2 + 8 + 24);
    double xi[81], w[27], xn[81];
    fcg::gauss_rule(fcg::kHex8, xi, w);
    fcg::node_param_coords(fcg::kHex8, xn);
    for (int g = 0; g < 8; ++g) fcg::shape_deriv(fcg::kHex8, &xi[3 * g], &tab[24 * g]);
    for (int g = 0; g < 8; ++g) fcg::shape_deriv(fcg::kHex8, &xn[3 * g], &tab[192 + 24 * g]);
    for (int g = 0; g < 8; ++g) tab[384 + g] = w[g];
    for (int k = 0; k < 24; ++k) tab[392 + k] = xi[k];
    chk(upload(&m.tables, tab.data(), int64_t(tab.size()), bytes));
    // diagnostics (tools/stamps.py): FCG_STAMPS=1 turns on the per-phase s_memtime counters
    const char* st = std::getenv("FCG_STAMPS");
    if (st && st[0] == '1')
    {
      const unsigned long long zero[16] = {};
      chk(upload(&m.stamps, zero, 16, bytes));
    }
  }
  else if (colored)
  {
    m.path = FCG_PATH_COLORED;
    chk(upload(&m.inc_of, inc_of.data(), d->n_ele * npe, bytes));
    chk(upload(&m.inc_pos, inc_pos.data(), n_inc * npe, bytes));
    chk(upload(&m.inc_row0, inc_row0.data(), n_inc, bytes));
    // hex27 StVK: the matrix-core element kernel in pencil order (4 launches, fcg_hex27.hip);
    // FCG_H27_LEGACY=1 or another material: the eight-colour element_kernel launches
    const char* legacy = std::getenv("FCG_H27_LEGACY");
    m.h27_pencil = d->material == FCG_MAT_STVK && !(legacy && legacy[0] == '1');
    if (m.h27_pencil)
    {
      fcg::upload_h27_tables();
      chk(upload(&m.col_ele, cp.pen_ele.data(), d->n_ele, bytes));
      chk(upload(&m.pen_ptr, cp.pen_ptr.data(), int64_t(cp.pen_ptr.size()), bytes));
      chk(upload(&m.ele_nb, cp.nb.data(), d->n_ele, bytes));
      for (int c = 0; c < 5; ++c) m.pen_color[c] = cp.pen_color[c];
    }
    else
    {
      chk(upload(&m.col_ele, cp.col_ele.data(), d->n_ele, bytes));
      chk(upload(&m.ele_ft, cp.ft.data(), d->n_ele, bytes));
      for (int c = 0; c < 9; ++c) m.color_ptr[c] = cp.color_ptr[c];
    }
  }
  else if (gather)
  {
    m.path = FCG_PATH_GATHER;
    // records of <= 8 incidences per row node (a node without elements keeps one empty record,
    // which zeroes its rows under OVERWRITE): first one record per node with <= 8 elements, in
    // row order, then the records of the other nodes, node by node
    //
    // Locality (input-file meshes carry arbitrary node and element numbers): the records follow
    // the Morton order of their row nodes' coordinates and the element data the Morton order of
    // the element centroids, so that the wavefronts working at the same time, and the records of
    // one XCD's contiguous range, share elements and displacements in L2 instead of re-reading
    // them from HBM (6.7 GB fetched per 1M-hex8 evaluate in random order).
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    for (int64_t n = 0; n < d->n_node; ++n)
      for (int k = 0; k < 3; ++k)
      {
        lo[k] = std::min(lo[k], d->node_x[3 * n + k]);
        hi[k] = std::max(hi[k], d->node_x[3 * n + k]);
      }
    std::vector<uint64_t> nkey(nrn), ekey(d->n_ele);
    parallel_for(nrn, [&](int64_t r) { nkey[r] = morton_key(d->node_x + 3 * int64_t(rownodes[r]), lo, hi); });
    parallel_for(d->n_ele, [&](int64_t e) {
      double c[3] = {0.0, 0.0, 0.0};
      for (int b = 0; b < 8; ++b)
        for (int k = 0; k < 3; ++k) c[k] += 0.125 * d->node_x[3 * int64_t(d->ele_nodes[e * 8 + b]) + k];
      ekey[e] = morton_key(c, lo, hi);
    });
    const std::vector<int64_t> rorder = morton_order(nkey);
    const std::vector<int64_t> eorder = morton_order(ekey);  // storage slot -> element
    std::vector<int32_t> eslot(d->n_ele);                     // element -> storage slot
    for (int64_t i = 0; i < d->n_ele; ++i) eslot[eorder[i]] = int32_t(i);
    std::vector<int64_t> rec_start(nrn), nrec(nrn), multi_ptr(1, 0);
    int64_t n_single = 0;
    for (int64_t i = 0; i < nrn; ++i)
    {
      const int64_t r = rorder[i];
      nrec[r] = std::max<int64_t>(1, (inc_ptr[r + 1] - inc_ptr[r] + 7) / 8);
      if (nrec[r] == 1) rec_start[r] = n_single++;
    }
    for (int64_t i = 0; i < nrn; ++i)
    {
      const int64_t r = rorder[i];
      if (nrec[r] > 1)
      {
        rec_start[r] = n_single + multi_ptr.back();
        multi_ptr.push_back(multi_ptr.back() + nrec[r]);
      }
    }
    for (auto& v : multi_ptr) v += n_single;
    const int64_t n_rec = multi_ptr.back();
    m.n_rec = n_rec;
    m.n_rec_single = n_single;
    m.n_multi = int64_t(multi_ptr.size()) - 1;
    std::vector<int32_t> rec_row0(n_rec), rec_meta(n_rec), rec_ele(n_rec * 8, -1);
    std::vector<int64_t> rec_base(n_rec);
    std::vector<uint8_t> rec_a(n_rec * 8, 0);
    std::vector<uint32_t> rec_tmap(n_rec * 32, 0x88888888u);
    parallel_for(nrn, [&](int64_t r) {
      const int64_t nr = nrec[r];
      for (int64_t i = 0; i < nr; ++i)
      {
        const int64_t R = rec_start[r] + i;
        const int64_t k0 = inc_ptr[r] + 8 * i;
        const int ns = int(std::min<int64_t>(8, std::max<int64_t>(0, inc_ptr[r + 1] - k0)));
        rec_row0[R] = row0[r];
        rec_meta[R] = ns | (i == 0 ? 16 : 0) | (i == nr - 1 ? 32 : 0) |
                      int32_t(d->rowptr[row0[r] + 1] - d->rowptr[row0[r]]) << 8;
        rec_base[R] = d->rowptr[row0[r]];
        // per column triple t of the rows: which element node of slot s lands there (nibble s;
        // 8 = none) -- stage 4 of the kernel sums a triple's blocks in slot (element) order
        for (int s = 0; s < ns; ++s)
        {
          rec_ele[R * 8 + s] = eslot[inc_ele[k0 + s]];
          rec_a[R * 8 + s] = inc_a[k0 + s];
          for (int b = 0; b < 8; ++b)
          {
            uint32_t& w = rec_tmap[R * 32 + inc_pos[(k0 + s) * 8 + b] / 3];
            w = (w & ~(15u << (4 * s))) | (uint32_t(b) << (4 * s));
          }
        }
      }
    });
    std::vector<double> ex(d->n_ele * 24);
    std::vector<int32_t> edof(d->n_ele * 8), eorig(d->n_ele);
    parallel_for(d->n_ele, [&](int64_t i) {
      const int64_t e = eorder[i];
      eorig[i] = int32_t(e);
      for (int b = 0; b < 8; ++b)
      {
        const int32_t nd = d->ele_nodes[e * 8 + b];
        for (int k = 0; k < 3; ++k) ex[i * 24 + 3 * b + k] = d->node_x[3 * int64_t(nd) + k];
        edof[i * 8 + b] = d->node_dof_col[nd];
      }
    });
    chk(upload(&m.ele_orig, eorig.data(), d->n_ele, bytes));
    chk(upload(&m.multi_ptr, multi_ptr.data(), int64_t(multi_ptr.size()), bytes));
    chk(upload(&m.rec_row0, rec_row0.data(), n_rec, bytes));
    chk(upload(&m.rec_meta, rec_meta.data(), n_rec, bytes));
    chk(upload(&m.rec_base, rec_base.data(), n_rec, bytes));
    chk(upload(&m.rec_ele, rec_ele.data(), n_rec * 8, bytes));
    chk(upload(&m.rec_a, rec_a.data(), n_rec * 8, bytes));
    chk(upload(&m.rec_tmap, rec_tmap.data(), n_rec * 32, bytes));
    chk(upload(&m.ele_x, ex.data(), d->n_ele * 24, bytes));
    chk(upload(&m.ele_dof, edof.data(), d->n_ele * 8, bytes));
    chk(upload<double>(&m.gather_dummy, nullptr, 4, bytes));
    // Gauss points of the hex8 stiffness rule: xi, eta, zeta, weight
    std::vector<double> tab(32);
    double xi[81], w[27];
    fcg::gauss_rule(fcg::kHex8, xi, w);
    for (int g = 0; g < 8; ++g)
    {
      for (int k = 0; k < 3; ++k) tab[4 * g + k] = xi[3 * g + k];
      tab[4 * g + 3] = w[g];
    }
    chk(upload(&m.tables, tab.data(), int64_t(tab.size()), bytes));
    // the Gauss points' reference Jacobians, inverted, once for the context's lifetime
    chk(upload<double>(&m.ele_gp, nullptr, d->n_ele * 80, bytes));
    chk(fcg::gather_precompute(m, d->n_ele, ctx->stream));
  }
  else
  {
    m.path = FCG_PATH_GENERAL;
    chk(upload(&m.inc_of, inc_of.data(), d->n_ele * npe, bytes));
    chk(upload(&m.inc_ptr, inc_ptr.data(), nrn + 1, bytes));
    chk(upload_big(&m.inc_pos, inc_pos.data(), n_inc * npe));
    // hex27 StVK: the matrix-core element kernel with symmetric per-element records
    // (fcg_hex27.hip; FCG_H27_LEGACY=1 keeps the incidence-record kernels for A/B runs)
    const char* legacy = std::getenv("FCG_H27_LEGACY");
    m.h27s = npe == 27 && d->material == FCG_MAT_STVK && !(legacy && legacy[0] == '1');
    if (m.h27s)
    {
      fcg::upload_h27_tables();
      chk(upload(&m.inc_ele, inc_ele.data(), n_inc, bytes));
      chk(upload(&m.inc_a, inc_a.data(), n_inc, bytes));
      // assembly order: Morton order of the row nodes' coordinates
      double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
      for (int64_t n = 0; n < d->n_node; ++n)
        for (int k = 0; k < 3; ++k)
        {
          lo[k] = std::min(lo[k], d->node_x[3 * n + k]);
          hi[k] = std::max(hi[k], d->node_x[3 * n + k]);
        }
      std::vector<uint64_t> key(nrn);
      parallel_for(nrn, [&](int64_t r) { key[r] = morton_key(d->node_x + 3 * int64_t(rownodes[r]), lo, hi); });
      const std::vector<int64_t> ord = morton_order(key);
      std::vector<int32_t> ord32(ord.begin(), ord.end());
      chk(upload(&m.asm_order, ord32.data(), nrn, bytes));
      // output: the owned incidences' block rows (assemble27_kernel reads each once, contiguous);
      // FCG_H27_SYMREC=1: one symmetric record per element (blocks a <= b) and h27_assemble_kernel
      const char* sym = std::getenv("FCG_H27_SYMREC");
      m.h27_increc = !(sym && sym[0] == '1');
      // slab schedule of the incidence records (DeviceMesh::h27_*): FCG_H27_SLAB elements per
      // slab (0 = one slab); by default only when one record per incidence would take more than a
      // quarter of the device's memory (1M hex27: 53 GB of 288 GB -> one slab).  Measured at 1M
      // hex27 TotLag: slabs of 5,000 / 10,000 / 20,000 elements keep a ring of 1.18 /
      // 1.24 / 2.30 GB instead of 53 GB, at 64.5 / 59.9 / 56.9 ms per evaluate instead of 51.5 ms
      // (every slab boundary drains the element kernel's two-element pipeline), so that meshes of
      // several million hex27 elements fit one GPU beside their tangent
      const char* sl = std::getenv("FCG_H27_SLAB");
      int64_t S = sl ? std::atoll(sl) : 0;
      int n_cu = 256;
      size_t mem_total = 0;
      {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d->device) == hipSuccess)
        {
          if (prop.multiProcessorCount > 0) n_cu = prop.multiProcessorCount;
          mem_total = prop.totalGlobalMem;
        }
        else
          (void)hipGetLastError();
      }
      const char* eg = std::getenv("FCG_H27_EL_GRID");
      m.h27_el_grid = eg ? std::max(1, std::atoi(eg)) : 2 * n_cu;  // the resident workgroups
      // the full scratch whenever it fits: the slab schedule costs about +25 % per evaluate, so
      // it is taken only when the records plus the caller's K values (and 4 GB of headroom for the
      // vectors and the solver) would not fit the device's free memory now
      const double full = double(n_inc) * double(fcg::record_doubles(npe)) * sizeof(double);
      size_t mem_free = 0, mem_tot2 = 0;
      if (hipMemGetInfo(&mem_free, &mem_tot2) != hipSuccess)
      {
        (void)hipGetLastError();
        mem_free = mem_total;
      }
      const double need = full + double(m.nnz) * sizeof(double) + double(int64_t(4) << 30);
      if (!sl && mem_free > 0 && need > double(mem_free))
        S = std::max<int64_t>(4096, d->n_ele / 200);
      int64_t n_slots = n_inc;
      if (m.h27_increc && S > 0 && S < d->n_ele)
      {
        H27Ring R;
        build_h27_ring(d->n_ele, S, 0, inc_ptr, inc_ele, inc_a, ord, R);
        m.h27_nslab = R.nslab;
        m.h27_slab = S;
        m.h27_ring = R.ring;
        m.h27_asm_ptr = R.asm_ptr;
        n_slots = R.ring;
        chk(upload(&m.h27_rows, R.rows.data(), nrn, bytes));
        chk(upload(&m.h27_rslot0, R.rslot0.data(), nrn, bytes));
        chk(upload(&m.h27_slot, R.slot.data(), d->n_ele * 27, bytes));
      }
      // FCG_H27_OVERLAP=1: the overlapped schedule (element chunks and row items in one launch,
      // DESIGN §7e) with the full scratch.  Bitwise the same K and f, but slower than the two
      // launches (40^3 TotLag 3.80 vs 3.45 ms, profiles/r06/r06_h27_overlap_v3_v4_ab.txt), so
      // not the default.  Knobs for A/B runs: FCG_H27_CHUNK elements per chunk, FCG_H27_BAND
      // chunks per band, FCG_H27_RITEM rows per row item, FCG_H27_LAG bands
      const char* ov = std::getenv("FCG_H27_OVERLAP");
      if (m.h27_increc && m.h27_nslab <= 1 && ov && ov[0] == '1')
      {
        auto knob = [](const char* name, int64_t dflt, int64_t lo = 1) {
          const char* e = std::getenv(name);
          return e ? std::max<int64_t>(lo, std::atoll(e)) : dflt;
        };
        const int64_t C = knob("FCG_H27_CHUNK", 8);
        const int64_t nch = (d->n_ele + C - 1) / C;
        const int64_t G = knob("FCG_H27_BAND", std::max<int64_t>(1, nch / 128));
        const int64_t Rr = knob("FCG_H27_RITEM", 64);
        const int64_t lag = knob("FCG_H27_LAG", 2 * ((m.h27_el_grid + G - 1) / G) + 1, 0);
        H27Overlap O;
        build_h27_overlap(d->n_ele, C, G, Rr, lag, inc_ptr, inc_ele, ord, O);
        m.h27_ovl = true;
        m.ovl_chunk = C;
        m.ovl_nchunks = O.nchunks;
        m.ovl_nbands = O.nbands;
        m.ovl_band_chunks = int(G);
        m.ovl_items = int64_t(O.queue.size());
        chk(upload(&m.ovl_queue, O.queue.data(), m.ovl_items, bytes));
        chk(upload(&m.ovl_ritem, O.ritem.data(), int64_t(O.ritem.size()), bytes));
        chk(upload(&m.ovl_rows, O.rows.data(), nrn, bytes));
        // per row position: {CSR offset of the node's rows, first row, first incidence,
        // row length | incidences << 16} -- one load instead of a chain of three
        std::vector<int64_t> meta(size_t(4) * nrn);
        parallel_for(nrn, [&](int64_t j) {
          const int64_t r = O.rows[j];
          const int64_t base = d->rowptr[row0[r]];
          meta[4 * j + 0] = base;
          meta[4 * j + 1] = row0[r];
          meta[4 * j + 2] = inc_ptr[r];
          meta[4 * j + 3] = (d->rowptr[row0[r] + 1] - base) | ((inc_ptr[r + 1] - inc_ptr[r]) << 16);
        });
        chk(upload(&m.ovl_rmeta, meta.data(), 4 * nrn, bytes));
        chk(upload<unsigned>(&m.ovl_sync, nullptr, 1 + O.nbands, bytes));
      }
      chk(upload<double>(&m.scratch, nullptr,
          m.h27_increc ? n_slots * fcg::record_doubles(npe) : d->n_ele * fcg::kH27RecDoubles, bytes));
    }
    else
      chk(upload<double>(&m.scratch, nullptr, n_inc * fcg::record_doubles(npe), bytes));
  }
  if (!structured)
  {
    // diagnostics: per-phase s_memtime counters of the element kernel (tools/stamps.py)
    const char* st = std::getenv("FCG_STAMPS");
    if (st && st[0] == '1')
    {
      const unsigned long long zero[16] = {};
      chk(upload(&m.stamps, zero, 16, bytes));
    }
  }
  for (auto& ev : ctx->timing.ev) chk(hipEventCreate(&ev));
  if (he != hipSuccess)
  {
    set_create_error(std::string("HIP allocation/copy failed: ") + hipGetErrorString(he));
    fcg_destroy(ctx);
    return fcg_device_error();
  }
  phase(6);
  ph[7] = std::chrono::duration<double>(t_last - t_start).count();
  for (int i = 0; i < 8; ++i) ctx->create_phase_s[i] = ph[i];
  *out = ctx;
  return FCG_OK;
}

int fcg_destroy(fcg_ctx* ctx)
{
  if (!ctx) return FCG_OK;
  (void)hipSetDevice(ctx->device);
  free_mesh(ctx->mesh);
  for (auto& ev : ctx->timing.ev)
    if (ev) (void)hipEventDestroy(ev);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->h_u) (void)hipFree(ctx->h_u);
  if (ctx->h_f) (void)hipFree(ctx->h_f);
  if (ctx->h_k) (void)hipFree(ctx->h_k);
  fcg::staging_free(ctx->staging);
  delete ctx;
  return FCG_OK;
}

}  // extern "C"

namespace {

// The error flags of the evaluates queued since the last check (4C's throws).
int report_error(fcg_ctx* ctx, int32_t* bad_ele_gid)
{
  fcg::DeviceMesh& m = ctx->mesh;
  const int32_t* errv = m.err_host;
  m.err_clean = errv[0] == 0;  // no failing element: err still {0, INT32_MAX}
  if (errv[0] == 0) return FCG_OK;
  int32_t gid = -1;
  if (errv[1] >= 0 && errv[1] < m.n_ele)
    (void)hipMemcpy(&gid, m.ele_gid + errv[1], sizeof(int32_t), hipMemcpyDeviceToHost);
  if (bad_ele_gid) *bad_ele_gid = gid;
  ctx->last_error = errv[0] == FCG_ERR_NODAL_DETJ
                        ? "determinant of jacobian <= 0 at one node of element " + std::to_string(gid)
                        : "singular 3x3 matrix in element " + std::to_string(gid);
  return errv[0];
}

void read_timing(fcg::Timing& T)
{
  if (!T.pending) return;
  T.pending = false;
  float a = 0.f, b = 0.f;
  if (hipEventSynchronize(T.ev[2]) != hipSuccess) return;
  (void)hipEventElapsedTime(&a, T.ev[0], T.ev[1]);
  (void)hipEventElapsedTime(&b, T.ev[1], T.ev[2]);
  T.ms_element = a;
  // fused kernels and the hex27 slab schedule: evaluate + assembly in ms_element
  T.ms_element = T.fused ? a + b : a;
  T.ms_assemble = T.path == FCG_PATH_GENERAL && !T.fused ? b : 0.0;
}

}  // namespace

namespace fcg {

hipError_t staged_copy(HostStaging& st, int device, void* dst, const void* src, int64_t bytes,
    bool to_device)
{
  if (bytes <= 0) return hipSuccess;
  if (st.threads <= 0)
    return hipMemcpy(dst, src, bytes, to_device ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost);
  hipError_t he = hipSuccess;
  if (!st.stream)
  {
    st.chunk = int64_t(32) << 20;  // bytes per chunk
    he = hipStreamCreateWithFlags(&st.stream, hipStreamNonBlocking);
    for (int b = 0; b < 2 && he == hipSuccess; ++b)
    {
      he = hipHostMalloc(reinterpret_cast<void**>(&st.pin[b]), st.chunk);
      if (he == hipSuccess) he = hipEventCreateWithFlags(&st.ev[b], hipEventDisableTiming);
    }
    if (he != hipSuccess) return he;
  }
  (void)device;
  const int64_t n_chunks = (bytes + st.chunk - 1) / st.chunk;
  auto host_copy = [&](char* d, const char* s, int64_t len) {
    const int nt = int(std::min<int64_t>(st.threads, std::max<int64_t>(1, len >> 22)));
    if (nt <= 1)
    {
      std::memcpy(d, s, len);
      return;
    }
    std::vector<std::thread> th;
    const int64_t part = (len + nt - 1) / nt;
    for (int t = 0; t < nt; ++t)
    {
      const int64_t a = t * part, e = std::min(len, a + part);
      if (a < e) th.emplace_back([=]() { std::memcpy(d + a, s + a, e - a); });
    }
    for (auto& x : th) x.join();
  };
  char* D = static_cast<char*>(dst);
  const char* S = static_cast<const char*>(src);
  if (to_device)
  {
    // host copy of chunk i into pin[i % 2] overlaps the DMA of chunk i - 1
    for (int64_t i = 0; i < n_chunks && he == hipSuccess; ++i)
    {
      const int b = int(i & 1);
      const int64_t off = i * st.chunk, len = std::min(st.chunk, bytes - off);
      if (i >= 2) he = hipEventSynchronize(st.ev[b]);  // the DMA that last read pin[b] is done
      if (he != hipSuccess) break;
      host_copy(reinterpret_cast<char*>(st.pin[b]), S + off, len);
      he = hipMemcpyAsync(D + off, st.pin[b], len, hipMemcpyHostToDevice, st.stream);
      if (he == hipSuccess) he = hipEventRecord(st.ev[b], st.stream);
    }
  }
  else
  {
    // DMA of chunk i + 1 overlaps the host copy of chunk i
    auto issue = [&](int64_t i) {
      const int b = int(i & 1);
      const int64_t off = i * st.chunk, len = std::min(st.chunk, bytes - off);
      hipError_t e = hipMemcpyAsync(st.pin[b], S + off, len, hipMemcpyDeviceToHost, st.stream);
      if (e == hipSuccess) e = hipEventRecord(st.ev[b], st.stream);
      return e;
    };
    he = issue(0);
    for (int64_t i = 0; i < n_chunks && he == hipSuccess; ++i)
    {
      const int b = int(i & 1);
      he = hipEventSynchronize(st.ev[b]);
      if (he == hipSuccess && i + 1 < n_chunks) he = issue(i + 1);
      if (he != hipSuccess) break;
      const int64_t off = i * st.chunk, len = std::min(st.chunk, bytes - off);
      host_copy(D + off, reinterpret_cast<const char*>(st.pin[b]), len);
    }
  }
  if (he == hipSuccess) he = hipStreamSynchronize(st.stream);
  return he;
}

void staging_free(HostStaging& st)
{
  for (int b = 0; b < 2; ++b)
  {
    if (st.pin[b]) (void)hipHostFree(st.pin[b]);
    if (st.ev[b]) (void)hipEventDestroy(st.ev[b]);
    st.pin[b] = nullptr;
    st.ev[b] = nullptr;
  }
  if (st.stream) (void)hipStreamDestroy(st.stream);
  st.stream = nullptr;
}

}  // namespace fcg

extern "C" {

int fcg_evaluate_device(fcg_ctx* ctx, int action, int mode, const double* d_u_col,
    double* d_fint_row, double* d_K_vals, void* stream_ptr, int32_t* bad_ele_gid)
{
  if (!ctx) return FCG_ERR_ARG;
  fcg::DeviceMesh& m = ctx->mesh;
  const bool want_k = (action == FCG_CALC_NLNSTIFF);
  if ((action != FCG_CALC_NLNSTIFF && action != FCG_CALC_INTERNALFORCE) ||
      (mode != FCG_ACCUMULATE && mode != FCG_OVERWRITE) ||
      (m.n_ele > 0 && !d_u_col) || (m.n_rows > 0 && !d_fint_row) ||
      (want_k && m.nnz > 0 && !d_K_vals))
  {
    ctx->last_error = "invalid evaluate arguments";
    return FCG_ERR_ARG;
  }
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream_ptr ? static_cast<hipStream_t>(stream_ptr) : ctx->stream;
  const int32_t init[2] = {0, INT32_MAX};
  hipError_t he = hipSuccess;
  // a pending evaluate on another stream must have written its flags first
  if (ctx->pending && ctx->pending_stream != s) he = hipStreamSynchronize(ctx->pending_stream);
  if (he == hipSuccess && !m.err_clean)
  {
    he = hipMemcpyAsync(m.err, init, sizeof(init), hipMemcpyHostToDevice, s);
    m.err_clean = true;  // re-initialised in stream order
  }
  auto& T = ctx->timing;
  if (T.enabled && he == hipSuccess) he = hipEventRecord(T.ev[0], s);
  if (m.path == FCG_PATH_STRUCTURED)
  {
    if (he == hipSuccess)
      he = fcg::launch_sweep_h8(m, d_u_col, want_k, mode == FCG_OVERWRITE, d_K_vals, d_fint_row, s);
    if (T.enabled && he == hipSuccess) he = hipEventRecord(T.ev[1], s);
  }
  else if (m.path == FCG_PATH_COLORED)
  {
    if (he == hipSuccess)
      he = m.h27_pencil ? fcg::launch_h27_pencil(m, d_u_col, want_k, mode == FCG_OVERWRITE, d_K_vals,
                              d_fint_row, s)
                        : fcg::launch_element_colored(m, d_u_col, want_k, mode == FCG_OVERWRITE,
                              d_K_vals, d_fint_row, s);
    if (T.enabled && he == hipSuccess) he = hipEventRecord(T.ev[1], s);
  }
  else if (m.path == FCG_PATH_GATHER)
  {
    if (he == hipSuccess)
      he = fcg::launch_gather_h8(m, d_u_col, want_k, mode == FCG_OVERWRITE, d_K_vals, d_fint_row, s);
    if (T.enabled && he == hipSuccess) he = hipEventRecord(T.ev[1], s);
  }
  else if (m.h27_nslab > 1)
  {
    // hex27 slab schedule: slab s's elements, then the rows whose last element it holds
    for (int64_t sl = 0; sl < m.h27_nslab && he == hipSuccess; ++sl)
    {
      he = fcg::launch_h27_element(m, d_u_col, want_k, s, sl * m.h27_slab,
          std::min(m.n_ele, (sl + 1) * m.h27_slab));
      if (he == hipSuccess)
        he = fcg::launch_assemble27_slab(m, sl, want_k, mode == FCG_OVERWRITE, d_K_vals, d_fint_row, s);
    }
    if (T.enabled && he == hipSuccess) he = hipEventRecord(T.ev[1], s);
  }
  else if (m.h27_ovl)
  {
    // hex27 overlapped schedule: elements and rows in one launch
    if (he == hipSuccess)
      he = fcg::launch_h27_overlap(m, d_u_col, want_k, mode == FCG_OVERWRITE, d_K_vals, d_fint_row, s);
    if (T.enabled && he == hipSuccess) he = hipEventRecord(T.ev[1], s);
  }
  else
  {
    if (he == hipSuccess)
      he = m.h27s ? fcg::launch_h27_element(m, d_u_col, want_k, s)
                  : fcg::launch_element(m, d_u_col, want_k, s);
    if (T.enabled && he == hipSuccess) he = hipEventRecord(T.ev[1], s);
    if (he == hipSuccess)
      he = m.h27s && !m.h27_increc
               ? fcg::launch_h27_assemble(m, want_k, mode == FCG_OVERWRITE, d_K_vals, d_fint_row, s)
               : fcg::launch_assemble(m, want_k, mode == FCG_OVERWRITE, d_K_vals, d_fint_row, s);
  }
  if (T.enabled && he == hipSuccess)
  {
    he = hipEventRecord(T.ev[2], s);
    T.pending = true;
    T.path = m.path;
    T.fused = m.path == FCG_PATH_GENERAL && (m.h27_nslab > 1 || m.h27_ovl);
  }
  // async: the flags stay sticky on the device across queued evaluates and fcg_check_error reads
  // them once (a read-back per evaluate would put a copy between every two evaluates' kernels)
  if (he == hipSuccess && !ctx->async)
    he = hipMemcpyAsync(m.err_host, m.err, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, s);
  if (he == hipSuccess && ctx->async)
  {
    ctx->pending = true;
    ctx->pending_stream = s;
    return FCG_OK;  // fcg_check_error reports what the queued work finds
  }
  if (he == hipSuccess) he = hipStreamSynchronize(s);
  if (he != hipSuccess)
  {
    m.err_clean = false;
    ctx->pending = false;
    ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
    return fcg_device_error();
  }
  ctx->pending = false;
  read_timing(T);
  return report_error(ctx, bad_ele_gid);
}

int fcg_set_async(fcg_ctx* ctx, int enable)
{
  if (!ctx) return FCG_ERR_ARG;
  if (!enable && ctx->pending)
  {
    const int rc = fcg_check_error(ctx, nullptr);
    ctx->async = false;
    return rc;
  }
  ctx->async = enable != 0;
  return FCG_OK;
}

int fcg_check_error(fcg_ctx* ctx, int32_t* bad_ele_gid)
{
  if (!ctx) return FCG_ERR_ARG;
  if (!ctx->pending) return FCG_OK;
  (void)hipSetDevice(ctx->device);
  ctx->pending = false;
  if (hipMemcpyAsync(ctx->mesh.err_host, ctx->mesh.err, 2 * sizeof(int32_t), hipMemcpyDeviceToHost,
          ctx->pending_stream) != hipSuccess ||
      hipStreamSynchronize(ctx->pending_stream) != hipSuccess)
  {
    ctx->mesh.err_clean = false;
    ctx->last_error = "HIP: stream failed";
    return fcg_device_error();
  }
  return report_error(ctx, bad_ele_gid);
}

int fcg_evaluate_host(fcg_ctx* ctx, int action, int mode, const double* u_col, double* fint_row,
    double* K_vals, int32_t* bad_ele_gid)
{
  if (!ctx) return FCG_ERR_ARG;
  fcg::DeviceMesh& m = ctx->mesh;
  const bool want_k = (action == FCG_CALC_NLNSTIFF) && K_vals;
  if ((action != FCG_CALC_NLNSTIFF && action != FCG_CALC_INTERNALFORCE) ||
      (mode != FCG_ACCUMULATE && mode != FCG_OVERWRITE) || (m.n_cols && !u_col) ||
      (m.n_rows && !fint_row))
  {
    ctx->last_error = "invalid evaluate arguments";
    return FCG_ERR_ARG;
  }
  (void)hipSetDevice(ctx->device);
  if (ctx->pending)
  {
    const int rc = fcg_check_error(ctx, bad_ele_gid);
    if (rc != FCG_OK) return rc;
  }
  static const char* thr = std::getenv("FCG_HOST_COPY_THREADS");
  ctx->staging.threads = thr ? std::atoi(thr) : 8;
  hipError_t he = hipSuccess;
  if (!ctx->h_u && m.n_cols) he = hipMalloc(&ctx->h_u, sizeof(double) * m.n_cols);
  if (he == hipSuccess && !ctx->h_f && m.n_rows) he = hipMalloc(&ctx->h_f, sizeof(double) * m.n_rows);
  if (he == hipSuccess && want_k && !ctx->h_k && m.nnz) he = hipMalloc(&ctx->h_k, sizeof(double) * m.nnz);
  const bool acc = mode == FCG_ACCUMULATE;
  if (he == hipSuccess)
    he = fcg::staged_copy(ctx->staging, ctx->device, ctx->h_u, u_col, sizeof(double) * m.n_cols, true);
  if (he == hipSuccess && acc)
    he = fcg::staged_copy(ctx->staging, ctx->device, ctx->h_f, fint_row, sizeof(double) * m.n_rows, true);
  if (he == hipSuccess && acc && want_k)
    he = fcg::staged_copy(ctx->staging, ctx->device, ctx->h_k, K_vals, sizeof(double) * m.nnz, true);
  if (he != hipSuccess)
  {
    ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
    return fcg_device_error();
  }
  const bool was_async = ctx->async;
  ctx->async = false;
  const int rc = fcg_evaluate_device(ctx, want_k ? FCG_CALC_NLNSTIFF : FCG_CALC_INTERNALFORCE, mode,
      ctx->h_u, ctx->h_f, ctx->h_k, nullptr, bad_ele_gid);
  ctx->async = was_async;
  if (rc != FCG_OK) return rc;
  he = fcg::staged_copy(ctx->staging, ctx->device, fint_row, ctx->h_f, sizeof(double) * m.n_rows, false);
  if (he == hipSuccess && want_k)
    he = fcg::staged_copy(ctx->staging, ctx->device, K_vals, ctx->h_k, sizeof(double) * m.nnz, false);
  if (he != hipSuccess)
  {
    ctx->last_error = std::string("HIP: ") + hipGetErrorString(he);
    return fcg_device_error();
  }
  return FCG_OK;
}

int fcg_evaluate(fcg_ctx* ctx, int action, const double* u_col, double* fint_row, double* K_vals,
    int32_t* bad_ele_gid)
{
  return fcg_evaluate_host(ctx, action, FCG_ACCUMULATE, u_col, fint_row, K_vals, bad_ele_gid);
}

int fcg_set_timing(fcg_ctx* ctx, int enable)
{
  if (!ctx) return FCG_ERR_ARG;
  ctx->timing.enabled = enable != 0;
  return FCG_OK;
}

int fcg_get_timing(const fcg_ctx* ctx, double* ms_element, double* ms_assemble)
{
  if (!ctx) return FCG_ERR_ARG;
  read_timing(const_cast<fcg_ctx*>(ctx)->timing);
  if (ms_element) *ms_element = ctx->timing.ms_element;
  if (ms_assemble) *ms_assemble = ctx->timing.ms_assemble;
  return 2;
}

int fcg_get_diagnostics(const fcg_ctx* ctx, uint64_t* out, int n)
{
  if (!ctx || !out || n < 0) return FCG_ERR_ARG;
  const fcg::DeviceMesh& m = ctx->mesh;
  unsigned long long v[16] = {};
  if (m.stamps && hipMemcpy(v, m.stamps, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess)
    return fcg_device_error();
  for (int i = 0; i < n && i < 16; ++i) out[i] = v[i];
  return m.stamps ? 16 : 0;
}

int fcg_get_create_phases(const fcg_ctx* ctx, double* out, int n)
{
  if (!ctx || (!out && n > 0)) return FCG_ERR_ARG;
  for (int i = 0; i < n && i < 8; ++i) out[i] = ctx->create_phase_s[i];
  return 8;
}

int fcg_get_info(const fcg_ctx* ctx, fcg_info* info)
{
  if (!ctx || !info) return FCG_ERR_ARG;
  const fcg::DeviceMesh& m = ctx->mesh;
  info->n_ele = m.n_ele;
  info->n_node = m.n_node;
  info->n_rows = m.n_rows;
  info->n_cols = m.n_cols;
  info->nnz = m.nnz;
  info->n_incidences = m.n_inc;
  info->scratch_bytes = !m.scratch ? 0
                        : m.h27s && !m.h27_increc ? m.n_ele * fcg::kH27RecDoubles * int64_t(sizeof(double))
                        : (m.h27_nslab > 1 ? m.h27_ring : m.n_inc) * fcg::record_doubles(m.npe) *
                              int64_t(sizeof(double));
  info->device_bytes = ctx->device_bytes;
  info->path = m.path;
  info->h27_slabs = m.path == FCG_PATH_GENERAL && m.h27s && m.h27_increc
                        ? int32_t(std::max<int64_t>(1, m.h27_nslab))
                        : 0;
  return FCG_OK;
}

int fcg_get_graph(const fcg_ctx* ctx, int64_t* rowptr, int32_t* col_lid, int64_t col_capacity,
    int64_t* nnz)
{
  if (!ctx || !nnz) return FCG_ERR_ARG;
  const fcg::DeviceMesh& m = ctx->mesh;
  *nnz = m.nnz;
  if (col_lid && col_capacity < m.nnz) return FCG_ERR_ARG;
  if (!fcg_use_device(ctx->device)) return fcg_device_error();
  hipError_t he = hipSuccess;
  if (rowptr && m.n_rows > 0)
    he = hipMemcpy(rowptr, m.rowptr, sizeof(int64_t) * size_t(m.n_rows + 1), hipMemcpyDeviceToHost);
  else if (rowptr)
    rowptr[0] = 0;
  if (he == hipSuccess && col_lid && m.nnz > 0)
    he = hipMemcpy(col_lid, m.col_lid, sizeof(int32_t) * size_t(m.nnz), hipMemcpyDeviceToHost);
  return he == hipSuccess ? FCG_OK : fcg_device_error();
}

int fcg_device_alloc(int device, int64_t bytes, void** d_ptr)
{
  if (!d_ptr || bytes < 0) return FCG_ERR_ARG;
  if (!fcg_use_device(device)) return fcg_device_error();
  return hipMalloc(d_ptr, bytes > 0 ? bytes : 1) == hipSuccess ? FCG_OK : fcg_device_error();
}
int fcg_device_free(void* p) { return hipFree(p) == hipSuccess ? FCG_OK : fcg_device_error(); }
int fcg_memcpy_h2d(void* dst, const void* src, int64_t n)
{
  return hipMemcpy(dst, src, n, hipMemcpyHostToDevice) == hipSuccess ? FCG_OK : fcg_device_error();
}
int fcg_memcpy_d2h(void* dst, const void* src, int64_t n)
{
  return hipMemcpy(dst, src, n, hipMemcpyDeviceToHost) == hipSuccess ? FCG_OK : fcg_device_error();
}
int fcg_memset_device(void* dst, int v, int64_t n)
{
  return hipMemset(dst, v, n) == hipSuccess ? FCG_OK : fcg_device_error();
}

}  // extern "C"
