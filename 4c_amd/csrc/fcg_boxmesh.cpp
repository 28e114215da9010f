// fcg_boxmesh.cpp -- per-rank discretization of a structured box, exactly as a 4C rank would hold
// it after GridGenerator + FillComplete + DofSet::assign_degrees_of_freedom, packaged as an
// fcg_desc.  Used by the benchmark and the tests to build synthetic meshes of any size natively.
//
//   element row map (box split over prime factors of nranks)  4C_io_gridgenerator.cpp:87-153
//   hex8/hex27 lattice node ids, 4C node order                4C_io_gridgenerator.cpp:329-392
//   node coordinates (+ rotation about the box midpoint)      4C_io_gridgenerator.cpp:254-323
//   node ownership: a node shared by several ranks' row elements belongs to the lowest rank
//                   (Rebalance::build_graph's broadcast/erase sweep, 4C_rebalance_graph_based.cpp:171-198)
//   column elements: every element with an owned node        4C_fem_discretization_partition.cpp:510-543
//   DOF gid = 3 * (node gid - min node gid) + d                4C_fem_dofset.cpp:343-351
//   matrix graph: row = owned DOF, columns = DOFs of every node sharing an element, column map
//                 ordered like Epetra's FillComplete (own DOFs first, then remote by owner, gid)
#include <algorithm>
#include <sys/mman.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "fourc_gpu.h"

namespace {

struct Section {
  int32_t lo[3], hi[3];  // element index ranges [lo, hi)
};

bool box_sections(const int32_t* interval, int nproc, std::vector<Section>& out)
{
  std::vector<int> factors;
  int np = nproc;
  for (int fac = 2; fac < np + 1;)
  {
    if (np % fac == 0)
    {
      factors.push_back(fac);
      np /= fac;
    }
    else
      fac++;
  }
  if (np != 1) return false;
  unsigned sub[3] = {1, 1, 1};
  const double di[3] = {double(interval[0]), double(interval[1]), double(interval[2])};
  for (auto f = factors.rbegin(); f != factors.rend(); ++f)
  {
    const double r[3] = {di[0] / sub[0], di[1] / sub[1], di[2] / sub[2]};
    if (r[0] >= r[1] && r[0] >= r[2])
      sub[0] *= *f;
    else if (r[1] >= r[0] && r[1] >= r[2])
      sub[1] *= *f;
    else if (r[2] >= r[0] && r[2] >= r[1])
      sub[2] *= *f;
  }
  out.resize(nproc);
  for (int q = 0; q < nproc; ++q)
  {
    const unsigned sec[3] = {q % sub[0], (q / sub[0]) % sub[1], q / (sub[0] * sub[1])};
    for (int d = 0; d < 3; ++d)
      for (int b = 0; b < 2; ++b)
      {
        long v = lround((sec[d] + b) * di[d] / sub[d]);
        v = std::max(0L, std::min(long(interval[d]), v));
        (b ? out[q].hi : out[q].lo)[d] = int32_t(v);
      }
  }
  return true;
}

uint64_t splitmix64(uint64_t x)
{
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <class F>
void parallel_for(int64_t n, F f)
{
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (n < 4096) nt = 1;
  std::atomic<int64_t> next{0};
  auto body = [&]() {
    for (;;)
    {
      const int64_t s = next.fetch_add(1024);
      if (s >= n) break;
      for (int64_t i = s; i < std::min(n, s + 1024); ++i) f(i);
    }
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(body);
  body();
  for (auto& t : th) t.join();
}

// std::vector without value-initialisation (the CSR arrays are written in full right after
// their allocation: no serial zero-fill of 18.5 GB of column indices at 1M hex27)
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = DefaultInitAlloc<U>;
  };
  using std::allocator<T>::allocator;
  // large arrays on transparent huge pages where the kernel offers them (madvise mode): the
  // first-touch page faults of 18.5 GB of column indices dominate the graph fill otherwise
  T* allocate(std::size_t n)
  {
    const std::size_t bytes = n * sizeof(T);
    if (bytes < (std::size_t(64) << 20)) return std::allocator<T>::allocate(n);
    constexpr std::size_t kHuge = std::size_t(2) << 20;
    void* p = std::aligned_alloc(kHuge, (bytes + kHuge - 1) / kHuge * kHuge);
    if (!p) throw std::bad_alloc();
    (void)madvise(p, bytes, MADV_HUGEPAGE);
    return static_cast<T*>(p);
  }
  void deallocate(T* p, std::size_t n)
  {
    if (n * sizeof(T) < (std::size_t(64) << 20))
      std::allocator<T>::deallocate(p, n);
    else
      std::free(p);
  }
  template <class U>
  void construct(U* p) noexcept
  {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a)
  {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};
template <class T>
using RawVec = std::vector<T, DefaultInitAlloc<T>>;

}  // namespace

struct fcg_box_mesh {
  fcg_box box;
  int rank = 0, nranks = 1, npe = 8;
  int64_t n_ele_global = 0, n_ele_row = 0, n_owned_rows = 0;
  int flags = 0;
  std::vector<int32_t> ele_nodes, ele_gid, ele_ijk;
  std::vector<double> node_x;
  std::vector<int64_t> node_gid;
  std::vector<int32_t> node_owner, node_dof_col, node_dof_row;
  std::vector<int32_t> row_gid, col_gid;
  RawVec<int64_t> rowptr;
  RawVec<int32_t> col_lid;
};

extern "C" {

int fcg_box_mesh_create(const fcg_box* box, int rank, int nranks, fcg_box_mesh** out)
{
  return fcg_box_mesh_create_ex(box, rank, nranks, FCG_BOX_GHOSTED, out);
}

int fcg_box_mesh_create_ex(const fcg_box* box, int rank, int nranks, int flags, fcg_box_mesh** out)
{
  if (flags != FCG_BOX_GHOSTED && flags != FCG_BOX_STRICT) return FCG_ERR_ARG;
  const bool strict = flags == FCG_BOX_STRICT;
  if (!box || !out || nranks < 1 || rank < 0 || rank >= nranks) return FCG_ERR_ARG;
  *out = nullptr;
  for (int d = 0; d < 3; ++d)
    if (box->interval[d] <= 0 || !(box->lower[d] < box->upper[d])) return FCG_ERR_ARG;
  if (box->celltype != FCG_HEX8 && box->celltype != FCG_HEX27) return FCG_ERR_ARG;
  std::vector<Section> secs;
  if (!box_sections(box->interval, nranks, secs)) return FCG_ERR_ARG;

  const bool tmr = std::getenv("FCG_BOX_TIMING") != nullptr;
  auto t_prev = std::chrono::steady_clock::now();
  auto tick = [&](const char* what) {
    if (!tmr) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "box %-12s %.3f s\n", what, std::chrono::duration<double>(now - t_prev).count());
    t_prev = now;
  };
  auto* m = new fcg_box_mesh();
  m->box = *box;
  m->rank = rank;
  m->nranks = nranks;
  m->flags = flags;
  const bool h27 = box->celltype == FCG_HEX27;
  const int npe = h27 ? 27 : 8;
  m->npe = npe;
  const int64_t IX = box->interval[0], IY = box->interval[1], IZ = box->interval[2];
  const int64_t NX = 2 * IX + 1, NY = 2 * IY + 1, NZ = 2 * IZ + 1;
  m->n_ele_global = IX * IY * IZ;
  const Section& my = secs[rank];
  m->n_ele_row = int64_t(my.hi[0] - my.lo[0]) * (my.hi[1] - my.lo[1]) * (my.hi[2] - my.lo[2]);

  // lowest rank whose closed lattice box holds the node
  auto owner_of = [&](int64_t i, int64_t j, int64_t k) -> int {
    for (int q = 0; q < nranks; ++q)
    {
      const Section& s = secs[q];
      if (s.hi[0] <= s.lo[0] || s.hi[1] <= s.lo[1] || s.hi[2] <= s.lo[2]) continue;
      if (i >= 2 * s.lo[0] && i <= 2 * s.hi[0] && j >= 2 * s.lo[1] && j <= 2 * s.hi[1] &&
          k >= 2 * s.lo[2] && k <= 2 * s.hi[2])
        return q;
    }
    return -1;
  };
  // create_hex_element node lattice positions (4C_io_gridgenerator.cpp:348-380), as offsets
  static const int off27[27][3] = {{0, 0, 0}, {2, 0, 0}, {2, 2, 0}, {0, 2, 0}, {0, 0, 2},
      {2, 0, 2}, {2, 2, 2}, {0, 2, 2}, {1, 0, 0}, {2, 1, 0}, {1, 2, 0}, {0, 1, 0}, {0, 0, 1},
      {2, 0, 1}, {2, 2, 1}, {0, 2, 1}, {1, 0, 2}, {2, 1, 2}, {1, 2, 2}, {0, 1, 2}, {1, 1, 0},
      {1, 0, 1}, {2, 1, 1}, {1, 2, 1}, {0, 1, 1}, {1, 1, 2}, {1, 1, 1}};

  // column elements: candidates in the section grown by one layer (strict: the section itself)
  int64_t clo[3], chi[3];
  for (int d = 0; d < 3; ++d)
  {
    clo[d] = strict ? my.lo[d] : std::max<int64_t>(0, my.lo[d] - 1);
    chi[d] = strict ? my.hi[d] : std::min<int64_t>(box->interval[d], my.hi[d] + 1);
  }
  const int64_t cex = std::max<int64_t>(0, chi[0] - clo[0]), cey = std::max<int64_t>(0, chi[1] - clo[1]),
                cez = std::max<int64_t>(0, chi[2] - clo[2]);
  std::vector<uint8_t> has(cex * cey * cez, strict ? 1 : 0);
  if (!strict)
    parallel_for(cex * cey * cez, [&](int64_t c) {
      const int64_t ex = clo[0] + c % cex, ey = clo[1] + (c / cex) % cey, ez = clo[2] + c / (cex * cey);
      bool h = false;
      for (int a = 0; a < npe && !h; ++a)
        h = owner_of(2 * ex + off27[a][0], 2 * ey + off27[a][1], 2 * ez + off27[a][2]) == rank;
      has[c] = h ? 1 : 0;
    });
  std::vector<int64_t> col_ele;
  for (int64_t c = 0; c < cex * cey * cez; ++c)
    if (has[c])
    {
      const int64_t ex = clo[0] + c % cex, ey = clo[1] + (c / cex) % cey, ez = clo[2] + c / (cex * cey);
      col_ele.push_back((ez * IY + ey) * IX + ex);
    }
  const int64_t nce = int64_t(col_ele.size());
  tick("elements");

  // column nodes: the lattice nodes of the column elements, marked in the node box of the grown
  // section and enumerated in lattice (GID) order
  // (a rank without column elements -- more ranks than element layers -- has an empty node box)
  const int64_t bx = nce > 0 ? 2 * cex + 1 : 0, by = nce > 0 ? 2 * cey + 1 : 0, bz = nce > 0 ? 2 * cez + 1 : 0;
  const int64_t bn = bx * by * bz;
  std::vector<uint8_t> used(bn, 0);
  auto box_of = [&](int64_t e, int a) -> int64_t {
    const int64_t ex = e % IX, ey = (e / IX) % IY, ez = e / (IX * IY);
    return ((2 * (ez - clo[2]) + off27[a][2]) * by + 2 * (ey - clo[1]) + off27[a][1]) * bx +
           2 * (ex - clo[0]) + off27[a][0];
  };
  // distinct elements may mark the same node: relaxed byte stores of the same value
  parallel_for(nce, [&](int64_t i) {
    for (int a = 0; a < npe; ++a)
      reinterpret_cast<std::atomic<uint8_t>*>(used.data())[box_of(col_ele[i], a)].store(1, std::memory_order_relaxed);
  });
  std::vector<int64_t> plane_cnt(bz + 1, 0);
  parallel_for(bz, [&](int64_t k) {
    int64_t c = 0;
    for (int64_t q = k * bx * by; q < (k + 1) * bx * by; ++q) c += used[q];
    plane_cnt[k + 1] = c;
  });
  for (int64_t k = 0; k < bz; ++k) plane_cnt[k + 1] += plane_cnt[k];
  const int64_t ncn = plane_cnt[bz];
  std::vector<int64_t> uniq(ncn);   // lattice linear index of every column node, ascending
  std::vector<int32_t> slot(bn, -1);  // node box position -> index into uniq
  parallel_for(bz, [&](int64_t k) {
    int64_t w = plane_cnt[k];
    for (int64_t q = k * bx * by; q < (k + 1) * bx * by; ++q)
      if (used[q])
      {
        const int64_t i = q % bx, j = (q / bx) % by;
        uniq[w] = ((2 * clo[2] + k) * NY + 2 * clo[1] + j) * NX + 2 * clo[0] + i;
        slot[q] = int32_t(w++);
      }
  });
  tick("nodes");
  std::vector<int32_t> own(ncn);
  parallel_for(ncn, [&](int64_t n) {
    const int64_t L = uniq[n];
    own[n] = owner_of(L % NX, (L / NX) % NY, L / (NX * NY));
  });
  // order: owned by gid, then ghosts by (owner, gid)  (Epetra column-map order): a stable
  // counting sort by owner class of the gid-ordered nodes
  std::vector<int64_t> cls_ptr(nranks + 2, 0);
  for (int64_t n = 0; n < ncn; ++n) cls_ptr[(own[n] == rank ? 0 : own[n] + 1) + 1]++;
  for (int q = 0; q <= nranks; ++q) cls_ptr[q + 1] += cls_ptr[q];
  std::vector<int64_t> order(ncn);
  std::vector<int32_t> newid(ncn);
  {
    std::vector<int64_t> fill(cls_ptr.begin(), cls_ptr.end() - 1);
    for (int64_t n = 0; n < ncn; ++n)
    {
      const int64_t i = fill[own[n] == rank ? 0 : own[n] + 1]++;
      order[i] = n;
      newid[n] = int32_t(i);
    }
  }

  m->node_gid.resize(ncn);
  m->node_owner.resize(ncn);
  m->node_x.resize(3 * ncn);
  m->node_dof_col.resize(ncn);
  m->node_dof_row.resize(ncn, -1);
  const int64_t n_owned = cls_ptr[1];
  parallel_for(ncn, [&](int64_t i) {
    const int64_t n = order[i];
    const int64_t L = uniq[n];
    m->node_gid[i] = box->first_node_gid + L;
    m->node_owner[i] = own[n];
    m->node_dof_col[i] = int32_t(3 * i);
    if (own[n] == rank) m->node_dof_row[i] = int32_t(3 * i);  // owned nodes come first, in gid order
    else if (strict) m->node_dof_row[i] = int32_t(3 * i);  // extended row (owned nodes come first)
    // coordinates (4C_io_gridgenerator.cpp:283-317)
    const int64_t ii = L % NX, jj = (L / NX) % NY, kk = L / (NX * NY);
    const int64_t lidx[3] = {ii, jj, kk};
    double c[3];
    for (int d = 0; d < 3; ++d)
      c[d] = double(lidx[d]) / (2 * box->interval[d]) * (box->upper[d] - box->lower[d]) + box->lower[d];
    if (box->jitter != 0.0 && ii > 0 && ii < NX - 1 && jj > 0 && jj < NY - 1 && kk > 0 && kk < NZ - 1)
    {
      for (int d = 0; d < 3; ++d)
      {
        const uint64_t z = splitmix64(box->jitter_seed + 3 * uint64_t(L) + d);
        const double u01 = double(z >> 11) * (1.0 / 9007199254740992.0);
        const double h = (box->upper[d] - box->lower[d]) / box->interval[d];
        c[d] += box->jitter * h * (2.0 * u01 - 1.0);
      }
    }
    double cm[3] = {0, 0, 0};
    if (box->rotation[0] != 0.0 || box->rotation[1] != 0.0 || box->rotation[2] != 0.0)
      for (int d = 0; d < 3; ++d) cm[d] = (box->upper[d] + box->lower[d]) / 2.;
    for (int ax = 0; ax < 3; ++ax)
    {
      if (box->rotation[ax] == 0.0) continue;
      double dx[3] = {c[0] - cm[0], c[1] - cm[1], c[2] - cm[2]};
      const double ca = std::cos(box->rotation[ax] * M_PI / 180), sa = std::sin(box->rotation[ax] * M_PI / 180);
      c[0] = cm[0];
      c[1] = cm[1];
      c[2] = cm[2];
      c[(ax + 1) % 3] += ca * dx[(ax + 1) % 3] + sa * dx[(ax + 2) % 3];
      c[(ax + 2) % 3] += ca * dx[(ax + 2) % 3] - sa * dx[(ax + 1) % 3];
      c[ax] += dx[ax];
    }
    for (int d = 0; d < 3; ++d) m->node_x[3 * i + d] = c[d];
  });
  tick("node data");
  // element connectivity in local column-node ids
  m->ele_nodes.resize(nce * npe);
  m->ele_gid.resize(nce);
  m->ele_ijk.resize(3 * nce);
  parallel_for(nce, [&](int64_t e) {
    // lattice position of the element (4C_io_gridgenerator.cpp:336-338)
    m->ele_ijk[3 * e + 0] = int32_t(col_ele[e] % IX);
    m->ele_ijk[3 * e + 1] = int32_t((col_ele[e] / IX) % IY);
    m->ele_ijk[3 * e + 2] = int32_t(col_ele[e] / (IX * IY));
    m->ele_gid[e] = int32_t(col_ele[e]);
    for (int a = 0; a < npe; ++a) m->ele_nodes[e * npe + a] = newid[slot[box_of(col_ele[e], a)]];
  });
  m->n_owned_rows = 3 * n_owned;
  // rows: the owned nodes, plus (strict) the extended rows of every other touched node
  const int64_t n_rn = strict ? ncn : n_owned;
  // dof gids of the maps
  m->row_gid.resize(3 * n_rn);
  m->col_gid.resize(3 * ncn);
  parallel_for(ncn, [&](int64_t i) {
    const int64_t dof0 = 3 * (m->node_gid[i] - box->first_node_gid);
    for (int d = 0; d < 3; ++d) m->col_gid[3 * i + d] = int32_t(dof0 + d);
    if (m->node_dof_row[i] >= 0)
      for (int d = 0; d < 3; ++d) m->row_gid[m->node_dof_row[i] + d] = int32_t(dof0 + d);
  });
  tick("connectivity");
  // graph (the FillComplete'd Epetra graph of the owned / extended rows): the column elements
  // holding a row node are the elements of the candidate box whose node box holds the node's
  // lattice position -- a box of elements per node, all of them column elements (a row node is
  // owned, so every element touching it is a column element; strict: the section's elements),
  // and the node's neighbours are the lattice nodes of those elements' node boxes (hex8: the
  // even positions, its corners).  Rows list them in column-LID order; with ghosts the LIDs are
  // not in lattice order and each list is sorted.
  std::vector<int64_t> pos_of(ncn);  // node box position of uniq index w
  parallel_for(bn, [&](int64_t q) {
    if (slot[q] >= 0) pos_of[slot[q]] = q;
  });
  const bool sorted_lids = ncn == n_owned;  // no ghosts: column LIDs follow the lattice order
  const int step = h27 ? 1 : 2;
  // neighbour LIDs of row node n into nbr (returns the count), the candidate element box checked
  auto neighbours = [&](int64_t n, int32_t* nbr) -> int {
    const int64_t q = pos_of[order[n]];
    const int64_t p[3] = {q % bx, (q / bx) % by, q / (bx * by)};
    const int64_t ce[3] = {cex, cey, cez};
    int64_t lo[3], hi[3];
    for (int d = 0; d < 3; ++d)
    {
      const int64_t elo = std::max<int64_t>(0, (p[d] - 1) / 2), ehi = std::min<int64_t>(ce[d] - 1, p[d] / 2);
      lo[d] = 2 * elo;
      hi[d] = 2 * ehi + 2;
    }
    int c = 0;
    for (int64_t k = lo[2]; k <= hi[2]; k += step)
      for (int64_t j = lo[1]; j <= hi[1]; j += step)
        for (int64_t i = lo[0]; i <= hi[0]; i += step)
          nbr[c++] = newid[slot[(k * by + j) * bx + i]];
    if (!sorted_lids) std::sort(nbr, nbr + c);
    return c;
  };
  // every element of a row node's element box must be a column element (else the lattice rule
  // above does not describe the graph)
  std::atomic<bool> box_ok{true};
  std::vector<int32_t> nnb(n_rn);
  parallel_for(n_rn, [&](int64_t n) {
    const int64_t q = pos_of[order[n]];
    const int64_t p[3] = {q % bx, (q / bx) % by, q / (bx * by)};
    const int64_t ce[3] = {cex, cey, cez};
    int64_t elo[3], ehi[3], cnt = 1;
    for (int d = 0; d < 3; ++d)
    {
      elo[d] = std::max<int64_t>(0, (p[d] - 1) / 2);
      ehi[d] = std::min<int64_t>(ce[d] - 1, p[d] / 2);
      cnt *= (2 * (ehi[d] - elo[d]) + 2) / step + 1;
    }
    for (int64_t ez = elo[2]; ez <= ehi[2]; ++ez)
      for (int64_t ey = elo[1]; ey <= ehi[1]; ++ey)
        for (int64_t ex = elo[0]; ex <= ehi[0]; ++ex)
          if (!has[(ez * cey + ey) * cex + ex]) box_ok.store(false, std::memory_order_relaxed);
    nnb[n] = int32_t(cnt);
  });
  if (!box_ok.load())
  {
    delete m;
    return FCG_ERR_ARG;  // not reached for GridGenerator sections
  }
  tick("neighbours");
  m->rowptr.resize(3 * n_rn + 1);
  m->rowptr[0] = 0;
  for (int64_t n = 0; n < n_rn; ++n)
    for (int d = 0; d < 3; ++d) m->rowptr[3 * n + d + 1] = m->rowptr[3 * n + d] + 3 * int64_t(nnb[n]);
  m->col_lid.resize(m->rowptr[3 * n_rn]);
  parallel_for(n_rn, [&](int64_t n) {
    int32_t v[125];
    const int c = neighbours(n, v);
    for (int d = 0; d < 3; ++d)
    {
      int32_t* cl = m->col_lid.data() + m->rowptr[3 * n + d];
      for (int k = 0; k < c; ++k)
        for (int j = 0; j < 3; ++j) cl[3 * k + j] = 3 * v[k] + j;  // node_dof_col == 3 * local id
    }
  });
  tick("csr");
  *out = m;
  return FCG_OK;
}

int fcg_box_mesh_destroy(fcg_box_mesh* m)
{
  delete m;
  return FCG_OK;
}

int fcg_box_mesh_desc(const fcg_box_mesh* m, int kinematics, double youngs, double poisson,
    int device, fcg_desc* o)
{
  if (!m || !o) return FCG_ERR_ARG;
  std::memset(o, 0, sizeof(*o));
  o->abi_version = FCG_ABI_VERSION;
  o->celltype = m->box.celltype;
  o->kinematics = kinematics;
  o->device = device;
  o->youngs = youngs;
  o->poisson = poisson;
  o->n_ele = int64_t(m->ele_gid.size());
  o->n_node = int64_t(m->node_gid.size());
  o->n_rows = int64_t(m->row_gid.size());
  o->n_cols = int64_t(m->col_gid.size());
  o->ele_nodes = m->ele_nodes.data();
  o->ele_gid = m->ele_gid.data();
  o->node_x = m->node_x.data();
  o->node_dof_col = m->node_dof_col.data();
  o->node_dof_row = m->node_dof_row.data();
  o->node_dof_kcol = nullptr;
  o->ele_ijk = m->ele_ijk.data();
  o->path = FCG_PATH_AUTO;
  o->rowptr = m->rowptr.data();
  o->col_lid = m->col_lid.data();
  return FCG_OK;
}

int fcg_box_mesh_maps(const fcg_box_mesh* m, const int32_t** row_gid, const int32_t** col_gid,
    const int64_t** node_gid, const int32_t** node_owner)
{
  if (!m) return FCG_ERR_ARG;
  if (row_gid) *row_gid = m->row_gid.data();
  if (col_gid) *col_gid = m->col_gid.data();
  if (node_gid) *node_gid = m->node_gid.data();
  if (node_owner) *node_owner = m->node_owner.data();
  return FCG_OK;
}

int fcg_box_mesh_counts(const fcg_box_mesh* m, int64_t* n_ele_global, int64_t* n_ele_row)
{
  if (!m) return FCG_ERR_ARG;
  if (n_ele_global) *n_ele_global = m->n_ele_global;
  if (n_ele_row) *n_ele_row = m->n_ele_row;
  return FCG_OK;
}

int fcg_box_mesh_owned_rows(const fcg_box_mesh* m, int64_t* n_owned_rows)
{
  if (!m || !n_owned_rows) return FCG_ERR_ARG;
  *n_owned_rows = m->n_owned_rows;
  return FCG_OK;
}

}  // extern "C"
