// fcg_graph.hip -- the matrix graph of the solid discretization built on the device: the
// FillComplete equivalent of 4C's first assembly.
//
// Reference: the stiffness is created with an estimated row length
// (SparseMatrix(dof_row_map, 81, explicitdirichlet, savegraph),
// 4C_structure_new_timint_basedataglobalstate.cpp:650-652); the first Discretization::evaluate runs
// SparseMatrix::assemble's unfilled path, InsertGlobalValues / SumIntoGlobalValues per entry
// (4C_linalg_sparsematrix.cpp:578-611), and complete() calls Epetra_CrsMatrix::FillComplete
// (:843-865), which sorts and merges the column indices of every row.  The resulting graph: one row
// per owned DOF, columns = the DOFs of every node sharing an element with the row's node, sorted by
// column LID.  Here (one rank's column elements, local LIDs):
//   1. incidences of the owned nodes (count, scan, fill);
//   2. one wavefront per owned node gathers the column LIDs of its elements' nodes into LDS, ranks
//      the distinct ones (sorted order without a sort: rank = number of distinct smaller LIDs);
//   3. row lengths -> row pointers (scan), then the same wavefronts write the 3 rows.
// Deterministic: the result does not depend on the order atomics hand out incidence slots.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_scan.hpp>

#include <climits>

#include "fourc_gpu.h"
#include "fcg_status.hpp"

namespace fcg {
namespace {

constexpr int kMaxInc = 16;  // elements per node handled by one wavefront

__global__ void graph_check_rows(int64_t n_node, const int32_t* dof_row, int64_t n_rows, int32_t* err)
{
  for (int64_t n = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; n < n_node;
       n += int64_t(gridDim.x) * blockDim.x)
  {
    const int32_t r = dof_row[n];
    if (r >= 0 && (r % 3 != 0 || r + 3 > n_rows)) atomicMax(err, 1);
  }
}

__global__ void graph_count(int64_t n_inc_all, const int32_t* ele_nodes, const int32_t* dof_row,
    int64_t n_node, int64_t* cnt, int32_t* err)
{
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n_inc_all;
       i += int64_t(gridDim.x) * blockDim.x)
  {
    const int32_t n = ele_nodes[i];
    if (n < 0 || n >= n_node)
    {
      atomicMax(err, 2);
      continue;
    }
    const int32_t r = dof_row[n];
    if (r >= 0) atomicAdd(reinterpret_cast<unsigned long long*>(&cnt[r / 3]), 1ull);
  }
}

__global__ void graph_fill(int64_t n_inc_all, int npe, const int32_t* ele_nodes,
    const int32_t* dof_row, const int64_t* inc_ptr, int64_t* cursor, int32_t* inc_ele)
{
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n_inc_all;
       i += int64_t(gridDim.x) * blockDim.x)
  {
    const int32_t r = dof_row[ele_nodes[i]];
    if (r < 0) continue;
    const int64_t rn = r / 3;
    const unsigned long long k = atomicAdd(reinterpret_cast<unsigned long long*>(&cursor[rn]), 1ull);
    inc_ele[inc_ptr[rn] + int64_t(k)] = int32_t(i / npe);
  }
}

// one wavefront per owned node: FILL = false writes the 3 row lengths, FILL = true the columns
template <int NPE, bool FILL>
__global__ __launch_bounds__(64) void graph_rows(int64_t n_rn, const int32_t* ele_nodes,
    const int32_t* dof_col, const int64_t* inc_ptr, const int32_t* inc_ele, int64_t* rowlen,
    const int64_t* rowptr, int32_t* col_lid, int32_t* err)
{
  constexpr int MAXC = kMaxInc * NPE;
  __shared__ int32_t cand[MAXC];
  __shared__ uint8_t first[MAXC];
  const int lane = threadIdx.x;
  for (int64_t rn = blockIdx.x; rn < n_rn; rn += gridDim.x)
  {
    const int64_t k0 = inc_ptr[rn], k1 = inc_ptr[rn + 1];
    const int ninc = int(k1 - k0);
    if (ninc > kMaxInc)
    {
      if (lane == 0) atomicMax(err, 3);
      continue;
    }
    const int nc = ninc * NPE;
    for (int v = lane; v < nc; v += 64)
    {
      const int k = v / NPE, b = v - NPE * k;
      cand[v] = dof_col[ele_nodes[int64_t(inc_ele[k0 + k]) * NPE + b]];
    }
    __syncthreads();
    // first occurrence of every column LID
    for (int v = lane; v < nc; v += 64)
    {
      const int32_t c = cand[v];
      bool f = true;
      for (int j = 0; j < v; ++j) f = f && cand[j] != c;
      first[v] = f ? 1 : 0;
    }
    __syncthreads();
    // rank among the distinct LIDs = position in the sorted row (FillComplete's sort + merge)
    int distinct = 0;
    for (int v = lane; v < nc; v += 64)
    {
      if (!first[v]) continue;
      ++distinct;
      if (FILL)
      {
        const int32_t c = cand[v];
        int rank = 0;
        for (int j = 0; j < nc; ++j) rank += (first[j] && cand[j] < c) ? 1 : 0;
        const int64_t base = rowptr[3 * rn];
        const int64_t len = rowptr[3 * rn + 1] - base;
#pragma unroll
        for (int d = 0; d < 3; ++d)
#pragma unroll
          for (int j = 0; j < 3; ++j) col_lid[base + d * len + 3 * rank + j] = c + j;
      }
    }
    if (!FILL)
    {
      // wavefront sum of the first occurrences
      for (int off = 32; off > 0; off >>= 1) distinct += __shfl_xor(distinct, off);
      if (lane == 0)
        for (int d = 0; d < 3; ++d) rowlen[3 * rn + d] = 3 * int64_t(distinct);
    }
    __syncthreads();
  }
}

int grid_for(int64_t work, int cap) { return int(work < cap ? (work > 0 ? work : 1) : cap); }

hipError_t exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, hipStream_t s)
{
  size_t bytes = 0;
  hipError_t e = rocprim::exclusive_scan(nullptr, bytes, in, out, int64_t(0), size_t(n),
      rocprim::plus<int64_t>(), s);
  if (e != hipSuccess) return e;
  void* tmp = nullptr;
  e = hipMallocAsync(&tmp, bytes > 0 ? bytes : 1, s);
  if (e != hipSuccess) return e;
  e = rocprim::exclusive_scan(tmp, bytes, in, out, int64_t(0), size_t(n), rocprim::plus<int64_t>(), s);
  hipError_t f = hipFreeAsync(tmp, s);
  return e != hipSuccess ? e : f;
}

}  // namespace
}  // namespace fcg

extern "C" int fcg_graph_build_device(int device, int celltype, int64_t n_ele,
    const int32_t* d_ele_nodes, int64_t n_node, const int32_t* d_node_dof_col,
    const int32_t* d_node_dof_row, int64_t n_rows, int64_t* d_rowptr, int32_t* d_col_lid,
    int64_t col_capacity, int64_t* nnz, void* stream_ptr)
{
  if ((celltype != FCG_HEX8 && celltype != FCG_HEX27) || n_ele < 0 || n_node < 0 || n_rows < 0 ||
      n_rows % 3 != 0 || !nnz || !d_rowptr || (n_ele > 0 && (!d_ele_nodes || !d_node_dof_col)) ||
      (n_node > 0 && !d_node_dof_row))
    return FCG_ERR_ARG;
  const int npe = celltype == FCG_HEX27 ? 27 : 8;
  const int64_t n_rn = n_rows / 3;
  const int64_t n_all = n_ele * npe;
  hipError_t he = hipSetDevice(device);
  hipStream_t s = static_cast<hipStream_t>(stream_ptr);
  int64_t *cnt = nullptr, *inc_ptr = nullptr, *cursor = nullptr, *rowlen = nullptr;
  int32_t *inc_ele = nullptr, *err = nullptr;
  auto chk = [&](hipError_t x) {
    if (he == hipSuccess) he = x;
  };
  chk(hipMallocAsync(reinterpret_cast<void**>(&cnt), sizeof(int64_t) * (n_rn + 1), s));
  chk(hipMallocAsync(reinterpret_cast<void**>(&inc_ptr), sizeof(int64_t) * (n_rn + 1), s));
  chk(hipMallocAsync(reinterpret_cast<void**>(&cursor), sizeof(int64_t) * (n_rn + 1), s));
  chk(hipMallocAsync(reinterpret_cast<void**>(&rowlen), sizeof(int64_t) * (n_rows + 1), s));
  chk(hipMallocAsync(reinterpret_cast<void**>(&err), sizeof(int32_t), s));
  if (he == hipSuccess)
  {
    chk(hipMemsetAsync(cnt, 0, sizeof(int64_t) * (n_rn + 1), s));
    chk(hipMemsetAsync(cursor, 0, sizeof(int64_t) * (n_rn + 1), s));
    chk(hipMemsetAsync(rowlen, 0, sizeof(int64_t) * (n_rows + 1), s));
    chk(hipMemsetAsync(err, 0, sizeof(int32_t), s));
  }
  const int gridn = fcg::grid_for((n_node + 255) / 256, 256 * 16);
  const int grida = fcg::grid_for((n_all + 255) / 256, 256 * 16);
  if (he == hipSuccess && n_node > 0)
  {
    hipLaunchKernelGGL(fcg::graph_check_rows, dim3(gridn), dim3(256), 0, s, n_node, d_node_dof_row,
        n_rows, err);
    chk(hipGetLastError());
  }
  // stop before any kernel indexes with invalid LIDs
  int32_t errv = 0;
  auto read_err = [&]() {
    if (he == hipSuccess) he = hipMemcpyAsync(&errv, err, sizeof(int32_t), hipMemcpyDeviceToHost, s);
    if (he == hipSuccess) he = hipStreamSynchronize(s);
    return he == hipSuccess && errv == 0;
  };
  if (read_err() && n_all > 0)
  {
    hipLaunchKernelGGL(fcg::graph_count, dim3(grida), dim3(256), 0, s, n_all, d_ele_nodes,
        d_node_dof_row, n_node, cnt, err);
    chk(hipGetLastError());
  }
  if (he == hipSuccess) he = fcg::exclusive_scan_i64(cnt, inc_ptr, n_rn + 1, s);
  int64_t n_inc = 0;
  if (he == hipSuccess)
    he = hipMemcpyAsync(&n_inc, inc_ptr + n_rn, sizeof(int64_t), hipMemcpyDeviceToHost, s);
  if (read_err())
    chk(hipMallocAsync(reinterpret_cast<void**>(&inc_ele), sizeof(int32_t) * (n_inc > 0 ? n_inc : 1), s));
  if (he == hipSuccess && errv == 0 && n_all > 0)
  {
    hipLaunchKernelGGL(fcg::graph_fill, dim3(grida), dim3(256), 0, s, n_all, npe, d_ele_nodes,
        d_node_dof_row, inc_ptr, cursor, inc_ele);
    chk(hipGetLastError());
  }
  const int gridr = fcg::grid_for(n_rn, 256 * 64);
  if (he == hipSuccess && errv == 0 && n_rn > 0)
  {
    if (npe == 8)
      hipLaunchKernelGGL((fcg::graph_rows<8, false>), dim3(gridr), dim3(64), 0, s, n_rn,
          d_ele_nodes, d_node_dof_col, inc_ptr, inc_ele, rowlen, nullptr, nullptr, err);
    else
      hipLaunchKernelGGL((fcg::graph_rows<27, false>), dim3(gridr), dim3(64), 0, s, n_rn,
          d_ele_nodes, d_node_dof_col, inc_ptr, inc_ele, rowlen, nullptr, nullptr, err);
    chk(hipGetLastError());
  }
  if (he == hipSuccess && errv == 0) he = fcg::exclusive_scan_i64(rowlen, d_rowptr, n_rows + 1, s);
  int64_t total = 0;
  if (he == hipSuccess) he = hipMemcpyAsync(&errv, err, sizeof(int32_t), hipMemcpyDeviceToHost, s);
  if (he == hipSuccess)
    he = hipMemcpyAsync(&total, d_rowptr + n_rows, sizeof(int64_t), hipMemcpyDeviceToHost, s);
  if (he == hipSuccess) he = hipStreamSynchronize(s);
  if (he == hipSuccess && errv == 0 && d_col_lid && col_capacity >= total && n_rn > 0)
  {
    if (npe == 8)
      hipLaunchKernelGGL((fcg::graph_rows<8, true>), dim3(gridr), dim3(64), 0, s, n_rn,
          d_ele_nodes, d_node_dof_col, inc_ptr, inc_ele, nullptr, d_rowptr, d_col_lid, err);
    else
      hipLaunchKernelGGL((fcg::graph_rows<27, true>), dim3(gridr), dim3(64), 0, s, n_rn,
          d_ele_nodes, d_node_dof_col, inc_ptr, inc_ele, nullptr, d_rowptr, d_col_lid, err);
    chk(hipGetLastError());
    if (he == hipSuccess) he = hipStreamSynchronize(s);
  }
  for (void* p : {static_cast<void*>(cnt), static_cast<void*>(inc_ptr), static_cast<void*>(cursor),
           static_cast<void*>(rowlen), static_cast<void*>(inc_ele), static_cast<void*>(err)})
    if (p) (void)hipFreeAsync(p, s);
  (void)hipStreamSynchronize(s);
  if (he != hipSuccess) return fcg_device_error();
  if (errv != 0) return FCG_ERR_ARG;
  *nnz = total;
  return FCG_OK;
}
