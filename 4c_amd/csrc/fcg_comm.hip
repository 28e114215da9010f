// fcg_comm.hip -- the multi-GPU data path over RCCL (xGMI within a node), SURVEY §8e.
//
//   fcg_comm            one RCCL communicator per rank (ncclCommInitRank on the rank's device)
//   fcg_halo_import     Discretization::set_state's row -> column Epetra_Import
//                       (4C_fem_discretization.cpp:542-548): the owned columns are copied on the
//                       device, the ghost values move by one grouped ncclSend / ncclRecv per
//                       neighbour -- straight into the column vector when a neighbour's ghost
//                       columns are contiguous (Epetra column maps group ghosts by owner)
//   fcg_shared_reduce   strict element partition (option B): the interface partial sums go into one
//                       compact buffer (position by (owner, GID), fcg_plan.cpp) reduced by
//                       ncclAllReduce (Core::Communication::sum_all, 4C_comm_mpi_utils.hpp:294-306)
//   fcg_norm2           the NOX residual norm: fixed-order block partials + an all-reduce
// Everything is queued on the caller's stream; RCCL orders its kernels on the same stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "fourc_gpu.h"
#include "fcg_status.hpp"

struct fcg_comm {
  ncclComm_t nccl = nullptr;
  int nranks = 1, rank = 0, device = 0;
  hipStream_t stream = nullptr;  // for the blocking host exchange
  double* d_scalar = nullptr;    // fcg_norm2 partials and result
  double* h_scalar = nullptr;    // pinned
};

struct fcg_halo {
  int device = 0, nranks = 1, rank = 0;
  int64_t n_same = 0, n_permute = 0, n_send = 0, n_recv = 0;
  int32_t* permute_from = nullptr;
  int32_t* permute_to = nullptr;
  int32_t* send_row = nullptr;
  int32_t* recv_col = nullptr;
  double* send = nullptr;
  double* recv = nullptr;
  std::vector<int64_t> send_off, recv_off;  // [nranks + 1]
  std::vector<int64_t> recv_first;          // first column of a contiguous peer block, else -1
  bool scatter_needed = false;              // some peer's ghost columns are not contiguous
};

struct fcg_shared {
  int device = 0;
  int64_t n_global = 0, n_local = 0, n_owned = 0;
  int32_t* row = nullptr;
  int64_t* pos = nullptr;
  double* buf = nullptr;
};

namespace {

constexpr int kBlock = 256;

template <class T>
hipError_t to_device(T** dst, const T* src, int64_t n)
{
  *dst = nullptr;
  if (n <= 0) return hipSuccess;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(dst), sizeof(T) * n);
  if (e == hipSuccess && src) e = hipMemcpy(*dst, src, sizeof(T) * n, hipMemcpyHostToDevice);
  return e;
}

unsigned grid_for(int64_t n, int64_t cap = 4096)
{
  return unsigned(std::max<int64_t>(1, std::min<int64_t>(cap, (n + kBlock - 1) / kBlock)));
}

// owned columns (same + permuted) and the send buffer, one grid-stride pass over all three ranges
__global__ __launch_bounds__(kBlock) void halo_local_kernel(const double* __restrict__ u_row,
    double* __restrict__ u_col, int64_t n_same, const int32_t* __restrict__ pfrom,
    const int32_t* __restrict__ pto, int64_t n_perm, const int32_t* __restrict__ send_row,
    double* __restrict__ send, int64_t n_send)
{
  const int64_t total = n_same + n_perm + n_send;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * kBlock)
  {
    if (i < n_same)
      u_col[i] = u_row[i];
    else if (i < n_same + n_perm)
    {
      const int64_t k = i - n_same;
      u_col[pto[k]] = u_row[pfrom[k]];
    }
    else
    {
      const int64_t k = i - n_same - n_perm;
      send[k] = u_row[send_row[k]];
    }
  }
}

__global__ __launch_bounds__(kBlock) void scatter_kernel(const double* __restrict__ src,
    const int32_t* __restrict__ idx, double* __restrict__ dst, int64_t n)
{
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
    dst[idx[i]] = src[i];
}

// d_buf[pos[i]] = f[row[i]] (positions distinct within a rank; the buffer was zeroed)
__global__ __launch_bounds__(kBlock) void shared_pack_kernel(const double* __restrict__ f,
    const int32_t* __restrict__ row, const int64_t* __restrict__ pos, double* __restrict__ buf,
    int64_t n)
{
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
    buf[pos[i]] = f[row[i]];
}

__global__ __launch_bounds__(kBlock) void shared_unpack_kernel(const double* __restrict__ buf,
    const int32_t* __restrict__ row, const int64_t* __restrict__ pos, double* __restrict__ f,
    int64_t n_owned)
{
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n_owned;
       i += int64_t(gridDim.x) * kBlock)
    f[row[i]] = buf[pos[i]];
}

// deterministic block sum (wave butterfly, then the waves in order); valid in thread 0
__device__ inline double block_sum(double v, double* sbuf)
{
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sbuf[w] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < int(blockDim.x >> 6); ++i) t += sbuf[i];
  return t;
}

constexpr int kNormBlocks = 1024;

__global__ __launch_bounds__(kBlock) void sumsq_kernel(const double* __restrict__ x, int64_t n,
    double* __restrict__ partial)
{
  __shared__ double sbuf[kBlock / 64];
  double s = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += int64_t(gridDim.x) * kBlock)
    s += x[i] * x[i];
  const double t = block_sum(s, sbuf);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

__global__ __launch_bounds__(kBlock) void sum_partials_kernel(double* __restrict__ partial, int n,
    double* __restrict__ out)
{
  __shared__ double sbuf[kBlock / 64];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += kBlock) s += partial[i];
  const double t = block_sum(s, sbuf);
  if (threadIdx.x == 0) *out = t;
}

int nccl_status(ncclResult_t r) { return r == ncclSuccess ? FCG_OK : fcg_device_error(); }

}  // namespace

extern "C" {

int fcg_comm_unique_id(void* id)
{
  if (!id) return FCG_ERR_ARG;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return fcg_device_error();
  std::memcpy(id, &u, sizeof(u));
  return FCG_OK;
}

int fcg_comm_create(const void* id, int nranks, int rank, int device, fcg_comm** out)
{
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return FCG_ERR_ARG;
  *out = nullptr;
  if (!fcg_use_device(device)) return fcg_device_error();
  auto* c = new fcg_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  hipError_t he = hipStreamCreate(&c->stream);
  if (he == hipSuccess) he = hipMalloc(&c->d_scalar, sizeof(double) * (kNormBlocks + 1));
  if (he == hipSuccess) he = hipHostMalloc(&c->h_scalar, sizeof(double));
  if (he != hipSuccess || ncclCommInitRank(&c->nccl, nranks, u, rank) != ncclSuccess)
  {
    c->nccl = nullptr;
    fcg_comm_destroy(c);
    return fcg_device_error();
  }
  *out = c;
  return FCG_OK;
}

int fcg_comm_destroy(fcg_comm* c)
{
  if (!c) return FCG_OK;
  (void)hipSetDevice(c->device);
  if (c->nccl) (void)ncclCommDestroy(c->nccl);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->d_scalar) (void)hipFree(c->d_scalar);
  if (c->h_scalar) (void)hipHostFree(c->h_scalar);
  delete c;
  return FCG_OK;
}

int fcg_comm_size(const fcg_comm* c, int* nranks)
{
  if (!c || !nranks) return FCG_ERR_ARG;
  int n = 0;
  if (ncclCommCount(c->nccl, &n) != ncclSuccess) return fcg_device_error();
  *nranks = n;
  return FCG_OK;
}

int fcg_comm_rank(const fcg_comm* c, int* rank)
{
  if (!c || !rank) return FCG_ERR_ARG;
  int r = 0;
  if (ncclCommUserRank(c->nccl, &r) != ncclSuccess) return fcg_device_error();
  *rank = r;
  return FCG_OK;
}

int fcg_comm_allreduce(fcg_comm* c, double* d_buf, int64_t n, int op, void* stream)
{
  if (!c || n < 0 || (n && !d_buf) || (op != FCG_OP_SUM && op != FCG_OP_MAX)) return FCG_ERR_ARG;
  if (n == 0) return FCG_OK;
  (void)hipSetDevice(c->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
  return nccl_status(ncclAllReduce(d_buf, d_buf, size_t(n), ncclFloat64,
      op == FCG_OP_SUM ? ncclSum : ncclMax, c->nccl, s));
}

int fcg_comm_alltoallv(const void* send_buf, const int64_t* send_counts, void* recv_buf,
    const int64_t* recv_counts, int64_t item_bytes, void* user)
{
  auto* c = static_cast<fcg_comm*>(user);
  if (!c || !send_counts || !recv_counts || item_bytes <= 0) return FCG_ERR_ARG;
  (void)hipSetDevice(c->device);
  int64_t ns = 0, nr = 0;
  for (int p = 0; p < c->nranks; ++p)
  {
    ns += send_counts[p];
    nr += recv_counts[p];
  }
  char* d_send = nullptr;
  char* d_recv = nullptr;
  hipError_t he = hipMalloc(&d_send, std::max<int64_t>(1, ns * item_bytes));
  if (he == hipSuccess) he = hipMalloc(&d_recv, std::max<int64_t>(1, nr * item_bytes));
  if (he == hipSuccess && ns)
    he = hipMemcpyAsync(d_send, send_buf, ns * item_bytes, hipMemcpyHostToDevice, c->stream);
  int rc = he == hipSuccess ? FCG_OK : fcg_device_error();
  if (rc == FCG_OK)
  {
    int64_t so = 0, ro = 0;
    ncclResult_t r = ncclGroupStart();
    for (int p = 0; p < c->nranks && r == ncclSuccess; ++p)
    {
      if (send_counts[p])
        r = ncclSend(d_send + so * item_bytes, size_t(send_counts[p] * item_bytes), ncclUint8, p,
            c->nccl, c->stream);
      if (r == ncclSuccess && recv_counts[p])
        r = ncclRecv(d_recv + ro * item_bytes, size_t(recv_counts[p] * item_bytes), ncclUint8, p,
            c->nccl, c->stream);
      so += send_counts[p];
      ro += recv_counts[p];
    }
    const ncclResult_t r2 = ncclGroupEnd();
    rc = (r == ncclSuccess && r2 == ncclSuccess) ? FCG_OK : fcg_device_error();
  }
  if (rc == FCG_OK && nr)
    rc = hipMemcpyAsync(recv_buf, d_recv, nr * item_bytes, hipMemcpyDeviceToHost, c->stream) ==
                 hipSuccess
             ? FCG_OK
             : fcg_device_error();
  if (hipStreamSynchronize(c->stream) != hipSuccess) rc = fcg_device_error();
  if (d_send) (void)hipFree(d_send);
  if (d_recv) (void)hipFree(d_recv);
  return rc;
}

int fcg_comm_exchange_device(void* comm, const double* d_send, const int64_t* send_counts,
    double* d_recv, const int64_t* recv_counts, void* stream)
{
  auto* c = static_cast<fcg_comm*>(comm);
  if (!c || !send_counts || !recv_counts) return FCG_ERR_ARG;
  (void)hipSetDevice(c->device);
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c->stream;
  int64_t so = 0, ro = 0;
  ncclResult_t r = ncclGroupStart();
  for (int p = 0; p < c->nranks && r == ncclSuccess; ++p)
  {
    if (send_counts[p] > 0) r = ncclSend(d_send + so, size_t(send_counts[p]), ncclFloat64, p, c->nccl, s);
    if (r == ncclSuccess && recv_counts[p] > 0)
      r = ncclRecv(d_recv + ro, size_t(recv_counts[p]), ncclFloat64, p, c->nccl, s);
    so += send_counts[p];
    ro += recv_counts[p];
  }
  const ncclResult_t r2 = ncclGroupEnd();
  return (r == ncclSuccess && r2 == ncclSuccess) ? FCG_OK : fcg_device_error();
}

int fcg_halo_create(const fcg_import_plan* p, int device, fcg_halo** out)
{
  if (!p || !out || p->nranks < 1 || p->rank < 0 || p->rank >= p->nranks || p->n_same < 0 ||
      p->n_permute < 0 || p->n_same > p->n_rows || p->n_same > p->n_cols)
    return FCG_ERR_ARG;
  *out = nullptr;
  auto* h = new fcg_halo();
  h->device = device;
  h->nranks = p->nranks;
  h->rank = p->rank;
  h->n_same = p->n_same;
  h->n_permute = p->n_permute;
  h->send_off.assign(p->nranks + 1, 0);
  h->recv_off.assign(p->nranks + 1, 0);
  h->recv_first.assign(p->nranks, -1);
  bool ok = true;
  for (int q = 0; q < p->nranks; ++q)
  {
    ok = ok && p->send_counts[q] >= 0 && p->recv_counts[q] >= 0;
    h->send_off[q + 1] = h->send_off[q] + p->send_counts[q];
    h->recv_off[q + 1] = h->recv_off[q] + p->recv_counts[q];
  }
  h->n_send = h->send_off[p->nranks];
  h->n_recv = h->recv_off[p->nranks];
  // host-side bounds of every index the kernels use
  for (int64_t i = 0; ok && i < p->n_permute; ++i)
    ok = p->permute_from[i] >= 0 && p->permute_from[i] < p->n_rows && p->permute_to[i] >= 0 &&
         p->permute_to[i] < p->n_cols;
  for (int64_t i = 0; ok && i < h->n_send; ++i) ok = p->send_row[i] >= 0 && p->send_row[i] < p->n_rows;
  for (int64_t i = 0; ok && i < h->n_recv; ++i) ok = p->recv_col[i] >= 0 && p->recv_col[i] < p->n_cols;
  if (!ok)
  {
    delete h;
    return FCG_ERR_ARG;
  }
  for (int q = 0; q < p->nranks; ++q)
  {
    const int64_t a = h->recv_off[q], n = h->recv_off[q + 1] - a;
    if (n == 0) continue;
    bool contig = true;
    for (int64_t i = 1; i < n && contig; ++i) contig = p->recv_col[a + i] == p->recv_col[a] + i;
    if (contig)
      h->recv_first[q] = p->recv_col[a];
    else
      h->scatter_needed = true;
  }
  if (!fcg_use_device(device))
  {
    delete h;
    return fcg_device_error();
  }
  hipError_t he = to_device(&h->permute_from, p->permute_from, p->n_permute);
  if (he == hipSuccess) he = to_device(&h->permute_to, p->permute_to, p->n_permute);
  if (he == hipSuccess) he = to_device(&h->send_row, p->send_row, h->n_send);
  if (he == hipSuccess) he = to_device(&h->recv_col, p->recv_col, h->n_recv);
  if (he == hipSuccess) he = to_device(&h->send, static_cast<const double*>(nullptr), h->n_send);
  if (he == hipSuccess) he = to_device(&h->recv, static_cast<const double*>(nullptr), h->n_recv);
  if (he != hipSuccess)
  {
    fcg_halo_destroy(h);
    return fcg_device_error();
  }
  *out = h;
  return FCG_OK;
}

int fcg_halo_destroy(fcg_halo* h)
{
  if (!h) return FCG_OK;
  (void)hipSetDevice(h->device);
  for (void* p : {static_cast<void*>(h->permute_from), static_cast<void*>(h->permute_to),
           static_cast<void*>(h->send_row), static_cast<void*>(h->recv_col),
           static_cast<void*>(h->send), static_cast<void*>(h->recv)})
    if (p) (void)hipFree(p);
  delete h;
  return FCG_OK;
}

int fcg_halo_pack(fcg_halo* h, const double* d_u_row, double* d_u_col, double* d_send, void* stream)
{
  if (!h || ((h->n_same || h->n_permute || h->n_send) && !d_u_row) ||
      ((h->n_same || h->n_permute) && !d_u_col) || (h->n_send && !d_send))
    return FCG_ERR_ARG;
  (void)hipSetDevice(h->device);
  const int64_t total = h->n_same + h->n_permute + h->n_send;
  if (total == 0) return FCG_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  halo_local_kernel<<<grid_for(total), kBlock, 0, s>>>(d_u_row, d_u_col, h->n_same,
      h->permute_from, h->permute_to, h->n_permute, h->send_row, d_send, h->n_send);
  return hipGetLastError() == hipSuccess ? FCG_OK : fcg_device_error();
}

int fcg_halo_unpack(fcg_halo* h, const double* d_recv, double* d_u_col, void* stream)
{
  if (!h || (h->n_recv && (!d_recv || !d_u_col))) return FCG_ERR_ARG;
  if (h->n_recv == 0) return FCG_OK;
  (void)hipSetDevice(h->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  scatter_kernel<<<grid_for(h->n_recv), kBlock, 0, s>>>(d_recv, h->recv_col, d_u_col, h->n_recv);
  return hipGetLastError() == hipSuccess ? FCG_OK : fcg_device_error();
}

int fcg_halo_import(fcg_halo* h, fcg_comm* c, const double* d_u_row, double* d_u_col, void* stream)
{
  if (!h || !c || c->nranks != h->nranks || c->rank != h->rank) return FCG_ERR_ARG;
  int rc = fcg_halo_pack(h, d_u_row, d_u_col, h->send, stream);
  if (rc != FCG_OK) return rc;
  if (h->n_send == 0 && h->n_recv == 0) return FCG_OK;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : nullptr;
  ncclResult_t r = ncclGroupStart();
  for (int q = 0; q < h->nranks && r == ncclSuccess; ++q)
  {
    const int64_t ns = h->send_off[q + 1] - h->send_off[q];
    const int64_t nr = h->recv_off[q + 1] - h->recv_off[q];
    if (ns) r = ncclSend(h->send + h->send_off[q], size_t(ns), ncclFloat64, q, c->nccl, s);
    if (r == ncclSuccess && nr)
    {
      double* dst = h->recv_first[q] >= 0 ? d_u_col + h->recv_first[q] : h->recv + h->recv_off[q];
      r = ncclRecv(dst, size_t(nr), ncclFloat64, q, c->nccl, s);
    }
  }
  const ncclResult_t r2 = ncclGroupEnd();
  if (r != ncclSuccess || r2 != ncclSuccess) return fcg_device_error();
  if (!h->scatter_needed) return FCG_OK;
  // peers with scattered ghost columns landed in h->recv: scatter those blocks
  for (int q = 0; q < h->nranks; ++q)
  {
    const int64_t a = h->recv_off[q], n = h->recv_off[q + 1] - a;
    if (n == 0 || h->recv_first[q] >= 0) continue;
    scatter_kernel<<<grid_for(n), kBlock, 0, s>>>(h->recv + a, h->recv_col + a, d_u_col, n);
  }
  return hipGetLastError() == hipSuccess ? FCG_OK : fcg_device_error();
}

int fcg_shared_create(const fcg_shared_plan* p, int device, fcg_shared** out)
{
  if (!p || !out || p->n_local < 0 || p->n_owned < 0 || p->n_owned > p->n_local || p->n_global < 0 ||
      (p->n_local && (!p->row || !p->pos)))
    return FCG_ERR_ARG;
  *out = nullptr;
  for (int64_t i = 0; i < p->n_local; ++i)
    if (p->row[i] < 0 || p->pos[i] < 0 || p->pos[i] >= p->n_global) return FCG_ERR_ARG;
  if (!fcg_use_device(device)) return fcg_device_error();
  auto* s = new fcg_shared();
  s->device = device;
  s->n_global = p->n_global;
  s->n_local = p->n_local;
  s->n_owned = p->n_owned;
  hipError_t he = to_device(&s->row, p->row, p->n_local);
  if (he == hipSuccess) he = to_device(&s->pos, p->pos, p->n_local);
  if (he == hipSuccess) he = to_device(&s->buf, static_cast<const double*>(nullptr), p->n_global);
  if (he != hipSuccess)
  {
    fcg_shared_destroy(s);
    return fcg_device_error();
  }
  *out = s;
  return FCG_OK;
}

int fcg_shared_destroy(fcg_shared* s)
{
  if (!s) return FCG_OK;
  (void)hipSetDevice(s->device);
  if (s->row) (void)hipFree(s->row);
  if (s->pos) (void)hipFree(s->pos);
  if (s->buf) (void)hipFree(s->buf);
  delete s;
  return FCG_OK;
}

int fcg_shared_pack(fcg_shared* s, const double* d_f, double* d_buf, void* stream)
{
  if (!s || (s->n_global && !d_buf) || (s->n_local && !d_f)) return FCG_ERR_ARG;
  if (s->n_global == 0) return FCG_OK;
  (void)hipSetDevice(s->device);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (hipMemsetAsync(d_buf, 0, sizeof(double) * s->n_global, st) != hipSuccess) return fcg_device_error();
  if (s->n_local)
    shared_pack_kernel<<<grid_for(s->n_local), kBlock, 0, st>>>(d_f, s->row, s->pos, d_buf, s->n_local);
  return hipGetLastError() == hipSuccess ? FCG_OK : fcg_device_error();
}

int fcg_shared_unpack(fcg_shared* s, const double* d_buf, double* d_f, void* stream)
{
  if (!s || (s->n_owned && (!d_buf || !d_f))) return FCG_ERR_ARG;
  if (s->n_owned == 0) return FCG_OK;
  (void)hipSetDevice(s->device);
  hipStream_t st = static_cast<hipStream_t>(stream);
  shared_unpack_kernel<<<grid_for(s->n_owned), kBlock, 0, st>>>(d_buf, s->row, s->pos, d_f, s->n_owned);
  return hipGetLastError() == hipSuccess ? FCG_OK : fcg_device_error();
}

int fcg_shared_reduce(fcg_shared* s, fcg_comm* c, double* d_f, void* stream)
{
  if (!s || !c) return FCG_ERR_ARG;
  int rc = fcg_shared_pack(s, d_f, s->buf, stream);
  if (rc != FCG_OK || s->n_global == 0) return rc;
  rc = fcg_comm_allreduce(c, s->buf, s->n_global, FCG_OP_SUM, stream);
  if (rc != FCG_OK) return rc;
  return fcg_shared_unpack(s, s->buf, d_f, stream);
}

int fcg_norm2(fcg_comm* c, const double* d_x, int64_t n, void* stream, double* out)
{
  if (!out || n < 0 || (n && !d_x)) return FCG_ERR_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  // without a communicator: small per-device buffers kept for the process lifetime
  static double* local_dev[64] = {};
  static double* local_host[64] = {};
  double* d_part;
  double* h_res;
  if (c)
  {
    (void)hipSetDevice(c->device);
    d_part = c->d_scalar;
    h_res = c->h_scalar;
  }
  else
  {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return fcg_device_error();
    if (!local_dev[dev] && (hipMalloc(&local_dev[dev], sizeof(double) * (kNormBlocks + 1)) != hipSuccess ||
                               hipHostMalloc(&local_host[dev], sizeof(double)) != hipSuccess))
      return fcg_device_error();
    d_part = local_dev[dev];
    h_res = local_host[dev];
  }
  const int nb = int(std::min<int64_t>(kNormBlocks, std::max<int64_t>(1, (n + kBlock - 1) / kBlock)));
  sumsq_kernel<<<nb, kBlock, 0, s>>>(d_x, n, d_part);
  sum_partials_kernel<<<1, kBlock, 0, s>>>(d_part, nb, d_part + kNormBlocks);
  if (hipGetLastError() != hipSuccess) return fcg_device_error();
  if (c && c->nranks > 1 &&
      ncclAllReduce(d_part + kNormBlocks, d_part + kNormBlocks, 1, ncclFloat64, ncclSum, c->nccl, s) !=
          ncclSuccess)
    return fcg_device_error();
  if (hipMemcpyAsync(h_res, d_part + kNormBlocks, sizeof(double), hipMemcpyDeviceToHost, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return fcg_device_error();
  *out = std::sqrt(*h_res);
  return FCG_OK;
}

}  // extern "C"
