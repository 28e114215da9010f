// fcg_plan.cpp -- host-side communication plans of the multi-GPU path (no device code, so the
// CPU tests drive them with gloo through the exchange callback).
//
//   fcg_import_plan_build: what Epetra_Import(colmap, rowmap) computes for
//       Discretization::set_state (4C_fem_discretization.cpp:542-548): the columns this rank owns
//       (same / permuted LIDs) and, per peer, the ghost columns it receives and the owned rows it
//       sends.  Epetra asks its directory for the owners; 4C knows them (node->owner()), so the
//       caller passes col_owner and one request exchange tells every owner what to send.
//   fcg_shared_plan_build: the interface of a strict element partition (SURVEY §8e option B) --
//       every DOF held by some rank as an extended (non-owned) row -- numbered globally by
//       (owner rank, GID) so that one all-reduce buffer serves all ranks
//       (Core::Communication::sum_all, 4C_comm_mpi_utils.hpp:294-306, on that buffer).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "fourc_gpu.h"

namespace {

struct ImportStorage {
  std::vector<int32_t> permute_from, permute_to, send_row, recv_col;
  std::vector<int64_t> send_counts, recv_counts;
};

struct SharedStorage {
  std::vector<int32_t> row;
  std::vector<int64_t> pos;
};

struct AnyStorage {
  int kind = 0;  // 1 = import, 2 = shared
  ImportStorage imp;
  SharedStorage sh;
};

// counts exchange: every rank tells every peer how many items follow
bool exchange_counts(int nranks, const std::vector<int64_t>& send, std::vector<int64_t>& recv,
    fcg_alltoallv_fn xchg, void* user)
{
  std::vector<int64_t> ones(nranks, 1);
  recv.assign(nranks, 0);
  return xchg(send.data(), ones.data(), recv.data(), ones.data(), sizeof(int64_t), user) == 0;
}

int64_t total(const std::vector<int64_t>& v)
{
  int64_t s = 0;
  for (int64_t x : v) s += x;
  return s;
}

}  // namespace

extern "C" {

void fcg_plan_free(void* storage) { delete static_cast<AnyStorage*>(storage); }

int fcg_import_plan_build(int rank, int nranks, int64_t n_rows, const int32_t* row_gid,
    int64_t n_cols, const int32_t* col_gid, const int32_t* col_owner, fcg_alltoallv_fn xchg,
    void* user, fcg_import_plan* out, void** storage)
{
  if (!out || !storage || !xchg || nranks < 1 || rank < 0 || rank >= nranks || n_rows < 0 ||
      n_cols < 0 || (n_rows && !row_gid) || (n_cols && (!col_gid || !col_owner)))
    return FCG_ERR_ARG;
  *storage = nullptr;
  auto* S = new AnyStorage();
  S->kind = 1;
  ImportStorage& P = S->imp;
  std::unordered_map<int32_t, int32_t> row_lid;
  row_lid.reserve(size_t(n_rows) * 2);
  for (int64_t i = 0; i < n_rows; ++i) row_lid.emplace(row_gid[i], int32_t(i));
  // owned columns: the longest common prefix is "same", the rest permuted (Epetra's split)
  int64_t n_same = 0;
  while (n_same < n_cols && n_same < n_rows && col_owner[n_same] == rank &&
         col_gid[n_same] == row_gid[n_same])
    ++n_same;
  std::vector<std::vector<int32_t>> want(nranks);  // column LIDs received from each owner
  bool bad = false;
  for (int64_t c = n_same; c < n_cols && !bad; ++c)
  {
    const int32_t o = col_owner[c];
    if (o < 0 || o >= nranks)
      bad = true;
    else if (o == rank)
    {
      auto it = row_lid.find(col_gid[c]);
      if (it == row_lid.end())
        bad = true;  // an owned column must be a row of this rank
      else
      {
        P.permute_from.push_back(it->second);
        P.permute_to.push_back(int32_t(c));
      }
    }
    else
      want[o].push_back(int32_t(c));
  }
  // a failing rank still takes part in both exchanges (the peers block on them)
  P.recv_counts.assign(nranks, 0);
  std::vector<int32_t> req;  // GIDs asked from each owner, in rank order
  for (int p = 0; p < nranks; ++p)
  {
    std::sort(want[p].begin(), want[p].end());  // ascending column LID (Epetra: by GID within owner)
    P.recv_counts[p] = int64_t(want[p].size());
    for (int32_t c : want[p])
    {
      P.recv_col.push_back(c);
      req.push_back(col_gid[c]);
    }
  }
  if (!exchange_counts(nranks, P.recv_counts, P.send_counts, xchg, user))
  {
    delete S;
    return FCG_ERR_DEVICE;
  }
  std::vector<int32_t> asked(total(P.send_counts));
  if (xchg(req.data(), P.recv_counts.data(), asked.data(), P.send_counts.data(), sizeof(int32_t),
          user) != 0)
  {
    delete S;
    return FCG_ERR_DEVICE;
  }
  P.send_row.resize(asked.size());
  for (size_t i = 0; i < asked.size() && !bad; ++i)
  {
    auto it = row_lid.find(asked[i]);
    if (it == row_lid.end())
      bad = true;  // a peer asks for a DOF this rank does not own: inconsistent owners
    else
      P.send_row[i] = it->second;
  }
  if (bad)
  {
    delete S;
    return FCG_ERR_ARG;
  }
  out->nranks = nranks;
  out->rank = rank;
  out->n_rows = n_rows;
  out->n_cols = n_cols;
  out->n_same = n_same;
  out->n_permute = int64_t(P.permute_from.size());
  out->permute_from = P.permute_from.data();
  out->permute_to = P.permute_to.data();
  out->send_counts = P.send_counts.data();
  out->send_row = P.send_row.data();
  out->recv_counts = P.recv_counts.data();
  out->recv_col = P.recv_col.data();
  *storage = S;
  return FCG_OK;
}

int fcg_shared_plan_build(int rank, int nranks, int64_t n_owned_rows, const int32_t* owned_gid,
    int64_t n_ext_rows, const int32_t* ext_gid, const int32_t* ext_owner, fcg_alltoallv_fn xchg,
    void* user, fcg_shared_plan* out, void** storage)
{
  if (!out || !storage || !xchg || nranks < 1 || rank < 0 || rank >= nranks || n_owned_rows < 0 ||
      n_ext_rows < 0 || (n_owned_rows && !owned_gid) || (n_ext_rows && (!ext_gid || !ext_owner)))
    return FCG_ERR_ARG;
  *storage = nullptr;
  bool bad = false;
  // extended rows grouped by owner, GID order inside a group
  std::vector<std::vector<int64_t>> by_owner(nranks);  // ext row indices
  for (int64_t k = 0; k < n_ext_rows; ++k)
  {
    const int32_t o = ext_owner[k];
    if (o < 0 || o >= nranks || o == rank)
    {
      bad = true;
      continue;
    }
    by_owner[o].push_back(k);
  }
  std::vector<int64_t> ask_counts(nranks, 0);
  std::vector<int32_t> ask;
  std::vector<int64_t> ask_row;  // ext index of every asked GID, same order
  for (int p = 0; p < nranks; ++p)
  {
    std::sort(by_owner[p].begin(), by_owner[p].end(),
        [&](int64_t a, int64_t b) { return ext_gid[a] < ext_gid[b]; });
    ask_counts[p] = int64_t(by_owner[p].size());
    for (int64_t k : by_owner[p])
    {
      ask.push_back(ext_gid[k]);
      ask_row.push_back(k);
    }
  }
  std::vector<int64_t> req_counts;
  if (!exchange_counts(nranks, ask_counts, req_counts, xchg, user)) return FCG_ERR_DEVICE;
  std::vector<int32_t> req(total(req_counts));
  if (xchg(ask.data(), ask_counts.data(), req.data(), req_counts.data(), sizeof(int32_t), user) != 0)
    return FCG_ERR_DEVICE;
  // owned interface list: the distinct requested GIDs, ascending
  std::unordered_map<int32_t, int32_t> owned_lid;
  owned_lid.reserve(size_t(n_owned_rows) * 2);
  for (int64_t i = 0; i < n_owned_rows; ++i) owned_lid.emplace(owned_gid[i], int32_t(i));
  std::vector<int32_t> mine(req);
  std::sort(mine.begin(), mine.end());
  mine.erase(std::unique(mine.begin(), mine.end()), mine.end());
  for (int32_t g : mine)
    if (owned_lid.find(g) == owned_lid.end()) bad = true;
  // global numbering: offset of this rank's block = sizes of the lower ranks' lists
  std::vector<int64_t> my_size(nranks, int64_t(mine.size())), sizes;
  if (!exchange_counts(nranks, my_size, sizes, xchg, user)) return FCG_ERR_DEVICE;
  int64_t offset = 0, n_global = 0;
  for (int p = 0; p < nranks; ++p)
  {
    if (p < rank) offset += sizes[p];
    n_global += sizes[p];
  }
  // reply with the positions of the requested GIDs, in request order
  std::vector<int64_t> reply(req.size());
  for (size_t i = 0; i < req.size(); ++i)
    reply[i] = offset + (std::lower_bound(mine.begin(), mine.end(), req[i]) - mine.begin());
  std::vector<int64_t> got(ask.size());
  if (xchg(reply.data(), req_counts.data(), got.data(), ask_counts.data(), sizeof(int64_t), user) != 0)
    return FCG_ERR_DEVICE;
  if (bad) return FCG_ERR_ARG;
  auto* S = new AnyStorage();
  S->kind = 2;
  SharedStorage& P = S->sh;
  for (size_t i = 0; i < mine.size(); ++i)
  {
    P.row.push_back(owned_lid[mine[i]]);
    P.pos.push_back(offset + int64_t(i));
  }
  for (size_t i = 0; i < ask.size(); ++i)
  {
    P.row.push_back(int32_t(n_owned_rows + ask_row[i]));
    P.pos.push_back(got[i]);
  }
  out->nranks = nranks;
  out->rank = rank;
  out->n_global = n_global;
  out->n_local = int64_t(P.row.size());
  out->n_owned = int64_t(mine.size());
  out->row = P.row.data();
  out->pos = P.pos.data();
  *storage = S;
  return FCG_OK;
}

}  // extern "C"
