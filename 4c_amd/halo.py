"""Multi-GPU glue: the row -> column import of the displacement state (Discretization::set_state,
4C_fem_discretization.cpp:503-548, an Epetra_Import over MPI in the reference) as one
`all_to_all_single` per evaluation over torch.distributed -- RCCL over xGMI with the "nccl"
backend on MI355X, gloo on CPU for the tests.

Only the ghost DOFs move (one ghost layer, SURVEY.md §8e option A): K and f_int need no
communication because every rank assembles exactly its owned rows.  The residual norm is a
scalar all-reduce.
"""

import numpy as np
import torch
import torch.distributed as dist


class HaloImport:
    """Plan + executor of u_row (owned DOFs) -> u_col (owned + ghost DOFs) on one rank."""

    def __init__(self, row_gid, col_gid, col_owner, rank, world, device):
        """row_gid: [n_rows] DOF gids owned here; col_gid: [n_cols] DOF gids of the column map;
        col_owner: [n_cols] owning rank of every column DOF."""
        self.rank, self.world, self.device = rank, world, device
        row_gid = np.asarray(row_gid, dtype=np.int64)
        col_gid = np.asarray(col_gid, dtype=np.int64)
        col_owner = np.asarray(col_owner, dtype=np.int64)
        row_lid = {int(g): i for i, g in enumerate(row_gid)}
        own = col_owner == rank
        # owned columns: copy from the row vector
        self.own_col = torch.from_numpy(np.nonzero(own)[0]).to(device)
        self.own_row = torch.from_numpy(np.array([row_lid[int(g)] for g in col_gid[own]],
                                                 dtype=np.int64)).to(device)
        # ghost columns grouped by owner (ascending), the order of the receive buffer
        ghost = np.nonzero(~own)[0]
        order = np.lexsort((col_gid[ghost], col_owner[ghost]))
        ghost = ghost[order]
        self.recv_col = torch.from_numpy(ghost).to(device)
        recv_counts = np.bincount(col_owner[ghost], minlength=world).astype(np.int64)
        want = col_gid[ghost]
        # tell every owner which gids we want (sizes first, then the gid lists)
        cpu = torch.device("cpu") if dist.get_backend() == "gloo" else device
        rc = torch.from_numpy(recv_counts).to(cpu)
        sc = torch.empty_like(rc)
        dist.all_to_all_single(sc, rc)
        send_counts = sc.cpu().numpy()
        req = torch.empty(int(send_counts.sum()), dtype=torch.int64, device=cpu)
        dist.all_to_all_single(req, torch.from_numpy(want).to(cpu),
                               output_split_sizes=send_counts.tolist(),
                               input_split_sizes=recv_counts.tolist())
        req = req.cpu().numpy()
        self.send_row = torch.from_numpy(np.array([row_lid[int(g)] for g in req],
                                                  dtype=np.int64)).to(device)
        self.send_counts = send_counts.tolist()
        self.recv_counts = recv_counts.tolist()
        self.sendbuf = torch.empty(len(req), dtype=torch.float64, device=device)
        self.recvbuf = torch.empty(len(ghost), dtype=torch.float64, device=device)
        # gloo moves host tensors only: stage device buffers through the host (tests/rehearsals)
        self.staged = cpu.type != torch.device(device).type
        self.n_ghost = len(ghost)
        # Epetra-style column maps (the BoxMesh ones): owned columns first in row order, then the
        # ghosts grouped by owner in GID order -- the import is then one contiguous copy plus a
        # receive straight into the column vector's tail (no scatter kernels)
        n_own = int(own.sum())
        self.n_own = n_own
        self.contiguous = (np.array_equal(np.nonzero(own)[0], np.arange(n_own))
                           and np.array_equal(self.own_row.cpu().numpy(), np.arange(n_own))
                           and np.array_equal(ghost, np.arange(n_own, n_own + len(ghost))))

    def __call__(self, u_row, u_col):
        if self.contiguous:
            u_col[:self.n_own].copy_(u_row[:self.n_own])
        else:
            u_col.index_copy_(0, self.own_col, u_row.index_select(0, self.own_row))
        torch.index_select(u_row, 0, self.send_row, out=self.sendbuf)
        if self.world > 1 and self.contiguous and not self.staged:
            dist.all_to_all_single(u_col[self.n_own:], self.sendbuf,
                                   output_split_sizes=self.recv_counts,
                                   input_split_sizes=self.send_counts)
            return u_col
        if self.world > 1 and self.staged:
            rb = torch.empty(self.n_ghost, dtype=torch.float64)
            dist.all_to_all_single(rb, self.sendbuf.cpu(), output_split_sizes=self.recv_counts,
                                   input_split_sizes=self.send_counts)
            self.recvbuf.copy_(rb)
        elif self.world > 1:
            dist.all_to_all_single(self.recvbuf, self.sendbuf,
                                   output_split_sizes=self.recv_counts,
                                   input_split_sizes=self.send_counts)
        u_col.index_copy_(0, self.recv_col, self.recvbuf)
        return u_col


def col_owner_of(mesh):
    """Owning rank of every column DOF of a BoxMesh rank."""
    owner = np.empty(mesh.n_cols, dtype=np.int64)
    for d in range(3):
        owner[mesh.node_dof_col + d] = mesh.node_owner
    return owner


def residual_norm(f_row):
    """||f||_2 over all ranks (NOX norm, an Allreduce in the reference)."""
    s = torch.dot(f_row, f_row).reshape(1)
    if dist.is_initialized() and dist.get_world_size() > 1:
        if dist.get_backend() == "gloo" and s.device.type != "cpu":
            h = s.cpu()
            dist.all_reduce(h)
            s = h.to(s.device)
        else:
            dist.all_reduce(s)
    return torch.sqrt(s)
