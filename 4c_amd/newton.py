"""Solid statics Newton loop on the device around the assembly.

Mirrors the static step of 4C's structure_new time integrator with a NOX full Newton:
  set_state(u) -> Discretization::evaluate(struct_calc_nlnstiff)   fcg_evaluate_device (OVERWRITE)
  r = f_int - f_ext                                                 Structure::assemble_force,
                                                                    4C_structure_new_model_evaluator_structure.cpp:245-261
  Dirichlet on r (reaction forces kept) and K                       fcg_dirichlet_apply,
                                                                    4C_structure_new_dbc.cpp:221-262
  convergence: |r|_2 <= tol_res and |du|_2 <= tol_inc (NOX normF / normUpdate tests, combined "And")
  K du = -r                                                         fcg_pcg_solve (block-Jacobi PCG)
  u += du
Homogeneous Dirichlet conditions (the increments of the constrained DOFs are zero); single rank
(the PCG needs the matrix column map to be the row map).  u, f, K, f_ext and the work vectors stay
in HBM; torch only supplies the device buffers and the vector updates.
"""

import numpy as np
import torch

from . import fcg


class StaticNewton:
    def __init__(self, evaluator, fext_row, dbc_rows, tol_res=1e-10, tol_inc=1e-10, max_iter=20,
                 lin_rtol=1e-13, lin_max_iter=100000):
        info = evaluator.info
        self.ev = evaluator
        self.dev = torch.device("cuda", evaluator.device)
        self.n = int(info.n_rows)
        if int(info.n_cols) != self.n:
            raise ValueError("StaticNewton is single-rank: the column map must be the row map")
        self.nnz = int(info.nnz)
        f64 = dict(dtype=torch.float64, device=self.dev)
        self.fext = torch.as_tensor(np.asarray(fext_row, dtype=np.float64)).to(self.dev)
        self.dbc = torch.as_tensor(np.asarray(dbc_rows, dtype=np.int32)).to(self.dev)
        self.K = torch.empty(self.nnz, **f64)
        self.fint = torch.empty(self.n, **f64)
        self.r = torch.empty(self.n, **f64)
        self.du = torch.empty(self.n, **f64)
        self.freact = torch.zeros(self.n, **f64)
        self.tol_res, self.tol_inc, self.max_iter = tol_res, tol_inc, max_iter
        self.lin_rtol, self.lin_max_iter = lin_rtol, lin_max_iter
        self.history = []

    def solve(self, u0=None):
        """Returns the converged displacement (row map, device tensor); raises if not converged."""
        u = (torch.zeros(self.n, dtype=torch.float64, device=self.dev) if u0 is None
             else torch.as_tensor(u0, dtype=torch.float64).to(self.dev).clone())
        self.history = []
        ndu = float("inf")
        for it in range(self.max_iter + 1):
            self.ev.evaluate_device(fcg.CALC_NLNSTIFF, fcg.OVERWRITE, u, self.fint, self.K)
            torch.sub(self.fint, self.fext, out=self.r)
            self.ev.dirichlet_apply(self.dbc, self.K, self.r, self.freact)
            nr = float(torch.linalg.vector_norm(self.r))
            rec = {"iter": it, "norm_res": nr, "norm_inc": ndu if it else None}
            if it > 0 and nr <= self.tol_res and ndu <= self.tol_inc:
                self.history.append(rec)
                return u
            torch.neg(self.r, out=self.r)
            lin_it, lin_res = self.ev.pcg_solve(self.K, self.r, self.du, self.lin_rtol,
                                                self.lin_max_iter)
            rec.update(lin_iter=lin_it, lin_relres=lin_res)
            self.history.append(rec)
            ndu = float(torch.linalg.vector_norm(self.du))
            u += self.du
            if nr == 0.0 and ndu == 0.0:
                return u
        raise RuntimeError(f"Newton did not converge in {self.max_iter} iterations: {self.history[-3:]}")
