"""Solid statics Newton loop on the device around the assembly.

Mirrors the static step of 4C's structure_new time integrator with a NOX full Newton:
  set_state(u) -> Discretization::evaluate(struct_calc_nlnstiff)   fcg_evaluate_device (OVERWRITE)
  r = f_int - f_ext                                                 Structure::assemble_force,
                                                                    4C_structure_new_model_evaluator_structure.cpp:245-261
  Dirichlet on r (reaction forces kept) and K                       fcg_dirichlet_apply,
                                                                    4C_structure_new_dbc.cpp:221-262
  convergence: |r|_2 <= tol_res and |du|_2 <= tol_inc (NOX normF / normUpdate tests, combined "And")
  K du = -r                                                         fcg_pcg_solve (block-Jacobi PCG),
                                                                    relative tolerance from ForcingTerm
  u += du
Homogeneous Dirichlet conditions (the increments of the constrained DOFs are zero); single rank
(the PCG needs the matrix column map to be the row map).  u, f, K, f_ext and the work vectors stay
in HBM; torch only supplies the device buffers and the vector updates.
"""

import math
import warnings

import numpy as np
import torch

from . import fcg


class ForcingTerm:
    """Relative tolerance of each Newton step's linear solve: the "STRUCT NOX/Direction/Newton"
    forcing-term parameters of 4C (4C_inpar_solver_nonlin.cpp:48-71: "Forcing Term Method"
    Constant | Type 1 | Type 2, initial 0.1, minimum 1e-6, maximum 0.01, alpha 1.5, gamma 0.9),
    which 4C hands to Trilinos NOX (sha 06db4c85, not vendored).  NOX's
    Direction::Utils::InexactNewton::computeForcingTerm is the Eisenstat-Walker choice
    (SIAM J. Sci. Comput. 17, 1996), restated here:
      Constant: eta = the linear solver's own tolerance, every step;
      step 0:   eta = initial (no clamp);
      Type 1:   eta = |‖F_k‖ - ‖F_{k-1} + J_{k-1} d_{k-1}‖| / ‖F_{k-1}‖,
                raised to eta_{k-1}^((1+√5)/2) when that exceeds 0.1;
      Type 2:   eta = gamma (‖F_k‖ / ‖F_{k-1}‖)^alpha, raised to gamma eta_{k-1}^alpha when that
                exceeds 0.1;
    then (Types 1, 2) clamped to [minimum, maximum].  Parity: unpinned (no reference test uses
    Types 1/2); the converged displacement does not depend on eta (the Newton tests on |r| and
    |du| decide), which tests/test_newton_gpu.py checks against the Constant method."""

    METHODS = ("Constant", "Type 1", "Type 2")

    def __init__(self, method="Constant", constant=1e-13, initial=0.1, minimum=1e-6,
                 maximum=0.01, alpha=1.5, gamma=0.9):
        if method not in self.METHODS:
            raise ValueError(f"Forcing Term Method must be one of {self.METHODS}, not {method!r}")
        self.method, self.constant = method, constant
        self.initial, self.minimum, self.maximum = initial, minimum, maximum
        self.alpha, self.gamma = alpha, gamma
        self.eta = None

    def compute(self, niter, normf, normoldf=None, normpredf=None):
        """eta for the linear solve of Newton step `niter`: normf = ‖F_k‖, normoldf = ‖F_{k-1}‖,
        normpredf = ‖F_{k-1} + J_{k-1} d_{k-1}‖ (the previous linear residual; Type 1 only)."""
        if self.method == "Constant":
            self.eta = self.constant
        elif niter == 0:
            self.eta = self.initial
        else:
            eta_km1 = self.eta
            if self.method == "Type 1":
                eta = abs(normf - normpredf) / normoldf
                safe = eta_km1 ** ((1.0 + math.sqrt(5.0)) / 2.0)
            else:
                eta = self.gamma * (normf / normoldf) ** self.alpha
                safe = self.gamma * eta_km1 ** self.alpha
            if safe > 0.1:
                eta = max(eta, safe)
            self.eta = min(max(eta, self.minimum), self.maximum)
        return self.eta


def accept_linear_solve(solve, tol, it, rescue, rec):
    """Run a Newton step's linear solve and decide whether its direction is used, as NOX's
    Newton direction does with "Rescue Bad Newton Solve" (4C_inpar_solver_nonlin.cpp:65-69):
    a finite solution above the tolerance is kept when `rescue` (marked in `rec`, warned);
    otherwise, or for a non-finite residual or an indefinite preconditioner, raise."""
    from .multigrid import MultigridError
    try:
        lin_it, lin_res = solve()
    except MultigridError as e:
        if not rescue or e.relres is None:
            raise
        lin_it, lin_res = e.iterations, e.relres
    if lin_res <= tol:
        return lin_it, lin_res
    msg = (f"linear solve of Newton step {it} stopped at relative residual {lin_res:.3e} above "
           f"its tolerance {tol:.3e} ({lin_it} iterations)")
    if not rescue or not math.isfinite(lin_res):
        raise RuntimeError(msg)
    warnings.warn(msg + "; direction kept (Rescue Bad Newton Solve)", RuntimeWarning, stacklevel=3)
    rec["lin_rescued"] = True
    return lin_it, lin_res


class StaticNewton:
    def __init__(self, evaluator, fext_row, dbc_rows, tol_res=1e-10, tol_inc=1e-10, max_iter=20,
                 lin_rtol=1e-13, lin_max_iter=100000, forcing=None, linear_solver=None,
                 rescue_bad_newton_solve=True):
        """forcing: ForcingTerm (None: Constant at lin_rtol).  linear_solver: an object with
        solve(K, b, x, rtol, max_iter) -> (iterations, relative residual), e.g.
        multigrid.Multigrid (None: the library's block-Jacobi PCG).
        rescue_bad_newton_solve: NOX's "Rescue Bad Newton Solve" (4C default true,
        4C_inpar_solver_nonlin.cpp:65-69): a linear solve that stops above its tolerance still
        gives the step (recorded in history, with a warning); false: raise."""
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
        self.rescue = rescue_bad_newton_solve
        self.forcing = forcing if forcing is not None else ForcingTerm("Constant", constant=lin_rtol)
        self.linear_solver = linear_solver
        if linear_solver is not None and hasattr(linear_solver, "check_dirichlet"):
            linear_solver.check_dirichlet(dbc_rows)
        self.history = []

    def warm_up(self):
        """The torch operations of a Newton step launched once on scratch vectors (their code
        objects load at the first launch); no state is kept."""
        t = torch.zeros(16, dtype=torch.float64, device=self.dev)
        w = torch.zeros_like(t)
        torch.sub(t, w, out=w)
        torch.neg(w, out=w)
        t += w
        float(torch.linalg.vector_norm(t))
        torch.cuda.synchronize(self.dev)

    def linear_solve(self, b, x, rtol):
        """K x = b to |r| <= rtol |b| from x = 0; returns (iterations, relative residual)."""
        if self.linear_solver is not None:
            return self.linear_solver.solve(self.K, b, x, rtol, self.lin_max_iter)
        return self.ev.pcg_solve(self.K, b, x, rtol, self.lin_max_iter)

    def solve(self, u0=None):
        """Returns the converged displacement (row map, device tensor); raises if not converged."""
        u = (torch.zeros(self.n, dtype=torch.float64, device=self.dev) if u0 is None
             else torch.as_tensor(u0, dtype=torch.float64).to(self.dev).clone())
        self.history = []
        ndu = float("inf")
        nr_old = lin_abs = None
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
            eta = self.forcing.compute(it, nr, nr_old, lin_abs)
            if hasattr(self.linear_solver, "set_state"):
                self.linear_solver.set_state(u)  # a matrix-free level applies K(u)
            lin_it, lin_res = accept_linear_solve(lambda: self.linear_solve(self.r, self.du, eta),
                                                  eta, it, self.rescue, rec)
            nr_old, lin_abs = nr, lin_res * nr  # ‖F_k + J_k d_k‖ (full step, no line search)
            rec.update(lin_iter=lin_it, lin_relres=lin_res, eta=eta)
            self.history.append(rec)
            ndu = float(torch.linalg.vector_norm(self.du))
            u += self.du
            if nr == 0.0 and ndu == 0.0:
                return u
        raise RuntimeError(f"Newton did not converge in {self.max_iter} iterations: {self.history[-3:]}")
