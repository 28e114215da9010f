"""Tiny dense FE driver used to pin the oracle end-to-end against the reference's RESULT
DESCRIPTION values (TEST INFRASTRUCTURE ONLY).

It restates just enough of 4C around the hot path to run the known-answer inputs:
  * live surface Neumann (4C_solid_3D_ele_surface_evaluate.cpp:262-320; quad_4point / quad_9point
    rules with the reference's truncated constants, 4C_fem_general_utils_integration.cpp:6151-6234;
    quad4/quad9 shape functions 4C_fem_general_utils_fem_shapefunctions.hpp:2003-2087,2148-2274),
  * live volume Neumann (4C_solid_3D_ele_neumann_evaluator.cpp:45-110),
  * Dirichlet elimination and a full Newton loop (statics) solved densely.
The element tangent and internal force come from the oracle (oracle_lib.solid_evaluate).
"""

import numpy as np

import oracle_lib as orc

# hex27 surface connectivity (4C_fem_general_utils_local_connectivity_matrices.hpp:51-54);
# the hex8 faces are the first four entries of each row.
HEX27_SURFACES = [[0, 3, 2, 1, 11, 10, 9, 8, 20], [0, 1, 5, 4, 8, 13, 16, 12, 21],
                  [1, 2, 6, 5, 9, 14, 17, 13, 22], [2, 3, 7, 6, 10, 15, 18, 14, 23],
                  [0, 4, 7, 3, 12, 19, 15, 11, 24], [4, 5, 6, 7, 16, 17, 18, 19, 25]]


def quad_rule(n):
    if n == 4:
        a = 0.5773502691896
        xg = [(-a, -a), (a, -a), (a, a), (-a, a)]
        return xg, [1.0] * 4
    b = 0.7745966692415
    w1, w2 = 0.5555555555556, 0.8888888888889
    xg = [(-b, -b), (b, -b), (b, b), (-b, b), (0.0, -b), (b, 0.0), (0.0, b), (-b, 0.0), (0.0, 0.0)]
    w = [w1 * w1] * 4 + [w2 * w1, w1 * w2, w2 * w1, w1 * w2, w2 * w2]
    return xg, w


def quad_shape(n, r, s):
    if n == 4:
        rp, rm, sp, sm = 1.0 + r, 1.0 - r, 1.0 + s, 1.0 - s
        N = np.array([0.25 * rm * sm, 0.25 * rp * sm, 0.25 * rp * sp, 0.25 * rm * sp])
        dN = np.array([[-0.25 * sm, 0.25 * sm, 0.25 * sp, -0.25 * sp],
                       [-0.25 * rm, -0.25 * rp, 0.25 * rp, 0.25 * rm]])
        return N, dN
    rp, rm, sp, sm = 1.0 + r, 1.0 - r, 1.0 + s, 1.0 - s
    r2, s2 = 1.0 - r * r, 1.0 - s * s
    rh, sh = 0.5 * r, 0.5 * s
    rs = rh * sh
    rhp, rhm, shp, shm = r + 0.5, r - 0.5, s + 0.5, s - 0.5
    N = np.array([rs * rm * sm, -rs * rp * sm, rs * rp * sp, -rs * rm * sp, -sh * sm * r2,
                  rh * rp * s2, sh * sp * r2, -rh * rm * s2, r2 * s2])
    dN = np.array([[-rhm * sh * sm, -rhp * sh * sm, rhp * sh * sp, rhm * sh * sp, 2.0 * r * sh * sm,
                    rhp * s2, -2.0 * r * sh * sp, rhm * s2, -2.0 * r * s2],
                   [-shm * rh * rm, shm * rh * rp, shp * rh * rp, -shp * rh * rm, shm * r2,
                    -2.0 * s * rh * rp, shp * r2, 2.0 * s * rh * rm, -2.0 * s * r2]])
    return N, dN


def make_function(expr):
    code = compile(expr, "<funct>", "eval")

    def f(x, t):
        return float(eval(code, {"__builtins__": {}}, {"x": x[0], "y": x[1], "z": x[2], "t": t}))
    return f


class Problem:
    def __init__(self, fx):
        self.fx = fx
        self.node_ids = sorted(int(k) for k in fx["nodes"])
        self.lid = {n: i for i, n in enumerate(self.node_ids)}
        self.X = np.array([fx["nodes"][str(n)] for n in self.node_ids])
        self.ndof = 3 * len(self.node_ids)
        self.E = fx["material"]["young"]
        self.nu = fx["material"]["nue"]
        self.material = (orc.MAT_NEOHOOKE if fx["material"].get("type") == "elasthyper_coupneohooke"
                         else orc.MAT_STVK)
        self.functs = {int(k): make_function(v) for k, v in fx.get("functions", {}).items()}

    def element_dofs(self, el):
        return np.array([3 * self.lid[n] + d for n in el["nodes"] for d in range(3)])

    def celltype(self, el):
        return orc.HEX8 if el["shape"] == "HEX8" else orc.HEX27

    def assemble(self, u):
        K = np.zeros((self.ndof, self.ndof))
        f = np.zeros(self.ndof)
        for el in self.fx["elements"]:
            ct = self.celltype(el)
            kin = orc.LINEAR if el["kinem"] == "linear" else orc.TOTLAG
            idx = self.element_dofs(el)
            Xe = self.X[[self.lid[n] for n in el["nodes"]]]
            err, Ke, fe = orc.solid_evaluate(ct, kin, self.E, self.nu, Xe, u[idx],
                                             material=self.material)
            assert err == 0, err
            K[np.ix_(idx, idx)] += Ke
            f[idx] += fe
        return K, f

    def funct_factor(self, fid, x, t):
        if fid and fid > 0:
            return self.functs[fid](x, t)
        return 1.0

    def fext(self, t):
        f = np.zeros(self.ndof)
        conds = self.fx["conditions"]
        topo = self.fx["topology"]
        for c in conds.get("DESIGN SURF NEUMANN CONDITIONS", []):
            nodeset = set(topo["DSURFACE"][str(c["entity"])])
            for el in self.fx["elements"]:
                nf = 4 if el["shape"] == "HEX8" else 9
                for face in HEX27_SURFACES:
                    fn = [el["nodes"][i] for i in face[:nf]]
                    if not set(fn) <= nodeset:
                        continue
                    x = self.X[[self.lid[n] for n in fn]]
                    xg, wg = quad_rule(nf)
                    for (r, s), w in zip(xg, wg):
                        N, dN = quad_shape(nf, r, s)
                        dxyz = dN @ x
                        g = dxyz @ dxyz.T
                        detA = np.sqrt(g[0, 0] * g[1, 1] - g[0, 1] * g[1, 0])
                        xgp = N @ x
                        for dof in range(3):
                            if c["onoff"][dof]:
                                fac = w * detA * c["val"][dof] * self.funct_factor(c["funct"][dof], xgp, t)
                                for k, n in enumerate(fn):
                                    f[3 * self.lid[n] + dof] += N[k] * fac
        for c in conds.get("DESIGN VOL NEUMANN CONDITIONS", []):
            for el in self.fx["elements"]:
                ct = self.celltype(el)
                Xe = self.X[[self.lid[n] for n in el["nodes"]]]
                gx, gw = orc.gauss_points(ct)
                for xi, w in zip(gx, gw):
                    N = orc.shape(ct, xi)
                    dN = orc.shape_deriv(ct, xi)
                    J = dN.T @ Xe
                    fac = np.linalg.det(J) * w
                    xgp = N @ Xe
                    for i in range(3):
                        if c["onoff"][i]:
                            v = c["val"][i] * self.funct_factor(c["funct"][i], xgp, t) * fac
                            for k, n in enumerate(el["nodes"]):
                                f[3 * self.lid[n] + i] += N[k] * v
        return f

    def dirichlet_dofs(self):
        fixed = set()
        topo = self.fx["topology"]
        kinds = {"DESIGN POINT DIRICH CONDITIONS": "DNODE", "DESIGN LINE DIRICH CONDITIONS": "DLINE",
                 "DESIGN SURF DIRICH CONDITIONS": "DSURFACE", "DESIGN VOL DIRICH CONDITIONS": "DVOL"}
        for key, kind in kinds.items():
            for c in self.fx["conditions"].get(key, []):
                assert all(v == 0.0 for v in c["val"]), "only homogeneous DBC supported"
                for n in topo[kind][str(c["entity"])]:
                    for d in range(3):
                        if c["onoff"][d]:
                            fixed.add(3 * self.lid[n] + d)
        return np.array(sorted(fixed), dtype=np.int64)

    def solve_statics(self, t=1.0, tol=1e-13, maxiter=50, nsteps=1, assemble=None):
        """Full Newton per load step at t_k = k t / nsteps (the reference's TIMESTEP sequence for
        large deformations); `assemble(u) -> (K, fint)` defaults to the oracle."""
        assemble = assemble or self.assemble
        u = np.zeros(self.ndof)
        fixed = self.dirichlet_dofs()
        free = np.setdiff1d(np.arange(self.ndof), fixed)
        for k in range(1, nsteps + 1):
            fe = self.fext(t * k / nsteps)
            for _ in range(maxiter):
                K, fint = assemble(u)
                r = fint - fe
                du = np.linalg.solve(K[np.ix_(free, free)], -r[free])
                u[free] += du
                if np.linalg.norm(du) < tol * max(1.0, np.linalg.norm(u)):
                    break
            else:
                raise RuntimeError(f"Newton did not converge in load step {k}")
        return u

    def disp(self, u, node, dof):
        return u[3 * self.lid[node] + dof]
