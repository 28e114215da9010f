"""Static monolithic thermo-structure interaction (TSI) driver for the reference's known-answer
inputs.  TEST INFRASTRUCTURE ONLY.

Restates just enough of 4C's monolithic TSI around the element evaluations to run
tsi_heatflux_monolithic.dat and tsi_heatflux_flexoutsurf_monolithic.dat (both fields statics,
KINEM linear, ThermoStVenantKirchhoff + Fourier):
  * time loop t_n = n dt (TSI DYNAMIC TIMESTEP), loads evaluated at t_{n+1};
  * velocity of the quasi-static structure V = (D_{n+1} - D_n) / dt
    (TSI::Algorithm::calc_velocity, 4C_tsi_algorithm.cpp:386-397; used in statics,
    4C_tsi_monolithic.cpp:882-889);
  * residuals r_S = f_int,S(D, T) - f_ext,S and r_T = f_int,T(T, V) - f_ext,T, tangent
    [[k_SS, k_ST], [k_TS, k_TT]] (TSI::Monolithic::setup_system_matrix, 4C_tsi_monolithic.cpp:982-1005;
    k_ST and k_TS without time scaling in statics, :1742-1745, :1823-1826);
  * thermal surface Neumann (Thermo::TemperBoundaryImpl::evaluate_neumann,
    4C_thermo_ele_boundary_impl.cpp:504-576) and Dirichlet conditions read with 4C's geometric
    hierarchy (4C_fem_discretization_utils_dbc.cpp:164-406);
  * a full Newton loop per step, solved densely.
The element blocks come from an `assemble(d, T, v, dt)` callback: the CPU oracle (below) or the
device library (tests/test_tsi.py).
"""

import numpy as np

import oracle_lib as orc
from fe_driver import HEX27_SURFACES, Problem, make_function, quad_rule, quad_shape

_DBC_LEVELS = (("VOL", "DVOL", 3), ("SURF", "DSURFACE", 2), ("LINE", "DLINE", 1),
               ("POINT", "DNODE", 0))


def dirichlet_dofs(fx, lid, ndof, thermo):
    """DOF indices (ndof per node, node-major) fixed by the DESIGN * [THERMO ]DIRICH conditions.
    Conditions are read volume -> surface -> line -> point; ONOFF 1 fixes a DOF, ONOFF 0 on a
    lower-dimensional entity releases a DOF fixed by a higher-dimensional one
    (4C_fem_discretization_utils_dbc.cpp:296-406).  Homogeneous values only."""
    toggle, level = {}, {}
    for name, topo, h in _DBC_LEVELS:
        key = f"DESIGN {name} {'THERMO ' if thermo else ''}DIRICH CONDITIONS"
        for c in fx["conditions"].get(key, []):
            assert all(v == 0.0 for v in c["val"][:ndof]), "only homogeneous DBC supported"
            for n in fx["topology"][topo][str(c["entity"])]:
                for d in range(ndof):
                    dof = ndof * lid[n] + d
                    cur = level.get(dof, 99)
                    if c["onoff"][d] == 0:
                        if h < cur:
                            toggle[dof] = 0
                            level[dof] = h
                    else:
                        toggle[dof] = 1
                        level[dof] = min(cur, h)
    return np.array(sorted(k for k, v in toggle.items() if v), dtype=np.int64)


class TsiProblem:
    def __init__(self, fx):
        self.fx = fx
        self.structure = Problem(fx)  # nodes, structural Neumann loads, functions
        self.lid = self.structure.lid
        self.X = self.structure.X
        self.nn = len(self.X)
        self.ns = 3 * self.nn
        mat = fx["material"]
        self.E, self.nu = mat["young"], mat["nue"]
        self.alpha, self.T0 = mat["thexpans"], mat["inittemp"]
        self.conduct = fx["thermo_material"]["conduct"]
        self.m = orc.st_modulus(self.E, self.nu, self.alpha)
        self.functs = {int(k): make_function(v) for k, v in fx.get("functions", {}).items()}
        tsi = fx["tsi_dynamic"]
        self.dt = float(tsi["TIMESTEP"])
        t_end = min(float(tsi["MAXTIME"]), int(tsi["NUMSTEP"]) * self.dt)
        self.nstep = int(round(t_end / self.dt))
        # initial temperature: zero_field or field_by_function (INITFUNCNO at t = 0)
        init = fx["thermal_dynamic"].get("INITIALFIELD", "zero_field")
        assert init in ("zero_field", "field_by_function"), init
        self.T_init = np.zeros(self.nn)
        if init == "field_by_function":
            f = self.functs[int(fx["thermal_dynamic"]["INITFUNCNO"])]
            self.T_init = np.array([f(x, 0.0) for x in self.X])
        self.dbc_s = dirichlet_dofs(fx, self.lid, 3, thermo=False)
        self.dbc_t = dirichlet_dofs(fx, self.lid, 1, thermo=True)
        shapes = {el["shape"] for el in fx["elements"]}
        assert len(shapes) == 1 and {el["kinem"] for el in fx["elements"]} == {"linear"}
        self.celltype = orc.HEX8 if shapes.pop() == "HEX8" else orc.HEX27
        self.elements = [[self.lid[n] for n in el["nodes"]] for el in fx["elements"]]

    def fext_s(self, t):
        return self.structure.fext(t)

    def fext_t(self, t):
        """Thermal surface Neumann (live heat flux): fext += N q fac functfac."""
        f = np.zeros(self.nn)
        nfn = 4 if self.celltype == orc.HEX8 else 9
        topo = self.fx["topology"]
        for c in self.fx["conditions"].get("DESIGN SURF THERMO NEUMANN CONDITIONS", []):
            if not c["onoff"][0]:
                continue
            nodeset = set(topo["DSURFACE"][str(c["entity"])])
            for el in self.fx["elements"]:
                for face in HEX27_SURFACES:
                    fn = [el["nodes"][i] for i in face[:nfn]]
                    if not set(fn) <= nodeset:
                        continue
                    x = self.X[[self.lid[n] for n in fn]]
                    xg, wg = quad_rule(nfn)
                    for (r, s), w in zip(xg, wg):
                        N, dN = quad_shape(nfn, r, s)
                        dxyz = dN @ x
                        g = dxyz @ dxyz.T
                        fac = w * np.sqrt(g[0, 0] * g[1, 1] - g[0, 1] * g[1, 0])
                        fid = c["funct"][0]
                        functfac = self.functs[fid](N @ x, t) if fid and fid > 0 else 1.0
                        q = c["val"][0] * fac * functfac
                        for k, n in enumerate(fn):
                            f[self.lid[n]] += N[k] * q
        return f

    def assemble_oracle(self, d, T, v):
        """Dense k_SS, k_ST, k_TS, k_TT, f_S, f_T from the CPU oracle (statics: timefac = 1,
        timefac_d = 1/dt, 4C_thermo_ele_impl.cpp:1096-1104)."""
        ns, nn = self.ns, self.nn
        Kss, Kst = np.zeros((ns, ns)), np.zeros((ns, nn))
        Kts, Ktt = np.zeros((nn, ns)), np.zeros((nn, nn))
        fs, fT = np.zeros(ns), np.zeros(nn)
        for en in self.elements:
            en = np.asarray(en)
            idx = (3 * en[:, None] + np.arange(3)).ravel()
            Xe, de, Te, ve = self.X[en], d[idx], T[en], v[idx]
            err, Ke, fe, Kste = orc.tsi_solid_evaluate(self.celltype, self.E, self.nu, self.alpha,
                                                        self.T0, Xe, de, Te)
            assert err == 0, err
            err, Ktte, fTe, Ktse = orc.tsi_thermo_evaluate(self.celltype, self.conduct, self.m, Xe,
                                                          Te, ve, 1.0, 1.0 / self.dt)
            assert err == 0, err
            Kss[np.ix_(idx, idx)] += Ke
            Kst[np.ix_(idx, en)] += Kste
            Kts[np.ix_(en, idx)] += Ktse
            Ktt[np.ix_(en, en)] += Ktte
            fs[idx] += fe
            fT[en] += fTe
        return Kss, Kst, Kts, Ktt, fs, fT

    def solve(self, assemble=None, tol=1e-13, maxiter=30):
        """Returns (D, T) at the end time; `assemble(d, T, v)` defaults to the oracle."""
        assemble = assemble or self.assemble_oracle
        ns, nn = self.ns, self.nn
        d, T = np.zeros(ns), self.T_init.copy()
        fixed = np.concatenate([self.dbc_s, ns + self.dbc_t])
        free = np.setdiff1d(np.arange(ns + nn), fixed)
        self.history = []
        for step in range(1, self.nstep + 1):
            t = step * self.dt
            fes, fet = self.fext_s(t), self.fext_t(t)
            d_n = d.copy()
            for it in range(maxiter):
                v = (d - d_n) / self.dt
                Kss, Kst, Kts, Ktt, fs, fT = assemble(d, T, v)
                r = np.concatenate([fs - fes, fT - fet])
                A = np.block([[Kss, Kst], [Kts, Ktt]])
                dx = np.linalg.solve(A[np.ix_(free, free)], -r[free])
                x = np.concatenate([d, T])
                x[free] += dx
                d, T = x[:ns], x[ns:]
                ninc = np.linalg.norm(dx)
                if ninc <= tol * max(1.0, np.linalg.norm(x)):
                    break
            else:
                raise RuntimeError(f"TSI Newton did not converge in step {step}")
            self.history.append({"step": step, "iterations": it + 1})
        return d, T

    def result(self, d, T, r):
        if r["dof"] == "temp":
            return T[self.lid[r["node"]]]
        return d[3 * self.lid[r["node"]] + r["dof"]]
