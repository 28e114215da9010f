"""Drivers for the reference known answers that need more than displacements: reaction forces,
the analytical-error CSV and the STRUCTURE DOMAIN (GridGenerator) input.  TEST INFRASTRUCTURE.

Each driver takes an `assemble` callback, so the same check runs on the oracle (CPU tests) and on
the library (GPU tests):
  * Problem-based (input meshes): assemble(u) -> (K dense, f_int), as fe_driver.Problem.assemble;
  * box-based (DOMAIN): assemble(mesh, u_col) -> (K values in the mesh's CSR, f_int owned rows).

Reaction forces follow Solid::Dbc::extract_freact (4C_structure_new_dbc.cpp:389-400): the
residual F = f_int - f_ext at the Dirichlet DOFs, scaled by -1, zero elsewhere.  The OP lines of
the RESULT DESCRIPTION sum / min / max a quantity over a condition's node set
(4C_structure_new_resulttest.cpp).
"""

import importlib

import numpy as np

fcg = importlib.import_module("4c_amd").fcg


def reactions(prob, u, assemble=None, t=1.0):
    """freact over all DOFs after the converged solve (zero off the Dirichlet DOFs)."""
    assemble = assemble or prob.assemble
    _, fint = assemble(u)
    F = fint - prob.fext(t)
    fr = np.zeros_like(F)
    dbc = prob.dirichlet_dofs()
    fr[dbc] = -F[dbc]
    return fr


def check_reactions(fx, prob, freact):
    """Every reactx/y/z line and OP line of the fixture; returns the list of failures."""
    bad = []
    for r in fx.get("reactions", []):
        got = freact[3 * prob.lid[r["node"]] + r["dof"]]
        if abs(got - r["value"]) > r["tol"]:
            bad.append((r, got))
    for r in fx.get("reaction_ops", []):
        nodes = fx["topology"][r["set"]][str(r["entity"])]
        vals = np.array([freact[3 * prob.lid[n] + r["dof"]] for n in nodes])
        got = {"sum": vals.sum(), "min": vals.min(), "max": vals.max()}[r["op"]]
        if abs(got - r["value"]) > r["tol"]:
            bad.append((r, got))
    return bad


def analytical_error(fx, prob, u):
    """struct_calc_analytical_error summed over the elements (calc_lib.hpp:1015-1060): integrated
    squared error against the analytical displacement function (time 0), integrated squared
    displacement and volume, at the stiffness Gauss rule; returns the CSV row's three values
    (displacement_error_l2_norm = sqrt of the first)."""
    import oracle_lib as orc
    from fe_driver import make_function
    fid = next(iter(fx["function_components"]))
    comp = [make_function(e) for e in fx["function_components"][fid]]
    err2 = disp2 = vol = 0.0
    for el in fx["elements"]:
        ct = orc.HEX8 if el["shape"] == "HEX8" else orc.HEX27
        idx = [prob.lid[n] for n in el["nodes"]]
        Xe = prob.X[idx]
        ue = u.reshape(-1, 3)[idx]
        gx, gw = orc.gauss_points(ct)
        for xi, w in zip(gx, gw):
            N = orc.shape(ct, xi)
            dN = orc.shape_deriv(ct, xi)
            fac = np.linalg.det(dN.T @ Xe) * w
            xg = N @ Xe
            ug = N @ ue
            ua = np.array([c(xg, 0.0) for c in comp])
            e = ua - ug
            err2 += e @ e * fac
            disp2 += ug @ ug * fac
            vol += fac
    return np.sqrt(err2), disp2, vol


# ----------------------------------------------------------------------------- DOMAIN input
def domain_meshes(fx, nranks):
    dom = fx["domain"]
    assert dom["shape"] == "HEX8"
    return [fcg.BoxMesh(fcg.HEX8, dom["intervals"], lower=dom["lower_bound"],
                        upper=dom["upper_bound"], rotation=dom.get("rotation", (0.0, 0.0, 0.0)),
                        rank=r, nranks=nranks) for r in range(nranks)]


def _node_set(fx, mesh, geo):
    """CORNER / SIDE node sets of a DOMAIN input on the mesh's column nodes."""
    lo, hi = np.array(fx["domain"]["lower_bound"]), np.array(fx["domain"]["upper_bound"])
    X = mesh.node_x
    sel = np.ones(len(X), dtype=bool)
    for s in geo["spec"]:
        d = "xyz".index(s[0])
        sel &= np.isclose(X[:, d], lo[d] if s[1] == "-" else hi[d], rtol=0, atol=1e-12)
    return np.nonzero(sel)[0]


def domain_solve(fx, meshes, assemble):
    """One Newton iteration from u = 0 (the input's MAXITER) of the DOMAIN problem, assembled rank
    by rank (owned rows, the reference's MPI semantics) into a global system by DOF GID.  Returns
    {dof gid: displacement}."""
    assert int(fx["dynamic"].get("MAXITER", 1)) == 1
    gids = np.unique(np.concatenate([m.row_gid for m in meshes]))
    pos = {int(g): i for i, g in enumerate(gids)}
    n = len(gids)
    K = np.zeros((n, n))
    fext = np.zeros(n)
    fixed = set()
    conds = fx["conditions"]
    for m in meshes:
        u0 = np.zeros(m.n_cols)
        Kv, fint = assemble(m, u0)
        rows = np.repeat(np.arange(m.n_rows), np.diff(m.rowptr))
        gr = np.array([pos[int(g)] for g in m.row_gid])
        gc = np.array([pos[int(g)] for g in m.col_gid[m.col_lid]])
        np.add.at(K, (gr[rows], gc), Kv)
        # u = 0: f_int is rounding only (hex8 TotLag takes F from current coordinates), but the
        # reference's first iteration solves K du = -(f_int - f_ext) with it, so it stays in
        fe = -fint
        for c in conds.get("DESIGN SURF NEUMANN CONDITIONS", []):
            geo = [g for g in fx["geometry_sets"] if g["set"] == "DSURFACE" and g["entity"] == c["entity"]]
            assert len(geo) == 1 and geo[0]["kind"] == "SIDE" and len(geo[0]["spec"]) == 1
            s = geo[0]["spec"][0]
            d = "xyz".index(s[0])
            # the side's faces: the column elements at the box end, their face in 4C node order
            end = 0 if s[1] == "-" else fx["domain"]["intervals"][d] - 1
            face = {("x", "+"): [1, 2, 6, 5], ("x", "-"): [0, 4, 7, 3], ("y", "+"): [2, 3, 7, 6],
                    ("y", "-"): [0, 1, 5, 4], ("z", "+"): [4, 5, 6, 7], ("z", "-"): [0, 3, 2, 1]}[(s[0], s[1])]
            faces = np.array([m.ele_nodes[e][face] for e in range(m.n_ele) if m.ele_ijk[e][d] == end])
            if len(faces):
                fcg.neumann_surface(fcg.HEX8, faces, m.node_x, m.node_dof_row, c["onoff"][:3],
                                    c["val"][:3], fe)
        fext[gr] += fe
        for key, kind in (("DESIGN POINT DIRICH CONDITIONS", "DNODE"),
                          ("DESIGN SURF DIRICH CONDITIONS", "DSURFACE")):
            for c in conds.get(key, []):
                assert all(v == 0.0 for v in c["val"])
                for g in fx["geometry_sets"]:
                    if g["set"] == kind and g["entity"] == c["entity"]:
                        for nd in _node_set(fx, m, g):
                            for dd in range(3):
                                if c["onoff"][dd]:
                                    fixed.add(pos[int(m.col_gid[m.node_dof_col[nd] + dd])])
    fixed = np.array(sorted(fixed))
    free = np.setdiff1d(np.arange(n), fixed)
    u = np.zeros(n)
    u[free] = np.linalg.solve(K[np.ix_(free, free)], fext[free])
    return {int(g): u[i] for i, g in enumerate(gids)}


def check_domain_results(fx, u_by_gid):
    """RESULT DESCRIPTION NODE ids are 1-based node GIDs; DOF gid = 3 gid + d (first gid 0)."""
    bad = []
    for r in fx["results"]:
        got = u_by_gid[3 * (r["node"] - 1) + r["dof"]]
        if abs(got - r["value"]) > r["tol"]:
            bad.append((r, got))
    return bad
