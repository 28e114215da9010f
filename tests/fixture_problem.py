"""A reference input fixture (tests/golden/*.json) as an fcg discretization: CSR of the element
couplings, external load through the library's Neumann routines, Dirichlet row LIDs.
TEST INFRASTRUCTURE (the face search reuses tests/fe_driver.py)."""
import importlib

import numpy as np

from fe_driver import HEX27_SURFACES, Problem

fcg = importlib.import_module("4c_amd").fcg


def celltype_of(fx):
    shapes = {el["shape"] for el in fx["elements"]}
    assert len(shapes) == 1, shapes
    return fcg.HEX8 if shapes.pop() == "HEX8" else fcg.HEX27


def kinematics_of(fx):
    k = {el["kinem"] for el in fx["elements"]}
    assert len(k) == 1, k
    return fcg.LINEAR if k.pop() == "linear" else fcg.TOTLAG


def discretization(prob, lattice=False):
    ct = celltype_of(prob.fx)
    en = [[prob.lid[n] for n in el["nodes"]] for el in prob.fx["elements"]]
    return fcg.Discretization.from_elements(ct, en, prob.X, lattice=lattice)


def fext(prob, t):
    """Surface + volume Neumann through fcg_neumann_surface / fcg_neumann_volume."""
    fx = prob.fx
    ct = celltype_of(fx)
    nfn = 4 if ct == fcg.HEX8 else 9
    dof_row = 3 * np.arange(len(prob.X), dtype=np.int32)
    f = np.zeros(prob.ndof)
    fn = (lambda fid, x, tt: prob.functs[fid](x, tt)) if prob.functs else None
    conds, topo = fx["conditions"], fx["topology"]
    for c in conds.get("DESIGN SURF NEUMANN CONDITIONS", []):
        nodeset = set(topo["DSURFACE"][str(c["entity"])])
        faces = []
        for el in fx["elements"]:
            for face in HEX27_SURFACES:
                fnod = [el["nodes"][i] for i in face[:nfn]]
                if set(fnod) <= nodeset:
                    faces.append([prob.lid[n] for n in fnod])
        if faces:
            fcg.neumann_surface(ct, np.array(faces), prob.X, dof_row, c["onoff"][:3], c["val"][:3], f,
                                funct=c["funct"][:3], fn=fn, time=t)
    for c in conds.get("DESIGN VOL NEUMANN CONDITIONS", []):
        en = np.array([[prob.lid[n] for n in el["nodes"]] for el in fx["elements"]])
        fcg.neumann_volume(ct, en, prob.X, dof_row, c["onoff"][:3], c["val"][:3], f,
                           funct=c["funct"][:3], fn=fn, time=t)
    return f


def end_time(fx):
    t_end = float(fx["dynamic"].get("MAXTIME", 1.0))
    nstep = int(fx["dynamic"].get("NUMSTEP", 1))
    dt = float(fx["dynamic"].get("TIMESTEP", 1.0))
    return min(t_end, nstep * dt)


def problem(fx):
    return Problem(fx)
