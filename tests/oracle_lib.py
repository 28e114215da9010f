"""ctypes binding of the CPU oracle (oracle/fourc_oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "_build", "liborc.so")

HEX8, HEX27 = 0, 1
LINEAR, TOTLAG = 0, 1
MAT_STVK, MAT_NEOHOOKE = 0, 1

_lib = None

_dp = ctypes.POINTER(ctypes.c_double)
_i64p = ctypes.POINTER(ctypes.c_int64)
_i32p = ctypes.POINTER(ctypes.c_int32)
_ip = ctypes.POINTER(ctypes.c_int)


class OrcCsr(ctypes.Structure):
    _fields_ = [("n_rows", ctypes.c_int64), ("rowptr", _i64p), ("col_lid", _i32p),
                ("vals", _dp), ("row_lid_of_gid", _i32p), ("col_lid_of_gid", _i32p),
                ("max_gid", ctypes.c_int64)]


def build(force=False, extra_flags=None, out=None):
    """Build the oracle shared library with make (gcc).  Returns the library path."""
    target = out or LIB_PATH
    if force or not os.path.exists(target):
        if out is None and extra_flags is None:
            subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
        else:
            flags = ["-O3", "-fopenmp", "-fPIC", "-std=gnu11"] + list(extra_flags or [])
            os.makedirs(os.path.dirname(target), exist_ok=True)
            subprocess.run(["gcc"] + flags + ["-shared", "-o", target,
                                              os.path.join(ORACLE_DIR, "fourc_oracle.c"), "-lm"],
                           check=True)
    return target


def load(path=None):
    global _lib
    if path is None and _lib is not None:
        return _lib
    p = path or build()
    lib = ctypes.CDLL(p)
    lib.orc_gauss_points.argtypes = [ctypes.c_int, _dp, _dp]
    lib.orc_shape.argtypes = [ctypes.c_int, _dp, _dp]
    lib.orc_node_param_coords.argtypes = [ctypes.c_int, _dp]
    lib.orc_shape_deriv1.argtypes = [ctypes.c_int, _dp, _dp]
    lib.orc_stvk_evaluate.argtypes = [ctypes.c_double, ctypes.c_double, _dp, _dp, _dp]
    lib.orc_stvk_strain_energy.argtypes = [ctypes.c_double, ctypes.c_double, _dp]
    lib.orc_stvk_strain_energy.restype = ctypes.c_double
    lib.orc_solid_evaluate.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                       _dp, _dp, _dp, _dp]
    lib.orc_hex_element_nodeids.argtypes = [ctypes.c_int, ctypes.c_int64, _i32p, ctypes.c_int64, _i64p]
    lib.orc_lattice_node_coords.argtypes = [ctypes.c_int64, _i32p, ctypes.c_int64, _dp, _dp, _dp, _dp]
    lib.orc_box_section.argtypes = [_i32p, ctypes.c_int, ctypes.c_int, _i32p]
    lib.orc_solid_evaluate_mat.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                           ctypes.c_double, _dp, _dp, _dp, _dp]
    lib.orc_elasthyper_coupneohooke.argtypes = [ctypes.c_double, ctypes.c_double, _dp, _dp, _dp]
    lib.orc_discretization_evaluate_mat.argtypes = [
        ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int64,
        _i64p, ctypes.c_int64, _dp, _i64p, _i32p, ctypes.c_int64, ctypes.c_int, _dp,
        ctypes.POINTER(OrcCsr), _dp, _i64p]
    lib.orc_discretization_evaluate.argtypes = [
        ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int64, _i64p,
        ctypes.c_int64, _dp, _i64p, _i32p, ctypes.c_int64, ctypes.c_int, _dp,
        ctypes.POINTER(OrcCsr), _dp, _i64p]
    lib.orc_tsi_discretization_evaluate.argtypes = (
        [ctypes.c_int] + [ctypes.c_double] * 7 + [ctypes.c_int64, _i64p, _dp, _i64p, _i32p,
                                                 ctypes.c_int64, ctypes.c_int, _dp, _dp, _dp]
        + [ctypes.POINTER(OrcCsr)] * 4 + [_dp, _dp, _i64p])
    lib.orc_thermo_stvk_st_modulus.argtypes = [ctypes.c_double] * 3
    lib.orc_thermo_stvk_st_modulus.restype = ctypes.c_double
    lib.orc_tsi_solid_evaluate.argtypes = [ctypes.c_int] + [ctypes.c_double] * 4 + [_dp] * 6
    lib.orc_tsi_thermo_evaluate.argtypes = ([ctypes.c_int] + [ctypes.c_double] * 2 + [_dp] * 3 +
                                            [ctypes.c_double] * 2 + [_dp] * 3)
    if path is None:
        _lib = lib
    return lib


def ptr(a, t):
    return a.ctypes.data_as(t)


def gauss_points(celltype):
    lib = load()
    n = 8 if celltype == HEX8 else 27
    xi = np.zeros((n, 3))
    w = np.zeros(n)
    lib.orc_gauss_points(celltype, ptr(xi, _dp), ptr(w, _dp))
    return xi, w


def shape(celltype, xi):
    lib = load()
    n = 8 if celltype == HEX8 else 27
    N = np.zeros(n)
    lib.orc_shape(celltype, ptr(np.ascontiguousarray(xi, dtype=np.float64), _dp), ptr(N, _dp))
    return N


def shape_deriv(celltype, xi):
    """dN[node, d] (the oracle stores column-major 3 x n == row-major n x 3)."""
    lib = load()
    n = 8 if celltype == HEX8 else 27
    dN = np.zeros((n, 3))
    lib.orc_shape_deriv1(celltype, ptr(np.ascontiguousarray(xi, dtype=np.float64), _dp), ptr(dN, _dp))
    return dN


def node_param_coords(celltype):
    lib = load()
    n = 8 if celltype == HEX8 else 27
    buf = np.zeros((n, 3))
    lib.orc_node_param_coords(celltype, ptr(buf, _dp))
    return buf


def stvk(E, nu, gl):
    lib = load()
    gl = np.ascontiguousarray(gl, dtype=np.float64)
    s = np.zeros(6)
    c = np.zeros(36)
    lib.orc_stvk_evaluate(E, nu, ptr(gl, _dp), ptr(s, _dp), ptr(c, _dp))
    return s, c.reshape(6, 6).T


def stvk_energy(E, nu, gl):
    return load().orc_stvk_strain_energy(E, nu, ptr(np.ascontiguousarray(gl, dtype=np.float64), _dp))


def solid_evaluate(celltype, kinem, E, nu, X, u, want_k=True, material=MAT_STVK):
    """Returns (err, Ke (3n x 3n), fe (3n))."""
    lib = load()
    n = 8 if celltype == HEX8 else 27
    X = np.ascontiguousarray(X, dtype=np.float64).reshape(n, 3)
    u = np.ascontiguousarray(u, dtype=np.float64).reshape(n, 3)
    Ke = np.zeros(9 * n * n)
    fe = np.zeros(3 * n)
    err = lib.orc_solid_evaluate_mat(celltype, kinem, material, E, nu, ptr(X, _dp), ptr(u, _dp),
                                     ptr(Ke, _dp) if want_k else None, ptr(fe, _dp))
    return err, Ke.reshape(3 * n, 3 * n).T.copy(), fe


def hex_nodeids(celltype, eleid, interval, offset):
    lib = load()
    n = 8 if celltype == HEX8 else 27
    out = np.zeros(n, dtype=np.int64)
    iv = np.asarray(interval, dtype=np.int32)
    lib.orc_hex_element_nodeids(celltype, eleid, ptr(iv, _i32p), offset, ptr(out, _i64p))
    return out


def node_coords(gid, interval, offset, lo, hi, rot=(0.0, 0.0, 0.0)):
    lib = load()
    x = np.zeros(3)
    iv = np.asarray(interval, dtype=np.int32)
    lo = np.asarray(lo, dtype=np.float64)
    hi = np.asarray(hi, dtype=np.float64)
    rot = np.asarray(rot, dtype=np.float64)
    lib.orc_lattice_node_coords(gid, ptr(iv, _i32p), offset, ptr(lo, _dp), ptr(hi, _dp),
                                ptr(rot, _dp), ptr(x, _dp))
    return x


def box_section(interval, nproc, rank):
    lib = load()
    iv = np.asarray(interval, dtype=np.int32)
    r = np.zeros(6, dtype=np.int32)
    if lib.orc_box_section(ptr(iv, _i32p), nproc, rank, ptr(r, _i32p)) != 0:
        raise ValueError("cannot split nproc")
    return r


def st_modulus(E, nu, alpha):
    return load().orc_thermo_stvk_st_modulus(E, nu, alpha)


def tsi_solid_evaluate(celltype, E, nu, alpha, T0, X, u, T, want=("K", "f", "Kst")):
    """SOLIDSCATRA + ThermoStVenantKirchhoff (linear): returns (err, Ke, fe, Kst (3n x n))."""
    lib = load()
    n = 8 if celltype == HEX8 else 27
    X = np.ascontiguousarray(X, dtype=np.float64).reshape(n, 3)
    u = np.ascontiguousarray(u, dtype=np.float64).reshape(n, 3)
    T = np.ascontiguousarray(T, dtype=np.float64).reshape(n)
    Ke, fe, Kst = np.zeros(9 * n * n), np.zeros(3 * n), np.zeros(3 * n * n)
    err = lib.orc_tsi_solid_evaluate(celltype, E, nu, alpha, T0, ptr(X, _dp), ptr(u, _dp), ptr(T, _dp),
                                     ptr(Ke, _dp) if "K" in want else None,
                                     ptr(fe, _dp) if "f" in want else None,
                                     ptr(Kst, _dp) if "Kst" in want else None)
    return err, Ke.reshape(3 * n, 3 * n).T.copy(), fe, Kst.reshape(n, 3 * n).T.copy()


def tsi_thermo_evaluate(celltype, conduct, m, X, T, v, timefac, timefac_d):
    """Thermo element, geometrically linear TSI: returns (err, Ktt (n x n), fT (n), Kts (n x 3n))."""
    lib = load()
    n = 8 if celltype == HEX8 else 27
    X = np.ascontiguousarray(X, dtype=np.float64).reshape(n, 3)
    T = np.ascontiguousarray(T, dtype=np.float64).reshape(n)
    v = np.ascontiguousarray(v, dtype=np.float64).reshape(n, 3)
    Ktt, fT, Kts = np.zeros(n * n), np.zeros(n), np.zeros(3 * n * n)
    err = lib.orc_tsi_thermo_evaluate(celltype, conduct, m, ptr(X, _dp), ptr(T, _dp), ptr(v, _dp),
                                      timefac, timefac_d, ptr(Ktt, _dp), ptr(fT, _dp), ptr(Kts, _dp))
    return err, Ktt.reshape(n, n).T.copy(), fT, Kts.reshape(3 * n, n).T.copy()


def neohooke(E, nu, gl):
    """ElastHyper/CoupNeoHooke: (S, cmat 6x6)."""
    lib = load()
    gl = np.ascontiguousarray(gl, dtype=np.float64)
    S, c = np.zeros(6), np.zeros(36)
    lib.orc_elasthyper_coupneohooke(E, nu, ptr(gl, _dp), ptr(S, _dp), ptr(c, _dp))
    return S, c.reshape(6, 6).T
