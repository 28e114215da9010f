"""CPU tests of the product's host side (no GPU): the C ABI library loads and exports every
declared symbol, the native GridGenerator/DofSet/graph builder reproduces the oracle's mesh and
the SURVEY §8 sizes, multi-rank partitions are consistent, and a context cannot silently fall
back to the CPU."""

import ctypes
import importlib
import os
import re

import numpy as np
import pytest

import oracle_lib as orc

fcg = importlib.import_module("4c_amd").fcg
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    L = fcg.lib()
    with open(os.path.join(ROOT, "include", "fourc_gpu.h")) as f:
        hdr = f.read()
    declared = set(re.findall(r"^(?:int|int64_t|double|void|const char\*)\s+\*?(fcg_[a-z0-9_]+)\s*\(", hdr, re.M))
    assert declared == set(fcg.EXPORTS), declared ^ set(fcg.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name


@pytest.mark.parametrize("celltype,n,nodes,dofs,nnz,maxgid", [
    (fcg.HEX8, 10, 1331, 3993, 268119, 27782),
    (fcg.HEX27, 4, 729, 2187, 9 * (8 * 4 + 1) ** 3, 3 * ((2 * 4 + 1) ** 3 - 1) + 2),
])
def test_box_sizes_match_survey_formulas(celltype, n, nodes, dofs, nnz, maxgid):
    m = fcg.BoxMesh(celltype, (n, n, n))
    assert m.n_ele == n ** 3 and m.n_node == nodes and m.n_rows == dofs and m.n_cols == dofs
    assert m.nnz == nnz
    assert m.row_gid.max() == maxgid


@pytest.mark.parametrize("celltype", [fcg.HEX8, fcg.HEX27])
def test_box_matches_oracle_gridgenerator(celltype):
    iv, lo, hi, off, rot = (3, 4, 5), (-1.0, -2.0, -3.0), (2.5, 3.5, 4.5), 17, (30.0, 10.0, 7.0)
    m = fcg.BoxMesh(celltype, iv, lo, hi, rotation=rot, first_node_gid=off)
    for e in range(m.n_ele):
        ref = orc.hex_nodeids(celltype, int(m.ele_gid[e]), iv, off)
        np.testing.assert_array_equal(m.node_gid[m.ele_nodes[e]], ref)
    for i in range(m.n_node):
        x = orc.node_coords(int(m.node_gid[i]), iv, off, lo, hi, rot)
        np.testing.assert_allclose(m.node_x[i], x, atol=1e-14, rtol=0)
    # DOF gid = 3 (node gid - min node gid) + d, bit-exact
    np.testing.assert_array_equal(m.col_gid.reshape(-1, 3)[:, 0], 3 * (m.node_gid - off))


def _pattern_from_connectivity(m):
    pairs = set()
    for e in range(m.n_ele):
        g = m.node_gid[m.ele_nodes[e]]
        dofs = (3 * g[:, None] + np.arange(3)[None, :]).reshape(-1)
        for r in dofs:
            for c in dofs:
                pairs.add((int(r), int(c)))
    return pairs


@pytest.mark.parametrize("celltype,n", [(fcg.HEX8, 4), (fcg.HEX27, 2)])
def test_graph_equals_element_couplings(celltype, n):
    m = fcg.BoxMesh(celltype, (n, n + 1, n + 2))
    got = set()
    for r in range(m.n_rows):
        for k in range(m.rowptr[r], m.rowptr[r + 1]):
            got.add((int(m.row_gid[r]), int(m.col_gid[m.col_lid[k]])))
    assert got == _pattern_from_connectivity(m)
    # sorted column LIDs inside each row (Epetra local indices after FillComplete)
    for r in range(m.n_rows):
        c = m.col_lid[m.rowptr[r]:m.rowptr[r + 1]]
        assert np.all(np.diff(c) > 0)


@pytest.mark.parametrize("nranks", [2, 3, 4, 8])
def test_partition_rows_and_ghost_layer(nranks):
    iv = (6, 5, 4)
    glob = fcg.BoxMesh(fcg.HEX8, iv)
    rows = []
    for r in range(nranks):
        m = fcg.BoxMesh(fcg.HEX8, iv, rank=r, nranks=nranks)
        rows.append(m.row_gid)
        owned = m.node_dof_row >= 0
        assert np.all(m.node_owner[owned] == r) and np.all(m.node_owner[~owned] != r)
        # every column element touches an owned node; every element touching an owned node is there
        has_owned = owned[m.ele_nodes].any(axis=1)
        assert has_owned.all()
        owned_gids = set(m.node_gid[owned].tolist())
        expect = set()
        for e in range(glob.n_ele):
            if owned_gids & set(glob.node_gid[glob.ele_nodes[e]].tolist()):
                expect.add(int(glob.ele_gid[e]))
        assert set(m.ele_gid.tolist()) == expect
        # the rank's rows of the global graph are identical
        gl = {int(g): i for i, g in enumerate(glob.row_gid)}
        for i in range(0, m.n_rows, 7):
            gi = gl[int(m.row_gid[i])]
            a = sorted(m.col_gid[m.col_lid[m.rowptr[i]:m.rowptr[i + 1]]].tolist())
            b = sorted(glob.col_gid[glob.col_lid[glob.rowptr[gi]:glob.rowptr[gi + 1]]].tolist())
            assert a == b
    allrows = np.concatenate(rows)
    assert len(allrows) == glob.n_rows
    assert set(allrows.tolist()) == set(glob.row_gid.tolist())


@pytest.mark.parametrize("celltype", [fcg.HEX8, fcg.HEX27])
@pytest.mark.parametrize("strict", [False, True])
def test_more_ranks_than_elements_leaves_empty_ranks(celltype, strict):
    """A split with more ranks than the box has element layers (GridGenerator gives some ranks no
    elements): those ranks get an empty mesh -- no elements, rows, columns or graph -- and the other
    ranks' rows still cover the global rows exactly once (this used to crash the builder)."""
    for iv, nranks in (((1, 1, 1), 3), ((2, 1, 1), 5), ((2, 2, 1), 8)):
        glob = fcg.BoxMesh(celltype, iv)
        rows, empty = [], 0
        for r in range(nranks):
            m = fcg.BoxMesh(celltype, iv, rank=r, nranks=nranks, strict=strict)
            if m.n_ele == 0:
                empty += 1
                assert m.n_rows == m.n_cols == m.nnz == m.n_owned_rows == 0
                assert len(m.rowptr) == 1 and m.rowptr[0] == 0
            rows.append(m.row_gid[:m.n_owned_rows])
        assert empty > 0, (iv, nranks)
        allrows = np.concatenate(rows)
        assert len(allrows) == glob.n_rows and set(allrows.tolist()) == set(glob.row_gid.tolist())


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    m = fcg.BoxMesh(fcg.HEX8, (2, 2, 2))
    with pytest.raises(fcg.FcgError) as ei:
        fcg.Evaluator(m)
    assert ei.value.code == 4  # FCG_ERR_DEVICE


def test_invalid_material_rejected_like_reference():
    # Mat::PAR::StVenantKirchhoff checks (4C_mat_stvenantkirchhoff.cpp:26-28) happen before any
    # device work, so they are testable without a GPU.
    m = fcg.BoxMesh(fcg.HEX8, (2, 2, 2))
    for E, nu in ((0.0, 0.3), (210.0, 0.5), (210.0, -1.5)):
        with pytest.raises(fcg.FcgError) as ei:
            fcg.Evaluator(m, youngs=E, poisson=nu)
        assert ei.value.code == 3


def test_jitter_is_deterministic_and_interior_only():
    a = fcg.BoxMesh(fcg.HEX8, (4, 4, 4), jitter=0.1, seed=20251015)
    b = fcg.BoxMesh(fcg.HEX8, (4, 4, 4), jitter=0.1, seed=20251015)
    c = fcg.BoxMesh(fcg.HEX8, (4, 4, 4))
    np.testing.assert_array_equal(a.node_x, b.node_x)
    d = np.abs(a.node_x - c.node_x)
    assert d.max() <= 0.1 * 0.25 + 1e-15 and d.max() > 0
    on_boundary = np.any((np.abs(c.node_x) < 1e-12) | (np.abs(c.node_x - 1) < 1e-12), axis=1)
    assert np.all(d[on_boundary] == 0)


@pytest.mark.parametrize("celltype", [fcg.HEX8, fcg.HEX27])
def test_structured_hint_is_verified_before_device_work(celltype):
    """A wrong lattice hint with PATH_STRUCTURED is rejected (FCG_ERR_ARG) on the host; a valid
    one passes verification and then needs the device (FCG_ERR_DEVICE here, no GPU).  hex8: the
    row-block sweep's plan; hex27: the colour-ordered direct assembly's plan."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    m = fcg.BoxMesh(celltype, (3, 4, 5) if celltype == fcg.HEX8 else (2, 3, 2))
    with pytest.raises(fcg.FcgError) as ei:
        fcg.Evaluator(m, path=fcg.PATH_STRUCTURED)
    assert ei.value.code == 4
    m.ele_ijk[[0, 1]] = m.ele_ijk[[1, 0]]  # swap two elements' lattice positions
    with pytest.raises(fcg.FcgError) as ei:
        fcg.Evaluator(m, path=fcg.PATH_STRUCTURED)
    assert ei.value.code == 3 and "lattice" in str(ei.value)


def test_lattice_detected_from_connectivity():
    """An input-file hex8 mesh without the lattice hint: fcg_create finds the lattice in the
    connectivity (shared faces, any proper rotation of an element's local numbering) when the
    elements stack like a box, and verifies it like a given hint (a renumbered box, or one with an
    element's local frame rotated, passes and then needs the device); an element whose local frame
    is mirrored is no such lattice, so PATH_STRUCTURED is refused on the host."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    box = fcg.BoxMesh(fcg.HEX8, (5, 4, 3), jitter=0.1, seed=4)
    dis = fcg.Discretization.renumbered(box, seed=2)
    assert dis.ele_ijk is None

    def relabel(en):
        return fcg.Discretization(fcg.HEX8, en, dis.node_x, dis.node_dof_col, dis.node_dof_row,
                                  dis.rowptr, dis.col_lid)

    with pytest.raises(fcg.FcgError) as ei:
        fcg.Evaluator(dis, path=fcg.PATH_STRUCTURED)
    assert ei.value.code == 4
    en = dis.ele_nodes.copy()
    en[0, :4] = np.roll(en[0, :4], 1)   # about local zeta
    en[0, 4:] = np.roll(en[0, 4:], 1)
    en[7] = en[7][[1, 5, 6, 2, 0, 4, 7, 3]]  # about local eta
    with pytest.raises(fcg.FcgError) as ei:
        fcg.Evaluator(relabel(en), path=fcg.PATH_STRUCTURED)
    assert ei.value.code == 4
    en = dis.ele_nodes.copy()
    en[3] = en[3][[4, 5, 6, 7, 0, 1, 2, 3]]  # top and bottom swapped: a mirrored frame
    with pytest.raises(fcg.FcgError) as ei:
        fcg.Evaluator(relabel(en), path=fcg.PATH_STRUCTURED)
    assert ei.value.code == 3 and "mirrored" in str(ei.value)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_weak_scaling_boxes(world):
    """bench.py's weak-scaling box: GridGenerator's own split gives every rank n^3 elements,
    N=8 is config 4's cube (2x2x2)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    n = 3
    iv = b.weak_interval(n, world)
    if world == 8:
        assert iv == (2 * n, 2 * n, 2 * n)
    for r in range(world):
        m = fcg.BoxMesh(fcg.HEX8, iv, rank=r, nranks=world)
        assert m.n_ele_row == n ** 3


def test_neohooke_needs_totlag_and_general_path():
    m = fcg.BoxMesh(fcg.HEX8, (1, 1, 1))
    with pytest.raises(fcg.FcgError) as ei:
        fcg.Evaluator(m, kinematics=fcg.LINEAR, material=fcg.MAT_ELASTHYPER_COUPNEOHOOKE)
    assert ei.value.code == 3
    with pytest.raises(fcg.FcgError) as ei:
        fcg.Evaluator(m, kinematics=fcg.TOTLAG, path=fcg.PATH_STRUCTURED,
                      material=fcg.MAT_ELASTHYPER_COUPNEOHOOKE)
    assert ei.value.code == 3
