"""The row-block sweep kernel's visit schedule (4c_amd/csrc/fcg_visit_table.h), replayed on the CPU.

The kernel (fcg_sweep.hip) assembles each 3x3 block (A, B) of the global matrix from the
elements that hold both nodes, two blocks per element visit, lane by lane and layer by layer;
the in-plane blocks (dz = 0) take their lower-layer part from an LDS hold written one layer
earlier, and the self block's two halves are summed across a lane pair.  This test replays
exactly that schedule on a small lattice with random per-(element, Gauss point, node) vectors v
and checks it against the direct element loop  G_AB = sum_e sum_g v_a v_b^T  (every block written
exactly once, every element contribution present).  CPU only (pure index logic).
"""
import os
import re

import numpy as np

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "4c_amd", "csrc",
                   "fcg_visit_table.h")
OFF = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (1, 1, 1), (0, 1, 1)]


def load_table():
    text = open(HDR).read()
    body = text[text.index("kVisit[16][2] = {"):]
    words = [int(w, 16) for w in re.findall(r"0x([0-9a-f]+)u", body)]
    assert len(words) == 32
    return np.array(words, dtype=np.int64).reshape(16, 2)


def decode(w):
    w = int(w)
    return dict(q=w & 3, a=(w >> 2) & 7, b1=(w >> 5) & 7, b2=(w >> 8) & 7, t1=(w >> 11) & 31,
                t2=(w >> 16) & 31, act=(w >> 21) & 7, flush2=(w >> 24) & 1, flush1=(w >> 25) & 1,
                pair=(w >> 26) & 3)


def offset(t):
    return t % 3 - 1, (t // 3) % 3 - 1, t // 9 - 1


def test_visits_are_geometrically_consistent():
    tab = load_table()
    for k in range(16):
        for v in range(2):
            d = decode(tab[k, v])
            qx, qy = d["q"] & 1, d["q"] >> 1
            oa = OFF[d["a"]]
            assert (oa[0], oa[1]) == (1 - qx, 1 - qy)
            for b, t in ((d["b1"], d["t1"]), (d["b2"], d["t2"])):
                ob = OFF[b]
                assert offset(t) == (ob[0] - oa[0], ob[1] - oa[1], ob[2] - oa[2])


def replay(nx, ny, nz, vec):
    """Kernel schedule: layers L = -1 .. nz-1, node columns, 16 lanes each; returns blocks."""
    tab = load_table()
    out = {}
    hold = {}  # (parity, column, t) -> block

    def emit(key_col, L, act, t, blk):
        i, j = key_col
        if act == 4:
            hold[((L + 1) & 1, i, j, t)] = blk.copy()
            return
        if act == 3:
            blk = hold.get((L & 1, i, j, t), np.full((3, 3), np.nan)) + blk
        plane = L + 1 if act == 2 else L
        if not 0 <= plane < nz:
            return
        dx, dy, dz = offset(t)
        B = (i + dx, j + dy, plane + dz)
        if 0 <= B[0] < nx and 0 <= B[1] < ny and 0 <= B[2] < nz:
            key = ((i, j, plane), B)
            assert key not in out, key
            assert np.all(np.isfinite(blk)), key
            out[key] = blk.copy()

    for L in range(-1, nz):
        for j in range(ny):
            for i in range(nx):
                acc1 = [np.zeros((3, 3)) for _ in range(16)]
                acc2 = [np.zeros((3, 3)) for _ in range(16)]
                pending = []
                for k in range(16):
                    for v in range(2):
                        d = decode(tab[k, v])
                        ex, ey = i - 1 + (d["q"] & 1), j - 1 + (d["q"] >> 1)
                        if 0 <= ex < nx - 1 and 0 <= ey < ny - 1 and 0 <= L < nz - 1:
                            ve = vec[(ex, ey, L)]
                            for g in range(8):
                                acc1[k] += np.outer(ve[g, d["a"]], ve[g, d["b1"]])
                                acc2[k] += np.outer(ve[g, d["a"]], ve[g, d["b2"]])
                        if d["flush2"]:
                            emit((i, j), L, d["act"], d["t2"], acc2[k])
                            acc2[k] = np.zeros((3, 3))
                        if d["flush1"]:
                            pending.append((k, d))
                # acc1 after the lane-pair exchange
                final = {k: acc1[k] + (acc1[k ^ 1] if d["pair"] == 1 else 0) for k, d in pending}
                for k, d in pending:
                    if d["pair"] != 2:
                        emit((i, j), L, d["act"], d["t1"], final[k])
    return out


def test_replay_matches_element_loop():
    rng = np.random.default_rng(7)
    nx, ny, nz = 4, 3, 4  # nodes
    vec = {(ex, ey, ez): rng.standard_normal((8, 8, 3))
           for ex in range(nx - 1) for ey in range(ny - 1) for ez in range(nz - 1)}
    direct = {}
    for (ex, ey, ez), ve in vec.items():
        nodes = [(ex + o[0], ey + o[1], ez + o[2]) for o in OFF]
        for a in range(8):
            for b in range(8):
                key = (nodes[a], nodes[b])
                direct[key] = direct.get(key, np.zeros((3, 3))) + sum(
                    np.outer(ve[g, a], ve[g, b]) for g in range(8))
    got = replay(nx, ny, nz, vec)
    assert set(got) == set(direct)
    for key, blk in direct.items():
        np.testing.assert_allclose(got[key], blk, rtol=1e-12, atol=1e-12)
