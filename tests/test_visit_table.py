"""The row-block sweep kernel's visit schedule (4c_amd/csrc/fcg_visit_table.h), replayed on the CPU.

The kernel (fcg_sweep.hip) assembles each 3x3 block (A, B) of the global matrix from the
elements that hold both nodes, lane by lane and layer by layer, carrying the in-plane blocks
(dz = 0) across two element layers in registers.  This test replays exactly that schedule on a
small lattice with random per-(element, Gauss point, node) vectors v and checks the result
against the direct element loop  G_AB = sum_e sum_g v_a v_b^T  (every block written exactly once,
every element contribution present).  CPU only; no oracle needed (pure index logic).
"""
import os
import re

import numpy as np

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "4c_amd", "csrc",
                   "fcg_visit_table.h")
OFF = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (1, 1, 1), (0, 1, 1)]


def load_table():
    text = open(HDR).read()
    body = text[text.index("kVisit[16][4] = {"):]
    words = [int(w, 16) for w in re.findall(r"0x([0-9a-f]+)u", body)]
    assert len(words) == 64
    return np.array(words, dtype=np.int64).reshape(16, 4)


def decode(w):
    return w & 3, (w >> 2) & 7, (w >> 5) & 7, (w >> 8) & 7, (w >> 12) & 31


def test_lane_visits_are_consistent():
    tab = load_table()
    seen = {}
    for k in range(16):
        for v in range(4):
            q, a, b, act, t = decode(int(tab[k, v]))
            qx, qy = q & 1, q >> 1
            oa, ob = OFF[a], OFF[b]
            # the row node sits at local (1-qx, 1-qy) in quadrant q's element
            assert (oa[0], oa[1]) == (1 - qx, 1 - qy)
            d = (ob[0] - oa[0], ob[1] - oa[1], ob[2] - oa[2])
            assert t == (d[2] + 1) * 9 + (d[1] + 1) * 3 + (d[0] + 1)
            side = "U" if oa[2] == 0 else "D"
            seen.setdefault((side, t), []).append((k, v, q, act))
    # 18 upper-side and 18 lower-side block parts, each visiting every element holding both nodes
    assert len(seen) == 36
    for (side, t), vis in seen.items():
        dz = t // 9 - 1
        dx, dy = t % 3 - 1, (t // 3) % 3 - 1
        assert dz in ((0, 1) if side == "U" else (-1, 0))
        assert len(vis) == (2 - abs(dx)) * (2 - abs(dy))
        assert len({k for k, _, _, _ in vis}) == 1  # one lane per block part
        assert sum(1 for *_, act in vis if act != 0) == 1  # finalised once, at its last visit
        assert vis[-1][3] != 0


def replay(nx, ny, nz, vec):
    """Kernel schedule: layers L = -1 .. nz-1, node columns, 16 lanes each; returns blocks."""
    tab = load_table()
    out = {}
    hold = {}
    for L in range(-1, nz):
        for j in range(ny):
            for i in range(nx):
                h = {k: hold.get((i, j, k), [np.zeros((3, 3)), np.zeros((3, 3))]) for k in range(16)}
                h[0][0] = h[1][0].copy()  # lane k0 takes lane k1's hold 0 (shuffle)
                for k in range(16):
                    acc = np.zeros((3, 3))
                    for v in range(4):
                        q, a, b, act, t = decode(int(tab[k, v]))
                        ex, ey = i - 1 + (q & 1), j - 1 + (q >> 1)
                        if 0 <= ex < nx - 1 and 0 <= ey < ny - 1 and 0 <= L < nz - 1:
                            ve = vec[(ex, ey, L)]
                            for g in range(8):
                                acc += np.outer(ve[g, a], ve[g, b])
                        if act == 0:
                            continue
                        blk = acc
                        if act in (3, 4):
                            blk = h[k][act - 3] + acc
                        if act in (5, 6):
                            h[k][act - 5] = acc
                        else:
                            plane = L if act in (1, 3, 4) else L + 1
                            if 0 <= plane < nz:
                                dx, dy, dz = t % 3 - 1, (t // 3) % 3 - 1, t // 9 - 1
                                B = (i + dx, j + dy, plane + dz)
                                if 0 <= B[0] < nx and 0 <= B[1] < ny and 0 <= B[2] < nz:
                                    key = ((i, j, plane), B)
                                    assert key not in out, key
                                    out[key] = blk.copy()
                        acc = np.zeros((3, 3))
                for k in range(16):
                    hold[(i, j, k)] = h[k]
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
