"""Extract known-answer fixtures from the reference's own integration-test input files.

Run in the build container only (it reads /root/reference, which does not exist on the GPU box):

    python tests/golden/make_fixtures.py

It copies DATA ONLY -- node coordinates, element connectivity, condition node sets and
parameters, material constants and the RESULT DESCRIPTION values -- out of the .dat files into
small JSON fixtures next to this script.  Nothing of the reference's code is copied.

Sources (paths relative to /root/reference):
  tests/input_files/solid_ele_hex8_Standard_linear.dat   (registered tests/list_of_tests.cmake:1338)
  tests/input_files/solid_ele_hex27_Standard_linear.dat  (tests/list_of_tests.cmake:1311)
  tests/input_files/sohex27_patchtest_nl_cost_drt.dat    (tests/list_of_tests.cmake:1265)
  tests/input_files/solid_ele_hex8_Standard_eas_none_volume_neumann.dat (ElastHyper/CoupNeoHooke)
  tests/input_files/solid_ele_hex27_Standard_volume_neumann.dat          (ElastHyper/CoupNeoHooke)
  tests/input_files/tsi_heatflux_monolithic.dat          (thermo-structure interaction, statics)
  tests/input_files/tsi_heatflux_flexoutsurf_monolithic.dat
"""

import json
import os
import re
import sys

REF = "/root/reference/tests/input_files"
HERE = os.path.dirname(os.path.abspath(__file__))


def sections(path):
    out, cur = {}, None
    with open(path) as f:
        for line in f:
            line = line.rstrip("\n")
            if line.startswith("---"):
                cur = line.strip("-").strip()
                out[cur] = []
                continue
            if cur is not None and line.strip() and not line.lstrip().startswith("//"):
                out[cur].append(line.strip())
    return out


def parse_condition(line):
    tok = line.split()
    d = {"entity": int(tok[1])}
    i = 2
    while i < len(tok):
        key = tok[i]
        if key == "NUMDOF":
            n = int(tok[i + 1])
            d["numdof"] = n
            i += 2
        elif key in ("ONOFF", "VAL", "FUNCT"):
            n = d["numdof"]
            vals = tok[i + 1 : i + 1 + n]
            d[key.lower()] = [float(v) if key == "VAL" else int(v) for v in vals]
            i += 1 + n
        elif key == "TYPE":
            d["type"] = tok[i + 1]
            i += 2
        else:
            i += 1
    return d


def topology(sec, kind):
    sets = {}
    for line in sec:
        tok = line.split()
        sets.setdefault(int(tok[3]), []).append(int(tok[1]))
    return sets


def extract(fname):
    s = sections(os.path.join(REF, fname))
    nodes = {}
    for line in s["NODE COORDS"]:
        tok = line.split()
        nodes[int(tok[1])] = [float(t) for t in tok[3:6]]
    elements = []
    for line in s["STRUCTURE ELEMENTS"]:
        tok = line.split()
        shape = tok[2]
        nn = {"HEX8": 8, "HEX27": 27}[shape]
        kin = tok[tok.index("KINEM") + 1]
        elements.append({"id": int(tok[0]), "shape": shape, "nodes": [int(t) for t in tok[3 : 3 + nn]],
                         "kinem": kin})
    mat = s["MATERIALS"][0].split()
    if "MAT_ElastHyper" in mat:
        # one ELAST_CoupNeoHooke summand (MATIDS)
        summ = [l.split() for l in s["MATERIALS"] if "ELAST_CoupNeoHooke" in l]
        assert len(summ) == 1 and mat[mat.index("NUMMAT") + 1] == "1"
        sm = summ[0]
        material = {"type": "elasthyper_coupneohooke", "young": float(sm[sm.index("YOUNG") + 1]),
                    "nue": float(sm[sm.index("NUE") + 1])}
    else:
        material = {"young": float(mat[mat.index("YOUNG") + 1]), "nue": float(mat[mat.index("NUE") + 1])}
    results = []
    for line in s["RESULT DESCRIPTION"]:
        m = re.match(r"STRUCTURE DIS structure NODE (\d+) QUANTITY (\w+) VALUE\s+(\S+) TOLERANCE (\S+)", line)
        if m and m.group(2) in ("dispx", "dispy", "dispz"):
            results.append({"node": int(m.group(1)), "dof": "xyz".index(m.group(2)[-1]),
                            "value": float(m.group(3)), "tol": float(m.group(4))})
    conds = {}
    for key in s:
        if key.startswith("DESIGN") and key.endswith("CONDITIONS"):
            conds[key] = [parse_condition(l) for l in s[key]]
    topo = {}
    for key, kind in (("DNODE-NODE TOPOLOGY", "DNODE"), ("DLINE-NODE TOPOLOGY", "DLINE"),
                      ("DSURF-NODE TOPOLOGY", "DSURFACE"), ("DVOL-NODE TOPOLOGY", "DVOL")):
        if key in s:
            topo[kind] = topology(s[key], kind)
    functs = {}
    for key in s:
        if key.startswith("FUNCT"):
            functs[key[5:]] = s[key][0].split("SYMBOLIC_FUNCTION_OF_SPACE_TIME")[1].strip()
    dyn = {}
    for line in s["STRUCTURAL DYNAMIC"]:
        tok = line.split()
        if tok[0] in ("TIMESTEP", "NUMSTEP", "MAXTIME", "DYNAMICTYPE"):
            dyn[tok[0]] = tok[1]
    return {"source": "tests/input_files/" + fname, "nodes": nodes, "elements": elements,
            "material": material, "results": results, "conditions": conds, "topology": topo,
            "functions": functs, "dynamic": dyn}


def extract_tsi(fname):
    """A monolithic TSI input: the structural data of extract() plus the thermo field's
    conditions, the ThermoStVenantKirchhoff / Fourier constants, the TSI time stepping and the
    THERMAL result lines."""
    data = extract(fname)
    s = sections(os.path.join(REF, fname))
    mats = {}
    for line in s["MATERIALS"]:
        tok = line.split()
        mats[tok[2]] = {tok[i]: tok[i + 1] for i in range(3, len(tok) - 1)}
    st = mats["MAT_Struct_ThermoStVenantK"]
    data["material"].update({"thexpans": float(st["THEXPANS"]), "inittemp": float(st["INITTEMP"]),
                             "dens": float(st["DENS"])})
    data["thermo_material"] = {"conduct": float(mats["MAT_Fourier"]["CONDUCT"]),
                               "capa": float(mats["MAT_Fourier"]["CAPA"])}
    for line in s["RESULT DESCRIPTION"]:
        m = re.match(r"THERMAL DIS thermo NODE (\d+) QUANTITY temp VALUE\s+(\S+) TOLERANCE (\S+)", line)
        if m:
            data["results"].append({"node": int(m.group(1)), "dof": "temp",
                                    "value": float(m.group(2)), "tol": float(m.group(3))})
    tsi = {}
    for line in s["TSI DYNAMIC"]:
        tok = line.split()
        if tok[0] in ("TIMESTEP", "NUMSTEP", "MAXTIME", "COUPALGO"):
            tsi[tok[0]] = tok[1]
    data["tsi_dynamic"] = tsi
    thr = {}
    for line in s["THERMAL DYNAMIC"]:
        tok = line.split()
        if tok[0] in ("DYNAMICTYPE", "INITIALFIELD", "INITFUNCNO"):
            thr[tok[0]] = tok[1]
    data["thermal_dynamic"] = thr
    return data


def main():
    if not os.path.isdir(REF):
        sys.exit("reference tree not present; fixtures are committed, nothing to do")
    for fname in ("solid_ele_hex8_Standard_linear.dat", "solid_ele_hex27_Standard_linear.dat",
                  "sohex27_patchtest_nl_cost_drt.dat",
                  "solid_ele_hex8_Standard_eas_none_volume_neumann.dat",
                  "solid_ele_hex27_Standard_volume_neumann.dat"):
        data = extract(fname)
        out = os.path.join(HERE, fname.replace(".dat", ".json"))
        with open(out, "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)
        print("wrote", out, len(data["nodes"]), "nodes", len(data["results"]), "results")
    for fname in ("tsi_heatflux_monolithic.dat", "tsi_heatflux_flexoutsurf_monolithic.dat"):
        data = extract_tsi(fname)
        out = os.path.join(HERE, fname.replace(".dat", ".json"))
        with open(out, "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)
        print("wrote", out, len(data["nodes"]), "nodes", len(data["results"]), "results")


if __name__ == "__main__":
    main()
