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
  tests/input_files/patch_test_cube_linear_test_react.dat     (reaction forces, list_of_tests.cmake:978)
  tests/input_files/patch_test_cube_h27_linear_test_react.dat (reaction forces, list_of_tests.cmake:982)
  tests/input_files/error_analytical_beam_cantilever_end_surface_load_with_poissons_effect.dat
      + its .csv (L2 error against the analytical solution, list_of_tests.cmake:509)
  tests/input_files/sohex8_disp_altgeogeneration.dat     (STRUCTURE DOMAIN = GridGenerator,
                                                          list_of_tests.cmake:1268, NP 2)
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
    results, reactions, reaction_ops = parse_results(s)
    conds = {}
    for key in s:
        if key.startswith("DESIGN") and key.endswith("CONDITIONS"):
            conds[key] = [parse_condition(l) for l in s[key]]
    topo = {}
    for key, kind in (("DNODE-NODE TOPOLOGY", "DNODE"), ("DLINE-NODE TOPOLOGY", "DLINE"),
                      ("DSURF-NODE TOPOLOGY", "DSURFACE"), ("DVOL-NODE TOPOLOGY", "DVOL")):
        if key in s:
            topo[kind] = topology(s[key], kind)
    functs, comps = parse_functions(s)
    dyn = {}
    for line in s["STRUCTURAL DYNAMIC"]:
        tok = line.split()
        if tok[0] in ("TIMESTEP", "NUMSTEP", "MAXTIME", "DYNAMICTYPE"):
            dyn[tok[0]] = tok[1]
    out = {"source": "tests/input_files/" + fname, "nodes": nodes, "elements": elements,
           "material": material, "results": results, "conditions": conds, "topology": topo,
           "functions": functs, "dynamic": dyn}
    if reactions:
        out["reactions"] = reactions
    if reaction_ops:
        out["reaction_ops"] = reaction_ops
    if comps:
        out["function_components"] = comps
    return out


def parse_results(s):
    """RESULT DESCRIPTION: nodal displacements, nodal reactions and the OP (sum/min/max) lines over
    condition node sets (4C_structure_new_resulttest.cpp)."""
    results, reactions, ops = [], [], []
    for line in s["RESULT DESCRIPTION"]:
        m = re.match(r"STRUCTURE DIS structure NODE (\d+) QUANTITY (\w+) VALUE\s+(\S+) TOLERANCE (\S+)", line)
        if m and m.group(2) in ("dispx", "dispy", "dispz"):
            results.append({"node": int(m.group(1)), "dof": "xyz".index(m.group(2)[-1]),
                            "value": float(m.group(3)), "tol": float(m.group(4))})
        elif m and m.group(2) in ("reactx", "reacty", "reactz"):
            reactions.append({"node": int(m.group(1)), "dof": "xyz".index(m.group(2)[-1]),
                              "value": float(m.group(3)), "tol": float(m.group(4))})
        m = re.match(r"STRUCTURE DIS structure (SURFACE|LINE) (\d+) OP (\w+) QUANTITY (react[xyz]) "
                     r"VALUE\s+(\S+) TOLERANCE (\S+)", line)
        if m:
            ops.append({"set": {"SURFACE": "DSURFACE", "LINE": "DLINE"}[m.group(1)],
                        "entity": int(m.group(2)), "op": m.group(3), "dof": "xyz".index(m.group(4)[-1]),
                        "value": float(m.group(5)), "tol": float(m.group(6))})
    return results, reactions, ops


def parse_functions(s):
    functs, comps = {}, {}
    for key in s:
        if key.startswith("FUNCT"):
            lines = s[key]
            if len(lines) > 1 and lines[0].startswith("COMPONENT"):
                comps[key[5:]] = [l.split("SYMBOLIC_FUNCTION_OF_SPACE_TIME")[1].strip() for l in lines]
            else:
                functs[key[5:]] = lines[0].split("SYMBOLIC_FUNCTION_OF_SPACE_TIME")[1].strip()
    return functs, comps


def extract_domain(fname):
    """A STRUCTURE DOMAIN input (GridGenerator box, 4C_io_meshreader.cpp:448-500): box bounds,
    intervals, element line, CORNER / SIDE node sets, conditions and results."""
    s = sections(os.path.join(REF, fname))
    dom = {}
    for line in s["STRUCTURE DOMAIN"]:
        tok = line.split()
        if tok[0] in ("LOWER_BOUND", "UPPER_BOUND"):
            dom[tok[0].lower()] = [float(t) for t in tok[1:4]]
        elif tok[0] == "INTERVALS":
            dom["intervals"] = [int(t) for t in tok[1:4]]
        elif tok[0] == "ELEMENTS":
            dom["shape"] = tok[2]
            dom["kinem"] = tok[tok.index("KINEM") + 1]
        elif tok[0] == "PARTITION":
            dom["partition"] = tok[1]
        elif tok[0] == "ROTATION":
            dom["rotation"] = [float(t) for t in tok[1:4]]
    mat = s["MATERIALS"][0].split()
    material = {"young": float(mat[mat.index("YOUNG") + 1]), "nue": float(mat[mat.index("NUE") + 1])}
    results, reactions, _ = parse_results(s)
    conds = {}
    for key in s:
        if key.startswith("DESIGN") and key.endswith("CONDITIONS"):
            conds[key] = [parse_condition(l) for l in s[key]]
    geo = []
    for key in ("DNODE-NODE TOPOLOGY", "DLINE-NODE TOPOLOGY", "DSURF-NODE TOPOLOGY"):
        for line in s.get(key, []):
            tok = line.split()
            # CORNER structure x- y- z- DNODE 1 / SIDE structure x- DSURFACE 1
            geo.append({"kind": tok[0], "spec": tok[2:-2], "set": tok[-2], "entity": int(tok[-1])})
    dyn = {}
    for line in s["STRUCTURAL DYNAMIC"]:
        tok = line.split()
        if tok[0] in ("TIMESTEP", "NUMSTEP", "MAXTIME", "DYNAMICTYPE", "MAXITER"):
            dyn[tok[0]] = tok[1]
    return {"source": "tests/input_files/" + fname, "domain": dom, "material": material,
            "results": results, "conditions": conds, "geometry_sets": geo, "dynamic": dyn}


def extract_csv(fname):
    """A CSV_COMPARISON reference file: header + rows (data)."""
    with open(os.path.join(REF, fname)) as f:
        rows = [l.strip().split(",") for l in f if l.strip()]
    return {"columns": rows[0], "rows": [[float(v) for v in r] for r in rows[1:]]}


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
    for fname in ("patch_test_cube_linear_test_react.dat", "patch_test_cube_h27_linear_test_react.dat",
                  "error_analytical_beam_cantilever_end_surface_load_with_poissons_effect.dat"):
        data = extract(fname)
        csv = fname.replace(".dat", ".csv")
        if os.path.exists(os.path.join(REF, csv)):
            data["csv_reference"] = extract_csv(csv)
            data["csv_tolerance"] = {"rtol": 1e-10, "atol": 1e-12}  # list_of_tests.cmake:509
        out = os.path.join(HERE, fname.replace(".dat", ".json"))
        with open(out, "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)
        print("wrote", out, len(data["nodes"]), "nodes", len(data["results"]), "results")
    data = extract_domain("sohex8_disp_altgeogeneration.dat")
    data["np"] = 2  # list_of_tests.cmake:1268
    out = os.path.join(HERE, "sohex8_disp_altgeogeneration.json")
    with open(out, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print("wrote", out, data["domain"])
    for fname in ("tsi_heatflux_monolithic.dat", "tsi_heatflux_flexoutsurf_monolithic.dat"):
        data = extract_tsi(fname)
        out = os.path.join(HERE, fname.replace(".dat", ".json"))
        with open(out, "w") as f:
            json.dump(data, f, indent=1, sort_keys=True)
        print("wrote", out, len(data["nodes"]), "nodes", len(data["results"]), "results")


if __name__ == "__main__":
    main()
