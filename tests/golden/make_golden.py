#!/usr/bin/env python3
"""Regenerates the golden fixtures in tests/golden/ from the reference.

Run here (where /root/reference exists); the fixtures are committed so the
tests never read the reference at run time.

  naming.json          format_hash_frame_placeholders evaluated by the
                       reference's OWN function: its source is read from
                       /root/reference/scripts/render-timing-script.py:69-78
                       with `ast` and executed on the inputs below (the module
                       itself cannot be imported: it imports bpy at line 11).
  fcurve_01_cube_z.json  cube z per frame: SURVEY.md §8c's golden table (decoded
                       from the 01 .blend's F-Curves with Blender Bezier
                       semantics) plus the value Blender saved in the file
                       (Object.loc.z at the saved frame RenderData.cfra = 60).
  reference_jobs.json  every job TOML under /root/reference/blender-projects:
                       the fields the master would read, or the serde error class
                       (missing `render_script_path`, unknown strategy variant).
"""
from __future__ import annotations

import ast
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"


def reference_function(path: str, name: str):
    src = open(path).read()
    tree = ast.parse(src)
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == name)
    mod = ast.Module(body=[fn], type_ignores=[])
    ns: dict = {}
    exec(compile(mod, path, "exec"), ns)
    return ns[name]


def make_naming():
    f = reference_function(os.path.join(REF, "scripts/render-timing-script.py"), "format_hash_frame_placeholders")
    cases = [("out/######", 7), ("out/######", 1), ("out/######", 14400), ("out/######", 1234567),
             ("out/#####", 1), ("out/#####", 600), ("out/rendered-#####", 42), ("out/frame_#", 3),
             ("out/frame_#", 12), ("out/no_hashes", 5), ("a/##/b_##", 9), ("a/##b##", 9), ("a/####", 0),
             ("a/###", -5), ("D:/Simon/output/######", 10), ("/x/y/#####.part", 77)]
    return [{"path": p, "frame": fr, "expected": f(p, fr)} for p, fr in cases]


def make_fcurve():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from sdna import BlendFile
    bf = BlendFile(os.path.join(REF, "blender-projects/01_simple-animation/01_simple-animation.blend"))
    sc = bf.blocks_with_code(b"SC")[0]
    cfra = bf.read_struct_at(bf.get(sc, "r"), "RenderData", "cfra")
    cube = next(b for b in bf.blocks_with_code(b"OB") if bf.get(b, "id.name") == "OBCube")
    saved_z = bf.get(cube, "loc")[2]
    table = {1: 0.0, 2: 0.0026213, 10: 0.1929112, 30: 1.4990573, 31: 1.5772613, 59: 3.0736972,
             60: 3.0763185, 61: 3.0763185, 120: 3.0763185, 600: 3.0763185}
    return {"source": "SURVEY.md §8c golden z table (7 significant digits) + saved Object.loc.z",
            "object": "Cube", "object_index": 1, "tolerance": 1e-6,
            "frames": {str(k): v for k, v in table.items()},
            "saved_frame": cfra, "saved_z": saved_z}


def make_jobs():
    try:
        import tomllib as toml
    except ModuleNotFoundError:
        import tomli as toml
    out = []
    for p in sorted(glob.glob(os.path.join(REF, "blender-projects/**/*.toml"), recursive=True)):
        with open(p, "rb") as f:
            d = toml.load(f)
        rel = os.path.relpath(p, REF)
        rec = {"file": rel}
        st = d.get("frame_distribution_strategy", {}).get("strategy_type")
        if "render_script_path" not in d:
            rec["error"] = "missing field `render_script_path`"
        elif st not in ("naive-fine", "eager-naive-coarse", "dynamic"):
            rec["error"] = f"unknown variant `{st}`"
        else:
            rec["job_name"] = d["job_name"]
            rec["frames"] = [d["frame_range_from"], d["frame_range_to"]]
            rec["workers"] = d["wait_for_number_of_workers"]
            rec["strategy"] = st
            rec["format"] = d["output_file_format"]
            rec["name_format"] = d["output_file_name_format"]
        rec["raw"] = d
        out.append(rec)
    return out


def main():
    if not os.path.isdir(REF):
        sys.exit("the reference checkout is needed to regenerate the fixtures")
    with open(os.path.join(HERE, "naming.json"), "w") as f:
        json.dump(make_naming(), f, indent=1)
    with open(os.path.join(HERE, "fcurve_01_cube_z.json"), "w") as f:
        json.dump(make_fcurve(), f, indent=1)
    with open(os.path.join(HERE, "reference_jobs.json"), "w") as f:
        json.dump(make_jobs(), f, indent=1)
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
