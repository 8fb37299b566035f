#!/usr/bin/env python3
"""Export a Blender .blend project into the renderer's .rrscene JSON.

One-time, per-project export: the reference re-opens the
.blend in Blender for every frame (/root/reference/worker/src/rendering/runner/mod.rs:142-146,
scripts/render-timing-script.py:81 `scene.frame_set`), the MI355X renderer loads
the exported scene once per worker and evaluates animation itself.

What is exported (the subset the path tracer consumes):
  * scene render block: resolution (RenderData.xsch/ysch/size), fps, frame range,
    filter width (RenderData.gauss), view transform (ColorManagedViewSettings),
    engine name (kept as provenance only);
  * objects: loc / rot (Euler, rotmode) / scale, parent index, data;
  * mesh: legacy MVert/MPoly/MLoop (3.5 "v305" writes them) fan-triangulated,
    per-poly material index, smooth flag;
  * camera: lens, sensor_x/y, sensor_fit, clip range;
  * light: type, energy, colour, radius (shadow_soft_size);
  * materials: Principled BSDF node socket defaults (base colour, metallic,
    specular, roughness, IOR, emission) or the legacy diffuse colour;
  * world: Background node colour/strength or horr/horg/horb;
  * animation: Action F-Curves (rna_path, array_index, extrapolation, Bezier
    keyframes with both handles and interpolation).

Render-quality settings the .blend does not carry for our engine (samples,
bounces, clamp, seed) come from --samples/--max-bounces etc. and are recorded in
the "render" block.

Usage: python tools/blend_export.py <in.blend> <out.rrscene> [--samples N] ...
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sdna import BlendFile  # noqa: E402

OB_EMPTY, OB_MESH, OB_LAMP, OB_CAMERA = 0, 1, 10, 11
LA_LOCAL, LA_SUN, LA_SPOT, LA_AREA = 0, 1, 2, 4
SENSOR_FIT = {0: "AUTO", 1: "HORIZONTAL", 2: "VERTICAL"}
ROTMODE = {1: "XYZ", 2: "XZY", 3: "YXZ", 4: "YZX", 5: "ZXY", 6: "ZYX"}
IPO = {0: "CONSTANT", 1: "LINEAR", 2: "BEZIER"}
EXTEND = {0: "CONSTANT", 1: "LINEAR"}


def idname(bf, blk):
    return bf.get(blk, "id.name")[2:]


def socket_defaults(bf, node_blk):
    """Map socket name -> default value for a bNode's inputs."""
    out = {}
    inputs_first = bf.read_struct_at(bf.get(node_blk, "inputs"), "ListBase", "first")
    for sb in bf.listbase(inputs_first, "bNodeSocket"):
        name = bf.get(sb, "name")
        typ = bf.get(sb, "type")
        dv = bf.deref(bf.get(sb, "default_value"))
        if dv is None:
            continue
        if typ == 2:  # SOCK_RGBA
            out[name] = bf.read_struct_at(dv.offset, "bNodeSocketValueRGBA", "value")
        elif typ == 0:  # SOCK_FLOAT
            out[name] = bf.read_struct_at(dv.offset, "bNodeSocketValueFloat", "value")
        elif typ == 1:  # SOCK_VECTOR
            out[name] = bf.read_struct_at(dv.offset, "bNodeSocketValueVector", "value")
    return out


def nodes_of(bf, ntree_ptr):
    nt = bf.deref(ntree_ptr)
    if nt is None:
        return []
    first = bf.read_struct_at(bf.get(nt, "nodes"), "ListBase", "first")
    return [(bf.get(nb, "idname"), nb) for nb in bf.listbase(first, "bNode")]


def export_material(bf, blk):
    mat = {
        "name": idname(bf, blk),
        "base_color": [bf.get(blk, "r"), bf.get(blk, "g"), bf.get(blk, "b")],
        "metallic": bf.get(blk, "metallic"),
        "specular": 0.5,
        "roughness": bf.get(blk, "roughness"),
        "ior": 1.45,
        "emission": [0.0, 0.0, 0.0],
        "emission_strength": 1.0,
        "source": "legacy",
    }
    if bf.get(blk, "use_nodes"):
        for idn, nb in nodes_of(bf, bf.get(blk, "nodetree")):
            if idn == "ShaderNodeBsdfPrincipled":
                d = socket_defaults(bf, nb)
                mat["base_color"] = list(d["Base Color"][:3])
                mat["metallic"] = d["Metallic"]
                mat["specular"] = d["Specular"]
                mat["roughness"] = d["Roughness"]
                mat["ior"] = d["IOR"]
                mat["emission"] = list(d["Emission"][:3])
                mat["emission_strength"] = d.get("Emission Strength", 1.0)
                mat["distribution"] = {0: "BECKMANN", 1: "SHARP", 2: "GGX", 4: "MULTI_GGX"}.get(
                    bf.get(nb, "custom1"), str(bf.get(nb, "custom1")))
                mat["source"] = "ShaderNodeBsdfPrincipled"
                break
    return mat


def export_world(bf, blk):
    w = {"color": [bf.get(blk, "horr"), bf.get(blk, "horg"), bf.get(blk, "horb")],
         "strength": 1.0, "source": "legacy"}
    if bf.get(blk, "use_nodes"):
        for idn, nb in nodes_of(bf, bf.get(blk, "nodetree")):
            if idn == "ShaderNodeBackground":
                d = socket_defaults(bf, nb)
                w["color"] = list(d["Color"][:3])
                w["strength"] = d["Strength"]
                w["source"] = "ShaderNodeBackground"
    return w


def export_mesh(bf, blk):
    totvert, totpoly = bf.get(blk, "totvert"), bf.get(blk, "totpoly")
    mv = bf.deref(bf.get(blk, "mvert"))
    mp = bf.deref(bf.get(blk, "mpoly"))
    ml = bf.deref(bf.get(blk, "mloop"))
    if mv is None or mp is None or ml is None:
        raise SystemExit("mesh without legacy MVert/MPoly/MLoop arrays is not supported yet")
    vs = bf.struct_by_name["MVert"].size
    ps = bf.struct_by_name["MPoly"].size
    ls = bf.struct_by_name["MLoop"].size
    verts = []
    for i in range(totvert):
        verts += bf.read_struct_at(mv.offset + i * vs, "MVert", "co")
    tris, mat_idx, smooth = [], [], []
    for p in range(totpoly):
        base = mp.offset + p * ps
        loopstart = bf.read_struct_at(base, "MPoly", "loopstart")
        totloop = bf.read_struct_at(base, "MPoly", "totloop")
        mnr = bf.read_struct_at(base, "MPoly", "mat_nr")
        flag = bf.read_struct_at(base, "MPoly", "flag")
        idx = [bf.read_struct_at(ml.offset + (loopstart + k) * ls, "MLoop", "v") for k in range(totloop)]
        for k in range(1, totloop - 1):  # fan triangulation (convex polys)
            tris += [idx[0], idx[k], idx[k + 1]]
            mat_idx.append(mnr)
            smooth.append(1 if (flag & 1) else 0)
    return {"name": idname(bf, blk), "vertices": verts, "triangles": tris,
            "material_indices": mat_idx, "smooth": smooth}


def export_action(bf, act_blk):
    curves_first = bf.read_struct_at(bf.get(act_blk, "curves"), "ListBase", "first")
    fcurves = []
    bs = bf.struct_by_name["BezTriple"].size
    for fb in bf.listbase(curves_first, "FCurve"):
        path_blk = bf.deref(bf.get(fb, "rna_path"))
        path = bf.data[path_blk.offset:path_blk.offset + path_blk.size].split(b"\0", 1)[0].decode()
        n = bf.get(fb, "totvert")
        bz = bf.deref(bf.get(fb, "bezt"))
        keys = []
        for k in range(n):
            base = bz.offset + k * bs
            vec = bf.read_struct_at(base, "BezTriple", "vec")
            keys.append({"handle_left": vec[0:2], "co": vec[3:5], "handle_right": vec[6:8],
                         "interpolation": IPO.get(bf.read_struct_at(base, "BezTriple", "ipo"), "BEZIER"),
                         "handle_left_type": bf.read_struct_at(base, "BezTriple", "h1"),
                         "handle_right_type": bf.read_struct_at(base, "BezTriple", "h2")})
        fcurves.append({"data_path": path, "index": bf.get(fb, "array_index"),
                        "extrapolation": EXTEND.get(bf.get(fb, "extend"), "CONSTANT"),
                        "keyframes": keys})
    return {"action": idname(bf, act_blk), "fcurves": fcurves}


def export(path: str, args) -> dict:
    bf = BlendFile(path)
    sc = bf.blocks_with_code(b"SC")[0]
    r = bf.get(sc, "r")  # RenderData offset (absolute)

    def rd(field):
        return bf.read_struct_at(r, "RenderData", field)

    vs = bf.get(sc, "view_settings")
    view_transform = bf.read_struct_at(vs, "ColorManagedViewSettings", "view_transform")
    out = {
        "format": "rrscene", "version": 1, "name": idname(bf, sc),
        "source": {"file": os.path.basename(path), "blender_version": bf.version,
                   "engine": rd("engine"), "exporter": "tools/blend_export.py"},
        "render": {
            "resolution_x": rd("xsch"), "resolution_y": rd("ysch"),
            "resolution_percentage": rd("size"), "fps": rd("frs_sec"),
            "frame_start": rd("sfra"), "frame_end": rd("efra"),
            "filter_width": rd("gauss"),
            "view_transform": view_transform,
            "look": bf.read_struct_at(vs, "ColorManagedViewSettings", "look"),
            "exposure": bf.read_struct_at(vs, "ColorManagedViewSettings", "exposure"),
            "gamma": bf.read_struct_at(vs, "ColorManagedViewSettings", "gamma"),
            "dither_intensity": rd("dither_intensity"),
            "samples": args.samples, "max_bounces": args.max_bounces,
            "clamp_indirect": args.clamp_indirect, "seed": args.seed,
        },
    }
    # ID blocks, indexed by old pointer
    mats = bf.blocks_with_code(b"MA")
    mat_index = {b.old_ptr: i for i, b in enumerate(mats)}
    out["materials"] = [export_material(bf, b) for b in mats]
    wo = bf.deref(bf.get(sc, "world"))
    out["world"] = export_world(bf, wo) if wo else {"color": [0.05, 0.05, 0.05], "strength": 1.0}
    meshes = bf.blocks_with_code(b"ME")
    mesh_index = {b.old_ptr: i for i, b in enumerate(meshes)}
    out["meshes"] = []
    for mb in meshes:
        m = export_mesh(bf, mb)
        # mesh material slots -> global material indices
        totcol = bf.get(mb, "totcol")
        mat_arr = bf.deref(bf.get(mb, "mat"))
        slots = []
        for k in range(totcol):
            ptr = bf.read_struct_at(mat_arr.offset + k * bf.ptr, "Link", "next") if mat_arr else 0
            slots.append(mat_index.get(ptr, -1))
        m["material_slots"] = slots
        out["meshes"].append(m)

    obs = bf.blocks_with_code(b"OB")
    ob_index = {b.old_ptr: i for i, b in enumerate(obs)}
    objects = []
    for ob in obs:
        typ = bf.get(ob, "type")
        o = {"name": idname(bf, ob),
             "type": {OB_EMPTY: "EMPTY", OB_MESH: "MESH", OB_LAMP: "LIGHT", OB_CAMERA: "CAMERA"}.get(typ, str(typ)),
             "location": bf.get(ob, "loc"), "rotation_euler": bf.get(ob, "rot"),
             "rotation_mode": ROTMODE.get(bf.get(ob, "rotmode"), "XYZ"), "scale": bf.get(ob, "size"),
             "parent": ob_index.get(bf.get(ob, "parent"), -1),
             "matrix_world_saved": bf.get(ob, "obmat")}
        data = bf.deref(bf.get(ob, "data"))
        if typ == OB_MESH:
            o["mesh"] = mesh_index[data.old_ptr]
        elif typ == OB_CAMERA:
            o["camera"] = {"type": {0: "PERSP", 1: "ORTHO", 2: "PANO"}.get(bf.get(data, "type")),
                           "lens": bf.get(data, "lens"), "sensor_width": bf.get(data, "sensor_x"),
                           "sensor_height": bf.get(data, "sensor_y"),
                           "sensor_fit": SENSOR_FIT.get(bf.get(data, "sensor_fit"), "AUTO"),
                           "clip_start": bf.get(data, "clipsta"), "clip_end": bf.get(data, "clipend")}
        elif typ == OB_LAMP:
            ltype = bf.get(data, "type")
            o["light"] = {"type": {LA_LOCAL: "POINT", LA_SUN: "SUN", LA_SPOT: "SPOT", LA_AREA: "AREA"}.get(ltype),
                          "energy": bf.get(data, "energy"),
                          "color": [bf.get(data, "r"), bf.get(data, "g"), bf.get(data, "b")],
                          "radius": bf.get(data, "radius") if ltype != LA_SUN else 0.0,
                          "angle": bf.get(data, "sun_angle")}
        adt = bf.deref(bf.get(ob, "adt"))
        if adt is not None:
            act = bf.deref(bf.read_struct_at(adt.offset, "AnimData", "action"))
            if act is not None:
                o["animation"] = export_action(bf, act)
        objects.append(o)
    out["objects"] = objects
    cam = bf.get(sc, "camera")
    out["camera"] = ob_index.get(cam, -1)
    out["saved_frame"] = rd("cfra")
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("blend")
    ap.add_argument("out")
    ap.add_argument("--samples", type=int, default=128)
    ap.add_argument("--max-bounces", type=int, default=12)
    ap.add_argument("--clamp-indirect", type=float, default=10.0)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args(argv)
    scene = export(args.blend, args)
    with open(args.out, "w") as f:
        json.dump(scene, f, indent=1)
    print(f"wrote {args.out}: {len(scene['objects'])} objects, "
          f"{sum(len(m['triangles']) // 3 for m in scene['meshes'])} triangles")


if __name__ == "__main__":
    main()
