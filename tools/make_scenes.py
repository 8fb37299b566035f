#!/usr/bin/env python3
"""Generate the committed scene files under scenes/ (DESIGN.md §3.3).

  01_simple-animation.rrscene   exported from the reference's only .blend
                                (blender-projects/01_simple-animation/01_simple-animation.blend)
                                when /root/reference is present; otherwise the
                                committed copy is kept.
  04_very-simple-standin.rrscene  stand-in for the missing 04_very-simple.blend
                                (/root/reference/.MISSING_LARGE_BLOBS:3): the 01
                                content (SURVEY.md §8d "04vs-standin"), Standard view.
  test_furnace.rrscene          Lambert sphere, albedo 0.5, uniform world: every
                                camera sample that hits the sphere returns
                                albedo * world exactly (convex, 1 bounce).
  test_pointlight.rrscene       Lambert plane under a point light of radius 0,
                                black world: closed-form irradiance.
Usage: python tools/make_scenes.py
"""
from __future__ import annotations

import copy
import json
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SCENES = os.path.join(ROOT, "scenes")
REF_BLEND = "/root/reference/blender-projects/01_simple-animation/01_simple-animation.blend"


def write(name: str, scene: dict):
    path = os.path.join(SCENES, name)
    with open(path, "w") as f:
        json.dump(scene, f, indent=1)
    print("wrote", path)


def export_01() -> dict:
    path = os.path.join(SCENES, "01_simple-animation.rrscene")
    if os.path.isfile(REF_BLEND):
        sys.path.insert(0, HERE)
        from blend_export import export

        class A:
            samples, max_bounces, clamp_indirect, seed = 128, 12, 10.0, 0

        s = export(REF_BLEND, A)
        write("01_simple-animation.rrscene", s)
        return s
    with open(path) as f:
        return json.load(f)


def camera_object(name, loc, target, lens=50.0):
    # XYZ Euler that points the camera's -Z at target with +Y up-ish (world Z up)
    dx, dy, dz = (target[i] - loc[i] for i in range(3))
    dist_xy = math.hypot(dx, dy)
    rx = math.atan2(dist_xy, -dz)       # tilt from looking straight down
    rz = math.atan2(dy, dx) - math.pi / 2
    return {"name": name, "type": "CAMERA", "location": list(loc), "rotation_euler": [rx, 0.0, rz],
            "rotation_mode": "XYZ", "scale": [1, 1, 1], "parent": -1,
            "camera": {"type": "PERSP", "lens": lens, "sensor_width": 36.0, "sensor_height": 24.0,
                       "sensor_fit": "AUTO", "clip_start": 0.1, "clip_end": 100.0}}


def main():
    os.makedirs(SCENES, exist_ok=True)
    s01 = export_01()

    s04 = copy.deepcopy(s01)
    s04["name"] = "04_very-simple-standin"
    s04["source"] = {"standin_for": "blender-projects/04_very-simple/04_very-simple.blend (missing: "
                                    ".MISSING_LARGE_BLOBS:3)", "content": "01_simple-animation export",
                     "generator": "tools/make_scenes.py"}
    s04["render"]["view_transform"] = "Standard"
    write("04_very-simple-standin.rrscene", s04)

    furnace = {
        "format": "rrscene", "version": 1, "name": "test_furnace",
        "source": {"generator": "tools/make_scenes.py", "purpose": "white-furnace known answer"},
        "render": {"resolution_x": 64, "resolution_y": 48, "resolution_percentage": 100, "fps": 24,
                   "frame_start": 1, "frame_end": 1, "filter_width": 1.5, "view_transform": "Raw",
                   "exposure": 0.0, "samples": 16, "max_bounces": 1, "clamp_indirect": 0.0, "seed": 7},
        "world": {"color": [0.8, 0.6, 0.4], "strength": 1.0},
        "materials": [{"name": "lambert50", "model": "lambert", "base_color": [0.5, 0.5, 0.5], "metallic": 0.0,
                       "specular": 0.0, "roughness": 1.0, "ior": 1.45, "emission": [0, 0, 0],
                       "emission_strength": 1.0}],
        "meshes": [{"name": "sphere", "generator": {"type": "icosphere", "subdivisions": 4, "radius": 1.0},
                    "material_slots": [0]}],
        "objects": [camera_object("Camera", (0.0, -6.0, 0.0), (0.0, 0.0, 0.0), lens=50.0),
                    {"name": "Sphere", "type": "MESH", "mesh": 0, "location": [0, 0, 0],
                     "rotation_euler": [0, 0, 0], "scale": [1, 1, 1], "parent": -1}],
        "camera": 0,
    }
    write("test_furnace.rrscene", furnace)

    plane = {
        "format": "rrscene", "version": 1, "name": "test_pointlight",
        "source": {"generator": "tools/make_scenes.py", "purpose": "point-light closed form"},
        "render": {"resolution_x": 64, "resolution_y": 64, "resolution_percentage": 100, "fps": 24,
                   "frame_start": 1, "frame_end": 1, "filter_width": 1.5, "view_transform": "Raw",
                   "exposure": 0.0, "samples": 4, "max_bounces": 1, "clamp_indirect": 0.0, "seed": 3},
        "world": {"color": [0.0, 0.0, 0.0], "strength": 1.0},
        "materials": [{"name": "lambert80", "model": "lambert", "base_color": [0.8, 0.8, 0.8], "metallic": 0.0,
                       "specular": 0.0, "roughness": 1.0, "ior": 1.45, "emission": [0, 0, 0],
                       "emission_strength": 1.0}],
        "meshes": [{"name": "plane", "generator": {"type": "plane", "size": 20.0}, "material_slots": [0]}],
        "objects": [{"name": "Camera", "type": "CAMERA", "location": [0.0, 0.0, 10.0],
                     "rotation_euler": [0.0, 0.0, 0.0], "rotation_mode": "XYZ", "scale": [1, 1, 1], "parent": -1,
                     "camera": {"type": "PERSP", "lens": 50.0, "sensor_width": 36.0, "sensor_height": 36.0,
                                "sensor_fit": "AUTO", "clip_start": 0.1, "clip_end": 100.0}},
                    {"name": "Plane", "type": "MESH", "mesh": 0, "location": [0, 0, 0],
                     "rotation_euler": [0, 0, 0], "scale": [1, 1, 1], "parent": -1},
                    {"name": "Light", "type": "LIGHT", "location": [1.0, 0.5, 2.0], "rotation_euler": [0, 0, 0],
                     "scale": [1, 1, 1], "parent": -1,
                     "light": {"type": "POINT", "energy": 100.0, "color": [1.0, 1.0, 1.0], "radius": 0.0}}],
        "camera": 0,
    }
    write("test_pointlight.rrscene", plane)


if __name__ == "__main__":
    main()
