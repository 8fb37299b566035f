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
  test_enclosure_diffuse.rrscene  camera inside a closed emissive white Lambert
                                sphere, black world: with per-lobe bounce caps
                                every path returns E (1 + 1 + ... ) over exactly
                                cap + 1 hits (Cycles max_diffuse_bounces).
  test_enclosure_glossy.rrscene the same with a white metallic near-mirror
                                (max_glossy_bounces).
  02_physics-standin.rrscene    stand-in for the missing 02_physics.blend (SURVEY.md
                                §8d C4): 2,000 falling/bouncing rigid bodies
                                (cubes + icospheres, ~92k triangles) over a ground
                                plane, closed-form motion => LBVH rebuild every
                                frame; frames 1..170 as the 02 job.
  03_physics-2-standin.rrscene  the same model with 3,000 bodies (~412k
                                triangles), frames 1..480 as the 03 jobs.
  c5_synthetic-10m.rrscene      SURVEY.md §8d C5: 512 displaced icospheres of
                                20,480 triangles (10,485,760) + ground plane,
                                3840x2160, 1024 spp, 4 bounces, 240 frames,
                                per-instance rigid motion (rebuild per frame).
Usage: python tools/make_scenes.py [--tests-only]
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


def look_at_euler(loc, target):
    return camera_object("Camera", loc, target)["rotation_euler"]


def physics_scene(name, standin_for, count, seed, frames, fmt_note, meshes_for_bodies, spawn_window,
                  resolution=(1920, 1080), samples=64, max_bounces=8, extra=None):
    cam = camera_object("Camera", (18.0, -18.0, 12.0), (0.0, 0.0, 1.5), lens=35.0)
    sun_rot = look_at_euler((6.0, -10.0, 14.0), (0.0, 0.0, 0.0))
    s = {
        "format": "rrscene", "version": 1, "name": name,
        "source": {"standin_for": standin_for, "generator": "tools/make_scenes.py", "note": fmt_note},
        "render": {"resolution_x": resolution[0], "resolution_y": resolution[1], "resolution_percentage": 100,
                   "fps": 24, "frame_start": 1, "frame_end": frames, "filter_width": 1.5,
                   "view_transform": "Standard", "exposure": 0.0, "samples": samples, "max_bounces": max_bounces,
                   "clamp_indirect": 10.0, "seed": 0},
        "world": {"color": [0.05, 0.06, 0.08], "strength": 1.0},
        "materials": [
            {"name": "ground", "base_color": [0.55, 0.55, 0.5], "metallic": 0.0, "specular": 0.5,
             "roughness": 0.8, "ior": 1.45, "emission": [0, 0, 0], "emission_strength": 1.0},
            {"name": "red", "base_color": [0.8, 0.15, 0.1], "metallic": 0.0, "specular": 0.5,
             "roughness": 0.4, "ior": 1.45, "emission": [0, 0, 0], "emission_strength": 1.0},
            {"name": "blue", "base_color": [0.1, 0.25, 0.8], "metallic": 0.0, "specular": 0.5,
             "roughness": 0.3, "ior": 1.45, "emission": [0, 0, 0], "emission_strength": 1.0},
            {"name": "gold", "base_color": [0.9, 0.7, 0.3], "metallic": 1.0, "specular": 0.5,
             "roughness": 0.35, "ior": 1.45, "emission": [0, 0, 0], "emission_strength": 1.0}],
        "meshes": [
            {"name": "ground", "generator": {"type": "plane", "size": 80.0}, "material_slots": [0]},
            {"name": "cube", "generator": {"type": "cube", "size": 2.0}, "material_slots": [1]},
            {"name": "ico1", "generator": {"type": "icosphere", "subdivisions": 1, "radius": 1.0},
             "material_slots": [2]},
            {"name": "ico2", "generator": {"type": "icosphere", "subdivisions": 2, "radius": 1.0},
             "material_slots": [3]}],
        "objects": [
            cam,
            {"name": "Ground", "type": "MESH", "mesh": 0, "location": [0, 0, 0], "rotation_euler": [0, 0, 0],
             "scale": [1, 1, 1], "parent": -1},
            {"name": "Sun", "type": "LIGHT", "location": [6.0, -10.0, 14.0], "rotation_euler": sun_rot,
             "rotation_mode": "XYZ", "scale": [1, 1, 1], "parent": -1,
             "light": {"type": "SUN", "energy": 3.0, "color": [1.0, 0.96, 0.9], "radius": 0.0}},
            {"name": "Lamp", "type": "LIGHT", "location": [4.0, -3.0, 10.0], "rotation_euler": [0, 0, 0],
             "scale": [1, 1, 1], "parent": -1,
             "light": {"type": "POINT", "energy": 2000.0, "color": [1.0, 0.9, 0.8], "radius": 0.5}}],
        "camera": 0,
        "rigid_bodies": [{"name": "body", "count": count, "seed": seed, "meshes": meshes_for_bodies,
                          "spawn_center": [0.0, 0.0, 9.0], "spawn_extent": [14.0, 14.0, 10.0],
                          "scale": [0.15, 0.35], "speed": 1.5, "up_speed": 2.0, "spin": 3.0,
                          "spawn_window": spawn_window, "gravity": 9.81, "restitution": 0.45,
                          "friction": 0.6, "ground_z": 0.0, "mesh_half_height": 1.0, "max_bounces": 6}],
    }
    if extra:
        extra(s)
    return s


def c5_scene():
    def tweak(s):
        s["meshes"].append({"name": "rock", "generator": {"type": "displaced_icosphere", "subdivisions": 5,
                                                          "radius": 1.0, "amplitude": 0.15, "frequency": 5.0},
                            "material_slots": [1]})
        g = s["rigid_bodies"][0]
        g.update({"count": 512, "seed": 1234, "meshes": [4], "spawn_center": [0.0, 0.0, 12.0],
                  "spawn_extent": [30.0, 30.0, 16.0], "scale": [0.4, 0.9], "spawn_window": [1, 200]})
        s["objects"][0] = camera_object("Camera", (34.0, -34.0, 22.0), (0.0, 0.0, 2.0), lens=35.0)
    return physics_scene("c5_synthetic-10m", "SURVEY.md §8d C5 synthetic scaled scene (no reference .blend)", 512,
                         1234, 240, "512 x 20,480-triangle displaced icospheres + ground = 10,485,762 triangles",
                         [4], [1, 200], resolution=(3840, 2160), samples=1024, max_bounces=4, extra=tweak)


def enclosure(name: str, material: dict, sub: int) -> dict:
    """Camera at the centre of a closed emissive icosphere (radius 5, emission
    0.25), black world, no lights, indirect clamp off: a path's radiance is
    0.25 x (number of hits before a bounce cap ends it), since white Lambert /
    white mirror-like metal keep the throughput at 1."""
    return {
        "format": "rrscene", "version": 1, "name": name,
        "source": {"generator": "tools/make_scenes.py", "purpose": "per-lobe bounce caps, known answer"},
        "render": {"resolution_x": 32, "resolution_y": 24, "resolution_percentage": 100, "fps": 24,
                   "frame_start": 1, "frame_end": 1, "filter_width": 1.5, "view_transform": "Raw",
                   "exposure": 0.0, "samples": 8, "max_bounces": 12, "max_diffuse_bounces": 4,
                   "max_glossy_bounces": 4, "clamp_indirect": 0.0, "seed": 11},
        "world": {"color": [0.0, 0.0, 0.0], "strength": 1.0},
        "materials": [dict(material, emission=[0.25, 0.25, 0.25], emission_strength=1.0)],
        "meshes": [{"name": "shell", "generator": {"type": "icosphere", "subdivisions": sub, "radius": 5.0},
                    "material_slots": [0]}],
        "objects": [camera_object("Camera", (0.0, 0.0, 0.0), (0.0, 0.0, 0.0), lens=35.0),
                    {"name": "Shell", "type": "MESH", "mesh": 0, "location": [0, 0, 0],
                     "rotation_euler": [0, 0, 0], "scale": [1, 1, 1], "parent": -1}],
        "camera": 0,
    }


def test_scenes():
    write("test_enclosure_diffuse.rrscene", enclosure(
        "test_enclosure_diffuse", {"name": "white_lambert", "model": "lambert", "base_color": [1.0, 1.0, 1.0],
                                   "metallic": 0.0, "specular": 0.0, "roughness": 1.0, "ior": 1.45}, 1))
    write("test_enclosure_glossy.rrscene", enclosure(
        "test_enclosure_glossy", {"name": "white_mirror", "model": "principled", "base_color": [1.0, 1.0, 1.0],
                                  "metallic": 1.0, "specular": 0.5, "roughness": 0.0, "ior": 1.45}, 3))


def main():
    os.makedirs(SCENES, exist_ok=True)
    test_scenes()
    if "--tests-only" in sys.argv:
        return
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

    write("02_physics-standin.rrscene", physics_scene(
        "02_physics-standin", "blender-projects/02_physics/02_physics.blend (missing: .MISSING_LARGE_BLOBS)", 2000, 2,
        170, "2,000 bodies (cube 12 + icosphere-1 80 triangles) + ground = 92,002 triangles; the 02 job writes PNG",
        [1, 2], [1, 120]))
    write("03_physics-2-standin.rrscene", physics_scene(
        "03_physics-2-standin", "blender-projects/03_physics-2/03_physics-2.blend (missing: .MISSING_LARGE_BLOBS)",
        3000, 3, 480, "3,000 bodies (cube 12 / icosphere-1 80 / icosphere-2 320 triangles) + ground = 412,002 triangles",
        [1, 2, 3], [1, 400]))
    write("c5_synthetic-10m.rrscene", c5_scene())


if __name__ == "__main__":
    main()
