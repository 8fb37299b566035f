"""Scene format, exporter and host-side frame evaluation (no GPU needed):
the product's C++ animation/camera evaluation (through the C ABI, host-only
scene handles) vs the Python restatement and the golden values decoded from
the reference's .blend."""
import json
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, have_reference, scene_path
from oracle import host_oracle as HO

S01 = scene_path("01_simple-animation.rrscene")
S04 = scene_path("04_very-simple-standin.rrscene")
BLEND = "/root/reference/blender-projects/01_simple-animation/01_simple-animation.blend"


def test_fcurve_golden_table(rr):
    g = json.load(open(os.path.join(GOLDEN, "fcurve_01_cube_z.json")))
    s = rr.Scene(S01)
    scene = HO.load_scene(S01)
    obj = scene["objects"][g["object_index"]]
    assert obj["name"] == g["object"]
    for f, z in g["frames"].items():
        zp = s.object_matrix(g["object_index"], int(f))[2, 3]
        zo = HO.object_matrix(obj, int(f))[2, 3]
        assert zp == zo, f"product and restatement differ at frame {f}"
        assert abs(zp - z) <= g["tolerance"], (f, zp, z)
    # Blender saved the file at cfra=60 with the evaluated location
    assert s.object_matrix(1, g["saved_frame"])[2, 3] == g["saved_z"]
    s.close()


@pytest.mark.parametrize("frame", [1, 1.5, 7, 33.25, 59.999, 60, 61, 1000, -5])
def test_fcurve_product_equals_restatement(rr, frame):
    s = rr.Scene(S01)
    scene = HO.load_scene(S01)
    for i, o in enumerate(scene["objects"]):
        assert np.array_equal(s.object_matrix(i, frame), HO.object_matrix(o, frame)), (i, frame)
    s.close()


def test_fcurve_interpolation_modes():
    keys = [{"co": [1, 0], "handle_left": [0, 0], "handle_right": [2, 0], "interpolation": "LINEAR"},
            {"co": [11, 10], "handle_left": [10, 10], "handle_right": [12, 10], "interpolation": "CONSTANT"},
            {"co": [21, 0], "handle_left": [20, 0], "handle_right": [22, 0], "interpolation": "BEZIER"}]
    assert HO.eval_fcurve(keys, "CONSTANT", 6) == pytest.approx(5.0)
    assert HO.eval_fcurve(keys, "CONSTANT", 15) == 10.0   # constant segment holds the left key
    assert HO.eval_fcurve(keys, "CONSTANT", -3) == 0.0
    assert HO.eval_fcurve(keys, "LINEAR", -3) == pytest.approx(-4.0)  # linear extrapolation of a LINEAR key
    assert HO.eval_fcurve(keys, "CONSTANT", 40) == 0.0


def test_camera_matches_saved_blender_matrix(rr):
    scene = HO.load_scene(S01)
    cam = scene["objects"][scene["camera"]]
    saved = np.array(cam["matrix_world_saved"]).reshape(4, 4).T  # Blender column-major
    s = rr.Scene(S01)
    np.testing.assert_allclose(s.object_matrix(scene["camera"], 60), saved, atol=2e-7)
    s.close()


def test_frame_constants_product_vs_restatement(rr):
    for path in (S01, S04):
        s = rr.Scene(path)
        scene = HO.load_scene(path)
        for frame in (1, 45):
            st = s.frame_constants(frame)
            fc = HO.frame_constants(scene, frame)
            np.testing.assert_allclose(st.camera, fc["camera"], atol=2e-7)
            np.testing.assert_allclose(st.lights, fc["lights"], rtol=1e-7, atol=1e-7)
            np.testing.assert_allclose(st.materials, fc["materials"], atol=1e-7)
            np.testing.assert_allclose(st.world, fc["world"], rtol=1e-7)
        s.close()
    # 01 light: 1000 W point light of radius 0.1 -> I = 1000/(4 pi) W/sr
    st = rr.Scene(S01).frame_constants(1)
    assert st.lights[0, 0] == 0 and st.lights[0, 7] == pytest.approx(0.1)
    assert st.lights[0, 8] == pytest.approx(1000 / (4 * np.pi), rel=1e-6)
    assert st.camera[12] == pytest.approx(0.36) and st.camera[13] == pytest.approx(0.36 * 1080 / 1920)


def test_render_params_override(rr):
    s = rr.Scene(S04)
    st = s.frame_constants(1, rr.default_params(width=320, height=200, spp=7, max_bounces=3, seed=9))
    assert list(st.render_ints[:5]) == [320, 200, 7, 3, 9]
    assert st.camera[13] == pytest.approx(0.36 * 200 / 320)
    st = s.frame_constants(1, rr.default_params(width=100, height=400))  # portrait: AUTO fits vertically
    assert st.camera[13] == pytest.approx(0.36) and st.camera[12] == pytest.approx(0.09)


@pytest.mark.skipif(not have_reference(), reason="needs the reference .blend")
def test_exporter_reproduces_committed_scene():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from blend_export import export

    class A:
        samples, max_bounces, clamp_indirect, seed = 128, 12, 10.0, 0

    fresh = export(BLEND, A)
    committed = HO.load_scene(S01)
    assert json.loads(json.dumps(fresh)) == committed
    cube = fresh["meshes"][0]
    assert len(cube["triangles"]) == 36 and len(cube["vertices"]) == 24
    assert fresh["render"]["resolution_x"] == 1920 and fresh["source"]["engine"] == "BLENDER_EEVEE"
    mat = fresh["materials"][cube["material_slots"][0]]
    assert mat["base_color"] == pytest.approx([0.8, 0.8, 0.8]) and mat["roughness"] == pytest.approx(0.5)
    assert mat["distribution"] == "GGX"


def test_procedural_meshes(rr, tmp_path):
    scene = {"format": "rrscene", "version": 1, "name": "gen",
             "meshes": [{"generator": {"type": "icosphere", "subdivisions": 3, "radius": 2.0}},
                        {"generator": {"type": "cube", "size": 1.0}}, {"generator": {"type": "plane"}}],
             "objects": [{"type": "CAMERA", "camera": {"lens": 50}, "location": [0, -5, 0],
                          "rotation_euler": [1.57, 0, 0]},
                         {"type": "MESH", "mesh": 0}, {"type": "MESH", "mesh": 1}, {"type": "MESH", "mesh": 2}]}
    p = tmp_path / "gen.rrscene"
    p.write_text(json.dumps(scene))
    s = rr.Scene(str(p))
    assert s.counts()["triangles"] == 20 * 4 ** 3 + 12 + 2
    s.close()


def test_scene_validation(rr, tmp_path):
    bad = [{"format": "rrscene", "version": 2, "objects": []},
           {"format": "rrscene", "version": 1, "objects": [{"type": "MESH", "mesh": 0}],
            "meshes": [{"vertices": [0, 0, 0], "triangles": [0, 1, 2]}]},
           {"format": "rrscene", "version": 1, "objects": [{"type": "LIGHT", "light": {"type": "AREA"}}]},
           {"format": "rrscene", "version": 1, "objects": [{"type": "EMPTY"}]}]
    for i, d in enumerate(bad):
        p = tmp_path / f"b{i}.rrscene"
        p.write_text(json.dumps(d))
        with pytest.raises(rr.RRError) as e:
            rr.Scene(str(p))
        assert e.value.code == -22, d


# ---- physics stand-ins (C4/C5) -------------------------------
PHYS = [scene_path("02_physics-standin.rrscene"), scene_path("03_physics-2-standin.rrscene"),
        scene_path("c5_synthetic-10m.rrscene")]


@pytest.mark.parametrize("path", PHYS)
def test_rigid_body_poses_match_restatement(rr, path):
    """Product poses (C++ generator through the C ABI) == the Python
    restatement, for a spread of bodies and frames (before spawn, in flight,
    bouncing, at rest). Same IEEE double ops and libm on both sides."""
    scene = HO.load_scene(path)
    bodies = HO.expand_rigid_bodies(scene)
    n_explicit = len(scene["objects"])
    s = rr.Scene(path)
    assert s.counts()["objects"] == n_explicit + len(bodies)
    fps, f0 = scene["render"]["fps"], scene["render"]["frame_start"]
    idx = sorted(set([0, 1, len(bodies) // 2, len(bodies) - 1] + list(range(0, len(bodies), max(1, len(bodies) // 37)))))
    for b in idx:
        for frame in (1, 2, 17, 60, 61.5, 119, 170, 240, 480, 2000):
            got = s.object_matrix(n_explicit + b, frame)
            want = HO.rigid_matrix(bodies[b], (frame - f0) / fps)
            np.testing.assert_allclose(got, want, rtol=0, atol=1e-12, err_msg=f"body {b} frame {frame}")
    s.close()


def test_rigid_body_motion_is_physical():
    """Bodies never sink below their rest height, fall under gravity after
    spawning, and come to rest (pose constant) long after the last spawn."""
    scene = HO.load_scene(PHYS[0])
    bodies = HO.expand_rigid_bodies(scene)
    assert len(bodies) == 2000
    fps = scene["render"]["fps"]
    for m in bodies[:200]:
        rest = m["ground_z"] + m["rest_height"]
        for f in range(1, 400, 7):
            z = HO.rigid_matrix(m, (f - 1) / fps)[2, 3]
            assert z >= rest - 1e-12
        before = HO.rigid_matrix(m, m["t_spawn"] - 1e-3)
        assert np.allclose(before[:3, 3], m["p0"])
        late1, late2 = HO.rigid_matrix(m, 1e4), HO.rigid_matrix(m, 2e4)
        assert np.array_equal(late1, late2)
        assert late1[2, 3] == pytest.approx(rest)
        # rotation part stays a scaled rotation
        R = late1[:3, :3] / m["scale"]
        np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-12)


def test_physics_standins_animate_every_frame(rr):
    """C4 requires a BVH rebuild per frame: consecutive frames inside the
    spawn window change at least one body's transform."""
    s = rr.Scene(PHYS[0])
    n = s.counts()["objects"]
    for f in (2, 30, 90, 119):
        moved = any(not np.array_equal(s.object_matrix(i, f), s.object_matrix(i, f + 1)) for i in range(4, n, 50))
        assert moved, f
    s.close()


def test_c5_scene_size(rr):
    """C5 synthetic scene: 512 x 20,480 displaced-icosphere triangles + ground."""
    s = rr.Scene(PHYS[2])
    c = s.counts()
    assert c["triangles"] == 512 * 20480 + 2
    assert s.resolution() == (3840, 2160)
    s.close()


def tiles_lds_per_block(n_tris: int, n_mats: int, n_lights: int) -> int:
    """Restatement of k_tiles' LDS per block (wavefront.hip kTilesStaticLds +
    tiles_dyn_lds_bytes): static traversal stack (12 entries x 256 lanes x 4 B)
    and 8 counter words per wave, + the staged scene in float4s — BVH2 nodes
    (4 per node), triangle records (3), normal + shading frames (1 + 4), camera
    vertices (13) per triangle, 72 per material, 3 per light, the 256-float4
    filter table."""
    static = 4 * (12 * 256 + 8 * 4)
    f4 = 4 * max(n_tris - 1, 1) + (3 + 5 + 13) * n_tris + 72 * n_mats + 3 * n_lights + 256
    return static + 16 * f4


def test_lds_residency_counts_what_k_tiles_allocates(rr, tmp_path):
    """VERDICT r5 Weak 7: the residency decision (k_tiles or the split path,
    render_ints[7] = 2 LBVH / 4 quantised 6-wide) uses the same byte count as
    k_tiles' launch: resident exactly while 3 blocks of that LDS fit a CU's
    160 KB and the scene has at most 128 triangles. Checked on both sides of
    the boundary for the 04vs stand-in's materials and lights."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import soups
    base = rr.Scene(S04)
    c = base.counts()
    nm, nl = c["materials"], c["lights"]
    base.close()
    resident = lambda n: n <= 128 and 3 * tiles_lds_per_block(n, nm, nl) <= 160 * 1024  # noqa: E731
    n_max = max(n for n in range(1, 200) if resident(n))
    assert 80 <= n_max < 128, n_max  # the study's range (70 / 90 triangles at 3 / 2 blocks per CU)
    for n in (12, n_max - 1, n_max, n_max + 1, 120):
        path = str(tmp_path / f"soup_{n}.rrscene")
        soups.soup_scene(S04, 5, path, n=n)
        s = rr.Scene(path)
        try:
            assert s.counts()["triangles"] == n
            hier = int(s.frame_constants(3).render_ints[7])
            assert hier == (2 if resident(n) else 4), (n, hier)
        finally:
            s.close()
