"""Parity of the HIP path (through the C ABI) with the CPU oracle (oracle/).

Integer/index work (Morton keys, sort order, BVH topology, hit primitive ids)
must be bit-exact; float work is ALSO expected bit-exact because both sides run
the same uncontracted IEEE single-precision op sequence (rr_device.h header);
the asserted tolerance is 0 and the mismatch counts are printed on failure.
"""
import os
import subprocess

import numpy as np
import pytest
from PIL import Image

from conftest import scene_path
from oracle import host_oracle as HO
from oracle import oracle as O

pytestmark = pytest.mark.gpu

S04 = scene_path("04_very-simple-standin.rrscene")
S01 = scene_path("01_simple-animation.rrscene")


@pytest.fixture(scope="module")
def s04(ctx):
    s = ctx.load_scene(S04)
    yield s
    s.close()


def _rays_random(rng, n, center, spread):
    o = center + rng.uniform(-spread, spread, (n, 3))
    tgt = center + rng.uniform(-1.5, 1.5, (n, 3))
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = np.zeros((n, 8), np.float32)
    r[:, 0:3] = o
    r[:, 3] = 0.0
    r[:, 4:7] = d
    r[:, 7] = 1e30
    return r


@pytest.mark.parametrize("frame", [1, 17, 30, 60, 300])
def test_lbvh_bit_exact(ctx, s04, frame):
    st = ctx.frame_state(s04, frame)
    keys, order, children, boxes = ctx.bvh(s04, frame)
    ok, oo, oc, ob = O.build_lbvh(st.tris)
    assert np.array_equal(keys, ok)
    assert np.array_equal(order, oo)
    assert np.array_equal(children, oc)
    assert np.array_equal(boxes, ob)


def test_world_transform_matches_host_oracle(ctx, s04):
    scene = HO.load_scene(S04)
    for frame in (1, 2, 30, 59, 60, 61):
        st = ctx.frame_state(s04, frame)
        obj = scene["objects"][1]
        M = HO.object_matrix(obj, frame).astype(np.float32)
        mesh = scene["meshes"][0]
        v = np.array(mesh["vertices"], np.float32).reshape(-1, 3)
        t = np.array(mesh["triangles"]).reshape(-1, 3)
        exp = np.empty((len(t), 3, 3), np.float32)
        for i, tri in enumerate(t):
            for k, vi in enumerate(tri):
                for r in range(3):
                    exp[i, k, r] = ((M[r, 0] * v[vi, 0] + M[r, 1] * v[vi, 1]) + M[r, 2] * v[vi, 2]) + M[r, 3]
        assert np.array_equal(st.tris, exp), f"frame {frame}"


def test_frame_constants_match_host_oracle(ctx, s04):
    scene = HO.load_scene(S04)
    for frame in (1, 30):
        st = ctx.frame_state(s04, frame)
        fc = HO.frame_constants(scene, frame)
        np.testing.assert_allclose(st.camera, fc["camera"], rtol=0, atol=2e-7)
        np.testing.assert_allclose(st.lights, fc["lights"], rtol=1e-7, atol=1e-7)
        np.testing.assert_allclose(st.materials, fc["materials"], rtol=0, atol=1e-7)
        np.testing.assert_allclose(st.world, fc["world"], rtol=1e-7)


def test_trace_batches_bit_exact(ctx, s04):
    rng = np.random.default_rng(1234)
    st = ctx.frame_state(s04, 30)
    center = st.tris.reshape(-1, 3).mean(axis=0)
    rays = np.concatenate([_rays_random(rng, 20000, center, 6.0),
                           _rays_random(rng, 2000, center, 0.5)])  # many origins inside the cube
    hits, prims, occ = ctx.trace(s04, 30, rays)
    oh, op, oo = O.trace(st.tris, rays)
    assert np.array_equal(prims, op), f"{np.count_nonzero(prims != op)} prim mismatches"
    assert np.array_equal(hits, oh), f"{np.count_nonzero(hits != oh)} hit-record mismatches"
    assert np.array_equal(occ, oo)
    assert (prims >= 0).mean() > 0.3
    # the LBVH result equals brute force over all triangles
    bh, bp = O.trace_brute(st.tris, rays)
    assert np.array_equal(bp, op)
    assert np.array_equal(bh[:, 0], oh[:, 0])


def test_trace_qbvh_small_scene(ctx, s04):
    """The quantised 6-wide walk on the 12-triangle scene (forced; frames use the LDS BVH2)."""
    rng = np.random.default_rng(99)
    st = ctx.frame_state(s04, 45)
    assert int(st.render_ints[7]) == 2
    center = st.tris.reshape(-1, 3).mean(axis=0)
    rays = np.concatenate([_rays_random(rng, 5000, center, 6.0), _rays_random(rng, 500, center, 0.5)])
    hits, prims, occ = ctx.trace(s04, 45, rays, width=4)
    oh, op, oo = O.trace(st.tris, rays, width=4)
    assert np.array_equal(prims, op) and np.array_equal(hits, oh) and np.array_equal(occ, oo)
    ch, bx, order = ctx.qbvh(s04, 45, with_order=True)
    och, obx, oorder = O.build_qbvh(st.tris, with_order=True)
    assert np.array_equal(ch, och) and np.array_equal(bx, obx) and np.array_equal(order, oorder)


def test_trace_edge_cases(ctx, s04):
    st = ctx.frame_state(s04, 1)
    v = st.tris[0, 0].astype(np.float64)
    rays = np.array([
        [*(v + [0, 0, 5]), 0.0, 0, 0, -1, 1e30],      # straight down through a vertex
        [*(v + [0, 0, 5]), 0.0, 0, 0, 1, 1e30],       # away from the mesh
        [0, 0, 10, 0.0, 0, 0, -1, 0.5],               # tmax too short
        [0, 0, 10, 20.0, 0, 0, -1, 1e30],             # tmin past the mesh
        [0, 0, 0, 0.0, 1, 0, 0, 1e30],                # axis-aligned, zero components
    ], np.float32)
    hits, prims, occ = ctx.trace(s04, 1, rays)
    oh, op, oo = O.trace(st.tris, rays)
    assert np.array_equal(prims, op) and np.array_equal(hits, oh) and np.array_equal(occ, oo)
    assert prims[1] == -1 and prims[2] == -1 and prims[3] == -1
    # empty batch
    h0, p0, o0 = ctx.trace(s04, 1, np.zeros((0, 8), np.float32))
    assert len(p0) == 0


# "tiles": k_tiles (default for LDS-resident scenes); "wavefront": the split
# trace / shade kernels over the quantised 6-wide hierarchy (RR_FLAG_WAVEFRONT), the path
# large scenes take (frame_state reports render_ints[7] == 4 for it, so the
# oracle walks the same hierarchy without the hull rule).
PATHS = {"tiles": 0, "wavefront": 4}


@pytest.mark.parametrize("path", sorted(PATHS))
@pytest.mark.parametrize("frame,w,h,spp,chunk", [(1, 160, 90, 16, 0), (30, 96, 54, 8, 3), (60, 64, 36, 5, 1),
                                                 (600, 33, 17, 7, 2), (30, 1, 1, 9, 0), (45, 7, 130, 3, 0),
                                                 # grids of 1..7 blocks (fewer than k_tiles' unit shards)
                                                 (30, 8, 130, 3, 0), (45, 16, 24, 2, 0), (5, 40, 40, 33, 0),
                                                 # > kFilmGroup (32) samples: grouped film sum, k_tiles
                                                 # sample-group slices, groups straddling chunks
                                                 (5, 40, 24, 72, 20), (10, 48, 32, 128, 0), (20, 24, 16, 65, 7)])
def test_full_frame_bit_exact(ctx, rr, s04, frame, w, h, spp, chunk, path):
    p = rr.default_params(width=w, height=h, spp=spp, spp_per_chunk=chunk, flags=PATHS[path])
    film, rgba, stats = ctx.render_to_memory(s04, frame, p)
    st = ctx.frame_state(s04, frame, p)
    of, orgba = O.render_state(st)
    assert stats.camera_rays == w * h * spp
    assert 0 <= stats.camera_rays_traced <= stats.camera_rays
    assert stats.width == w and stats.height == h and stats.spp == spp
    nbad = int(np.count_nonzero(rgba != orgba))
    assert nbad == 0, f"{nbad} 8-bit mismatches"
    assert np.array_equal(film, of), f"max film diff {np.max(np.abs(film - of))}"
    assert film[..., :3].mean() > 0.01


def test_tiles_equal_wavefront_full_resolution(ctx, rr, s04):
    """BASELINE size (1920x1080) at low spp: k_tiles (tile-binned camera rays,
    LDS BVH2) and the split path (quantised 6-wide hierarchy) give the same
    bits. Both decide hits with the watertight woop_test and open every box that
    can hold an accepted triangle (box margins), so neither the hierarchy nor
    the camera-ray binning changes a hit. (Round 3's Moeller-Trumbore test with
    an unwidened quantised slab test let a few edge-grazing camera rays differ
    between the paths.)"""
    out, traced = {}, {}
    for path, flags in PATHS.items():
        p = rr.default_params(spp=4, flags=flags)
        film, rgba, st = ctx.render_to_memory(s04, 30, p)
        out[path] = (film, rgba, st.extension_rays, st.shadow_rays, st.primary_continued, st.primary_shadow)
        traced[path] = st.camera_rays_traced
    a, b = out["tiles"], out["wavefront"]
    # 40 samples: two film groups, k_tiles' box tiles in two slices
    f40 = [ctx.render_to_memory(s04, 7, rr.default_params(spp=40, flags=flags))[0] for flags in PATHS.values()]
    n40 = int(np.count_nonzero(f40[0] != f40[1]))
    n4 = int(np.count_nonzero(a[0] != b[0]))
    print(f"film values differing between the paths: {n4} at 4 spp, {n40} at 40 spp (of {a[0].size})")
    assert a[0].shape == (1080, 1920, 4)
    assert n40 == 0 and n4 == 0
    assert np.array_equal(a[1], b[1])
    assert a[2:] == b[2:], (a[2:], b[2:])  # ray counts
    assert a[2] > 0 and a[3] > 0
    # k_tiles also skips camera rays whose tile meets no triangle: fewer traced
    assert 0 < traced["tiles"] <= traced["wavefront"] < 1920 * 1080 * 4


@pytest.mark.parametrize("path", sorted(PATHS))
def test_ray_counts_match_oracle(ctx, rr, s04, path):
    """rr_frame_stats' ray counts equal the oracle's (04vs frame 6, 1920x1080 x
    4 spp), and no path reaches a second surface: the cube is closed and
    convex, so a continuation leaves it for good unless a camera ray slipped
    through an edge crack into it. Round 3's triangle test let such paths in
    (this frame had one, bouncing inside); the watertight test does not.
    k_tiles once counted its ballots inside the live-lane branch, which lost
    bounces run while the wave's lane 0 was already dead, without changing a
    pixel."""
    p = rr.default_params(spp=4, flags=PATHS[path])
    film, _, st = ctx.render_to_memory(s04, 6, p)
    of, _ = O.render_state(ctx.frame_state(s04, 6, rr.default_params(spp=4)))
    assert np.array_equal(film, of)
    (c0, s0, c1, s1), late = O.ray_counts()
    print(f"{path}: oracle continuations {c0} + {c1}, shadow rays {s0} + {s1}, late paths {late[:3]}")
    assert (st.primary_continued, st.primary_shadow) == (c0, s0)
    assert (st.extension_rays, st.shadow_rays) == (c0 + c1, s0 + s1)
    assert c0 > 0 and c1 == 0 and s1 == 0
    # escaped rays (left a hull side, resolved without a traversal): on the
    # cube every face is a hull side, so k_tiles traverses no secondary ray;
    # the split path has no hull rule and traverses them all
    if path == "tiles":
        assert (st.extension_rays_escaped, st.shadow_rays_escaped) == (st.extension_rays, st.shadow_rays)
    else:
        assert (st.extension_rays_escaped, st.shadow_rays_escaped) == (0, 0)
    assert st.stack_drops == 0  # counted in every frame, not only the counting pass


def test_no_path_enters_the_cube(ctx, rr, s04):
    """Frames 1..60 of 04vs at 1920x1080 x 4 spp through the split path (every
    secondary ray traversed, no hull rule): a path reaches a second surface
    only after a camera ray grazed the cube's silhouette, i.e. met the far
    face exactly at the edge it shares with a visible one (where the two
    faces' hit distances differ by rounding); no camera ray enters the cube
    through a crack. The frames with such paths, and four others, are
    rendered by the oracle too: the same ray counts, and every late path's
    camera ray hits within 1e-6 of the scene's extent of a triangle edge
    (test_oracle.py late_paths_at_edges)."""
    from test_oracle import late_paths_at_edges
    p = rr.default_params(spp=4, flags=PATHS["wavefront"])
    late_frames, n_late = [], 0
    for f in range(1, 61):
        _, _, st = ctx.render_to_memory(s04, f, p)
        extra = st.extension_rays - st.primary_continued
        n_late += extra
        if extra or f in (1, 6, 30, 60):
            fs = ctx.frame_state(s04, f, p)
            O.render_state(fs, film=False, rgba=False)
            (c0, s0, c1, s1), late = O.ray_counts()
            assert (c0, s0, c0 + c1, s0 + s1) == (st.primary_continued, st.primary_shadow, st.extension_rays,
                                                   st.shadow_rays), f
            if extra:
                late_frames.append(f)
                d_edge = late_paths_at_edges(fs.tris, fs, late)
                print(f"frame {f}: {extra} late continuations, camera hits {d_edge} from an edge")
                assert max(d_edge) < 1e-6
    print(f"60 frames: {n_late} continuations past bounce 0 in frames {late_frames}")
    assert n_late <= 60 * 1920 * 1080 * 4 * 1e-7


def test_watertight_edge_rays_on_device(ctx, s04):
    """Rays aimed at the 04vs cube's vertices and edges from outside
    (tests/test_oracle.py edge_vertex_rays): on the device's BVH2 and its
    quantised 6-wide walk, bit for bit the oracle's, no ray that passes
    through the cube misses it, and none hits it past its entry point."""
    from test_oracle import convex_leaks, edge_vertex_rays
    st = ctx.frame_state(s04, 30)
    rays = edge_vertex_rays(st.tris, 20000, 11)
    for width in (2, 4):
        hits, prims, occ = ctx.trace(s04, 30, rays, width=width)
        oh, op, oo = O.trace(st.tris, rays, width=width)
        assert np.array_equal(prims, op) and np.array_equal(hits, oh) and np.array_equal(occ, oo)
        # prims are original ids: st.tris is in original order
        leaks, lost, through = convex_leaks(st.tris, rays, prims, hits[:, 0])
        print(f"width {width}: {int(through.sum())} rays through the cube, {lost} lost, {leaks} past the entry")
        assert leaks == 0 and lost == 0 and through.sum() > 5000


def test_chunking_and_determinism(ctx, rr, s04):
    outs = []
    for chunk in (1, 4, 0):
        p = rr.default_params(width=80, height=45, spp=12, spp_per_chunk=chunk)
        film, rgba, _ = ctx.render_to_memory(s04, 30, p)
        outs.append((film, rgba))
    for f, r in outs[1:]:
        assert np.array_equal(f, outs[0][0]) and np.array_equal(r, outs[0][1])


def test_seed_changes_noise(ctx, rr, s04):
    a = ctx.render_to_memory(s04, 30, rr.default_params(width=64, height=36, spp=4, seed=1))[0]
    b = ctx.render_to_memory(s04, 30, rr.default_params(width=64, height=36, spp=4, seed=2))[0]
    assert not np.array_equal(a, b)
    assert abs(float(a.mean()) - float(b.mean())) < 0.02


def test_furnace_known_answer(ctx, rr):
    """Lambert sphere, albedo 0.5, world (0.8, 0.6, 0.4): every camera sample on the
    sphere is exactly 0.5*world after one bounce (zero variance)."""
    s = ctx.load_scene(scene_path("test_furnace.rrscene"))
    film, _, _ = ctx.render_to_memory(s, 1, None)
    center = film[20:28, 28:36, :3].reshape(-1, 3)
    np.testing.assert_allclose(center, np.tile([0.4, 0.3, 0.2], (len(center), 1)), rtol=2e-6)
    corner = film[0, 0, :3]
    np.testing.assert_allclose(corner, [0.8, 0.6, 0.4], rtol=1e-6)
    st = ctx.frame_state(s, 1)
    of, _ = O.render_state(st)
    assert np.array_equal(film, of)
    s.close()


def test_point_light_closed_form(ctx, rr):
    s = ctx.load_scene(scene_path("test_pointlight.rrscene"))
    film, _, _ = ctx.render_to_memory(s, 1, rr.default_params(spp=64))
    st = ctx.frame_state(s, 1)
    cam = st.camera
    W, H = 64, 64
    # analytic radiance at the pixel centre's plane point (camera looks straight down)
    py, px = np.mgrid[0:H, 0:W]
    sx = ((px + 0.5) * (2.0 / W) - 1.0) * cam[12]
    sy = (1.0 - (py + 0.5) * (2.0 / H)) * cam[13]
    x, y = cam[0] + sx * 10.0, cam[1] + sy * 10.0
    lx, ly, lz = 1.0, 0.5, 2.0
    r2 = (x - lx) ** 2 + (y - ly) ** 2 + lz ** 2
    I = 100.0 / (4 * np.pi)
    L = 0.8 / np.pi * I * lz / r2 ** 1.5
    rel = np.abs(film[..., 0] - L) / L
    assert np.median(rel) < 0.01, np.median(rel)
    of, _ = O.render_state(ctx.frame_state(s, 1, rr.default_params(spp=64)))
    assert np.array_equal(film, of)
    s.close()


def test_render_frame_writes_named_files(ctx, rr, s04, tmp_path):
    p = rr.default_params(width=128, height=72, spp=4)
    out = str(tmp_path / "frames" / "000007")
    os.makedirs(tmp_path / "frames")
    t, stats = ctx.render_frame(s04, 7, p, out, "JPEG", 90)
    f = tmp_path / "frames" / "000007.jpg"
    assert f.is_file() and stats.output_bytes == f.stat().st_size
    assert t.loaded_at <= t.started_rendering_at <= t.finished_rendering_at == t.file_saving_started_at
    assert t.file_saving_started_at <= t.file_saving_finished_at
    _, rgba, _ = ctx.render_to_memory(s04, 7, p)
    # the device JPEG path (jpeg.hip: transform + Huffman coding) produces the
    # same bytes as the all-host encoder on the same 8-bit image
    rr.encode_image(rgba, str(tmp_path / "host_encoded"), "JPEG", 90)
    assert (tmp_path / "host_encoded.jpg").read_bytes() == f.read_bytes()
    jpg = np.asarray(Image.open(f).convert("RGB")).astype(np.float64)
    mse = np.mean((jpg - rgba[..., :3]) ** 2)
    assert 10 * np.log10(255 ** 2 / max(mse, 1e-9)) > 35.0
    t2, _ = ctx.render_frame(s04, 7, p, str(tmp_path / "frames" / "00007"), "PNG", 90)
    png = np.asarray(Image.open(tmp_path / "frames" / "00007.png").convert("RGBA"))
    assert np.array_equal(png, rgba)
    with pytest.raises(rr.RRError) as e:
        ctx.render_frame(s04, 7, p, str(tmp_path / "x"), "TIFF", 90)
    assert e.value.code == -95
    with pytest.raises(rr.RRError) as e:
        ctx.render_frame(s04, 7, p, str(tmp_path / "missing_dir" / "x"), "PNG", 90)
    assert e.value.code == -5


def _hit_rows(film, world, n, rng):
    """n 4-row bands spread over the rows whose pixels show the cube (film
    differs from the world colour), each with its cube-pixel count."""
    hit = np.any(np.abs(film[..., :3] - world[None, None, :]) > 1e-4 * np.abs(world).max(), axis=-1)
    rows = np.nonzero(hit.sum(axis=1) > 0)[0]
    assert len(rows) >= 4 * n, len(rows)
    starts = np.linspace(rows[0], rows[-1] - 3, n).astype(int)
    return [(int(r), int(hit[r:r + 4].sum())) for r in starts]


@pytest.mark.parametrize("frame", [1, 5, 10])
def test_bench_config_properties(ctx, rr, s04, frame):
    """The bench workload (1920x1080, 128 spp) on frames 1, 5 and 10 of the 04vs
    job: too big for the oracle whole, so size-independent properties plus
    four bit-exact oracle bands per frame, each through the cube."""
    film, rgba, stats = ctx.render_to_memory(s04, frame, None)
    assert film.shape == (1080, 1920, 4)
    assert stats.camera_rays == 1920 * 1080 * 128
    assert 0 < stats.camera_rays_traced < stats.camera_rays
    assert stats.extension_rays > 0 and stats.shadow_rays > 0
    film2, rgba2, _ = ctx.render_to_memory(s04, frame, None)
    assert np.array_equal(film, film2)
    st = ctx.frame_state(s04, frame)
    bands = _hit_rows(film, st.world, 4, None)
    for r0, n_hit in bands:
        of, orgba = O.render_state(st, rows=(r0, r0 + 4))
        print(f"frame {frame} rows {r0}..{r0 + 3}: {n_hit} cube pixels")
        assert n_hit > 0
        assert np.array_equal(rgba[r0:r0 + 4], orgba[r0:r0 + 4])
        assert np.array_equal(film[r0:r0 + 4], of[r0:r0 + 4])
    bg = film[1060:1080, 0:20, :3]
    np.testing.assert_allclose(bg, 0.050876088, rtol=1e-5)


def test_01_full_resolution_slices(ctx, rr):
    """The 01 scene at its own 1920x1080 x 128 spp (C3's frame): two oracle
    bands through the cube, bit for bit (rendered with Standard here: no
    OCIO LUTs are configured on the context, and the frame says so)."""
    s = ctx.load_scene(S01)
    try:
        film, rgba, stats = ctx.render_to_memory(s, 20, None)
        assert stats.view_transform_substituted == 1
        st = ctx.frame_state(s, 20)
        for r0, n_hit in _hit_rows(film, st.world, 2, None):
            of, orgba = O.render_state(st, rows=(r0, r0 + 4))
            print(f"01 frame 20 rows {r0}..{r0 + 3}: {n_hit} cube pixels")
            assert n_hit > 0
            assert np.array_equal(rgba[r0:r0 + 4], orgba[r0:r0 + 4])
            assert np.array_equal(film[r0:r0 + 4], of[r0:r0 + 4])
    finally:
        s.close()


def test_01_scene_renders(ctx, rr):
    s = ctx.load_scene(S01)
    p = rr.default_params(width=64, height=36, spp=4)
    film, rgba, _ = ctx.render_to_memory(s, 45, p)
    of, orgba = O.render_state(ctx.frame_state(s, 45, p))
    assert np.array_equal(rgba, orgba)
    s.close()


def test_backend_runner_job(rr, tmp_path):
    """BackendRunner.render_frame over a job TOML: file names per the reference
    naming rule, seven ordered timestamps in the trace."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    job = rr.BlenderJob.load_from_file(os.path.join(root, "jobs", "04_very-simple_demo_10f-1w.toml"))
    job = rr.BlenderJob.from_dict({**job.to_dict(), "output_directory_path": str(tmp_path / "out")})
    runner = rr.BackendRunner(root, params=rr.default_params(width=64, height=36, spp=2))
    try:
        for f in job.frames()[:3]:
            frt = runner.render_frame(job, f)
            vals = [getattr(frt, k) for k in rr.traces.FRAME_FIELDS]
            assert vals == sorted(vals), vals
    finally:
        runner.close()
    names = sorted(os.listdir(tmp_path / "out"))
    assert names == ["000001.jpg", "000002.jpg", "000003.jpg"]
    assert [i for i, _ in runner.tracer.frames()] == [1, 2, 3]


def test_blender_cli_shim(rr, tmp_path):
    """The --blenderBinary seam: the reference argv in, the reference stdout out."""
    out_fmt = str(tmp_path / "######")
    argv = [rr.SHIM_PATH, S04.replace(".rrscene", ".blend"), "--background", "--python", "script.py", "--",
            "--render-output", out_fmt, "--render-format", "PNG", "--render-frame", "12"]
    env = dict(os.environ, RR_WIDTH="64", RR_HEIGHT="36", RR_SPP="2")
    # the .blend does not exist: the shim resolves <stem>.rrscene next to it
    res = subprocess.run(argv, capture_output=True, text=True, env=env, timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    stats = HO.parse_blender_stdout(res.stdout)
    assert (tmp_path / "000012.png").is_file()
    assert f"Saved: '{tmp_path}/000012.png'" in res.stdout
    assert stats["loaded_at"] <= stats["started_rendering_at"] <= stats["file_saving_finished_at"]
    bad = subprocess.run([rr.SHIM_PATH, S04, "--", "--render-format", "PNG"], capture_output=True, text=True,
                         timeout=60)
    assert "Missing render-and-timing-script arguments!" in bad.stdout


def test_pipelined_frames_match_serial(ctx, rr, tmp_path, s04):
    """rr_frame_submit / rr_frame_complete with two frames in flight writes
    byte-identical files to rr_render_frame, in submission order."""
    p = rr.default_params(width=160, height=90, spp=4)
    serial = {}
    for f in (3, 4, 5, 7):
        ctx.render_frame(s04, f, p, str(tmp_path / f"s{f}"), "JPEG", 90)
        serial[f] = (tmp_path / f"s{f}.jpg").read_bytes()
    t3 = ctx.submit_frame(s04, 3, p, str(tmp_path / "p3"), "JPEG", 90)
    t4 = ctx.submit_frame(s04, 4, p, str(tmp_path / "p4"), "JPEG", 90)
    t7 = ctx.submit_frame(s04, 7, p, str(tmp_path / "p7"), "JPEG", 90)
    assert rr.native.RR_MAX_FRAMES_IN_FLIGHT == 3
    with pytest.raises(rr.RRError) as e:  # a fourth frame in flight
        ctx.submit_frame(s04, 5, p, str(tmp_path / "p5"), "JPEG", 90)
    assert e.value.code == rr.native.RR_EBUSY
    with pytest.raises(rr.RRError):  # out of order
        ctx.complete_frame(t4)
    tm3, st3 = ctx.complete_frame(t3)
    t5 = ctx.submit_frame(s04, 5, p, str(tmp_path / "p5"), "PNG", 90)
    tm4, _ = ctx.complete_frame(t4)
    ctx.complete_frame(t7)
    tm5, _ = ctx.complete_frame(t5)
    assert (tmp_path / "p3.jpg").read_bytes() == serial[3]
    assert (tmp_path / "p4.jpg").read_bytes() == serial[4]
    assert (tmp_path / "p7.jpg").read_bytes() == serial[7]
    assert (tmp_path / "p5.png").is_file()
    for tm in (tm3, tm4, tm5):
        assert tm.loaded_at <= tm.started_rendering_at <= tm.finished_rendering_at <= tm.file_saving_finished_at
    assert st3.camera_rays == 160 * 90 * 4
    # a synchronous call works again once nothing is pending
    ctx.render_frame(s04, 6, p, str(tmp_path / "s6"), "JPEG", 90)


def test_overlapped_frames_match_serial_across_paths(ctx, rr, tmp_path, s04):
    """Two k_tiles frames in flight run side by side on the slots' streams
    (each with its own hierarchy build, tile buffers and JPEG scratch); a
    split-path frame (02 stand-in, 92k triangles) in between waits for its
    predecessor. Every file equals the serial render byte for byte, also when
    consecutive tile frames of different resolutions and sample counts share
    the device."""
    s02 = ctx.load_scene(scene_path("02_physics-standin.rrscene"))
    try:
        plan = [(s04, 5, rr.default_params(width=480, height=270, spp=64)),
                (s04, 9, rr.default_params(width=320, height=180, spp=40)),
                (s02, 60, rr.default_params(width=160, height=90, spp=4)),
                (s04, 2, rr.default_params(width=480, height=270, spp=64)),
                (s04, 60, rr.default_params(width=480, height=270, spp=64)),
                (s04, 30, rr.default_params(width=480, height=270, spp=64))]
        serial = []
        for i, (s, f, p) in enumerate(plan):
            ctx.render_frame(s, f, p, str(tmp_path / f"s{i}"), "JPEG", 90)
            serial.append((tmp_path / f"s{i}.jpg").read_bytes())
        pending = []
        for i, (s, f, p) in enumerate(plan):
            if len(pending) == rr.native.RR_MAX_FRAMES_IN_FLIGHT:
                ctx.complete_frame(pending.pop(0))
            pending.append(ctx.submit_frame(s, f, p, str(tmp_path / f"p{i}"), "JPEG", 90))
        for t in pending:
            ctx.complete_frame(t)
        for i in range(len(plan)):
            assert (tmp_path / f"p{i}.jpg").read_bytes() == serial[i], f"frame {i} of the plan differs"
    finally:
        s02.close()


def test_backend_runner_render_frames_pipelined(rr, tmp_path):
    """BackendRunner.render_frames: every frame written, traced once, in order."""
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    job = rr.BlenderJob.load_from_file(os.path.join(root, "jobs", "04_very-simple_demo_10f-1w.toml"))
    job = rr.BlenderJob.from_dict({**job.to_dict(), "output_directory_path": str(tmp_path)})
    runner = rr.BackendRunner(root, params=rr.default_params(width=96, height=54, spp=2))
    seen = []
    frts = runner.render_frames(job, job.frames(), on_frame=lambda f, frt, st: seen.append(f))
    assert seen == job.frames() and len(frts) == len(seen)
    assert sorted(os.listdir(tmp_path)) == [f"{f:06d}.jpg" for f in job.frames()]
    # render spans from the device clock (rr_api.cpp rr_frame_complete): frames
    # overlap on the device, yet the spans are consecutive and together cover
    # no more than the wall time the frames took (timings straight from the
    # library, before traces.py's clamping)
    import time
    p = rr.default_params(width=480, height=270, spp=64)
    scene = runner._scene(rr.parse_with_base_directory_prefix(job.project_file_path, root))
    t0 = time.time()
    pending, timings = [], []
    for f in range(1, 13):
        if len(pending) == rr.native.RR_MAX_FRAMES_IN_FLIGHT:
            timings.append(runner.ctx.complete_frame(pending.pop(0))[0])
        pending.append(runner.ctx.submit_frame(scene, f, p, str(tmp_path / f"span{f}"), "JPEG", 90))
    timings += [runner.ctx.complete_frame(t)[0] for t in pending]
    wall = time.time() - t0
    runner.close()
    spans = [(t.started_rendering_at, t.finished_rendering_at) for t in timings]
    assert all(a <= b for a, b in spans)
    assert all(spans[i][1] <= spans[i + 1][0] for i in range(len(spans) - 1)), spans
    total = sum(b - a for a, b in spans)
    print(f"12 overlapped frames: render spans {total * 1e3:.1f} ms of {wall * 1e3:.1f} ms wall")
    assert t0 <= spans[0][0] and spans[-1][1] <= t0 + wall and 0 < total <= wall


@pytest.mark.parametrize("seed", [0, 3, 6, 7, 11, 14])
def test_random_soups_bit_exact_against_traversed_oracle(ctx, rr, tmp_path, seed):
    """Random non-convex LDS-resident soups (tests/soups.py, <= 60 triangles):
    k_tiles (tile-binned camera rays, hull rule, screen culling) equals the
    oracle rendering the same frame with every camera ray and every
    secondary ray traversed, bit for bit."""
    import soups
    path = str(tmp_path / f"soup{seed}.rrscene")
    tris = soups.soup_scene(S04, seed, path)
    s = ctx.load_scene(path)
    try:
        frame = 1 + (3 * seed) % 30
        p = rr.default_params(width=160, height=90, spp=24)
        film, rgba, stats = ctx.render_to_memory(s, frame, p)
        st = ctx.frame_state(s, frame, p)
        assert int(st.render_ints[7]) == 2  # LDS-resident: k_tiles
        with O.rules(cull=False, hull=False):
            of, orgba = O.render_state(st)
        print(f"soup {seed}: {len(tris)} triangles, {soups.hull_sides(tris)} hull sides, "
              f"{stats.camera_rays_traced} camera rays traced")
        assert np.array_equal(film, of), f"{np.count_nonzero(film != of)} film mismatches"
        assert np.array_equal(rgba, orgba)
    finally:
        s.close()


def test_lds_residency_boundary_renders_bit_exact(ctx, rr, tmp_path):
    """at the LDS residency boundary (tests/test_scene.py
    restates the byte count k_tiles allocates; 3 blocks per CU) the largest
    resident soup renders through k_tiles and the next size up through the split
    path, and both equal the oracle bit for bit (the k_tiles launch at the
    boundary runs at the residency rule's 3 blocks per CU, not the launch
    bounds' 4-5, so its grid is the occupancy query's, never more blocks than
    fit)."""
    import soups
    from test_scene import tiles_lds_per_block
    base = rr.Scene(S04)
    c = base.counts()
    base.close()
    n_max = max(n for n in range(1, 129) if 3 * tiles_lds_per_block(n, c["materials"], c["lights"]) <= 160 * 1024)
    for n, hier in ((n_max, 2), (n_max + 1, 4)):
        path = str(tmp_path / f"soup_{n}.rrscene")
        soups.soup_scene(S04, 9, path, n=n)
        s = ctx.load_scene(path)
        try:
            p = rr.default_params(width=192, height=108, spp=40)
            film, rgba, stats = ctx.render_to_memory(s, 7, p)
            st = ctx.frame_state(s, 7, p)
            assert int(st.render_ints[7]) == hier and (int(stats.tile_slices) > 0) == (hier == 2), (n, hier)
            of, orgba = O.render_state(st)
            print(f"{n} triangles: hierarchy {hier}, tile_slices {stats.tile_slices}, "
                  f"{stats.camera_rays_traced} camera rays traced")
            assert np.array_equal(film, of), f"{n}: {np.count_nonzero(film != of)} film mismatches"
            assert np.array_equal(rgba, orgba)
        finally:
            s.close()


@pytest.mark.parametrize("job_name,frames", [("04_very-simple_demo_10f-1w.toml", list(range(1, 11))),
                                             ("01_simple-animation_600f-8w_dynamic.toml", [1, 20, 60, 61])])
def test_timed_configuration_full_frames_bit_exact(rr, tmp_path, job_name, frames):
    """The bench's timed configuration under the oracle: BackendRunner.render_frames
    exactly as bench.py times it (scene defaults 1920x1080 x 128 spp, three
    frames in flight, so every k_tiles frame after the first overlaps a pending
    one and runs as whole-tile work units, tile_slices == 1), one write_still
    per frame (render-timing-script.py:90) under the worker's queue loop
    (queue.rs:79-118), PNG so the written file is lossless. Every pixel of
    every written frame, all 1,080 rows, equals the oracle's bit for bit."""
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    job = rr.BlenderJob.load_from_file(os.path.join(root, "jobs", job_name))
    job = rr.BlenderJob.from_dict({**job.to_dict(), "output_directory_path": str(tmp_path),
                                   "output_file_format": "PNG"})
    runner = rr.BackendRunner(root, params=rr.default_params())
    slices = {}
    try:
        runner.render_frames(job, frames, on_frame=lambda f, frt, st: slices.__setitem__(f, int(st.tile_slices)))
        print(f"{job_name}: tile_slices per frame {slices}")
        assert slices[frames[0]] == 4 and all(slices[f] == 1 for f in frames[1:])
        scene = runner._scene(rr.parse_with_base_directory_prefix(job.project_file_path, root))
        for f in frames:
            out = rr.naming.output_path_without_extension(str(tmp_path), job.output_file_name_format, f)
            img = np.asarray(Image.open(out + ".png").convert("RGBA"))
            assert img.shape == (1080, 1920, 4)
            st = runner.ctx.frame_state(scene, f)
            t0 = time.time()
            _, orgba = O.render_state(st, film=False)
            n_cube = int(np.count_nonzero(np.any(img[..., :3] != img[-1, 0, :3], axis=-1)))
            nbad = int(np.count_nonzero(img != orgba))
            print(f"  frame {f}: {n_cube} cube pixels, {nbad} mismatches (oracle {time.time() - t0:.1f} s)")
            assert n_cube > 0
            assert nbad == 0, f"frame {f}: {nbad} mismatches"
    finally:
        runner.close()


def test_empty_scene_is_the_world(ctx, rr, tmp_path):
    """A scene without triangles (k_world): every sample is the world term, the
    film its grouped sum, equal to the oracle's frame of an empty hierarchy."""
    import json
    with open(S04) as f:
        sc = json.load(f)
    m = sc["meshes"][0]
    m["vertices"], m["triangles"], m["material_indices"], m["smooth"] = [], [], [], []
    path = str(tmp_path / "empty.rrscene")
    with open(path, "w") as f:
        json.dump(sc, f)
    s = ctx.load_scene(path)
    try:
        p = rr.default_params(width=40, height=24, spp=40)
        film, rgba, st = ctx.render_to_memory(s, 3, p)
        fs = ctx.frame_state(s, 3, p)
        assert s.counts()["triangles"] == 0 and st.camera_rays_traced == 0 and st.extension_rays == 0
        of, orgba = O.render_state(fs)
        assert np.array_equal(film, of) and np.array_equal(rgba, orgba)
        np.testing.assert_allclose(film[..., :3], np.broadcast_to(fs.world, (24, 40, 3)), rtol=1e-6)
    finally:
        s.close()


def test_tile_schedule_record(ctx, rr, s04):
    """rr_debug_tile_costs after a counting tile frame: every screen tile of the
    scene's box that holds work has a unit time, the hand-out order of the
    launch is a permutation of the box tiles, and the unit log holds a start
    before the end of every sliced unit (4 per box tile at 128 spp)."""
    p = rr.default_params(width=320, height=180, spp=128, flags=rr.native.RR_FLAG_COUNT_TRAVERSAL)
    for _ in range(4):  # every frame slot has run a launch, so the last order is built from costs
        _, _, st = ctx.render_to_memory(s04, 5, p, film=False, rgba=True)
    assert st.tile_slices == 4
    costs, order, log = ctx.tile_costs()
    n = ((320 + 7) // 8) * ((180 + 7) // 8)
    assert costs.shape[0] >= n
    busy = np.nonzero(costs[:n])[0]
    assert busy.size > 0
    xs, ys = busy % ((320 + 7) // 8), busy // ((320 + 7) // 8)
    nb = int((xs.max() - xs.min() + 1) * (ys.max() - ys.min() + 1))
    assert sorted(order[:nb].tolist()) == list(range(nb))
    logged = np.nonzero(log[:, 1])[0]
    assert logged.size >= 4 * busy.size
    assert (log[logged, 0] <= log[logged, 1]).all() and (log[logged, 0] > 0).all()
