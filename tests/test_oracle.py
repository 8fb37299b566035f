"""Pins the CPU oracle itself (oracle/rr_oracle.c) before it is trusted as the
GPU's checker: Cycles (the reference's renderer) is third-party and absent, so
the oracle is pinned by analytic known answers instead:
ray/triangle cases, LBVH == brute force, uniform RNG and disk sampling, BSDF
identities, the white furnace and the point-light closed form."""
import dataclasses
import math

import numpy as np
import pytest

from conftest import walk_lbvh, scene_path
from oracle import host_oracle as HO
from oracle import oracle as O


def world_tris(scene, frame):
    tris, mats = [], []
    for o in scene["objects"]:
        if o["type"] != "MESH":
            continue
        m = scene["meshes"][o["mesh"]]
        if "generator" in m:
            raise NotImplementedError
        M = HO.object_matrix(o, frame).astype(np.float32)
        v = np.array(m["vertices"], np.float32).reshape(-1, 3)
        for tri in np.array(m["triangles"]).reshape(-1, 3):
            tris.append([[((M[r, 0] * v[i, 0] + M[r, 1] * v[i, 1]) + M[r, 2] * v[i, 2]) + M[r, 3]
                          for r in range(3)] for i in tri])
            mats.append(m["material_slots"][0])
    return np.array(tris, np.float32), np.array(mats, np.int32)


def icosphere_tris(sub=3, radius=1.0):
    t = (1 + 5 ** 0.5) / 2
    v = [[-1, t, 0], [1, t, 0], [-1, -t, 0], [1, -t, 0], [0, -1, t], [0, 1, t], [0, -1, -t], [0, 1, -t],
         [t, 0, -1], [t, 0, 1], [-t, 0, -1], [-t, 0, 1]]
    v = [list(np.array(p) / np.linalg.norm(p)) for p in v]
    f = [[0, 11, 5], [0, 5, 1], [0, 1, 7], [0, 7, 10], [0, 10, 11], [1, 5, 9], [5, 11, 4], [11, 10, 2],
         [10, 7, 6], [7, 1, 8], [3, 9, 4], [3, 4, 2], [3, 2, 6], [3, 6, 8], [3, 8, 9], [4, 9, 5], [2, 4, 11],
         [6, 2, 10], [8, 6, 7], [9, 8, 1]]
    for _ in range(sub):
        cache, nf = {}, []

        def mid(a, b):
            k = (min(a, b), max(a, b))
            if k not in cache:
                p = (np.array(v[a]) + np.array(v[b])) / 2
                v.append(list(p / np.linalg.norm(p)))
                cache[k] = len(v) - 1
            return cache[k]
        for a, b, c in f:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [[a, ab, ca], [b, bc, ab], [c, ca, bc], [ab, bc, ca]]
        f = nf
    V = np.array(v) * radius
    return V[np.array(f)].astype(np.float32)


def test_rng_uniform():
    u = np.concatenate([O.rng(0, p, s, 16) for p in range(200) for s in range(4)])
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 0.01 and abs(u.var() - 1 / 12) < 0.005
    assert not np.array_equal(O.rng(0, 1, 0, 8), O.rng(1, 1, 0, 8))


def test_concentric_disk_uniform():
    u = np.random.default_rng(0).random((200000, 2), dtype=np.float32)
    xy = O.disk(u)
    r2 = (xy ** 2).sum(1)
    assert r2.max() <= 1.0 + 1e-6
    assert abs((r2 < 0.25).mean() - 0.25) < 0.005  # area-uniform
    ang = np.arctan2(xy[:, 1], xy[:, 0])
    hist = np.histogram(ang, bins=16)[0]
    assert hist.min() > 0.9 * hist.mean()


def test_ray_triangle_known_cases():
    tri = np.array([[[0, 0, 0], [1, 0, 0], [0, 1, 0]]], np.float32)
    rays = np.array([[0.25, 0.25, 1, 0, 0, 0, -1, 10],     # hit, t=1, u=v=0.25
                     [0.25, 0.25, -1, 0, 0, 0, 1, 10],     # back side (two-sided)
                     [0.9, 0.9, 1, 0, 0, 0, -1, 10],       # outside (u+v>1)
                     [0.25, 0.25, 1, 0, 1, 0, 0, 10],      # parallel
                     [0.25, 0.25, 1, 0, 0, 0, -1, 0.5],    # beyond tmax
                     [0.25, 0.25, 1, 2, 0, 0, -1, 10]],    # before tmin
                    np.float32)
    hits, prims, occ = O.trace(tri, rays)
    assert list(prims) == [0, 0, -1, -1, -1, -1]
    assert hits[0, 0] == 1.0 and hits[0, 1] == 0.25 and hits[0, 2] == 0.25
    assert list(occ) == [1, 1, 0, 0, 0, 0]


def _rot(seed):
    q, _ = np.linalg.qr(np.random.default_rng(seed).normal(size=(3, 3)))
    return q.astype(np.float32)


def closed_meshes():
    """Closed convex meshes whose triangles share their vertices bit for bit:
    the 04vs cube at two frames (the product's own float32 transform,
    world_tris), an icosphere of 1,280 triangles rotated in float32, and an
    axis-aligned cube (rays can run exactly along its faces)."""
    scene = HO.load_scene(scene_path("04_very-simple-standin.rrscene"))
    out = {f"04vs-{f}": world_tris(scene, f)[0] for f in (1, 30)}
    ico = icosphere_tris(3, 1.5)
    out["ico3"] = (ico.reshape(-1, 3) @ _rot(3).T + np.float32(0.25)).astype(np.float32).reshape(-1, 3, 3)
    c = np.array([[x, y, z] for x in (-1, 1) for y in (-1, 1) for z in (-1, 1)], np.float32)
    quads = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    out["aabb"] = np.array([[c[a], c[b], c[cc]] for a, b, cc, _ in quads] +
                           [[c[a], c[cc], c[d]] for a, _, cc, d in quads], np.float32)
    return out


def edge_vertex_rays(tris, n_edge, seed):
    """Rays from outside aimed at the mesh's vertices (exactly: d = the
    normalised difference, in float32) and at random points of its edges, from
    origins on a sphere three times the mesh's radius."""
    rng = np.random.default_rng(seed)
    verts = np.unique(tris.reshape(-1, 3), axis=0)
    edges = np.concatenate([tris[:, [0, 1]], tris[:, [1, 2]], tris[:, [2, 0]]])
    t = rng.random((n_edge, 1)).astype(np.float32)
    e = edges[rng.integers(0, len(edges), n_edge)]
    pts = np.concatenate([verts, (e[:, 0] + t * (e[:, 1] - e[:, 0])).astype(np.float32)])
    ctr = tris.reshape(-1, 3).mean(axis=0)
    rad = np.linalg.norm(tris.reshape(-1, 3) - ctr, axis=1).max()
    u = rng.normal(size=(len(pts), 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    o = (ctr + 3.0 * rad * u).astype(np.float32)
    d = pts - o
    d = (d / np.linalg.norm(d.astype(np.float64), axis=1, keepdims=True)).astype(np.float32)
    return np.concatenate([o, np.zeros((len(o), 1)), d, np.full((len(o), 1), 1e30)], axis=1).astype(np.float32)


def outward_normals(tris):
    n = np.cross(tris[:, 1] - tris[:, 0], tris[:, 2] - tris[:, 0]).astype(np.float64)
    ctr = tris.reshape(-1, 3).mean(axis=0)
    s = np.sign(np.einsum("ij,ij->i", n, tris.mean(axis=1) - ctr))
    return n * s[:, None]


@pytest.mark.parametrize("name", ["04vs-1", "04vs-30", "ico3", "aabb"])
def test_watertight_edges_and_vertices(name):
    """Closed meshes hit from outside at their edges and vertices: every ray
    that reaches the mesh hits a front face first — no ray slips through a
    shared edge or vertex into the interior (a back face), on the BVH2, the
    quantised 6-wide walk and brute force alike (woop_test with margins on the
    box tests). A ray aimed at a surface point can only miss when it grazes
    the silhouette."""
    tris = closed_meshes()[name]
    rays = edge_vertex_rays(tris, 20000, 7)
    if name == "aabb":  # rays exactly along the faces' planes, at the edges
        extra = []
        for a in range(3):
            for s in (-1.0, 1.0):
                for b in range(3):
                    if b == a:
                        continue
                    o = np.zeros(3, np.float32)
                    o[a] = 5.0 * s
                    o[b] = 1.0
                    d = np.zeros(3, np.float32)
                    d[a] = -s
                    extra.append([*o, 0.0, *d, 1e30])
        rays = np.concatenate([rays, np.array(extra, np.float32)])
    bh, bp = O.trace_brute(tris, rays)
    for width in (2, 4):
        h, p, occ = O.trace(tris, rays, width=width)
        assert np.array_equal(p, bp), f"width {width}: {np.count_nonzero(p != bp)} differ from brute force"
        assert np.array_equal(occ.astype(bool), p >= 0)
    leaks, lost, through = convex_leaks(tris, rays, bp, bh[:, 0])
    print(f"{name}: {len(rays)} rays, {int(through.sum())} through the solid, {lost} of them lost, "
          f"{leaks} hits past the entry point")
    assert leaks == 0 and lost == 0
    assert through.mean() > 0.5


def convex_leaks(tris, rays, prims, t_hit):
    """Against the exact (double) entry / exit distances of a closed convex
    mesh (the largest entering, the smallest leaving face-plane distance):
    hits farther than the entry point (a path through a crack to the inside
    of a far face) and rays that pass through the solid, entry to exit longer
    than 1e-4 of their distance, yet hit nothing (a path through a crack to
    the other side). A ray grazing the silhouette may hit or miss; on an edge
    it may hit either face, at the entry distance. Returns (hits past the
    entry, rays lost, mask of the rays through the solid)."""
    n = outward_normals(tris)
    o, d = rays[:, 0:3].astype(np.float64), rays[:, 4:7].astype(np.float64)
    den = d @ n.T                                            # (rays, faces)
    num = np.einsum("fk,fk->f", n, tris[:, 0].astype(np.float64))[None, :] - o @ n.T
    with np.errstate(divide="ignore", invalid="ignore"):
        tf = num / den
        t_entry = np.where(den < 0, tf, -np.inf).max(axis=1)
        t_exit = np.where(den > 0, tf, np.inf).min(axis=1)
    hit = prims >= 0
    scale = np.linalg.norm(o - tris.reshape(-1, 3).mean(axis=0), axis=1)
    late = hit & (t_hit.astype(np.float64) > t_entry + 1e-4 * scale)
    through = (t_exit - t_entry > 1e-4 * scale) & (t_entry > 0)
    return int(late.sum()), int((through & ~hit).sum()), through


def late_paths_at_edges(tris, state, late):
    """For late paths (pixel, sample) of oracle.ray_counts(): the distance of
    each one's camera hit from the nearest triangle edge, relative to the
    scene's extent (the camera ray traced by the oracle, O.camera_rays)."""
    pix = [int(p) for p, _ in late]
    smp = [int(q) for _, q in late]
    rays = O.camera_rays(state, pix, smp)
    h, p, _ = O.trace(tris, rays, width=2)
    t = tris.astype(np.float64)
    ext = float(np.ptp(t.reshape(-1, 3), axis=0).max())
    out = []
    for r, hh, pp in zip(rays, h, p):
        assert pp >= 0
        P = r[0:3].astype(np.float64) + float(hh[0]) * r[4:7].astype(np.float64)
        best = np.inf
        for a, b in ((0, 1), (1, 2), (2, 0)):
            A, B = t[:, a], t[:, b]
            u = np.clip(np.einsum("ij,ij->i", P - A, B - A) / np.einsum("ij,ij->i", B - A, B - A), 0, 1)
            best = min(best, float(np.linalg.norm(P - (A + u[:, None] * (B - A)), axis=1).min()))
        out.append(best / ext)
    return out


@pytest.mark.parametrize("frame", [6, 47, 50])
def test_late_paths_start_at_silhouette_edges(rr, frame):
    """04vs at 1920x1080 x 4 spp through the traversed hierarchy (the split
    path's, no hull rule): a path that reaches a second surface of the closed,
    convex cube started with a camera ray that met the cube exactly on an edge
    (its hit within 1e-6 of the cube's extent of a triangle edge) — a graze of
    the silhouette, where the far face's hit distance can round below the near
    one's; no camera ray passes through a crack (test_watertight_edges_and_
    vertices). Frames 47 and 50 have such paths, frame 6 (the frame whose
    path leaked through an edge crack under round 3's triangle test) has none."""
    scene = HO.load_scene(scene_path("04_very-simple-standin.rrscene"))
    s = rr.Scene(scene_path("04_very-simple-standin.rrscene"))
    try:
        st = s.frame_constants(frame, rr.default_params(spp=4))
    finally:
        s.close()
    tris, mats = world_tris(scene, frame)
    ri = np.array(st.render_ints, np.int32)
    ri[7] = 4  # the quantised 6-wide walk of the split path
    O.render(tris, mats, st.camera, st.lights, st.materials, st.world, ri, st.render_floats, film=False, rgba=False)
    (c0, s0, c1, s1), late = O.ray_counts()
    print(f"frame {frame}: continuations {c0} + {c1}, late paths {late}")
    assert c0 > 0
    assert (c1 > 0) == (frame != 6) and len(late) == c1
    st = dataclasses.replace(st, render_ints=ri)
    d = late_paths_at_edges(tris, st, late)
    print(f"  camera hits of the late paths: {d} of the extent from an edge")
    assert all(x < 1e-6 for x in d)


def test_lbvh_structure_and_brute_force():
    rng = np.random.default_rng(5)
    n = 3000
    c = rng.uniform(-10, 10, (n, 1, 3))
    tris = (c + rng.normal(0, 0.4, (n, 3, 3))).astype(np.float32)
    keys, order, children, boxes = O.build_lbvh(tris)
    assert np.all(np.diff(keys.astype(np.int64)) >= 0)
    assert sorted(order) == list(range(n))
    leaves, inner, refs = walk_lbvh(children)
    assert sorted(leaves) == list(range(n))  # the walk covers every leaf exactly once
    assert len(set(inner)) == len(inner)
    assert max(c for (_, _, _, c) in refs) <= 8  # ORC_LEAF_MAX (1: one triangle per leaf)
    # boxes contain their triangles
    for node, side, first, count in refs[::37]:
        t = tris[order[first:first + count]]
        lo, hi = boxes[node, 6 * side:6 * side + 3], boxes[node, 6 * side + 3:6 * side + 6]
        assert np.all(t >= lo) and np.all(t <= hi)
    o = rng.uniform(-15, 15, (4000, 3))
    d = rng.normal(size=(4000, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, np.zeros((4000, 1)), d, np.full((4000, 1), 1e30)], axis=1).astype(np.float32)
    hits, prims, occ = O.trace(tris, rays)
    bh, bp = O.trace_brute(tris, rays)
    assert np.array_equal(prims, bp)
    assert np.array_equal(hits[:, 0], bh[:, 0])
    assert np.array_equal(occ.astype(bool), bp >= 0)
    assert (prims >= 0).mean() > 0.1


def test_lbvh_degenerate_inputs():
    tri = np.array([[[0, 0, 0], [1, 0, 0], [0, 1, 0]]], np.float32)
    k, o, ch, b = O.build_lbvh(tri)
    assert list(ch[0]) == [~0, ~0]
    same = np.repeat(tri, 50, axis=0)  # 50 identical triangles: duplicate Morton keys
    k, o, ch, b = O.build_lbvh(same)
    assert np.all(k == k[0]) and sorted(o) == list(range(50))
    hits, prims, _ = O.trace(same, np.array([[0.2, 0.2, 1, 0, 0, 0, -1, 5]], np.float32))
    assert prims[0] == 0  # equal t: the smallest original id wins


def test_lambert_and_principled_bsdf():
    n = [0, 0, 1]
    wo = [0, 0.6, 0.8]
    wi = [0.6, 0, 0.8]
    lam = [0.5, 0.25, 1.0, 0, 0, 1.0, 1.45, 0, 0, 0, 1.0, 0]
    f, pdf = O.bsdf_eval(lam, n, wo, wi)
    np.testing.assert_allclose(f, np.array([0.5, 0.25, 1.0]) / np.pi, rtol=1e-6)
    assert pdf == pytest.approx(0.8 / np.pi, rel=1e-6)
    pr = [0.8, 0.8, 0.8, 0.0, 0.5, 0.5, 1.45, 0, 0, 0, 0.0, 0]
    f1, _ = O.bsdf_eval(pr, n, wo, wi)
    f2, _ = O.bsdf_eval(pr, n, wi, wo)
    np.testing.assert_allclose(f1, f2, rtol=1e-6)  # reciprocity
    f3, p3 = O.bsdf_eval(pr, n, wo, [0.6, 0, -0.8])
    assert np.all(f3 == 0) and p3 == 0


@pytest.mark.parametrize("cos_v", [0.95, 0.6, 0.2])
@pytest.mark.parametrize("roughness,metallic", [(0.5, 0.0), (0.3, 1.0)])
def test_principled_sampling_matches_evaluation(cos_v, roughness, metallic):
    """The lobe sampler and the BSDF's pdf agree (what makes the path estimator
    unbiased): E[f cos / pdf] over sample_bsdf draws equals a quadrature of
    the same integral over the hemisphere (the directional albedo), and the
    pdf integrates over the hemisphere to the fraction of draws that continue."""
    mat = [0.8, 0.7, 0.6, metallic, 0.5, roughness, 1.45, 0, 0, 0, 0.0, 0]
    n = [0.0, 0.0, 1.0]
    wo = [math.sqrt(1.0 - cos_v * cos_v), 0.0, cos_v]
    k = 400_000
    g = np.random.default_rng(11)
    wi, f, pdf, ok = O.bsdf_sample(mat, n, wo, g.random((k, 3), dtype=np.float32))
    assert np.all(pdf[ok] > 0) and np.all(wi[ok, 2] > 0)
    w = np.where(ok, wi[:, 2] / np.where(ok, pdf, 1.0), 0.0)
    est_is = (f * w[:, None]).mean(0)
    # midpoint quadrature over the hemisphere in (z = cos theta, phi): dω = dz dphi
    nz, nphi = 2048, 512
    z = (np.arange(nz) + 0.5) / nz
    phi = (np.arange(nphi) + 0.5) * (2.0 * math.pi / nphi)
    zz, pp = np.meshgrid(z, phi, indexing="ij")
    r = np.sqrt(1.0 - zz * zz)
    wu = np.stack([r * np.cos(pp), r * np.sin(pp), zz], -1).reshape(-1, 3)
    fu, pu = O.bsdf_eval_n(mat, n, wo, wu)
    dw = (1.0 / nz) * (2.0 * math.pi / nphi)
    est_q = (fu.astype(np.float64) * (zz.reshape(-1) * dw)[:, None]).sum(0)
    np.testing.assert_allclose(est_is, est_q, rtol=0.02)
    assert 0.05 < est_is.min() and est_is.max() < 1.0          # energy: albedo below 1
    assert float(pu.astype(np.float64).sum() * dw) == pytest.approx(float(ok.mean()), rel=0.01)


def _render_scene(name, frame=1, **over):
    """Oracle render from the Python restatement (no product code involved)."""
    scene = HO.load_scene(scene_path(name))
    r = scene["render"]
    W, H = r["resolution_x"], r["resolution_y"]
    fc = HO.frame_constants(scene, frame)
    tris, mats = [], []
    for o in scene["objects"]:
        if o["type"] != "MESH":
            continue
        g = scene["meshes"][o["mesh"]]["generator"]
        if g["type"] == "icosphere":
            t = icosphere_tris(g["subdivisions"], g["radius"])
        else:
            h = g["size"] / 2
            t = np.array([[[-h, -h, 0], [h, -h, 0], [h, h, 0]], [[-h, -h, 0], [h, h, 0], [-h, h, 0]]], np.float32)
        tris.append(t + np.array(o["location"], np.float32))
        mats += [0] * len(t)
    ri = np.array([W, H, over.get("spp", r["samples"]), over.get("max_bounces", r["max_bounces"]), r["seed"],
                   1 if r["view_transform"] == "Raw" else 0, 0, 0,
                   over.get("max_diffuse", r.get("max_diffuse_bounces", 4)),
                   over.get("max_glossy", r.get("max_glossy_bounces", 4))], np.int32)
    rf = np.array([r["clamp_indirect"], r["filter_width"], 1.0, 0], np.float32)
    return O.render(np.concatenate(tris), np.array(mats), fc["camera"], fc["lights"], fc["materials"],
                    fc["world"], ri, rf, threads=4)


def test_white_furnace():
    film, rgba = _render_scene("test_furnace.rrscene")
    center = film[20:28, 28:36, :3].reshape(-1, 3)
    np.testing.assert_allclose(center, np.tile([0.4, 0.3, 0.2], (len(center), 1)), rtol=2e-6)
    np.testing.assert_allclose(film[0, 0, :3], [0.8, 0.6, 0.4], rtol=1e-6)
    assert rgba[0, 0, 0] == 204 and rgba[24, 32, 0] == 102  # Raw view: round(0.8*255), round(0.4*255)


def test_point_light_closed_form():
    film, _ = _render_scene("test_pointlight.rrscene", spp=64)
    scene = HO.load_scene(scene_path("test_pointlight.rrscene"))
    cam = HO.frame_constants(scene, 1)["camera"]
    py, px = np.mgrid[0:64, 0:64]
    sx = ((px + 0.5) * (2.0 / 64) - 1.0) * cam[12]
    sy = (1.0 - (py + 0.5) * (2.0 / 64)) * cam[13]
    x, y = sx * 10.0, sy * 10.0
    r2 = (x - 1.0) ** 2 + (y - 0.5) ** 2 + 4.0
    L = 0.8 / math.pi * (100.0 / (4 * math.pi)) * 2.0 / r2 ** 1.5
    rel = np.abs(film[..., 0] - L) / L
    assert np.median(rel) < 0.01 and np.percentile(rel, 95) < 0.05


def test_04_frame_is_plausible():
    scene = HO.load_scene(scene_path("04_very-simple-standin.rrscene"))
    fc = HO.frame_constants(scene, 30, 96, 54)
    tris, mats = world_tris(scene, 30)
    ri = np.array([96, 54, 8, 12, 0, 0, 0, 0], np.int32)
    rf = np.array([10.0, 1.5, 1.0, 0], np.float32)
    film, rgba = O.render(tris, mats, fc["camera"], fc["lights"], fc["materials"], fc["world"], ri, rf,
                          threads=4)
    bg = film[50, 2, :3]
    np.testing.assert_allclose(bg, fc["world"], rtol=1e-6)  # background pixel = world colour
    assert film[..., 0].max() > 0.3  # the lit cube face
    # deterministic, and row slices reproduce the full render exactly
    f2, r2 = O.render(tris, mats, fc["camera"], fc["lights"], fc["materials"], fc["world"], ri, rf,
                      rows=(10, 20), threads=2)
    assert np.array_equal(f2[10:20], film[10:20]) and np.array_equal(r2[10:20], rgba[10:20])
    # and so do rows picked anywhere in one call (one hierarchy build)
    rows = [0, 3, 17, 18, 40, 53]
    f3, r3 = O.render(tris, mats, fc["camera"], fc["lights"], fc["materials"], fc["world"], ri, rf,
                      row_list=rows, threads=3)
    assert np.array_equal(f3[rows], film[rows]) and np.array_equal(r3[rows], rgba[rows])
    others = [y for y in range(54) if y not in rows]
    assert not f3[others].any() and not r3[others].any()


@pytest.mark.parametrize("frame,ground", [(1, False), (30, False), (60, True), (5, True)])
def test_hull_escape_changes_no_pixel(frame, ground):
    """LDS-resident scenes (render_ints[7] == 2) skip the traversal of a
    secondary ray that leaves a triangle on a side the whole scene lies behind
    (tri_hull). Such a ray meets nothing, so the frame equals the one rendered
    with every secondary ray traversed (render_ints[7] == 3: PLOC hierarchy,
    no hull rule) bit for bit — on the cube, where every face is a hull side,
    and with a ground quad under it, where the side faces are not."""
    scene = HO.load_scene(scene_path("04_very-simple-standin.rrscene"))
    fc = HO.frame_constants(scene, frame, 64, 36)
    tris, mats = world_tris(scene, frame)
    if ground:
        g = np.array([[[-6, -6, -1.5], [6, -6, -1.5], [6, 6, -1.5]], [[-6, -6, -1.5], [6, 6, -1.5], [-6, 6, -1.5]]],
                     np.float32)
        tris, mats = np.concatenate([tris, g]), np.concatenate([mats, mats[:2]])
    rf = np.array([10.0, 1.5, 1.0, 0], np.float32)
    films = []
    for hier in (2, 3):
        ri = np.array([64, 36, 16, 12, 0, 0, 0, hier, 4, 4], np.int32)
        f, _ = O.render(tris, mats, fc["camera"], fc["lights"], fc["materials"], fc["world"], ri, rf, threads=4)
        films.append(f)
    assert films[0][..., 0].max() > 0.3
    assert np.array_equal(films[0], films[1])


def _soup_frame(tmp_path, seed, frame, W=128, H=72):
    """Frame inputs of random soup `seed` (tests/soups.py) in the 04vs stand-in."""
    import soups
    path = str(tmp_path / f"soup{seed}.rrscene")
    soups.soup_scene(scene_path("04_very-simple-standin.rrscene"), seed, path)
    scene = HO.load_scene(path)
    tris, mats = world_tris(scene, frame)
    return HO.frame_constants(scene, frame, W, H), tris, mats


@pytest.mark.parametrize("seed", list(range(20)))
def test_hull_rule_random_soups(tmp_path, seed):
    """The hull rule (tri_hull) on 20 random non-convex LDS-resident soups of
    <= 60 triangles (star-shaped closed blobs, free shards, half with a ground
    quad): frames with the rule equal frames with every secondary ray
    traversed, bit for bit, on the same hierarchy (render_ints[7] == 2)."""
    import soups
    fc, tris, mats = _soup_frame(tmp_path, seed, 1 + (3 * seed) % 30)
    n_sides = soups.hull_sides(tris)
    rf = np.array([10.0, 1.5, 1.0, 0], np.float32)
    ri = np.array([128, 72, 16, 12, 0, 0, 0, 2, 4, 4], np.int32)
    args = (tris, mats, fc["camera"], fc["lights"], fc["materials"], fc["world"], ri, rf)
    f_rule, r_rule = O.render(*args, threads=4)
    with O.rules(hull=False):
        f_all, r_all = O.render(*args, threads=4)
    print(f"soup {seed}: {len(tris)} triangles, {n_sides} hull sides")
    assert len(tris) <= 60 and n_sides > 0
    assert np.any(np.abs(f_rule[..., :3] - fc["world"][None, None, :]) > 1e-3)  # the soup is on screen
    assert np.array_equal(f_rule, f_all), f"{np.count_nonzero(f_rule != f_all)} film mismatches"
    assert np.array_equal(r_rule, r_all)


@pytest.mark.parametrize("case", ["04vs-1", "04vs-30", "04vs-60", "soup-3", "soup-6", "soup-11"])
@pytest.mark.parametrize("hier", [2, 3])
def test_screen_cull_changes_no_pixel(tmp_path, case, hier):
    """Camera rays outside the scene's projected bounding rectangle (screen_rect,
    one pixel of slack) are misses without a traversal. Rendering with the
    rule and with every camera ray traced gives the same film bit for bit, on
    the LBVH (LDS-resident path, camera rays against every triangle) and on
    the PLOC hierarchy."""
    kind, k = case.split("-")
    if kind == "04vs":
        scene = HO.load_scene(scene_path("04_very-simple-standin.rrscene"))
        fc = HO.frame_constants(scene, int(k), 96, 54)
        tris, mats = world_tris(scene, int(k))
    else:
        fc, tris, mats = _soup_frame(tmp_path, int(k), 20, 96, 54)
    rf = np.array([10.0, 1.5, 1.0, 0], np.float32)
    ri = np.array([96, 54, 8, 12, 0, 0, 0, hier, 4, 4], np.int32)
    args = (tris, mats, fc["camera"], fc["lights"], fc["materials"], fc["world"], ri, rf)
    f_cull, _ = O.render(*args, threads=4)
    with O.rules(cull=False):
        f_all, _ = O.render(*args, threads=4)
    bg = np.all(np.abs(f_cull[..., :3] - fc["world"][None, None, :]) <= 1e-7, axis=-1)
    print(f"{case} hier {hier}: {int(bg.sum())} of {bg.size} pixels background")
    assert 0 < bg.sum() < bg.size  # the rectangle leaves background pixels to cull
    assert np.array_equal(f_cull, f_all), f"{np.count_nonzero(f_cull != f_all)} film mismatches"


def _q6_child_boxes(node):
    """Decoded child boxes of one quantised 6-wide node (rr_device.h QNode6),
    in double: lo/hi = org + q * 2^e per axis, (6, 3) each."""
    org = node[0:3].view(np.float32).astype(np.float64)
    e = np.array([((int(node[3]) >> (8 * a)) & 255) - 128 for a in range(3)])
    q = np.zeros((6, 6), np.float64)  # [child, lo x lo y lo z hi x hi y hi z]
    for c in range(6):
        for k in range(6):
            if c < 4:
                q[c, k] = (int(node[6 + k]) >> (8 * c)) & 255
            else:
                q[c, k] = (int(node[12 + k // 2]) >> (16 * (k & 1) + 8 * (c - 4))) & 255
    return org + q[:, 0:3] * np.exp2(e), org + q[:, 3:6] * np.exp2(e)


def _q6_refs(node):
    """The implicit child references of a node, spelled out as rr_debug_qbvh
    does: internal slot c -> first internal child + internal slots before c,
    leaf slot -> ~(first leaf triangle + leaf slots before c), unused
    (lo 255 / hi 0) -> 0x7fffffff."""
    inner = int(node[3]) >> 24
    out = []
    for c in range(6):
        below = bin(inner & ((1 << c) - 1)).count("1")
        lox = (int(node[6]) >> (8 * c)) & 255 if c < 4 else (int(node[12]) >> (8 * (c - 4))) & 255
        hix = (int(node[9]) >> (8 * c)) & 255 if c < 4 else (int(node[13]) >> (16 + 8 * (c - 4))) & 255
        if (inner >> c) & 1:
            out.append(int(node[4]) + below)
        elif lox == 255 and hix == 0:
            out.append(0x7FFFFFFF)
        else:
            out.append(~(int(node[5]) + c - below))
    return out


def leaf_range(r):
    """(first, count) of a leaf ref ~(first | (count - 1) << 28)."""
    x = ~int(r)
    return x & 0x0FFFFFFF, (x >> 28) + 1


def qbvh_leaf_positions(ch):
    """Positions of the hierarchy's triangle array its leaf refs name, in node order."""
    out = []
    for r in ch[(ch < 0)].tolist():
        f, k = leaf_range(r)
        out += list(range(f, f + k))
    return out


def _check_q4_contains(tris, ch, nodes, order):
    """Every quantised child box contains the boxes of all triangles below it
    (order: original triangle id of each position of the hierarchy's triangle array)."""
    bvh4_tris = tris.reshape(-1, 9)[order].reshape(-1, 3, 3)

    def walk(i):
        lo4, hi4 = _q6_child_boxes(nodes[i])
        under = []
        for c in range(6):
            r = int(ch[i, c])
            if r == 0x7FFFFFFF:
                continue
            if r < 0:
                f, k = leaf_range(r)
                ids = list(range(f, f + k))
            else:
                ids = walk(r)
            under += ids
            t = bvh4_tris[ids].reshape(-1, 3).astype(np.float64)
            assert np.all(lo4[c] <= t.min(0)) and np.all(t.max(0) <= hi4[c]), (i, c)
        return under

    assert sorted(walk(0)) == list(range(tris.shape[0]))
    assert sorted(order.tolist()) == list(range(tris.shape[0]))  # a permutation


@pytest.mark.parametrize("n,seed", [(1, 0), (2, 1), (7, 2), (300, 3), (5000, 4)])
def test_qbvh_collapse_and_walk_equal_brute_force(n, seed):
    """Quantised 6-wide collapse of the PLOC hierarchy: every leaf once, every
    node but the root once, quantised boxes containing their subtrees, the
    implicit child references as spelled out; the wide walk finds the
    brute-force closest hits."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(-5, 5, (n, 1, 3))
    tris = (c + rng.normal(0, 0.6, (n, 3, 3))).astype(np.float32)
    ch, nodes, order = O.build_qbvh(tris, with_order=True)
    assert np.array_equal(np.array([_q6_refs(x) for x in nodes], np.int32).reshape(ch.shape), ch)
    leaves = qbvh_leaf_positions(ch)
    assert sorted(leaves) == list(range(n))
    assert all(leaf_range(r)[1] == 1 for r in ch[ch < 0].tolist())  # one triangle per leaf
    assert n < 300 or np.mean((ch != 0x7FFFFFFF).sum(1)) > 3.5  # (nodes over two single-triangle leaves stay 2-wide)
    inner = ch[(ch >= 0) & (ch != 0x7FFFFFFF)]
    assert np.array_equal(np.sort(inner), np.arange(1, ch.shape[0]))
    if n > 1:
        _check_q4_contains(tris, ch, nodes, order)
    m = 4000
    rays = np.zeros((m, 8), np.float32)
    rays[:, 0:3] = rng.uniform(-8, 8, (m, 3))
    d = rng.normal(0, 1, (m, 3))
    rays[:, 4:7] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 7] = 1e30
    h4, p4, o4 = O.trace(tris, rays, width=4)
    h2, p2, o2 = O.trace(tris, rays, width=2)
    bh, bp = O.trace_brute(tris, rays)
    assert np.array_equal(p4, bp) and np.array_equal(p2, bp)
    assert np.array_equal(h4[:, 0], bh[:, 0])
    assert np.array_equal(o4, o2)


def test_qbvh_axis_aligned_geometry_and_rays():
    """Flat boxes (an axis-aligned grid of quads and a cube) and rays with
    exactly zero direction components: the finite reciprocal of the quantised
    walk (q4_rcp) keeps every plane distance finite, and the hits still equal
    brute force. Ray origins stay off the box planes: a ray parallel to a box
    face and exactly on it is a boundary case both the BVH2 slab test (0 * inf)
    and this walk may reject."""
    quads = []
    for i in range(8):
        for j in range(8):
            x0, z0 = i - 4.0, j - 4.0
            a, b, c, d = (x0, 0, z0), (x0 + 1, 0, z0), (x0 + 1, 0, z0 + 1), (x0, 0, z0 + 1)
            quads += [(a, b, c), (a, c, d)]
    for ax in range(3):  # a unit cube's faces at +-0.5 around (0, 1, 0)
        for s in (-0.5, 0.5):
            p = [[0.0, 1.0, 0.0] for _ in range(4)]
            u, v = (ax + 1) % 3, (ax + 2) % 3
            for k, (du, dv) in enumerate(((-.5, -.5), (.5, -.5), (.5, .5), (-.5, .5))):
                p[k][ax] += s
                p[k][u] += du
                p[k][v] += dv
            quads += [(p[0], p[1], p[2]), (p[0], p[2], p[3])]
    tris = np.array(quads, np.float32)
    ch, nodes, order = O.build_qbvh(tris, with_order=True)
    _check_q4_contains(tris, ch, nodes, order)
    rng = np.random.default_rng(7)
    rays = []
    for _ in range(3000):
        o = rng.uniform(-5, 5, 3).round(1) + 0.0123
        o[1] = abs(o[1]) + 0.25
        d = np.zeros(3)
        axes = rng.choice(3, rng.integers(1, 3), replace=False)
        d[axes] = rng.choice([-1.0, 1.0], len(axes)) * rng.uniform(0.2, 1.0, len(axes))
        d /= np.linalg.norm(d)
        rays.append([*o, 0.0, *d, 1e30])
    for _ in range(1000):  # straight down onto the grid, straight across through the cube
        x, z = rng.uniform(-4, 4, 2).round(2) + 0.0031
        rays.append([x, 3.0, z, 0.0, 0.0, -1.0, 0.0, 1e30])
        y, w = rng.uniform(0.5, 1.5), rng.uniform(-0.5, 0.5)
        rays.append([-6.0, y, w, 0.0, 1.0, 0.0, 0.0, 1e30])
    rays = np.array(rays, np.float32)
    h4, p4, o4 = O.trace(tris, rays, width=4)
    bh, bp = O.trace_brute(tris, rays)
    assert np.count_nonzero(bp >= 0) > 2000
    assert np.array_equal(p4, bp) and np.array_equal(h4[:, 0], bh[:, 0])


@pytest.mark.parametrize("n,seed", [(3, 0), (50, 1), (2000, 2)])
def test_ploc_structure_and_walk_equal_brute_force(n, seed):
    """PLOC (hier 3): a binary tree over all leaves with node 0 as the root,
    boxes containing their subtrees, closest hits equal to brute force."""
    rng = np.random.default_rng(seed)
    c = rng.uniform(-8, 8, (n, 1, 3)) * rng.uniform(0.2, 1.0, (n, 1, 1))
    tris = (c + rng.normal(0, 0.3, (n, 3, 3)) * rng.uniform(0.1, 3.0, (n, 1, 1))).astype(np.float32)
    keys, order, children, boxes = O.build_lbvh(tris, hier=3)
    k2, o2, _, _ = O.build_lbvh(tris, hier=2)
    assert np.array_equal(keys, k2) and np.array_equal(order, o2)  # same sorted leaves
    leaves, inner, refs = walk_lbvh(children)
    assert sorted(leaves) == list(range(n))
    assert sorted(inner) == list(range(n - 1))
    for node, side, first, count in refs:
        t = tris[order[first]]
        lo, hi = boxes[node, 6 * side:6 * side + 3], boxes[node, 6 * side + 3:6 * side + 6]
        assert np.all(t >= lo) and np.all(t <= hi)
    m = 3000
    rays = np.zeros((m, 8), np.float32)
    rays[:, 0:3] = rng.uniform(-10, 10, (m, 3))
    d = rng.normal(0, 1, (m, 3))
    rays[:, 4:7] = d / np.linalg.norm(d, axis=1, keepdims=True)
    rays[:, 7] = 1e30
    h3, p3, o3 = O.trace(tris, rays, width=3)
    bh, bp = O.trace_brute(tris, rays)
    assert np.array_equal(p3, bp)
    assert np.array_equal(h3[:, 0], bh[:, 0])


# ---- Cycles per-lobe bounce caps (path_state_next) --------------------------
@pytest.mark.parametrize("caps,hits", [((12, 4, 4), 5), ((12, 2, 4), 3), ((3, 4, 4), 4), ((12, 1, 4), 2),
                                       ((12, 4, 1), 5)])
def test_diffuse_bounce_cap_known_answer(caps, hits):
    """Camera inside a closed emissive (E = 0.25) white Lambert shell: the
    throughput stays 1, so every path returns E times the number of hits it
    makes before a cap ends it. Diffuse cap d (Cycles max_diffuse_bounces):
    the scatter that makes the d-th diffuse bounce ends the path at the next
    hit, whose emission still counts -> E (d + 1), the truncated series
    E (1 + rho + ... + rho^d) at rho = 1; total cap b likewise -> E (b + 1);
    the glossy cap does not touch a diffuse-only path."""
    mb, md, mg = caps
    film, _ = _render_scene("test_enclosure_diffuse.rrscene", max_bounces=mb, max_diffuse=md, max_glossy=mg)
    np.testing.assert_allclose(film[..., :3], 0.25 * hits, rtol=2e-5)


def test_glossy_bounce_cap_known_answer():
    """The same shell as a white metallic near-mirror (roughness 0: alpha
    1e-4, G1 ~ 1, F = cspec0 = 1): E (g + 1) with the glossy cap g."""
    for mg, hits in ((4, 5), (2, 3)):
        film, _ = _render_scene("test_enclosure_glossy.rrscene", spp=4, max_glossy=mg)
        assert abs(float(film[..., :3].mean()) - 0.25 * hits) < 2e-3 * hits, (mg, float(film[..., :3].mean()))
    # without per-lobe caps (caps above the total) the same shell runs to the total cap
    film, _ = _render_scene("test_enclosure_glossy.rrscene", spp=4, max_bounces=6, max_glossy=64)
    assert abs(float(film[..., :3].mean()) - 0.25 * 7) < 2e-2


def _fresnel_dielectric(c, eta):
    g = np.sqrt(eta * eta - 1 + c * c)
    A = (g - c) / (g + c)
    B = (c * (g + c) - 1) / (c * (g - c) + 1)
    return 0.5 * A * A * (1 + B * B)


def test_principled_fresnel_is_cycles_interpolated_dielectric():
    """Specular lobe at a metallic-0 grey surface against Cycles' Principled v1
    Fresnel in float64: F = cspec0 (1 - FH) + FH, FH = (Fd(L.H, ior) - F0) /
    (1 - F0), ior = 2 / (1 - sqrt(0.08 specular)) - 1 (specular 0.5 -> 1.5,
    F0 = 0.04), measured by isolating the specular term (base colour 0 turns
    the diffuse closure off; metallic 0, specular 0.5)."""
    mat = np.array([0.0, 0.0, 0.0, 0.0, 0.5, 0.4, 1.45, 0, 0, 0, 0, 0], np.float32)
    n = np.array([0, 0, 1], np.float32)
    for th_o, th_i, ph in ((0.3, 0.5, 2.0), (1.2, 0.7, 1.0), (1.45, 1.4, 3.0)):
        wo = np.array([np.sin(th_o), 0, np.cos(th_o)], np.float32)
        wi = np.array([np.sin(th_i) * np.cos(ph), np.sin(th_i) * np.sin(ph), np.cos(th_i)], np.float32)
        f, _ = O.bsdf_eval(mat, n, wo, wi)
        h = (wo.astype(np.float64) + wi) / np.linalg.norm(wo.astype(np.float64) + wi)
        a2 = (0.4 * 0.4) ** 2
        cv, cl, nh = wo[2], wi[2], h[2]
        D = a2 / (np.pi * (nh * nh * (a2 - 1) + 1) ** 2)
        G1 = lambda c: 2 * c / (c + np.sqrt(a2 + (1 - a2) * c * c))  # noqa: E731
        eta = 2 / (1 - np.sqrt(0.08 * 0.5)) - 1
        F0 = _fresnel_dielectric(1.0, eta)
        FH = (_fresnel_dielectric(float(np.dot(wi, h)), eta) - F0) / (1 - F0)
        cspec0 = 0.5 * 0.08
        F = cspec0 * (1 - FH) + FH
        ref = F * D * G1(cv) * G1(cl) / (4 * cv * cl)
        # FH is read from the material's table (128 intervals of cos, error < 4e-4)
        np.testing.assert_allclose(f, ref, rtol=1e-2)
        assert abs(eta - 1.5) < 1e-12 and abs(F0 - 0.04) < 1e-12


# ---- Filmic view transform (csrc/view.hpp) ----------------------------------
def _filmic_f64(rgb, luts):
    """The Filmic chain in float64 (the oracle's float32 result must agree to
    within one 8-bit code value)."""
    cube, lut, lo, hi = luts["cube"].astype(np.float64), luts["lut1"][:, 0].astype(np.float64), luts["lo1"], luts["hi1"]
    n = cube.shape[0]
    a = (np.log2(np.maximum(rgb, 1.17549435e-38)) + 12.473931188) / 25.0
    x = np.clip(a, 0, 1) * (n - 1)
    i0 = np.minimum(x.astype(int), n - 2)
    f = x - i0
    out = np.zeros(3)
    # tetrahedral interpolation == the barycentric interpolation inside the
    # tetrahedron of the cell containing f: sort the fractions descending
    order = np.argsort(-f, kind="stable")
    corner = i0.copy()
    prev = 1.0
    out = (1 - f[order[0]]) * cube[tuple(corner)]
    for k in range(3):
        corner[order[k]] += 1
        w = f[order[k]] - (f[order[k + 1]] if k < 2 else 0.0)
        out = out + w * cube[tuple(corner)]
    c = out / 0.66
    t = np.clip((c - lo) / (hi - lo) * (len(lut) - 1), 0, len(lut) - 1)
    j = np.minimum(t.astype(int), len(lut) - 2)
    v = lut[j] + (lut[j + 1] - lut[j]) * (t - j)
    return np.clip(np.floor(np.clip(v, 0, 1) * 255 + 0.5), 0, 255)


def test_filmic_chain_on_synthetic_luts(tmp_path):
    HO.write_synthetic_filmic_luts(str(tmp_path))
    luts = HO.load_filmic_luts(str(tmp_path))
    assert luts["cube"].shape == (17, 17, 17, 3) and luts["lut1"].shape == (1024, 1)
    O.set_filmic(luts)
    try:
        rng = np.random.default_rng(3)
        rgb = np.concatenate([np.exp2(rng.uniform(-14, 14, (3000, 3))), np.zeros((1, 3)), np.full((1, 3), 1e30),
                              np.full((1, 3), 0.18)]).astype(np.float32)
        got = O.filmic(rgb)
        exp = np.array([_filmic_f64(x.astype(np.float64), luts) for x in rgb])
        assert np.abs(got.astype(int) - exp).max() <= 1
        assert (got.astype(int) == exp).mean() > 0.97
        # rendering with view 2 applies the same chain to the film
        film, rgba = _render_scene("test_furnace.rrscene")
        r = HO.load_scene(scene_path("test_furnace.rrscene"))
        f2, rgba2 = _render_scene_view("test_furnace.rrscene", 2)
        assert np.array_equal(f2, film)
        assert np.array_equal(rgba2[..., :3].reshape(-1, 3), O.filmic(film[..., :3].reshape(-1, 3)))
    finally:
        O.set_filmic(None)


def _render_scene_view(name, view):
    scene = HO.load_scene(scene_path(name))
    scene["render"]["view_transform"] = "Raw"
    import oracle.oracle as OO
    orig = OO.render

    def patched(*a, **k):
        ri = np.array(a[6], np.int32).copy()
        ri[5] = view
        return orig(*a[:6], ri, *a[7:], **k)
    OO.render = patched
    try:
        return _render_scene(name)
    finally:
        OO.render = orig


def test_log2_fixed_accuracy():
    """The libm-free log2 of the Filmic shaper (view.hip log2_fixed) is within
    3e-7 of log2 over the normal range: checked through the shaper's
    allocation a = (log2 x + 12.47) / 25 on a 1x1x1 identity cube + identity
    curve, where one 8-bit step is 25/255 stops."""
    import os
    d = "/tmp/rr_identity_luts"
    os.makedirs(os.path.join(d, "luts"), exist_ok=True)
    with open(os.path.join(d, "luts", HO.FILMIC_LUT_FILES[0]), "w") as fh:
        fh.write("SPILUT 1.0\n3 3\n2 2 2\n")
        for i in range(2):
            for j in range(2):
                for k in range(2):
                    fh.write(f"{i} {j} {k} {0.66 * i} {0.66 * j} {0.66 * k}\n")
    with open(os.path.join(d, "luts", HO.FILMIC_LUT_FILES[1]), "w") as fh:
        fh.write("Version 1\nFrom 0 1\nLength 2\nComponents 1\n{\n0\n1\n}\n")
    O.set_filmic(HO.load_filmic_luts(d))
    try:
        x = np.exp2(np.linspace(-12.4, 12.5, 4001)).astype(np.float32)
        got = O.filmic(np.stack([x, x, x], 1))[:, 0].astype(int)
        a = (np.log2(x.astype(np.float64)) + 12.473931188) / 25.0
        exp = np.floor(np.clip(a, 0, 1) * 255 + 0.5)
        assert np.abs(got - exp).max() <= 1 and (got == exp).mean() > 0.99
    finally:
        O.set_filmic(None)


def test_material_table_matches_cycles_fresnel():
    """The material table's Fresnel channel against Cycles' exact
    interpolate_fresnel_color blend in float64, and its pick-probability
    channel against the closure sample weights (bsdf_microfacet_fresnel_color
    / principled diffuse), over specular 0..1."""
    for spec, met, base in ((0.5, 0.0, (0.8, 0.8, 0.8)), (0.2, 0.3, (0.9, 0.2, 0.1)), (1.0, 0.0, (0.1, 0.5, 0.9))):
        mat = np.array([*base, met, spec, 0.4, 1.45, 0, 0, 0, 0, 0], np.float32)
        t = O.material_lut(mat)
        eta = 2 / (1 - np.sqrt(0.08 * np.float32(spec))) - 1
        F0 = _fresnel_dielectric(1.0, eta)
        c = np.linspace(0, 1, 1001)
        fh = (_fresnel_dielectric(c, eta) - F0) / (1 - F0)
        got = np.interp(c, np.arange(129) / 128, t[:129])
        assert np.abs(got - fh).max() < 5e-4
        c0 = np.clip(np.float32(spec) * 0.08 * (1 - np.float32(met)) + np.array(base, np.float64) * np.float32(met), 0, 1)
        wsp = (c0[None, :] * (1 - fh[:, None]) + fh[:, None]).mean(1)
        wd = (1 - np.float32(met)) * np.mean(np.array(base, np.float32).astype(np.float64))
        ps = wsp / (wsp + wd)
        got = np.interp(c, np.arange(129) / 128, t[130:259])
        assert np.abs(got - ps).max() < 5e-4
        assert t[129] == t[128] and t[259] == t[258]  # repeated last entries (branch-free device lerp)
