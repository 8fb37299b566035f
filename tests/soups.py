"""Random LDS-resident triangle soups for the shortcut tests (test infrastructure).

Each soup is <= 60 triangles in the 04vs cube's object space ([-1, 1]^3 around
the animated cube's location): one or two star-shaped closed blobs (an
icosahedron with every vertex pushed to its own radius, so the mesh is closed
and non-convex: faces on the convex hull are hull sides, the others are not),
a few free-floating shards and, for half the seeds, a ground quad under them.
`soup_scene` writes the soup as a copy of the 04vs stand-in .rrscene (same
camera, light, materials and F-Curve), so the product renders it exactly as it
renders 04vs: an LDS-resident scene through k_tiles.
"""
from __future__ import annotations

import json

import numpy as np

_ICO_V = None
_ICO_F = np.array([[0, 11, 5], [0, 5, 1], [0, 1, 7], [0, 7, 10], [0, 10, 11], [1, 5, 9], [5, 11, 4], [11, 10, 2],
                   [10, 7, 6], [7, 1, 8], [3, 9, 4], [3, 4, 2], [3, 2, 6], [3, 6, 8], [3, 8, 9], [4, 9, 5],
                   [2, 4, 11], [6, 2, 10], [8, 6, 7], [9, 8, 1]])


def _ico_vertices():
    global _ICO_V
    if _ICO_V is None:
        t = (1 + 5 ** 0.5) / 2
        v = np.array([[-1, t, 0], [1, t, 0], [-1, -t, 0], [1, -t, 0], [0, -1, t], [0, 1, t], [0, -1, -t],
                      [0, 1, -t], [t, 0, -1], [t, 0, 1], [-t, 0, -1], [-t, 0, 1]], np.float64)
        _ICO_V = v / np.linalg.norm(v, axis=1, keepdims=True)
    return _ICO_V


def _rotation(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def random_soup(seed: int) -> np.ndarray:
    """(n, 3, 3) float32 triangles, n <= 60, object space of the 04vs cube."""
    rng = np.random.default_rng(seed)
    tris = []
    n_blobs = 1 + seed % 2
    for b in range(n_blobs):
        radii = rng.uniform(0.45, 1.0, 12) * (0.8 if n_blobs == 1 else 0.5)
        centre = rng.uniform(-0.3, 0.3, 3) if n_blobs == 1 else np.array([(-0.6 if b == 0 else 0.6), 0.0, 0.0])
        v = (_ico_vertices() * radii[:, None]) @ _rotation(rng).T + centre
        tris.extend(v[_ICO_F])
    for _ in range(int(rng.integers(2, 8))):  # shards, some poking out of the blobs
        c = rng.uniform(-0.5, 0.5, 3)
        tris.append(c + np.clip(rng.normal(0.0, 0.25, (3, 3)), -0.6, 0.6))
    if seed % 4 < 2:  # ground quad below everything
        z = -1.3
        tris.append([[-2.5, -2.5, z], [2.5, -2.5, z], [2.5, 2.5, z]])
        tris.append([[-2.5, -2.5, z], [2.5, 2.5, z], [-2.5, 2.5, z]])
    out = np.array(tris, np.float32)
    assert len(out) <= 60
    return out


def hull_sides(tris: np.ndarray) -> int:
    """Triangle sides that the whole soup lies behind (tri_hull's rule in float64,
    for reporting / asserting that a soup exercises the rule)."""
    t = tris.astype(np.float64)
    pts = t.reshape(-1, 3)
    n_sides = 0
    for tri in t:
        n = np.cross(tri[1] - tri[0], tri[2] - tri[0])
        r = pts - tri[0]
        h = r @ n
        lim = np.abs(n).sum() * np.abs(r).sum(axis=1) * 2.0 ** -12
        n_sides += int(np.all(h <= lim)) + int(np.all(-h <= lim))
    return n_sides


def padded_soup(seed: int, n: int) -> np.ndarray:
    """random_soup(seed) with small shards added (or triangles dropped) until it
    holds exactly n triangles: scenes at the LDS residency boundary."""
    tris = random_soup(seed)[:n]
    rng = np.random.default_rng(1000 + seed)
    extra = []
    while len(tris) + len(extra) < n:
        c = rng.uniform(-0.9, 0.9, 3)
        extra.append(c + np.clip(rng.normal(0.0, 0.12, (3, 3)), -0.3, 0.3))
    return np.concatenate([tris, np.array(extra, np.float32).reshape(-1, 3, 3)]).astype(np.float32)


def soup_scene(base_scene_path: str, seed: int, out_path: str, n: int | None = None) -> np.ndarray:
    """Writes the soup of `seed` (padded_soup(seed, n) when n is given) as a
    copy of the scene at base_scene_path (the 04vs stand-in) with its mesh
    replaced; returns the triangles."""
    with open(base_scene_path) as f:
        scene = json.load(f)
    tris = random_soup(seed) if n is None else padded_soup(seed, n)
    mesh = scene["meshes"][0]
    mesh["vertices"] = [float(x) for x in tris.reshape(-1)]
    mesh["triangles"] = list(range(3 * len(tris)))
    mesh["material_indices"] = [0] * len(tris)
    mesh["smooth"] = [0] * len(tris)
    scene["name"] = f"soup-{seed}"
    with open(out_path, "w") as f:
        json.dump(scene, f)
    return tris
