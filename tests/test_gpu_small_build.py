"""Parity of the one-launch LBVH build (bvh.hip k_build_small: scenes of at
most 512 triangles, one workgroup) and of the multi-kernel build above that
size, against the oracle's Karras LBVH (oracle/rr_oracle.c), node for node.

Scenes are the committed furnace scene with the icosphere subdivided 0..3
times (20, 80, 320, 1280 triangles) and the point-light plane (2 triangles),
plus the 12-triangle 04vs cube; 1280 crosses the one-launch cap, so both
builders are covered by the same assertions.
"""
import json
import os

import numpy as np
import pytest

from conftest import scene_path
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _variant(tmp_path, base: str, subdiv: int | None) -> str:
    with open(scene_path(base)) as f:
        s = json.load(f)
    if subdiv is not None:
        s["meshes"][0]["generator"]["subdivisions"] = subdiv
    p = os.path.join(tmp_path, f"{os.path.splitext(base)[0]}_{subdiv}.rrscene")
    with open(p, "w") as f:
        json.dump(s, f)
    return p


CASES = [("test_pointlight.rrscene", None, 2), ("test_furnace.rrscene", 0, 20),
         ("test_furnace.rrscene", 1, 80), ("test_furnace.rrscene", 2, 320),
         ("test_furnace.rrscene", 3, 1280), ("04_very-simple-standin.rrscene", None, 12)]


@pytest.mark.parametrize("base,subdiv,n", CASES)
def test_lbvh_small_and_multi_kernel_bit_exact(ctx, tmp_path, base, subdiv, n):
    s = ctx.load_scene(_variant(tmp_path, base, subdiv))
    try:
        assert s.counts()["triangles"] == n
        for frame in (1, 30):
            st = ctx.frame_state(s, frame)
            keys, order, children, boxes = ctx.bvh(s, frame, hier=2)
            ok, oo, oc, ob = O.build_lbvh(st.tris, hier=2)
            assert np.array_equal(keys, ok)
            assert np.array_equal(order, oo)
            assert np.array_equal(children, oc)
            assert np.array_equal(boxes, ob), f"{np.count_nonzero(boxes != ob)} box mismatches"
    finally:
        s.close()


@pytest.mark.parametrize("subdiv", [2, 3])
def test_trace_through_lbvh_of_both_builders(ctx, tmp_path, subdiv):
    """Ray batches through the LBVH each builder made equal the oracle's walk."""
    s = ctx.load_scene(_variant(tmp_path, "test_furnace.rrscene", subdiv))
    try:
        st = ctx.frame_state(s, 1)
        rng = np.random.default_rng(7 + subdiv)
        n = 4096
        o = rng.uniform(-3.0, 3.0, (n, 3))
        d = rng.uniform(-0.8, 0.8, (n, 3)) - o
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        rays = np.zeros((n, 8), np.float32)
        rays[:, 0:3], rays[:, 4:7], rays[:, 7] = o, d, 1e30
        hits, prims, occ = ctx.trace(s, 1, rays, width=2)
        oh, op, oo = O.trace(st.tris, rays, width=2)
        assert np.array_equal(prims, op)
        assert np.array_equal(hits, oh)
        assert np.array_equal(occ, oo)
        assert (prims >= 0).mean() > 0.5
    finally:
        s.close()
