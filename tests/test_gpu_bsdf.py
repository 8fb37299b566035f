"""Device BSDF sampling (rr_debug_bsdf_sample: the frame kernels' mat_derive,
bsdf_view and bsdf_sample) against the oracle's sample_bsdf, bit for bit, over
materials spanning the Principled subset (roughness down to the GGX alpha
floor, metallic, specular, closure cut-offs) and view angles from normal to
grazing incidence."""
import itertools

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROUGH = [0.0, 0.02, 0.05, 0.2, 0.5, 1.0]
METAL = [0.0, 0.5, 1.0]
SPEC = [0.0, 0.5, 1.0]


def _views(rng):
    th = np.concatenate([[0.0, 1e-6, 1e-3, 0.3, 0.8, 1.2, 1.5, 1.5707], rng.uniform(0, 1.57, 4)])
    ph = rng.uniform(0, 2 * np.pi, len(th))
    return np.stack([np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), np.cos(th)], 1).astype(np.float32)


@pytest.mark.parametrize("rough", ROUGH)
def test_bsdf_sampling_bit_exact(ctx, rough):
    rng = np.random.default_rng(int(rough * 1000) + 5)
    n = np.array([0.0, 0.0, 1.0], np.float32)
    u = rng.random((2048, 3), dtype=np.float32)
    u[:4] = [[0.0, 0.5, 0.5], [0.999999, 0.0, 0.0], [0.3, 1.0, 0.0], [0.7, 0.5, 0.5]]
    bad = []
    for metal, spec in itertools.product(METAL, SPEC):
        mat = np.array([0.8, 0.6, 0.3, metal, spec, rough, 1.45, 0, 0, 0, 0, 0], np.float32)
        for wo in _views(rng):
            wo = wo / np.float32(np.linalg.norm(wo))
            g = ctx.bsdf_sample(mat, n, wo, u)
            o = O.bsdf_sample_lobes(mat, n, wo, u)
            for k, (a, b) in enumerate(zip(g, o)):
                same = np.array_equal(a, b) or (a.dtype.kind == "f" and np.array_equal(a, b, equal_nan=True))
                if not same:
                    idx = np.nonzero(~np.all((a == b) | (np.isnan(a) & np.isnan(b)), axis=tuple(range(1, a.ndim))))[0]
                    bad.append((metal, spec, tuple(float(x) for x in wo), ["wi", "f", "pdf", "ok"][k], len(idx),
                                int(idx[0]), a[idx[0]].tolist(), b[idx[0]].tolist()))
    assert not bad, "\n".join(map(str, bad[:12]))
