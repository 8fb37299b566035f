import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
if os.path.join(ROOT, "tools") not in sys.path:  # fixture generators (tools/make_split_golden.py)
    sys.path.append(os.path.join(ROOT, "tools"))

PKG = "diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd"
SCENES = os.path.join(ROOT, "scenes")
GOLDEN = os.path.join(ROOT, "tests", "golden")
REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu on the GPU box")


@pytest.fixture(scope="session")
def rr():
    return importlib.import_module(PKG)


@pytest.fixture(scope="session")
def ctx(rr):
    c = rr.RenderContext(0)
    yield c
    c.close()


def scene_path(name: str) -> str:
    return os.path.join(SCENES, name)


def qbvh_leaf_positions(ch):
    """Positions of the quantised hierarchy's triangle array its leaf refs
    ~(first | (count - 1) << 28) name (one triangle each: ~position), in node
    order."""
    out = []
    for r in ch[ch < 0].tolist():
        x = ~int(r)
        f, k = x & 0x0FFFFFFF, (x >> 28) + 1
        out += list(range(f, f + k))
    return out


def have_reference() -> bool:
    return os.path.isdir(os.path.join(REFERENCE, "worker"))


def walk_lbvh(children):
    """Walk a BVH2 child-ref array from the root (refs >= 0: internal node,
    < 0: leaf range ~(first | (count-1) << 28)). Returns (covered sorted leaf
    indices in walk order, reachable internal nodes, leaf refs as (node, side,
    first, count))."""
    import numpy as np
    children = np.asarray(children).reshape(-1, 2)
    leaves, inner, refs = [], [], []
    stack = [0]
    while stack:
        v = stack.pop()
        inner.append(v)
        for side in range(2):
            c = int(children[v, side])
            if c >= 0:
                stack.append(c)
            else:
                x = ~c
                first, count = x & 0x0FFFFFFF, (x >> 28) + 1
                leaves.extend(range(first, first + count))
                refs.append((v, side, first, count))
    return leaves, inner, refs
