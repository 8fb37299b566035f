#!/usr/bin/env python3
"""How many node visits of the quantised 6-wide walk a pop-time distance test
would skip (CPU, research tool): a node is visited although its entry distance,
as its parent's box test computed it, already exceeds the ray's closest hit
(the hit shrank after the push, or in the leaf tests of the same visit). Runs
the oracle's walk built with ORC_WALK_STUDY (a separate library under /tmp;
the product oracle is untouched) over collapse_study.py's rays: camera rays of
the frame, a cosine bounce ray and a shadow ray from each hit.
  python tools/walk_study.py [02|03|c5] [frame] [n_pixels]"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from oracle import oracle as O  # noqa: E402

STUDY_LIB = "/tmp/orc_walk_study/liboracle.so"


def build_study_lib():
    os.makedirs(os.path.dirname(STUDY_LIB), exist_ok=True)
    subprocess.run(["gcc", "-O2", "-std=c11", "-D_GNU_SOURCE", "-DORC_WALK_STUDY", "-fPIC", "-shared",
                    "-ffp-contract=off", "-mfma", "-fopenmp", "-o", STUDY_LIB,
                    os.path.join(ROOT, "oracle", "rr_oracle.c"), "-lm"], check=True)


def main():
    build_study_lib()
    O.LIB = STUDY_LIB
    import collapse_study as CS
    L = O.lib()
    study = np.zeros(2, np.int64)
    orig_walk = CS.walk

    def walk(tris, rays, mode):
        L.orc_walk_study(study.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), 1)
        r = orig_walk(tris, rays, mode)
        L.orc_walk_study(study.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), 1)
        if mode == 0:
            n = len(rays)
            cnt = r[3]
            print(f"    visits beyond the closest hit: {study[0] / n:.2f} of {cnt[0] / n:.2f} per ray "
                  f"({study[0] / max(cnt[0], 1):.3f}); grouped pops wholly beyond it {study[1] / n:.2f} per ray")
        return r

    CS.walk = walk
    L.orc_study_order(int(os.environ.get("WALK_ORDER", "0")))
    CS.main()


if __name__ == "__main__":
    main()
