#!/usr/bin/env python3
"""A/B timing of library variants (tools/ab_variants.sh builds) on the GPU box:
for each variant and scene, per-class kernel ms of one frame (second of two
renders) via RR_LIB_PATH, one subprocess per variant.
  python tools/ab_run.py VARIANT... -- SCENE:FRAME:SPP ..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd"

CHILD = r'''
import importlib, json, sys
sys.path.insert(0, %r)
rr = importlib.import_module(%r)
out = {}
with rr.RenderContext(0) as ctx:
    for spec in %r:
        path, frame, spp = spec.split(":")
        s = ctx.load_scene(path)
        p = rr.default_params(spp=int(spp), flags=rr.native.RR_FLAG_PROFILE_KERNELS)
        ctx.render_to_memory(s, int(frame), p, film=False, rgba=True)
        best = None
        for _ in range(3):
            _, _, st = ctx.render_to_memory(s, int(frame), p, film=False, rgba=True)
            ms = {n: round(st.kernel_ms[k], 2) for k, n in enumerate(rr.native.KERNEL_CLASSES) if st.kernel_ms[k] > 0}
            tot = sum(ms.values())
            if best is None or tot < best[0]:
                best = (tot, ms)
        out[path.split("/")[-1].split(".")[0][:6] + ":" + frame + ":" + spp] = {"total": round(best[0], 2), **best[1]}
        s.close()
print(json.dumps(out))
'''


def main():
    k = sys.argv.index("--")
    variants, scenes = sys.argv[1:k], sys.argv[k + 1:]
    for v in variants:
        env = dict(os.environ)
        if v != "main":
            env["RR_LIB_PATH"] = os.path.join(ROOT, PKG, "build", "ab_" + v, "librr.so")
        r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, PKG, scenes)], env=env, capture_output=True,
                           text=True, timeout=600)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-500:]
        print(f"{v:10s} {line}", flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
