#!/usr/bin/env python3
"""A/B timing of library variants (tools/ab_variants.sh builds) on the GPU box,
one subprocess per variant (RR_LIB_PATH = ab_builds/<variant>/librr.so),
variants interleaved over `rounds`
rounds so that clock drift hits them alike. Per variant and scene:
  * solo: per-class kernel ms of one frame rendered alone (best of 3,
    render_to_memory: k_tiles in sample-group slices);
  * pipe: frames/s of `frames` frames through rr_frame_submit /
    rr_frame_complete with three in flight and JPEG files written, as bench.py
    times them (k_tiles frames in whole-tile units).
  python tools/ab_run.py [--rounds R] [--frames N] VARIANT... -- SCENE:FRAME:SPP ..."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd"

CHILD = r'''
import importlib, json, sys, tempfile, time
sys.path.insert(0, %r)
rr = importlib.import_module(%r)
import os as _os
if _os.environ.get("AB_ABI"):  # an older library (its stats struct is a prefix of this binding's)
    rr.native.RR_ABI_VERSION = int(_os.environ["AB_ABI"])
specs, n_pipe = %r, %d
out = {}
with rr.RenderContext(0) as ctx:
    for spec in specs:
        path, frame, spp = spec.split(":")
        s = ctx.load_scene(path)
        p = rr.default_params(spp=int(spp), flags=rr.native.RR_FLAG_PROFILE_KERNELS)
        ctx.render_to_memory(s, int(frame), p, film=False, rgba=True)
        best = None
        for _ in range(3):
            _, _, st = ctx.render_to_memory(s, int(frame), p, film=False, rgba=True)
            ms = {n: round(st.kernel_ms[k], 3) for k, n in enumerate(rr.native.KERNEL_CLASSES) if st.kernel_ms[k] > 0}
            tot = sum(ms.values())
            if best is None or tot < best[0]:
                best = (tot, ms)
        key = path.split("/")[-1].split(".")[0][:6] + ":" + frame + ":" + spp
        res = {"solo": {"total": round(best[0], 3), **best[1]}}
        if n_pipe:
            pp = rr.default_params(spp=int(spp))
            d = tempfile.mkdtemp()
            frames = [1 + (int(frame) - 1 + i) %% 10 for i in range(n_pipe + 3)]
            def run(fs):
                pend = []
                for i, f in enumerate(fs):
                    if len(pend) == rr.native.RR_MAX_FRAMES_IN_FLIGHT:
                        ctx.complete_frame(pend.pop(0))
                    pend.append(ctx.submit_frame(s, f, pp, d + "/f%%d" %% i, "JPEG", 90))
                for t in pend:
                    ctx.complete_frame(t)
            run(frames[:3])
            ctx.synchronize()
            t0 = time.perf_counter()
            run(frames[3:])
            ctx.synchronize()
            res["pipe_fps"] = round(n_pipe / (time.perf_counter() - t0), 1)
        out[key] = res
        s.close()
print(json.dumps(out))
'''


def main():
    argv = sys.argv[1:]
    rounds, frames = 1, 0
    while argv and argv[0].startswith("--") and argv[0] != "--":
        if argv[0] == "--rounds":
            rounds = int(argv[1])
        elif argv[0] == "--frames":
            frames = int(argv[1])
        argv = argv[2:]
    k = argv.index("--")
    variants, scenes = argv[:k], argv[k + 1:]
    for r in range(rounds):
        for v in variants:
            env = dict(os.environ)
            if v != "main":
                env["RR_LIB_PATH"] = os.path.join(ROOT, "ab_builds", v, "librr.so")
                abi = os.path.join(ROOT, "ab_builds", v, "ABI")
                if os.path.exists(abi):  # e.g. a previous round's library, ABI 6
                    env["AB_ABI"] = open(abi).read().strip()
            res = subprocess.run([sys.executable, "-c", CHILD % (ROOT, PKG, scenes, frames)], env=env,
                                 capture_output=True, text=True, timeout=600)
            line = res.stdout.strip().splitlines()[-1] if res.stdout.strip() else res.stderr[-500:]
            print(f"r{r} {v:10s} {line}", flush=True)
            if res.returncode != 0:
                sys.exit(res.returncode)


if __name__ == "__main__":
    main()
