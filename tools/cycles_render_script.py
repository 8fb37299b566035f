"""Blender-side render harness for the Cycles CPU baseline / image oracle.

The jobs under jobs/ point `render_script_path` here. The MI355X backend does
not execute it (frames are rendered in-process through include/rr.h); it exists
so the 04 and 01 job TOMLs can drive the REFERENCE worker with a real Blender
3.6 (`--blenderBinary /path/to/blender`) when one is available: their
project_file_path names a .blend (blender-projects/01_simple-animation/
01_simple-animation.blend, the reference's own; blender-projects/04_very-simple/
04_very-simple-standin.blend, written by tools/make_standin_blend.py), which
the worker hands to Blender as the project (worker/src/rendering/runner/
mod.rs:140-146). Cycles is pinned to the settings the MI355X renderer
implements (SURVEY.md §7 hard parts b-d): engine CYCLES on the CPU, fixed
samples (no adaptive sampling, no denoiser), bounce limit, indirect clamp,
Blackman-Harris 1.5 px filter, seed, no dithering. Resolution, frame range and
the view transform are the .blend's own (1920x1080 at 100 % in both; the 04
stand-in is Standard, 01 is Filmic, as the GPU backend renders them when the
context has Blender's OCIO LUTs).

CLI (after the last "--"), stdout protocol and timing semantics are those the
reference worker parses (worker/src/rendering/runner/utilities.rs:105-203):
  --render-output PATH --render-format FMT --render-frame N
prints RESULTS={"project_loaded_at", "project_started_rendering_at",
"project_finished_rendering_at"} after Blender's own "Saved:" / " Time:" lines.
Environment overrides: RR_SPP (default 128), RR_MAX_BOUNCES (12),
RR_CLAMP_INDIRECT (10), RR_SEED (0).
"""
import json
import os
import sys
import time

import bpy  # noqa: F401  (only importable inside Blender)

T_LOADED = time.time()


def script_args(argv):
    rest = argv[len(argv) - 1 - argv[::-1].index("--") + 1:] if "--" in argv else []
    out = {}
    it = iter(rest)
    for a in it:
        if a in ("--render-output", "--render-format", "--render-frame"):
            out[a[2:]] = next(it, None)
    return out


def hash_substitute(path, frame):
    n = path.count("#")
    return path.replace("#" * n, str(frame).rjust(n, "0"))


def main():
    a = script_args(sys.argv)
    if not all(a.get(k) for k in ("render-output", "render-format", "render-frame")):
        print("Missing render-and-timing-script arguments!")
        bpy.ops.wm.quit_blender()
        return
    frame = int(a["render-frame"])
    scene = bpy.context.scene
    scene.render.engine = "CYCLES"
    cy = scene.cycles
    cy.device = "CPU"
    cy.samples = int(os.environ.get("RR_SPP", "128"))
    cy.use_adaptive_sampling = False
    cy.use_denoising = False
    cy.max_bounces = int(os.environ.get("RR_MAX_BOUNCES", "12"))
    cy.sample_clamp_indirect = float(os.environ.get("RR_CLAMP_INDIRECT", "10"))
    cy.sample_clamp_direct = 0.0
    cy.seed = int(os.environ.get("RR_SEED", "0"))
    cy.pixel_filter_type = "BLACKMAN_HARRIS"
    cy.filter_width = 1.5
    scene.render.dither_intensity = 0.0  # the GPU backend does not dither
    scene.frame_set(frame)
    scene.render.filepath = hash_substitute(a["render-output"], frame)
    scene.render.image_settings.file_format = a["render-format"]
    scene.render.image_settings.quality = 90
    t0 = time.time()
    bpy.ops.render.render(animation=False, write_still=True, use_viewport=False)
    t1 = time.time()
    print("RESULTS=" + json.dumps({"project_loaded_at": T_LOADED, "project_started_rendering_at": t0,
                                   "project_finished_rendering_at": t1}))
    bpy.ops.wm.quit_blender()


main()
