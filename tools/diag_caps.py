"""Diagnostic: roughness-0 metal enclosure, cube (LDS: k_tiles / wavefront) vs icosphere (split)."""
import importlib, json, os, sys, tempfile
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rr = importlib.import_module("diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd")
from oracle import oracle as O
d = tempfile.mkdtemp()
ctx = rr.RenderContext(0)
cube_v = [[x, y, z] for x in (-5, 5) for y in (-5, 5) for z in (-5, 5)]
cube_t = [0, 1, 3, 0, 3, 2, 4, 6, 7, 4, 7, 5, 0, 4, 5, 0, 5, 1, 2, 3, 7, 2, 7, 6, 0, 2, 6, 0, 6, 4, 1, 5, 7, 1, 7, 3]
for shape in ("cube", "ico1"):
    for rough in (0.0, 0.05):
        sc = json.load(open(os.path.join(ROOT, "scenes", "test_enclosure_glossy.rrscene")))
        sc["materials"][0]["roughness"] = rough
        if shape == "cube":
            sc["meshes"][0] = {"name": "box", "vertices": sum(cube_v, []), "triangles": cube_t, "material_slots": [0]}
        else:
            sc["meshes"][0]["generator"]["subdivisions"] = 1
        p = os.path.join(d, f"g_{shape}_{rough}.rrscene")
        json.dump(sc, open(p, "w"))
        s = ctx.load_scene(p)
        for flags in (0, 4):
            prm = rr.default_params(spp=4, flags=flags)
            film, rgba, st = ctx.render_to_memory(s, 1, prm)
            state = ctx.frame_state(s, 1, prm)
            of, _ = O.render_state(state)
            print(f"{shape} rough {rough} flags {flags} hier {int(state.render_ints[7])}: gpu "
                  f"{float(film[..., 0].mean()) / 0.25:.4f} oracle {float(of[..., 0].mean()) / 0.25:.4f} "
                  f"ext/cam {st.extension_rays / st.camera_rays:.4f} mism {int(np.count_nonzero(film != of))}",
                  flush=True)
        s.close()
ctx.close()
