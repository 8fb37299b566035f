"""TEST INFRASTRUCTURE ONLY — host-side restatements used as checkers.

Each function restates a reference behaviour on the hot path's host side, for
tests/ to compare the product (C++ in librr.so, Python in the package) against:

  * eval_fcurve        Blender 3.6 F-Curve evaluation (third-party; the
                       reference pins Blender 3.6.0, pull-blender-image.sh:3-4,
                       and calls it through scene.frame_set,
                       scripts/render-timing-script.py:81). Pinned by the
                       golden z table of the 01 cube (tests/golden/fcurve_01_cube_z.json,
                       SURVEY.md §8c) and the saved ob.loc.z at cfra=60.
  * object_matrix      Blender loc / XYZ-Euler / scale object matrix.
  * frame_constants    camera / light / material constants the integrator reads.
  * rigid_matrix / expand_rigid_bodies
                       closed-form rigid-body poses of the physics stand-ins
                       (C4/C5; the reference's 02/03 .blend
                       files and simulation caches are missing,
                       .MISSING_LARGE_BLOBS), restating csrc/scene.cpp's
                       generator so the product's poses are checked against an
                       independent statement of the same model.
  * parse_blender_stdout  worker/src/rendering/runner/utilities.rs:105-203
                       (extract_blender_render_information) and :51-96.
"""
from __future__ import annotations

import json
import math
import re

import numpy as np

F = np.float32


# ------------------------------------------------------------ F-Curves ----
def _sqrt3d(d: float) -> float:
    if d == 0.0:
        return 0.0
    if d < 0.0:
        return -math.exp(math.log(-d) / 3.0)
    return math.exp(math.log(d) / 3.0)


def _ok(x: np.float32) -> bool:
    return x >= F(-1.0e-10) and x <= F(1.000001)


def _solve_cubic(c0, c1, c2, c3):
    """Roots in [0,1] of c0 + c1 t + c2 t^2 + c3 t^3 (double), as float32."""
    out = []
    if c3 != 0.0:
        a, b, c = c2 / c3, c1 / c3, c0 / c3
        a = a / 3
        p = b / 3 - a * a
        q = (2 * a * a * a - a * b + c) / 2
        d = q * q + p * p * p
        if d > 0.0:
            t = math.sqrt(d)
            r = F(_sqrt3d(-q + t) + _sqrt3d(-q - t) - a)
            return [r] if _ok(r) else []
        if d == 0.0:
            t = _sqrt3d(-q)
            cands = [F(2 * t - a), F(-t - a)]
        else:
            phi = math.acos(-q / math.sqrt(-(p * p * p)))
            t = math.sqrt(-p)
            p = math.cos(phi / 3)
            q = math.sqrt(3 - 3 * p * p)
            cands = [F(2 * t * p - a), F(-t * (p + q) - a), F(-t * (p - q) - a)]
        return [r for r in cands if _ok(r)]
    a, b, c = c2, c1, c0
    if a != 0.0:
        p = b * b - 4 * a * c
        if p > 0:
            p = math.sqrt(p)
            return [r for r in (F((-b - p) / (2 * a)), F((-b + p) / (2 * a))) if _ok(r)]
        if p == 0:
            r = F(-b / (2 * a))
            return [r] if _ok(r) else []
        return []
    if b != 0.0:
        r = F(-c / b)
        return [r] if _ok(r) else []
    return [F(0.0)] if c == 0.0 else []


def eval_fcurve(keys: list, extrapolation: str, t: float) -> np.float32:
    """keys: [{"co":[x,y], "handle_left":[..], "handle_right":[..], "interpolation": ...}]."""
    K = [{k: [F(v) for v in kk[k]] for k in ("co", "handle_left", "handle_right")} | {"ipo": kk["interpolation"]}
         for kk in keys]
    t = F(t)
    n = len(K)

    def extrap(e, nb_dir):
        E = K[e]
        if E["ipo"] == "CONSTANT" or extrapolation != "LINEAR":
            return E["co"][1]
        if E["ipo"] == "LINEAR":
            if n == 1:
                return E["co"][1]
            N = K[e + nb_dir]
            dx = F(E["co"][0] - t)
            fac = F(N["co"][0] - E["co"][0])
            if fac == 0:
                return E["co"][1]
            fac = F(F(N["co"][1] - E["co"][1]) / fac)
            return F(E["co"][1] - F(fac * dx))
        h = E["handle_left"] if nb_dir > 0 else E["handle_right"]
        dx = F(E["co"][0] - t)
        fac = F(E["co"][0] - h[0])
        if fac == 0:
            return E["co"][1]
        fac = F(F(E["co"][1] - h[1]) / fac)
        return F(E["co"][1] - F(fac * dx))

    if t <= K[0]["co"][0]:
        return extrap(0, +1)
    if K[-1]["co"][0] <= t:
        return extrap(n - 1, -1)
    # segment containing t (keys strictly increasing in x)
    for a in range(1, n):
        if K[a]["co"][0] >= t:
            break
    B, P = K[a], K[a - 1]
    if abs(float(B["co"][0] - t)) <= 0.0001 or abs(float(P["co"][0] - t)) <= 0.0001:
        return B["co"][1] if abs(float(B["co"][0] - t)) <= 0.0001 else P["co"][1]
    if P["ipo"] == "CONSTANT":
        return P["co"][1]
    if P["ipo"] == "LINEAR":
        return F(F(F(B["co"][1] - P["co"][1]) * F(t - P["co"][0])) / F(B["co"][0] - P["co"][0]) + P["co"][1])
    v1, v2 = list(P["co"]), list(P["handle_right"])
    v3, v4 = list(B["handle_left"]), list(B["co"])
    eps = F(np.finfo(np.float32).eps)
    if abs(v1[1] - v4[1]) < eps and abs(v2[1] - v3[1]) < eps and abs(v3[1] - v4[1]) < eps:
        return v1[1]
    h1 = [F(v1[0] - v2[0]), F(v1[1] - v2[1])]
    h2 = [F(v4[0] - v3[0]), F(v4[1] - v3[1])]
    ln, l1, l2 = F(v4[0] - v1[0]), abs(h1[0]), abs(h2[0])
    if F(l1 + l2) != 0 and F(l1 + l2) > ln:
        fac = F(ln / F(l1 + l2))
        v2 = [F(v1[0] - F(fac * h1[0])), F(v1[1] - F(fac * h1[1]))]
        v3 = [F(v4[0] - F(fac * h2[0])), F(v4[1] - F(fac * h2[1]))]
    q0, q1, q2, q3 = v1[0], v2[0], v3[0], v4[0]
    c0 = float(F(q0 - t))
    c1 = float(F(F(3.0) * F(q1 - q0)))
    c2 = float(F(F(3.0) * F(F(q0 - F(F(2.0) * q1)) + q2)))
    c3 = float(F(F(q3 - q0) + F(F(3.0) * F(q1 - q2))))
    roots = _solve_cubic(c0, c1, c2, c3)
    if not roots:
        return F(0.0)
    u = roots[0]
    f1, f2, f3, f4 = v1[1], v2[1], v3[1], v4[1]
    k0 = f1
    k1 = F(F(3.0) * F(f2 - f1))
    k2 = F(F(3.0) * F(F(f1 - F(F(2.0) * f2)) + f3))
    k3 = F(F(f4 - f1) + F(F(3.0) * F(f2 - f3)))
    return F(F(F(k0 + F(u * k1)) + F(F(u * u) * k2)) + F(F(F(u * u) * u) * k3))


# ------------------------------------------------------------ matrices ----
def euler_xyz(rx, ry, rz) -> np.ndarray:
    ci, cj, ch = math.cos(rx), math.cos(ry), math.cos(rz)
    si, sj, sh = math.sin(rx), math.sin(ry), math.sin(rz)
    cc, cs, sc, ss = ci * ch, ci * sh, si * ch, si * sh
    return np.array([[cj * ch, sj * sc - cs, sj * cc + ss],
                     [cj * sh, sj * ss + cc, sj * cs - sc],
                     [-sj, cj * si, cj * ci]], dtype=np.float64)


def object_matrix(obj: dict, frame: float) -> np.ndarray:
    loc = list(map(float, obj.get("location", [0, 0, 0])))
    rot = list(map(float, obj.get("rotation_euler", [0, 0, 0])))
    scl = list(map(float, obj.get("scale", [1, 1, 1])))
    for fc in obj.get("animation", {}).get("fcurves", []):
        v = float(eval_fcurve(fc["keyframes"], fc.get("extrapolation", "CONSTANT"), frame))
        tgt = {"location": loc, "rotation_euler": rot, "scale": scl}.get(fc["data_path"])
        if tgt is not None and 0 <= fc["index"] < 3:
            tgt[fc["index"]] = v
    if obj.get("rotation_mode", "XYZ") != "XYZ":
        raise NotImplementedError("oracle restates XYZ Euler only")
    R = euler_xyz(*rot)
    M = np.eye(4)
    M[:3, :3] = R * np.array(scl)[None, :]
    M[:3, 3] = loc
    return M


# ------------------------------------------------------ rigid bodies ----
_M64 = (1 << 64) - 1


class _SplitMix:
    def __init__(self, state: int):
        self.s = state & _M64

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & _M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
        return z ^ (z >> 31)

    def u01(self) -> float:
        return (self.next() >> 11) * (1.0 / 9007199254740992.0)


def expand_rigid_bodies(scene: dict) -> list:
    """The motion parameters of every body of every "rigid_bodies" group, in
    object order after the scene's explicit objects."""
    r = scene["render"]
    fps, f0 = float(r.get("fps", 24)), float(r.get("frame_start", 1))
    out = []
    for g in scene.get("rigid_bodies", []):
        c = [float(x) for x in g.get("spawn_center", [0, 0, 5])]
        e = [float(x) for x in g.get("spawn_extent", [10, 10, 4])]
        sc = [float(x) for x in g.get("scale", [0.3, 0.6])]
        speed, vup, spin = float(g.get("speed", 1.0)), float(g.get("up_speed", 1.0)), float(g.get("spin", 2.0))
        win = [float(x) for x in g.get("spawn_window", [f0, f0])]
        meshes = g["meshes"]
        for i in range(int(g["count"])):
            rng = _SplitMix(int(g.get("seed", 0)) ^ ((i * 0xD1B54A32D192ED03) & _M64))
            p0 = [c[k] + (rng.u01() - 0.5) * e[k] for k in range(3)]
            scale = sc[0] + rng.u01() * (sc[1] - sc[0])
            v0 = [(rng.u01() - 0.5) * 2.0 * speed, (rng.u01() - 0.5) * 2.0 * speed, rng.u01() * vup]
            a = [rng.u01() * 2.0 - 1.0 for _ in range(3)]
            ln = math.sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2])
            if ln < 1e-6:
                a, ln = [0.0, 0.0, 1.0], 1.0
            w = spin * (0.5 + rng.u01())
            f = win[0] + rng.u01() * (win[1] - win[0])
            out.append({"mesh": meshes[i % len(meshes)], "p0": p0, "v0": v0, "axis": [x / ln for x in a],
                        "w": w, "scale": scale, "t_spawn": (f - f0) / fps,
                        "gravity": float(g.get("gravity", 9.81)), "restitution": float(g.get("restitution", 0.5)),
                        "friction": float(g.get("friction", 0.7)), "ground_z": float(g.get("ground_z", 0.0)),
                        "rest_height": scale * float(g.get("mesh_half_height", 1.0)),
                        "min_speed": float(g.get("min_speed", 0.05)), "max_bounces": int(g.get("max_bounces", 8))})
    return out


def rigid_matrix(m: dict, t: float) -> np.ndarray:
    """Pose at t seconds after frame_start: hang until t_spawn, ballistic
    flight, bounces with restitution, per-bounce friction on horizontal and
    angular travel, rest."""
    travel, zr = 0.0, 0.0
    trel = t - m["t_spawn"]
    g = m["gravity"]
    if trel > 0.0:
        z = max(m["p0"][2] - m["ground_z"] - m["rest_height"], 0.0)
        vz, tt, fac = m["v0"][2], trel, 1.0
        tau = (vz + math.sqrt(vz * vz + 2.0 * g * z)) / g
        k = 0
        while True:
            if tt <= tau:
                zr = z + vz * tt - 0.5 * g * tt * tt
                travel += fac * tt
                break
            travel += fac * tau
            tt -= tau
            vimp = g * tau - vz
            vz = m["restitution"] * vimp
            z = 0.0
            fac = fac * m["friction"]
            k += 1
            tau = 2.0 * vz / g
            if k > m["max_bounces"] or vz < m["min_speed"]:
                zr = 0.0
                break
        zr = max(zr, 0.0)
    else:
        zr = m["p0"][2] - m["ground_z"] - m["rest_height"]
    th = m["w"] * travel
    c, s = math.cos(th), math.sin(th)
    oc = 1.0 - c
    x, y, z = m["axis"]
    R = np.array([[c + x * x * oc, x * y * oc - z * s, x * z * oc + y * s],
                  [y * x * oc + z * s, c + y * y * oc, y * z * oc - x * s],
                  [z * x * oc - y * s, z * y * oc + x * s, c + z * z * oc]], np.float64)
    M = np.eye(4)
    M[:3, :3] = R * m["scale"]
    M[0, 3] = m["p0"][0] + m["v0"][0] * travel
    M[1, 3] = m["p0"][1] + m["v0"][1] * travel
    M[2, 3] = m["ground_z"] + m["rest_height"] + zr
    return M


def frame_constants(scene: dict, frame: int, width: int | None = None, height: int | None = None) -> dict:
    """Camera (16 floats), lights (n x 12), materials (n x 12), world (3)."""
    r = scene["render"]
    W = width or (r["resolution_x"] * r["resolution_percentage"]) // 100
    H = height or (r["resolution_y"] * r["resolution_percentage"]) // 100
    cam_obj = scene["objects"][scene["camera"]]
    M = object_matrix(cam_obj, frame)
    axes = [M[:3, a] / np.linalg.norm(M[:3, a]) for a in range(3)]
    c = cam_obj["camera"]
    fit = c.get("sensor_fit", "AUTO")
    sensor = c["sensor_height"] if fit == "VERTICAL" else c["sensor_width"]
    horiz = fit == "HORIZONTAL" or (fit == "AUTO" and W >= H)
    if horiz:
        hw = 0.5 * sensor / c["lens"]
        hh = hw * H / W
    else:
        hh = 0.5 * sensor / c["lens"]
        hw = hh * W / H
    cam = np.array([*M[:3, 3], *axes[0], *axes[1], *axes[2], hw, hh, c["clip_start"], c["clip_end"]], np.float32)
    lights = []
    for o in scene["objects"]:
        if o["type"] != "LIGHT":
            continue
        Lm = object_matrix(o, frame)
        li = o["light"]
        dz = -Lm[:3, 2] / np.linalg.norm(Lm[:3, 2])
        k = li["energy"] / (4.0 * math.pi) if li["type"] == "POINT" else li["energy"]
        lights.append([0.0 if li["type"] == "POINT" else 1.0, *Lm[:3, 3], *dz,
                       li.get("radius", 0.0) if li["type"] == "POINT" else 0.0, *(k * np.array(li["color"])), 0.0])
    mats = []
    for m in scene["materials"] + [{"base_color": [0.8] * 3, "metallic": 0.0, "specular": 0.5, "roughness": 0.5,
                                    "ior": 1.45, "emission": [0, 0, 0], "emission_strength": 1.0}]:
        mats.append([*m["base_color"], m["metallic"], m["specular"], m["roughness"], m["ior"],
                     *(np.array(m["emission"]) * m.get("emission_strength", 1.0)),
                     1.0 if m.get("model") == "lambert" else 0.0, 0.0])
    w = scene["world"]
    return {"camera": cam, "lights": np.array(lights, np.float32).reshape(-1, 12),
            "materials": np.array(mats, np.float32), "world": np.array(w["color"], np.float64) * w["strength"],
            "W": W, "H": H}


def load_scene(path: str) -> dict:
    with open(path) as f:
        return json.load(f)


# ------------------------------------------------------ stdout protocol ----
_TIME_RE = re.compile(r"Time: (?P<total_time>\d+:\d+\.\d+) \(Saving: (?P<saving_time>\d+:\d+\.\d+)\)")


class StdoutError(ValueError):
    pass


def parse_blender_human_time(s: str) -> float:
    """utilities.rs:51-84: 'mm:ss.ff' -> seconds (exactly two ':'-separated parts)."""
    parts = s.split(":")
    if len(parts) != 2:
        raise StdoutError(f"Invalid human time, not in 00:00.00 format: {s}")
    try:
        return float(parts[0]) * 60.0 + float(parts[1])
    except ValueError as e:
        raise StdoutError(str(e)) from e


def f64_to_utc(ts: float) -> float:
    """utilities.rs:86-96: whole seconds (as i64 truncation) + ns truncated."""
    whole = int(ts)  # `timestamp as i64` truncates toward zero
    sub = ts - math.floor(ts)
    ns = int(sub * 1e9)
    return whole + ns / 1e9


def parse_blender_stdout(stdout: str) -> dict:
    """utilities.rs:105-203. Returns the five PartialRenderStatistics fields."""
    lines = stdout.splitlines()
    i = 0
    while i < len(lines) and not lines[i].startswith("Saved: '"):
        i += 1
    saving = None
    raw = None
    for line in lines[i:]:
        if line.startswith(" Time:"):
            m = _TIME_RE.search(line)
            if not m:
                continue
            if saving is not None:
                raise StdoutError('Invalid Blender output: " Time... (Saving ...)" line appears more than once.')
            saving = parse_blender_human_time(m.group("saving_time"))
        elif line.startswith("RESULTS="):
            raw = json.loads(line[len("RESULTS="):])
    if raw is None or saving is None:
        raise StdoutError("Invalid output, missing data")
    fin = raw["project_finished_rendering_at"] - saving
    return {"loaded_at": f64_to_utc(raw["project_loaded_at"]),
            "started_rendering_at": f64_to_utc(raw["project_started_rendering_at"]),
            "finished_rendering_at": f64_to_utc(fin),
            "file_saving_started_at": f64_to_utc(fin),
            "file_saving_finished_at": f64_to_utc(raw["project_finished_rendering_at"])}


# --------------------------------------------------------------- OCIO LUTs --
# Readers of OpenColorIO's Sony Pictures Imageworks LUT formats, restated from
# the formats' published layout (OCIO FileFormatSpi3D / FileFormatSpi1D), for
# the Filmic view transform of Blender 3.6's colour-management config
# (csrc/view.hpp). Independent of the product's C++ parser: the parity tests
# feed these arrays to the oracle and the files to the product.

def parse_spi3d(path: str) -> np.ndarray:
    """.spi3d: 'SPILUT 1.0', '3 3', 'N N N', then 'i j k r g b' per entry (i =
    red index). Returns the cube as (N, N, N, 3) float32 indexed [i, j, k]."""
    with open(path) as fh:
        lines = fh.read().splitlines()
    if not lines or not lines[0].startswith("SPILUT"):
        raise ValueError(f"{path}: not an SPILUT file")
    n = [int(x) for x in lines[2].split()]
    if len(n) != 3 or len(set(n)) != 1:
        raise ValueError(f"{path}: bad cube size")
    n = n[0]
    cube = np.zeros((n, n, n, 3), np.float32)
    seen = np.zeros((n, n, n), bool)
    for ln in lines[3:]:
        f = ln.split()
        if not f:
            continue
        i, j, k = (int(x) for x in f[:3])
        cube[i, j, k] = [np.float32(float(x)) for x in f[3:6]]
        seen[i, j, k] = True
    if not seen.all():
        raise ValueError(f"{path}: missing cube entries")
    return cube


def parse_spi1d(path: str) -> dict:
    """.spi1d: 'Version 1', 'From lo hi', 'Length N', 'Components C', '{',
    N rows of C values, '}'. Returns {"lut1": (N, C) float32, "lo1", "hi1"}."""
    with open(path) as fh:
        toks_lines = fh.read().splitlines()
    lo, hi, n, comps, body = 0.0, 1.0, None, None, []
    it = iter(toks_lines)
    for ln in it:
        f = ln.split()
        if not f or f[0] == "Version":
            continue
        if f[0] == "From":
            lo, hi = float(f[1]), float(f[2])
        elif f[0] == "Length":
            n = int(f[1])
        elif f[0] == "Components":
            comps = int(f[1])
        elif f[0] == "{":
            for ln2 in it:
                for t in ln2.split():
                    if t == "}":
                        break
                    body.append(np.float32(float(t)))
                else:
                    continue
                break
            break
    lut = np.array(body, np.float32).reshape(n, comps)
    return {"lut1": lut, "lo1": np.float32(lo), "hi1": np.float32(hi)}


FILMIC_LUT_FILES = ("filmic_desat65cube.spi3d", "filmic_to_0-70_1-03.spi1d")


def load_filmic_luts(directory: str) -> dict:
    """The two Filmic LUTs under a Blender colour-management directory (or its luts/)."""
    import os
    found = []
    for name in FILMIC_LUT_FILES:
        for sub in ("luts", ""):
            p = os.path.join(directory, sub, name)
            if os.path.isfile(p):
                found.append(p)
                break
        else:
            raise FileNotFoundError(name)
    d = parse_spi1d(found[1])
    d["cube"] = parse_spi3d(found[0])
    return d


def write_synthetic_filmic_luts(directory: str, n3: int = 17, n1: int = 1024, seed: int = 7,
                                lo: float = -0.125, hi: float = 1.125) -> None:
    """Synthetic LUT files in the two formats, shaped like Filmic's (a
    desaturating cube into [0, 0.66], an S-shaped display curve), for tests
    only: Blender's own LUT files are not in this image."""
    import os
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(directory, "luts"), exist_ok=True)
    g = np.linspace(0.0, 1.0, n3)
    with open(os.path.join(directory, "luts", FILMIC_LUT_FILES[0]), "w") as fh:
        fh.write(f"SPILUT 1.0\n3 3\n{n3} {n3} {n3}\n")
        for i in range(n3):
            for j in range(n3):
                for k in range(n3):
                    rgb = np.array([g[i], g[j], g[k]])
                    y = rgb.mean()
                    v = 0.66 * (0.8 * rgb + 0.2 * y) + rng.normal(0, 0.004, 3)
                    fh.write(f"{i} {j} {k} {v[0]:.6f} {v[1]:.6f} {v[2]:.6f}\n")
    x = np.linspace(lo, hi, n1)
    curve = 1.0 / (1.0 + np.exp(-8.0 * (x - 0.5)))
    with open(os.path.join(directory, "luts", FILMIC_LUT_FILES[1]), "w") as fh:
        fh.write(f"Version 1\nFrom {lo} {hi}\nLength {n1}\nComponents 1\n{{\n")
        for v in curve:
            fh.write(f"  {v:.8f}\n")
        fh.write("}\n")


# ------------------------------------------------------- worker accounting --
def worker_performance(trace: dict) -> dict:
    """WorkerPerformance::from_worker_trace (/root/reference/shared/src/results/
    performance.rs:47-143) over a WorkerTrace dict (traces.WorkerTrace.to_dict):
    the per-frame loading / rendering / saving durations and the idle time
    between frames. Every `signed_duration_since(..).to_std()` of the reference
    fails on a negative duration; the same checks raise ValueError here with
    the reference's messages."""
    def dur(a, b, msg):
        d = a - b
        if d < 0:
            raise ValueError(msg)
        return d
    frames = [f["details"] for f in trace["frame_render_traces"]]
    total = dur(trace["job_finish_time"], trace["job_start_time"], "Could not calculate total job duration.")
    load = rend = save = idle = 0.0
    n = len(frames)
    for i, f in enumerate(frames):
        load += dur(f["finished_loading_at"], f["started_process_at"], "Invalid file reading duration.")
        rend += dur(f["finished_rendering_at"], f["started_rendering_at"], "Invalid rendering duration.")
        save += dur(f["file_saving_finished_at"], f["file_saving_started_at"], "Invalid file saving duration.")
        if i == 0:
            idle += dur(f["started_process_at"], trace["job_start_time"],
                        "Failed to calculate idle time before first frame.")
        elif i == n - 1:
            idle += dur(trace["job_finish_time"], f["exited_process_at"],
                        "Failed to calculate idle time after last frame.")
        else:
            idle += dur(f["started_process_at"], frames[i - 1]["exited_process_at"], "Invalid idle duration.")
    return {"total_frames_rendered": n, "total_time": total, "total_blend_file_reading_time": load,
            "total_rendering_time": rend, "total_image_saving_time": save, "total_idle_time": idle}
