#!/usr/bin/env python3
"""Whole-job frames/s of the per-frame render step on 1..N MI355X.

One step = one frame of the 04_very-simple job through BackendRunner.render_frame
(the reference's BlenderJobRunner::render_frame semantics, /root/reference/worker/
src/rendering/runner/mod.rs:72-203): animation eval, LBVH rebuild, wavefront path
tracing at the scene's 1920x1080 / 128 spp, tonemap, JPEG q90 encode and file
write. Frames are independent; each rank (one per GPU) renders its own frames
(static frame partition, no data-path collective) => weak scaling.

Timed region: barrier + device sync on both sides, max over ranks (the only
cross-rank exchange, over gloo: frames are independent, there is no data-path
collective and no RCCL). Per-kernel device times come from HIP events recorded
by the library on its own stream around every launch (RR_FLAG_PROFILE_KERNELS):
during the timed steps, or — when consecutive k_tiles frames overlap on the
device in the timed steps — over frames rendered one at a time right after it
(roofline.launch_timing says which). Traversal counts for the algorithmic-byte model
come from one extra counting frame after the timed region
(RR_FLAG_COUNT_TRAVERSAL).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1 without a launcher: bench.py starts N worker processes itself, one per
  GPU (HIP_VISIBLE_DEVICES=i, before any GPU call in this process), as the
  reference starts one worker per node (scripts/arnes/
  queue-batch_04vs_14400f-10w_dynamic.sh:49,59); under torchrun (RANK /
  WORLD_SIZE set) each process is one rank on GPU LOCAL_RANK.
  --dry-run: the launch, frame partition and reduction without rendering (CPU
  containers; the line carries value null).
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "diploma_thesis-distributed_rendering_of_cgi_using_a_render_cluster_amd"

METRIC = "job frames/sec at 1/2/4/8 MI355X (04_very-simple); Mrays/s per GPU"
JOB = os.path.join(ROOT, "jobs", "04_very-simple_demo_10f-1w.toml")
# --workload: the default is BASELINE.json's metric config (configs[1], 04vs on
# one MI355X); the others are the C4/C5 configs, reported in DESIGN.md/profiles.
WORKLOADS = {
    # 40 steps (4 passes over the 10-frame job): at ~3 ms a frame the fill and
    # drain of the two-frame pipeline would otherwise weigh ~15 % of a 10-step run
    "04vs": {"job": JOB, "metric": METRIC, "steps": 40, "warmup": 4, "device_warmup_s": 0.3,
             "data": "synthetic: 04_very-simple stand-in scene (01_simple-animation content; the 04 .blend is "
                     "missing from the reference), frames of the 04vs demo job, JPEG q90 written per frame",
             "workload": "04vs-standin, 1 frame per step: 1920x1080, 128 spp, max 12 bounces, "
                         "LBVH rebuild + path trace (k_tiles: every sample of an 8x8 tile in one wave) + "
                         "JPEG q90 encode/write"},
    "01": {"job": os.path.join(ROOT, "jobs", "01_simple-animation_600f-8w_dynamic.toml"),
           "metric": "job frames/sec at 1/2/4/8 MI355X (01_simple-animation)", "steps": 40, "warmup": 4,
           "device_warmup_s": 0.3,
           "data": "01_simple-animation.rrscene exported from the reference's .blend (Filmic rendered as "
                   "Standard: no OCIO LUTs in the image), frames of the 600-frame job, JPEG q90 written per frame",
           "workload": "01-simple-animation, 1 frame per step: 1920x1080, 128 spp, max 12 bounces, "
                       "LBVH rebuild + path trace (k_tiles) + JPEG q90 encode/write"},
    "02": {"job": os.path.join(ROOT, "jobs", "02_physics-standin_170f-5w_naive-fine.toml"),
           "metric": "job frames/sec at 1/2/4/8 MI355X (02_physics stand-in)", "steps": 10, "warmup": 2,
           "data": "synthetic: 02_physics stand-in (2,000 closed-form rigid bodies, 92,002 triangles; the 02 .blend "
                   "is missing from the reference), PNG written per frame",
           "workload": "02-physics-standin, 1 frame per step: 1920x1080, 64 spp, max 8 bounces, full hierarchy "
                       "rebuild every frame + wavefront path trace + PNG encode/write"},
    "03": {"job": os.path.join(ROOT, "jobs", "03_physics-2-standin_480f-8w_dynamic.toml"),
           "metric": "job frames/sec at 1/2/4/8 MI355X (03_physics-2 stand-in)", "steps": 10, "warmup": 2,
           "data": "synthetic: 03_physics-2 stand-in (3,000 closed-form rigid bodies, 412,002 triangles), JPEG q90",
           "workload": "03-physics-2-standin, 1 frame per step: 1920x1080, 64 spp, max 8 bounces, full hierarchy "
                       "rebuild every frame + wavefront path trace + JPEG q90 encode/write"},
    "c5": {"job": os.path.join(ROOT, "jobs", "c5_synthetic-10m_240f-8w_dynamic.toml"),
           "metric": "job frames/sec at 1/2/4/8 MI355X (C5 synthetic 10M triangles, 4K, 1024 spp)",
           "steps": 2, "warmup": 1,
           "data": "synthetic: 512 displaced icospheres x 20,480 triangles + ground (10,485,762 triangles), "
                   "per-instance rigid motion, JPEG q90",
           "workload": "c5-synthetic-10m, 1 frame per step: 3840x2160, 1024 spp, max 4 bounces, full hierarchy "
                       "rebuild every frame + wavefront path trace + JPEG q90 encode/write"},
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
MALL_BYTES = 256 << 20  # Infinity Cache (MALL) capacity
# Vector-issue peak: a wave64 VALU instruction issues over 2 cycles on a SIMD-32
# (MI355X_MICROARCH.md, wave scheduling), 4 SIMDs per CU, 256 CUs.
VALU_ISSUE_PER_CLK_PER_SIMD = 0.5
SIMDS = 256 * 4
PEAK_CLOCK_GHZ = 2.4  # MI355X peak engine clock (MI355X_MICROARCH.md)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default: 10 (2 for c5)")
    ap.add_argument("--warmup", type=int, default=None, help="default: 2 (1 for c5)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="04vs")
    ap.add_argument("--spp", type=int, default=0, help="override the scene's samples (0 = scene)")
    ap.add_argument("--device-warmup-s", type=float, default=None,
                    help="frames of the job rendered for this long before the warmup steps (GPU clock ramp; "
                         "default 0.3 s for the k_tiles workloads 04vs / 01, 0 otherwise)")
    ap.add_argument("--no-profile", action="store_true", help="time without per-kernel HIP events")
    ap.add_argument("--serial", action="store_true",
                    help="one rr_render_frame per step (no overlap of frame N's encode with N+1's render)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc-summary", default=None,
                    help="PMC traffic summary for roofline.traffic (tools/pmc_summary.py; default the newest "
                         "profiles/r<N>_pmc.json for 04vs, profiles/r<N>_pmc_<workload>.json otherwise)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch, partition and reduce without rendering (no GPU needed; value is null)")
    a = ap.parse_args()
    wl = WORKLOADS[a.workload]
    if a.steps is None:
        a.steps = wl["steps"]
    if a.warmup is None:
        a.warmup = wl["warmup"]
    return a


def algorithmic_bytes(cls: str, stats, scene_bytes: float, split: bool) -> tuple[float, float]:
    """Algorithmic HBM bytes of one kernel class over a frame.

    Returns (compulsory, survey): `compulsory` is the stream every launch must
    move through HBM (radiance records, queue entries, hit records, film) plus
    the scene's BVH and triangles read once; `survey` is SURVEY.md §8(d)'s
    literal figure, which prices every counted node visit (64 B) and triangle
    test (48 B) as HBM traffic even when the scene is cache/LDS resident.
    `split`: the large-scene path (separate trace and shade kernels, 8 B hit
    records; the shading stream is class "shade")."""
    npaths = stats.camera_rays
    ext = stats.extension_rays
    sh = stats.shadow_rays
    c0, s0 = stats.primary_continued, stats.primary_shadow
    ce, se = ext - c0, sh - s0
    node, tri = 64.0, 48.0
    trav = None
    if cls == "primary":
        if split:
            stream = npaths * 8.0
        else:
            stream = npaths * 16.0 + c0 * 48.0 + s0 * 48.0
        trav = node * stats.trav_nodes[0] + tri * stats.trav_tris[0]
    elif cls == "extend":
        if split:
            stream = ext * (32.0 + 8.0)
        else:
            stream = ext * (48.0 + 32.0) + ce * 48.0 + se * 48.0
        trav = node * stats.trav_nodes[1] + tri * stats.trav_tris[1]
    elif cls == "shadow":
        stream = sh * (48.0 + 32.0)
        trav = node * stats.trav_nodes[2] + tri * stats.trav_tris[2]
    elif cls == "shade":
        stream = (npaths * (8.0 + 16.0) + ext * (48.0 + 8.0 + 32.0) + (c0 + ce) * 48.0 + (s0 + se) * 48.0
                  + tri * (npaths + ext))
        return stream, stream
    elif cls == "tiles":
        # k_tiles (LDS-resident scenes): no per-path stream at all; HBM sees the
        # film (16 B) and RGBA8 (4 B) write per pixel. SURVEY 8(d)'s figure
        # prices every ray (48 B), node visit, triangle test, path segment
        # (128 B) and sample (32 B) as if they went through memory.
        npix = stats.width * stats.height
        stream = npix * (16.0 + 4.0)
        trav = sum(node * stats.trav_nodes[k] + tri * stats.trav_tris[k] for k in range(3))
        rays_all = npaths + ext + sh
        survey = stream + trav + 48.0 * rays_all + 128.0 * (npaths + ext) + 32.0 * npaths
        return stream + scene_bytes, survey
    elif cls == "accumulate":
        npix = stats.width * stats.height
        return (npix * (stats.spp * 16.0 + 32.0 * max(stats.chunks - 1, 0) + 16.0 + 4.0),) * 2
    else:
        return 0.0, 0.0
    return stream + min(trav, scene_bytes), stream + trav


# kernel names per class: the split path (large scenes) and k_tiles (LDS-resident scenes)
KERNEL_OF_CLASS = {"build": [], "primary": ["k_trace_primary", "k_trace_primary_packet"],
                   "extend": ["k_trace_extend"], "shadow": ["k_shadow_refill"],
                   "shade": ["k_shade_extend", "k_shade_primary"], "accumulate": ["k_accumulate"],
                   "tiles": ["k_tiles"]}


def pmc_kernels(path: str | None) -> dict:
    """Per-kernel entries of a committed rocprofv3 PMC summary
    (tools/pmc_summary.py traffic), {} when absent."""
    if not path or not os.path.exists(path):
        return {}
    with open(path) as fh:
        return json.load(fh)["kernels"]


# kernels reported one by one in kernels_pmc (BASELINE north star: achieved HBM
# GB/s of the traversal and shading kernels, occupancy), in frame order
PMC_KERNELS = ("k_trace_primary_packet", "k_trace_primary", "k_shade_primary", "k_shadow_refill", "k_trace_extend",
               "k_shade_extend", "k_accumulate", "k_tiles")


def occupancy_figures(e: dict, clock_ghz: float = PEAK_CLOCK_GHZ) -> dict:
    """Wave life and occupancy of one kernel from its PMC pass. The span is the
    kernel's own mean dispatch time in that pass (pmc_pass_avg_ms) x the engine
    clock (`clock_ghz`: the kernel clock the library measured, else the 2.4 GHz
    peak): wave_life_frac = a wave's mean lifetime (4 x SQ_WAVE_CYCLES / SQ_WAVES,
    quad-cycle units) over that span (how full the persistent grid stays),
    occupancy_waves_per_simd = 4 x SQ_WAVE_CYCLES / span / 1024 SIMDs.
    GRBM_GUI_ACTIVE / 8, the span used until round 5, counts every cycle the GPU
    was busy while the kernel's dispatches ran, other kernels' and copies'
    included; for k_tiles in the pipelined pass it was 3.4x the dispatch (VERDICT
    r5 Weak 4), so it is kept only as the ratio grbm_span_over_dispatch."""
    gr, wc, nw, ms = e.get("GRBM_GUI_ACTIVE"), e.get("SQ_WAVE_CYCLES"), e.get("SQ_WAVES"), e.get("pmc_pass_avg_ms")
    if not (wc and nw and ms):
        return {}
    span = ms * 1e-3 * clock_ghz * 1e9
    row = {"wave_life_frac": round(4.0 * wc / nw / span, 3),
           "occupancy_waves_per_simd": round(4.0 * wc / span / SIMDS, 2),
           "occupancy_span": f"PMC-pass dispatch time x {clock_ghz:g} GHz"}
    if gr:
        row["grbm_span_over_dispatch"] = round(gr / 8.0 / span, 2)
    return row


def pmc_kernel_block(ks: dict, src: str | None, clock_ghz: float = PEAK_CLOCK_GHZ) -> dict:
    """Per-kernel PMC figures of the path's traversal and shading kernels (the
    timed instantiation, not the counting one): HBM GB/s = PMC bytes per launch
    (FETCH_SIZE x fetch_scale + WRITE_SIZE) over that pass's own mean dispatch
    time, its fraction of the 8 TB/s peak, L2 hit rate, wait_frac = SQ_WAIT_ANY /
    SQ_WAVE_CYCLES, valu_lane_util (active lanes per VALU instruction), wave
    life and occupancy over the same dispatch time (occupancy_figures)."""
    out = {}
    for name in PMC_KERNELS:
        for k, e in ks.items():
            if k.split("<")[0] != name:
                continue
            targs = k.split("<")[1].rstrip(">").split(",") if "<" in k else []
            if targs and targs[0] != "false":
                continue  # the counting instantiation
            ms = e.get("pmc_pass_avg_ms")
            row = {"launches": e.get("launches")}
            if ms:
                gbs = e["traffic_bytes"] / (ms * 1e-3) / 1e9
                row.update({"pmc_pass_avg_ms": round(ms, 4), "hbm_gbs": round(gbs, 1),
                            "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)})
            row["traffic_bytes"] = round(e["traffic_bytes"])
            for f in ("l2_hit_rate", "wait_frac", "valu_lane_util"):
                if f in e:
                    row[f] = round(e[f], 3)
            row.update(occupancy_figures(e, clock_ghz))
            out[k] = row
    return {"source": src, "timing": "each kernel's own mean dispatch time in the PMC pass (profiler-serialised)",
            "kernels": out} if out else {}


def pmc_entry(ks: dict, cls: str, variant: str | None = None):
    """(name, entry) of the class's timed kernel (not the counting
    instantiation) in a PMC summary: `variant` = the template arguments after
    kCount (k_tiles: "true" whole-tile units, "false" sample-group slices)."""
    for name in KERNEL_OF_CLASS.get(cls, []):
        for k, v in ks.items():
            if k.split("<")[0] != name:
                continue
            targs = k.split("<")[1].rstrip(">").split(",") if "<" in k else []
            if targs and targs[0] != "false":
                continue  # the counting instantiation
            if variant is not None and (len(targs) < 2 or targs[1] != variant):
                continue
            return k, v
    return None, None


def frame_partition(frames, step: int, rank: int, world: int):
    """Frame a rank renders at a step: static round-robin over the job's frame set
    (frames are independent, so ranks never exchange data)."""
    return frames[(step * world + rank) % len(frames)]


def reduce_max_seconds(elapsed: float, dist=None) -> float:
    """Max of the per-rank timed-region wall time (the job ends with its slowest
    rank), over the gloo group on host tensors."""
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def newest_profile(name_fmt: str):
    """profiles/<name_fmt % round> of the newest round that has it (r9 .. r1)."""
    for r in range(9, 0, -1):
        p = os.path.join(ROOT, "profiles", name_fmt % f"r{r}")
        if os.path.exists(p):
            return p
    return None


def host_cpu():
    """(cores usable by this process, nproc of the machine, CPU model)."""
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return usable, os.cpu_count() or 1, model


def _read_sysfs(path: str):
    try:
        with open(path) as fh:
            return fh.read().strip()
    except OSError:
        return None


def parse_cpulist(s: str | None) -> set:
    """sysfs cpulist ("0-3,8,10-11") -> set of CPU ids."""
    out = set()
    for part in (s or "").split(","):
        part = part.strip()
        if not part:
            continue
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


def gpu_numa_nodes(sysfs: str = "/sys") -> list:
    """NUMA node of every GPU in HIP's enumeration order — the GPU nodes of the
    KFD topology in node order — read from sysfs without touching a GPU:
    the node's PCI address (properties domain / location_id = bus << 8 |
    device << 3 | function) -> /sys/bus/pci/devices/<bdf>/numa_node. -1 where
    unknown; [] without a KFD topology (CPU containers)."""
    base = os.path.join(sysfs, "class/kfd/kfd/topology/nodes")
    try:
        ids = sorted(int(x) for x in os.listdir(base) if x.isdigit())
    except OSError:
        return []
    out = []
    for i in ids:
        props = _read_sysfs(os.path.join(base, str(i), "properties")) or ""
        kv = dict(ln.split()[:2] for ln in props.splitlines() if len(ln.split()) >= 2)
        if int(kv.get("simd_count", "0")) <= 0:
            continue  # a CPU node
        loc, dom = int(kv.get("location_id", "0")), int(kv.get("domain", "0"))
        bdf = f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}"
        node = _read_sysfs(os.path.join(sysfs, "bus/pci/devices", bdf, "numa_node"))
        out.append(int(node) if node not in (None, "") else -1)
    return out


def gpu_placement(devices: list, allowed: set, numa: list, node_cpus) -> list:
    """Host CPUs per rank (rank r drives GPU devices[r]): the CPUs of its GPU's
    NUMA node that this process may use, split into disjoint contiguous
    shares among the ranks whose GPUs sit on that node; ranks whose GPU's
    node is unknown (or has none of the allowed CPUs) share what is left of
    `allowed` the same way. One worker pinned per GPU as the reference pins
    one per node slot (scripts/arnes/queue-batch_04vs_14400f-10w_dynamic.sh:
    6-10,59). node_cpus(n) -> set of CPU ids of NUMA node n."""
    groups: dict = {}
    for r, d in enumerate(devices):
        n = numa[d] if 0 <= d < len(numa) else -1
        if n < 0 or not (node_cpus(n) & allowed):
            n = None
        groups.setdefault(n, []).append(r)
    plan: list = [set() for _ in devices]
    used = set()
    for n in sorted((k for k in groups if k is not None)):
        pool = sorted(node_cpus(n) & allowed)
        used.update(pool)
        _split(pool, groups[n], plan)
    if None in groups:
        rest = sorted(allowed - used) or sorted(allowed)
        _split(rest, groups[None], plan)
    return plan


def _split(pool: list, ranks: list, plan: list):
    k = len(ranks)
    for j, r in enumerate(ranks):
        share = pool[j * len(pool) // k:(j + 1) * len(pool) // k]
        plan[r] = set(share) if share else {pool[j % len(pool)]}


def rank_placement(local_rank: int, devices: list) -> dict:
    """This rank's CPU set and GPU NUMA node (computed identically by every
    local rank, so the sets are disjoint)."""
    numa = gpu_numa_nodes()
    allowed = set(os.sched_getaffinity(0))
    plan = gpu_placement(devices, allowed, numa,
                         lambda n: parse_cpulist(_read_sysfs(f"/sys/devices/system/node/node{n}/cpulist")))
    d = devices[local_rank]
    return {"device": d, "numa_node": numa[d] if 0 <= d < len(numa) else -1, "cpus": sorted(plan[local_rank])}


def pin_rank(place: dict):
    """Pins this process (before any GPU call) to its CPU share and caps the
    host threads of the oracle / OpenMP to it; librr's encoders size their
    pools from the affinity mask (image_io.cpp encoder_threads)."""
    os.sched_setaffinity(0, place["cpus"])
    cap = len(place["cpus"])
    omp = int(os.environ.get("OMP_NUM_THREADS") or cap)
    os.environ["OMP_NUM_THREADS"] = str(max(1, min(omp, cap)))


def cpuset_str(cpus) -> str:
    """[0, 1, 2, 5] -> "0-2,5"."""
    cpus, out = sorted(cpus), []
    i = 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


def physical_devices(n: int) -> list:
    """GPU indices (HIP's enumeration of the whole machine) of local ranks 0..n-1:
    the parent's HIP_VISIBLE_DEVICES list when set, else 0..n-1."""
    visible = os.environ.get("HIP_VISIBLE_DEVICES")
    devs = visible.split(",") if visible else [str(i) for i in range(n)]
    return [int(x) if x.strip().isdigit() else i for i, x in enumerate(devs[:n])]


def spawn_ranks(args) -> int:
    """--gpus N with no launcher: N child processes of this script, rank i on
    GPU i (HIP_VISIBLE_DEVICES, mapped through the parent's own list), each
    pinned to its GPU's NUMA node share (gpu_placement), gloo rendezvous on
    127.0.0.1. Started before this process touches a GPU; the children's
    rank 0 prints the line. Returns the worst exit code."""
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    visible = os.environ.get("HIP_VISIBLE_DEVICES")
    devs = visible.split(",") if visible else [str(i) for i in range(args.gpus)]
    if len(devs) < args.gpus:
        print(f"bench.py: --gpus {args.gpus} but HIP_VISIBLE_DEVICES lists {len(devs)}", file=sys.stderr)
        return 2
    phys = physical_devices(args.gpus)
    procs = []
    for r in range(args.gpus):
        place = rank_placement(r, phys)
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HIP_VISIBLE_DEVICES=devs[r], RR_BENCH_DEVICE="0",
                   HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
                   RR_BENCH_PLACEMENT=json.dumps(place))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    return max(abs(p.wait()) for p in procs)


def cpu_baseline(oracle_mod, state, budget_s: float, label: str = "04vs-standin frame 1", spp_scale: float = 1.0,
                 threads: int | None = None):
    """Oracle (C restatement, OpenMP) on the host cores: bands of the same
    frame (4 rows, or more where each call's hierarchy build outweighs a 4-row
    band's render), taken in an order spread over the image, until the budget
    is spent or the frame is done; extrapolated to frames/s with ONE hierarchy
    build per frame (each band call rebuilds it; its build time,
    orc_last_build_seconds, is taken out of the band's time and counted once). Threads: OMP_NUM_THREADS
    when the environment sets it (the GPU box gives one GPU's job a 16-core
    share and sets it; nproc there counts the whole machine), else every core
    this process may run on. spp_scale: the frame's samples over the samples
    rendered (render time is linear in spp; the build is not)."""
    H = int(state.render_ints[1])
    usable, nproc, model = host_cpu()
    if threads is None:
        threads = int(os.environ.get("OMP_NUM_THREADS") or usable)
    done_rows, t_used, t_render, builds = 0, 0.0, 0.0, []
    band_h = 4

    def band(b, h):
        nonlocal done_rows, t_used, t_render
        t0 = time.perf_counter()
        oracle_mod.render_state(state, rows=(b, min(b + h, H)), threads=threads, film=False)
        dt = time.perf_counter() - t0
        tb = min(oracle_mod.last_build_seconds(), dt)
        builds.append(tb)
        t_used += dt
        t_render += dt - tb
        done_rows += min(b + h, H) - b
        return tb, dt - tb

    # the first 4-row band (the middle rows) measures the per-call hierarchy
    # build against the render; where the build dominates (C5: ~3.5 s a call),
    # later bands grow to about the build's cost in rows, so the budget renders
    # more rows. The later bands tile the other rows and are taken in an order
    # spread over the frame; the extrapolation uses them alone unless there are
    # none (then the middle band stands for the frame) or the frame gets done
    # whole.
    b0 = (H // 2) // 4 * 4
    tb0, tr0 = band(b0, 4)
    if tr0 > 0.0:
        band_h = 4 * max(1, min(16, int(round(tb0 / tr0))))
    first = (done_rows, t_render)
    bands = [b for b in range(0, H, band_h) if b + band_h <= b0 or b >= b0 + 4]
    order = [b for k in range(16) for b in bands[k::16]]
    for b in order:
        if t_used >= budget_s:
            break
        band(b, band_h)
    if done_rows < H and done_rows > first[0]:  # a sample: the spread bands only
        frac = (done_rows - first[0]) / H
        rendered = t_render - first[1]
    else:
        frac, rendered = done_rows / H, t_render
    t_build = sum(builds) / len(builds)
    t_frame = t_build + rendered / frac * spp_scale
    return {"value": 1.0 / t_frame, "unit": "frames/s", "cores": threads, "kind": "port",
            "host": {"nproc": nproc, "affinity_cores": usable, "cpu_model": model,
                     "omp_num_threads": os.environ.get("OMP_NUM_THREADS")},
            "sample": f"{done_rows} of {H} rows ({band_h}-row bands spread over the frame after a first 4-row band at "
                      f"row {b0} that sizes them and stands for the frame only when no other band fits the budget) "
                      f"of {label} "
                      f"at {int(state.render_ints[0])}x{H}, {int(state.render_ints[2])} spp, "
                      f"{t_used:.1f} s in {len(builds)} band calls; frame time = one hierarchy build "
                      f"({t_build:.3f} s) + the bands' render time extrapolated to the whole frame; "
                      f"render only (no encode)"
                      + (f"; rendered at {int(state.render_ints[2])} spp, render time scaled by {spp_scale:g}"
                         if spp_scale != 1.0 else "")}


# The reference master's frame-dispatch loops (master/src/cluster/strategies.rs):
# each pass tops the workers' queues up and then sleeps, so a worker receives at
# most `per_pass` frames per sleep period whatever its render speed.
DISPATCH = {"naive-fine": {"sleep_ms": 50, "source": "strategies.rs:20-64 (one frame to an empty queue, 50 ms sleep)"},
            "eager-naive-coarse": {"sleep_ms": 100,
                                   "source": "strategies.rs:70-146 (queue topped up to target_queue_size, 100 ms sleep)"},
            "dynamic": {"sleep_ms": 50,
                        "source": "strategies.rs:171-401 (queue topped up to target_queue_size, 50 ms sleep)"}}


def dispatch_ceiling(job_dict: dict, workers: int) -> dict:
    """Upper bound on the whole-job frames/s of BASELINE's metric (frames over
    the master trace's job_finish_time - job_start_time, master/src/cluster/
    mod.rs:590,666-668) set by the unchanged master's dispatch cadence alone
    (no message latency, instant renders): workers x frames per pass / sleep."""
    strat = job_dict.get("frame_distribution_strategy") or {}
    kind = strat.get("strategy_type", "naive-fine")
    d = DISPATCH.get(kind, DISPATCH["naive-fine"])
    per_pass = 1 if kind == "naive-fine" else int(strat.get("target_queue_size", 1))
    return {"value": round(workers * per_pass * 1000.0 / d["sleep_ms"], 1), "unit": "frames/s",
            "strategy": kind, "frames_per_pass_per_worker": per_pass, "sleep_ms": d["sleep_ms"], "workers": workers,
            "source": "/root/reference/master/src/cluster/" + d["source"],
            "note": "what the reference master can dispatch to this many workers; bench.py's value times the "
                    "worker's render loop with its queue kept full (no master in the loop), i.e. the renderer's "
                    "rate: under the unchanged master the job runs at most min(value, this ceiling)"}


def names_idx(cls: str, rr) -> int:
    return list(rr.native.KERNEL_CLASSES).index(cls)


def valu_peak_per_s() -> float:
    return VALU_ISSUE_PER_CLK_PER_SIMD * SIMDS * PEAK_CLOCK_GHZ * 1e9


def roofline_line(args, cls, cstats, kernel_ms, launches, names, steps, timed=None):
    """The dominant kernel class against the roofline that actually bounds it
    (DESIGN.md §6):
      * LDS-resident scenes (k_tiles, 04vs / 01): VALU issue. The scene lives
        in LDS; HBM sees only the film (hbm_frac) and the bound is vector-
        instruction issue: SQ_INSTS_VALU wave-instructions against 0.5 per
        clock per SIMD x 1024 SIMDs at the 2.4 GHz peak clock. Headline = the
        TIMED REGION: the launches the timed frames ran (whole-tile units for
        every frame that overlapped a pending one, sample-group slices for a
        frame alone; each kind priced by its own PMC count) over the timed
        region's wall time; avg_launch_ms = that wall time per launch (<=
        ms_per_step). The same launches timed alone by HIP events after the
        timed region are the secondary `solo` figure.
      * split path over a hierarchy that fits in L2 / MALL (02 / 03): bound by
        memory latency (L2 hits waited on), reported as l2_hit_rate and
        wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES beside the PMC HBM rate.
      * split path over a hierarchy far above MALL (C5): HBM, SURVEY §8(d)'s
        algorithmic bytes (64 B per node visit, 48 B per triangle test + the
        ray / hit stream); the PMC traffic beside it."""
    dom = names.index(cls)
    n = int(cstats.n_triangles)
    scene_bytes = 64.0 * max(n - 1, 1) + 48.0 * n
    split = launches[5] > 0
    bytes_frame, survey_frame = algorithmic_bytes(cls, cstats, scene_bytes, split)
    launches_frame = max(launches[dom] / max(steps, 1), 1)
    avg_ms = kernel_ms[dom] / max(launches[dom], 1)
    wl_key = "" if args.workload == "04vs" else f"_{args.workload}"
    pmc_path = args.pmc_summary or newest_profile("%s_pmc" + wl_key + ".json")
    ks = pmc_kernels(pmc_path)
    src = os.path.relpath(pmc_path, ROOT) if ks else None
    if cls == "tiles" and not split:
        _, e_sl = pmc_entry(ks, cls, "false")
        _, e_wh = pmc_entry(ks, cls, "true")
        if e_sl is None:  # a summary from before the whole-tile variant (k_tiles<false>)
            _, e_sl = pmc_entry(ks, cls)
        v_sl = e_sl.get("SQ_INSTS_VALU") if e_sl else None
        v_wh = e_wh.get("SQ_INSTS_VALU") if e_wh else None
        peak = valu_peak_per_s()
        out = {"kernel": cls, "bound": "valu", "unit": "G wave-instr/s", "peak": round(peak / 1e9, 1),
               "clock_ghz": PEAK_CLOCK_GHZ, "clock_source": "peak engine clock (MI355X_MICROARCH.md)",
               "valu_source": src, "launches_per_frame": launches_frame,
               "bytes_per_launch_algorithmic": round(bytes_frame / launches_frame)}
        if timed is not None:
            n_wh, n_sl, t_s = timed["whole"], timed["sliced"], timed["elapsed"]
            eff_ms = t_s / max(n_wh + n_sl, 1) * 1e3
            out["avg_launch_ms"] = round(eff_ms, 4)
            out["launch_timing"] = (f"timed region: {n_wh + n_sl} k_tiles launches ({n_wh} whole-tile, {n_sl} "
                                    f"sample-group sliced) over {t_s * 1e3:.2f} ms of wall time; consecutive "
                                    "frames overlap on the device, so this is the time per launch the timed "
                                    "frames sustained")
            if v_sl is not None and (v_wh is not None or n_wh == 0):
                valu = (n_wh * (v_wh or 0.0) + n_sl * v_sl) / max(n_wh + n_sl, 1)
                ach = valu / (eff_ms * 1e-3)
                out.update({"achieved": round(ach / 1e9, 1), "frac": round(ach / peak, 3),
                            "valu_per_launch": round(valu),
                            "valu_per_launch_whole": round(v_wh) if v_wh is not None else None,
                            "valu_per_launch_sliced": round(v_sl)})
            else:
                out.update({"achieved": None, "frac": None, "valu_per_launch": None,
                            "note_valu": "no PMC count for the timed launches' kernel variant"})
        if v_sl is not None:
            out["solo"] = {"avg_launch_ms": round(avg_ms, 4), "valu_per_launch": round(v_sl),
                           "achieved": round(v_sl / (avg_ms * 1e-3) / 1e9, 1),
                           "frac": round(v_sl / (avg_ms * 1e-3) / peak, 3),
                           "launch_timing": f"HIP events around each launch, {steps} frames rendered one at a "
                                            "time after the timed region (sample-group slices)"}
        kc = float(getattr(cstats, "kernel_clock_ghz", 0.0))
        if kc > 0 and out.get("achieved"):
            out["kernel_clock_ghz"] = round(kc, 3)
            out["issue_util_at_kernel_clock"] = round(out["achieved"] * 1e9 /
                                                      (VALU_ISSUE_PER_CLK_PER_SIMD * SIMDS * kc * 1e9), 3)
        # the counting launch (k_tiles<true, false>: a slower variant of the sliced
        # kernel) — its waves' mean life over the launch and the spread of their
        # starts and ends; a production launch's own unit log (DESIGN.md,
        # tools/tiles_fill_probe.py) shows a shorter tail
        out["wave_fill_solo"] = round(float(getattr(cstats, "kernel_wave_fill", 0.0)), 3)
        out["wave_entry_spread_solo"] = round(float(getattr(cstats, "kernel_entry_spread", 0.0)), 3)
        out["wave_exit_spread_solo"] = round(float(getattr(cstats, "kernel_exit_spread", 0.0)), 3)
        # the same occupancy from the PMC pass (sliced launches, dispatch-time span),
        # to set beside wave_fill_solo
        if e_sl is not None:
            occ = occupancy_figures(e_sl, kc if 1.0 < kc <= PEAK_CLOCK_GHZ * 1.05 else PEAK_CLOCK_GHZ)
            if occ:
                out["wave_life_pmc_sliced"] = occ["wave_life_frac"]
                out["occupancy_waves_per_simd_pmc_sliced"] = occ["occupancy_waves_per_simd"]
        lu = (e_wh or {}).get("valu_lane_util") if (timed and timed["whole"]) else (e_sl or {}).get("valu_lane_util")
        if lu is not None:  # active lanes per issued VALU instruction (PMC, SQ_THREAD_CYCLES_VALU)
            out["valu_lane_util"] = round(lu, 3)
            if out.get("frac") is not None:
                out["frac_lane_weighted"] = round(out["frac"] * lu, 3)
        t_ms = out.get("avg_launch_ms", avg_ms)
        comp = bytes_frame / launches_frame / (t_ms * 1e-3) / 1e9
        tr = e_wh if (e_wh and timed and timed["whole"]) else e_sl
        out.update({"hbm_compulsory_gbs": round(comp, 2), "hbm_frac": round(comp / HBM_PEAK_GBS, 4),
                    "hbm_survey_formula_gbs": round(survey_frame / launches_frame / (t_ms * 1e-3) / 1e9, 2),
                    "traffic": round(tr["traffic_bytes"]) if tr else None,
                    "traffic_gbs": round(tr["traffic_bytes"] / (t_ms * 1e-3) / 1e9, 1) if tr else None,
                    "traffic_source": src if tr else None,
                    "note": "k_tiles: scene in LDS, bound by vector-instruction issue (SQ_INSTS_VALU per launch / "
                            "launch time vs 0.5 wave-instr/clk/SIMD x 1024 SIMDs at 2.4 GHz); HBM sees only the "
                            "film + RGBA8 (hbm_frac)"})
        return out
    per_s = lambda b: b / launches_frame / (avg_ms * 1e-3) / 1e9  # noqa: E731
    _, e = pmc_entry(ks, cls)
    hbm = {"hbm_compulsory_gbs": round(per_s(bytes_frame), 2),
           "hbm_survey_formula_gbs": round(per_s(survey_frame), 2),
           "frac_survey_formula": round(per_s(survey_frame) / HBM_PEAK_GBS, 4),
           "traffic": round(e["traffic_bytes"]) if e else None,
           "traffic_gbs": round(e["traffic_bytes"] / (avg_ms * 1e-3) / 1e9, 1) if e else None,
           "traffic_source": src if e else None,
           "launch_timing": "HIP events around each launch on the library's stream over the timed region"}
    # PMC bytes per ray the class traced (counting frame's ray counts)
    cls_rays = {"primary": cstats.camera_rays_traced, "extend": cstats.extension_rays,
                "shadow": cstats.shadow_rays}.get(cls, 0)
    if e and cls_rays:
        hbm["traffic_bytes_per_ray"] = round(e["traffic_bytes"] * launches_frame / float(cls_rays), 1)
        hbm["fetch_scale"] = e.get("fetch_scale", 2.0)
    base = {"kernel": cls, "avg_launch_ms": round(avg_ms, 4), "launches_per_frame": launches_frame,
            "bytes_per_launch_algorithmic": round((survey_frame if split else bytes_frame) / launches_frame)}
    lat = {k: round(e[k], 3) for k in ("l2_hit_rate", "wait_frac", "valu_lane_util") if e and k in e}
    if e is None:  # no PMC summary for this workload: the survey formula, flagged
        ach = per_s(survey_frame)
        return {**base, "bound": "unmeasured", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), **hbm,
                "note": "no PMC summary: achieved = SURVEY 8(d) algorithmic bytes per launch / launch time, which "
                        "prices every node visit and triangle test as HBM traffic (an upper bound, not a measurement)"}
    # the bound from the counters: the PMC HBM rate against the peak, how much
    # of a wave's life it waits (SQ_WAIT_ANY / SQ_WAVE_CYCLES) and its vector
    # issue rate (SQ_INSTS_VALU per launch / launch time against 0.5 wave-
    # instructions per clock per SIMD at 2.4 GHz). At half the HBM peak or
    # more: hbm. Below it, waves waiting more than half their lives: bound by
    # the latency of the gathers (cache hits included), not bandwidth.
    # Otherwise the waves are issuing: valu (achieved / frac are then the issue
    # rate, the HBM rate stays beside it).
    ach = e["traffic_bytes"] / (avg_ms * 1e-3) / 1e9
    wf = e.get("wait_frac")
    v = e.get("SQ_INSTS_VALU")
    issue = v / (avg_ms * 1e-3) if v else None
    if ach >= 0.5 * HBM_PEAK_GBS:
        bound = "hbm"
    elif wf is not None and wf > 0.5:
        bound = "latency"
    else:
        bound = "valu" if issue else "hbm"
    resident = n * (64.0 + 48.0) < MALL_BYTES  # hierarchy + triangles fit in the 256 MB MALL
    out = {**base, "bound": bound, "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(ach / HBM_PEAK_GBS, 4), **lat, **hbm,
           "hbm_gbs_pmc": round(ach, 2), "hbm_frac_pmc": round(ach / HBM_PEAK_GBS, 4),
           "scene_fits_mall": resident,
           "note": "hbm_gbs_pmc = PMC HBM bytes per launch (FETCH_SIZE x fetch_scale, 1 for these 64 B gathers per "
                   "tools/fetch_probe.hip, + WRITE_SIZE; FETCH_SIZE counts Infinity-Cache hits, so an upper "
                   "bound on HBM reads) / the bench's launch time; bound = hbm at half the HBM peak or more, "
                   "else latency when waves wait more than half their lives (wait_frac), else valu (issue rate "
                   "SQ_INSTS_VALU / launch time vs 0.5 wave-instr/clk/SIMD x 1024 SIMDs at 2.4 GHz: achieved / "
                   "frac are then that rate); frac_survey_formula = SURVEY 8(d)'s algorithmic bytes (64 B per "
                   "node visit, 48 B per triangle test + ray/hit stream, every one priced as HBM traffic) over the "
                   "same time"}
    if issue:
        out["valu_per_launch"] = round(v)
        out["valu_issue_frac"] = round(issue / valu_peak_per_s(), 4)
    if bound == "valu":
        out.update({"achieved": round(issue / 1e9, 1), "peak": round(valu_peak_per_s() / 1e9, 1),
                    "unit": "G wave-instr/s", "frac": round(issue / valu_peak_per_s(), 4)})
    return out


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = int(os.environ.get("RR_BENCH_DEVICE", local))
    placement = None
    if world > 1:  # one worker pinned per GPU, before any GPU call (spawn_ranks or torchrun)
        if "RR_BENCH_PLACEMENT" in os.environ:
            placement = json.loads(os.environ["RR_BENCH_PLACEMENT"])
        else:
            n_local = int(os.environ.get("LOCAL_WORLD_SIZE", world))
            phys = ([device] * n_local if "RR_BENCH_DEVICE" in os.environ else physical_devices(n_local))
            placement = rank_placement(local, phys)
        pin_rank(placement)
        placement = {**placement, "cpus": cpuset_str(placement["cpus"]),
                     "omp_num_threads": int(os.environ["OMP_NUM_THREADS"])}
    import torch  # first, as in every bench run so far: the HIP runtime librr binds to is torch's
    gpu = torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(device)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # gloo: the only exchange is the timed region's max (host scalars); no RCCL
        dist.init_process_group("gloo", init_method="env://")

    def barrier(ctx=None):
        if dist is not None:
            dist.barrier()
        if gpu:
            torch.cuda.synchronize()
        if ctx is not None:
            ctx.synchronize()  # the renderer's own streams (rr_synchronize)

    rr = importlib.import_module(PKG)
    wl = WORKLOADS[args.workload]
    job = rr.BlenderJob.load_from_file(wl["job"])
    outdir = tempfile.mkdtemp(prefix=f"rr_bench_r{rank}_")
    job = rr.BlenderJob.from_dict({**job.to_dict(), "output_directory_path": outdir})
    frames = job.frames()

    def frame_of(step):
        return frame_partition(frames, step, rank, world)

    if args.dry_run:
        barrier()
        t0 = time.perf_counter()
        mine = [frame_of(args.warmup + s) for s in range(args.steps)]
        barrier()
        t_max = reduce_max_seconds(time.perf_counter() - t0, dist)
        by_rank, places = [mine], [placement]
        if dist is not None:
            by_rank, places = [None] * world, [None] * world
            dist.all_gather_object(by_rank, mine)
            dist.all_gather_object(places, placement)
        if rank == 0:
            print(json.dumps({"metric": wl["metric"], "value": None, "unit": "frames/s", "n_gpus": world,
                              "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(t_max / args.steps * 1e3, 6),
                              "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
                              "data": "dry run: no frames rendered", "dry_run": True,
                              "config": {"workload": wl["workload"], "job": os.path.basename(wl["job"]),
                                         "parallelism": f"frame-parallel x{world} (one worker per GPU, no collective)"},
                              "frames_by_rank": by_rank, "placement_by_rank": places}), flush=True)
        shutil.rmtree(outdir, ignore_errors=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    flags = 0 if args.no_profile else rr.native.RR_FLAG_PROFILE_KERNELS
    runner = rr.BackendRunner(ROOT, device=device, params=rr.default_params(flags=flags, spp=args.spp))

    # Device warm-up before the W warmup steps: frames of the same job, pipelined
    # as the timed loop renders them, for a fixed wall time. A k_tiles frame is
    # ~1 ms, so W = 5 warmup steps keep the GPU busy for ~6 ms, and the timed
    # region then starts before the engine clock has ramped: on one box, 20
    # timed frames after 5 warmup frames ran at 1,057-1,072 frames/s, the same
    # 20 frames after 100 more at 1,125 (tools/pipeline_timeline.py,
    # profiles/r6_pipeline_timeline.txt); every later repetition in the same
    # process ran at 1,123-1,132. The timed region is unchanged: exactly K steps
    # of full per-frame work between barrier + synchronize.
    warm_s = wl.get("device_warmup_s", 0.0) if args.device_warmup_s is None else args.device_warmup_s
    device_warmup = {"frames": 0, "seconds": 0.0}
    if warm_s > 0:
        tw = time.perf_counter()
        # the timed steps' own frames, so that per-launch averages over the whole
        # process (the PMC passes of tools/profile_round.sh) stay those frames'
        # (--serial: one frame at a time, as its timed loop renders them)
        while time.perf_counter() - tw < warm_s:
            batch = [frame_of(args.warmup + (device_warmup["frames"] + i) % args.steps) for i in range(8)]
            if args.serial:
                for f in batch:
                    runner.render_frame(job, f)
            else:
                runner.render_frames(job, batch)
            device_warmup["frames"] += 8
        device_warmup["seconds"] = round(time.perf_counter() - tw, 3)

    if args.serial:
        for w in range(args.warmup):
            runner.render_frame(job, frame_of(w))
    else:
        runner.render_frames(job, [frame_of(w) for w in range(args.warmup)])
    kernel_ms = [0.0] * 8
    launches = [0] * 8
    rays = {"camera": 0, "camera_traced": 0, "extension": 0, "extension_escaped": 0, "shadow": 0,
            "shadow_escaped": 0}
    substituted = []
    tile_modes = {"whole": 0, "sliced": 0}

    def account(st):
        for k in range(8):
            kernel_ms[k] += st.kernel_ms[k]
            launches[k] += st.kernel_launches[k]
        rays["camera"] += st.camera_rays
        rays["camera_traced"] += st.camera_rays_traced
        rays["extension"] += st.extension_rays
        rays["shadow"] += st.shadow_rays
        rays["extension_escaped"] += st.extension_rays_escaped
        rays["shadow_escaped"] += st.shadow_rays_escaped
        substituted.append(st.view_transform_substituted)
        if st.tile_slices == 1:
            tile_modes["whole"] += 1
        elif st.tile_slices > 1:
            tile_modes["sliced"] += 1

    barrier(runner.ctx)
    t0 = time.perf_counter()
    if args.serial:
        for s in range(args.steps):
            runner.render_frame(job, frame_of(args.warmup + s))
            account(runner.last_stats)
    else:
        # the worker's queued frames, frame N+1 rendering while N is encoded and
        # written (rr_frame_submit / rr_frame_complete); every frame is written
        runner.render_frames(job, [frame_of(args.warmup + s) for s in range(args.steps)],
                             on_frame=lambda f, frt, st: account(st))
    barrier(runner.ctx)
    elapsed = time.perf_counter() - t0
    last_stats = runner.last_stats
    t_max = reduce_max_seconds(elapsed, dist)
    places = [placement]
    if dist is not None:
        places = [None] * world
        dist.all_gather_object(places, placement)

    # Per-launch kernel times for the roofline. When consecutive k_tiles frames
    # overlap on the device (the two frame slots' streams, rr_api.cpp
    # enqueue_frame), an event pair around a launch also spans the wait for the
    # CUs the previous frame still holds; so those frames are timed again one at
    # a time after the timed region (rr_render_frame: nothing else in flight),
    # the same HIP events around the same launches. Frames of other paths never
    # overlap, and their timed-region events are used as they are.
    solo = not args.serial and launches[names_idx("tiles", rr)] > 0
    roof_ms, roof_launches, roof_steps = kernel_ms, launches, args.steps
    if solo:
        roof_ms, roof_launches = [0.0] * 8, [0] * 8
        roof_steps = min(args.steps, 10)
        for i in range(roof_steps):  # spread over the timed steps' frames
            runner.render_frame(job, frame_of(args.warmup + i * args.steps // roof_steps))
            for k in range(8):
                roof_ms[k] += runner.last_stats.kernel_ms[k]
                roof_launches[k] += runner.last_stats.kernel_launches[k]

    # traversal counts for the byte model: one counting frame, outside the timed region
    scene = runner._scene(rr.parse_with_base_directory_prefix(job.project_file_path, ROOT))
    f_count = frame_of(args.warmup)
    _, _, cstats = runner.ctx.render_to_memory(scene, f_count, rr.default_params(
        flags=rr.native.RR_FLAG_COUNT_TRAVERSAL, spp=args.spp), film=False, rgba=True)

    if rank == 0:
        total_frames = args.steps * world
        value = total_frames / t_max
        names = rr.native.KERNEL_CLASSES
        per_class = {names[k]: {"ms_total": kernel_ms[k], "launches": launches[k]} for k in range(len(names))}
        if solo:
            per_class = {names[k]: {"ms_total": roof_ms[k], "launches": roof_launches[k],
                                    "timed_region_event_ms_total": kernel_ms[k]} for k in range(len(names))}
        roofline = None
        if not args.no_profile:
            dom = max(range(len(names)), key=lambda k: roof_ms[k])
            timed = ({**tile_modes, "elapsed": elapsed} if names[dom] == "tiles" and sum(tile_modes.values()) else None)
            roofline = roofline_line(args, names[dom], cstats, roof_ms, roof_launches, names, roof_steps, timed)
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            try:
                from oracle import oracle as O
                # the oracle renders at most 128 spp per sample and is scaled to
                # the frame's spp (path cost is linear in spp)
                spp_full = int(last_stats.spp)
                spp_cpu = min(spp_full, 128)
                state = runner.ctx.frame_state(scene, f_count, rr.default_params(spp=spp_cpu))
                cpu = cpu_baseline(O, state, args.cpu_seconds, f"{args.workload} frame {f_count}",
                                   spp_scale=spp_full / spp_cpu)
                # the thesis' own single-worker point: one worker with 4 CPU cores
                # (scripts/arnes/queue-batch_04vs_14400f-1w.sh:6-7)
                w1 = cpu_baseline(O, state, args.cpu_seconds / 2, f"{args.workload} frame {f_count}",
                                  spp_scale=spp_full / spp_cpu, threads=4)
                cpu["thesis_point_w1_t4"] = {k: w1[k] for k in ("value", "unit", "cores", "sample")}
                # BASELINE.md §2 times W x T = nproc; this job may use a 16-core
                # share of the box (OMP_NUM_THREADS), so the whole host is a
                # projection from the measured points, never a measurement
                usable, nproc, _ = host_cpu()
                if cpu.get("value") and w1.get("value") and cpu["cores"] > w1["cores"]:
                    eff = (cpu["value"] / w1["value"]) / (cpu["cores"] / w1["cores"])
                    cpu["whole_host_projection"] = {
                        "value": round(cpu["value"] * nproc / cpu["cores"], 4), "unit": "frames/s", "cores": nproc,
                        "kind": "projection",
                        "scaling_eff_measured": round(eff, 3),
                        "note": f"linear in threads from the {cpu['cores']}-thread point to nproc = {nproc} "
                                f"(an upper bound: {w1['cores']} -> {cpu['cores']} threads scaled at {eff:.2f} of "
                                f"linear); not run: the job's CPU share on the GPU box is OMP_NUM_THREADS = "
                                f"{os.environ.get('OMP_NUM_THREADS')} of {usable} usable"}
            except Exception as e:  # baseline is reported, never the target
                cpu = {"value": None, "unit": "frames/s", "error": str(e)}
        # rays that entered a traversal: escaped continuations / shadow rays
        # (k_tiles' hull rule) are spawned and counted, but never walk a node
        traced = (rays["camera_traced"] + rays["extension"] - rays["extension_escaped"] + rays["shadow"]
                  - rays["shadow_escaped"])
        spawned = rays["camera_traced"] + rays["extension"] + rays["shadow"]
        wl_key = "" if args.workload == "04vs" else f"_{args.workload}"
        pmc_path = args.pmc_summary or newest_profile("%s_pmc" + wl_key + ".json")
        kc = float(getattr(cstats, "kernel_clock_ghz", 0.0) or 0.0) if cstats is not None else 0.0
        kernels_pmc = pmc_kernel_block(pmc_kernels(pmc_path),
                                       os.path.relpath(pmc_path, ROOT) if pmc_path else None,
                                       kc if 1.0 < kc <= PEAK_CLOCK_GHZ * 1.05 else PEAK_CLOCK_GHZ)
        result = {
            "metric": wl["metric"], "value": round(value, 4), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(t_max / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": wl["data"],
            "device_warmup": {**device_warmup, "note": "the timed steps' frames rendered before the W warmup steps "
                              "so the timed region starts at the engine clock it keeps (GPU clock ramp); not timed"},
            "config": {"workload": wl["workload"], "job": os.path.basename(wl["job"]),
                       "resolution": f"{int(last_stats.width)}x{int(last_stats.height)}", "spp": int(last_stats.spp),
                       "parallelism": f"frame-parallel x{world} (one worker per GPU, no collective)",
                       "pipelining": "serial (rr_render_frame per frame)" if args.serial else
                                     "3 frames in flight: frame N encoded + written while N+1 renders and N+2 waits on its stream",
                       "view_transform_substituted": int(any(substituted)),
                       "k_tiles_units": tile_modes,
                       "placement_by_rank": places},
            "mrays_per_s_per_gpu": round(traced / elapsed / 1e6, 1),
            # SURVEY 8(d)'s form: rays traced over the summed render-kernel time
            # (kernels timed alone, see roofline.launch_timing)
            "mrays_per_s_per_gpu_kernel_time": (
                round(traced / args.steps / (sum(roof_ms) / max(roof_steps, 1) * 1e-3) / 1e6, 1)
                if sum(roof_ms) > 0 else None),
            "mrays_spawned_per_s_per_gpu": round(spawned / elapsed / 1e6, 1),
            "rays_per_frame": {**{k: v // max(args.steps, 1) for k, v in rays.items()},
                               "traversed": traced // max(args.steps, 1)},
            "rays_note": "camera = W x H x spp samples; camera_traced = those tested against a triangle (the rest "
                         "lie outside the scene's screen rectangle or meet no triangle of their tile and are "
                         "resolved as background without a ray); extension / shadow = continuation / NEE shadow "
                         "rays spawned, of which *_escaped left a hull side of their triangle (every vertex of the "
                         "scene behind that side's plane: they meet nothing) and were resolved without a traversal; "
                         "traversed = camera_traced + extension + shadow - the escaped ones. mrays_per_s_per_gpu "
                         "counts traversed rays only; mrays_spawned_per_s_per_gpu counts the escaped ones too",
            "kernels_pmc": kernels_pmc,
            "whole_job_ceiling_frames_s": dispatch_ceiling(job.to_dict(), world),
            "value_under_reference_master_max": round(min(value, dispatch_ceiling(job.to_dict(), world)["value"]), 4),
            "device_ms_per_frame": round(sum(roof_ms) / max(roof_steps, 1), 3),
            "kernels": per_class,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    runner.close()
    shutil.rmtree(outdir, ignore_errors=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
