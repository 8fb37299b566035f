"""N>1 path of bench.py on CPU (gloo, world_size 2): the static frame partition
gives every rank disjoint frames that together cover the job, per-rank renders
of those frames equal a single-process render of the same frames (frames are
independent: no data-path collective), and the timed region reduces to the max
over ranks. Rendering here is the oracle (no GPU in this container); the GPU
path is the same per-frame call on each rank."""
import hashlib
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from oracle import host_oracle as HO  # noqa: E402
from oracle import oracle as O  # noqa: E402

JOB_FRAMES = list(range(1, 11))  # jobs/04_very-simple_demo_10f-1w.toml
W, H, SPP = 32, 18, 2


def _render_hash(frame: int) -> str:
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_oracle import world_tris
    from conftest import scene_path
    scene = HO.load_scene(scene_path("04_very-simple-standin.rrscene"))
    fc = HO.frame_constants(scene, frame, W, H)
    tris, mats = world_tris(scene, frame)
    ri = np.array([W, H, SPP, 12, 0, 0, 0, 0], np.int32)
    rf = np.array([10.0, 1.5, 1.0, 0], np.float32)
    _, rgba = O.render(tris, mats, fc["camera"], fc["lights"], fc["materials"], fc["world"], ri, rf, threads=1)
    return hashlib.sha256(rgba.tobytes()).hexdigest()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = [bench.frame_partition(JOB_FRAMES, s, rank, world) for s in range(steps)]
        hashes = {f: _render_hash(f) for f in mine}
        # each rank reports a different elapsed time; every rank must see the max
        t = bench.reduce_max_seconds(1.0 + rank * 0.5, dist)
        # verification only (the bench itself exchanges nothing but the time)
        gathered = [None] * world
        dist.all_gather_object(gathered, (rank, mine, hashes))
        if rank == 0:
            q.put((t, gathered))
    finally:
        dist.destroy_process_group()


def test_partition_single_rank_is_job_order():
    assert [bench.frame_partition(JOB_FRAMES, s, 0, 1) for s in range(10)] == JOB_FRAMES


def test_partition_covers_job_disjointly():
    for world in (2, 4, 8):
        steps = len(JOB_FRAMES) // world or 1
        seen = [bench.frame_partition(JOB_FRAMES, s, r, world) for s in range(steps) for r in range(world)]
        assert len(seen) == len(set(seen)) == min(steps * world, len(JOB_FRAMES))


def test_reduce_max_without_group():
    assert bench.reduce_max_seconds(2.5) == 2.5


@pytest.mark.timeout(300)
def test_two_rank_gloo_frame_parallel():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, steps = 2, 5
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    t, gathered = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == pytest.approx(1.5)
    frames = [f for _, mine, _ in gathered for f in mine]
    assert sorted(frames) == JOB_FRAMES  # 2 ranks x 5 steps = the whole 10-frame job, once each
    a, b = gathered[0][1], gathered[1][1]
    assert not set(a) & set(b)
    # sharded renders == single-process renders of the same frames
    for _, mine, hashes in gathered:
        for f in mine[:2]:
            assert hashes[f] == _render_hash(f)
    # frames differ (the animation moves the cube), so the check is not vacuous
    assert len({h for _, _, hs in gathered for h in hs.values()}) > 1


@pytest.mark.timeout(300)
def test_bench_spawns_one_rank_per_gpu_dry_run():
    """`bench.py --gpus 2` with no launcher starts 2 rank processes itself (gloo
    rendezvous, HIP_VISIBLE_DEVICES per rank) that take disjoint frames of the
    job; rank 0 prints one line with n_gpus 2. --dry-run: nothing is rendered
    (no GPU here)."""
    import json
    import subprocess
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                          "--steps", "5", "--warmup", "0"], capture_output=True, text=True, timeout=240,
                         env=dict(os.environ, HIP_VISIBLE_DEVICES="0,1"))
    assert res.returncode == 0, res.stderr[-2000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] is None and line["dry_run"]
    a, b = line["frames_by_rank"]
    assert not set(a) & set(b) and sorted(a + b) == JOB_FRAMES
    # each rank pinned to its own non-empty CPU share before any GPU call
    pa, pb = line["placement_by_rank"]
    print(pa, pb)
    assert (pa["device"], pb["device"]) == (0, 1)
    ca, cb = _bench().parse_cpulist(pa["cpus"]), _bench().parse_cpulist(pb["cpus"])
    assert ca and cb and not ca & cb
    assert 1 <= pa["omp_num_threads"] <= len(ca) and 1 <= pb["omp_num_threads"] <= len(cb)


def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_gpu_placement_follows_numa_nodes(tmp_path):
    """gpu_placement on an 8-GPU, 2-socket topology written as sysfs files: the
    KFD topology (CPU nodes first, then GPUs in HIP's order) gives each GPU's
    PCI address, the PCI device its NUMA node; each rank gets a disjoint,
    non-empty share of its own GPU's node, and ranks of one node split it."""
    b = _bench()
    topo = tmp_path / "class/kfd/kfd/topology/nodes"
    numa_of = [0, 0, 0, 0, 1, 1, 1, 1]
    for i in range(2):  # CPU nodes
        (topo / str(i)).mkdir(parents=True)
        (topo / str(i) / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    for g in range(8):
        bus = 0x10 + 0x10 * g
        (topo / str(2 + g)).mkdir(parents=True)
        (topo / str(2 + g) / "properties").write_text(f"simd_count 1024\nlocation_id {bus << 8}\ndomain 0\n")
        dev = tmp_path / "bus/pci/devices" / f"0000:{bus:02x}:00.0"
        dev.mkdir(parents=True)
        (dev / "numa_node").write_text(f"{numa_of[g]}\n")
    numa = b.gpu_numa_nodes(str(tmp_path))
    assert numa == numa_of
    node_cpus = {0: set(range(0, 64)) | set(range(128, 192)), 1: set(range(64, 128)) | set(range(192, 256))}
    allowed = set(range(256))
    plan = b.gpu_placement(list(range(8)), allowed, numa, lambda n: node_cpus[n])
    for r, cpus in enumerate(plan):
        assert len(cpus) == 32 and cpus <= node_cpus[numa_of[r]]
    assert len(set().union(*plan)) == 256  # disjoint
    assert [sum(1 for c in plan if c <= node_cpus[n]) for n in (0, 1)] == [4, 4]  # four ranks per socket
    # two ranks on one GPU (the one-GPU rehearsal) split that GPU's node
    p2 = b.gpu_placement([5, 5], allowed, numa, lambda n: node_cpus[n])
    assert p2[0] and p2[1] and not p2[0] & p2[1] and p2[0] | p2[1] == node_cpus[1]
    # no topology (CPU containers): the allowed set split evenly
    p3 = b.gpu_placement([0, 1], {0, 1, 2, 3, 4, 5, 6, 7}, [], lambda n: set())
    assert p3 == [{0, 1, 2, 3}, {4, 5, 6, 7}]
    assert b.cpuset_str([0, 1, 2, 5, 7, 8]) == "0-2,5,7-8" and b.parse_cpulist("0-2,5,7-8") == {0, 1, 2, 5, 7, 8}
