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
