"""Replica layout of the multi-GPU path (turtlevsr_amd/replicas.py), world_size 2 over gloo on CPU.

bench.py runs one independent clip per GPU and reports frames of all ranks / slowest rank time;
these tests run that aggregation in two real processes (gloo, 127.0.0.1) with unequal per-rank
times and frame counts, and the clip assignment / seeding it relies on."""
import os
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from turtlevsr_amd.replicas import assign_clips, clip_seed, replica_throughput


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        elapsed = [2.0, 2.5][rank]          # rank 1 is the slow replica
        frames = [10, 12][rank]
        r = replica_throughput(elapsed, frames)
        q.put((rank, r.value, r.t_max, r.frames_total, clip_seed(rank), assign_clips(5, rank, world)))
    finally:
        dist.destroy_process_group()


def test_replica_throughput_two_ranks_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    for rank, value, tmax, frames, seed, clips in res:
        assert tmax == pytest.approx(2.5)              # the slowest rank's time
        assert frames == 22                            # every rank's frames
        assert value == pytest.approx(22 / 2.5)        # whole-job value, identical on every rank
    assert [r[4] for r in res] == [100, 101]           # distinct clips per replica
    assert [r[5] for r in res] == [[0, 2, 4], [1, 3]]


def test_replica_throughput_single_process():
    r = replica_throughput(4.0, 10)
    assert (r.value, r.t_max, r.frames_total) == (2.5, 4.0, 10)


def test_assign_clips_partition():
    for world in (1, 2, 3, 8):
        got = sorted(c for rank in range(world) for c in assign_clips(17, rank, world))
        assert got == list(range(17))
        sizes = [len(assign_clips(17, rank, world)) for rank in range(world)]
        assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        assign_clips(4, 2, 2)


def _probe(args, env=None):
    import json
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(here, "_launch_probe.py")] + args, env=e,
                       capture_output=True, text=True, timeout=300)
    return r.returncode, [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")], r.stderr


def test_launcher_spawns_one_worker_per_gpu_gloo():
    """`--gpus N` without an external launcher spawns N workers (the bench's own launcher); the
    gloo replica reduction over them gives frames of all ranks / slowest rank time."""
    rc, lines, err = _probe(["3"])
    assert rc == 0, err
    assert len(lines) == 1                                   # rank 0 only prints
    assert lines[0]["world"] == 3 and lines[0]["frames"] == 5 + 6 + 7
    assert lines[0]["t_max"] == pytest.approx(3.0) and lines[0]["value"] == pytest.approx(18 / 3.0)


def test_launcher_refuses_mismatched_world():
    rc, lines, err = _probe(["2"], env={"WORLD_SIZE": "4", "RANK": "0"})
    assert rc != 0 and not lines and "WORLD_SIZE=4" in err


def test_launcher_stops_the_group_when_a_worker_fails():
    """One shared deadline for the whole group; a worker failing (here rank 1, before any
    rendezvous) ends its siblings at once and its exit code is returned."""
    import time
    from turtlevsr_amd.replicas import launch_workers
    code = "import os, sys, time; r = int(os.environ['RANK']); sys.exit(3) if r == 1 else time.sleep(60)"
    t0 = time.monotonic()
    assert launch_workers(3, [sys.executable, "-c", code]) == 3
    assert time.monotonic() - t0 < 30
    t0 = time.monotonic()
    assert launch_workers(2, [sys.executable, "-c", "import time; time.sleep(60)"], timeout=1.0) == 124
    assert time.monotonic() - t0 < 30
    assert launch_workers(2, [sys.executable, "-c", "pass"]) == 0
