"""Multi-GPU layout of the Turtle frame path: independent replicas, one process per GPU.

Inference of a clip is a sequential recurrence (each frame's forward consumes the history caches
the previous frame produced: turtle_t1_arch.py:861-872), so one clip never shards; the unit of
parallel work is a whole clip. Each rank restores its own clip on its own GPU with no data-path
collective, and the job's throughput is the frames of all ranks over the slowest rank's time
(bench.py contract, "scaling": "weak"). The only collectives are these two scalar reductions,
over whatever backend the process group uses (RCCL on the GPU box, gloo in the CPU tests).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class ReplicaResult:
    value: float           # frames of all ranks / max rank time (frames/s)
    t_max: float           # slowest rank's timed-region seconds
    frames_total: int      # frames restored by all ranks


def clip_seed(rank: int, base: int = 100) -> int:
    """Seed of rank `rank`'s synthetic clip: every replica restores a different clip."""
    return base + rank


def assign_clips(n_clips: int, rank: int, world: int) -> list[int]:
    """Clip indices of rank `rank` when `n_clips` clips are spread over `world` replicas
    (round-robin, so any prefix of the clip list is balanced to within one clip)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    return list(range(rank, n_clips, world))


def replica_throughput(elapsed_s: float, frames_local: int, device: torch.device | str = "cpu") -> ReplicaResult:
    """Whole-job throughput of the replicas: SUM of frames over ranks / MAX of elapsed over ranks.
    Without an initialised process group this is the single-replica value."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return ReplicaResult(frames_local / elapsed_s, float(elapsed_s), int(frames_local))
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    n = torch.tensor([int(frames_local)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(n, op=dist.ReduceOp.SUM)
    tmax, frames = float(t.item()), int(n.item())
    return ReplicaResult(frames / tmax, tmax, frames)


def check_world(n_gpus: int) -> int | None:
    """World size this process belongs to. None: no launcher set one (the caller may spawn
    `n_gpus` workers itself); raises when an external launcher's WORLD_SIZE disagrees with the
    requested GPU count, so a mismatched launch never reports another configuration's numbers."""
    import os
    w = os.environ.get("WORLD_SIZE")
    if w is None:
        return None
    if int(w) != n_gpus:
        raise SystemExit(f"WORLD_SIZE={w} but --gpus {n_gpus}: launch one process per requested GPU")
    return int(w)


def launch_workers(n: int, argv: list[str], extra_env: dict | None = None, timeout: float | None = None,
                   poll_s: float = 0.2) -> int:
    """Run `argv` as `n` worker processes, one per GPU (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR=127.0.0.1 / MASTER_PORT set as torch.distributed.run does), and return an exit
    code: 0 when every worker succeeded, otherwise the code of the first worker seen failing.
    Called BEFORE the parent touches the GPU: the workers are children, never an exec of an
    initialised process. All workers are polled against ONE deadline (`timeout` seconds for the
    whole group); as soon as one exits non-zero - e.g. before the rendezvous, where its siblings
    would otherwise block until the process group's own timeout - the others are terminated.
    At the deadline every survivor is killed and the result is 124 (as `timeout(1)`)."""
    import os
    import socket
    import subprocess
    import time
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.update(extra_env or {})
        procs.append(subprocess.Popen(argv, env=env))
    deadline = None if timeout is None else time.monotonic() + timeout
    rc = 0

    def stop_all():
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_kill = time.monotonic() + 10.0
        for p in procs:
            try:
                p.wait(timeout=max(0.0, t_kill - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            rc = bad[0]
            stop_all()
            return rc
        if all(c == 0 for c in codes):
            return 0
        if deadline is not None and time.monotonic() >= deadline:
            stop_all()
            return 124
        time.sleep(poll_s)
