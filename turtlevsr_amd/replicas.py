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
