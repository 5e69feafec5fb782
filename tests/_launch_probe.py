"""Worker script for tests/test_replicas.py: the bench's launcher contract on CPU (gloo).
Prints one JSON line on rank 0 with the aggregated replica throughput."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch.distributed as dist  # noqa: E402

from turtlevsr_amd.replicas import check_world, launch_workers, replica_throughput  # noqa: E402


def main():
    n = int(sys.argv[1])
    world = check_world(n)
    if world is None and n > 1:
        sys.exit(launch_workers(n, [sys.executable] + sys.argv))
    rank = int(os.environ.get("RANK", "0"))
    if world:
        dist.init_process_group("gloo")
    r = replica_throughput(1.0 + rank, 5 + rank)
    if rank == 0:
        print(json.dumps(dict(value=r.value, t_max=r.t_max, frames=r.frames_total, world=world or 1)), flush=True)
    if world:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
