"""Worker of test_shard.py::test_status_guard_exits_when_a_peer_is_stuck (gloo, 2 ranks, CPU).

Rank 0 waits for a step's status report that never arrives (the sharded engine's
_check_reports on a host-side stand-in: an empty pinned-ring image); rank 1 sits in a
collective that rank 0 never joins — a peer stuck in RCCL in the real run.  Rank 0's guard
(DLAMD_SHARD_GUARD_S) must end its process non-zero and say where it stopped; the launcher
then stops rank 1."""
import os
import sys
import types

import numpy as np
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_learning_amd.shard import ShardedCTREngine  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    if rank == 0:
        st = types.SimpleNamespace(rank=rank, world=world, _ring_sent=5, _ring_checked=2, steps=5, cap=64,
                                   _ring_np=np.zeros(8, np.int32), host_wait=0.0, _hist_b={},
                                   guard_s=float(os.environ.get("DLAMD_SHARD_GUARD_S", "60")))
        st._guard_exit = lambda k: ShardedCTREngine._guard_exit(st, k)
        ShardedCTREngine._check_reports(st, 0)
        print("guard did not fire", flush=True)
        sys.exit(0)
    dist.barrier()   # rank 0 never joins: stuck until the launcher stops this rank
    sys.exit(0)


if __name__ == "__main__":
    main()
