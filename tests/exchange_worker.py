"""Worker for test_block_exchange (CPU, gloo): shard.Exchange.blocks moves the fixed-capacity
blocks of the sharded step (shard.hip's layout: 2W - 1 blocks, block p < W = what peer p sent
this rank, block W + p - (p > rank) = this rank's side of its traffic with p) — checked against
what every peer put there, in both directions, for several dtypes and block shapes."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_learning_amd.shard import Exchange  # noqa: E402


def val(src, dst, j, dt):
    """What rank src puts in slot j of its block for rank dst."""
    return torch.tensor(1000 * src + 100 * dst + j).to(dt)


def main():
    dist.init_process_group("gloo")
    ex = Exchange()
    W, me = ex.world, ex.rank
    assert ex.staged
    for dt, blk in ((torch.int32, 5), (torch.float32, 7), (torch.int64, 3)):
        # direction 0: this rank's request block for peer p travels to p's block `me`
        a = torch.full((2 * W - 1, blk), -7, dtype=dt)
        for p in range(W):
            for j in range(blk):
                a[ex.block(p), j] = val(me, p, j, dt)
        own = a[me].clone()
        ex.blocks([a], 0)
        for p in range(W):
            for j in range(blk):
                want = val(p, me, j, dt)       # block p: what p sent to this rank (own block unchanged)
                assert a[p, j] == want, (me, p, j, a[p, j], want)
        assert torch.equal(a[me], own)
        # direction 1: the answers in block p go back to p's block for this rank
        b = torch.full((2 * W - 1, blk), -7, dtype=dt)
        for p in range(W):
            for j in range(blk):
                b[p, j] = val(me, p, j, dt)
        ex.blocks([b], 1)
        for p in range(W):
            if p == me:
                continue
            for j in range(blk):
                assert b[ex.block(p), j] == val(p, me, j, dt), (me, p, j)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
