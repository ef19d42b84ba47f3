"""Worker for test_exchange_p2p_matches_all_to_all (CPU, gloo): the grouped point-to-point
all-to-all of shard.Exchange (own segment copied locally, one send / receive per peer,
zero-size transfers skipped) against the all-to-all it replaces, on uneven splits."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_learning_amd.shard import Exchange  # noqa: E402


def main():
    dist.init_process_group("gloo")
    ex = Exchange()
    W, me = ex.world, ex.rank
    g = torch.Generator().manual_seed(7)
    # rows rank r sends to rank p: splits[r][p] (zeros included), 3 floats per row
    splits = torch.randint(0, 5, (W, W), generator=g)
    splits[0, W - 1] = 0
    splits[W - 1, 0] = 0
    send = list(splits[me].tolist())
    recv = [int(splits[r][me]) for r in range(W)]
    src = torch.arange(sum(send) * 3, dtype=torch.float32).view(-1, 3) + 1000 * me
    res = torch.full((sum(recv), 3), float("nan"))
    for w in ex._exchange_p2p(res, src, send, recv):
        w.wait()
    ref = torch.empty_like(res)
    dist.all_to_all_single(ref, src, output_split_sizes=recv, input_split_sizes=send)
    assert torch.equal(res, ref), (me, res, ref)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
