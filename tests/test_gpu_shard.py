"""The sharded step's device-side pieces on one GPU (shard.hip, optim.hip, comm.cpp):

* dl_shard_route against a numpy restatement of its block layout, from the batch index the
  kernel reads (index build already pinned bit-exact by test_index_build_matches_numpy): the
  request blocks, the replicated group, the headers, every unique row's slot and the remapped
  inverse map — with roomy blocks and with blocks too small (overflow flagged, no slot past cap);
* dl_shard_step_begin's one decision from the headers (bad ids, overflow, steps that disagree);
* the one-rank sharded engine as a captured step while an asynchronous torch RCCL work is
  still outstanding (the round-4 watchdog abort, now deterministic to reproduce: thread-local
  capture lets the process group's watchdog query its events mid-capture).
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch

from deep_learning_amd import _lib
from deep_learning_amd._lib import call, ptr

pytestmark = pytest.mark.gpu


def _s():
    return _lib.stream_handle()


def _route_ref(uniq, counts, world, rank, cap, rep_cap, inv0):
    """numpy restatement of dl_shard_route (shard.hip)."""
    mask = (1 << 27) - 1
    nb = 2 * world - 1
    blk = lambda p: p if p == rank else world + p - (1 if p > rank else 0)
    off = np.concatenate([[0], np.cumsum(counts)])
    ids = np.zeros(nb * cap, np.int64)      # blocks p != rank of [0, W): the peers' (not written)
    hdr = np.zeros((nb, 4), np.int64)
    for p in range(world):
        c = counts[p]
        take = min(c, cap)
        ids[blk(p) * cap: (blk(p) + 1) * cap] = -1
        ids[blk(p) * cap: blk(p) * cap + take] = uniq[off[p]: off[p] + take] & mask
        hdr[blk(p)] = [take, 0, rank, 0]
    rep = np.full(max(rep_cap, 1), -1, np.int64)
    take = min(counts[world], rep_cap)
    rep[:take] = uniq[off[world]: off[world] + take] & mask

    def slot(u):
        p = int(np.searchsorted(off[1:], u, side="right"))
        j = u - off[p]
        if p < world:
            return blk(p) * cap + j if j < cap else -1
        return nb * cap + j if j < rep_cap else -1
    upos = np.array([slot(u) for u in range(off[-1])], np.int64)
    inv = np.where(inv0 >= 0, np.array([slot(u) if u >= 0 else -1 for u in inv0]), -1)
    ovf = any(counts[p] > cap for p in range(world)) or counts[world] > rep_cap
    return ids, hdr, rep, upos, inv, ovf


@pytest.mark.parametrize("world,rank,room", [(3, 1, "roomy"), (3, 1, "tight"), (1, 0, "all"), (4, 3, "roomy"),
                                             (4, 0, "tight")])
def test_shard_route_matches_numpy(hip_lib, world, rank, room):
    from deep_learning_amd.engine import CTREngine, ModelSpec
    from deep_learning_amd.synthetic import make_batch
    B, C = 300, 13
    spec = ModelSpec("deepfm_pipeline", C=C, S=26, E=16, cate_index_size=20000, hidden=[16])
    eng = CTREngine(spec, max_batch=B, init="none")
    b = make_batch(B, cate_index_size=20000, seed=11)
    b["cate_feats"][0, :6] = [0, 0, 3, 3, 12, 19999]     # row 0, replicated rows (< 13 deep), repeats
    eng.stage(b)
    L = eng.layout
    L.batch = B
    n = B * 52
    zi = lambda k: torch.zeros(k, dtype=torch.int32, device="cuda")
    ws = torch.zeros(hip_lib.dl_index_workspace_bytes(n), dtype=torch.uint8, device="cuda")
    keys, refs, uniq, off, nu, inv, oc = zi(n), zi(n), zi(n), zi(n + 1), zi(4), zi(n), zi(world + 1)
    call("dl_index_build", ctypes.byref(L), ptr(eng.in_cate), world, C, ptr(ws), ws.numel(), ptr(keys), ptr(refs),
         ptr(uniq), ptr(off), ptr(nu), ptr(inv), ptr(oc), ptr(eng.err), _s())
    torch.cuda.synchronize()
    nuv = int(nu[0])
    u_h = uniq[:nuv].cpu().numpy().astype(np.uint32).astype(np.int64)
    counts = oc.cpu().numpy().astype(np.int64)
    inv0 = inv.cpu().numpy().astype(np.int64)
    rep_cap = 16
    # blocks just large enough for the biggest owner, 100 slots short of it, or every reference
    cap = {"roomy": int(counts[:world].max()), "tight": int(counts[:world].max()) - 100, "all": n}[room]
    nb = 2 * world - 1
    ids, hdr, rep = zi(nb * cap), zi(nb * 4), zi(rep_cap)
    upos = torch.full((n,), -7, dtype=torch.int32, device="cuda")
    call("dl_shard_route", ptr(uniq), ptr(nu), ptr(oc), world, rank, cap, rep_cap, ptr(eng.err), ptr(ids), ptr(hdr),
         ptr(rep), ptr(upos), ptr(inv), n, n, _s())
    torch.cuda.synchronize()
    e_ids, e_hdr, e_rep, e_upos, e_inv, ovf = _route_ref(u_h, counts, world, rank, cap, rep_cap, inv0)
    assert counts[world] > 0 and ovf == (room == "tight"), (counts, cap)
    np.testing.assert_array_equal(ids.cpu().numpy(), e_ids)
    h = hdr.cpu().numpy().reshape(nb, 4)
    np.testing.assert_array_equal(h[:, [0, 2, 3]], e_hdr[:, [0, 2, 3]])
    sent = [p if p == rank else world + p - (1 if p > rank else 0) for p in range(world)]   # the route's blocks
    assert (h[sent, 1] == (_lib.STATUS_OVERFLOW if ovf else 0)).all(), h[:, 1]
    np.testing.assert_array_equal(rep.cpu().numpy(), e_rep[:rep_cap])
    np.testing.assert_array_equal(upos[:nuv].cpu().numpy(), e_upos)
    np.testing.assert_array_equal(inv.cpu().numpy(), e_inv)


def test_shard_step_begin_one_decision(hip_lib):
    """Every rank's header: counts within cap, flags, rank, step.  A bad id anywhere skips the
    step (not sticky) and names the rank; an overflow or a header from another step poisons it
    and stays (sticky) until cleared; otherwise the Adam step begins as dl_step_begin's."""
    W, cap = 3, 100

    def run(hdrs, opt0=None):
        opt = torch.zeros(32, device="cuda")
        opt[:8] = torch.tensor([0.9, 0.999, 1e-3, 0.0, 0.9, 0.999, 1e-8, 5.0])
        if opt0 is not None:
            opt.copy_(opt0)
        h = torch.tensor(hdrs, dtype=torch.int32, device="cuda").reshape(-1)
        hist = torch.zeros(8, device="cuda")
        call("dl_shard_step_begin", ptr(h), None, W, cap, 0, ptr(opt), 0.9, 1e7, ptr(hist), 8, _s())
        torch.cuda.synchronize()
        return opt
    st = lambda o: int(o.view(torch.int32)[_lib.OPT_STATUS])
    sk = lambda o: int(o.view(torch.int32)[_lib.OPT_SKIP])
    ok = [[10, 0, p, 5] for p in range(W)]
    o = run(ok)
    assert sk(o) == 0 and st(o) == 0 and float(o[7]) == 6.0 and float(o[3]) > 0
    bad = [list(r) for r in ok]
    bad[2][1] = _lib.STATUS_BAD_ID
    o = run(bad)
    assert sk(o) == _lib.STATUS_BAD_ID and float(o[7]) == 5.0
    assert int(o.view(torch.int32)[_lib.OPT_BAD_RANKS]) == 1 << 2
    o2 = run(ok, o)                                       # the next good step applies
    assert sk(o2) == 0 and float(o2[7]) == 6.0
    ovf = [list(r) for r in ok]
    ovf[0][1] = _lib.STATUS_OVERFLOW
    o = run(ovf)
    assert sk(o) & _lib.STATUS_OVERFLOW and float(o[7]) == 5.0
    o2 = run(ok, o)                                       # sticky: the next step is skipped too
    assert sk(o2) & _lib.STATUS_OVERFLOW and float(o2[7]) == 5.0
    desync = [list(r) for r in ok]
    desync[1][3] = 4
    assert sk(run(desync)) & _lib.STATUS_DESYNC
    big = [list(r) for r in ok]
    big[1][0] = cap + 1
    assert sk(run(big)) & _lib.STATUS_INDEX


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_step_capture_with_outstanding_rccl_work(hip_lib):
    """The sharded step captured into its hipGraph while a torch RCCL collective issued
    asynchronously is still outstanding on the same rank (the process group's watchdog polls its
    events during the capture): thread-local capture mode lets it, so the capture completes and
    the captured steps give the eager steps' logits bit for bit."""
    import torch.distributed as dist
    from deep_learning_amd.engine import ModelSpec
    from deep_learning_amd.shard import Exchange, ShardedCTREngine
    from deep_learning_amd.synthetic import make_batch
    own = not dist.is_initialized()
    if own:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    try:
        spec = ModelSpec("deepfm_pipeline", C=13, S=26, E=16, cate_index_size=50000, hidden=[64, 32])
        bs = [{k: torch.from_numpy(v).cuda() for k, v in make_batch(512, cate_index_size=50000, seed=70 + i).items()}
              for i in range(4)]
        zs = []
        for graph in (False, True):
            eng = ShardedCTREngine(spec, 512, Exchange(), seed=3, adam="lazy")
            eng.init_device(3)
            out = []
            for i, b in enumerate(bs):
                if graph and i == 1:   # this call captures the step graph (the first step ran eagerly)
                    t = torch.ones(1 << 22, device="cuda")
                    work = dist.all_reduce(t, async_op=True)
                    eng.train_step(b, graph=True, next_batch=bs[i + 1])
                    work.wait()
                    assert eng.graphs, "the step was not captured"
                else:
                    eng.train_step(b, graph=graph, next_batch=bs[i + 1] if i + 1 < len(bs) else None)
                torch.cuda.synchronize()
                out.append(eng.z[:512].clone())
            eng.check_error()
            zs.append(torch.stack(out))
            eng.exch.close()
            del eng
        assert torch.equal(zs[0], zs[1])
    finally:
        if own:
            dist.destroy_process_group()
