"""Worker for the multi-rank tests (launched by torch.distributed.run, 127.0.0.1).

mode "sim"  (CPU, gloo): numpy restatement of the sharded step — ids partitioned by
            owner (row % world), deduplicated, exchanged with the real Exchange
            all-to-alls, rows gathered from per-rank shards, gradients returned to
            owners, dense gradients all-reduced — must equal the single-process
            oracle at the global batch.
mode "gpu"  (ranks share cuda:0, gloo-staged exchange): the real ShardedCTREngine.
Writes rank-local results to OUT_DIR/rank{r}.npz.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from deep_learning_amd.synthetic import make_batch  # noqa: E402
from oracle import ctr_ref as R  # noqa: E402

KW = dict(C=13, V=0, S=26, E=8, cate_index_size=4000, hidden=[24, 16])


def global_batches(Bg, steps):
    out = []
    for i in range(steps):
        b = make_batch(Bg, cont=KW["C"], vector=KW["V"], cate_fields=KW["S"], cate_index_size=KW["cate_index_size"],
                       seed=100 + i)
        b["cate_feats"][0, :4] = [0, 1, 5, 12]
        b["cate_feats"][1, :3] = [2, 2, 2]
        out.append(b)
    return out


def local(b, rank, world):
    B = b["label"].shape[0] // world
    return {k: v[rank * B:(rank + 1) * B] for k, v in b.items()}


def run_sim(rank, world, steps, Bl, out_dir):
    """numpy sharded step over the real fixed-capacity block exchange (gloo): each owner's
    unique rows routed into a block of `cap` slots with a header, blocks exchanged both ways."""
    from deep_learning_amd.shard import Exchange
    ex = Exchange()
    cfg = R.make_cfg("deepfm_pipeline", **KW)
    P = R.init_params(cfg, np.random.default_rng(42))          # same global init everywhere
    N = R.n_rows(cfg)
    C, E = cfg.C, cfg.E
    own = lambda r: r % world
    nb = 2 * world - 1
    cap = -(-(Bl * 2 * KW["S"]) // world) * 2                # roomy: the sim never overflows
    # shard state: this rank's rows of the tables (+ Adam moments) keyed by global row
    opt = R.AdamTF1(cfg, P)
    for step, bg in enumerate(global_batches(Bl * world, steps)):
        b = local(bg, rank, world)
        cate = b["cate_feats"].astype(np.int64)
        rows = np.unique(np.concatenate([(cate + C).reshape(-1), cate.reshape(-1)]))
        rows = rows[rows >= C]                                  # replicated rows stay local
        owners = own(rows)
        send = [rows[owners == p] for p in range(world)]
        ids = torch.full((nb, cap), -1, dtype=torch.int32)
        hdr = torch.zeros((nb, 4), dtype=torch.int32)
        for p in range(world):
            ids[ex.block(p), : len(send[p])] = torch.from_numpy((send[p] // world).astype(np.int32))
            hdr[ex.block(p), 0] = len(send[p])
        ex.blocks([ids, hdr], 0)
        counts = [int(hdr[p, 0]) for p in range(world)]
        req = np.concatenate([ids[p, : counts[p]].numpy().astype(np.int64) * world + rank for p in range(world)])
        # owner side: answer from its own rows only
        assert np.all(own(req) == rank)
        ans = torch.zeros((nb, cap, E + 1), dtype=torch.float32)
        o = 0
        for p in range(world):
            r = req[o: o + counts[p]]
            ans[p, : len(r)] = torch.from_numpy(np.concatenate([P["feats_emb"][r], P["fm_first_order_emb"][r]], 1))
            o += counts[p]
        ans_v = ans.view(nb, -1)
        ex.blocks([ans_v], 1)
        back = np.concatenate([ans[ex.block(p), : len(send[p])].numpy() for p in range(world)])
        # the local view of the table: own/exchanged rows + replicated rows; others poisoned
        view = {k: np.full_like(v, np.nan) for k, v in P.items() if k in ("feats_emb", "fm_first_order_emb")}
        got = np.concatenate(send)
        view["feats_emb"][got] = back[:, :E]
        view["fm_first_order_emb"][got] = back[:, E:]
        view["feats_emb"][:C] = P["feats_emb"][:C]
        view["fm_first_order_emb"][:C] = P["fm_first_order_emb"][:C]
        Pl = dict(P)
        Pl.update(view)
        fw = R.forward(cfg, Pl, b)
        # global-batch mean: scale the local loss gradient by B_local / B_global
        G, dz = R.backward(cfg, Pl, b, fw)
        for k in G:
            if k not in ("feats_emb", "fm_first_order_emb"):
                G[k] = (G[k] - (cfg.l2 * P[k] if k == "deep_fm_weight" else 0)) / world \
                       + (cfg.l2 * P[k] if k == "deep_fm_weight" else 0)
        Gt = G["feats_emb"] / world
        G1 = G["fm_first_order_emb"] / world
        # embedding grads: requested rows go back to their owners
        gb = torch.zeros((nb, cap, E + 1), dtype=torch.float32)
        for p in range(world):
            gb[ex.block(p), : len(send[p])] = torch.from_numpy(
                np.concatenate([Gt[send[p]], G1[send[p]]], 1).astype(np.float32))
        ex.blocks([gb.view(nb, -1)], 0)
        grecv = np.concatenate([gb[p, : counts[p]].numpy() for p in range(world)])
        full_t = np.zeros_like(P["feats_emb"])
        full_1 = np.zeros_like(P["fm_first_order_emb"])
        np.add.at(full_t, req, grecv[:, :E])
        np.add.at(full_1, req, grecv[:, E:])
        # dense + replicated grads: one all-reduce (emulated per tensor)
        dense = {k: torch.from_numpy(np.ascontiguousarray(G[k])) for k in G if k not in ("feats_emb", "fm_first_order_emb")}
        l2w = cfg.l2 * P["deep_fm_weight"]
        dense["deep_fm_weight"] = torch.from_numpy(np.ascontiguousarray(G["deep_fm_weight"] - l2w))
        for k, t in dense.items():
            ex.all_reduce(t)
        rep_t = torch.from_numpy(np.ascontiguousarray(Gt[:C]))
        rep_1 = torch.from_numpy(np.ascontiguousarray(G1[:C]))
        ex.all_reduce(rep_t)
        ex.all_reduce(rep_1)
        Gall = {k: t.numpy() for k, t in dense.items()}
        Gall["deep_fm_weight"] = Gall["deep_fm_weight"] + l2w
        full_t[:C] = rep_t.numpy()
        full_1[:C] = rep_1.numpy()
        # rows not owned here keep zero gradient; after Adam only owned rows are meaningful
        Gall["feats_emb"], Gall["fm_first_order_emb"] = full_t, full_1
        opt.apply(P, Gall)
        # exchange the owned rows so every rank holds the true global table (test-only broadcast)
        for key in ("feats_emb", "fm_first_order_emb"):
            part = torch.from_numpy(np.ascontiguousarray(P[key]))
            mask = torch.from_numpy((np.arange(N) % world == rank) | (np.arange(N) < C))
            part[~mask] = 0
            if rank != 0:
                part[:C] = 0
            ex.all_reduce(part)
            P[key] = part.numpy()
            for mk in (opt.m, opt.v):
                mm = torch.from_numpy(np.ascontiguousarray(mk[key]))
                mm[~mask] = 0
                if rank != 0:
                    mm[:C] = 0
                ex.all_reduce(mm)
                mk[key] = mm.numpy()
        np.savez(os.path.join(out_dir, "rank%d_step%d.npz" % (rank, step)), z=fw["z"])
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), **P)


def run_gpu(rank, world, steps, Bl, out_dir, adam="dense", prefetch=False, owner_update=None, slack=None):
    """slack: the blocks' slack over an even split (-0.6: blocks too small for these batches, so
    the first step overflows, every rank grows its blocks and replays the skipped steps)."""
    from deep_learning_amd.engine import ModelSpec
    from deep_learning_amd.shard import Exchange, ShardedCTREngine
    torch.cuda.set_device(0)
    ex = Exchange()
    cfg = R.make_cfg("deepfm_pipeline", **KW)
    P = R.init_params(cfg, np.random.default_rng(42))
    eng = ShardedCTREngine(ModelSpec("deepfm_pipeline", **KW), Bl, ex, adam=adam, hist_len=4,
                           owner_update=owner_update, slack=slack)
    cap0 = eng.cap
    eng.load_params(P)
    batches = [local(bg, rank, world) for bg in global_batches(Bl * world, steps)]
    for step, b in enumerate(batches):
        # dense middle as a hipGraph from step 2; prefetch: the next batch's index and counts
        # on the side stream during this step
        nxt = batches[step + 1] if prefetch and step + 1 < len(batches) else None
        eng.train_step(b, graph=step >= 2, next_batch=nxt)
        torch.cuda.synchronize()
        np.savez(os.path.join(out_dir, "rank%d_step%d.npz" % (rank, step)), z=eng.z[:Bl].cpu().numpy(),
                 loss=eng.loss())
    # sharded eval (reference eval: predict every rank's half of two unseen global batches,
    # one AUC over all of them)
    evb = [local(bg, rank, world) for bg in global_batches(Bl * world, steps + 2)[steps:]]
    scores = [eng.predict(b) for b in evb]
    auc = eng.evaluate(evb)
    np.savez(os.path.join(out_dir, "rank%d_eval.npz" % rank), s0=scores[0], s1=scores[1], auc=auc)
    rows, t, f = eng.shard_state()
    dense = {"W%d" % l: eng.W[l].cpu().numpy() for l in range(len(KW["hidden"]))}
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), rows=rows, table=t, first=f,
             rep=eng.rep_t[:KW["C"]].cpu().numpy(), head=eng.w_head.cpu().numpy(),
             overflows=getattr(eng, "overflows", 0), cap=np.array([cap0, eng.cap]), **dense)


def run_gpu_badid(rank, world, steps, Bl, out_dir):
    """Lazy + prefetch; global batch 1 carries an out-of-range id on rank 1 only.  Every rank
    must raise at that step (one collective decides) with nothing applied, then train on."""
    from deep_learning_amd import _lib
    from deep_learning_amd.engine import ModelSpec
    from deep_learning_amd.shard import Exchange, ShardedCTREngine
    torch.cuda.set_device(0)
    ex = Exchange()
    cfg = R.make_cfg("deepfm_pipeline", **KW)
    P = R.init_params(cfg, np.random.default_rng(42))
    eng = ShardedCTREngine(ModelSpec("deepfm_pipeline", **KW), Bl, ex, adam="lazy", hist_len=4)
    eng.load_params(P)
    batches = [local(bg, rank, world) for bg in global_batches(Bl * world, steps)]
    if rank == 1:
        batches[1]["cate_feats"][3, 5] = KW["cate_index_size"] + 7
    raised, trained = [], 0
    for step, b in enumerate(batches):
        nxt = batches[step + 1] if step + 1 < len(batches) else None
        try:
            eng.train_step(b, graph=step >= 2, next_batch=nxt)
        except _lib.DLError as e:
            # reported `lag` calls after the skipped step, on every rank at the same call; this
            # call's own batch was trained
            assert "out of range" in str(e) and "rank(s) [1]" in str(e), str(e)
            raised.append(step)
        torch.cuda.synchronize()
        if step == 1:            # the skipped step: nothing applied, its logits are not a result
            continue
        np.savez(os.path.join(out_dir, "rank%d_step%d.npz" % (rank, trained)), z=eng.z[:Bl].cpu().numpy())
        trained += 1
    eng.check_error()
    assert float(eng.opt[7].item()) == steps - 1   # the skipped step never advanced global_step
    rows, t, f = eng.shard_state()
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), rows=rows, table=t, first=f, raised=np.array(raised),
             rep=eng.rep_t[:KW["C"]].cpu().numpy(), head=eng.w_head.cpu().numpy())


WKW = dict(C=13, S=26, E=16, cate_index_size=8000, hidden=[32, 24], Fw=26)


def wdl_batches(Bg, steps):
    out = []
    for i in range(steps):
        b = make_batch(Bg, cont=WKW["C"], cate_fields=WKW["S"], cate_index_size=WKW["cate_index_size"], seed=300 + i,
                       wide_fields=WKW["Fw"])
        b["wide_feats"][0, :3] = [WKW["Fw"], WKW["Fw"] + 1, 3]   # wide ids aliasing deep-output rows
        out.append(b)
    return out


def run_gpu_wdl(rank, world, steps, Bl, out_dir, adam, tower, prefetch):
    """Row-sharded Wide&Deep (table and wdl_weights sharded, bf16 or fp32 tower)."""
    from deep_learning_amd.engine import ModelSpec
    from deep_learning_amd.shard import Exchange, ShardedCTREngine
    torch.cuda.set_device(0)
    ex = Exchange()
    cfg = R.make_cfg("wdl", **WKW)
    P = R.init_params(cfg, np.random.default_rng(42))
    eng = ShardedCTREngine(ModelSpec("wdl", tower=tower, **WKW), Bl, ex, adam=adam, hist_len=4)
    eng.load_params(P)
    batches = [local(bg, rank, world) for bg in wdl_batches(Bl * world, steps)]
    for step, b in enumerate(batches):
        nxt = batches[step + 1] if prefetch and step + 1 < len(batches) else None
        eng.train_step(b, graph=step >= 2, next_batch=nxt)
        torch.cuda.synchronize()
        np.savez(os.path.join(out_dir, "rank%d_step%d.npz" % (rank, step)), z=eng.z[:Bl].cpu().numpy(),
                 loss=eng.loss())
    evb = [local(bg, rank, world) for bg in wdl_batches(Bl * world, steps + 2)[steps:]]
    scores = [eng.predict(b) for b in evb]
    auc = eng.evaluate(evb)
    rows, t, _ = eng.shard_state()
    wrows, wv = eng.wide_state()
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), rows=rows, table=t, wrows=wrows, ww=wv,
             wb=eng.wb[:1].cpu().numpy(), s0=scores[0], s1=scores[1], auc=auc,
             **{"W%d" % l: eng.W[l].cpu().numpy() for l in range(len(WKW["hidden"]))})


if __name__ == "__main__":
    mode, steps, Bl, out_dir = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    if mode == "sim":
        run_sim(rank, world, steps, Bl, out_dir)
    elif mode == "gpu_badid":
        run_gpu_badid(rank, world, steps, Bl, out_dir)
    elif mode.startswith("gpu_wdl"):
        run_gpu_wdl(rank, world, steps, Bl, out_dir, adam="lazy" if "lazy" in mode else "dense",
                    tower="bf16" if "bf16" in mode else "f32", prefetch=mode.endswith("_pf"))
    else:
        run_gpu(rank, world, steps, Bl, out_dir, adam="lazy" if mode.startswith("gpu_lazy") else "dense",
                prefetch=mode.endswith("_pf"), owner_update="chain" if "_chain" in mode else None,
                slack=-0.6 if "_ovf" in mode else None)
    dist.barrier()
    dist.destroy_process_group()
