"""Oracle self-checks (CPU): analytic backward vs torch autograd (fp64), TF1-Adam
formula, AUC vs sklearn (the reference's own AUC call)."""
import numpy as np
import pytest
import torch

from deep_learning_amd.synthetic import make_batch
from oracle import ctr_ref as R


MULTI = [[0, 6, "a"], [6, 11, "b"]]


def _cfg(model):
    kw = dict(S=4, E=8, cate_index_size=200, hidden=[12, 10])
    if model == "deepfm_pipeline":
        return R.make_cfg(model, C=5, **kw)
    if model in ("dnn_pipeline", "dnn_cate"):
        return R.make_cfg(model, C=5, V=3, **kw)
    if model == "deepfm":
        return R.make_cfg(model, C=5, V=3, **kw)
    if model == "dnn":
        return R.make_cfg(model, C=7, **kw)
    if model == "deepfm_cate":
        return R.make_cfg(model, V=2, **kw)
    if model in ("deepfm_multi_cate", "dnn_multi_cate"):
        return R.make_cfg(model, C=0, V=2, multi_ranges=MULTI, **dict(kw, cate_index_size=300))
    if model in ("deepfm_multi", "dnn_multi"):
        return R.make_cfg(model, C=5, V=2, multi_ranges=MULTI, **dict(kw, cate_index_size=300))
    return R.make_cfg("wdl", C=5, **kw)


def _batch(cfg, B=16, seed=3):
    if cfg.multi_ranges:
        b = make_batch(B, cont=cfg.C, vector=cfg.V, cate_fields=cfg.S, cate_index_size=cfg.cate_index_size,
                       multi_slots=0, seed=seed, cate_only=cfg.C == 0)
        rng = np.random.default_rng(seed)
        W = R.multi_width(cfg)
        multi = rng.integers(1, cfg.cate_index_size, size=(B, W))
        multi[rng.random((B, W)) < 0.4] = 0
        multi[0, :] = 0  # an all-padding sample: div_no_nan path
        b["cate_feats"] = np.concatenate([b["cate_feats"], multi], 1)
        return b
    b = make_batch(B, cont=cfg.C, vector=cfg.V, cate_fields=cfg.S, cate_index_size=cfg.cate_index_size,
                   seed=seed, wide_fields=6 if cfg.model == "wdl" else 0, cate_only=cfg.C == 0)
    b["cate_feats"][1, 0] = 0   # padding id hits the zeroed row
    return b


def _torch_loss(cfg, P, batch):
    """Independent torch fp64 restatement used only to check the analytic grads
    (each branch follows its reference model file)."""
    T = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in P.items()}
    E, S, C = cfg.E, cfg.S, cfg.C
    lab = torch.tensor(batch["label"][:, 0], dtype=torch.float64)
    B = lab.shape[0]
    vec = torch.tensor(batch["vector_feats"], dtype=torch.float64)
    cate = torch.tensor(batch["cate_feats"], dtype=torch.long)
    cont = torch.tensor(batch["cont_feats"], dtype=torch.float64) if C else torch.zeros(B, 0, dtype=torch.float64)
    ones = torch.ones(B, S, dtype=torch.float64)

    def z0(t):
        return torch.cat([torch.zeros_like(t[:1]), t[1:]], 0)

    def pool(tab, multi):   # nonzero_reduce_mean per slot (deepfm_multi.py:82-87)
        out = []
        for a, b_, _ in cfg.multi_ranges:
            emb = tab[multi[:, a:b_]]
            cnt = (emb.sum(2) != 0).sum(1, keepdim=True).double()
            s_ = emb.sum(1)
            out.append(torch.where(cnt > 0, s_ / torch.clamp(cnt, min=1), torch.zeros_like(s_)))
        return out

    def fm(firsts, embs):
        first = torch.cat(firsts, 1)
        e = torch.cat(embs, 1)
        s = e.sum(1)
        return first, 0.5 * (s * s - (e * e).sum(1))

    if cfg.model == "deepfm_pipeline":           # deepfm_pipeline.py:83-123
        V, w1 = z0(T["feats_emb"]), z0(T["fm_first_order_emb"])[:, 0]
        idx = torch.cat([torch.arange(C).repeat(B, 1), cate + C], 1)
        val = torch.cat([cont, ones], 1)
        first, second = fm([w1[idx] * val], [V[idx] * val[:, :, None]])
        x = torch.cat([cont, vec, V[cate].reshape(B, -1)], 1)
    elif cfg.model == "deepfm_cate":             # deepfm_cate.py:84-118
        V, w1 = z0(T["feats_emb"]), z0(T["fm_first_order_emb"])[:, 0]
        first, second = fm([w1[cate] * ones], [V[cate] * ones[:, :, None]])
        x = torch.cat([vec, V[cate].reshape(B, -1)], 1)
    elif cfg.model in ("dnn_pipeline", "dnn_cate"):   # dnn_pipeline.py:72-83, dnn_cate.py:71-76
        V = z0(T["feats_emb"])
        x = torch.cat([cont, vec, V[cate].reshape(B, -1)], 1)
    elif cfg.model in ("dnn_multi", "dnn_multi_cate"):   # dnn_multi.py:74-106, dnn_multi_cate.py:68-103
        V = z0(T["feats_emb"])
        single, multi = cate[:, :S], cate[:, S:]
        x = torch.cat([cont, vec, V[single].reshape(B, -1)] + pool(V, multi), 1)
    elif cfg.model == "deepfm_multi_cate":       # deepfm_multi_cate.py:113-171
        V, w1 = z0(T["feats_emb"]), z0(T["fm_first_order_emb"])
        single, multi = cate[:, :S], cate[:, S:]
        pf, pv = pool(w1, multi), pool(V, multi)
        first, second = fm([w1[single][:, :, 0]] + pf, [V[single], torch.stack(pv, 1)])
        x = torch.cat([vec, V[single].reshape(B, -1), torch.stack(pv, 1).reshape(B, -1)], 1)
    elif cfg.model == "deepfm_multi":            # deepfm_multi.py:124-188
        V, w1 = z0(T["feats_emb"]), z0(T["fm_first_order_emb"])
        single, multi = cate[:, :S], cate[:, S:]
        cidx = torch.arange(C).repeat(B, 1) + cfg.cate_index_size
        pf, pv = pool(w1, multi), pool(V, multi)
        first, second = fm([w1[cidx][:, :, 0] * cont, w1[single][:, :, 0]] + pf,
                           [V[cidx] * cont[:, :, None], V[single], torch.stack(pv, 1)])
        x = torch.cat([cont, vec, V[single].reshape(B, -1), torch.stack(pv, 1).reshape(B, -1)], 1)
    elif cfg.model == "deepfm":                  # deepfm.py:56-115 (no zero row; FM fields [cate | cont])
        V, w1 = T["feats_emb"], T["feats"][:, 0]
        idx = torch.cat([cate, torch.arange(C).repeat(B, 1) + S], 1)
        val = torch.cat([ones, cont], 1)
        first, second = fm([w1[idx] * val], [V[idx] * val[:, :, None]])
        x = torch.cat([cont, vec, V[cate].reshape(B, -1)], 1)
    else:                                        # wdl.py:132-179, dnn.py:49-60
        V = T["weight_mat"]
        x = torch.cat([cont, V[cate].reshape(B, -1)], 1)
    h = x
    for i in range(len(cfg.hidden)):
        h = torch.relu(h @ T["deep_%d" % i] + T["deep_bias_%d" % i])
    if cfg.model.startswith("deepfm"):
        z = (torch.cat([first, second, h], 1) @ T["deep_fm_weight"])[:, 0] + T["deep_fm_bias"][0]
        reg = 0.5 * (T["deep_fm_weight"] ** 2).sum()
    elif cfg.model == "dnn":
        z = (h @ T["deep_res"])[:, 0] + T["deep_res_bias"][0, 0]
        reg = sum(T["deep_%d" % i].abs().sum() for i in range(len(cfg.hidden)))   # l1_regularizer
    elif cfg.model.startswith("dnn"):
        z = (h @ T["deep_res"])[:, 0] + T["deep_res_bias"][0, 0]
        reg = 0.5 * (T["deep_res"] ** 2).sum()
    else:
        wide = torch.tensor(batch["wide_feats"], dtype=torch.long)
        w = T["wdl_weights"][:, 0]
        Fw, H = wide.shape[1], cfg.hidden[-1]
        z = w[wide].sum(1) + (w[Fw:Fw + H][None, :] * h).sum(1) + T["wdl_bias"][0]
        reg = 0.5 * (T["wdl_weights"] ** 2).sum() + sum(0.5 * (T["deep_%d" % i] ** 2).sum()
                                                       for i in range(len(cfg.hidden)))
    p = torch.sigmoid(z)
    eps = cfg.logloss_eps
    loss = (-lab * torch.log(p + eps) - (1 - lab) * torch.log(1 - p + eps)).mean() + cfg.l2 * reg
    loss.backward()
    return loss.item(), z.detach().numpy(), {k: t.grad.numpy() for k, t in T.items()}


ALL_MODELS = ["deepfm_pipeline", "deepfm_cate", "deepfm_multi_cate", "deepfm_multi", "dnn_pipeline", "dnn_cate",
              "dnn_multi", "dnn_multi_cate", "wdl", "deepfm", "dnn"]


@pytest.mark.parametrize("model", ALL_MODELS)
def test_backward_matches_autograd(model):
    cfg = _cfg(model)
    P = R.init_params(cfg, np.random.default_rng(7))
    P64 = {k: v.astype(np.float64) for k, v in P.items()}
    batch = _batch(cfg)
    fw = R.forward(cfg, P64, batch, dtype=np.float64)
    G, _ = R.backward(cfg, P64, batch, fw, dtype=np.float64)
    loss_t, z_t, G_t = _torch_loss(cfg, P, batch)
    np.testing.assert_allclose(fw["z"], z_t, rtol=1e-10, atol=1e-12)
    assert abs(fw["loss"] - loss_t) < 1e-10
    for k in P:
        np.testing.assert_allclose(G[k], G_t[k], rtol=1e-8, atol=1e-12, err_msg=k)


def test_adam_tf1_formula():
    cfg = R.make_cfg("dnn_pipeline")
    P = {"w": np.array([1.0, -2.0, 0.5], np.float32)}
    opt = R.AdamTF1(cfg, P)
    g = {"w": np.array([0.1, 0.0, -0.3], np.float32)}
    m = np.zeros(3); v = np.zeros(3); w = P["w"].astype(np.float64).copy()
    for t in range(1, 4):
        opt.apply(P, g)
        a = 0.001 * np.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
        m = m + (g["w"] - m) * 0.1
        v = v + (g["w"] ** 2 - v) * 0.001
        w = w - m * a / (np.sqrt(v) + 1e-8)
    np.testing.assert_allclose(P["w"], w, rtol=1e-6)
    assert opt.step == 3


def test_weighted_pool_matches_autograd():
    """dnn_multi_textline.py:89-103 weighted nonzero-mean pooling: forward vs a torch
    restatement, backward vs autograd (fp64); the count ignores the values."""
    rng = np.random.default_rng(5)
    V = rng.standard_normal((50, 8))
    V[0] = 0                      # the concatenated zero row (:43)
    V[7] = 0                      # a real id whose row is zero: not counted
    ids = rng.integers(0, 50, (9, 11))
    ids[0] = 0                    # an all-padding sample: div_no_nan -> 0
    ids[1, :6] = 7
    vals = rng.random((9, 11)) * 3
    vals[2, 1] = 0.0              # a zero value still counts (count is on the plain row)
    ranges = [[0, 6, "a"], [6, 11, "b"]]
    pooled, cnt = R.pool_weighted(V, ids, vals, ranges)
    Vt = torch.tensor(V, requires_grad=True)
    tab = torch.cat([torch.zeros(1, 8, dtype=torch.float64), Vt[1:]], 0)
    outs = []
    for a, b_, _ in ranges:
        e = tab[torch.tensor(ids[:, a:b_])]
        c = (e.sum(2) != 0).sum(1, keepdim=True).double()
        s = (e * torch.tensor(vals[:, a:b_, None])).sum(1)
        outs.append(torch.where(c > 0, s / c.clamp(min=1), torch.zeros_like(s)))
    pt = torch.stack(outs, 1)
    np.testing.assert_allclose(pooled, pt.detach().numpy(), rtol=1e-12, atol=1e-14)
    assert cnt[0].tolist() == [0, 0] and cnt[1, 0] == 0
    d = rng.standard_normal(pooled.shape)
    (pt * torch.tensor(d)).sum().backward()
    G = R.pool_weighted_bwd(50, ids, vals, ranges, cnt, d)
    np.testing.assert_allclose(G, Vt.grad.numpy(), rtol=1e-10, atol=1e-12)


def test_auc_matches_sklearn():
    from sklearn.metrics import roc_auc_score
    rng = np.random.default_rng(0)
    y = (rng.random(5000) < 0.3).astype(np.float32)
    s = np.round(rng.random(5000) * 20) / 20  # heavy ties
    assert abs(R.auc(y, s) - roc_auc_score(y, s)) < 1e-12
    s2 = rng.random(777)
    y2 = (rng.random(777) < s2).astype(np.float32)
    assert abs(R.auc(y2, s2) - roc_auc_score(y2, s2)) < 1e-12


def test_torch_cpu_restatement_matches_numpy_oracle():
    """bench.py's cpu_baseline times oracle/torch_cpu.py: it must compute what the numpy
    oracle computes (same deepfm_pipeline graph, dense TF1 Adam) — 3 steps, logits, loss
    and every parameter."""
    from oracle.torch_cpu import DeepFMPipelineCPU
    kw = dict(C=13, V=0, S=26, E=16, cate_index_size=3000, hidden=[48, 32])
    cfg = R.make_cfg("deepfm_pipeline", **kw)
    P = R.init_params(cfg, np.random.default_rng(3))
    m = DeepFMPipelineCPU(13, 26, 16, 3000, [48, 32], P)
    opt = R.AdamTF1(cfg, P)
    for i in range(3):
        b = make_batch(256, cate_index_size=3000, seed=50 + i)
        fw = R.train_step(cfg, P, opt, b)
        z, loss = m.train_step(b)
        np.testing.assert_allclose(z.numpy(), fw["z"], atol=1e-5, rtol=0)
        assert abs(loss - fw["loss"]) < 1e-5
    for k in P:
        np.testing.assert_allclose(m.params[k].detach().numpy(), P[k], atol=1e-5, rtol=0, err_msg=k)


def test_torch_cpu_restatement_dnn_pipeline_matches_numpy_oracle():
    """The C1 leg of bench.py's cpu_baseline (dnn_pipeline, fm=False) against the numpy oracle:
    3 steps, logits, loss and every parameter."""
    from oracle.torch_cpu import DeepFMPipelineCPU
    kw = dict(C=13, V=0, S=26, E=8, cate_index_size=2000, hidden=[48, 32, 16])
    cfg = R.make_cfg("dnn_pipeline", **kw)
    P = R.init_params(cfg, np.random.default_rng(4))
    m = DeepFMPipelineCPU(13, 26, 8, 2000, [48, 32, 16], P, fm=False)
    opt = R.AdamTF1(cfg, P)
    for i in range(3):
        b = make_batch(256, cate_index_size=2000, seed=60 + i)
        fw = R.train_step(cfg, P, opt, b)
        z, loss = m.train_step(b)
        np.testing.assert_allclose(z.numpy(), fw["z"], atol=1e-5, rtol=0)
        assert abs(loss - fw["loss"]) < 1e-5
    for k in P:
        np.testing.assert_allclose(m.params[k].detach().numpy(), P[k], atol=1e-5, rtol=0, err_msg=k)
