"""numpy restatement of the reference CTR graphs — TEST INFRASTRUCTURE ONLY.

PARITY UNPINNED (model math): TensorFlow 1.x is absent, the reference has no
tests or fixtures.  Every step below cites the reference line it restates
(paths relative to the reference repo root).  Only tests/, smoke() and
bench.py's cpu_baseline leg may import this module.

Models restated:
  deepfm_pipeline   models/deepfm_pipeline.py:43-191
  dnn_pipeline      models/dnn_pipeline.py:40-137
  deepfm_multi_cate models/deepfm_multi_cate.py:45-240
  wdl               models/wdl.py:43-285
Optimizer: tf.train.AdamOptimizer (TF1 ApplyAdam, dense — see ledger item 6
in SURVEY.md: the embedding gradient reaches the Variable through
concat/strided-slice and is densified, so every row's m, v decay each step).
"""
import math

import numpy as np

F32 = np.float32

# ---------------------------------------------------------------------------
# configuration


class Cfg(dict):
    """Plain config: model, C (cont), V (vector), S (single cate fields),
    E (embedding), cate_index_size, hidden, multi_ranges, Fw (wdl wide ids),
    lr, l2, decay_steps, decay_rate, beta1, beta2, eps."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k)


def make_cfg(model, **kw):
    c = Cfg(model=model, C=13, V=0, S=26, E=16, cate_index_size=1000, hidden=[32, 32],
            multi_ranges=[], Fw=0, lr=0.001, l2=1e-5, decay_steps=10000000, decay_rate=0.9,
            beta1=0.9, beta2=0.999, eps=1e-8, logloss_eps=1e-7)
    c.update(kw)
    if model in ("deepfm_multi_cate",):
        c["C"] = 0
    return c


def n_rows(cfg):
    """Embedding-table rows (index_max_size)."""
    if cfg.model == "deepfm_pipeline":
        return cfg.C + cfg.cate_index_size          # deepfm_pipeline.py:77
    return cfg.cate_index_size                      # dnn_pipeline.py:69, deepfm_multi_cate.py:114, wdl.py:46


def multi_width(cfg):
    return sum(e - s for s, e, *_ in cfg.multi_ranges)


def deep_in(cfg):
    M = len(cfg.multi_ranges)
    if cfg.model == "deepfm_multi_cate":
        return cfg.V + cfg.S * cfg.E + M * cfg.E    # deepfm_multi_cate.py:169-174
    if cfg.model == "wdl":
        return cfg.C + cfg.S * cfg.E                # wdl.py:179-186
    return cfg.C + cfg.V + cfg.S * cfg.E            # deepfm_pipeline.py:123-127


def fm_fields(cfg):
    if cfg.model == "deepfm_pipeline":
        return cfg.C + cfg.S                        # deepfm_pipeline.py:92
    if cfg.model == "deepfm_multi_cate":
        return cfg.S + len(cfg.multi_ranges)        # deepfm_multi_cate.py:128
    return 0


def head_in(cfg):
    if cfg.model in ("deepfm_pipeline", "deepfm_multi_cate"):
        return fm_fields(cfg) + cfg.E + cfg.hidden[-1]   # deepfm_pipeline.py:158
    return cfg.hidden[-1]


# ---------------------------------------------------------------------------
# parameters (initial values are injected for parity: the reference draws the
# dense weights from UNSEEDED np.random — ledger item 7)


def init_params(cfg, rng):
    E, H = cfg.E, cfg.hidden
    N = n_rows(cfg)
    P = {}
    if cfg.model == "wdl":
        lim = math.sqrt(6.0 / (N + E))              # xavier_initializer, wdl.py:44-47
        P["weight_mat"] = rng.uniform(-lim, lim, (N, E)).astype(F32)
    else:
        P["feats_emb"] = (rng.standard_normal((N, E)) * 0.01).astype(F32)   # deepfm_pipeline.py:78
    if cfg.model in ("deepfm_pipeline", "deepfm_multi_cate"):
        P["fm_first_order_emb"] = rng.uniform(0.0, 1.0, (N, 1)).astype(F32)  # :80
    fan = deep_in(cfg)
    dims = [fan] + list(H)
    for i in range(len(H)):
        g = math.sqrt(2.0 / (dims[i] + dims[i + 1]))                         # :131,140
        P["deep_%d" % i] = (rng.standard_normal((dims[i], dims[i + 1])) * g).astype(F32)
        P["deep_bias_%d" % i] = (rng.standard_normal((1, dims[i + 1])) * g).astype(F32)
    if cfg.model in ("deepfm_pipeline", "deepfm_multi_cate"):
        F = head_in(cfg)
        g = math.sqrt(2.0 / (F + 1))                                         # :166
        P["deep_fm_weight"] = (rng.standard_normal((F, 1)) * g).astype(F32)
        P["deep_fm_bias"] = rng.standard_normal((1,)).astype(F32)            # :169
    elif cfg.model == "dnn_pipeline":
        g = math.sqrt(2.0 / (H[-1] + 1))                                     # dnn_pipeline.py:114
        P["deep_res"] = (rng.standard_normal((H[-1], 1)) * g).astype(F32)
        P["deep_res_bias"] = (rng.standard_normal((1, 1)) * g).astype(F32)   # :117
    elif cfg.model == "wdl":
        W = N + H[-1]
        g = math.sqrt(2.0 / W)                                               # wdl.py:241-244
        P["wdl_weights"] = (rng.standard_normal((W, 1)) * g).astype(F32)
        P["wdl_bias"] = rng.standard_normal((1,)).astype(F32)                # wdl.py:246
    return P


# ---------------------------------------------------------------------------
# forward


def _zero_row0(t):
    """tf.concat((zeros([1,E]), table[1:]), 0) — deepfm_pipeline.py:83-86."""
    t = t.copy()
    t[0] = 0
    return t


def _nonzero_reduce_mean(emb):
    """deepfm_multi_cate.py:73-78: cnt = count_nonzero(sum_E emb) over L;
    out = div_no_nan(sum_L emb, cnt).  emb: [B, L, E]."""
    axis2 = emb.sum(axis=2)
    cnt = (axis2 != 0).sum(axis=1, keepdims=True).astype(emb.dtype)
    s = emb.sum(axis=1)
    out = np.where(cnt > 0, s / np.where(cnt > 0, cnt, 1), 0).astype(emb.dtype)
    return out, cnt


def forward(cfg, P, batch, dtype=F32):
    """Returns dict with x0, hs (post-ReLU activations), feats (head input),
    z (logit), p (score) and model-specific intermediates."""
    E, S, C = cfg.E, cfg.S, cfg.C
    lab = batch["label"].astype(dtype).reshape(-1)
    B = lab.shape[0]
    out = {}
    vec = batch.get("vector_feats")
    vec = np.zeros((B, 0), dtype) if vec is None else vec.astype(dtype)
    if cfg.model == "deepfm_pipeline":
        V = _zero_row0(P["feats_emb"].astype(dtype))
        w1 = _zero_row0(P["fm_first_order_emb"].astype(dtype))[:, 0]
        cont = batch["cont_feats"].astype(dtype)
        cate = batch["cate_feats"].astype(np.int64)
        idx = np.concatenate([np.tile(np.arange(C, dtype=np.int64), (B, 1)), cate + C], 1)  # :58-61,89-90
        val = np.concatenate([cont, np.ones((B, S), dtype)], 1)                              # :62,91
        first = w1[idx] * val                                                                # :95-97
        e = V[idx] * val[:, :, None]                                                         # :102-104
        s = e.sum(1)                                                                         # :105
        second = (dtype(0.5) * (s * s - (e * e).sum(1))).astype(dtype)                       # :106-109
        cat_emb = V[cate].reshape(B, S * E)                                                  # :120-121
        x0 = np.concatenate([cont, vec, cat_emb], 1)                                         # :123
        out.update(idx=idx, val=val, e=e, s=s, first=first, second=second)
    elif cfg.model == "dnn_pipeline":
        V = _zero_row0(P["feats_emb"].astype(dtype))                                         # dnn_pipeline.py:72
        cont = batch["cont_feats"].astype(dtype)
        cate = batch["cate_feats"].astype(np.int64)
        x0 = np.concatenate([cont, vec, V[cate].reshape(B, S * E)], 1)                       # :78-83
    elif cfg.model == "deepfm_multi_cate":
        V = _zero_row0(P["feats_emb"].astype(dtype))                                         # deepfm_multi_cate.py:120
        w1 = _zero_row0(P["fm_first_order_emb"].astype(dtype))                               # :122 ([N,1])
        cate = batch["cate_feats"].astype(np.int64)
        single, multi = cate[:, :S], cate[:, S:]                                             # :58-59
        pf, pv, c1, cV = [], [], [], []
        for (a, b_, *_) in cfg.multi_ranges:                                                 # :80-108
            ids = multi[:, a:b_]
            f1, n1 = _nonzero_reduce_mean(w1[ids])                                           # :89,95
            fv, nv = _nonzero_reduce_mean(V[ids])                                            # :92,96
            pf.append(f1); pv.append(fv); c1.append(n1); cV.append(nv)
        M = len(cfg.multi_ranges)
        pooled_first = np.concatenate(pf, 1) if M else np.zeros((B, 0), dtype)
        pooled = np.stack(pv, 1) if M else np.zeros((B, 0, E), dtype)
        first = np.concatenate([w1[single][:, :, 0], pooled_first], 1)                       # :132-136
        e = np.concatenate([V[single], pooled], 1)                                           # :142-147
        s = e.sum(1)
        second = (dtype(0.5) * (s * s - (e * e).sum(1))).astype(dtype)                       # :149-153
        x0 = np.concatenate([vec, V[single].reshape(B, S * E), pooled.reshape(B, M * E)], 1)  # :169-171
        out.update(single=single, multi=multi, e=e, s=s, first=first, second=second,
                   cnt_first=np.concatenate(c1, 1) if M else None,
                   cnt_emb=np.concatenate(cV, 1) if M else None, pooled=pooled)
    elif cfg.model == "wdl":
        V = P["weight_mat"].astype(dtype)                                                    # wdl.py:44 (no zero row)
        cont = batch["cont_feats"].astype(dtype)
        cate = batch["cate_feats"].astype(np.int64)
        x0 = np.concatenate([cont, V[cate].reshape(B, S * E)], 1)                            # wdl.py:132-133,179
    else:
        raise ValueError(cfg.model)

    h = x0
    hs = []
    for i in range(len(cfg.hidden)):                                                         # :149-153
        h = np.maximum(h @ P["deep_%d" % i].astype(dtype) + P["deep_bias_%d" % i].astype(dtype), 0).astype(dtype)
        hs.append(h)

    if cfg.model in ("deepfm_pipeline", "deepfm_multi_cate"):
        feats = np.concatenate([out["first"], out["second"], h], 1)                          # :157
        z = (feats @ P["deep_fm_weight"].astype(dtype))[:, 0] + P["deep_fm_bias"].astype(dtype)[0]  # :171
    elif cfg.model == "dnn_pipeline":
        feats = h
        z = (h @ P["deep_res"].astype(dtype))[:, 0] + P["deep_res_bias"].astype(dtype)[0, 0]  # dnn_pipeline.py:119
    else:
        wide = batch["wide_feats"].astype(np.int64)
        Fw, H = wide.shape[1], cfg.hidden[-1]
        w = P["wdl_weights"].astype(dtype)[:, 0]
        widx = np.concatenate([wide, np.tile(np.arange(H) + Fw, (B, 1))], 1)                 # wdl.py:225-228,248
        wval = np.concatenate([np.ones((B, Fw), dtype), h], 1)                               # :249
        z = (w[widx] * wval).sum(1) + P["wdl_bias"].astype(dtype)[0]                         # :250-253
        feats = h
        out.update(widx=widx, wval=wval)
    z = z.astype(dtype)
    p = (1.0 / (1.0 + np.exp(-z.astype(np.float64)))).astype(dtype)                          # :173
    eps = dtype(cfg.logloss_eps)
    per = -lab * np.log(p + eps) - (1 - lab) * np.log(1 - p + eps)                           # :179 (tf.losses.log_loss)
    loss = per.astype(np.float64).mean()
    loss += _reg_loss(cfg, P)
    out.update(x0=x0, hs=hs, feats=feats, z=z, p=p, loss=loss, label=lab, V=V)
    return out


def _reg_loss(cfg, P):
    if cfg.l2 <= 0:
        return 0.0
    sq = lambda a: 0.5 * float((a.astype(np.float64) ** 2).sum())   # tf.nn.l2_loss
    if cfg.model in ("deepfm_pipeline", "deepfm_multi_cate"):
        return cfg.l2 * sq(P["deep_fm_weight"])                     # deepfm_pipeline.py:183
    if cfg.model == "dnn_pipeline":
        return cfg.l2 * sq(P["deep_res"])                           # dnn_pipeline.py:131
    r = cfg.l2 * sq(P["wdl_weights"])                               # wdl.py:270-271
    for i in range(len(cfg.hidden)):
        r += cfg.l2 * sq(P["deep_%d" % i])                          # wdl.py:272-275
    return r


# ---------------------------------------------------------------------------
# analytic backward (cross-checked against torch autograd in tests)


def dlogit(cfg, p, lab, dtype=F32):
    """d loss / d z for tf.losses.log_loss(labels, sigmoid(z)), mean over B:
    dp = (-y/(p+eps) + (1-y)/(1-p+eps)) / B ; dz = dp * p * (1-p) (SigmoidGrad)."""
    B = p.shape[0]
    eps = dtype(cfg.logloss_eps)
    dp = (-lab / (p + eps) + (1 - lab) / (1 - p + eps)) / dtype(B)
    return (dp * p * (1 - p)).astype(dtype)


def backward(cfg, P, batch, fw, dtype=F32):
    E, S, C = cfg.E, cfg.S, cfg.C
    B = fw["z"].shape[0]
    G = {k: np.zeros_like(v, dtype=dtype) for k, v in P.items()}
    dz = dlogit(cfg, fw["p"], fw["label"], dtype)
    l2 = dtype(cfg.l2)
    H = cfg.hidden
    h = fw["hs"][-1]
    if cfg.model in ("deepfm_pipeline", "deepfm_multi_cate"):
        W = P["deep_fm_weight"].astype(dtype)
        G["deep_fm_weight"] = (fw["feats"].T @ dz[:, None]).astype(dtype) + l2 * W
        G["deep_fm_bias"] = np.array([dz.sum()], dtype)
        dfeats = dz[:, None] * W[:, 0][None, :]
        nF = fm_fields(cfg)
        dfirst, dsec, dh = dfeats[:, :nF], dfeats[:, nF:nF + E], dfeats[:, nF + E:]
    elif cfg.model == "dnn_pipeline":
        W = P["deep_res"].astype(dtype)
        G["deep_res"] = (h.T @ dz[:, None]).astype(dtype) + l2 * W
        G["deep_res_bias"] = np.array([[dz.sum()]], dtype)
        dh = dz[:, None] * W[:, 0][None, :]
    else:
        w = P["wdl_weights"].astype(dtype)[:, 0]
        gw = np.zeros(w.shape[0], dtype)
        np.add.at(gw, fw["widx"].reshape(-1), (dz[:, None] * fw["wval"]).reshape(-1))
        G["wdl_weights"] = (gw + l2 * w).astype(dtype)[:, None]
        G["wdl_bias"] = np.array([dz.sum()], dtype)
        Fw = batch["wide_feats"].shape[1]
        dh = dz[:, None] * w[fw["widx"][:, Fw:]]
    # MLP backward
    xs = [fw["x0"]] + fw["hs"][:-1]
    g = (dh * (fw["hs"][-1] > 0)).astype(dtype)
    for i in reversed(range(len(H))):
        Wi = P["deep_%d" % i].astype(dtype)
        G["deep_%d" % i] = (xs[i].T @ g).astype(dtype)
        if cfg.model == "wdl":
            G["deep_%d" % i] += l2 * Wi
        G["deep_bias_%d" % i] = g.sum(0, keepdims=True).astype(dtype)
        dx = (g @ Wi.T).astype(dtype)
        g = (dx * (xs[i] > 0)).astype(dtype) if i > 0 else dx
    dx0 = g
    # embedding backward
    if cfg.model == "deepfm_pipeline":
        tab, t1 = "feats_emb", "fm_first_order_emb"
        idx, val, e, s = fw["idx"], fw["val"], fw["e"], fw["s"]
        de = dsec[:, None, :] * (s[:, None, :] - e)                 # d second / d e_f
        gV = (de * val[:, :, None]).reshape(-1, E)
        np.add.at(G[tab], idx.reshape(-1), gV)
        np.add.at(G[t1][:, 0], idx.reshape(-1), (dfirst * val).reshape(-1))
        cate = batch["cate_feats"].astype(np.int64)
        col = C + cfg.V
        np.add.at(G[tab], cate.reshape(-1), dx0[:, col:col + S * E].reshape(-1, E))
        G[tab][0] = 0                                              # concat zero-row: no grad to Var row 0
        G[t1][0] = 0
    elif cfg.model == "dnn_pipeline":
        cate = batch["cate_feats"].astype(np.int64)
        col = C + cfg.V
        np.add.at(G["feats_emb"], cate.reshape(-1), dx0[:, col:col + S * E].reshape(-1, E))
        G["feats_emb"][0] = 0
    elif cfg.model == "deepfm_multi_cate":
        tab, t1 = "feats_emb", "fm_first_order_emb"
        single, multi = fw["single"], fw["multi"]
        M = len(cfg.multi_ranges)
        e, s = fw["e"], fw["s"]
        de = dsec[:, None, :] * (s[:, None, :] - e)                # [B, S+M, E]
        # single fields: FM second + deep
        np.add.at(G[tab], single.reshape(-1), de[:, :S].reshape(-1, E))
        np.add.at(G[t1][:, 0], single.reshape(-1), dfirst[:, :S].reshape(-1))
        col = cfg.V
        np.add.at(G[tab], single.reshape(-1), dx0[:, col:col + S * E].reshape(-1, E))
        dpool = de[:, S:] + dx0[:, col + S * E: col + S * E + M * E].reshape(B, M, E)
        dpool1 = dfirst[:, S:]
        for m, (a, b_, *_) in enumerate(cfg.multi_ranges):
            ids = multi[:, a:b_]
            L = b_ - a
            cV = fw["cnt_emb"][:, m]
            c1 = fw["cnt_first"][:, m]
            gV = np.where(cV[:, None] > 0, dpool[:, m] / np.where(cV > 0, cV, 1)[:, None], 0).astype(dtype)
            g1 = np.where(c1 > 0, dpool1[:, m] / np.where(c1 > 0, c1, 1), 0).astype(dtype)
            np.add.at(G[tab], ids.reshape(-1), np.repeat(gV, L, axis=0).reshape(-1, E))
            np.add.at(G[t1][:, 0], ids.reshape(-1), np.repeat(g1, L))
        G[tab][0] = 0
        G[t1][0] = 0
    else:  # wdl
        cate = batch["cate_feats"].astype(np.int64)
        col = C
        np.add.at(G["weight_mat"], cate.reshape(-1), dx0[:, col:col + S * E].reshape(-1, E))
    return G, dz


# ---------------------------------------------------------------------------
# TF1 Adam (training_ops.cc ApplyAdam; optimizer state shared beta powers)


class AdamTF1:
    """tf.train.AdamOptimizer(learning_rate=exponential_decay(...)) — deepfm_pipeline.py:184-188.
    alpha = lr_t*sqrt(1-beta2^t)/(1-beta1^t); m += (g-m)(1-b1); v += (g^2-v)(1-b2);
    var -= (m*alpha)/(sqrt(v)+eps).  beta powers are float32 variables multiplied
    by beta after every apply; global_step increments after the apply."""

    def __init__(self, cfg, P, chunk=1 << 22):
        self.cfg = cfg
        self.m = {k: np.zeros_like(v) for k, v in P.items()}
        self.v = {k: np.zeros_like(v) for k, v in P.items()}
        self.b1p = F32(cfg.beta1)
        self.b2p = F32(cfg.beta2)
        self.step = 0
        self.chunk = chunk

    def lr_t(self):
        c = self.cfg
        p = math.floor(self.step / c.decay_steps)                 # staircase=True
        return F32(F32(c.lr) * F32(c.decay_rate) ** F32(p))

    def alpha(self):
        one = F32(1)
        return F32(self.lr_t() * np.sqrt(one - self.b2p) / (one - self.b1p))

    def apply(self, P, G):
        c = self.cfg
        a = self.alpha()
        b1, b2, eps = F32(1) - F32(c.beta1), F32(1) - F32(c.beta2), F32(c.eps)   # T(1) - beta1() in f32
        for k in P:
            p, m, v, g = P[k].reshape(-1), self.m[k].reshape(-1), self.v[k].reshape(-1), G[k].reshape(-1)
            for s in range(0, p.size, self.chunk):
                sl = slice(s, s + self.chunk)
                gs = g[sl].astype(F32)
                m[sl] += (gs - m[sl]) * b1
                v[sl] += (gs * gs - v[sl]) * b2
                p[sl] -= (m[sl] * a) / (np.sqrt(v[sl]) + eps)
        self.b1p = F32(self.b1p * F32(c.beta1))
        self.b2p = F32(self.b2p * F32(c.beta2))
        self.step += 1


def train_step(cfg, P, opt, batch):
    fw = forward(cfg, P, batch)
    G, dz = backward(cfg, P, batch, fw)
    opt.apply(P, G)
    return fw


# ---------------------------------------------------------------------------
# AUC (sklearn.metrics.roc_auc_score semantics: trapezoid with ties) —
# deepfm_pipeline.py:311,344


def auc(labels, scores):
    y = np.asarray(labels, np.float64).reshape(-1)
    s = np.asarray(scores, np.float64).reshape(-1)
    order = np.argsort(-s, kind="mergesort")
    s, y = s[order], y[order]
    distinct = np.where(np.diff(s))[0]
    thr = np.r_[distinct, y.size - 1]
    tps = np.cumsum(y)[thr]
    fps = 1 + thr - tps
    tps = np.r_[0, tps]
    fps = np.r_[0, fps]
    if tps[-1] <= 0 or fps[-1] <= 0:
        return float("nan")
    tpr = tps / tps[-1]
    fpr = fps / fps[-1]
    return float(np.trapezoid(tpr, fpr))
