"""numpy restatement of the reference CTR graphs — TEST INFRASTRUCTURE ONLY.

PARITY UNPINNED (model math): TensorFlow 1.x is absent, the reference has no
tests or fixtures.  Every step below cites the reference line it restates
(paths relative to the reference repo root).  Only tests/, smoke() and
bench.py's cpu_baseline leg may import this module.

Models restated:
  deepfm_pipeline   models/deepfm_pipeline.py:43-191
  deepfm_cate       models/deepfm_cate.py:73-182
  deepfm_multi_cate models/deepfm_multi_cate.py:45-240
  deepfm_multi      models/deepfm_multi.py:46-260
  dnn_pipeline      models/dnn_pipeline.py:40-137
  dnn_cate          models/dnn_cate.py:62-131
  dnn_multi         models/dnn_multi.py:70-167
  dnn_multi_cate    models/dnn_multi_cate.py:64-162
  wdl               models/wdl.py:43-285
  deepfm (load)     models/deepfm.py:39-162
  dnn (load)        models/dnn.py:35-96
Optimizer: tf.train.AdamOptimizer.  Pipeline models: TF1 ApplyAdam, dense — see
ledger item 6 in SURVEY.md: the embedding gradient reaches the Variable through
concat/strided-slice and is densified, so every row's m, v decay each step.
wdl / deepfm / dnn (load-style): the table Variables are read by
tf.nn.embedding_lookup directly, so their gradient is an IndexedSlices and TF
applies Adam._apply_sparse_shared (tensorflow/python/training/adam.py, TF 1.x):
dedup-sum the slices (unsorted_segment_sum), m = m*b1 then scatter_add(g*(1-b1)),
v = v*b2 then scatter_add((g*g)*(1-b2)), var -= lr*m/(sqrt(v)+eps) over every row.
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


# fm: FM outputs feed the head (deep_fm_weight), else deep_res; cont: "first" = FM cont rows
# 0..C-1 with cate ids at +C (deepfm_pipeline.py:58-61,89), "last" = FM cont rows at
# cate_index_size + j (deepfm_multi.py:139), "deep" = cont only in the deep input, None = no
# cont_feats (the cate algs of utils/data_loader.py:8); multi: nonzero-mean pooled slots.
FAMILIES = {
    "deepfm_pipeline": dict(fm=True, cont="first", multi=False),
    "deepfm_cate": dict(fm=True, cont=None, multi=False),
    "deepfm_multi_cate": dict(fm=True, cont=None, multi=True),
    "deepfm_multi": dict(fm=True, cont="last", multi=True),
    "dnn_pipeline": dict(fm=False, cont="deep", multi=False),
    "dnn_cate": dict(fm=False, cont=None, multi=False),
    "dnn_multi": dict(fm=False, cont="deep", multi=True),
    "dnn_multi_cate": dict(fm=False, cont=None, multi=True),
    "wdl": dict(fm=False, cont="deep", multi=False),
    "deepfm": dict(fm=True, cont="field", multi=False),   # FM fields [cate | cont], cont rows at S + j
    "dnn": dict(fm=False, cont="deep", multi=False),      # xavier weight_mat, L1 on hidden weights
}


def zero_row0(cfg):
    # deepfm_pipeline.py:83-86; none in wdl.py:44, deepfm.py:58-60, dnn.py:49-52
    return cfg.model not in ("wdl", "deepfm", "dnn")


def sparse_keys(cfg):
    """Variables TF updates with the sparse-apply Adam: read by embedding_lookup with no
    concat in between (wdl.py:44-47,132; deepfm.py:57-60,78,85,98; dnn.py:49-54).  wdl's
    wdl_weights is also looked up directly (wdl.py:250) but its L2 term (:270-271) adds a
    dense gradient, and TF's aggregation of an IndexedSlices with a Tensor is a dense add_n:
    ApplyAdam."""
    if cfg.model in ("wdl", "dnn"):
        return {"weight_mat"}
    if cfg.model == "deepfm":
        return {"feats_emb", "feats"}
    return set()


def table_key(cfg):
    return "weight_mat" if cfg.model in ("wdl", "dnn") else "feats_emb"


def first_key(cfg):
    return "feats" if cfg.model == "deepfm" else "fm_first_order_emb"   # deepfm.py:60


def make_cfg(model, **kw):
    c = Cfg(model=model, C=13, V=0, S=26, E=16, cate_index_size=1000, hidden=[32, 32],
            multi_ranges=[], Fw=0, lr=0.001, l2=1e-5, decay_steps=10000000, decay_rate=0.9,
            beta1=0.9, beta2=0.999, eps=1e-8, logloss_eps=1e-7)
    c.update(kw)
    fam = FAMILIES[model]
    if not fam["cont"]:
        c["C"] = 0
    if not fam["multi"]:
        c["multi_ranges"] = []
    return c


def is_fm(cfg):
    return FAMILIES[cfg.model]["fm"]


def fm_cont(cfg):
    return is_fm(cfg) and FAMILIES[cfg.model]["cont"] in ("first", "last", "field") and cfg.C > 0


def n_rows(cfg):
    """Embedding-table rows (index_max_size)."""
    if fm_cont(cfg):
        return cfg.C + cfg.cate_index_size          # deepfm_pipeline.py:77, deepfm_multi.py:125, deepfm.py:57
    return cfg.cate_index_size                      # dnn_pipeline.py:69, deepfm_multi_cate.py:114, wdl.py:46


def multi_width(cfg):
    return sum(e - s for s, e, *_ in cfg.multi_ranges)


def deep_in(cfg):
    # [cont, vector, single cate, pooled]: deepfm_pipeline.py:123, deepfm_multi.py:188,
    # dnn_multi.py:106, deepfm_multi_cate.py:169-174, wdl.py:179-186 (V = 0)
    return cfg.C + cfg.V + cfg.S * cfg.E + len(cfg.multi_ranges) * cfg.E


def fm_fields(cfg):
    if not is_fm(cfg):
        return 0
    # deepfm_pipeline.py:92 (C + S), deepfm_multi.py:128 (C + S + M), deepfm_multi_cate.py:128 (S + M)
    return (cfg.C if fm_cont(cfg) else 0) + cfg.S + len(cfg.multi_ranges)


def head_in(cfg):
    if is_fm(cfg):
        return fm_fields(cfg) + cfg.E + cfg.hidden[-1]   # deepfm_pipeline.py:158
    return cfg.hidden[-1]


# ---------------------------------------------------------------------------
# parameters (initial values are injected for parity: the reference draws the
# dense weights from UNSEEDED np.random — ledger item 7)


def init_params(cfg, rng):
    E, H = cfg.E, cfg.hidden
    N = n_rows(cfg)
    P = {}
    if table_key(cfg) == "weight_mat":
        lim = math.sqrt(6.0 / (N + E))              # xavier_initializer, wdl.py:44-47, dnn.py:49-52
        P["weight_mat"] = rng.uniform(-lim, lim, (N, E)).astype(F32)
    else:
        P["feats_emb"] = (rng.standard_normal((N, E)) * 0.01).astype(F32)   # deepfm_pipeline.py:78
    if is_fm(cfg):
        P[first_key(cfg)] = rng.uniform(0.0, 1.0, (N, 1)).astype(F32)       # :80
    fan = deep_in(cfg)
    dims = [fan] + list(H)
    for i in range(len(H)):
        g = math.sqrt(2.0 / (dims[i] + dims[i + 1]))                         # :131,140
        P["deep_%d" % i] = (rng.standard_normal((dims[i], dims[i + 1])) * g).astype(F32)
        P["deep_bias_%d" % i] = (rng.standard_normal((1, dims[i + 1])) * g).astype(F32)
    if is_fm(cfg):
        F = head_in(cfg)
        g = math.sqrt(2.0 / (F + 1))                                         # :166
        P["deep_fm_weight"] = (rng.standard_normal((F, 1)) * g).astype(F32)
        P["deep_fm_bias"] = rng.standard_normal((1,)).astype(F32)            # :169
    elif cfg.model != "wdl":
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


def _pool(cfg, V, w1, multi):
    """Per slot: nonzero-mean pooled V rows (and first-order weights when w1 is given),
    concatenated in range order (deepfm_multi_cate.py:80-108, dnn_multi.py:83-104)."""
    B, E = multi.shape[0], cfg.E
    pf, pv, c1, cV = [], [], [], []
    for (a, b_, *_) in cfg.multi_ranges:
        ids = multi[:, a:b_]
        if w1 is not None:
            f1, n1 = _nonzero_reduce_mean(w1[ids])                               # :89,95
            pf.append(f1); c1.append(n1)
        fv, nv = _nonzero_reduce_mean(V[ids])                                    # :92,96
        pv.append(fv); cV.append(nv)
    M = len(cfg.multi_ranges)
    dtype = V.dtype
    pooled = np.stack(pv, 1) if M else np.zeros((B, 0, E), dtype)
    pooled_first = np.concatenate(pf, 1) if (M and w1 is not None) else np.zeros((B, 0), dtype)
    return (pooled, pooled_first, np.concatenate(cV, 1) if M else None,
            np.concatenate(c1, 1) if (M and w1 is not None) else None)


def pool_weighted(V, ids, values, ranges):
    """Weighted nonzero-mean pooling of models/dnn_multi_textline.py:89-103 (deep-only).
    V: table with row 0 already zeroed (:43); ids, values: [B, W] multi-hot block and its
    per-position values (mul_cat_feats / mul_cat_feats_value, :57-58).  Per slot:
    cnt = count_nonzero(reduce_sum(V[ids], axis=2)) (:94-95, UNweighted rows),
    out = div_no_nan(reduce_sum(V[ids] * value, axis=1), cnt) (:97-102).
    Returns pooled [B, M, E] and cnt [B, M]."""
    outs, cnts = [], []
    for (a, b_, *_) in ranges:
        emb = V[ids[:, a:b_]]                                                    # :88-89
        cnt = (emb.sum(axis=2) != 0).sum(axis=1, keepdims=True).astype(V.dtype)  # :94-95
        s = (emb * values[:, a:b_, None].astype(V.dtype)).sum(axis=1)            # :97-101
        outs.append(np.where(cnt > 0, s / np.where(cnt > 0, cnt, 1), 0).astype(V.dtype))  # :102
        cnts.append(cnt)
    return np.stack(outs, 1), np.concatenate(cnts, 1)


def pool_weighted_bwd(n_rows, ids, values, ranges, cnt, d_pooled, zero_row0=True):
    """Gradient of pool_weighted w.r.t. the table (dense [n_rows, E]): every position l of
    slot m adds value_l * d_pooled[b, m] / cnt[b, m] (0 when cnt = 0) to its row; row 0
    (the concatenated zero row, :43) receives none."""
    E = d_pooled.shape[2]
    G = np.zeros((n_rows, E), d_pooled.dtype)
    for m, (a, b_, *_) in enumerate(ranges):
        c = cnt[:, m:m + 1]
        gv = np.where(c > 0, d_pooled[:, m] / np.where(c > 0, c, 1), 0)         # [B, E]
        idl = ids[:, a:b_]
        contrib = values[:, a:b_, None].astype(G.dtype) * gv[:, None, :]
        np.add.at(G, idl.reshape(-1), contrib.reshape(-1, E))
    if zero_row0:
        G[0] = 0
    return G


def forward(cfg, P, batch, dtype=F32):
    """Returns dict with x0, hs (post-ReLU activations), feats (head input),
    z (logit), p (score) and model-specific intermediates."""
    E, S, C = cfg.E, cfg.S, cfg.C
    lab = batch["label"].astype(dtype).reshape(-1)
    B = lab.shape[0]
    out = {}
    vec = batch.get("vector_feats")
    vec = np.zeros((B, 0), dtype) if vec is None else vec.astype(dtype)
    cont = batch["cont_feats"].astype(dtype) if C else np.zeros((B, 0), dtype)
    cate = batch["cate_feats"].astype(np.int64)
    if cfg.model == "wdl":
        V = P["weight_mat"].astype(dtype)                                                    # wdl.py:44 (no zero row)
        x0 = np.concatenate([cont, V[cate].reshape(B, S * E)], 1)                            # wdl.py:132-133,179
    else:
        zr = _zero_row0 if zero_row0(cfg) else (lambda t: t)
        V = zr(P[table_key(cfg)].astype(dtype))                                              # deepfm_pipeline.py:83-86
        w1 = zr(P[first_key(cfg)].astype(dtype)) if is_fm(cfg) else None                     # :85-86
        single, multi = cate[:, :S], cate[:, S:]                                             # deepfm_multi.py:64-65
        M = len(cfg.multi_ranges)
        pooled, pooled_first, cnt_emb, cnt_first = _pool(cfg, V, w1, multi)
        if is_fm(cfg):
            fam = FAMILIES[cfg.model]["cont"]
            Cf = C if fm_cont(cfg) else 0
            cont_off = cfg.cate_index_size if fam == "last" else 0                          # deepfm_multi.py:139
            cate_off = C if fam == "first" else 0                                            # deepfm_pipeline.py:89
            # FM fields [cont (row cont_off + j, value cont) | single (row id + cate_off, value 1)]
            cidx = np.tile(np.arange(Cf, dtype=np.int64) + cont_off, (B, 1))
            if fam == "field":    # deepfm.py:66-73: [cate | cont], cont rows at cate_field_size + j
                idx = np.concatenate([single, cidx + S], 1)
                val = np.concatenate([np.ones((B, S), dtype), cont[:, :Cf]], 1)
            else:
                idx = np.concatenate([cidx, single + cate_off], 1)                           # :58-61,89-90
                val = np.concatenate([cont[:, :Cf], np.ones((B, S), dtype)], 1)              # :62,91
            first = np.concatenate([w1[idx][:, :, 0] * val, pooled_first], 1)               # :95-97; multi :132-136
            e = np.concatenate([V[idx] * val[:, :, None], pooled], 1)                        # :102-104; multi :142-147
            s = e.sum(1)                                                                     # :105
            second = (dtype(0.5) * (s * s - (e * e).sum(1))).astype(dtype)                   # :106-109
            out.update(idx=idx, val=val, e=e, s=s, first=first, second=second)
        # deep input [cont, vector, single (raw ids: deepfm_pipeline.py:120), pooled]
        x0 = np.concatenate([cont, vec, V[single].reshape(B, S * E), pooled.reshape(B, M * E)], 1)
        out.update(single=single, multi=multi, pooled=pooled, cnt_emb=cnt_emb, cnt_first=cnt_first)

    h = x0
    hs = []
    for i in range(len(cfg.hidden)):                                                         # :149-153
        h = np.maximum(h @ P["deep_%d" % i].astype(dtype) + P["deep_bias_%d" % i].astype(dtype), 0).astype(dtype)
        hs.append(h)

    if is_fm(cfg):
        feats = np.concatenate([out["first"], out["second"], h], 1)                          # :157
        z = (feats @ P["deep_fm_weight"].astype(dtype))[:, 0] + P["deep_fm_bias"].astype(dtype)[0]  # :171
    elif cfg.model != "wdl":
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
    if is_fm(cfg):
        return cfg.l2 * sq(P["deep_fm_weight"])                     # deepfm_pipeline.py:183
    if cfg.model == "dnn":                                          # dnn.py:88-90: L1 on every hidden W
        return sum(cfg.l2 * float(np.abs(P["deep_%d" % i].astype(np.float64)).sum())
                   for i in range(len(cfg.hidden)))
    if cfg.model != "wdl":
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


def backward(cfg, P, batch, fw, dtype=F32, trace=None):
    """Analytic gradients of every parameter.  trace (a dict, tests only) receives each dense
    layer's input X_i and output gradient g_i (G[deep_i] = X_i^T g_i) and dz, so a test can
    measure how ill-conditioned a gradient sum is (sum_b |X_i[b, r]| |g_i[b, c]| against |G|)."""
    E, S, C = cfg.E, cfg.S, cfg.C
    B = fw["z"].shape[0]
    G = {k: np.zeros_like(v, dtype=dtype) for k, v in P.items()}
    dz = dlogit(cfg, fw["p"], fw["label"], dtype)
    l2 = dtype(cfg.l2)
    H = cfg.hidden
    h = fw["hs"][-1]
    if is_fm(cfg):
        W = P["deep_fm_weight"].astype(dtype)
        G["deep_fm_weight"] = (fw["feats"].T @ dz[:, None]).astype(dtype) + l2 * W
        G["deep_fm_bias"] = np.array([dz.sum()], dtype)
        dfeats = dz[:, None] * W[:, 0][None, :]
        nF = fm_fields(cfg)
        dfirst, dsec, dh = dfeats[:, :nF], dfeats[:, nF:nF + E], dfeats[:, nF + E:]
    elif cfg.model != "wdl":
        W = P["deep_res"].astype(dtype)
        G["deep_res"] = (h.T @ dz[:, None]).astype(dtype) + (l2 * W if cfg.model != "dnn" else 0)
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
    if trace is not None:
        trace.update(dz=dz, xs=xs, g={})
    for i in reversed(range(len(H))):
        Wi = P["deep_%d" % i].astype(dtype)
        if trace is not None:
            trace["g"][i] = g
        G["deep_%d" % i] = (xs[i].T @ g).astype(dtype)
        if cfg.model == "wdl":
            G["deep_%d" % i] += l2 * Wi
        elif cfg.model == "dnn":
            G["deep_%d" % i] += l2 * np.sign(Wi)                    # d/dW l1_regularizer
        G["deep_bias_%d" % i] = g.sum(0, keepdims=True).astype(dtype)
        dx = (g @ Wi.T).astype(dtype)
        g = (dx * (xs[i] > 0)).astype(dtype) if i > 0 else dx
    dx0 = g
    # embedding backward
    if cfg.model == "wdl":
        cate = batch["cate_feats"].astype(np.int64)
        col = C
        np.add.at(G["weight_mat"], cate.reshape(-1), dx0[:, col:col + S * E].reshape(-1, E))
        return G, dz
    tab, t1 = table_key(cfg), first_key(cfg)
    single, multi = fw["single"], fw["multi"]
    M = len(cfg.multi_ranges)
    col = C + cfg.V
    dpool = dx0[:, col + S * E: col + S * E + M * E].reshape(B, M, E)
    if is_fm(cfg):
        idx, val, e, s = fw["idx"], fw["val"], fw["e"], fw["s"]
        nI = idx.shape[1]                                          # cont + single FM fields
        de = dsec[:, None, :] * (s[:, None, :] - e)                # d second / d e_f
        gV = (de[:, :nI] * val[:, :, None]).reshape(-1, E)
        np.add.at(G[tab], idx.reshape(-1), gV)
        np.add.at(G[t1][:, 0], idx.reshape(-1), (dfirst[:, :nI] * val).reshape(-1))
        dpool = de[:, nI:] + dpool
        dpool1 = dfirst[:, nI:]
    np.add.at(G[tab], single.reshape(-1), dx0[:, col:col + S * E].reshape(-1, E))   # deep lookups (raw ids)
    for m, (a, b_, *_) in enumerate(cfg.multi_ranges):         # div_no_nan gradient to every member
        ids = multi[:, a:b_]
        L = b_ - a
        cV = fw["cnt_emb"][:, m]
        gV = np.where(cV[:, None] > 0, dpool[:, m] / np.where(cV > 0, cV, 1)[:, None], 0).astype(dtype)
        np.add.at(G[tab], ids.reshape(-1), np.repeat(gV, L, axis=0).reshape(-1, E))
        if is_fm(cfg):
            c1 = fw["cnt_first"][:, m]
            g1 = np.where(c1 > 0, dpool1[:, m] / np.where(c1 > 0, c1, 1), 0).astype(dtype)
            np.add.at(G[t1][:, 0], ids.reshape(-1), np.repeat(g1, L))
    if zero_row0(cfg):
        G[tab][0] = 0                                              # concat zero-row: no grad to Var row 0
        if is_fm(cfg):
            G[t1][0] = 0
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
        self.sparse = sparse_keys(cfg)
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
        beta1, beta2 = F32(c.beta1), F32(c.beta2)
        for k in P:
            p, m, v, g = P[k].reshape(-1), self.m[k].reshape(-1), self.v[k].reshape(-1), G[k].reshape(-1)
            for s in range(0, p.size, self.chunk):
                sl = slice(s, s + self.chunk)
                gs = g[sl].astype(F32)
                if k in self.sparse:
                    # _apply_sparse_shared: rows outside the batch are the g = 0 case (x + 0 = x)
                    m[sl] = m[sl] * beta1 + gs * b1
                    v[sl] = v[sl] * beta2 + (gs * gs) * b2
                    p[sl] -= (a * m[sl]) / (np.sqrt(v[sl]) + eps)
                else:
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
