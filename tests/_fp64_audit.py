"""Stage-wise fp64 audit of one GPU training step (test infrastructure for test_gpu_fullsize.py).

The GPU's step keeps its intermediates on the device (x0, every layer's activations h_l and
output gradients dh_l, dx0, z, dz, the FM outputs and sums, the pre-update head weights).
Each stage of the step is recomputed in float64 from the GPU's OWN inputs to that stage and
the GPU's output must agree within that stage's f32 error bound

    |gpu - fp64| <= K * 2^-24 * S

where S is the stage's running-error scale (the same expression on absolute values: |X| |W|
for a product, |a| + |b| for a difference) and K the stage's summation depth (Higham's
forward-error bound; the three-plane bf16 products of the s3 GEMMs are exact to 2^-24).  A
ReLU whose fp64 pre-activation is within that bound of zero may go either way.  The stages,
following models/deepfm_pipeline.py:89-191 and deepfm_multi_cate.py:71-240:

    x0 (the gathered rows bit-exact, pooled means), FM first / second order and sums,
    each hidden layer h_l = relu(X_l W_l + b_l), the logit z, dz = dlogloss/dz of the GPU's z,
    each output gradient dh_l (ReluGrad by the GPU's own h_l), dx0.

Parameter gradients are audited per element (audit_elements): the gradient the GPU applied,
read back from its Adam moments (ApplyAdam: m1 = m0 + (g - m0)(1 - b1)), against the fp64 sum
of the GPU's own terms (X_l^T dh_l, feats^T dz, each table row's references), within the sum's
own bound; its v and p must have moved by TF1 Adam on that gradient.  Together: every stage of
the GPU's step is an f32 evaluation of the reference graph, so an element whose value differs
from the f32 oracle's (numpy's evaluation order) is ill-conditioned, not wrong.

Supported: the pipeline models with a zero row 0 — the FM ones (deepfm_pipeline,
deepfm_multi_cate: BASELINE configs C2, C3) and the DNN ones (dnn_pipeline: C1, whose head is
deep_res on the last hidden layer, dnn_pipeline.py).
"""
import numpy as np

from oracle import ctr_ref as R

U32 = 2.0 ** -24
F64 = np.float64
K_GEMM = 512        # forward / input-gradient products: 6 bf16 planes x <= 512 / 32 MFMA chunks + bias
K_WGRAD = 2048      # weight gradients: 6 planes x (65,536 / 32 slabs) / 32 chunks + 32 slab sums, rounded up
K_TABLE = 512       # table rows: a row's references summed in fixed-order segments / chunks (segment.h) and
                    # the FM cont rows' 65,536 references as block partials + a reduce (pairwise-like
                    # depth); measured worst 92 u*S over 20 full-size C2/C3 steps (round 4: was 8,192)


def read_gpu(eng, B):
    """The step's intermediates from the engine (host float64/float32, reference layouts)."""
    sp = eng.spec
    L = len(sp.hidden)
    x0i = eng.x0[:B].cpu().numpy()
    x0 = np.zeros((B, sp.deep_in), np.float32)
    x0[:, sp.x0_ref_rows()] = x0i[:, :sp.deep_in]
    d = dict(x0=x0, h=[eng.h[l][:B, :sp.hidden[l]].cpu().numpy() for l in range(L)],
             dh=[eng.dh[l][:B, :sp.hidden[l]].cpu().numpy() for l in range(L)],
             dx0=eng.dx0[:B, :(sp.S + sp.M) * sp.E].cpu().numpy(), z=eng.z[:B].cpu().numpy(),
             dz=eng.dz[:B].cpu().numpy(), fm_out=eng.fm_out[:B, :sp.fm_cols].cpu().numpy(),
             fm_sum=eng.fm_sum[:B, :sp.E].cpu().numpy(), w_head=eng.w_head_prev[:eng.head_n].cpu().numpy())
    if sp.M:
        d["cnt_emb"] = eng.cnt_emb[:B].cpu().numpy()
        if sp.fm:
            d["cnt_first"] = eng.cnt_first[:B].cpu().numpy()
    return d


class StepAudit:
    def __init__(self, cfg, P, batch, gpu):
        """P: the GPU's pre-step parameters (reference layout); gpu: read_gpu() after the step."""
        assert R.zero_row0(cfg) and cfg.model not in ("wdl", "deepfm", "dnn"), "the audit covers the pipeline models"
        fm = self.fm = R.is_fm(cfg)
        self.cfg, self.gpu = cfg, gpu
        self.fails, self.stats = [], {}
        E, S, C = cfg.E, cfg.S, cfg.C
        lab = batch["label"].astype(F64).reshape(-1)
        B = lab.shape[0]
        self.B = B
        tab, t1 = R.table_key(cfg), R.first_key(cfg)
        self.tab, self.t1 = tab, t1
        cate = batch["cate_feats"].astype(np.int64)
        single, multi = cate[:, :S], cate[:, S:]
        cont = batch["cont_feats"].astype(F64) if C else np.zeros((B, 0))
        vec = batch.get("vector_feats")
        vec = np.zeros((B, 0)) if vec is None else vec.astype(F64)
        M = len(cfg.multi_ranges)
        L = len(cfg.hidden)

        def rows32(ids):                     # gathered f32 rows, row 0 zeroed (deepfm_pipeline.py:83-86)
            r = P[tab][ids]
            r[ids == 0] = 0
            return r

        def w1(ids):
            r = P[t1][ids, 0].astype(F64)
            return np.where(ids == 0, 0, r)

        fam = R.FAMILIES[cfg.model]["cont"]
        Cf = C if R.fm_cont(cfg) else 0
        cidx = np.tile(np.arange(Cf, dtype=np.int64) + (cfg.cate_index_size if fam == "last" else 0), (B, 1))
        idx = np.concatenate([cidx, single + (C if fam == "first" else 0)], 1)
        val = np.concatenate([cont[:, :Cf], np.ones((B, S))], 1)
        nI = idx.shape[1]
        nF = R.fm_fields(cfg) if fm else 0
        # ---- x0: the deep lookups bit-exact, the pooled means within their bound
        x0g = gpu["x0"].astype(F64)
        col = C + cfg.V
        single_rows = rows32(single).reshape(B, S * E)
        self._exact("x0 cate rows", gpu["x0"][:, col:col + S * E], single_rows)
        self._exact("x0 cont/vector", gpu["x0"][:, :col], np.concatenate([cont, vec], 1).astype(np.float32))
        pooled, pooled_a, p1, p1_a = [], [], [], []
        for m, (a, b_, *_) in enumerate(cfg.multi_ranges):
            ids = multi[:, a:b_]
            v32 = rows32(ids)
            n = (v32.sum(axis=2) != 0).sum(1)
            f32 = np.where(ids == 0, 0, P[t1][ids, 0]) if fm else np.zeros(ids.shape, np.float32)
            n1 = (f32 != 0).sum(1)
            # the counts are integers: bit-exact
            self._exact("pool count slot %d" % m, gpu["cnt_emb"][:, m], n.astype(np.float32))
            if fm:
                self._exact("pool first-order count slot %d" % m, gpu["cnt_first"][:, m], n1.astype(np.float32))
            dv = np.where(n > 0, n, 1)[:, None].astype(F64)
            pooled.append(np.where(n[:, None] > 0, v32.astype(F64).sum(1) / dv, 0))
            pooled_a.append(np.where(n[:, None] > 0, np.abs(v32.astype(F64)).sum(1) / dv, 0))
            d1 = np.where(n1 > 0, n1, 1).astype(F64)
            p1.append(np.where(n1 > 0, f32.astype(F64).sum(1) / d1, 0))
            p1_a.append(np.where(n1 > 0, np.abs(f32.astype(F64)).sum(1) / d1, 0))
        if M:
            pc = col + S * E
            pooled, pooled_a = np.stack(pooled, 1), np.stack(pooled_a, 1)
            p1, p1_a = np.stack(p1, 1), np.stack(p1_a, 1)
            self._close("x0 pooled", x0g[:, pc:pc + M * E], pooled.reshape(B, -1), pooled_a.reshape(B, -1), 128)
            pg = x0g[:, pc:pc + M * E].reshape(B, M, E)      # the GPU's pooled rows feed its FM
        else:
            pg = np.zeros((B, 0, E))
            p1 = np.zeros((B, 0))
        # ---- FM first / second order (deepfm_pipeline.py:89-110) from the GPU's pooled rows
        e = ea = fs = sa = None
        fo = np.zeros((B, 0))
        if fm:
            ei = rows32(idx).astype(F64) * val[:, :, None]
            e = np.concatenate([ei, pg], 1)
            ea = np.abs(e)
            s64, sa = e.sum(1), ea.sum(1)
            fo = gpu["fm_out"].astype(F64)
            fs = gpu["fm_sum"].astype(F64)
            self._close("fm first order", fo[:, :nI], w1(idx) * val, np.abs(w1(idx) * val), 4)
            if M:
                self._close("fm pooled first order", fo[:, nI:nF], p1, p1_a, 128)
            self._close("fm sum", fs, s64, sa, 128)
            second = 0.5 * (fs * fs - (e * e).sum(1))
            self._close("fm second order", fo[:, nF:nF + E], second,
                        0.5 * (fs * fs + (ea * ea).sum(1) + 2 * sa * sa), 256)
        # ---- tower forward: h_l = relu(X_l W_l + b_l) from the GPU's X_l
        Ws = [P["deep_%d" % i].astype(F64) for i in range(L)]
        bs = [P["deep_bias_%d" % i].astype(F64) for i in range(L)]
        X = [x0g] + [gpu["h"][i].astype(F64) for i in range(L)]
        for i in range(L):
            pre = X[i] @ Ws[i] + bs[i]
            A = np.abs(X[i]) @ np.abs(Ws[i]) + np.abs(bs[i])
            h = X[i + 1]
            bound = K_GEMM * U32 * A
            on = h > 0
            err = np.where(on, np.abs(h - pre), np.maximum(pre, 0))    # off: the pre-activation must be <= ~0
            self._count("layer %d forward" % i, err, bound)
        # ---- logit and its gradient (deepfm_pipeline.py:157-179)
        Wh = gpu["w_head"].astype(F64)
        feats = np.concatenate([fo, X[L]], 1)
        z64 = feats @ Wh[:-1] + Wh[-1]
        self._close("logit", gpu["z"].astype(F64), z64, np.abs(feats) @ np.abs(Wh[:-1]) + abs(Wh[-1]), K_GEMM)
        zg = gpu["z"].astype(F64)
        p = 1.0 / (1.0 + np.exp(-zg))
        eps = cfg.logloss_eps
        dz64 = (-lab / (p + eps) + (1 - lab) / (1 - p + eps)) / B * p * (1 - p)
        dzg = gpu["dz"].astype(F64)
        self._close("dz", dzg, dz64, np.abs(dz64) + 1.0 / B, 64)
        # ---- tower backward from the GPU's own gradients
        hoff = nF + E if fm else 0          # head weights of the last hidden layer (FM outputs first)
        dh_top = np.outer(dzg, Wh[hoff:-1]) * (X[L] > 0)
        G = [gpu["dh"][i].astype(F64) for i in range(L)]
        self._close("dh %d" % (L - 1), G[L - 1], dh_top, np.abs(dh_top), 4)
        for i in range(L - 1, 0, -1):
            dx = (G[i] @ Ws[i].T) * (X[i] > 0)
            self._close("dh %d" % (i - 1), G[i - 1], dx, np.abs(G[i]) @ np.abs(Ws[i]).T, K_GEMM)
        emb = slice(col, col + (S + M) * E)
        dx0 = G[0] @ Ws[0][emb].T
        dx0g = gpu["dx0"].astype(F64)
        self._close("dx0", dx0g, dx0, np.abs(G[0]) @ np.abs(Ws[0][emb]).T, K_GEMM)
        # ---- parameter gradients of the GPU's own terms (values and scales), per element on demand
        l2 = cfg.l2
        hw, hb = ("deep_fm_weight", "deep_fm_bias") if fm else ("deep_res", "deep_res_bias")
        Wfm = P[hw][:, 0].astype(F64)       # the head's L2 term (deepfm_pipeline.py:167, dnn_pipeline.py)
        self.dense = {hw: ((feats.T @ dzg + l2 * Wfm)[:, None],
                           (np.abs(feats).T @ np.abs(dzg) + l2 * np.abs(Wfm))[:, None]),
                      hb: (np.array([dzg.sum()]).reshape(P[hb].shape),
                           np.array([np.abs(dzg).sum()]).reshape(P[hb].shape))}
        for i in range(L):
            self.dense["deep_%d" % i] = (X[i].T @ G[i], np.abs(X[i]).T @ np.abs(G[i]))
            self.dense["deep_bias_%d" % i] = (G[i].sum(0, keepdims=True), np.abs(G[i]).sum(0, keepdims=True))
        dsec = np.outer(dzg, Wh[nF:nF + E]) if fm else None
        dfirst = np.outer(dzg, Wh[:nF]) if fm else None
        self.ref = dict(idx=idx, val=val, nI=nI, single=single, multi=multi, e=e, ea=ea, fs=fs, sa=sa, dsec=dsec,
                        dfirst=dfirst, dx0=dx0g, cnt=gpu.get("cnt_emb"), cnt1=gpu.get("cnt_first"))

    # ---- stage checks
    def _exact(self, what, got, want):
        bad = int((np.asarray(got) != np.asarray(want)).sum())
        self.stats[what] = {"n_bad": bad}
        if bad:
            self.fails.append("%s: %d elements not bit-exact" % (what, bad))

    def _count(self, what, err, bound):
        ratio = err / np.maximum(bound, 1e-300)
        bad = int((err > bound).sum())
        self.stats[what] = {"n_bad": bad, "max_err_over_bound": float(ratio.max()) if ratio.size else 0.0,
                            "max_err": float(err.max()) if err.size else 0.0}
        if bad:
            j = int(np.argmax(ratio))
            self.fails.append("%s: %d elements beyond the f32 bound (worst %g x the bound, err %g)" % (
                what, bad, ratio.reshape(-1)[j], err.reshape(-1)[j]))

    def _close(self, what, got, want, scale, K):
        self._count(what, np.abs(np.asarray(got, F64) - want), K * U32 * scale)

    # ---- per-element gradients
    def dense_elements(self, key, flat_idx):
        G, S = self.dense[key]
        return G.reshape(-1)[flat_idx], np.broadcast_to(S, G.shape).reshape(-1)[flat_idx]

    def table_elements(self, first, rows, dims):
        """(G, S) of table elements (rows[i], dims[i]) — first-order weights when `first` —
        summed over every reference of the batch to those rows, from the GPU's dx0, dz, FM sums
        and pooled counts (the terms of deepfm_pipeline.py:102-110,120 and the multi-hot
        div_no_nan gradient of deepfm_multi_cate.py:73-78)."""
        cfg, r = self.cfg, self.ref
        E, S = cfg.E, cfg.S
        B = self.B
        rows = np.asarray(rows, np.int64)
        uniq, inv = np.unique(rows, return_inverse=True)
        w = 1 if first else E
        acc = [np.zeros((len(uniq), w)), np.zeros((len(uniq), w))]

        def add(ids, contrib, scale):
            hit = np.isin(ids, uniq)
            if hit.any():
                k = np.searchsorted(uniq, ids[hit])
                np.add.at(acc[0], k, contrib[hit].reshape(len(k), w))
                np.add.at(acc[1], k, scale[hit].reshape(len(k), w))

        idx, val, nI = r["idx"], r["val"], r["nI"]
        if first:
            t = r["dfirst"][:, :nI] * val
            add(idx, t[..., None], np.abs(t)[..., None])
        elif not self.fm:                                          # DNN: the deep lookups only
            dx = r["dx0"][:, :S * E].reshape(B, S, E)
            add(r["single"], dx, np.abs(dx))
        else:
            de = r["dsec"][:, None, :] * (r["fs"][:, None, :] - r["e"][:, :nI]) * val[..., None]
            dea = np.abs(r["dsec"])[:, None, :] * (r["sa"][:, None, :] + r["ea"][:, :nI]) * np.abs(val)[..., None]
            add(idx, de, dea)
            dx = r["dx0"][:, :S * E].reshape(B, S, E)                 # deep lookups of the raw ids (:120)
            add(r["single"], dx, np.abs(dx))
        for m, (a, b_, *_) in enumerate(cfg.multi_ranges):
            ids = r["multi"][:, a:b_]
            Lm = b_ - a
            j = nI + m
            if first:
                n = r["cnt1"][:, m]
                g = np.where(n > 0, r["dfirst"][:, j] / np.where(n > 0, n, 1), 0)
                add(ids, np.repeat(g[:, None], Lm, 1)[..., None], np.repeat(np.abs(g)[:, None], Lm, 1)[..., None])
                continue
            n = r["cnt"][:, m][:, None]
            fm = r["dsec"] * (r["fs"] - r["e"][:, j]) if self.fm else 0
            fma = np.abs(r["dsec"]) * (r["sa"] + r["ea"][:, j]) if self.fm else 0
            dp = r["dx0"][:, (S + m) * E:(S + m + 1) * E]
            g = np.where(n > 0, (dp + fm) / np.where(n > 0, n, 1), 0)
            ga = np.where(n > 0, (np.abs(dp) + fma) / np.where(n > 0, n, 1), 0)
            add(ids, np.repeat(g[:, None, :], Lm, 1), np.repeat(ga[:, None, :], Lm, 1))
        pick = (lambda a: a[inv, 0]) if first else (lambda a: a[inv, np.asarray(dims, np.int64)])
        Gv, Sv = pick(acc[0]), pick(acc[1])
        zero = rows == 0                      # the concat zero row gets no gradient (:83-86)
        return np.where(zero, 0, Gv), np.where(zero, 0, Sv)


def gpu_gradient(m0, m1, beta1):
    """The gradient the GPU applied, from its ApplyAdam first moment (m1 = m0 + (g - m0)(1 - b1)),
    and the reconstruction's own rounding slack."""
    m0 = np.asarray(m0, F64)
    m1 = np.asarray(m1, F64)
    omb1 = float(np.float32(1) - np.float32(beta1))
    g = m0 + (m1 - m0) / omb1
    slack = 8 * U32 * (np.abs(m0) + np.abs(m1)) / omb1 + 4 * U32 * np.abs(g)
    return g, slack


def adam_consistent(g, slack, p0, m1, v0, v1, p1, alpha, beta2, eps):
    """Did (v, p) move by TF1 ApplyAdam on gradient g (within its reconstruction slack)?
    Returns a boolean array."""
    g, p0, m1, v0, v1, p1 = (np.asarray(a, F64) for a in (g, p0, m1, v0, v1, p1))
    omb2 = float(np.float32(1) - np.float32(beta2))
    v_exp = v0 + (g * g - v0) * omb2
    v_ok = np.abs(v1 - v_exp) <= 16 * U32 * (np.abs(v1) + np.abs(v0)) + 2 * omb2 * (np.abs(g) + slack) * slack
    upd = m1 * alpha / (np.sqrt(v1) + eps)
    p_ok = np.abs(p1 - (p0 - upd)) <= 4 * U32 * (np.abs(p1) + np.abs(p0)) + 8 * U32 * np.abs(upd)
    return v_ok & p_ok


def audit_elements(audit, key, idx, shape, m0, m1, v0, v1, p0, p1, alpha, beta1, beta2, eps, table_cols=None):
    """The gradient the GPU applied to elements idx of parameter `key` against the fp64 sum of
    its own terms, and its Adam step.  Returns (ok mask, stats dict)."""
    if key in (audit.tab, audit.t1):
        r_, c_ = np.unravel_index(idx, shape)
        G, S = audit.table_elements(key == audit.t1, r_, c_)
        K = K_TABLE
    else:
        G, S = audit.dense_elements(key, idx)
        K = K_WGRAD
    g, slack = gpu_gradient(m0, m1, beta1)
    err = np.abs(g - G)
    allowed = K * U32 * S + slack
    ok = (err <= allowed) & adam_consistent(g, slack, p0, m1, v0, v1, p1, alpha, beta2, eps)
    st = dict(n=len(idx), n_fail=int((~ok).sum()),
              min_g_over_S=float((np.abs(G) / np.maximum(S, 1e-300)).min()),
              max_err_over_uS=float((err / np.maximum(U32 * S, 1e-300)).max()),
              max_err_over_allowed=float((err / np.maximum(allowed, 1e-300)).max()))
    return ok, st, (g, G, S)
