"""C1 defaults (dnn_pipeline, hidden [512, 256, 128], B = 1,024): where the GPU's dense weight
gradients differ from the f32 oracle's, compare both with the fp64 product of the GPU's own
layer inputs and output gradients (x0 / h_l, dh_l).  Prints, per layer and step, how many
elements differ by more than 1e-5 and the worst |g - G64| / (u S) of the GPU's and the oracle's
gradients (u S: the sum's f32 scale).  Diagnostic only (GPU)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from deep_learning_amd.engine import CTREngine, ModelSpec  # noqa: E402
from oracle import ctr_ref as R  # noqa: E402
from tests import _fp64_audit as A  # noqa: E402
from tests.test_gpu_parity import _batches  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
kw = dict(C=13, V=0, S=26, E=8, cate_index_size=10000, hidden=[512, 256, 128])
cfg = R.make_cfg("dnn_pipeline", **kw)
P = R.init_params(cfg, np.random.default_rng(42))
eng = CTREngine(ModelSpec("dnn_pipeline", **kw), max_batch=B, init="none", adam="dense")
eng.load_params(P)
opt = R.AdamTF1(cfg, P)
sp = eng.spec
for step, b in enumerate(_batches("dnn_pipeline", kw, B, 3)):
    gp = eng.params()
    ds = eng.dense_state()
    Ps = {k: v.copy() for k, v in gp.items()}
    st = eng.adam_state()
    tk = sp.table_key
    opt.m = {k: (st["m"].reshape(P[k].shape) if k == tk else ds["m"][k]).copy() for k in gp}
    opt.v = {k: (st["v"].reshape(P[k].shape) if k == tk else ds["v"][k]).copy() for k in gp}
    fw = R.forward(cfg, Ps, b)
    G32, _ = R.backward(cfg, Ps, b, fw)
    eng.train_step(b, graph=False)
    torch.cuda.synchronize()
    ds1 = eng.dense_state()
    x0i = eng.x0[:B].cpu().numpy().astype(np.float64)
    X = np.zeros((B, sp.deep_in))
    X[:, sp.x0_ref_rows()] = x0i[:, :sp.deep_in]
    xs = [X] + [eng.h[l][:B, :sp.hidden[l]].cpu().numpy().astype(np.float64) for l in range(len(sp.hidden) - 1)]
    for l in range(len(sp.hidden)):
        k = "deep_%d" % l
        dh = eng.dh[l][:B, :sp.hidden[l]].cpu().numpy().astype(np.float64)
        G64 = xs[l].T @ dh
        S = np.abs(xs[l]).T @ np.abs(dh)
        g, slack = A.gpu_gradient(ds["m"][k], ds1["m"][k], cfg.beta1)
        us = A.U32 * np.maximum(S, 1e-30)
        rg = np.abs(g - G64) / us
        ro = np.abs(G32[k].astype(np.float64) - G64) / us
        # the oracle's own gradient vs its own fp64 (its xs / g)
        print("step %d %s: gpu |g-G64|/uS max %.1f p99 %.2f | oracle max %.1f p99 %.2f | |G64| med %.3g, S med %.3g"
              % (step, k, rg.max(), np.percentile(rg, 99), ro.max(), np.percentile(ro, 99),
                 np.median(np.abs(G64)), np.median(S)), flush=True)
        i = np.unravel_index(np.argmax(rg), rg.shape)
        print("    worst gpu elem", i, "g", g[i], "G64", G64[i], "oracle", G32[k][i], "S", S[i])
    opt_fw = R.train_step(cfg, Ps, opt, b)
