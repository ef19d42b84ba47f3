"""Parity at the BASELINE configurations' own sizes (SURVEY.md §8 config keys C2, C3, C5).

The per-model parity tests (test_gpu_parity.py) run at B <= 1536 and small tables; these
run the product path (row records, lazy-exact Adam, hipGraph replay) at full size against
the numpy oracle fed the same injected initial parameters and the same batches:

  C2  deepfm_pipeline, 26,000,013 x 16 table, MLP [400]x3, B = 65,536        (fp32, TOL 1e-5)
  C3  deepfm_multi_cate, 26 single + 6 multi-hot slots x 60, 26M rows, B = 65,536 (fp32)
  C5  wdl, bf16 deep tower, 26M rows + 26 wide ids, B = 65,536  (stated bf16 tolerance)

Each of 2 training steps is checked from identical state: before step t the oracle takes
the GPU's parameters and Adam moments (step 0: the injected parameters, zero moments), so
every comparison is one step of the reference math against one step of the HIP path:
every logit and the loss (fp32 tolerance 1e-5), then the updated table rows (values and both
Adam moments) of a sample of rows the batch touched plus a sample of rows it did not, and
every dense parameter.

Sign flips of near-zero gradient sums: the first Adam steps move an element by ~±alpha
whatever the gradient's size (m/sqrt(v) saturates), so an element whose summed gradient is
within fp32 rounding of 0 can move the other way when the summation order differs from
numpy's (a [400, 400] weight gradient sums 65,536 products per element).  Parameters are
therefore held to 1e-5 except for at most 1e-4 of the elements (at least one for small
arrays), which must still be within 2*FLIP*alpha (the size of such a flip).  Re-syncing before
each step keeps flips of one step from feeding the next step's gradients (a flipped hidden
weight moves the next step's embedding gradients by ~0.2 %, enough to flip ~1e-3 of the
near-zero ones: measured, and the reason the comparison is per step).
"""
import numpy as np
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

from deep_learning_amd.engine import CTREngine, ModelSpec  # noqa: E402
from deep_learning_amd.synthetic import make_batch  # noqa: E402
from oracle import ctr_ref as R  # noqa: E402

TOL = 1e-5
N_CATE = 26 * 1_000_000
B = 65536
HIDDEN = [400, 400, 400]


# |m / sqrt(v)| <= (1 - b1) / sqrt(1 - b2) for TF1 Adam's moments (b1^2 < b2), so one update
# moves an element by at most FLIP * alpha and a sign flip of it by twice that
FLIP = (1 - 0.9) / np.sqrt(1 - 0.999)


def _check_table(got, want, alpha, what, loose=False):
    d = np.abs(got.astype(np.float64) - want.astype(np.float64))
    bound = 2 * FLIP * alpha + TOL
    if loose:   # bf16 tower: every element within the size of a sign flip of its update
        assert d.max() <= bound, "%s: max error %g > 2*FLIP*alpha" % (what, d.max())
        return
    bad = d > TOL
    assert bad.sum() <= max(1, 1e-4 * d.size), "%s: %d of %d elements off by > %g (max %g)" % (what, bad.sum(), d.size, TOL, d.max())
    assert d.max() <= bound, "%s: max error %g > 2*FLIP*alpha" % (what, d.max())


def _sync_oracle(eng, cfg, opt):
    """Oracle state := the GPU's parameters and Adam moments (beta powers and step already
    advance in lockstep)."""
    P = eng.params()
    st = eng.adam_state()
    ds = eng.dense_state()
    spec = eng.spec
    tk = spec.table_key
    opt.m[tk], opt.v[tk] = st["m"], st["v"]
    if spec.fm:
        opt.m[spec.first_key], opt.v[spec.first_key] = st["m1"][:, None], st["v1"][:, None]
    for k in ds["m"]:
        opt.m[k] = ds["m"][k].reshape(opt.m[k].shape)
        opt.v[k] = ds["v"][k].reshape(opt.v[k].shape)
    return P


def _run(model, kw, batches, tower="f32", z_tol=TOL, loss_tol=TOL, auc_tol=None, seed=42):
    cfg = R.make_cfg(model, **kw)
    P = R.init_params(cfg, np.random.default_rng(seed))
    eng = CTREngine(ModelSpec(model, tower=tower, **kw), max_batch=B, init="none", adam="lazy")
    eng.load_params(P)
    opt = R.AdamTF1(cfg, P)
    spec = eng.spec
    tk = spec.table_key
    loose = tower == "bf16"
    rng = np.random.default_rng(1)
    for step, b in enumerate(batches):
        if step:
            P = _sync_oracle(eng, cfg, opt)
        alpha = float(opt.alpha())           # this step's alpha (before the oracle advances it)
        fw = R.train_step(cfg, P, opt, b)
        eng.train_step(b, graph=step >= 1)
        torch.cuda.synchronize()
        eng.check_error()
        z = eng.z[:B].cpu().numpy()
        np.testing.assert_allclose(z, fw["z"], atol=z_tol, rtol=0, err_msg="logits step %d" % step)
        assert abs(eng.loss() - fw["loss"]) < loss_tol, (eng.loss(), fw["loss"])
        if auc_tol is not None:
            s = eng.score[:B].cpu().numpy()
            assert abs(R.auc(b["label"], s) - R.auc(b["label"], fw["p"])) < auc_tol
        # the step's update: touched rows (FM rows id + offset, deep rows id, multi-hot ids) and others
        ids = b["cate_feats"].reshape(-1).astype(np.int64)
        touched = np.unique(np.concatenate([ids + spec.fm_cate_offset, ids]))
        touched = touched[touched < spec.n_rows]
        pick = np.concatenate([rng.choice(touched, 20000, replace=False), rng.integers(0, spec.n_rows, 20000)])
        got = eng.params()
        st = eng.adam_state()
        what = lambda k: "%s (step %d)" % (k, step)
        _check_table(got[tk][pick], P[tk][pick], alpha, what(tk), loose)
        if loose:   # moments: the bf16 gradients' relative error
            np.testing.assert_allclose(st["m"][pick], opt.m[tk][pick], rtol=0.1, atol=1e-7)
            np.testing.assert_allclose(st["v"][pick], opt.v[tk][pick], rtol=0.2, atol=1e-10)
        else:
            _check_table(st["m"][pick], opt.m[tk][pick], alpha, what("m"))
            _check_table(st["v"][pick], opt.v[tk][pick], alpha, what("v"))
        if spec.fm:
            fk = spec.first_key
            _check_table(got[fk][pick], P[fk][pick], alpha, what(fk))
        for k in P:
            if k in (tk, spec.first_key):
                continue
            _check_table(got[k], P[k], alpha, what(k), loose)
        del got, st
    return eng


def test_c2_deepfm_pipeline_full_size(hip_lib):
    kw = dict(C=13, V=0, S=26, E=16, cate_index_size=N_CATE, hidden=HIDDEN)
    bs = [make_batch(B, cate_index_size=N_CATE, seed=100 + i) for i in range(2)]
    _run("deepfm_pipeline", kw, bs)


def test_c3_deepfm_multi_cate_full_size(hip_lib):
    ranges = [[60 * i, 60 * (i + 1), "slot%d" % i] for i in range(6)]
    kw = dict(C=0, V=0, S=26, E=16, cate_index_size=N_CATE, hidden=HIDDEN, multi_ranges=ranges)
    bs = [make_batch(B, cont=0, cate_fields=26, cate_index_size=N_CATE, multi_slots=6, multi_width=60,
                     seed=200 + i, cate_only=True) for i in range(2)]
    _run("deepfm_multi_cate", kw, bs)


def test_c5_wdl_bf16_full_size(hip_lib):
    """C5 with the bf16 tower against the fp32 oracle, at the bf16 tolerance stated in
    test_gpu_parity.py::test_wdl_bf16_tower_tracks_oracle (logits 3e-2, loss 5e-3, AUC 2e-3)."""
    kw = dict(C=13, S=26, E=16, cate_index_size=N_CATE, hidden=HIDDEN, Fw=26)
    bs = [make_batch(B, cate_index_size=N_CATE, seed=300 + i, wide_fields=26) for i in range(2)]
    _run("wdl", kw, bs, tower="bf16", z_tol=3e-2, loss_tol=5e-3, auc_tol=2e-3)
