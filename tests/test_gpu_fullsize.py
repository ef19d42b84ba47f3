"""Parity at the BASELINE configurations' own sizes (SURVEY.md §8 config keys C2, C3, C5).

The per-model parity tests (test_gpu_parity.py) run at B <= 1536 and small tables; these
run the product path (row records, lazy-exact Adam, hipGraph replay) at full size against
the numpy oracle fed the same injected initial parameters and the same batches:

  C2  deepfm_pipeline, 26,000,013 x 16 table, MLP [400]x3, B = 65,536        (fp32, TOL 1e-5)
  C3  deepfm_multi_cate, 26 single + 6 multi-hot slots x 60, 26M rows, B = 65,536 (fp32)
  C5  wdl, bf16 deep tower, 26M rows + 26 wide ids, B = 65,536  (stated bf16 tolerance)

Checked after each of 2 training steps: every logit, the loss; after the last step every
dense parameter, and the table rows (values and both Adam moments) of a sample of rows the
batches touched plus a sample of rows they did not (those still move: dense Adam).

Sign flips of near-zero gradient sums: the first Adam steps move an element by ~±alpha
whatever the gradient's size (m/sqrt(v) saturates), so an element whose summed gradient is
within fp32 rounding of 0 can move the other way when the summation order differs from
numpy's.  Table elements are therefore held to 1e-5 except for at most 1e-4 of them, which
must still be within 2*alpha (the size of such a flip); the logits see these at 1e-5 too.
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


def _check_table(got, want, alpha_sum, what, loose=False):
    d = np.abs(got.astype(np.float64) - want.astype(np.float64))
    if loose:   # bf16 tower: every element within the size of a sign flip of its update
        assert d.max() <= 2 * alpha_sum + TOL, "%s: max error %g > 2*alpha" % (what, d.max())
        return
    bad = d > TOL
    assert bad.mean() <= 1e-4, "%s: %d of %d elements off by > %g (max %g)" % (what, bad.sum(), d.size, TOL, d.max())
    assert d.max() <= 2 * alpha_sum + TOL, "%s: max error %g > 2*alpha" % (what, d.max())


def _run(model, kw, batches, tower="f32", z_tol=TOL, loss_tol=TOL, auc_tol=None, seed=42):
    cfg = R.make_cfg(model, **kw)
    P = R.init_params(cfg, np.random.default_rng(seed))
    eng = CTREngine(ModelSpec(model, tower=tower, **kw), max_batch=B, init="none", adam="lazy")
    eng.load_params(P)
    opt = R.AdamTF1(cfg, P)
    alphas = 0.0
    for step, b in enumerate(batches):
        alphas += float(opt.alpha())        # this step's alpha (before the oracle advances it)
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
    got = eng.params()
    st = eng.adam_state()
    spec = eng.spec
    # touched rows (FM rows id + C, deep rows id; multi-hot ids) and untouched ones
    rows = set()
    for b in batches:
        ids = b["cate_feats"].reshape(-1)
        rows.update(np.unique(ids + spec.fm_cate_offset).tolist()[:200000])
        rows.update(np.unique(ids).tolist()[:200000])
    rng = np.random.default_rng(1)
    touched = np.array(sorted(rows), np.int64)
    touched = touched[touched < spec.n_rows]
    pick = np.concatenate([rng.choice(touched, 20000, replace=False),
                           rng.integers(0, spec.n_rows, 20000)])
    tk = spec.table_key
    loose = tower == "bf16"
    _check_table(got[tk][pick], P[tk][pick], alphas, tk, loose)
    if loose:   # moments: the bf16 gradients' relative error
        np.testing.assert_allclose(st["m"][pick], opt.m[tk][pick], rtol=0.1, atol=1e-7)
        np.testing.assert_allclose(st["v"][pick], opt.v[tk][pick], rtol=0.2, atol=1e-10)
    else:
        _check_table(st["m"][pick], opt.m[tk][pick], alphas, "m")
        _check_table(st["v"][pick], opt.v[tk][pick], alphas, "v")
    if spec.fm:
        fk = spec.first_key
        _check_table(got[fk][pick], P[fk][pick], alphas, fk)
    for k in P:
        if k in (tk, spec.first_key):
            continue
        _check_table(got[k], P[k], alphas, k, loose)
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
