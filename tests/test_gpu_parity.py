"""End-to-end parity of the HIP training step against the CPU oracle.

Identical injected initial parameters, identical unshuffled batches; after each
of several TF1-Adam steps the logits must agree within 1e-5 (north_star
tolerance, fp32) and the parameters within 1e-5; the loss within 1e-5."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from deep_learning_amd import _lib  # noqa: E402
from deep_learning_amd.engine import CTREngine, ModelSpec  # noqa: E402
from deep_learning_amd.synthetic import make_batch  # noqa: E402
from oracle import ctr_ref as R  # noqa: E402

TOL = 1e-5

CASES = {
    "deepfm_pipeline": dict(C=13, V=0, S=26, E=16, cate_index_size=20000, hidden=[64, 48, 32]),
    "deepfm_pipeline_e8_vec": dict(C=13, V=5, S=26, E=8, cate_index_size=3000, hidden=[40, 24]),
    "dnn_pipeline": dict(C=13, V=3, S=26, E=8, cate_index_size=10000, hidden=[64, 32, 16]),
    "deepfm_multi_cate": dict(V=4, S=8, E=16, cate_index_size=6000, hidden=[48, 32],
                              multi_ranges=[[0, 30, "a"], [30, 50, "b"]]),
    "wdl": dict(C=13, S=26, E=16, cate_index_size=8000, hidden=[64, 32], Fw=26),
    "deepfm_cate": dict(V=4, S=26, E=16, cate_index_size=9000, hidden=[48, 32]),
    "deepfm_multi": dict(C=13, V=3, S=10, E=16, cate_index_size=7000, hidden=[48, 32],
                         multi_ranges=[[0, 24, "a"], [24, 40, "b"], [40, 41, "c"]]),
    "dnn_cate": dict(V=3, S=26, E=8, cate_index_size=5000, hidden=[40, 24]),
    "dnn_multi": dict(C=13, V=2, S=12, E=16, cate_index_size=6000, hidden=[48, 32],
                      multi_ranges=[[0, 30, "a"], [30, 50, "b"]]),
    "dnn_multi_cate": dict(V=4, S=8, E=8, cate_index_size=6000, hidden=[40, 24],
                           multi_ranges=[[0, 20, "a"], [20, 64, "b"]]),
    "deepfm": dict(C=13, V=3, S=26, E=8, cate_index_size=5000, hidden=[48, 32]),
    "dnn": dict(C=16, S=26, E=16, cate_index_size=6000, hidden=[64, 32], l2=1e-3),
}


def _stat(name, **kw):
    """DLAMD_TEST_STATS=<dir>: measured maxima appended as json lines (as test_gpu_fullsize.py)."""
    import json
    import os
    d = os.environ.get("DLAMD_TEST_STATS")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "parity_stats.jsonl"), "a") as f:
            f.write(json.dumps(dict(test=name, **{k: float(v) for k, v in kw.items()})) + "\n")


def _model(name):
    return name.split("_e8")[0]


def _batches(name, kw, B, n, seed=11):
    out = []
    for i in range(n):
        if "multi_ranges" in kw:
            C = kw.get("C", 0)
            b = make_batch(B, cont=C, vector=kw["V"], cate_fields=kw["S"], cate_index_size=kw["cate_index_size"],
                           seed=seed + i, cate_only=C == 0)
            rng = np.random.default_rng(seed + 100 + i)
            W = sum(e - s for s, e, _ in kw["multi_ranges"])
            multi = rng.integers(1, kw["cate_index_size"], size=(B, W))
            multi[rng.random((B, W)) < 0.5] = 0
            b["cate_feats"] = np.concatenate([b["cate_feats"], multi], 1)
        else:
            C = kw.get("C", 0)
            b = make_batch(B, cont=C, vector=kw.get("V", 0), cate_fields=kw["S"],
                           cate_index_size=kw["cate_index_size"], seed=seed + i, wide_fields=kw.get("Fw", 0),
                           cate_only=C == 0)
            b["cate_feats"][0, :4] = [0, 1, 5, 12]   # padding id + ids that alias cont rows
            b["cate_feats"][1, :2] = [27, 30]        # deepfm.py: ids aliasing its cont rows (S + j)
        out.append(b)
    return out


@pytest.mark.parametrize("bwd", ["atomic", "sorted", "lazy"])
@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("B", [256, 1536])
def test_train_steps_match_oracle(hip_lib, name, B, bwd):
    kw = CASES[name]
    model = _model(name)
    cfg = R.make_cfg(model, **kw)
    spec = ModelSpec(model, **kw)
    P = R.init_params(cfg, np.random.default_rng(42))
    if bwd == "lazy":
        eng = CTREngine(spec, max_batch=B, init="none", adam="lazy")
    else:
        eng = CTREngine(spec, max_batch=B, init="none", bwd=bwd)
    eng.load_params(P)
    opt = R.AdamTF1(cfg, P)
    for step, b in enumerate(_batches(name, kw, B, 4)):
        fw = R.train_step(cfg, P, opt, b)
        eng.train_step(b, graph=(step >= 2))
        torch.cuda.synchronize()
        z = eng.z[:B].cpu().numpy()
        np.testing.assert_allclose(z, fw["z"], atol=TOL, rtol=0, err_msg="logits step %d" % step)
        assert abs(eng.loss() - fw["loss"]) < TOL
    got = eng.params()
    for k in P:
        np.testing.assert_allclose(got[k], P[k], atol=TOL, rtol=0, err_msg=k)


@pytest.mark.parametrize("B", [256, 1024])
@pytest.mark.parametrize("adam", ["dense", "lazy"])
def test_dnn_pipeline_c1_defaults_same_state(hip_lib, B, adam):
    """BASELINE config C1 at the reference's own defaults: dnn_pipeline, 13 dense + 26 cate over
    a 10k vocab, embedding 8, hidden [512, 256, 128] (local_run.py:28-35), batch 256 (configs[0])
    and 1,024 (local_run.py:35).  Every step is checked from the GPU's own state (the full-size
    tests' same-state track): the oracle takes the GPU's exported parameters and Adam moments,
    then the f32 TF1 step — every logit and the loss within 1e-5; every stage of the GPU's step
    against fp64 of its own inputs (tests/_fp64_audit.py); every parameter element within 1e-5 or
    else audited in fp64 (the gradient the GPU applied, from its moments, against the fp64 sum of
    its own terms within that sum's f32 bound, and TF1 Adam on it).  At these widths the f32
    oracle's own ReLU decisions near zero differ from the GPU's for a few units a step, and each
    such unit moves a whole column of W_0's gradient: a count bar on the elements off by more than
    1e-5 would measure the oracle's conditioning, not the GPU's step."""
    from tests import _fp64_audit as A
    kw = dict(C=13, V=0, S=26, E=8, cate_index_size=10000, hidden=[512, 256, 128])
    cfg = R.make_cfg("dnn_pipeline", **kw)
    P = R.init_params(cfg, np.random.default_rng(42))
    eng = CTREngine(ModelSpec("dnn_pipeline", **kw), max_batch=B, init="none", adam=adam)
    eng.load_params(P)
    opt = R.AdamTF1(cfg, P)
    tk = eng.spec.table_key
    flip = (1 - 0.9) / np.sqrt(1 - 0.999)
    worst, audited = 0.0, 0
    fails = []
    for step, b in enumerate(_batches("dnn_pipeline", kw, B, 6)):
        # the oracle from the GPU's state: parameters and both moments
        gp = eng.params()
        ds, st = eng.dense_state(), eng.adam_state()
        m0 = {k: (st["m"].reshape(P[k].shape) if k == tk else ds["m"][k]) for k in gp}
        v0 = {k: (st["v"].reshape(P[k].shape) if k == tk else ds["v"][k]) for k in gp}
        Ps = {k: v.copy() for k, v in gp.items()}
        opt.m = {k: v.copy() for k, v in m0.items()}
        opt.v = {k: v.copy() for k, v in v0.items()}
        alpha = float(opt.alpha())
        fw = R.train_step(cfg, Ps, opt, b)
        eng.train_step(b, graph=(step >= 2))
        torch.cuda.synchronize()
        z = eng.z[:B].cpu().numpy()
        worst = max(worst, float(np.abs(z - fw["z"]).max()))
        np.testing.assert_allclose(z, fw["z"], atol=TOL, rtol=0, err_msg="logits step %d" % step)
        assert abs(eng.loss() - fw["loss"]) < TOL
        audit = A.StepAudit(cfg, gp, b, A.read_gpu(eng, B))
        fails += ["step %d: %s" % (step, f) for f in audit.fails]
        got = eng.params()
        ds1, st1 = eng.dense_state(), eng.adam_state()
        m1 = {k: (st1["m"].reshape(P[k].shape) if k == tk else ds1["m"][k]) for k in gp}
        v1 = {k: (st1["v"].reshape(P[k].shape) if k == tk else ds1["v"][k]) for k in gp}
        for k in Ps:
            d = np.abs(got[k].astype(np.float64) - Ps[k])
            assert d.max() <= 2 * flip * alpha + TOL, (k, step, float(d.max()))
            idx = np.flatnonzero(d.reshape(-1) > TOL)
            if not len(idx):
                continue
            fl = lambda a: np.asarray(a).reshape(-1)[idx]
            ok, st_, (g, G64, S) = A.audit_elements(audit, k, idx, P[k].shape, fl(m0[k]), fl(m1[k]), fl(v0[k]),
                                                    fl(v1[k]), fl(gp[k]), fl(got[k]), alpha, cfg.beta1, cfg.beta2,
                                                    cfg.eps)
            audited = max(audited, len(idx))
            _stat("c1 defaults B=%d %s step %d %s audited" % (B, adam, step, k), **st_)
            if not ok.all():
                j = int(np.flatnonzero(~ok)[0])
                fails.append("step %d %s: %d of %d audited elements fail (e.g. flat %d: GPU gradient %r, fp64 %r, "
                             "scale %r)" % (step, k, (~ok).sum(), len(idx), idx[j], g[j], G64[j], S[j]))
    assert not fails, fails[:8]
    _stat("c1 defaults B=%d %s" % (B, adam), z_max_err=worst, audited_max=audited)


def test_graph_replay_equals_eager(hip_lib):
    kw = CASES["deepfm_pipeline"]
    spec = ModelSpec("deepfm_pipeline", **kw)
    bs = _batches("deepfm_pipeline", kw, 512, 3)
    res = []
    for graph in (False, True):
        eng = CTREngine(spec, max_batch=512, seed=5)
        for b in bs:
            eng.train_step(b, graph=graph)
        torch.cuda.synchronize()
        res.append(eng.z[:512].cpu().numpy())
    np.testing.assert_allclose(res[0], res[1], atol=1e-6)


@pytest.mark.parametrize("name,tower", [("deepfm_pipeline", "f32"), ("wdl", "bf16"), ("dnn_pipeline", "f32")])
def test_fused_dense_adam_bit_identical(hip_lib, name, tower, monkeypatch):
    """The tower's dense Adams as one launch after the backward's GEMMs (dl_adam_dense_layers)
    against one launch per layer after its input gradient: the same per-element operations, so
    parameters, moments and the GEMM operand copies the next steps read are bit-identical."""
    kw = CASES[name]
    spec = ModelSpec(name, tower=tower, **kw)
    bs = _batches(name, kw, 512, 4)
    res = []
    for fused in ("0", "1"):
        monkeypatch.setenv("DLAMD_ADAM_FUSED", fused)
        eng = CTREngine(spec, max_batch=512, seed=5, adam="lazy")
        assert eng._adam_fused() == (fused == "1")
        for i, b in enumerate(bs):
            eng.train_step(b, graph=i >= 1)
        torch.cuda.synchronize()
        res.append((eng.z[:512].cpu().numpy(), eng.params(), eng.dense_state()))
    (z0, p0, d0), (z1, p1, d1) = res
    assert np.array_equal(z0, z1)
    for k in p0:
        assert np.array_equal(p0[k], p1[k]), k
    for k in d0["m"]:
        assert np.array_equal(d0["m"][k], d1["m"][k]) and np.array_equal(d0["v"][k], d1["v"][k]), k


def test_opt_restore_mid_process_keeps_status_ring(hip_lib):
    """A checkpoint's optimizer block restored into an engine that has already trained
    (_ctr_model.py _restore -> set_opt): the status ring's step sequence stays the device's, so
    the next steps report on time — no 10-s resynchronisation stall — and train exactly as an
    engine given the same state from the start."""
    import time
    kw = CASES["deepfm_pipeline"]
    spec = ModelSpec("deepfm_pipeline", **kw)
    bs = _batches("deepfm_pipeline", kw, 512, 8)
    eng = CTREngine(spec, max_batch=512, seed=5, adam="lazy")
    assert eng._ring is not None
    for b in bs[:3]:
        eng.train_step(b, graph=True)
    torch.cuda.synchronize()
    saved = eng.opt.clone()
    for b in bs[3:5]:
        eng.train_step(b, graph=True)
    eng.set_opt(saved)
    t0 = time.perf_counter()
    for b in bs[5:]:
        eng.train_step(b, graph=True)
    torch.cuda.synchronize()
    eng.check_error()
    assert time.perf_counter() - t0 < 5.0
    assert eng.host_wait < 5.0
    assert np.isfinite(eng.z[:512].cpu().numpy()).all()


@pytest.mark.parametrize("stash", [False, True])
# (multi-hot models are left out: the dense engine adds pooled gradients with atomics, whose
# order varies, while the record path sums every row's references in a fixed order)
@pytest.mark.parametrize("name", ["deepfm_pipeline", "dnn_pipeline", "wdl", "deepfm_cate", "dnn_cate", "deepfm",
                                  "dnn"])
def test_lazy_adam_bit_identical_to_dense(hip_lib, name, stash):
    """Row records + lazy catch-up (rec.hip) against the dense sweep with the same
    (sorted, deterministic) gradients: parameters, Adam moments, logits and
    predictions must be bit-identical.  A large table, a small batch and an 8-entry
    alpha ring make rows lag many steps and force periodic flushes.  (wdl included: its
    wide-weight gradient is an integer fixed-point segment sum, order-independent, and its
    wide weights are lazy records too (wide.hip) against the dense L2 sweep — wide ids
    aliasing the deep-output rows included; the loss's L2 term within 1e-6 relative.)"""
    kw = dict(CASES[name], cate_index_size=50000)
    same = np.testing.assert_array_equal
    model = _model(name)
    spec = ModelSpec(model, **kw)
    dense = CTREngine(spec, max_batch=128, seed=3, bwd="sorted")
    lazy = CTREngine(spec, max_batch=128, seed=3, adam="lazy", hist_len=8, rec_stash=stash)
    np.testing.assert_array_equal(lazy.params()[spec.table_key], dense.params()[spec.table_key])
    bs = _batches(name, kw, 128, 21, seed=7)
    if "wide_feats" in bs[0]:   # wide ids on the deep-output rows Fw .. Fw+H (wdl.py:225-228 aliasing)
        Fw, H = kw["Fw"], kw["hidden"][-1]
        for j, b in enumerate(bs):
            b["wide_feats"][j % 7, :3] = [Fw + j % H, Fw + H - 1, Fw]
    assert lazy.wide_lazy == (name == "wdl")
    for i, b in enumerate(bs):
        dense.train_step(b, graph=i >= 3)
        lazy.train_step(b, graph=i >= 3)
        torch.cuda.synchronize()
        same(lazy.z[:128].cpu().numpy(), dense.z[:128].cpu().numpy(), err_msg="logits step %d" % i)
        if i == 10:
            same(lazy.predict(bs[0]), dense.predict(bs[0]))
    np.testing.assert_allclose(lazy.loss(), dense.loss(), rtol=1e-6)
    pd, pl = dense.params(), lazy.params()
    for k in pd:
        same(pl[k], pd[k], err_msg=k)
    sd, sl = dense.adam_state(), lazy.adam_state()
    for k in sd:
        same(sl[k], sd[k], err_msg=k)
    dd, dl = dense.dense_state(), lazy.dense_state()
    for mv in ("m", "v"):
        for k in dd[mv]:
            same(dl[mv][k], dd[mv][k], err_msg="%s %s" % (mv, k))


@pytest.mark.parametrize("name", ["deepfm_pipeline", "dnn_pipeline", "wdl"])
def test_record_forward_bit_identical_to_gather(hip_lib, name):
    """dl_embed_fwd_rec (cate rows read and caught up straight from the records) against
    the gather + indexed forward pair: logits every step, predictions and all parameters
    bit-identical (8-entry alpha ring: lagging rows and flushes included)."""
    kw = dict(CASES[name], cate_index_size=50000)
    spec = ModelSpec(_model(name), **kw)
    a = CTREngine(spec, max_batch=128, seed=3, adam="lazy", hist_len=8, fwd_rec=True, rec_stash=False)
    b = CTREngine(spec, max_batch=128, seed=3, adam="lazy", hist_len=8, fwd_rec=False)
    assert a.fwd_rec and not b.fwd_rec
    bs = _batches(name, kw, 128, 15, seed=11)
    for i, bt in enumerate(bs):
        a.train_step(bt, graph=i >= 2)
        b.train_step(bt, graph=i >= 2)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(a.z[:128].cpu().numpy(), b.z[:128].cpu().numpy(), err_msg="step %d" % i)
        np.testing.assert_array_equal(a.fm_out[:128].cpu().numpy(), b.fm_out[:128].cpu().numpy())
    np.testing.assert_array_equal(a.predict(bs[0]), b.predict(bs[0]))
    pa, pb = a.params(), b.params()
    for k in pa:
        np.testing.assert_array_equal(pa[k], pb[k], err_msg=k)


@pytest.mark.parametrize("name", ["deepfm_pipeline", "dnn_pipeline", "wdl"])
def test_flat_lookup_after_flush_bit_identical(hip_lib, name):
    """predict() on a flushed table reads each reference's record first line only
    (dl_embed_fwd_rec_flat) — the same scores and forward outputs as the gather + indexed
    forward at lag 0 on the same table; after a further training step predict() leaves the flat
    path; and the flat lookup on a table that is not caught up raises (DL_STATUS_LAG) instead of
    reading stale rows."""
    kw = dict(CASES[name], cate_index_size=50000)
    spec = ModelSpec(_model(name), **kw)
    e = CTREngine(spec, max_batch=128, seed=3, adam="lazy", hist_len=8)
    bs = _batches(name, kw, 128, 6, seed=13)
    for i, bt in enumerate(bs[:5]):
        e.train_step(bt, graph=i >= 2)
    ref = e.predict(bs[5], logits=True)           # gather + indexed forward, lag 0
    ref_fm = e.fm_out[:128].cpu().numpy().copy()
    e.flush()
    assert e.since_flush == 0
    got = e.predict(bs[5], logits=True)           # flat lookup on the flushed planes
    assert e.planes_step == e.steps
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(e.fm_out[:128].cpu().numpy(), ref_fm)
    e.flat_planes = False                         # the record form of the flat lookup
    e.planes_step = -1
    np.testing.assert_array_equal(e.predict(bs[5], logits=True), ref)
    np.testing.assert_array_equal(e.fm_out[:128].cpu().numpy(), ref_fm)
    e.flat_planes = True
    e.train_step(bs[0])
    assert e.since_flush == 1
    np.testing.assert_array_equal(e.predict(bs[5], logits=True), e.predict(bs[5], logits=True))
    # the record form of the flat lookup (without planes) forced onto a table whose touched
    # rows lag: the status word, then the host raise
    e.train_step(bs[1])
    e.since_flush = 0
    e.flat_planes = False
    with pytest.raises(_lib.DLError, match="lagged"):
        e.predict(bs[5])


@pytest.mark.parametrize("name,kw", [
    ("deepfm_pipeline", dict(CASES["deepfm_pipeline"], cate_index_size=50000)),
    ("dnn_pipeline", dict(C=13, V=3, S=24, E=8, cate_index_size=10000, hidden=[64, 32])),
    ("deepfm_pipeline", dict(C=13, V=0, S=6, E=16, cate_index_size=7000, hidden=[48, 32]))])
def test_fused_gather_predict_bit_identical(hip_lib, name, kw, monkeypatch):
    """predict() on current planes with the deep lookup inside the first tower layer against
    the lookup writing x0 followed by the plain GEMM (DLAMD_FUSED_GATHER=0): logits, FM outputs
    and the first layer's activations bit-identical, over a batch that is not a multiple of the
    256-row block with padding ids (the zero row) in every field; and the engine really took
    the fused path.  The table form (DLAMD_GATHER_TAB=1: dl_embed_fwd_gtab +
    dl_gemm_s3_nt_gather_tab; the offset table the lookup wrote equals the ids' rows times the
    plane stride) and the id form (the default, dl_gemm_s3_nt_gather) both; x0's deep columns
    are neither written nor read by either — they keep a NaN sentinel."""
    monkeypatch.setenv("DLAMD_GATHER_TAB", "1")
    spec = ModelSpec(name, **kw)
    e = CTREngine(spec, max_batch=300, seed=3, adam="lazy", hist_len=8)
    bs = _batches(name, kw, 300, 5, seed=29)
    for i, bt in enumerate(bs[:4]):
        e.train_step(bt, graph=i >= 2)
    b = dict(bs[4])
    cate = np.array(b["cate_feats"], copy=True)
    cate[::9, :] = 0                         # padding ids: the zero row
    b["cate_feats"] = cate
    e.flush(planes=True)
    assert e.fused_gather_l0()
    assert e.fused_gather_tab(300)
    calls = []
    orig = e._c
    monkeypatch.setattr(e, "_c", lambda tag, fn, *a: (calls.append(fn), orig(tag, fn, *a))[1])
    D = spec.S * spec.E
    e.x0[:, :D] = float("nan")
    got = e.predict(b, logits=True)
    got_fm = e.fm_out[:300].cpu().numpy().copy()
    got_h = e.h[0][:300].cpu().numpy().copy()
    assert "dl_gemm_s3_nt_gather_tab" in calls and "dl_embed_fwd_gtab" in calls
    assert torch.isnan(e.x0[:, :D]).all()   # x0's deep columns not written (nor read: finite outputs)
    S, E = spec.S, spec.E
    ids = e.in_cate[:300, :S].cpu().numpy().astype(np.int64)
    FL = e._flat_layout(300)
    rows = ids + FL.deep_cate_offset
    ok = (rows >= (1 if FL.zero_row0 else 0)) & (rows < FL.n_rows)
    want = np.where(ok, rows * e.p_plane.shape[1] * 4, 0xFFFFFF00).astype(np.uint32)
    gt = e.gtab.cpu().numpy().view(np.uint32).reshape(-1, S, 272)
    m = np.arange(300)
    np.testing.assert_array_equal(gt[m // 256, :, m % 256], want)
    calls.clear()
    monkeypatch.setenv("DLAMD_GATHER_TAB", "0")
    ref_id = e.predict(b, logits=True)
    assert "dl_gemm_s3_nt_gather" in calls and "dl_gemm_s3_nt_gather_tab" not in calls
    assert torch.isnan(e.x0[:, :D]).all()
    np.testing.assert_array_equal(got, ref_id)
    np.testing.assert_array_equal(got_h, e.h[0][:300].cpu().numpy())
    assert np.isfinite(got).all()
    monkeypatch.setenv("DLAMD_FUSED_GATHER", "0")
    calls.clear()
    ref = e.predict(b, logits=True)
    assert "dl_gemm_s3_nt_gather" not in calls and "dl_gemm_s3_nt_gather_tab" not in calls
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(got_fm, e.fm_out[:300].cpu().numpy())
    np.testing.assert_array_equal(got_h, e.h[0][:300].cpu().numpy())


@pytest.mark.parametrize("name", ["deepfm_pipeline", "dnn_pipeline"])
def test_lookup_without_deep_columns(hip_lib, name):
    """The FM-only form of the plane lookup (x0_cat_col = -1, what the fused predict runs):
    FM outputs and sums bit-identical to the full lookup's, x0's cont / vector columns the same,
    its deep columns never written (a sentinel survives), and a bad id still reported."""
    kw = dict(CASES[name], cate_index_size=30000)
    e = CTREngine(ModelSpec(_model(name), **kw), max_batch=200, seed=5, adam="lazy", hist_len=8)
    bs = _batches(name, kw, 200, 3, seed=41)
    for bt in bs[:2]:
        e.train_step(bt)
    e.flush(planes=True)
    B = 200
    e.stage(bs[2])
    s = _lib.stream_handle()
    D = e.spec.S * e.spec.E
    e.x0.fill_(7.0)
    e.plane_lookup(B, e.x0, s, deep=True)
    full_x0 = e.x0[:B].clone()
    full_fm = (e.fm_out[:B].clone(), e.fm_sum[:B].clone()) if e.spec.fm else None
    e.x0.fill_(7.0)
    e.fm_out.fill_(3.0)
    e.plane_lookup(B, e.x0, s, deep=False)
    torch.cuda.synchronize()
    e.check_error()
    assert (e.x0[:B, e.cat_col:e.cat_col + D] == 7.0).all()
    assert torch.equal(e.x0[:B, D:], full_x0[:, D:])
    if full_fm is not None:
        nf = e.spec.fm_cols   # the pad columns past fm_cols are not outputs
        assert torch.equal(e.fm_out[:B, :nf], full_fm[0][:, :nf])
        assert torch.equal(e.fm_sum[:B], full_fm[1])
    bad = dict(bs[2])
    cate = np.array(bad["cate_feats"], copy=True)
    cate[3, 2] = kw["cate_index_size"] * 10          # outside the table
    bad["cate_feats"] = cate
    e.stage(bad)
    e.plane_lookup(B, e.x0, s, deep=False)
    with pytest.raises(_lib.DLError):
        e.check_error()


@pytest.mark.parametrize("name,kw", [
    ("deepfm_pipeline", dict(CASES["deepfm_pipeline"], cate_index_size=40000)),
    ("deepfm_multi_cate", dict(V=4, S=8, E=16, cate_index_size=6000, hidden=[48, 32],
                               multi_ranges=[[0, 30, "a"], [30, 50, "b"]])),
    ("dnn", dict(CASES["dnn"], cate_index_size=9000))])
def test_fused_gather_training_bit_identical(hip_lib, name, kw, monkeypatch):
    """The lazy training forward with the deep rows gathered by the first s3 layer
    (dl_gemm_s3_nt_gather_rows, the default where it applies: the lookup writes only the FM side
    and x0's cont / pooled columns, the layer writes x0's deep columns for dw_l0) against the
    indexed lookup writing them (DLAMD_FUSED_GATHER=0): the same losses, logits and tables, bit
    for bit, over graph-captured steps with a prefetched next batch."""
    bs = _batches(name, kw, 300, 6, seed=53)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("DLAMD_FUSED_GATHER", mode)
        e = CTREngine(ModelSpec(_model(name), **kw), max_batch=300, seed=9, adam="lazy", hist_len=8)
        assert e.fused_gather_rows() == (mode == "1")
        losses = []
        for i, bt in enumerate(bs[:5]):
            e.train_step(bt, graph=i >= 1, next_batch=bs[i + 1] if i + 1 < 5 else None)
            losses.append(e.loss())
        z = e.predict(bs[5], logits=True)
        out[mode] = (losses, z, e.params())
        del e
    assert out["1"][0] == out["0"][0]
    np.testing.assert_array_equal(out["1"][1], out["0"][1])
    for k in out["0"][2]:
        np.testing.assert_array_equal(out["1"][2][k], out["0"][2][k], err_msg=k)


def test_lazy_multi_hot_tracks_oracle(hip_lib):
    """Multi-hot pooling on row records (deepfm_multi_cate): pooled rows come from the
    caught-up records through the batch index, their gradients join each row's ordered
    segment sum.  A large table and an 8-entry alpha ring force lagging rows and flushes;
    the dense path's pooled scatter is atomic, so the bar is the oracle at TOL."""
    name = "deepfm_multi_cate"
    kw = dict(CASES[name], cate_index_size=40000)
    cfg = R.make_cfg(name, **kw)
    spec = ModelSpec(name, **kw)
    P = R.init_params(cfg, np.random.default_rng(5))
    eng = CTREngine(spec, max_batch=192, init="none", adam="lazy", hist_len=8)
    eng.load_params(P)
    opt = R.AdamTF1(cfg, P)
    bs = _batches(name, kw, 192, 15, seed=21)
    for step, b in enumerate(bs):
        fw = R.train_step(cfg, P, opt, b)
        eng.train_step(b, graph=(step >= 2))
        torch.cuda.synchronize()
        np.testing.assert_allclose(eng.z[:192].cpu().numpy(), fw["z"], atol=TOL, rtol=0,
                                   err_msg="logits step %d" % step)
        if step == 7:
            np.testing.assert_allclose(eng.predict(bs[0]), R.forward(cfg, P, bs[0])["p"], atol=TOL, rtol=0)
    got = eng.params()
    for k in P:
        np.testing.assert_allclose(got[k], P[k], atol=TOL, rtol=0, err_msg=k)


@pytest.mark.parametrize("adam", ["dense", "lazy"])
def test_wdl_bf16_tower_tracks_oracle(hip_lib, adam):
    """Config C5: the deep tower on bf16 MFMA (fp32 master weights, fp32 wide cross logit).
    Stated bf16 tolerance: logits within 3e-2 absolute of the fp32 oracle over
    4 steps (the bf16 operand rounding of a small, fast-moving tower), loss within 5e-3, and the
    AUC of the scores within 1e-4 (north star).  The measured maxima are recorded
    (DLAMD_TEST_STATS)."""
    kw = CASES["wdl"]
    cfg = R.make_cfg("wdl", **kw)
    P = R.init_params(cfg, np.random.default_rng(42))
    eng = CTREngine(ModelSpec("wdl", tower="bf16", **kw), max_batch=1536, init="none", adam=adam)
    eng.load_params(P)
    opt = R.AdamTF1(cfg, P)
    worst, worst_loss, worst_auc = 0.0, 0.0, 0.0
    for step, b in enumerate(_batches("wdl", kw, 1536, 4)):
        fw = R.train_step(cfg, P, opt, b)
        eng.train_step(b, graph=(step >= 2))
        torch.cuda.synchronize()
        z = eng.z[:1536].cpu().numpy()
        worst = max(worst, float(np.abs(z - fw["z"]).max()))
        worst_loss = max(worst_loss, abs(eng.loss() - fw["loss"]))
        worst_auc = max(worst_auc, abs(R.auc(b["label"], eng.score[:1536].cpu().numpy()) - R.auc(b["label"], fw["p"])))
    _stat("wdl bf16 B=1536 %s" % adam, z_max_err=worst, loss_err=worst_loss, auc_delta=worst_auc)
    assert worst < 3e-2 and worst_loss < 5e-3 and worst_auc < 1e-4, (worst, worst_loss, worst_auc)


@pytest.mark.parametrize("name,adam,depth,mid", [("deepfm_pipeline", "lazy", 1, 0), ("deepfm_pipeline", "dense", 1, 0),
                                                 ("deepfm_multi_cate", "lazy", 1, 0), ("wdl", "lazy", 1, 0),
                                                 ("deepfm_pipeline", "lazy", 2, 0), ("wdl", "lazy", 2, 0),
                                                 ("deepfm_pipeline", "lazy", 1, 1), ("wdl", "lazy", 1, 1),
                                                 ("deepfm_multi_cate", "lazy", 2, 1)])
def test_prefetch_matches_inline_index(hip_lib, name, adam, depth, mid, monkeypatch):
    """train_step(next_batch=...) stages and indexes the next batch (depth 2: the next two,
    three buffer sets) into idle buffer sets on the side stream during the current step:
    results are bit-identical to building each index at the start of its own step (graph and
    eager replays, a predict between, a step that prefetches nothing).  mid=1: the step in two
    launches with the prefetch released between them (DLAMD_PF_MID)."""
    monkeypatch.setenv("DLAMD_PF_DEPTH", str(depth))
    monkeypatch.setenv("DLAMD_PF_MID", str(mid))
    kw = CASES[name]
    model = _model(name)
    spec = ModelSpec(model, **kw)
    bs = _batches(name, kw, 256, 8, seed=3)
    runs = []
    for pf in (False, True):
        eng = CTREngine(spec, max_batch=256, seed=9, adam=adam, **({} if adam == "lazy" else {"bwd": "sorted"}))
        assert eng.pf_depth == depth
        zs = []
        for i, b in enumerate(bs[:6]):
            # step 3: no prefetch (depth 1: step 4 indexes inline)
            nxt = (bs[i + 1] if depth == 1 else bs[i + 1: i + 1 + depth]) if pf and i != 3 else None
            eng.train_step(b, graph=i >= 2, next_batch=nxt)
            torch.cuda.synchronize()
            zs.append(eng.z[:256].cpu().numpy().copy())
            if i == 4:
                zs.append(eng.predict(bs[6]))
        p = eng.params()
        runs.append((zs, p))
    # (wdl's wide-weight gradient is int64 fixed point with integer atomics: order-free, exact)
    eq = np.testing.assert_array_equal
    for a, b in zip(runs[0][0], runs[1][0]):
        eq(a, b)
    for k in runs[0][1]:
        eq(runs[0][1][k], runs[1][1][k], err_msg=k)


@pytest.mark.parametrize("name,adam,where,ring", [
    ("deepfm_pipeline", "lazy", "cate", 0), ("deepfm_pipeline", "dense", "cate", 0),
    ("wdl", "lazy", "cate", 0), ("wdl", "lazy", "wide", 0), ("wdl", "dense", "wide", 0),
    ("deepfm_multi_cate", "lazy", "multi", 0), ("deepfm_multi_cate", "dense", "multi", 0),
    ("deepfm_pipeline", "lazy", "cate", 1), ("wdl", "lazy", "wide", 1)])
def test_bad_id_batch_skipped_alone_and_raises(hip_lib, name, adam, where, ring, monkeypatch):
    """TF raises InvalidArgumentError inside the failing sess.run, before anything is applied
    (deepfm_pipeline.py:219-221), and the next sess.run applies normally.  Here every id is
    validated before its step begins (dl_index_build, dl_validate_batch for the dense-layout
    gathers and wdl's wide ids), the step of the bad batch is skipped whole (the per-step skip
    word, include/dlamd.h), the batches after it apply, and train_step raises within two calls
    naming the global step skipped.  The final state is bit-identical to an engine that never
    saw the bad batch: parameters, Adam moments, the step counter (adam='dense' runs the
    dense-layout gather and the float-atomic backward, whose summation order varies: 1e-5).
    ring=1: the status reported by the step's last kernel into pinned memory (DLAMD_STATUS_RING)."""
    from deep_learning_amd import _lib
    monkeypatch.setenv("DLAMD_STATUS_RING", str(ring))
    kw = CASES[name]
    spec = ModelSpec(_model(name), **kw)
    mk = lambda: CTREngine(spec, max_batch=256, seed=4, adam=adam)
    eng, twin = mk(), mk()
    bs = _batches(name, kw, 256, 6, seed=13)
    bad = {k: v.copy() for k, v in bs[3].items()}
    if where == "cate":
        bad["cate_feats"][5, 3] = kw["cate_index_size"] + 7
    elif where == "multi":
        bad["cate_feats"][7, -2] = kw["cate_index_size"] + 3
    else:
        bad["wide_feats"][9, 1] = kw["cate_index_size"] + kw["hidden"][-1] + 1
    seq = bs[:3] + [bad] + bs[4:]
    raised = []
    for i, b in enumerate(seq):
        try:
            eng.train_step(b, graph=i >= 1)        # the batch's step is issued even if this raises
        except _lib.DLError as e:
            raised.append(str(e))
    torch.cuda.synchronize()
    try:
        eng.check_error()
    except _lib.DLError as e:
        raised.append(str(e))
    assert len(raised) == 1 and "out of range" in raised[0] and "global_step 3" in raised[0], raised
    for i, b in enumerate(bs[:3] + bs[4:]):
        twin.train_step(b, graph=i >= 1)
    torch.cuda.synchronize()
    twin.check_error()
    assert float(eng.opt[7].item()) == float(twin.opt[7].item()) == 5
    same = (np.testing.assert_array_equal if adam == "lazy" else
            lambda a, b, err_msg: np.testing.assert_allclose(a, b, atol=TOL, rtol=0, err_msg=err_msg))
    pe, pt = eng.params(), twin.params()
    for k in pt:
        same(pe[k], pt[k], err_msg=k)
    se, st = eng.adam_state(), twin.adam_state()
    for k in st:
        same(se[k], st[k], err_msg=k)


def _hot(bs, seed=5):
    """Zipf-like hot rows: one field all one id, one field over five ids, 10 % of every
    other entry one shared id — segments of hundreds of references (the wave-cooperative
    long-segment sums of segment.h), beside ordinary short ones."""
    rng = np.random.default_rng(seed)
    for b in bs:
        c = b["cate_feats"]
        c[:, 3] = 77
        c[:, 5] = 100 + rng.integers(0, 5, size=c.shape[0])
        m = rng.random(c.shape) < 0.1
        m[:, 3] = m[:, 5] = False
        c[m] = 9
    return bs


@pytest.mark.parametrize("name", ["deepfm_pipeline", "wdl", "dnn_pipeline"])
def test_hot_rows_lazy_bit_identical_to_dense(hip_lib, name):
    """Hot rows: the lazy record update and the dense sorted backward sum every long
    segment by the same wave-cooperative order — bit-identical parameters and moments."""
    kw = dict(CASES[name], cate_index_size=50000)
    same = np.testing.assert_array_equal
    spec = ModelSpec(_model(name), **kw)
    dense = CTREngine(spec, max_batch=1024, seed=3, bwd="sorted")
    lazy = CTREngine(spec, max_batch=1024, seed=3, adam="lazy", hist_len=8)
    bs = _hot(_batches(name, kw, 1024, 6, seed=9))
    for i, b in enumerate(bs):
        dense.train_step(b, graph=i >= 2)
        lazy.train_step(b, graph=i >= 2)
        torch.cuda.synchronize()
        same(lazy.z[:1024].cpu().numpy(), dense.z[:1024].cpu().numpy(), err_msg="logits step %d" % i)
    pd, pl = dense.params(), lazy.params()
    for k in pd:
        same(pl[k], pd[k], err_msg=k)


@pytest.mark.parametrize("bwd", ["sorted", "lazy"])
@pytest.mark.parametrize("name", ["deepfm_pipeline", "deepfm_multi_cate"])
def test_hot_rows_match_oracle(hip_lib, name, bwd):
    """Hot rows against the oracle (its segment sums run in reference order; the long
    segments here are summed in the wave's fixed order): logits, loss, parameters 1e-5."""
    kw = CASES[name]
    model = _model(name)
    cfg = R.make_cfg(model, **kw)
    spec = ModelSpec(model, **kw)
    P = R.init_params(cfg, np.random.default_rng(42))
    B = 1536
    eng = (CTREngine(spec, max_batch=B, init="none", adam="lazy") if bwd == "lazy"
           else CTREngine(spec, max_batch=B, init="none", bwd=bwd))
    eng.load_params(P)
    opt = R.AdamTF1(cfg, P)
    for step, b in enumerate(_hot(_batches(name, kw, B, 3))):
        fw = R.train_step(cfg, P, opt, b)
        eng.train_step(b, graph=(step >= 1))
        torch.cuda.synchronize()
        np.testing.assert_allclose(eng.z[:B].cpu().numpy(), fw["z"], atol=TOL, rtol=0, err_msg="logits %d" % step)
        assert abs(eng.loss() - fw["loss"]) < TOL
    got = eng.params()
    for k in P:
        np.testing.assert_allclose(got[k], P[k], atol=TOL, rtol=0, err_msg=k)


@pytest.mark.parametrize("name,tower", [("deepfm_pipeline", "f32"), ("wdl", "f32"), ("wdl", "bf16"),
                                        ("deepfm_multi_cate", "f32"), ("dnn_pipeline", "f32")])
def test_scatter_forward_bit_identical_to_indexed(hip_lib, name, tower):
    """The lazy forward's scatter form (dl_rec_gather_scatter + dl_embed_fwd_staged: rows
    written to their references' FM staging rows / first-order outputs / x0 columns) against
    the indexed form (compact rows read back through the inverse map): logits, x0 (bf16 for
    the bf16 tower), the FM outputs and the trained parameters bit for bit, on batches with
    hot rows (segments far past the 32-reference per-row limit: the block-per-row pass),
    padding id 0 (no row: zeros written by the staged forward) and ids aliasing cont rows."""
    kw = CASES[name]
    spec = ModelSpec(_model(name), tower=tower, **kw)
    a = CTREngine(spec, max_batch=1024, seed=5, adam="lazy", fwd_scatter=True)
    b = CTREngine(spec, max_batch=1024, seed=5, adam="lazy", fwd_scatter=False)
    assert a.fwd_scatter and not b.fwd_scatter
    same = np.testing.assert_array_equal
    for i, bt in enumerate(_hot(_batches(name, kw, 1024, 4, seed=21))):
        a.train_step(bt, graph=i >= 1)
        b.train_step(bt, graph=i >= 1)
        torch.cuda.synchronize()
        same(a.z[:1024].cpu().numpy(), b.z[:1024].cpu().numpy(), err_msg="logits step %d" % i)
        xa, xb = (a.x0b, b.x0b) if a.x0_direct else (a.x0, b.x0)
        same(xa[:1024].float().cpu().numpy(), xb[:1024].float().cpu().numpy(), err_msg="x0 step %d" % i)
        if spec.fm:
            same(a.fm_out[:1024].cpu().numpy(), b.fm_out[:1024].cpu().numpy(), err_msg="fm_out step %d" % i)
    pa, pb = a.params(), b.params()
    for k in pa:
        same(pa[k], pb[k], err_msg=k)
    # predict (lag 0, no stash) through both forms
    same(a.predict(bt), b.predict(bt))


@pytest.mark.parametrize("name", ["wdl", "deepfm_pipeline", "dnn"])
def test_running_loss_sum_and_partial_last_batch(hip_lib, name):
    """The load-style fit's epoch loss (wdl.py:305-313: sum of loss_t * batch_size) summed on
    the device (loss_sum_begin / loss_sum_end: no host read, no wide-table flush per step)
    against the oracle's per-step losses; an 8-entry alpha ring forces lagging wide rows and
    flushes mid-sum.  The last batch is smaller than the others: the per-step loss() of that
    step (lazy wide records: only the update blocks that batch launched) must match too."""
    kw = dict(CASES[name], cate_index_size=30000)
    model = _model(name)
    cfg = R.make_cfg(model, **kw)
    P = R.init_params(cfg, np.random.default_rng(17))
    spec = ModelSpec(model, **kw)
    run = CTREngine(spec, max_batch=256, init="none", adam="lazy", hist_len=8)
    step = CTREngine(spec, max_batch=256, init="none", adam="lazy", hist_len=8)
    run.load_params(P)
    step.load_params(P)
    opt = R.AdamTF1(cfg, P)
    bs = _batches(name, kw, 256, 13, seed=31)
    last = _batches(name, kw, 96, 1, seed=77)[0]
    bs.append(last)
    run.loss_sum_begin()
    ref = []
    for i, b in enumerate(bs):
        fw = R.train_step(cfg, P, opt, b)
        ref.append(fw["loss"])
        full = b["label"].shape[0] == 256
        nxt = bs[i + 1] if i + 1 < len(bs) else None
        run.train_step(b, graph=full and i >= 2, **({"next_batch": nxt} if nxt is not None else {}))
        step.train_step(b, graph=full and i >= 2)
        assert abs(step.loss() - fw["loss"]) < TOL, "per-step loss at step %d (B=%d)" % (i, b["label"].shape[0])
    total, n = run.loss_sum_end()
    assert n == len(bs)
    np.testing.assert_allclose(total, float(np.sum(ref)), rtol=0, atol=TOL * len(bs))
    # the running sum and the exact per-step sum agree far below the oracle bar
    np.testing.assert_allclose(run.params()[spec.table_key], step.params()[spec.table_key], rtol=0, atol=0)
