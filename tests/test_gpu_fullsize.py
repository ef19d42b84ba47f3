"""Parity at the BASELINE configurations' own sizes (SURVEY.md §8 config keys C2-C5).

The per-model parity tests (test_gpu_parity.py) run at B <= 1536 and small tables; these
run the product path (row records, lazy-exact Adam, hipGraph replay) at full size:

  C2  deepfm_pipeline, 26,000,013 x 16 table, MLP [400]x3, B = 65,536          (fp32, TOL 1e-5)
  C3  deepfm_multi_cate, 26 single + 6 multi-hot slots x 60, 26M rows, B = 65,536 (fp32)
  C4  deepfm_pipeline, 100,000,013-row table in the row-sharded engine (RCCL, one rank)
      against the single-GPU engine on the same table and batches
  C5  wdl, bf16 deep tower, 26M rows + 26 wide ids, B = 65,536  (stated bf16 tolerance)

C2 / C3 run 10 steps (logits within 1e-5 at steps 0-10) in two tracks against
the numpy oracle, from the same injected initial parameters and the same batches:

  same-state (all 10 steps): before every step the oracle takes the GPU's whole state
    (parameters and Adam moments, exported), takes the f32 TF1 step, and the GPU's step must
    agree: every logit and the loss within 1e-5, every parameter element within 1e-5 —
    or else the element is AUDITED in fp64 (tests/_fp64_audit.py): the gradient the GPU
    applied (read back from its Adam moments) must equal the element's gradient of the GPU's
    own pre-step state recomputed in float64 within the a-priori f32 error bound
    K u S (S the element's running-error scale, K = K_SUM the summation depth) plus the
    envelope of ReLU pre-activations within rounding of zero, and its v and p must have moved
    by TF1 Adam on that gradient.  An element that fails the audit fails the test; the
    audited elements' count and conditioning (min |G| / S, max |g' - G| / (u S)) go to the
    stats, table and dense alike.
  trajectory (first TRAJ_STEPS steps): the oracle is never re-synced except for the elements
    off by more than 1e-5 (ill-conditioned sums, counted and bounded: at most 1e-4 of an
    array after the first step, 1e-3 / 5e-4 later, each within one step's flip size), and
    the logits along it must stay within 1e-5 for all but 1e-3 of the samples, every one
    within Z_DRIFT — the drift of two f32 evaluation orders, which the same-state track
    shows is not an error of either step.

Why the same-state track and not a longer trajectory: the elements whose summed gradient is
within f32 rounding of zero (a [400, 400] weight gradient sums 65,536 products per element)
move by up to 2 * FLIP * alpha in Adam's sign-saturated first steps whichever way the sum
rounds, so two correct f32 implementations drift apart step by step (measured: 770, 3,827,
13,644 such table elements at steps 0-2 of the never-re-synced C2 run, profiles/r03zl).

C5 (bf16 tower) follows the TRAJ_STEPS trajectory at its stated bf16 bounds, never repaired.

DLAMD_TEST_STATS=<dir>: each test appends its measured maxima / flip fractions there (json).
"""
import json
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

from deep_learning_amd.engine import CTREngine, ModelSpec  # noqa: E402
from deep_learning_amd.synthetic import make_batch  # noqa: E402
from oracle import ctr_ref as R  # noqa: E402
from tests import _fp64_audit as A  # noqa: E402

TOL = 1e-5
N_CATE = 26 * 1_000_000
B = 65536
HIDDEN = [400, 400, 400]
STEPS = 10           # fp32 C2 / C3, same-state track
TRAJ_STEPS = 3       # the never-re-synced trajectory (fp32) and the C5 bf16 run
K_SUM = 2048         # summation-depth bound of the fp64 audit (|g' - G64| <= K_SUM u S + U)

# |m / sqrt(v)| <= (1 - b1) / sqrt(1 - b2) for TF1 Adam's moments (b1^2 < b2), so one update
# moves an element by at most FLIP * alpha and a sign flip of it by twice that
FLIP = (1 - 0.9) / np.sqrt(1 - 0.999)

# bf16 tower (C5): the tower's gradients carry bf16 operand rounding (relative ~2^-9 per
# product), so the table's gradients, and through Adam's sign-saturated first steps the
# updates, differ from the fp32 oracle's by a sign flip wherever the fp32 gradient is within
# that rounding of zero (and move by a different amount where it is near Adam's epsilon).
# Stated bf16 bounds: elements within BF16_ATOL except at most BF16_FRAC of them (measured
# after one step: hidden weights 0.1 % beyond 1e-5, max 8.7e-4; biases 3.75 % beyond 1e-5,
# max 8.8e-5 — profiles/r03b/fullsize_stats.jsonl), every element within the flip size;
# Adam moments within BF16_MRTOL relative (+ a floor) except the same fraction.
BF16_ATOL = 1e-4
# logits along the fp32 trajectory (steps >= 1) against the never-re-synced oracle state
Z_DRIFT = 5 * TOL
BF16_FRAC = 0.01
BF16_MRTOL = 0.05


def _stat(name, **kw):
    d = os.environ.get("DLAMD_TEST_STATS")
    if not d:
        return
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "fullsize_stats.jsonl"), "a") as f:
        f.write(json.dumps(dict(test=name, **{k: float(v) for k, v in kw.items()})) + "\n")


def _terms(key, idx, trace, fw):
    """sum_b |terms| of the gradient sums of dense parameter `key` at flat indices idx (the
    scale the sums' f32 rounding lives on): hidden weights X_i^T g_i, biases sum_b g_i, the
    FM / deep_res head weights feats^T dz (hs[-1]^T dz), its bias sum_b dz."""
    dz = np.abs(trace["dz"]).astype(np.float64)
    if key.startswith("deep_bias_"):
        g = np.abs(trace["g"][int(key.rsplit("_", 1)[1])]).astype(np.float64)
        return g.sum(0)[idx]
    if key.startswith("deep_") and key[5:].isdigit():
        i = int(key[5:])
        X, g = np.abs(trace["xs"][i]), np.abs(trace["g"][i])
        r, c = np.unravel_index(idx, (X.shape[1], g.shape[1]))
        return np.array([float(np.dot(X[:, a].astype(np.float64), g[:, b].astype(np.float64))) for a, b in zip(r, c)])
    if key in ("deep_fm_weight", "deep_res"):
        F = np.abs(fw["feats"] if key == "deep_fm_weight" else fw["hs"][-1]).astype(np.float64)
        return (F[:, idx] * dz[:, None]).sum(0)
    return np.full(len(idx), dz.sum())


def _run(name, model, kw, batches, tower="f32", z_tol=TOL, loss_tol=TOL, auc_tol=None, seed=42, heldout=()):
    cfg = R.make_cfg(model, **kw)
    P = R.init_params(cfg, np.random.default_rng(seed))
    eng = CTREngine(ModelSpec(model, tower=tower, **kw), max_batch=B, init="none", adam="lazy")
    eng.load_params(P)
    opt = R.AdamTF1(cfg, P)
    spec = eng.spec
    tk = spec.table_key
    bf = tower == "bf16"
    rng = np.random.default_rng(1)
    touched_all = []
    fails = []

    def check(cond, msg):
        if not cond:
            fails.append(msg)

    def compare(got, want, bound, what, frac, atol=TOL, rtol=0.0):
        g64, w64 = got.astype(np.float64), want.astype(np.float64)
        d = np.abs(g64 - w64)
        bad = d > atol + rtol * np.abs(w64)
        _stat("%s %s" % (name, what), max_err=d.max() if d.size else 0.0, frac_bad=bad.mean() if d.size else 0.0)
        check(bad.sum() <= max(1, frac * d.size), "%s: %d of %d elements off by > %g (max %g)" % (
            what, bad.sum(), d.size, atol, d.max()))
        check(d.max() <= bound, "%s: max error %g > %g" % (what, d.max(), bound))
        return bad

    for step, b in enumerate(batches):
        alpha = float(opt.alpha())           # this step's alpha (before the oracle advances it)
        trace = {}
        fw = R.forward(cfg, P, b)
        G, _ = R.backward(cfg, P, b, fw, trace=trace)
        opt.apply(P, G)
        eng.train_step(b, graph=step >= 1)
        torch.cuda.synchronize()
        eng.check_error()
        z = eng.z[:B].cpu().numpy()
        dz = np.abs(z.astype(np.float64) - fw["z"])
        _stat("%s step %d" % (name, step), z_max_err=dz.max(), z_frac_bad=(dz > z_tol).mean(),
              loss_err=abs(eng.loss() - fw["loss"]))
        if step == 0 or bf:
            check(dz.max() <= z_tol, "logits step %d: max error %g > %g (%d samples)" % (
                step, dz.max(), z_tol, (dz > z_tol).sum()))
        else:
            # from identical state (the GPU's own state after the last step, through the
            # oracle's forward): the reference's 1e-5 on every logit
            z1 = R.forward(cfg, prev, b)["z"]
            d1 = np.abs(z.astype(np.float64) - z1)
            _stat("%s step %d same-state" % (name, step), z_max_err=d1.max())
            check(d1.max() <= z_tol, "logits step %d from the GPU's state: max error %g > %g" % (
                step, d1.max(), z_tol))
            # along the trajectory the oracle's state carries its own sub-TOL summation-order
            # differences (never re-synced): within TOL but for at most 1e-3 of the samples,
            # every one within Z_DRIFT
            check((dz > z_tol).mean() <= 1e-3 and dz.max() <= Z_DRIFT,
                  "logits step %d: max error %g, %d samples > %g" % (step, dz.max(), (dz > z_tol).sum(), z_tol))
        check(abs(eng.loss() - fw["loss"]) < loss_tol, "loss step %d: %r vs %r" % (step, eng.loss(), fw["loss"]))
        if auc_tol is not None:
            s = eng.score[:B].cpu().numpy()
            check(abs(R.auc(b["label"], s) - R.auc(b["label"], fw["p"])) < auc_tol, "AUC step %d" % step)
        # rows the step touched (FM rows id + offset, deep rows id, multi-hot ids)
        ids = b["cate_feats"].reshape(-1).astype(np.int64)
        t = np.unique(np.concatenate([ids + spec.fm_cate_offset, ids]))
        touched_all.append(t[t < spec.n_rows])
        # dense parameters and moments after every step
        bound = 2 * FLIP * alpha + TOL
        got = eng.dense_params()
        ds = eng.dense_state()
        for key in got:
            what = "%s (step %d)" % (key, step)
            if bf:
                compare(got[key], P[key], bound, what, BF16_FRAC, BF16_ATOL)
                continue
            bad = compare(got[key], P[key], bound, what, 1e-4 if step == 0 else 1e-3).reshape(-1)
            if not bad.any() or key == "wdl_weights":
                continue
            # the elements off take the GPU's state (recorded: how many, how ill-conditioned)
            idx = np.flatnonzero(bad)
            gabs = np.abs(G[key].reshape(-1)[idx].astype(np.float64))
            terms = _terms(key, idx, trace, fw)
            _stat("%s %s repaired" % (name, what), n=len(idx),
                  min_g_over_terms=(gabs / np.maximum(terms, 1e-300)).min(), max_abs_g=gabs.max())
            for arr, src in ((P[key], got[key]), (opt.m[key], ds["m"][key]), (opt.v[key], ds["v"][key])):
                arr.reshape(-1)[idx] = np.asarray(src).reshape(-1)[idx]
        # the table (never re-synced except its elements off by > TOL, which are counted and
        # bounded like the dense ones): all rows after every step (the fp32 path), a sample of
        # touched and untouched rows after the first and the last step (the bf16 tower)
        k = step + 1
        tbound = k * 2 * FLIP * alpha + TOL
        frac = 1e-4 if step == 0 else 5e-4
        last = step == len(batches) - 1
        what = lambda key: "%s (step %d)" % (key, step)
        if bf:
            if step not in (0, len(batches) - 1):
                continue
            pick = np.concatenate([rng.choice(touched_all[-1], 20000, replace=False),
                                   rng.choice(touched_all[0], 5000, replace=False),
                                   rng.integers(0, spec.n_rows, 20000)])
            gp = eng.params()
            st = eng.adam_state()
            compare(gp[tk][pick], P[tk][pick], tbound, what(tk), BF16_FRAC, BF16_ATOL)
            compare(st["m"][pick], opt.m[tk][pick], np.inf, what("m"), BF16_FRAC, 1e-7, BF16_MRTOL)
            compare(st["v"][pick], opt.v[tk][pick], np.inf, what("v"), BF16_FRAC, 1e-10, 2 * BF16_MRTOL)
            del gp, st
            continue
        gp = eng.params()
        st = eng.adam_state()
        prev = gp
        keys = [(tk, "m", "v")] + ([(spec.first_key, "m1", "v1")] if spec.fm else [])
        for key, mk, vk in keys:
            bad = compare(gp[key], P[key], tbound, what(key), frac if not last else 5e-4)
            compare(st[mk].reshape(P[key].shape), opt.m[key], tbound, what(mk), frac if not last else 5e-4)
            if bad.any():
                idx = np.flatnonzero(bad.reshape(-1))
                _stat("%s %s repaired" % (name, what(key)), n=len(idx))
                for arr, src in ((P[key], gp[key]), (opt.m[key], st[mk]), (opt.v[key], st[vk])):
                    arr.reshape(-1)[idx] = np.asarray(src).reshape(-1)[idx]
        del st
    if heldout:
        # the reference's evaluate (wdl.py:343-358: sklearn roc_auc_score over the held-out
        # batches' predictions) on the trained state, against the oracle's trained parameters
        ys, sg, so, zerr = [], [], [], 0.0
        for hb in heldout:
            zg = eng.predict(hb, logits=True).astype(np.float64)
            fo = R.forward(cfg, P, hb)
            zerr = max(zerr, float(np.abs(zg - fo["z"]).max()))
            ys.append(hb["label"].reshape(-1))
            sg.append(1.0 / (1.0 + np.exp(-zg)))
            so.append(fo["p"])
        y = np.concatenate(ys)
        a_gpu, a_ref = R.auc(y, np.concatenate(sg)), R.auc(y, np.concatenate(so))
        _stat("%s heldout" % name, n=len(y), auc_gpu=a_gpu, auc_oracle=a_ref, auc_delta=abs(a_gpu - a_ref),
              z_max_err=zerr)
        check(zerr <= z_tol, "held-out logits: max error %g > %g" % (zerr, z_tol))
        check(abs(a_gpu - a_ref) < auc_tol, "held-out AUC %r vs oracle %r (|d| %g >= %g)" % (
            a_gpu, a_ref, abs(a_gpu - a_ref), auc_tol))
    assert not fails, "; ".join(fails)
    return eng


def _run_fp32(name, model, kw, batches, seed=42):
    """The fp32 configs (C2, C3): the same-state track over every batch with the fp64 audit of
    every element off by more than TOL, and the never-re-synced trajectory over the first
    TRAJ_STEPS batches (module docstring)."""
    cfg = R.make_cfg(model, **kw)
    P0 = R.init_params(cfg, np.random.default_rng(seed))
    eng = CTREngine(ModelSpec(model, **kw), max_batch=B, init="none", adam="lazy")
    eng.load_params(P0)
    spec = eng.spec
    tk, fk = spec.table_key, spec.first_key
    tab_moments = {tk: ("m", "v"), fk: ("m1", "v1")}
    fails = []

    def check(cond, msg):
        if not cond:
            fails.append(msg)

    # the GPU's state before the next step, in the reference layout
    gpu_p = {k: v.copy() for k, v in P0.items()}
    gpu_m = {k: np.zeros_like(v) for k, v in P0.items()}
    gpu_v = {k: np.zeros_like(v) for k, v in P0.items()}
    opt_s = R.AdamTF1(cfg, gpu_p)
    Pt = {k: v.copy() for k, v in P0.items()}          # the never-re-synced trajectory
    opt_t = R.AdamTF1(cfg, Pt)
    b1, b2, eps = cfg.beta1, cfg.beta2, cfg.eps
    for step, b in enumerate(batches):
        alpha = float(opt_s.alpha())
        # ---- the same-state oracle step: from the GPU's whole state after the previous step
        Ps = {k: v.copy() for k, v in gpu_p.items()}
        opt_s.m = {k: v.copy() for k, v in gpu_m.items()}
        opt_s.v = {k: v.copy() for k, v in gpu_v.items()}
        fw = R.forward(cfg, Ps, b)
        G, _ = R.backward(cfg, Ps, b, fw)
        opt_s.apply(Ps, G)
        del G
        traj = step < TRAJ_STEPS
        if traj:
            trace = {}
            fwt = R.forward(cfg, Pt, b)
            Gt, _ = R.backward(cfg, Pt, b, fwt, trace=trace)
            opt_t.apply(Pt, Gt)
        eng.train_step(b, graph=step >= 1)
        torch.cuda.synchronize()
        eng.check_error()
        gpu_mid = A.read_gpu(eng, B)
        z = eng.z[:B].cpu().numpy().astype(np.float64)
        loss = eng.loss()
        d = np.abs(z - fw["z"])
        _stat("%s step %d same-state" % (name, step), z_max_err=d.max(), loss_err=abs(loss - fw["loss"]))
        check(d.max() <= TOL, "logits step %d from the GPU's state: max error %g (%d samples > %g)" % (
            step, d.max(), (d > TOL).sum(), TOL))
        check(abs(loss - fw["loss"]) < TOL, "loss step %d: %r vs %r" % (step, loss, fw["loss"]))
        gp = eng.params()
        ds = eng.dense_state()
        st = eng.adam_state()
        new_m = {k: (st[tab_moments[k][0]].reshape(P0[k].shape) if k in tab_moments else ds["m"][k]) for k in gp}
        new_v = {k: (st[tab_moments[k][1]].reshape(P0[k].shape) if k in tab_moments else ds["v"][k]) for k in gp}
        del st, ds
        # ---- every stage of the GPU's step against fp64 of its own inputs (tests/_fp64_audit.py)
        audit = A.StepAudit(cfg, gpu_p, b, gpu_mid)
        for what, st_ in audit.stats.items():
            _stat("%s step %d stage %s" % (name, step, what), **st_)
        fails += ["step %d: %s" % (step, f) for f in audit.fails]
        # ---- every element of the GPU's step against the oracle's step from the same state;
        # the elements off by more than TOL are audited in fp64
        for key in P0:
            diff = np.abs(gp[key].astype(np.float64) - Ps[key])
            idx = np.flatnonzero(diff.reshape(-1) > TOL)
            what = "%s (step %d)" % (key, step)
            _stat("%s %s same-state" % (name, what), max_err=diff.max(), n_off=len(idx))
            if not len(idx):
                continue
            check(len(idx) <= max(1, 1e-3 * diff.size), "%s: %d of %d elements off by > %g" % (
                what, len(idx), diff.size, TOL))
            fl = lambda a: np.asarray(a).reshape(-1)[idx]
            ok, st_, (g, G64, S) = A.audit_elements(audit, key, idx, P0[key].shape, fl(gpu_m[key]), fl(new_m[key]),
                                                    fl(gpu_v[key]), fl(new_v[key]), fl(gpu_p[key]), fl(gp[key]),
                                                    alpha, b1, b2, eps)
            _stat("%s %s audited" % (name, what), **st_)
            if not ok.all():
                j = int(np.flatnonzero(~ok)[0])
                fails.append("%s: %d of %d audited elements fail the fp64 audit (e.g. flat %d: GPU gradient %r, "
                             "fp64 %r, scale %r)" % (what, (~ok).sum(), len(idx), idx[j], g[j], G64[j], S[j]))
        del audit
        # ---- the never-re-synced trajectory (first TRAJ_STEPS steps)
        if traj:
            dz = np.abs(z - fwt["z"])
            _stat("%s step %d" % (name, step), z_max_err=dz.max(), z_frac_bad=(dz > TOL).mean(),
                  loss_err=abs(loss - fwt["loss"]))
            check((dz > TOL).mean() <= 1e-3 and dz.max() <= Z_DRIFT,
                  "trajectory logits step %d: max error %g, %d samples > %g" % (step, dz.max(), (dz > TOL).sum(), TOL))
            bound = 2 * FLIP * alpha + TOL
            tbound = (step + 1) * 2 * FLIP * alpha + TOL
            for key in P0:
                tab = key in tab_moments
                diff = np.abs(gp[key].astype(np.float64) - Pt[key])
                bad = diff > TOL
                frac = 1e-4 if step == 0 else (5e-4 if tab else 1e-3)
                _stat("%s %s (step %d) trajectory" % (name, key, step), max_err=diff.max(), frac_bad=bad.mean())
                check(bad.sum() <= max(1, frac * diff.size) and diff.max() <= (tbound if tab else bound),
                      "trajectory %s step %d: %d elements off by > %g (max %g)" % (key, step, bad.sum(), TOL,
                                                                                    diff.max()))
                if not bad.any():
                    continue
                idx = np.flatnonzero(bad.reshape(-1))
                rec = dict(n=len(idx))
                if not tab:
                    gabs = np.abs(Gt[key].reshape(-1)[idx].astype(np.float64))
                    terms = _terms(key, idx, trace, fwt)
                    rec.update(min_g_over_terms=(gabs / np.maximum(terms, 1e-300)).min(), max_abs_g=gabs.max())
                _stat("%s %s (step %d) repaired" % (name, key, step), **rec)
                # those elements take the GPU's value and moments; the rest is never re-synced
                for arr, src in ((Pt[key], gp[key]), (opt_t.m[key], new_m[key]), (opt_t.v[key], new_v[key])):
                    arr.reshape(-1)[idx] = np.asarray(src).reshape(-1)[idx]
            del Gt, trace
        gpu_p, gpu_m, gpu_v = gp, new_m, new_v
        del Ps
    assert not fails, "; ".join(fails[:8])
    return eng


def test_c2_deepfm_pipeline_full_size_trajectory(hip_lib):
    kw = dict(C=13, V=0, S=26, E=16, cate_index_size=N_CATE, hidden=HIDDEN)
    bs = [make_batch(B, cate_index_size=N_CATE, seed=100 + i) for i in range(STEPS)]
    _run_fp32("c2", "deepfm_pipeline", kw, bs)


def test_c3_deepfm_multi_cate_full_size_trajectory(hip_lib):
    ranges = [[60 * i, 60 * (i + 1), "slot%d" % i] for i in range(6)]
    kw = dict(C=0, V=0, S=26, E=16, cate_index_size=N_CATE, hidden=HIDDEN, multi_ranges=ranges)
    bs = [make_batch(B, cont=0, cate_fields=26, cate_index_size=N_CATE, multi_slots=6, multi_width=60,
                     seed=200 + i, cate_only=True) for i in range(STEPS)]
    _run_fp32("c3", "deepfm_multi_cate", kw, bs)


def test_c5_wdl_bf16_full_size_trajectory(hip_lib):
    """C5 with the bf16 tower against the fp32 oracle (never re-synced): every logit within 1e-3
    (measured <= 2.9e-4 over these steps, profiles/r04zp), the loss within 1e-4, the per-step
    AUC and — north star — the AUC of 4 held-out full-size batches predicted with the trained
    state within 1e-4 of the oracle's (wdl.py:343-358), the BF16_* parameter bounds above."""
    kw = dict(C=13, S=26, E=16, cate_index_size=N_CATE, hidden=HIDDEN, Fw=26)
    bs = [make_batch(B, cate_index_size=N_CATE, seed=300 + i, wide_fields=26) for i in range(TRAJ_STEPS)]
    hb = [make_batch(B, cate_index_size=N_CATE, seed=900 + i, wide_fields=26) for i in range(4)]
    _run("c5", "wdl", kw, bs, tower="bf16", z_tol=1e-3, loss_tol=1e-4, auc_tol=1e-4, heldout=hb)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_c4_sharded_100m_rows_equals_single_gpu(hip_lib):
    """C4's workload at one rank: the 100,000,013-row table (25.6 GB of row records) in the
    row-sharded engine (shard.py: index, count all-gather, RCCL id / row / gradient exchanges,
    owner gather and update, flat all-reduce) against the single-GPU engine on the same table,
    parameters and batches (B = 65,536, 3 steps): logits and loss every step, then the records
    (p, both moments, first-order triple) of sampled touched rows, the replicated FM cont rows
    and every dense parameter.  At one rank both engines sum every gradient in the same order,
    so the bar is bit-identity, with 1e-5 allowed for the replicated rows' dense update."""
    import torch.distributed as dist
    from deep_learning_amd.shard import Exchange, ShardedCTREngine
    n_cate = 100_000_000
    spec = ModelSpec("deepfm_pipeline", C=13, V=0, S=26, E=16, cate_index_size=n_cate, hidden=HIDDEN)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1")
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    try:
        one = CTREngine(spec, max_batch=B, seed=2019, adam="lazy")
        sh = ShardedCTREngine(spec, B, Exchange(), seed=2019, adam="lazy")
        # the same state: records copied (local row i == global row i at one rank), the
        # replicated FM cont rows taken from the same records, the dense parameters copied
        assert sh.rec.shape == one.rec.shape
        sh.rec.copy_(one.rec)
        E, rep = spec.E, sh.rep
        sh.rep_t[:rep].copy_(one.rec[:rep, :E])
        sh.rep_f[:rep].copy_(one.rec[:rep, E])
        for l in range(len(HIDDEN)):
            sh.W[l].copy_(one.W[l])
            sh._refresh_wb(l)
        sh.w_head.copy_(one.w_head)
        sh.opt.copy_(one.opt)
        torch.cuda.synchronize()
        bs = [make_batch(B, cate_index_size=n_cate, seed=400 + i) for i in range(TRAJ_STEPS)]
        dev = [{k: torch.from_numpy(v).cuda() for k, v in b.items()} for b in bs]
        for step, b in enumerate(dev):
            one.train_step(b, graph=step >= 1)
            sh.train_step(b, graph=step >= 1)
            torch.cuda.synchronize()
            one.check_error()
            za, zb = one.z[:B].cpu().numpy(), sh.z[:B].cpu().numpy()
            _stat("c4 step %d" % step, z_max_err=np.abs(za - zb).max(), z_bit_equal=(za == zb).mean())
            np.testing.assert_allclose(zb, za, atol=TOL, rtol=0, err_msg="logits step %d" % step)
            assert abs(sh.loss() - one.loss()) < TOL
        one.flush()
        sh.flush()
        torch.cuda.synchronize()
        ids = np.concatenate([b["cate_feats"].reshape(-1) for b in bs]).astype(np.int64)
        rows = np.unique(np.concatenate([ids + 13, ids]))
        rows = rows[rows >= rep]        # rows < 13 are the replicated FM cont rows (checked below)
        rng = np.random.default_rng(5)
        pick = torch.from_numpy(np.concatenate([rng.choice(rows, 200_000, replace=False),
                                                rng.integers(rep, spec.n_rows, 50_000)])).cuda()
        ra, rb = one.rec[pick, : 3 * E + 4], sh.rec[pick, : 3 * E + 4]
        _stat("c4 records", max_err=(ra - rb).abs().max().item(), bit_equal=(ra == rb).float().mean().item())
        assert torch.equal(ra, rb), "records differ: max %g" % (ra - rb).abs().max().item()
        # replicated FM cont-field rows (dense Adam on the replica) against the single-GPU records
        np.testing.assert_allclose(sh.rep_t[:rep].cpu().numpy(), one.rec[:rep, :E].cpu().numpy(), atol=TOL, rtol=0)
        np.testing.assert_allclose(sh.rep_f[:rep].cpu().numpy(), one.rec[:rep, E].cpu().numpy(), atol=TOL, rtol=0)
        for l in range(len(HIDDEN)):
            np.testing.assert_allclose(sh.W[l].cpu().numpy(), one.W[l].cpu().numpy(), atol=TOL, rtol=0)
        np.testing.assert_allclose(sh.w_head.cpu().numpy(), one.w_head.cpu().numpy(), atol=TOL, rtol=0)
        del one, sh
        torch.cuda.empty_cache()
    finally:
        dist.destroy_process_group()
