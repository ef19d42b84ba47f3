"""GPU tests of the drop-in surface: the engine against the committed oracle
fixtures, and local_run.py (train -> checkpoint/export -> pred) end to end on
TFRecord files, with the final AUC checked against the oracle trained on the
identical (unshuffled) batches."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.mark.parametrize("name", ["deepfm_pipeline", "dnn_pipeline", "deepfm_multi_cate"])
def test_engine_matches_committed_fixtures(hip_lib, name):
    from deep_learning_amd.engine import CTREngine, ModelSpec
    from tests.golden.make_golden import MODEL_CASES
    d = np.load(os.path.join(GOLD, "model_%s.npz" % name))
    eng = CTREngine(ModelSpec(name, **MODEL_CASES[name]), max_batch=64, init="none")
    eng.load_params({k[5:]: d[k] for k in d.files if k.startswith("init/")})
    for i in range(3):
        b = {k.split("/", 1)[1]: d[k] for k in d.files if k.startswith("batch%d/" % i)}
        eng.train_step(b)
        torch.cuda.synchronize()
        np.testing.assert_allclose(eng.z[:64].cpu().numpy(), d["z%d" % i], atol=1e-5, rtol=0)
        assert abs(eng.loss() - d["loss%d" % i][0]) < 1e-5
    got = eng.params()
    for k in got:
        np.testing.assert_allclose(got[k], d["final/" + k], atol=1e-5, rtol=0, err_msg=k)


def _conf(d):
    lines = ["f%d\tx\tfloat" % i for i in range(13)] + ["c%d\tx\tstring" % i for i in range(26)]
    with open(os.path.join(d, "dnn.conf"), "w") as f:
        f.write("\n".join(lines) + "\n")


def test_local_run_train_and_pred_end_to_end(hip_lib, tmp_path):
    from deep_learning_amd.synthetic import make_batch
    from deep_learning_amd.utils import data_loader
    from oracle import ctr_ref as R
    conf, tr, pr = tmp_path / "conf", tmp_path / "train", tmp_path / "pred"
    for p in (conf, tr, pr):
        p.mkdir()
    _conf(str(conf))
    V = 3000
    train_parts = [make_batch(256, cate_index_size=V, seed=i) for i in range(3)]
    pred_part = make_batch(200, cate_index_size=V, seed=99)
    for i, b in enumerate(train_parts):
        data_loader.write_tfrecord_part(str(tr / ("part-%d" % i)), b)
    data_loader.write_tfrecord_part(str(pr / "part-0"), pred_part)
    args = ["deepfm_pipeline", "train", "1", "8", str(V), "3", str(conf), str(tr) + "/", str(pr) + "/",
            str(tmp_path / "model_pb"), str(tmp_path / "ckpt"), "0", str(tmp_path / "ckpt"),
            "batch_size=64", "hidden_units=32,16", "shuffle=0"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "local_run.py")] + args, capture_output=True,
                       text=True, timeout=900, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    out = r.stdout
    assert "val_auc:" in out and "--------------End of dataset-------------" in out
    assert "model training time:" in out and "val of auc:" in out
    auc_gpu = float(out.split("val of auc:")[-1].split()[0])
    assert os.path.exists(tmp_path / "model_pb" / "variables.npz")
    assert any(f.startswith("model-") for f in os.listdir(tmp_path / "ckpt"))
    # pred-only run reproduces the AUC from the export
    r2 = subprocess.run([sys.executable, os.path.join(ROOT, "local_run.py"), "deepfm_pipeline", "pred"] + args[2:],
                        capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert abs(float(r2.stdout.split("val of auc:")[-1].split()[0]) - auc_gpu) < 1e-5
    # oracle on the identical batches, from the exported initial state is not available
    # (random init); instead retrain the oracle from the GPU model's checkpoint-free init:
    # compare the exported model's scores with the oracle forward of the same params.
    d = np.load(tmp_path / "model_pb" / "variables.npz")
    P = {k: d[k] for k in d.files}
    cfg = R.make_cfg("deepfm_pipeline", C=13, V=0, S=26, E=8, cate_index_size=V, hidden=[32, 16])
    b = {k: v[:192] for k, v in pred_part.items()}
    fw = R.forward(cfg, P, b)
    auc_oracle = R.auc(b["label"], fw["p"])
    assert abs(auc_oracle - auc_gpu) < 1e-4


@pytest.mark.parametrize("alg", ["deepfm_multi", "dnn_multi_cate", "deepfm_cate", "dnn_multi"])
def test_local_run_family_models_end_to_end(hip_lib, tmp_path, alg):
    """local_run.py dispatch of the other pipeline-style models (local_run.py:47-62): a conf with
    two multi-hot `arr` columns (feat_size -> multi ranges for the pool algs, plain cate columns
    otherwise), TFRecord parts, train -> export -> pred, exported scores vs the oracle forward."""
    from deep_learning_amd.synthetic import make_batch
    from deep_learning_amd.utils import data_loader, my_utils
    from oracle import ctr_ref as R
    conf, tr, pr = tmp_path / "conf", tmp_path / "train", tmp_path / "pred"
    for p in (conf, tr, pr):
        p.mkdir()
    lines = ["f%d\tx\tfloat" % i for i in range(5)] + ["c%d\tx\tstring" % i for i in range(8)]
    lines += ["tags\tx\tarr\tx\tx\tx\tx\tk=12\ttags", "kw\tx\tarr\tx\tx\tx\tx\tk=7\tkw"]
    with open(str(conf / "dnn.conf"), "w") as f:
        f.write("\n".join(lines) + "\n")
    C, S, Mw = 5, 8, 19
    fs = my_utils.feat_size(str(conf), alg)
    cate_alg = alg in data_loader.CATE_ALGS
    V = 2000
    rng = np.random.default_rng(5)

    def part(n, seed):
        b = make_batch(n, cont=0 if cate_alg else C, cate_fields=S, cate_index_size=V, seed=seed,
                       cate_only=cate_alg)
        multi = rng.integers(1, V, size=(n, Mw))
        multi[rng.random((n, Mw)) < 0.5] = 0
        b["cate_feats"] = np.concatenate([b["cate_feats"], multi], 1)
        return b
    for i in range(3):
        data_loader.write_tfrecord_part(str(tr / ("part-%d" % i)), part(256, i))
    pred_part = part(200, 99)
    data_loader.write_tfrecord_part(str(pr / "part-0"), pred_part)
    args = [alg, "train", "1", "8", str(V), "3", str(conf), str(tr) + "/", str(pr) + "/",
            str(tmp_path / "model_pb"), str(tmp_path / "ckpt"), "0", str(tmp_path / "ckpt"),
            "batch_size=64", "hidden_units=32,16", "shuffle=0"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "local_run.py")] + args, capture_output=True,
                       text=True, timeout=900, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    auc_gpu = float(r.stdout.split("val of auc:")[-1].split()[0])
    d = np.load(tmp_path / "model_pb" / "variables.npz")
    P = {k: d[k] for k in d.files}
    cfg = R.make_cfg(alg, C=fs[0], V=fs[1], S=fs[2], E=8, cate_index_size=V, hidden=[32, 16],
                     multi_ranges=fs[5])
    b = {k: v[:192] for k, v in pred_part.items()}
    fw = R.forward(cfg, P, b)
    assert abs(R.auc(b["label"], fw["p"]) - auc_gpu) < 1e-4


def test_wdl_load_style_fit_evaluate_predict(hip_lib, tmp_path):
    from oracle import ctr_ref as R
    from deep_learning_amd.models import wdl
    from deep_learning_amd.synthetic import make_batch
    from deep_learning_amd.utils import data_loader_load as dll

    class Args:
        hidden_units, epochs, batch_size, learning_rate = [32, 16], 2, 64, 0.001
        model_pb, learning_rate_decay_steps, learning_rate_decay_rate, l2_reg = str(tmp_path / "pb"), 10000000, 0.9, 1e-5
        cont_field_size, cate_field_size, cate_index_size, embedding_size, wide_field_size = 13, 26, 4000, 8, 26
        alg_name, vector_field_size = "wdl", 0
    (tmp_path / "tr").mkdir()
    (tmp_path / "va").mkdir()
    dll.write_lines(str(tmp_path / "tr" / "part-0"), make_batch(300, cate_index_size=4000, seed=1, wide_fields=26))
    dll.write_lines(str(tmp_path / "va" / "part-0"), make_batch(200, cate_index_size=4000, seed=2, wide_fields=26))
    tr = dll.load_input_file(Args, str(tmp_path / "tr"))
    va = dll.load_input_file(Args, str(tmp_path / "va"))
    m = wdl.DeepModel(Args)
    # the training trajectory against the oracle: the epoch losses the fit prints (the
    # device-summed per-step losses, wdl.py:305-313) over two epochs of the same pickled
    # batches (the last one partial: 300 = 4 x 64 + 44) from the engine's own initial state
    eng = m.model_optimizer()
    P = eng.params()
    cfg = R.make_cfg("wdl", C=13, S=26, E=8, cate_index_size=4000, hidden=[32, 16], Fw=26)
    opt = R.AdamTF1(cfg, P)
    for epoch in range(2):
        ref = [R.train_step(cfg, P, opt, m.batch(item))["loss"] for item in tr]
        got, steps = m.train_epoch(tr)
        assert steps == len(ref) == 5
        np.testing.assert_allclose(got, float(np.sum(ref)), rtol=1e-5, err_msg="epoch %d loss sum" % epoch)
    Pg = eng.params()
    for k in P:
        np.testing.assert_allclose(Pg[k], P[k], atol=1e-5, rtol=0, err_msg=k)
    m.fit(tr, va)
    auc_eval = m.evaluate(None, va)
    auc_pred = m.predict(va)
    assert abs(auc_eval - auc_pred) < 1e-6 and 0.0 < auc_pred < 1.0


@pytest.mark.parametrize("alg", ["wdl", "deepfm", "dnn"])
def test_native_pickle_feed_trains_like_the_default_loop(hip_lib, tmp_path, alg, monkeypatch):
    """DLAMD_PINNED_FEED=1: worker threads decode each pickled batch with libdlio's decoder
    (dlio_unpickle_batch, no GIL) straight into pinned buffers and the engine stages them with
    async copies — two epochs over the same batches (the last one partial, lists-of-lists
    batches as the reference's own loader pickles them, and numpy-array batches) end with the
    same parameters, bit for bit, as the default loop's pickle.loads path (and the same epoch
    losses to an f32 unit); the second epoch decodes into the first epoch's pinned ring."""
    import importlib
    import pickle
    from deep_learning_amd.synthetic import make_batch
    from deep_learning_amd.utils import data_loader_load as dll
    mod = importlib.import_module("deep_learning_amd.models." + alg)

    class Args:
        hidden_units, epochs, batch_size, learning_rate = [32, 16], 1, 64, 0.001
        model_pb, learning_rate_decay_steps, learning_rate_decay_rate, l2_reg = str(tmp_path / "pb"), 10000000, 0.9, 1e-5
        cont_field_size, cate_field_size, embedding_size, wide_field_size = 13, 26, 8, 26
        cate_index_size = cate_feats_size = 4000
        vector_feats_size = vector_field_size = 0
        alg_name = alg
    (tmp_path / "tr").mkdir()
    dll.write_lines(str(tmp_path / "tr" / "part-0"),
                    make_batch(300, cate_index_size=4000, seed=1, wide_fields=26 if alg == "wdl" else 0))
    tr = dll.load_input_file(Args, str(tmp_path / "tr"))
    # half the batches re-pickled as the reference's loader writes them: lists of rows
    tr = [pickle.dumps({k: (v.tolist() if hasattr(v, "tolist") else v) for k, v in pickle.loads(it).items()})
          if i % 2 else it for i, it in enumerate(tr)]
    from deep_learning_amd.utils.native_reader import unpickle_batch_into
    m0 = mod.DeepModel(Args)
    f = m0.native_fields()
    outs = [np.zeros((64, sz), np.float32 if kind == 0 else np.int64) for _, _, kind, sz in f]
    assert all(unpickle_batch_into(it, [(k, kind, sz) for k, _, kind, sz in f], outs, 64) is not None for it in tr)
    res = {}
    for feed in ("0", "1"):
        monkeypatch.setenv("DLAMD_PINNED_FEED", feed)
        m = mod.DeepModel(Args)
        losses, ptrs = [], []
        for _ in range(2):
            losses.append(m.train_epoch(tr))
            ring = getattr(m, "_feed_ring", ([], []))[0]
            ptrs.append(sorted(t.data_ptr() for d in ring for t in d.values()))
        if feed == "1":   # the ring's pinned buffers are the model's: the second epoch reuses them
            assert ptrs[0] and ptrs[0] == ptrs[1]
        res[feed] = (losses, m.model_optimizer().params())
    for k in res["0"][1]:
        np.testing.assert_array_equal(res["1"][1][k], res["0"][1][k], err_msg=k)
    # the epoch loss: the same per-step losses, bit for bit (the parameters above are
    # bit-identical, the data term is summed in a fixed order and the regulariser sums are int64
    # fixed point, so the order in which blocks land does not matter: common.h block_fixed_add)
    assert res["1"][0] == res["0"][0], (res["0"][0], res["1"][0])


def test_pinned_feed_bad_id_batch_raises_without_hang(hip_lib, tmp_path, monkeypatch):
    """A DLError raised mid-epoch by the default PinnedFeed loop (a batch with an out-of-range id,
    reported through the status ring a step or two later, while the loop still holds batches)
    propagates as the reference's InvalidArgumentError does: the feed's workers that wait for a
    slot the loop will never release are let go, so the pool's shutdown cannot hang
    (PinnedFeed.close(abort=True)); a later epoch on the same model still trains."""
    import pickle
    import threading
    from deep_learning_amd import _lib
    from deep_learning_amd.models import wdl
    from deep_learning_amd.synthetic import make_batch
    from deep_learning_amd.utils import data_loader_load as dll

    class Args:
        hidden_units, epochs, batch_size, learning_rate = [32, 16], 1, 64, 0.001
        model_pb, learning_rate_decay_steps, learning_rate_decay_rate, l2_reg = str(tmp_path / "pb"), 10000000, 0.9, 1e-5
        cont_field_size, cate_field_size, embedding_size, wide_field_size = 13, 26, 8, 26
        cate_index_size = cate_feats_size = 4000
        vector_feats_size = vector_field_size = 0
        alg_name = "wdl"
    monkeypatch.setenv("DLAMD_PINNED_FEED", "1")
    (tmp_path / "tr").mkdir()
    dll.write_lines(str(tmp_path / "tr" / "part-0"), make_batch(64 * 8, cate_index_size=4000, seed=3, wide_fields=26))
    tr = dll.load_input_file(Args, str(tmp_path / "tr"))
    d = pickle.loads(tr[1])
    d["cate_feats"][5, 3] = 10 ** 7          # batch 1: one id far outside [0, 4000)
    bad = list(tr)
    bad[1] = pickle.dumps(d)
    m = wdl.DeepModel(Args)
    out = {}

    def run():
        try:
            m.train_epoch(bad)
        except Exception as e:   # noqa: BLE001 — the thread reports what ended the epoch
            out["err"] = e
    t = threading.Thread(target=run, daemon=True)
    t.start()
    t.join(60)
    assert not t.is_alive(), "train_epoch hung after the bad-id error"
    assert isinstance(out.get("err"), _lib.DLError) and "InvalidArgumentError" in str(out["err"]), out
    loss, steps = m.train_epoch(tr)
    assert steps == 8 and np.isfinite(loss)


@pytest.mark.parametrize("alg", ["deepfm", "dnn"])
def test_load_style_deepfm_dnn_fit_evaluate_predict(hip_lib, tmp_path, alg):
    """models/deepfm.py and models/dnn.py surfaces over the load-style loader
    (utils/data_loader_load.py): fit prints per epoch, evaluate and predict agree, and
    the exported parameters reproduce the predicted AUC through the oracle forward."""
    import importlib
    from deep_learning_amd.synthetic import make_batch
    from deep_learning_amd.utils import data_loader_load as dll
    from oracle import ctr_ref as R
    mod = importlib.import_module("deep_learning_amd.models." + alg)

    class Args:
        hidden_units, epochs, batch_size, learning_rate = [32, 16], 2, 64, 0.001
        model_pb, learning_rate_decay_steps, learning_rate_decay_rate, l2_reg = str(tmp_path / "pb"), 10000000, 0.9, 1e-4
        cont_field_size, cate_field_size, cate_feats_size, embedding_size = 13, 26, 4000, 8
        vector_feats_size = vector_field_size = 0
        alg_name = alg
    (tmp_path / "tr").mkdir()
    (tmp_path / "va").mkdir()
    dll.write_lines(str(tmp_path / "tr" / "part-0"), make_batch(300, cate_index_size=4000, seed=1))
    va_b = make_batch(192, cate_index_size=4000, seed=2)
    dll.write_lines(str(tmp_path / "va" / "part-0"), va_b)
    tr = dll.load_input_file(Args, str(tmp_path / "tr"))
    va = dll.load_input_file(Args, str(tmp_path / "va"))
    m = mod.DeepModel(Args)
    m.fit(tr, va)
    auc_eval = m.evaluate(None, va)
    auc_pred = m.predict(va)
    assert abs(auc_eval - auc_pred) < 1e-6 and 0.0 < auc_pred < 1.0
    d = np.load(tmp_path / "pb" / "variables.npz")
    P = {k: d[k] for k in d.files}
    cfg = R.make_cfg(alg, C=13, V=0, S=26, E=8, cate_index_size=4000, hidden=[32, 16])
    fw = R.forward(cfg, P, va_b)
    assert abs(R.auc(va_b["label"], fw["p"]) - auc_pred) < 1e-4


def test_tfrecord_two_epoch_trajectory_matches_oracle(hip_lib, tmp_path):
    """The drop-in fit() fed by the native TFRecord reader (utils/data_loader.py:29-40 order:
    shuffle(off) -> batch(drop_remainder) -> repeat(2)) trains on exactly the batches the
    reference iterator yields: 3 part files of 70 + 90 + 50 records at B = 64 give 3 batches per
    epoch (18 records dropped per epoch, never carried into epoch 2).  The oracle trained on those
    reference-ordered batches from the same injected parameters matches every step's logits and
    the final parameters at 1e-5."""
    from deep_learning_amd.local_run import ModelParams
    from deep_learning_amd.models import deepfm_pipeline as M
    from deep_learning_amd.synthetic import make_batch
    from deep_learning_amd.utils import data_loader
    from oracle import ctr_ref as R
    conf, tr, pr = tmp_path / "conf", tmp_path / "train", tmp_path / "pred"
    for p in (conf, tr, pr):
        p.mkdir()
    _conf(str(conf))
    V, Bsz = 3000, 64
    parts = {"part-a": make_batch(70, cate_index_size=V, seed=1), "part-b": make_batch(90, cate_index_size=V, seed=2),
             "part-c": make_batch(50, cate_index_size=V, seed=3)}
    for n, b in parts.items():
        data_loader.write_tfrecord_part(str(tr / n), b)
    data_loader.write_tfrecord_part(str(pr / "part-0"), make_batch(128, cate_index_size=V, seed=9))
    argv = ["local_run.py", "deepfm_pipeline", "train", "2", "8", str(V), "1000", str(conf), str(tr) + "/",
            str(pr) + "/", str(tmp_path / "model_pb"), str(tmp_path / "ckpt"), "0", str(tmp_path / "ckpt"),
            "batch_size=%d" % Bsz, "hidden_units=32,16", "shuffle=0"]
    mp = ModelParams(argv)
    m = M.DeepModel(mp, data_loader.load_input_file(mp, mp.train_path, "train"),
                    data_loader.load_input_file(mp, mp.predict_path, "pred"))
    m.model_optimizer()
    eng = m.engine
    cfg = R.make_cfg("deepfm_pipeline", C=13, V=0, S=26, E=8, cate_index_size=V, hidden=[32, 16])
    P = R.init_params(cfg, np.random.default_rng(17))
    eng.load_params(P)
    zs = []
    inner = eng.train_step

    def hooked(*a, **k):
        r = inner(*a, **k)
        torch.cuda.synchronize()
        zs.append(eng.z[:Bsz].cpu().numpy().copy())
        return r
    eng.train_step = hooked
    m.fit(mp.num_batch_size)
    # the reference's batches: files in get_file_list (directory-listing) order, per epoch
    order = [os.path.basename(f) for f in data_loader.get_file_list(str(tr) + "/")]
    recs = {k: np.concatenate([parts[n][k] for n in order]) for k in parts["part-a"]}
    n_per_epoch = 210 // Bsz
    assert len(zs) == 2 * n_per_epoch
    opt = R.AdamTF1(cfg, P)
    for ep in range(2):
        for j in range(n_per_epoch):
            b = {k: v[j * Bsz:(j + 1) * Bsz] for k, v in recs.items()}
            fw = R.train_step(cfg, P, opt, b)
            np.testing.assert_allclose(zs[ep * n_per_epoch + j], fw["z"], atol=1e-5, rtol=0,
                                       err_msg="epoch %d batch %d" % (ep, j))
    got = eng.params()
    for k in P:
        np.testing.assert_allclose(got[k], P[k], atol=1e-5, rtol=0, err_msg=k)


def test_device_batch_iterator_matches_host_batches(hip_lib, tmp_path):
    """load_input_file(..., device="cuda") yields DEVICE tensors (the reference's get_next()
    tensors, utils/data_loader.py:29-46) with the host iterator's keys, dtypes, shapes and
    values, epoch by epoch (shuffle off, drop_remainder, repeat 2), and trains the drop-in
    model exactly as the host batches do (logits of every step equal)."""
    from deep_learning_amd.local_run import ModelParams
    from deep_learning_amd.models import deepfm_pipeline as M
    from deep_learning_amd.synthetic import make_batch
    from deep_learning_amd.utils import data_loader
    from oracle import ctr_ref as R
    conf, tr = tmp_path / "conf", tmp_path / "train"
    for p in (conf, tr):
        p.mkdir()
    _conf(str(conf))
    V, Bsz = 3000, 64
    for i, n in enumerate((70, 90, 50)):
        data_loader.write_tfrecord_part(str(tr / ("part-%d" % i)), make_batch(n, cate_index_size=V, seed=i + 1))
    argv = ["local_run.py", "deepfm_pipeline", "train", "2", "8", str(V), "1000", str(conf), str(tr) + "/",
            str(tr) + "/", str(tmp_path / "model_pb"), str(tmp_path / "ckpt"), "0", str(tmp_path / "ckpt"),
            "batch_size=%d" % Bsz, "hidden_units=32,16", "shuffle=0"]
    mp = ModelParams(argv)
    host = list(data_loader.load_input_file(mp, mp.train_path, "train"))
    dev = list(data_loader.load_input_file(mp, mp.train_path, "train", device="cuda"))
    assert len(host) == len(dev) == 6     # 3 batches per epoch (210 records // 64), 2 epochs
    for h, d in zip(host, dev):
        assert set(h) == set(d)
        for k in h:
            assert d[k].is_cuda and d[k].dtype == torch.from_numpy(h[k]).dtype and tuple(d[k].shape) == h[k].shape
            np.testing.assert_array_equal(d[k].cpu().numpy(), h[k], err_msg=k)
    cfg = R.make_cfg("deepfm_pipeline", C=13, V=0, S=26, E=8, cate_index_size=V, hidden=[32, 16])
    zs = []
    for batches in (host, dev):
        m = M.DeepModel(mp, batches)
        m.model_optimizer()
        eng = m.engine
        eng.load_params(R.init_params(cfg, np.random.default_rng(3)))
        out = []
        for b in batches:
            eng.train_step(b)
            torch.cuda.synchronize()
            out.append(eng.z[:Bsz].cpu().numpy().copy())
        zs.append(out)
    for a, b in zip(*zs):
        np.testing.assert_array_equal(a, b)
