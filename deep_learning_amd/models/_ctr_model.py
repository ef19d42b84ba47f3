"""Shared implementation of the reference's DeepModel surface on the MI355X engine.

The reference builds one TF-1.x graph per model file (models/deepfm_pipeline.py,
dnn_pipeline.py, deepfm_multi_cate.py) with the same public surface:

    DeepModel(args, data_dict)                 (deepfm_pipeline.py:16)
    .model_optimizer() -> (loss, train_op, global_step)      (:176-191)
    .fit(print_num_batch, predict_data)        (:193-265)
    DeepModel.get_val_data(sess, data)         (:267-292, staticmethod)
    .eval(sess, val_data) -> auc               (:294-311)
    predict(predict_data, model_pb)            (:314-346, module level)

Here the graph is the HIP engine (deep_learning_amd/engine.py).  Both call forms
in the reference's runners work: ``DeepModel(mp, train, pred)`` + ``fit(n)``
(local_run.py:74-76) and ``DeepModel(mp, train)`` + ``fit(n, pred)``
(local_run_test.py:77-79).  ``sess`` arguments are accepted and ignored.
Printed lines follow the reference formats (log-scrape parity).
Checkpoints / exported models are this package's own format (npz + JSON with the
reference's signature names: cont_feats, cate_feats, vector_feats,
input_data_size -> score); TF checkpoint/SavedModel byte-compatibility is out of scope.
"""
import glob
import json
import os
import re
import sys
import time

import numpy as np
import torch

import inspect

from ..engine import FAMILIES, CTREngine, ModelSpec, default_adam
from ..metrics import AucAccumulator


def _spec_from_args(model, args):
    hidden = [int(h) for h in args.hidden_units]
    kw = dict(E=int(args.embedding_size), cate_index_size=int(args.cate_feats_size), hidden=hidden,
              lr=float(args.learning_rate), l2=float(args.l2_reg),
              decay_steps=float(args.learning_rate_decay_steps), decay_rate=float(args.learning_rate_decay_rate),
              V=int(getattr(args, "vector_feats_size", 0)))
    kw.update(S=int(args.cate_field_size), C=int(getattr(args, "cont_field_size", 0) or 0))
    if FAMILIES[model]["multi"]:   # slot ranges within the multi block (my_utils.feat_size)
        kw.update(multi_ranges=[list(r) for r in args.multi_feats_range])
    return ModelSpec(model, **kw)


class CTRModel:
    MODEL = None  # set by the per-file subclasses

    def __init__(self, args, data_dict, predict_data=None):
        self.args = args
        self.epochs = args.epochs
        self.batch_size = int(args.batch_size)
        self.model_pb = args.model_pb
        self.save_model_checkpoint = args.save_model_checkpoint
        self.restore_model_checkpoint = args.restore_model_checkpoint
        self.model_restore = args.model_restore
        self.metric_type = "auc"
        self.random_seed = 2019
        self.data_dict = data_dict
        self.predict_data = predict_data
        self.spec = _spec_from_args(self.MODEL, args)
        self.engine = None
        self.global_step = 0

    # --------------------------------------------------------------- graph
    def model_optimizer(self):
        """Builds the engine (the reference builds the graph here): returns
        (loss_fn, train_fn, global_step_fn)."""
        if self.engine is None:
            self.engine = CTREngine(self.spec, max_batch=self.batch_size, seed=self.random_seed,
                                    adam=default_adam(self.spec))
        eng = self.engine
        return (eng.loss, lambda batch, next_batch=None: eng.train_step(batch, graph=True, next_batch=next_batch),
                lambda: eng.steps)

    # --------------------------------------------------------------- training
    def fit(self, print_num_batch, predict_data=None):
        loss_fn, train_fn, _ = self.model_optimizer()
        predict_data = predict_data if predict_data is not None else self.predict_data
        if self.model_restore == 1:
            try:
                self._restore(self.restore_model_checkpoint)
                print("@_@~ Old Model Restored Successfully!")
            except Exception as e:
                print("=_=!! Error: There is no model checkpoint in %s" % self.restore_model_checkpoint)
                print(e)
                sys.exit(-1)
        val_data = self.get_val_data(None, predict_data) if predict_data is not None else [[], [], [], []]
        print("Start of training")
        start_time = time.time()
        batch_count = 0
        i = 0
        feed = _Feed(self.data_dict)
        for batch, nxt in feed:
            train_fn(batch, nxt)
            feed.mark(self.engine)
            if batch_count == print_num_batch:
                batch_end_time = time.time()
                loss = loss_fn()
                auc = self.eval(None, val_data)
                print("[{}] val_auc:{}\t loss:{} time:{:.2f}s".format(i, auc, loss, batch_end_time - start_time))
                sys.stdout.flush()
                start_time = time.time()
                batch_count = 0
            batch_count += 1
            i += 1
        print("--------------End of dataset-------------")
        self.engine.check_error()
        print("--------------save checkpoint model-------------")
        if self.save_model_checkpoint:
            self._save_checkpoint(self.save_model_checkpoint)
        print("--------------save pb model-------------")
        try:
            export_model(self.engine, self.model_pb)
        except Exception as e:
            print("Fail to export saved model, exception: {}".format(e))
            sys.stdout.flush()

    @staticmethod
    def get_val_data(sess, data):
        labels, cont, cate, vec = [], [], [], []
        for b in data:
            labels.append(b["label"])
            cont.append(b.get("cont_feats"))
            cate.append(b["cate_feats"])
            vec.append(b.get("vector_feats"))
        return [labels, cont, cate, vec]

    def eval(self, sess, val_data):
        if self.engine is None:
            self.model_optimizer()
        acc = AucAccumulator()
        for i in range(len(val_data[0])):
            batch = {"label": val_data[0][i], "cate_feats": val_data[2][i]}
            if val_data[1][i] is not None:
                batch["cont_feats"] = val_data[1][i]
            if val_data[3][i] is not None:
                batch["vector_feats"] = val_data[3][i]
            acc.add(val_data[0][i], _predict_batches(self.engine, batch))
        return acc.result()

    # --------------------------------------------------------------- checkpoints
    def _save_checkpoint(self, directory):
        os.makedirs(directory, exist_ok=True)
        eng = self.engine
        state = {"param/" + k: v for k, v in eng.params().items()}
        state.update(_adam_state(eng))
        path = os.path.join(directory, "model-%d.npz" % eng.steps)
        for old in glob.glob(os.path.join(directory, "model-*.npz")):   # Saver(max_to_keep=1)
            os.remove(old)
        np.savez(path, **state)

    def _restore(self, directory):
        files = glob.glob(os.path.join(directory, "model-*.npz"))
        if not files:
            raise FileNotFoundError("no checkpoint in %s" % directory)
        path = max(files, key=lambda f: int(re.findall(r"model-(\d+)\.npz", f)[0]))
        d = np.load(path, allow_pickle=False)
        P = {k[len("param/"):]: d[k] for k in d.files if k.startswith("param/")}
        self.engine.load_params(P)
        _load_adam_state(self.engine, d)


def _adam_state(eng):
    out = {"adam/opt": eng.opt.cpu().numpy(), "adam/steps": np.array([eng.steps])}
    out.update({"adam/table_" + k: v for k, v in eng.adam_state().items()})
    out["adam/hm"], out["adam/hv"] = eng.hm.cpu().numpy(), eng.hv.cpu().numpy()
    for l in range(len(eng.W)):
        out["adam/Wm%d" % l] = eng.Wm[l].cpu().numpy()
        out["adam/Wv%d" % l] = eng.Wv[l].cpu().numpy()
    return out


def _load_adam_state(eng, d):
    eng.set_opt(torch.from_numpy(d["adam/opt"]))
    eng.steps = int(d["adam/steps"][0])
    eng.set_adam_state({k[len("adam/table_"):]: d[k] for k in d.files if k.startswith("adam/table_")})
    eng.hm.copy_(torch.from_numpy(d["adam/hm"]))
    eng.hv.copy_(torch.from_numpy(d["adam/hv"]))
    for l in range(len(eng.W)):
        eng.Wm[l].copy_(torch.from_numpy(d["adam/Wm%d" % l]))
        eng.Wv[l].copy_(torch.from_numpy(d["adam/Wv%d" % l]))


class _Feed:
    """Training batches as (batch, next batch) pairs.  From the native TFRecord reader the
    batches are decoded into pinned host buffers (PinnedFeed) and the next one is handed to
    train_step as next_batch, so its upload and index build run on the engine's side
    stream during the current step.  Other iterables (lists, generators) pass through
    with no lookahead."""

    def __init__(self, data):
        from ..utils.native_reader import NativeReader, PinnedFeed
        self.it = iter(data)
        self.pinned = PinnedFeed(self.it) if isinstance(self.it, NativeReader) else None
        self.pair = None

    def __iter__(self):
        if self.pinned is None:
            for b in self.it:
                yield b, None
            return
        cur = self.pinned.next()
        while cur is not None:
            nxt = self.pinned.next()
            self.pair = (cur, nxt)
            yield cur, nxt
            cur = nxt

    def mark(self, eng):
        """After train_step(cur, next_batch=nxt): cur's buffers were read by copies queued on
        the compute stream (or by an earlier prefetch), nxt's by the side-stream prefetch."""
        if self.pinned is None or self.pair is None:
            return
        cur, nxt = self.pair
        ev = torch.cuda.Event()
        ev.record()
        self.pinned.mark(cur, ev)
        if nxt is not None and getattr(eng, "_pf", None) is not None:
            self.pinned.mark(nxt, eng._pf[2])


def _predict_batches(eng, batch, logits=False):
    """Forward in chunks of the engine's max batch; returns the scores (or logits) as one
    device tensor."""
    n = np.asarray(batch["label"]).shape[0]
    out = []
    for s in range(0, n, eng.B):
        part = {k: np.asarray(v)[s:s + eng.B] for k, v in batch.items()}
        out.append(eng.predict(part, logits=logits, device=True))
    return torch.cat(out) if len(out) > 1 else out[0]


SIGNATURE = {"inputs": ["cont_feats", "cate_feats", "vector_feats", "input_data_size"], "outputs": ["score"],
             "method_name": "tensorflow/serving/predict"}


def export_model(eng, model_pb):
    """The SavedModel export of deepfm_pipeline.py:243-262, in this package's format."""
    os.makedirs(model_pb, exist_ok=True)
    sp = eng.spec
    meta = dict(SIGNATURE, model=sp.model, spec={k: v for k, v in sp.__dict__.items()}, batch_size=eng.B)
    with open(os.path.join(model_pb, "signature.json"), "w") as f:
        json.dump(meta, f, indent=1)
    np.savez(os.path.join(model_pb, "variables.npz"), **eng.params())


def load_model(model_pb, max_batch=None):
    with open(os.path.join(model_pb, "signature.json")) as f:
        meta = json.load(f)
    keys = set(inspect.signature(ModelSpec.__init__).parameters) - {"self", "model"}
    spec = ModelSpec(meta["model"], **{k: v for k, v in meta["spec"].items() if k in keys})
    eng = CTREngine(spec, max_batch=max_batch or meta["batch_size"], init="none", adam=default_adam(spec))
    d = np.load(os.path.join(model_pb, "variables.npz"), allow_pickle=False)
    eng.load_params({k: d[k] for k in d.files})
    return eng


def predict(predict_data, model_pb):
    """Loads the exported model and scores predict_data (deepfm_pipeline.py:314-346)."""
    eng = None
    acc = AucAccumulator()
    for b in predict_data:
        if eng is None:
            eng = load_model(model_pb, max_batch=np.asarray(b["label"]).shape[0])
        acc.add(b["label"], _predict_batches(eng, b))
    print("-----------end of data_set-----------")
    auc = acc.result()
    print("val of auc:%.5f" % auc)
    sys.stdout.flush()
    print('---end---')
    return auc
