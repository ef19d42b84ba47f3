"""Drop-in for the reference's models/wdl.py (Wide&Deep, load-style surface).

    DeepModel(args)                      (wdl.py:19-51; args as built by local_run_textline.py:45-67)
    .model_optimizer()                   (:261-285)
    .fit(train_data, val_data)           (:287-341) lists of pickled batch dicts
    .evaluate(sess, data_val) -> auc     (:343-358)
    .predict(data_val)                   (:360-384) from the exported model

Math (engine, model "wdl"): xavier embedding table with no zero row, deep tower
over [cont, V[cate]], cross logit sum_f w[wide_f] + sum_j w[Fw+j] h_j + b with the
deep-output weights aliasing wide rows (wdl.py:225-253), eps-log-loss, L2 on
wdl_weights and every hidden weight matrix (:269-275), TF1 Adam.  The deep tower
runs the fp32 MFMA GEMMs (the reference's numerics) unless ``args.tower_dtype == "bf16"``
(BASELINE config C5: bf16 MFMA tower, fp32 master weights and fp32 wide cross logit).
"""
import pickle
import sys
import time

import numpy as np

from ..engine import CTREngine, ModelSpec, default_adam
from ..metrics import roc_auc
from ._ctr_model import _predict_batches, export_model, load_model


def _batch(item):
    d = pickle.loads(item) if isinstance(item, (bytes, bytearray)) else item
    return {"label": np.asarray(d["labels"], np.float32).reshape(-1, 1),
            "cont_feats": np.asarray(d["cont_feats"], np.float32),
            "cate_feats": np.asarray(d["cate_feats"], np.int64),
            "wide_feats": np.asarray(d["wide_feats"], np.int64)}


class DeepModel:
    def __init__(self, args):
        self.hidden_units = [int(h) for h in args.hidden_units]
        self.epochs = int(args.epochs)
        self.batch_size = int(args.batch_size)
        self.learning_rate = args.learning_rate
        self.model_pb = args.model_pb
        self.l2_reg = args.l2_reg
        self.metric_type = "auc"
        self.random_seed = 2019
        self.cont_field_size = int(args.cont_field_size)
        self.cate_field_size = int(args.cate_field_size)
        self.cate_index_size = int(args.cate_index_size)
        self.embedding_size = int(args.embedding_size)
        self.wide_feats_field_size = int(args.wide_field_size)
        self.spec = ModelSpec("wdl", C=self.cont_field_size, S=self.cate_field_size, E=self.embedding_size,
                              cate_index_size=self.cate_index_size, hidden=self.hidden_units,
                              Fw=self.wide_feats_field_size, lr=float(args.learning_rate), l2=float(args.l2_reg),
                              decay_steps=float(args.learning_rate_decay_steps),
                              decay_rate=float(args.learning_rate_decay_rate),
                              tower=str(getattr(args, "tower_dtype", "f32")))
        self.engine = None

    def model_optimizer(self):
        if self.engine is None:
            self.engine = CTREngine(self.spec, max_batch=self.batch_size, seed=self.random_seed,
                                    adam=default_adam(self.spec))
        return self.engine

    def fit(self, train_data, val_data):
        eng = self.model_optimizer()
        losses = []
        num_samples = 0
        for epoch in range(self.epochs):
            st = time.time()
            for item in train_data:
                b = _batch(item)
                eng.train_step(b, graph=b["label"].shape[0] == eng.B)
                losses.append(eng.loss() * self.batch_size)
                num_samples += self.batch_size
            end_time = time.time()
            total_loss = float(np.sum(losses) / num_samples)
            valid_metric = self.evaluate(None, val_data)
            print('[%s] valid-%s=%.5f\tloss=%.5f [%.1f s]' % (epoch + 1, self.metric_type, valid_metric,
                                                               total_loss, end_time - st))
            sys.stdout.flush()
        eng.check_error()
        try:
            export_model(eng, self.model_pb)
        except Exception as e:
            print("Fail to export saved model, exception: {}".format(e))
            sys.stdout.flush()

    def evaluate(self, sess, data_val):
        eng = self.model_optimizer()
        preds, labels = [], []
        for item in data_val:
            b = _batch(item)
            labels.extend(b["label"].reshape(-1).tolist())
            preds.extend(_predict_batches(eng, b))
        return roc_auc(labels, preds)

    def predict(self, data_val):
        eng = load_model(self.model_pb, max_batch=self.batch_size)
        preds, labels = [], []
        for item in data_val:
            b = _batch(item)
            labels.extend(b["label"].reshape(-1).tolist())
            preds.extend(_predict_batches(eng, b))
        auc = roc_auc(labels, preds)
        print("val of auc:%.5f" % auc)
        sys.stdout.flush()
        print('---end---')
        return auc
