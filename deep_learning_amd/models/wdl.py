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
import numpy as np

from ..engine import ModelSpec
from ._load_style import LoadStyleModel, unpickle


class DeepModel(LoadStyleModel):
    def make_spec(self, args):
        self.cont_field_size = int(args.cont_field_size)
        self.cate_field_size = int(args.cate_field_size)
        self.cate_index_size = int(args.cate_index_size)
        self.embedding_size = int(args.embedding_size)
        self.wide_feats_field_size = int(args.wide_field_size)
        return ModelSpec("wdl", C=self.cont_field_size, S=self.cate_field_size, E=self.embedding_size,
                         cate_index_size=self.cate_index_size, hidden=self.hidden_units,
                         Fw=self.wide_feats_field_size, lr=float(args.learning_rate), l2=float(args.l2_reg),
                         decay_steps=float(args.learning_rate_decay_steps),
                         decay_rate=float(args.learning_rate_decay_rate),
                         tower=str(getattr(args, "tower_dtype", "f32")))

    def native_fields(self):
        sp = self.spec
        return [("labels", "label", 0, 1), ("cont_feats", "cont_feats", 0, sp.C), ("cate_feats", "cate_feats", 1, sp.S),
                ("wide_feats", "wide_feats", 1, sp.Fw)]

    def batch(self, item):
        d = unpickle(item)
        return {"label": np.asarray(d["labels"], np.float32).reshape(-1, 1),
                "cont_feats": np.asarray(d["cont_feats"], np.float32),
                "cate_feats": np.asarray(d["cate_feats"], np.int64),
                "wide_feats": np.asarray(d["wide_feats"], np.int64)}
