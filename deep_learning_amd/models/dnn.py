"""Drop-in for the reference's models/dnn.py (DNN, load-style surface).

    DeepModel(args)                      (dnn.py:15-33; the graph is built in the constructor)
    .fit(train_data, val_data)           (:98-145) lists of pickled batch dicts
    .evaluate(sess, data_val) -> auc     (:147-161)
    .predict(data_val)                   (:163-185) from the exported model

Math (engine, model "dnn"): xavier table weight_mat [cate_feats_size, E] with no zero
row (:49-52); deep input [cont_feats (cont_field_size + vector_feats_size columns, :28),
V[cate]] (:56); output layer deep_res (:74-78); eps-log-loss on the sigmoid plus
l1_regularizer(l2_reg) on every hidden weight matrix (:82-90; no term on deep_res);
TF1 Adam.
"""
import numpy as np

from ..engine import ModelSpec
from ._load_style import LoadStyleModel, unpickle


class DeepModel(LoadStyleModel):
    def make_spec(self, args):
        self.cont_field_size = int(args.cont_field_size) + int(args.vector_feats_size)
        self.cate_field_size = int(args.cate_field_size)
        self.cate_feats_size = int(args.cate_feats_size)
        self.embedding_size = int(args.embedding_size)
        return ModelSpec("dnn", C=self.cont_field_size, V=0, S=self.cate_field_size, E=self.embedding_size,
                         cate_index_size=self.cate_feats_size, hidden=self.hidden_units,
                         lr=float(args.learning_rate), l2=float(args.l2_reg),
                         decay_steps=float(args.learning_rate_decay_steps),
                         decay_rate=float(args.learning_rate_decay_rate))

    def native_fields(self):
        return [("labels", "label", 0, 1), ("cont_feats", "cont_feats", 0, self.cont_field_size),
                ("cate_feats", "cate_feats", 1, self.cate_field_size)]

    def batch(self, item):
        d = unpickle(item)
        B = len(d["labels"])
        return {"label": np.asarray(d["labels"], np.float32).reshape(B, 1),
                "cont_feats": np.asarray(d["cont_feats"], np.float32).reshape(B, self.cont_field_size),
                "cate_feats": np.asarray(d["cate_feats"], np.int64)}
