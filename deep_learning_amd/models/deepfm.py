"""Drop-in for the reference's models/deepfm.py (DeepFM, load-style surface).

    DeepModel(args)                      (deepfm.py:15-37)
    .model_optimizer()                   (:146-162)
    .fit(train_data, val_data)           (:164-214) lists of pickled batch dicts
    .evaluate(sess, data_val) -> auc     (:216-232, AUC of the pre-sigmoid output self.out)
    .predict(data_val)                   (:234-255) from the exported model

Math (engine, model "deepfm"): tables feats_emb ~ N(0, 0.01) and feats ~ U[0, 1) over
cont_field_size + cate_feats_size rows with NO zero row (:56-60); FM fields are
[cate ids (value 1) | cont (row cate_field_size + j, value cont)] (:62-73: the cont rows
sit at the field count, aliasing cate ids in [S, S + C)); deep input [cont, vector,
V[cate]] (:98); head [first | second | deep] (:131); eps-log-loss + L2 on the head
weights (:151-155); TF1 Adam.
"""
import numpy as np

from ..engine import ModelSpec
from ._load_style import LoadStyleModel, unpickle


class DeepModel(LoadStyleModel):
    EVAL_OUTPUT = "logit"

    def make_spec(self, args):
        self.embedding_size = int(args.embedding_size)
        self.cont_field_size = int(args.cont_field_size)
        self.vector_field_size = int(args.vector_feats_size)
        self.cate_field_size = int(args.cate_field_size)
        self.cate_feats_size = int(args.cate_feats_size)
        return ModelSpec("deepfm", C=self.cont_field_size, V=self.vector_field_size, S=self.cate_field_size,
                         E=self.embedding_size, cate_index_size=self.cate_feats_size, hidden=self.hidden_units,
                         lr=float(args.learning_rate), l2=float(args.l2_reg),
                         decay_steps=float(args.learning_rate_decay_steps),
                         decay_rate=float(args.learning_rate_decay_rate))

    def native_fields(self):
        f = [("labels", "label", 0, 1), ("cont_feats", "cont_feats", 0, self.cont_field_size),
             ("cate_feats", "cate_feats", 1, self.cate_field_size)]
        return f + ([("vector_feats", "vector_feats", 0, self.vector_field_size)] if self.vector_field_size else [])

    def native_extra(self, rows):
        return {} if self.vector_field_size else {"vector_feats": np.zeros((rows, 0), np.float32)}

    def batch(self, item):
        d = unpickle(item)
        B = len(d["labels"])
        return {"label": np.asarray(d["labels"], np.float32).reshape(B, 1),
                "cont_feats": np.asarray(d["cont_feats"], np.float32).reshape(B, self.cont_field_size),
                "vector_feats": np.asarray(d["vector_feats"], np.float32).reshape(B, self.vector_field_size),
                "cate_feats": np.asarray(d["cate_feats"], np.int64)}   # tf.int32 placeholder (:44)
