"""Drop-in for the reference's models/deepfm_cate.py (DeepFM over the categorical fields only: FM over S cate fields, deep input [vector, cate embeddings]).

Same surface: DeepModel(args, data_dict[, predict_data]), .fit, .eval,
DeepModel.get_val_data, .model_optimizer, module-level predict(predict_data, model_pb).
Implementation: deep_learning_amd/models/_ctr_model.py on the MI355X engine.
"""
from ._ctr_model import CTRModel, predict  # noqa: F401


class DeepModel(CTRModel):
    MODEL = "deepfm_cate"
