"""Drop-in for the reference's models/dnn_multi.py (deep tower over [cont, vector, cate embeddings, pooled multi-hot slots], output layer deep_res).

Same surface: DeepModel(args, data_dict[, predict_data]), .fit, .eval,
DeepModel.get_val_data, .model_optimizer, module-level predict(predict_data, model_pb).
Implementation: deep_learning_amd/models/_ctr_model.py on the MI355X engine.
"""
from ._ctr_model import CTRModel, predict  # noqa: F401


class DeepModel(CTRModel):
    MODEL = "dnn_multi"
