"""Exact ROC-AUC with ties on the GPU (``dl_auc``, csrc/metrics.hip) — the semantics of
sklearn.metrics.roc_auc_score, which the reference calls on the collected scores
(models/deepfm_pipeline.py:311,344; wdl.py:343-358; deepfm.py:229; dnn.py:147-161).

Scores stay on the device: the eval/predict loops hand their per-batch score tensors to
an :class:`AucAccumulator` and one ``dl_auc`` call sorts and counts them.  Like sklearn,
a label set with a single class raises ``ValueError``.
"""
import numpy as np
import torch

from . import _lib
from ._lib import call, ptr

_SINGLE_CLASS = "Only one class present in y_true. ROC AUC score is not defined in that case."


def _dev_f32(x):
    if isinstance(x, torch.Tensor):
        return x.detach().to(device="cuda", dtype=torch.float32).reshape(-1).contiguous()
    return torch.from_numpy(np.ascontiguousarray(np.asarray(x, np.float32).reshape(-1))).cuda()


def roc_auc(labels, scores):
    """AUC of scores (host arrays/lists or device tensors) against 0/1 labels."""
    s, y = _dev_f32(scores), _dev_f32(labels)
    if s.numel() != y.numel():
        raise ValueError("labels and scores differ in length")
    n = s.numel()
    if n == 0:
        raise ValueError(_SINGLE_CLASS)
    ws = torch.empty(int(_lib.lib().dl_auc_workspace_bytes(n)), dtype=torch.uint8, device="cuda")
    out = torch.empty(1, dtype=torch.float64, device="cuda")
    call("dl_auc", ptr(s), 1, ptr(y), 1, n, ptr(ws), ws.numel(), ptr(out), _lib.stream_handle())
    v = float(out.item())
    if v != v:
        raise ValueError(_SINGLE_CLASS)
    return v


class AucAccumulator:
    """Collects device score and label tensors batch by batch; ``result()`` is one dl_auc."""

    def __init__(self):
        self.scores, self.labels = [], []

    def add(self, labels, scores):
        self.scores.append(_dev_f32(scores))
        self.labels.append(_dev_f32(labels))

    def result(self):
        if not self.scores:
            raise ValueError(_SINGLE_CLASS)
        return roc_auc(torch.cat(self.labels), torch.cat(self.scores))
