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


class ShardedAucAccumulator(AucAccumulator):
    """AUC over every rank's scores (row-sharded eval, shard.py): the local device scores and
    labels are all-gathered (padded to the largest rank's count) and dl_auc runs on the global
    concatenation, so every rank gets the single-GPU value of the whole set."""

    def __init__(self, exch):
        super().__init__()
        self.exch = exch

    def result(self):
        import torch.distributed as dist
        ex = self.exch
        s = torch.cat(self.scores) if self.scores else torch.empty(0, device="cuda")
        y = torch.cat(self.labels) if self.labels else torch.empty(0, device="cuda")
        dev = "cpu" if ex.staged else "cuda"
        n = torch.tensor([s.numel()], dtype=torch.int64, device=dev)
        ns = [torch.empty_like(n) for _ in range(ex.world)]
        dist.all_gather(ns, n, group=ex.group)
        counts = [int(c.item()) for c in ns]
        cap = max(counts)
        if cap == 0:
            raise ValueError(_SINGLE_CLASS)
        pad = torch.zeros(2, cap, dtype=torch.float32, device=dev)
        pad[0, : s.numel()] = s.to(dev)
        pad[1, : y.numel()] = y.to(dev)
        parts = [torch.empty_like(pad) for _ in range(ex.world)]
        dist.all_gather(parts, pad, group=ex.group)
        scores = torch.cat([p[0, :c] for p, c in zip(parts, counts)])
        labels = torch.cat([p[1, :c] for p, c in zip(parts, counts)])
        return roc_auc(labels, scores)
