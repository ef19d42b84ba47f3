"""Exact ROC-AUC with ties (the semantics of sklearn.metrics.roc_auc_score, which the
reference calls at models/deepfm_pipeline.py:311,344).  Rank statistic form:
AUC = (sum over negatives of [#positives ranked above + 0.5 * #positives tied]) / (P * N).
"""
import numpy as np


def roc_auc(labels, scores):
    y = np.asarray(labels, np.float64).reshape(-1)
    s = np.asarray(scores, np.float64).reshape(-1)
    if y.size != s.size:
        raise ValueError("labels and scores differ in length")
    pos = y > 0.5
    P = int(pos.sum())
    N = y.size - P
    if P == 0 or N == 0:
        raise ValueError("Only one class present in y_true. ROC AUC score is not defined in that case.")
    order = np.argsort(s, kind="mergesort")
    s_sorted = s[order]
    # average ranks over ties (1-based)
    starts = np.r_[0, np.flatnonzero(np.diff(s_sorted)) + 1]
    ends = np.r_[starts[1:], s.size]
    avg = (starts + ends + 1) / 2.0
    ranks = np.empty(s.size)
    ranks[order] = np.repeat(avg, ends - starts)
    return float((ranks[pos].sum() - P * (P + 1) / 2.0) / (P * N))
