"""Seeded synthetic Criteo-shaped batches (SURVEY.md §8(d) "Synthetic inputs").

Dense features: log1p(Exponential(scale=10)) as float32.
Categorical field f: ids in [f*Vf + 1, (f+1)*Vf - 1] (id 0 is padding only),
drawn uniform (worst-case gather) or Zipf(alpha) over a seeded per-field
permutation.  Multi-hot slots: width L, valid length ~ U[1, L-1], padded with 0.
Labels ~ Bernoulli(sigmoid(teacher . features)) with base rate ~0.25.
"""
import numpy as np


def _field_ids(rng, B, field, per_field, dist, alpha, perm_cache):
    lo = field * per_field + 1
    span = per_field - 1
    if dist == "uniform":
        return lo + rng.integers(0, span, size=B, dtype=np.int64)
    # Zipf over a seeded permutation of the field's id range.
    r = rng.zipf(alpha, size=B).astype(np.int64) - 1
    r = np.minimum(r, span - 1)
    key = (field, span)
    if key not in perm_cache:
        prng = np.random.default_rng(1000 + field)
        perm_cache[key] = prng.permutation(span).astype(np.int64)
    return lo + perm_cache[key][r]


def make_batch(B, cont=13, vector=0, cate_fields=26, cate_index_size=26_000_000, multi_slots=0,
               multi_width=60, wide_fields=0, seed=2019, dist="uniform", alpha=1.1,
               cate_only=False, with_cont=True):
    """Returns a dict of numpy arrays with the reference loader's keys
    (utils/data_loader.py:12-24): label [B,1] f32, cont_feats [B,C] f32,
    vector_feats [B,V] f32, cate_feats [B, S + M*L] int64 (+ wide_feats for wdl)."""
    rng = np.random.default_rng(seed)
    perm = {}
    S = cate_fields
    per_field = max(2, cate_index_size // max(1, S + multi_slots))
    out = {}
    feats = []
    if with_cont and cont > 0 and not cate_only:
        c = np.log1p(rng.exponential(10.0, size=(B, cont))).astype(np.float32)
        out["cont_feats"] = c
        feats.append(c / 4.0)
    elif not cate_only:
        out["cont_feats"] = np.zeros((B, 0), np.float32)
    out["vector_feats"] = rng.standard_normal((B, vector)).astype(np.float32) * 0.1
    cols = [_field_ids(rng, B, f, per_field, dist, alpha, perm) for f in range(S)]
    for m in range(multi_slots):
        f = S + m
        L = multi_width
        ids = np.stack([_field_ids(rng, B, f, per_field, dist, alpha, perm) for _ in range(L)], 1)
        ln = rng.integers(1, L, size=B)
        ids[np.arange(L)[None, :] >= ln[:, None]] = 0
        cols.append(ids)
    cate = np.concatenate([c.reshape(B, -1) for c in cols], 1).astype(np.int64)
    out["cate_feats"] = cate
    # teacher: per-id hash weight + dense weights
    tw = ((cate[:, :S] * 2654435761) % 1000).astype(np.float64) / 1000.0 - 0.5
    logit = tw.sum(1) * 0.6 - 1.1
    for f in feats:
        logit += f @ np.linspace(-0.5, 0.5, f.shape[1])
    p = 1.0 / (1.0 + np.exp(-logit))
    out["label"] = (rng.random(B) < p).astype(np.float32).reshape(B, 1)
    if wide_fields:
        out["wide_feats"] = np.stack(
            [_field_ids(rng, B, f % max(S, 1), per_field, dist, alpha, perm) for f in range(wide_fields)], 1)
    return out
