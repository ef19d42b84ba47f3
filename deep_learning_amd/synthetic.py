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


def make_batch_device(B, cont=13, vector=0, cate_fields=26, cate_index_size=26_000_000, multi_slots=0,
                      multi_width=60, wide_fields=0, seed=2019, cate_only=False, device="cuda"):
    """The same distributions as make_batch (uniform ids only), drawn on the device with a
    seeded torch generator: fresh batches every bench step cost no host time (a host draw of
    one C3 batch takes ~0.3 s).  Values differ from make_batch's for the same seed; keys,
    dtypes and shapes are the reference loader's (utils/data_loader.py:12-24)."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    S = cate_fields
    per_field = max(2, cate_index_size // max(1, S + multi_slots))
    span = per_field - 1
    out = {}
    dense = None
    if cont > 0 and not cate_only:
        c = torch.empty(B, cont, device=device).exponential_(0.1, generator=g).log1p_()
        out["cont_feats"] = c
        dense = c / 4.0
    elif not cate_only:
        out["cont_feats"] = torch.zeros(B, 0, device=device)
    out["vector_feats"] = torch.randn(B, vector, device=device, generator=g) * 0.1
    lo = torch.arange(S, device=device, dtype=torch.int64) * per_field + 1
    cols = [lo + torch.randint(0, span, (B, S), device=device, generator=g)]
    for m in range(multi_slots):
        ids = (S + m) * per_field + 1 + torch.randint(0, span, (B, multi_width), device=device, generator=g)
        ln = torch.randint(1, multi_width, (B, 1), device=device, generator=g)
        ids[torch.arange(multi_width, device=device)[None, :] >= ln] = 0
        cols.append(ids)
    cate = torch.cat(cols, 1).contiguous()
    out["cate_feats"] = cate
    tw = ((cate[:, :S] * 2654435761) % 1000).double() / 1000.0 - 0.5
    logit = tw.sum(1) * 0.6 - 1.1
    if dense is not None:
        logit = logit + dense.double() @ torch.linspace(-0.5, 0.5, dense.shape[1], device=device, dtype=torch.float64)
    p = torch.sigmoid(logit)
    out["label"] = (torch.rand(B, device=device, generator=g, dtype=torch.float64) < p).float().reshape(B, 1)
    if wide_fields:
        f = torch.arange(wide_fields, device=device, dtype=torch.int64) % max(S, 1)
        out["wide_feats"] = (f * per_field + 1 + torch.randint(0, span, (B, wide_fields), device=device,
                                                                generator=g)).contiguous()
    return out
