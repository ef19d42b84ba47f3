#!/usr/bin/env python
"""Headline benchmark: DeepFM training throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--dist uniform|zipf] [--no-cpu-baseline]

Workload (BASELINE.json configs[1], "C2"): deepfm_pipeline, 13 dense + 26
categorical fields x 1M vocab each (table 26,000,013 x 16 fp32), MLP
[400,400,400], batch 65,536 per GPU, fp32, TF1-dense Adam.  One step = one full
training step (embedding gather + FM + MLP fwd/bwd + log-loss + Adam over every
table row) on a synthetic batch already resident in HBM (a fresh one per step,
drawn on the device before the timed region).  The timed region replays the
hipGraph of the step K times, bracketed by barrier + synchronize.

Then, inside the same run, a few eager steps are bracketed per kernel with HIP
events on the launch stream: those durations give the per-kernel algorithmic GB/s
and TFLOP/s (`kernels`) and the `roofline` of the dominant kernel.  At N=1 the other
single-GPU BASELINE configurations (C3 deepfm_multi_cate, C5 wdl with the bf16
tower) are timed the same way with fewer steps (`extra_workloads`), and rank 0 times
the torch-CPU restatement of the reference graph (oracle/torch_cpu.py) on a bounded
sample of the C2 workload (`cpu_baseline`).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
F32_MFMA_PEAK_TFLOPS = 157.3    # v_mfma_f32_16x16x4_f32 dense peak
BF16_MFMA_PEAK_TFLOPS = 2516.6  # dense bf16 MFMA peak (MI355X_MICROARCH.md; no sparsity)

C2 = dict(C=13, V=0, S=26, E=16, per_field_vocab=1_000_000, hidden=[400, 400, 400], B=65536)


def log(*a):
    print("[bench %s]" % time.strftime("%H:%M:%S"), *a, file=sys.stderr, flush=True)


def kernel_work(spec, B, touched_rows, rows=None, uniq=None, shard=None, wide_rows=None, stash=False, scatter=False,
                wide_uniq=None):
    """Algorithmic bytes / flops per launch."""
    E, S, C = spec.E, spec.S, spec.C
    N = rows if rows is not None else spec.n_rows
    w = {}
    # gather: FM rows (c+C) + deep rows (c) x 64 B + first-order 4 B + ids 8 B  (3,640 B/sample)
    w["embed_fwd"] = ("hbm", B * (S * (2 * E * 4 + 4 + 8)))
    # dense TF1 Adam: read+write p, m, v for every element; gradient rows read+reset only where touched
    w["adam_table"] = ("hbm", N * E * 4 * 6 + touched_rows * E * 4 * 2 + N)
    w["adam_first"] = ("hbm", N * 4 * 6 + touched_rows * 4 * 2 + N)
    dims = [spec.deep_in] + spec.hidden
    for l in range(len(spec.hidden)):
        f = 2.0 * B * (dims[l] + 1) * dims[l + 1]
        w["gemm_fwd_l%d" % l] = ("mfma", f)
        w["gemm_dw_l%d" % l] = ("mfma", f)
        w["gemm_dx_l%d" % l] = ("mfma", 2.0 * B * dims[l + 1] * (dims[l] if l else S * E))
    # backward scatter: FM + deep row gradients (f32 adds) + ids + dx0 read
    w["embed_bwd"] = ("hbm", B * (S * (E * 4 * 2 + 4 * 2 + 8) + S * E * 4))
    if uniq is not None:
        # row records (adam='lazy'): U unique rows of the batch, record = p, w1 triple + stamp, m, v
        rec_b = (3 * E + 4) * 4
        refs = 2 * S if spec.fm else S            # FM + deep references per sample (wdl/dnn: deep only)
        xb = 2 if spec.tower == "bf16" else 4      # x0 element bytes (the bf16 tower's x0 is written as bf16)
        # gather: read U records, write the compact rows (E + 1 floats) + keys; with the moment
        # stash (default) also the caught-up m, v (+ first-order m1, v1) for the backward
        from deep_learning_amd import _lib
        sf = int(_lib.lib().dl_rec_stash_floats(E))
        stash_b = sf * 4 if stash else 0
        # with the m-only stash (sf = E + 4) the backward reads the row's s (E floats) from its record
        s_rec = E * 4 if (stash and sf < 2 * E + 4) else 0
        w["rec_gather"] = ("hbm", uniq * (rec_b + (E + 1) * 4 + 4 + stash_b))
        # indexed x0 assembly: refs/sample x (compact row + inv) + first-order (FM) + x0 cat write
        w["embed_fwd"] = ("hbm", B * (refs * (E * 4 + 4) + (S * 4 if spec.fm else 0) + S * E * xb))
        if scatter:
            # scatter form: the gather also writes every reference's row (64 B) and the FM
            # references' first-order outputs, reading the index's segments and references;
            # the staged forward reads the FM staging rows and the inverse map in order
            w["rec_gather"] = ("hbm", uniq * (rec_b + (E + 1) * 4 + 4 + stash_b + 8) + B * refs * (4 + E * 4) +
                               (B * S * 4 if spec.fm else 0))
            w["embed_fwd"] = ("hbm", B * ((S * E * 4 + S * 4 + C * 4 + spec.fm_cols * 4 + E * 4) if spec.fm else 0) +
                              B * refs * 4 + B * C * xb)
        # fused backward + Adam: U records written and read back (stash: the compact row and
        # stashed moments read instead), per ref: ref id + dx0/fm_sum row + dz
        rd_b = ((E + 1) * 4 + stash_b + s_rec) if stash else rec_b
        w["embed_bwd"] = ("hbm", uniq * (rec_b + rd_b + 4 + 8) + B * refs * (4 + E * 4 + 4))
    if shard is not None:
        # row-sharded engine (shard.py): this rank's batch needs U = nsend + nrep unique rows;
        # as an owner it serves nrecv of them (gather) and updates nrecv arrivals (rec_apply)
        nsend, nrep, nrecv = shard
        rec_b = (3 * E + 4) * 4
        w["rec_gather"] = ("hbm", nrecv * (rec_b + (E + 1) * 4 + 4))
        w["embed_fwd"] = ("hbm", B * (2 * S * (E * 4 + 4) + S * 4 + S * E * 4))
        # per-unique-row gradient from its sorted references: ref + dx0/fm_sum row + dz per
        # reference, compact (E + 1)-float gradient row out
        w["embed_bwd"] = ("hbm", B * 2 * S * (4 + E * 4 + 4) + (nsend + nrep) * ((E + 1) * 4 + 8))
        # owner update: record read + written, gradient row + id in
        w["rec_apply"] = ("hbm", nrecv * (2 * rec_b + (E + 1) * 4 + 4))
        w.pop("adam_table", None)
        w.pop("adam_first", None)
    H = spec.hidden[-1]
    w["head"] = ("hbm", B * (spec.fm_cols + H) * 4 * 2)
    Fw = getattr(spec, "Fw", 0)
    if Fw:
        # wdl cross logit: per sample Fw ids + weights + gradient atomics + touched bytes, the h row,
        # the dY row (bf16 tower: bf16), label/score/z/dz
        dyb = 2 if spec.tower == "bf16" else 4
        w["head"] = ("hbm", B * (Fw * (8 + 4 + 8 + 1) + H * 4 + H * dyb + 16))
        # wide Adam (L2 on every row: a dense sweep): p, m, v read + written, touched flag read;
        # int64 fixed-point gradient read + reset where touched (at most B * Fw rows)
        w["adam_wide"] = ("hbm", (wide_rows or 0) * (12 * 2 + 1) + B * Fw * 16)
        if wide_uniq is not None:
            # lazy wide records: the unique wide rows' stash read, record written, gradient read +
            # reset; the deep-output rows' records; the wide gather: record read, stash + local w written
            w["adam_wide"] = ("hbm", wide_uniq * (16 + 16 + 16) + H * 40)
            w["wide_gather"] = ("hbm", wide_uniq * (4 + 16 + 16 + 4) + H * 20)
    return w


# bench label -> rocprofv3 kernel name in profiles/*/pmc_summary.json
PMC_KERNEL = {"adam_table": "adam_rows4_kernel", "adam_first": "adam_rows1_kernel",
              "embed_fwd": "embed_fwd_kernel<16, 5>", "embed_bwd": "embed_bwd_kernel<16, false>",
              "head": "head_kernel"}
PMC_KERNEL_LAZY = {"rec_gather": ("rec_gather_kernel<16, false, false>", "rec_gather_kernel<16, true, false>",
                                  "rec_gather_kernel<16, false>", "rec_gather_kernel<16, true>",
                                  "rec_gather_kernel<16>"),     # the last: summaries before the SPARSE template
                   "embed_bwd": ("rec_bwd_adam_kernel<16, true, false>", "rec_bwd_adam_kernel<16, true, true>",
                                 "rec_bwd_adam_kernel<16, true>", "rec_bwd_adam_kernel<16>"),
                   "head": "head_kernel"}


def pmc_traffic(label, world, lazy=False, workload="c2", id_dist="uniform"):
    """HBM bytes per launch of `label` from the newest committed PMC summary of the same
    workload (scripts/pmc_summary.py: (2*FETCH_SIZE + WRITE_SIZE)*1024, gfx950 correction;
    a summary without a "workload" key was collected on C2; one without "id_dist" on uniform ids,
    and a workload's zipf traffic is only taken from a zipf summary).  Newest = the latest round tag
    (profiles/r02s > r02q > r01r): file times do not survive a checkout or a copy."""
    import glob
    names = PMC_KERNEL_LAZY if lazy else PMC_KERNEL
    if world != 1 or label not in names:
        return None
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_summary*.json")))
    for f in reversed(files):
        d = json.load(open(f))
        if d.get("workload", "c2") != workload or d.get("id_dist", "uniform") != id_dist:
            continue
        want = names[label] if isinstance(names[label], tuple) else (names[label],)
        for n in want:
            k = d["kernels"].get(n)
            if k and "hbm_bytes" in k:
                return {"hbm_bytes": int(k["hbm_bytes"]), "source": os.path.relpath(f, ROOT)}
    return None


def bwd_calibrated(label, world, lazy=False, workload="c2", id_dist="uniform"):
    """The lazy backward's HBM bytes with the x2 FETCH_SIZE correction applied only to its
    coalesced streams (scripts/bwd_split.py: diagnostic builds show each random 64-B slice read
    is one 64-B request, already counted at its size) — C2 uniform only, where it was measured."""
    import glob
    if label != "embed_bwd" or not lazy or world != 1 or workload != "c2" or id_dist != "uniform":
        return None
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "bwd_split.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    return {"traffic_calibrated": int(d["hbm_bytes_calibrated"]),
            "traffic_calibrated_source": os.path.relpath(files[-1], ROOT)}


def cpu_baseline(spec_kw, B, steps_big=12, warm_big=2, steps_small=50, warm_small=10):
    """The CPU baseline of BASELINE.md §2: the torch-CPU restatement of
    models/deepfm_pipeline.py (oracle/torch_cpu.py; the reference's TF-CPU path cannot run
    without TensorFlow) timed on this host's cores at the full C2 table (26M rows, dense TF1
    Adam over every row), at the reference's default batch (1,024: SURVEY §8(d)'s >= 50 steps
    after 10 warmups) and at the headline batch (65,536: `value`, as many steps as the
    default bench's time budget allows — each sweeps the 26M-row table, ~2.5-3.4 s).
    Median step time; the counts are in the label."""
    import torch
    from oracle import ctr_ref as R
    from oracle.torch_cpu import DeepFMPipelineCPU
    from deep_learning_amd.synthetic import make_batch
    torch.set_num_threads(os.cpu_count() if not os.environ.get("OMP_NUM_THREADS")
                          else int(os.environ["OMP_NUM_THREADS"]))
    threads = torch.get_num_threads()
    N = spec_kw["S"] * spec_kw["per_field_vocab"]
    cfg = R.make_cfg("deepfm_pipeline", C=spec_kw["C"], V=0, S=spec_kw["S"], E=spec_kw["E"],
                     cate_index_size=N, hidden=spec_kw["hidden"])
    m = DeepFMPipelineCPU(spec_kw["C"], spec_kw["S"], spec_kw["E"], N, spec_kw["hidden"],
                          R.init_params(cfg, np.random.default_rng(0)))
    res = {}
    for bsz, n, warm in ((1024, steps_small, warm_small), (B, steps_big, warm_big)):
        bs = [make_batch(bsz, cate_index_size=N, seed=7 + i) for i in range(4)]
        for i in range(warm):
            m.train_step(bs[i % 4])
        ts = []
        for i in range(n):
            t0 = time.perf_counter()
            m.train_step(bs[i % 4])
            ts.append(time.perf_counter() - t0)
        res[bsz] = (float(np.median(ts)), len(ts), warm)
        log("cpu baseline B=%d: median %.3f s over %d steps after %d warmup" % (bsz, res[bsz][0], n, warm))
    med, n, w = res[B]
    med1, n1, w1 = res[1024]
    return {"value": B / med, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": "torch-CPU restatement of deepfm_pipeline.py (oracle/torch_cpu.py), full C2 table "
                      "(26M rows, dense TF1 Adam over every row, autograd backward), %d intra-op threads; "
                      "value: median of %d steps at B=%d (%.2f s/step) after %d warmup steps (the bench's time "
                      "budget); B=1024: median of %d steps after %d warmup (SURVEY §8(d))"
                      % (threads, n, B, med, w, n1, w1),
            "b1024": {"value": 1024 / med1, "median_s": round(med1, 3), "steps": n1, "warmup": w1}}


C1 = dict(C=13, V=0, S=26, E=8, cate_index_size=10_000, hidden=[512, 256, 128])


def hbm_peak_measured(gib=1.0, reps=10):
    """The chip's streaming rate measured here, reported beside HBM_PEAK_GBS (the 8 TB/s
    specification the roofline fractions use): dl_hbm_copy (metrics.hip: 16-B pieces, read once,
    written once) and torch's own device copy (a yardstick only) on the same buffers; the faster
    of the two is the measured peak (the two trade places from box to box, profiles/r06f)."""
    import torch
    from deep_learning_amd import _lib
    from deep_learning_amd._lib import call, ptr
    n = int(gib * (1 << 30))
    a = torch.empty(n, dtype=torch.uint8, device="cuda").fill_(1)
    b = torch.empty_like(a)
    s = _lib.stream_handle()

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    us_dl = timed(lambda: call("dl_hbm_copy", ptr(a), ptr(b), n, s))
    assert bool((b[:: 1 << 20] == 1).all())
    b.zero_()
    us_t = timed(lambda: b.copy_(a))
    assert bool((b[:: 1 << 20] == 1).all())
    del a, b
    torch.cuda.empty_cache()
    gbs = lambda us: round(2 * n / (us * 1e-6) / 1e9, 1)
    best = min(us_dl, us_t)
    return {"GB/s": gbs(best), "kernel": "dl_hbm_copy (metrics.hip)" if us_dl <= us_t else "torch copy_",
            "bytes_per_launch": 2 * n, "us": round(best, 1),
            "dl_hbm_copy": {"us": round(us_dl, 1), "GB/s": gbs(us_dl)},
            "torch_copy": {"us": round(us_t, 1), "GB/s": gbs(us_t)}}


def c1_leg(steps_time=50, warm=10, steps_auc=60, n_eval=4, seed=11):
    """BASELINE configs[0] (C1): models/dnn_pipeline.py at local_run.py's defaults (13 dense +
    26 cat over a 10k vocab, embedding 8, hidden [512, 256, 128]) — the reference's CPU-runnable
    plumbing case.  The torch-CPU restatement (oracle/torch_cpu.py, fm=False; TF is absent) is
    timed at B = 256 (configs[0]) and 1,024 (local_run.py:35): median of `steps_time` steps after
    `warm`.  Then the restatement and the GPU engine train `steps_auc` steps at B = 256 from the
    same initial parameters on the same seeded batches, and both score the same `n_eval` unseen
    batches: their ROC-AUCs (exact tie-aware AUC on each side) and the difference (north star:
    AUC within 1e-4 of the CPU path)."""
    import torch
    from oracle import ctr_ref as R
    from oracle.torch_cpu import DeepFMPipelineCPU
    from deep_learning_amd.engine import CTREngine, ModelSpec
    from deep_learning_amd.synthetic import make_batch
    threads = torch.get_num_threads()
    cfg = R.make_cfg("dnn_pipeline", **C1)
    P0 = R.init_params(cfg, np.random.default_rng(seed))
    new_cpu = lambda: DeepFMPipelineCPU(C1["C"], C1["S"], C1["E"], C1["cate_index_size"], C1["hidden"], P0, fm=False)
    out = {"workload": "C1 dnn_pipeline: 13 dense + 26 cat over a 10k vocab, E=8, MLP [512,256,128], TF1 Adam",
           "kind": "port", "cores": threads}
    for bsz in (256, 1024):
        m = new_cpu()
        bs = [make_batch(bsz, cate_index_size=C1["cate_index_size"], seed=seed + 1 + i) for i in range(8)]
        for i in range(warm):
            m.train_step(bs[i % 8])
        ts = []
        for i in range(steps_time):
            t0 = time.perf_counter()
            m.train_step(bs[i % 8])
            ts.append(time.perf_counter() - t0)
        med = float(np.median(ts))
        out["b%d" % bsz] = {"samples_per_s": round(bsz / med, 1), "median_ms": round(med * 1e3, 3),
                            "steps": steps_time, "warmup": warm}
    tr = [make_batch(256, cate_index_size=C1["cate_index_size"], seed=1000 + i) for i in range(steps_auc)]
    ev = [make_batch(1024, cate_index_size=C1["cate_index_size"], seed=2000 + i) for i in range(n_eval)]
    y = np.concatenate([b["label"].reshape(-1) for b in ev])
    sig = lambda z: 1.0 / (1.0 + np.exp(-z.astype(np.float64)))
    # three f32 trajectories from P0 over the same batches: the timed torch restatement, the
    # numpy oracle (the parity oracle, oracle/ctr_ref.py) and the GPU engine
    m = new_cpu()
    for b in tr:
        m.train_step(b)
    with torch.no_grad():
        s_cpu = np.concatenate([torch.sigmoid(m.forward(b)[0]).double().numpy() for b in ev])
    P = {k: v.copy() for k, v in P0.items()}
    opt = R.AdamTF1(cfg, P)
    for b in tr:
        R.train_step(cfg, P, opt, b)
    s_orc = np.concatenate([sig(R.forward(cfg, P, b)["z"]) for b in ev])
    eng = CTREngine(ModelSpec("dnn_pipeline", **C1), max_batch=1024, init="none")
    eng.load_params(P0)
    for b in tr:
        eng.train_step(b)
    s_gpu = np.concatenate([eng.predict(b).astype(np.float64) for b in ev])
    # the same parameters on both sides: the torch restatement's trained weights scored by the engine
    eng.load_params({k: v.detach().numpy().copy() for k, v in m.params.items()})
    s_same = np.concatenate([eng.predict(b).astype(np.float64) for b in ev])
    a_cpu, a_orc, a_gpu, a_same = R.auc(y, s_cpu), R.auc(y, s_orc), R.auc(y, s_gpu), R.auc(y, s_same)
    d = lambda v: float("%.3g" % v)
    out["auc"] = {"gpu_engine": round(a_gpu, 7), "numpy_oracle": round(a_orc, 7), "torch_cpu_restatement": round(a_cpu, 7),
                  "gpu_vs_oracle_abs_diff": d(abs(a_gpu - a_orc)),
                  "gpu_vs_oracle_max_abs_score_diff": d(np.abs(s_gpu - s_orc).max()),
                  "torch_vs_oracle_max_abs_score_diff": d(np.abs(s_cpu - s_orc).max()),
                  "same_params": {"gpu_scores_auc": round(a_same, 7), "abs_diff_vs_torch_cpu": d(abs(a_same - a_cpu)),
                                  "max_abs_score_diff": d(np.abs(s_same - s_cpu).max())},
                  "train_steps": steps_auc, "batch": 256, "eval_samples": int(y.size),
                  "note": "independent f32 trajectories: the two CPU restatements themselves part after ~10 steps "
                          "(sign-saturated early Adam steps on near-zero gradient sums), so the engine is compared "
                          "with the numpy oracle's trajectory and, on identical parameters, with the torch "
                          "restatement's scores"}
    del eng
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    log("C1 leg: CPU %s samples/s at B=256; AUC gpu %.7f oracle %.7f torch-cpu %.7f (same params: gpu %.7f)"
        % (out["b256"]["samples_per_s"], a_gpu, a_orc, a_cpu, a_same))
    return out


def vocab_for(wl, args, sharded):
    """Per-field vocab of a workload: --vocab, else 1M (C2, C3, C5 at every N) or, for the
    sharded DeepFM (C4), 100M rows over the 26 fields."""
    if args.vocab:
        return args.vocab
    return C2["per_field_vocab"] if (not sharded or wl != "c2") else -(-100_000_000 // C2["S"])


def make_spec(wl, vocab):
    from deep_learning_amd.engine import ModelSpec
    if wl == "c3":
        return ModelSpec("deepfm_multi_cate", C=0, V=0, S=C2["S"], E=C2["E"], cate_index_size=C2["S"] * vocab,
                         hidden=C2["hidden"], multi_ranges=[[60 * i, 60 * (i + 1), "slot%d" % i] for i in range(6)])
    if wl == "c5":
        return ModelSpec("wdl", C=C2["C"], S=C2["S"], E=C2["E"], cate_index_size=C2["S"] * vocab,
                         hidden=C2["hidden"], Fw=26, tower="bf16")
    return ModelSpec("deepfm_pipeline", C=C2["C"], V=0, S=C2["S"], E=C2["E"], cate_index_size=C2["S"] * vocab,
                     hidden=C2["hidden"])


def workload_name(wl, vocab, n_rows, sharded):
    return {"c2": ("C4 deepfm_pipeline, table row-sharded over the ranks" if sharded else "C2 deepfm_pipeline")
                  + ": 13 dense + 26 cat x %d vocab (table %d x 16 f32), MLP [400,400,400], TF1-dense Adam",
            "c3": "C3 deepfm_multi_cate: 26 cat + 6 multi-hot slots x 60 over %d vocab "
                  "(table %d x 16 f32), MLP [400,400,400], TF1-dense Adam",
            "c5": "C5 wdl: 13 dense + 26 deep cat + 26 wide ids x %d vocab (table %d x 16), "
                  "bf16 MLP [400,400,400] (fp32 master), fp32 wide logit, TF1-dense Adam",
            }[wl] % (vocab, n_rows)


def lookup_alone(eng, batch, B, per_sample, reps=20):
    """SURVEY §8(d)'s embedding gather as a lookup kernel alone, the one CTREngine.predict runs
    on a flushed table: the flush writes every row's p and first-order weight out as a slot plane
    (dl_rec_flush with DL_REC_PLANE_SLOTS: 128-B slots, the weight beside the row) and the lookup
    reads them (dl_embed_fwd_slots: an FM reference's row and weight one random request; the FM
    sums and x0 assembled) — bit-identical to the rec_gather + embed_fwd pair at lag 0 by test.
    Also timed: the same lookup reading each record's first 128-B line (dl_embed_fwd_rec_flat,
    the form without planes).  HIP events on the launch stream."""
    import torch
    from deep_learning_amd import _lib
    from deep_learning_amd._lib import call, ptr
    from deep_learning_amd.engine import C_ref
    sp = eng.spec
    eng.flush(planes=True)
    eng.stage(batch)
    L = eng.layout
    L.batch = B
    FL = eng._flat_layout(B)
    s = _lib.stream_handle()
    x0 = eng.x0b if eng.x0_direct else eng.x0

    def planes():
        if sp.fm:   # the slot plane: an FM reference's row and first-order weight in one 128-B slot
            call("dl_embed_fwd_slots", C_ref(FL), ptr(eng.p_plane), ptr(eng.in_cate), ptr(eng.in_cont), ptr(eng.in_vec),
                 ptr(x0), ptr(eng.fm_out), ptr(eng.fm_sum), ptr(eng.err), s)
        else:
            call("dl_embed_fwd", C_ref(FL), ptr(eng.p_plane), None, ptr(eng.in_cate), ptr(eng.in_cont),
                 ptr(eng.in_vec), ptr(x0), ptr(eng.fm_out), ptr(eng.fm_sum), ptr(eng.err), s)

    def records():
        if eng.n_rep:
            call("dl_rec_gather", C_ref(L), ptr(eng.rec), eng.rec_ld, eng.rec_flags, eng.n_rep, ptr(eng.idx_uniq), None,
                 0, 1, ptr(eng.hist), eng.hist_len, ptr(eng.opt), 0, ptr(eng.rows_u), ptr(eng.rows_u1), None, s)
        call("dl_embed_fwd_rec_flat", C_ref(L), ptr(eng.rec), eng.rec_ld, eng.rec_flags, ptr(eng.rows_u),
             ptr(eng.rows_u1) if sp.fm else None, ptr(eng.in_cate), ptr(eng.in_cont), ptr(eng.in_vec), ptr(eng.opt),
             ptr(x0), ptr(eng.fm_out), ptr(eng.fm_sum), ptr(eng.err), s)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        eng.check_error()
        us = e0.elapsed_time(e1) * 1e3 / reps
        gb = B * per_sample / (us * 1e-6) / 1e9
        return round(us, 1), round(gb, 1), round(gb / HBM_PEAK_GBS, 3)

    us, gb, fr = timed(planes)
    rus, rgb, rfr = timed(records)
    fused = None
    if eng.fused_gather_l0():
        # predict's fused form (the default on current planes): the lookup writes only the FM
        # outputs and x0's cont columns, the first tower layer reads the deep rows from the plane
        # through the ids (dl_gemm_s3_nt_gather).  What the gather costs there is the FM lookup
        # plus what the fused layer takes beyond the same layer over a written x0.
        FLn = eng._flat_layout(B)
        FLn.x0_cat_col = -1
        hd, ld0, ol0 = sp.hidden[0], eng.in_ld[0], eng.out_ld[0]
        bits = (ptr(eng.hbits[0]), eng.hbits_ld[0]) if eng.hbits else (None, 0)

        def fm_only():
            if sp.fm:
                call("dl_embed_fwd_slots", C_ref(FLn), ptr(eng.p_plane), ptr(eng.in_cate), ptr(eng.in_cont),
                     ptr(eng.in_vec), ptr(x0), ptr(eng.fm_out), ptr(eng.fm_sum), ptr(eng.err), s)
            else:
                call("dl_embed_fwd", C_ref(FLn), ptr(eng.p_plane), None, ptr(eng.in_cate), ptr(eng.in_cont),
                     ptr(eng.in_vec), ptr(x0), ptr(eng.fm_out), ptr(eng.fm_sum), ptr(eng.err), s)

        def l0_plain():
            call("dl_gemm_s3_nt_bits", B, hd, ld0, ptr(x0), ld0, ptr(eng.WTp[0]), ld0, ld0 * ol0, ptr(eng.h[0]),
                 eng.h_ld[0], 1, None, 0, *bits, s)

        def l0_gather():
            call("dl_gemm_s3_nt_gather", B, hd, ld0, ptr(x0), ld0, ptr(eng.p_plane), FLn.n_rows,
                 eng.p_plane.shape[1], ptr(eng.in_cate), FLn.cate_ld, FLn.deep_cate_offset, FLn.zero_row0, sp.S,
                 sp.E, ptr(eng.WTp[0]), ld0, ld0 * ol0, ptr(eng.h[0]), eng.h_ld[0], 1, *bits, s)

        fus = timed(fm_only)[0]
        l0u = timed(l0_plain)[0]
        l0g = timed(l0_gather)[0]
        pair_u = timed(lambda: (planes(), l0_plain()))[0]
        pair_f = timed(lambda: (fm_only(), l0_gather()))[0]
        g_us = fus + max(l0g - l0u, 0.0)
        g_gb = B * per_sample / (g_us * 1e-6) / 1e9
        fused = {"kernels": ["embed_fwd (FM only)", "gemm_fwd_l0 (gather)"], "fm_lookup_us": fus,
                 "fwd_l0_gather_us": l0g, "fwd_l0_plain_us": l0u,
                 "us": round(g_us, 1), "GB/s": round(g_gb, 1), "frac": round(g_gb / HBM_PEAK_GBS, 3),
                 "lookup_plus_l0_us": {"unfused": pair_u, "fused": pair_f},
                 "note": "us = the FM-only lookup + (fused first layer - the same layer over a written x0): "
                         "what the 3,640 B/sample gather adds to predict's forward when it feeds the MFMA "
                         "tiles directly"}
        # the same cost read off the back-to-back pair (lookup + fused layer, minus the plain
        # layer alone): the two kernels' cache interactions included
        fused["pair_minus_plain_us"] = round(pair_f - l0u, 1)
        fused["frac_by_pair"] = round(B * per_sample / ((pair_f - l0u) * 1e-6) / 1e9 / HBM_PEAK_GBS, 3)
        if eng.fused_gather_tab(B, force=True):
            # the table form (DLAMD_GATHER_TAB=1, not the default): the lookup writes the deep rows'
            # plane offsets too (dl_embed_fwd_gtab, no fm_sum) and the first layer stages them as
            # they stand instead of loading and range-checking the ids
            def fm_tab():
                call("dl_embed_fwd_gtab", C_ref(FLn), ptr(eng.p_plane), 1 if sp.fm else 0, ptr(eng.in_cate),
                     ptr(eng.in_cont), ptr(eng.in_vec), ptr(x0), ptr(eng.fm_out), None, ptr(eng.gtab),
                     ptr(eng.err), s)

            def l0_tab():
                call("dl_gemm_s3_nt_gather_tab", B, hd, ld0, ptr(x0), ld0, ptr(eng.p_plane), FLn.n_rows,
                     eng.p_plane.shape[1], ptr(eng.gtab), sp.S, sp.E, ptr(eng.WTp[0]), ld0, ld0 * ol0,
                     ptr(eng.h[0]), eng.h_ld[0], 1, *bits, s)

            fut = timed(fm_tab)[0]
            l0t = timed(l0_tab)[0]
            pair_t = timed(lambda: (fm_tab(), l0_tab()))[0]
            t_us = fut + max(l0t - l0u, 0.0)
            t_gb = B * per_sample / (t_us * 1e-6) / 1e9
            fused["table_form"] = {
                "kernels": ["embed_fwd (FM + row offsets)", "gemm_fwd_l0 (gather, offset table)"],
                "fm_lookup_us": fut, "fwd_l0_gather_us": l0t, "us": round(t_us, 1), "GB/s": round(t_gb, 1),
                "frac": round(t_gb / HBM_PEAK_GBS, 3), "lookup_plus_l0_us": pair_t,
                "pair_minus_plain_us": round(pair_t - l0u, 1),
                "frac_by_pair": round(B * per_sample / ((pair_t - l0u) * 1e-6) / 1e9 / HBM_PEAK_GBS, 3),
                "note": "DLAMD_GATHER_TAB=1, not the default: its layer alone is faster than the id form's, "
                        "the back-to-back pair is not (frac_by_pair)"}
    return {"kernels": ["embed_fwd (slot plane)"], "us": us, "GB/s": gb, "frac": fr, "fused": fused,
            "records": {"kernels": ["rec_gather (13 cont rows)", "embed_fwd_rec_flat"], "us": rus, "GB/s": rgb,
                        "frac": rfr},
            "note": "flushed table: the lookup without lazy Adam's catch-up, as predict runs it with "
                    "DLAMD_FUSED_GATHER=0 (the flush writes a slot plane, each row's p and first-order weight in one "
                    "128-B slot; 'records' reads each record's first line instead; 'fused': predict's default on "
                    "current planes, the deep rows read by the first tower layer itself); the "
                    "training step's gather above also replays each row's pending zero-gradient Adam steps and "
                    "stashes its moments"}


def dropin_fit(args, n_batches=24, warm=3):
    """The Wide&Deep drop-in's own training loop at C5 shapes: models/wdl.DeepModel (the
    load-style surface of /root/reference/models/wdl.py:287-316) trained over pickled host
    batches (utils/data_loader_load.py's format: a dict of arrays per batch, unpickled each
    step as wdl.py:296 does) — unpickle, host-to-device staging of the next batch during the
    current step, the step, and the per-step loss summed on the device (read once per epoch).
    Timed over one pass of n_batches after a warmup pass of `warm`."""
    import pickle
    import torch
    from deep_learning_amd.models import wdl
    from deep_learning_amd.synthetic import make_batch

    class A:
        hidden_units, epochs, batch_size, learning_rate = list(C2["hidden"]), 1, args.batch, 0.001
        model_pb, learning_rate_decay_steps, learning_rate_decay_rate, l2_reg = "", 10000000, 0.9, 1e-5
        cont_field_size, cate_field_size, embedding_size, wide_field_size = C2["C"], C2["S"], C2["E"], 26
        cate_index_size = C2["S"] * C2["per_field_vocab"]
        alg_name, vector_field_size, tower_dtype = "wdl", 0, "bf16"
    items = []
    for i in range(n_batches):
        b = make_batch(args.batch, cate_index_size=A.cate_index_size, seed=500 + i, wide_fields=26)
        items.append(pickle.dumps({"labels": b["label"], "cont_feats": b["cont_feats"], "cate_feats": b["cate_feats"],
                                   "wide_feats": b["wide_feats"]}, protocol=pickle.HIGHEST_PROTOCOL))
    m = wdl.DeepModel(A)
    m.train_epoch(items[:warm])
    eng = m.model_optimizer()
    eng.step_events = []     # the compute stream's step spans and the gaps between steps
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss_sum, steps = m.train_epoch(items)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ev, eng.step_events = eng.step_events or [], None
    starts = [e for k, e in ev if k == 0]
    ends = [e for k, e in ev if k == 1]
    span = [a.elapsed_time(b) for a, b in zip(starts, ends)]
    gap = [b.elapsed_time(a) for b, a in zip(ends, starts[1:])]
    out = {"ms_per_step": round(dt / steps * 1e3, 4), "steps": steps, "samples_per_s": round(steps * args.batch / dt, 1),
           "epoch_mean_loss": round(loss_sum / steps, 6),
           "compute_stream": {"step_span_ms": round(sum(span) / max(1, len(span)), 4),
                              "gap_ms": round(sum(gap) / max(1, len(gap)), 4)},
           "note": "wdl.DeepModel.train_epoch over one %d-batch epoch of pickled C5 batches (B=%d, 26M-row table, "
                   "bf16 tower): decode + staging + step + device-summed loss per step, the epoch's start included; "
                   "after a %d-batch warmup pass. compute_stream: the steps' own span and the gap between steps "
                   "on the device" % (n_batches, args.batch, warm)}
    del m
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def run_workload(wl, args, world, rank, sharded, steps, warmup, age, ksteps, barrier, dist_ids=None):
    """The workload on the default stream, or (DLAMD_MAIN_PRIORITY set, an A/B switch) on a
    compute stream of that priority.  dist_ids: the id distribution (default --dist)."""
    import torch
    pr = os.environ.get("DLAMD_MAIN_PRIORITY")
    if pr is None:
        return _run_workload(wl, args, world, rank, sharded, steps, warmup, age, ksteps, barrier, dist_ids)
    st = torch.cuda.Stream(priority=int(pr))
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        r = _run_workload(wl, args, world, rank, sharded, steps, warmup, age, ksteps, barrier, dist_ids)
    torch.cuda.current_stream().wait_stream(st)
    return r


def _run_workload(wl, args, world, rank, sharded, steps, warmup, age, ksteps, barrier, dist_ids=None):
    """Build the engine of workload `wl`, age its table, time `steps` steps (hipGraph replay,
    next batch prefetched), then `ksteps` eager steps bracketed per kernel by HIP events.
    Uniform ids: a fresh device-drawn batch every step (no batch repeats, so the model never
    memorises the set and the data-dependent paths see a real loss); zipf: 32 host-drawn batches
    cycled (the Zipf permutations are host-side)."""
    import torch
    from deep_learning_amd.engine import CTREngine
    from deep_learning_amd.synthetic import make_batch, make_batch_device
    B = args.batch
    id_dist = dist_ids or args.dist
    spec = make_spec(wl, vocab_for(wl, args, sharded))
    log("%s rank %d/%d: building engine, table rows %d" % (wl, rank, world, spec.n_rows))
    use_graph = not args.no_graph
    prefetch = not args.no_prefetch
    if not sharded:
        eng = CTREngine(spec, max_batch=B, seed=2019, adam=args.adam, rec_stash=not args.no_rec_stash)
    else:
        from deep_learning_amd.shard import Exchange, ShardedCTREngine
        eng = ShardedCTREngine(spec, B, Exchange(), seed=2019, adam=args.adam, owner_update=args.owner_update)
        eng.init_device(2019)
    kw = dict(cont=0, cate_fields=C2["S"], cate_index_size=spec.cate_index_size, multi_slots=6, multi_width=60,
              cate_only=True) if wl == "c3" else dict(cate_index_size=spec.cate_index_size, wide_fields=spec.Fw)
    total = age + warmup + steps + ksteps + 1
    if id_dist == "uniform":
        nb = total
        batches = [make_batch_device(B, seed=100_000 * rank + i, **kw) for i in range(nb)]
    else:
        nb = 16 if wl == "c3" else 32
        batches = [{k: torch.from_numpy(v).cuda() for k, v in
                    make_batch(B, seed=1000 * rank + i, dist=id_dist, **kw).items()} for i in range(nb)]
    torch.cuda.synchronize()

    depth = getattr(eng, "pf_depth", 1)

    def step(i, graph=use_graph, pf=prefetch):
        # the batches after step i are prefetched during it (pf_depth of them in flight; each
        # step still builds exactly one index: the last timed step builds one after the region)
        ahead = [batches[(i + j) % nb] for j in range(1, depth + 1)]
        eng.train_step(batches[i % nb], graph=graph, **({"next_batch": ahead if depth > 1 else ahead[0]} if pf else {}))

    # table age: untimed steps before the warmup, so the rows the timed steps reference carry
    # the steady-state lag of lazy Adam (the zero-gradient steps a row replays when next
    # touched; geometric, mean ~15 steps for C2's uniform 1M-id fields, capped by the age)
    log("%s: table age %d steps" % (wl, age))
    for i in range(age):
        step(i)
    base = age
    torch.cuda.synchronize()
    log("%s: warmup %d" % (wl, warmup))
    for i in range(base, base + max(1, warmup)):
        step(i)
    base += max(1, warmup)
    torch.cuda.synchronize()
    eng.check_error()
    log("%s: timed %d steps" % (wl, steps))
    barrier()
    torch.cuda.synchronize()
    if os.environ.get("DLAMD_STEP_EVENTS", "0") == "1":   # the compute stream's span / gap per step
        eng.step_events = []
    if getattr(eng, "host_marks", None) is not None:
        eng.host_marks.clear()
    t0 = time.perf_counter()
    w0 = getattr(eng, "host_wait", 0.0)
    for i in range(base, base + steps):
        step(i)
    # the host's own submission time per step (the time train_step spent waiting for the GPU to
    # catch up excluded): close to ms_per_step would mean the host, not the GPU, sets the pace
    host_ms = (time.perf_counter() - t0 - (getattr(eng, "host_wait", 0.0) - w0)) / steps * 1e3
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    base += steps
    marks = getattr(eng, "host_marks", None)
    if marks:   # sharded engine, DLAMD_HOST_TIMING=1: host time per phase of the step (ms)
        ph = {}
        for (n0, t0_), (n1, t1_) in zip(marks[:-1], marks[1:]):
            if n1 != "start":
                ph.setdefault(n1, []).append((t1_ - t0_) * 1e3)
        log("%s: host ms per phase %s" % (wl, {k: round(sum(v) / len(v), 4) for k, v in ph.items()}))
    step_ev = None
    if getattr(eng, "step_events", None):
        ev, eng.step_events = eng.step_events, None
        starts = [e for k, e in ev if k == 0]
        ends = [e for k, e in ev if k == 1]
        span = [a.elapsed_time(b) for a, b in zip(starts, ends)]
        gap = [b.elapsed_time(a) for b, a in zip(ends, starts[1:])]
        step_ev = {"span_ms": round(sum(span) / len(span), 4), "gap_ms": round(sum(gap) / max(1, len(gap)), 4),
                   "gap_max_ms": round(max(gap, default=0.0), 4)}
        log("%s: step span %.4f ms, gap to the next step %.4f ms" % (wl, step_ev["span_ms"], step_ev["gap_ms"]))
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = tt.item()
    ms = dt / steps * 1e3
    value = world * B * steps / dt
    eng.check_error()
    loss = eng.loss()
    log("%s: %.4f ms/step, %.1f M samples/s, loss %.4f" % (wl, ms, value / 1e6, loss))

    # ---- live per-kernel timing (HIP events on the launch stream), eager steps
    eng.prof = []
    for i in range(base, base + ksteps):
        step(i, graph=False, pf=False)
    torch.cuda.synchronize()
    times = {}
    for label, e0, e1 in eng.prof:
        times.setdefault(label, []).append(e0.elapsed_time(e1) * 1e3)   # us
    eng.prof = None
    ids = batches[0]["cate_feats"]
    touched_rows = int(torch.unique(torch.cat([ids.reshape(-1) + spec.C, ids.reshape(-1)])).numel()) + spec.C
    shard_counts = getattr(eng, "last_counts", None) if sharded and getattr(eng, "lazy", False) else None
    uniq = int(eng.idx_n[0].item()) if getattr(eng, "lazy", False) and not sharded else None
    ww = getattr(eng, "ww", None)
    wide_uniq = int(eng.widx_n[0].item()) if getattr(eng, "wide_lazy", False) else None
    work = kernel_work(spec, B, touched_rows, rows=getattr(eng, "local_rows", spec.n_rows), uniq=uniq,
                       shard=shard_counts, wide_rows=int(ww.shape[0]) if ww is not None else None,
                       stash=getattr(eng, "mv_u", None) is not None, scatter=getattr(eng, "fwd_scatter", False),
                       wide_uniq=wide_uniq)
    s3 = getattr(eng, "s3", False)
    # the tower GEMMs' own peak: f32 products as six bf16 plane products (gemm_s3.hip) run at
    # 1/6 of the bf16 MFMA peak; the bf16 tower at the bf16 peak; f32 MFMA otherwise
    gemm_peak = BF16_MFMA_PEAK_TFLOPS if spec.tower == "bf16" else (
        BF16_MFMA_PEAK_TFLOPS / 6 if s3 else F32_MFMA_PEAK_TFLOPS)
    kernels = {}
    for label, ts in times.items():
        us = float(np.mean(ts))
        ent = {"us": round(us, 2), "launches": len(ts)}
        if label in work:
            kind, amount = work[label]
            if kind == "hbm":
                ent["GB/s"] = round(amount / (us * 1e-6) / 1e9, 1)
                ent["frac_hbm"] = round(amount / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 3)
            else:
                ent["TFLOP/s"] = round(amount / (us * 1e-6) / 1e12, 2)
                ent["frac_mfma"] = round(amount / (us * 1e-6) / 1e12 / gemm_peak, 3)
                if s3:   # against the native f32 matrix peak too (157.3 TF): above 1.0 by design
                    ent["frac_f32_mfma_peak"] = round(amount / (us * 1e-6) / 1e12 / F32_MFMA_PEAK_TFLOPS, 3)
        kernels[label] = ent
    # where the step's time went, one compact line on stderr (kept by a log's tail)
    log("%s per-kernel us/launch: %s" % (wl, ", ".join(
        "%s %.0f%s" % (k, v["us"], "x%d" % v["launches"] if v["launches"] > 1 else "")
        for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["us"] * kv[1]["launches"]))))
    # the dominant kernel among those with an algorithmic work figure
    dom = max((l for l in kernels if l in work), key=lambda l: kernels[l]["us"])
    kind, amount = work.get(dom, ("hbm", 0))
    us = kernels[dom]["us"]
    if kind == "hbm":
        ach = amount / (us * 1e-6) / 1e9
        roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 3), "traffic": None, "algorithmic_bytes": amount}
    else:
        ach = amount / (us * 1e-6) / 1e12
        roof = {"kernel": dom, "bound": "mfma", "achieved": round(ach, 2), "peak": round(gemm_peak, 1),
                "unit": "TFLOP/s", "frac": round(ach / gemm_peak, 3), "traffic": None,
                "algorithmic_flops": amount}
        if s3:
            roof["frac_f32_mfma_peak"] = round(ach / F32_MFMA_PEAK_TFLOPS, 3)
    pmc = pmc_traffic(dom, world, lazy=uniq is not None, workload=wl, id_dist=id_dist)
    if pmc is not None:
        roof["traffic"] = pmc["hbm_bytes"]
        roof["traffic_source"] = pmc["source"]
        cal = bwd_calibrated(dom, world, lazy=uniq is not None, workload=wl, id_dist=id_dist)
        if cal is not None:
            roof.update(cal)
    # the embedding lookup by SURVEY §8(d)'s own byte count (C2: 26 FM + 26 deep rows x 64 B +
    # 26 first-order x 4 B + 26 ids x 8 B = 3,640 B/sample; C3: 17,096 B/sample) over the
    # kernels that do it here (record gather + indexed forward); the per-kernel figures above
    # count the bytes those kernels move (records include the Adam moments the lazy scheme needs)
    gather = None
    per_sample = {"c2": 3640, "c3": 17096}.get(wl)
    fwd_kernels = [k for k in ("rec_gather", "pool_fwd", "embed_fwd") if k in kernels]
    if per_sample and not sharded and "embed_fwd" in kernels:
        gus = sum(kernels[k]["us"] for k in fwd_kernels)
        gb = B * per_sample / (gus * 1e-6) / 1e9
        gather = {"bytes_per_sample": per_sample, "kernels": fwd_kernels,
                  "us": round(gus, 1), "GB/s": round(gb, 1), "frac": round(gb / HBM_PEAK_GBS, 3)}
    # the lazy table's periodic catch-up of every row (dl_rec_flush every hist_len - 2 steps),
    # timed once and amortised per step (not inside the timed region: it runs once per ~4094)
    flush = None
    if getattr(eng, "lazy", False) and hasattr(eng, "hist_len") and not sharded:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.flush()
        torch.cuda.synchronize()
        fus = (time.perf_counter() - t0) * 1e6
        flush = {"us": round(fus, 1), "every_steps": eng.hist_len - 2,
                 "us_per_step_amortised": round(fus / (eng.hist_len - 2), 2)}
        if per_sample and not spec.M:
            gather_lookup = lookup_alone(eng, batches[base % nb], B, per_sample)
            if id_dist == "uniform":
                # the same lookup over a Zipf batch (SURVEY §8(d)'s realistic ids: hot rows re-read)
                zb = {k: torch.from_numpy(v).cuda() for k, v in
                      make_batch(B, seed=4242, dist="zipf", **kw).items()}
                z = lookup_alone(eng, zb, B, per_sample)
                gather_lookup["zipf"] = {k: z[k] for k in ("us", "GB/s", "frac")}
                gather_lookup["zipf"]["records"] = z["records"]
                gather_lookup["zipf"]["fused"] = z["fused"]
                del zb
            if gather is not None:
                gather["lookup_alone"] = gather_lookup
    out = dict(spec=spec, value=value, ms=ms, loss=loss, roofline=roof, gather=gather, flush=flush, kernels=kernels,
               kernel_sum=sum(k["us"] for k in kernels.values()), nb=nb, gemm_peak=gemm_peak, host_ms=host_ms,
               step_events=step_ev)
    if sharded:
        out["shard"] = {"cap": eng.cap, "overflows": getattr(eng, "overflows", 0), "report_lag": eng.lag,
                        "all_reduce_serial": eng.ar_serial, "exchange_bytes_per_rank": eng.exchange_bytes()}
        eng.exch.close()
    del eng, batches
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def free_port():
    """A free TCP port on 127.0.0.1 for the ranks' rendezvous."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(n, argv, port, script=None):
    """The command that runs this bench as `n` ranks, one process per GPU (the driver's own
    form: torch.distributed.run on one node, rendezvous on 127.0.0.1).  `argv` is this
    process's argument list; every rank parses the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port),
            script or os.path.abspath(__file__)] + list(argv)


def world_check(gpus, env):
    """(world, need_launch): under a launcher (WORLD_SIZE set) the world must be --gpus;
    without one, --gpus N > 1 means this process starts the N ranks itself."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return 1, gpus > 1
    if int(ws) != gpus:
        raise SystemExit("bench.py: WORLD_SIZE=%s from the launcher but --gpus %d: the line would misreport "
                         "n_gpus; launch --nproc-per-node %d or pass --gpus %s" % (ws, gpus, gpus, ws))
    return int(ws), False


def relay_ranks(n, argv, json_fd, script=None):
    """Run the bench as n rank processes (started before this process touches the GPU: it
    never initialises HIP, so no exec or fork of a GPU-holding process happens), relay rank
    0's JSON line to our stdout and return the launcher's exit code."""
    import subprocess
    cmd = launch_command(n, argv, free_port(), script)
    log("launching %d ranks: %s" % (n, " ".join(cmd)))
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=None, env=dict(os.environ))
    lines = [l for l in p.stdout.decode(errors="replace").splitlines() if l.startswith("{")]
    for l in lines[-1:]:
        os.write(json_fd, (l + "\n").encode())
    if p.returncode == 0 and not lines:
        log("the ranks exited 0 without a result line")
        return 1
    return p.returncode


def main():
    # stdout carries exactly one JSON line: libraries that print banners at init (RCCL does)
    # are sent to stderr by pointing fd 1 there; the result goes to the saved stdout fd.
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dist", default="uniform", choices=["uniform", "zipf"])
    ap.add_argument("--batch", type=int, default=C2["B"])
    ap.add_argument("--vocab", type=int, default=0,
                    help="per-field vocab (default: 1M at N=1 = C2; 100M/26 at N>1 = C4's 100M-row table)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c5"],
                    help="c2 DeepFM (the headline, default); c3 deepfm_multi_cate 6 multi-hot slots x 60; "
                         "c5 Wide&Deep with the bf16 tower (single GPU, or row-sharded at N>1 / --sharded)")
    ap.add_argument("--no-extra", action="store_true",
                    help="N=1: skip the other single-GPU BASELINE workloads (C3, C5) timed after the headline")
    ap.add_argument("--extra-steps", type=int, default=10, help="timed steps of each extra workload")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph replay")
    ap.add_argument("--owner-update", default=None, choices=["sort", "chain"],
                    help="sharded owners: group arriving rows by a sort (default) or by arrival chains")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="build each batch's index at the start of its own step (default: during the "
                         "previous step, on a second hardware queue)")
    ap.add_argument("--sharded", action="store_true",
                    help="run the row-sharded multi-GPU engine even at N=1 (measures its overhead)")
    ap.add_argument("--age-steps", type=int, default=64,
                    help="untimed steps before the warmup that bring the table's row lags to steady state")
    ap.add_argument("--no-rec-stash", action="store_true",
                    help="lazy records: the backward re-reads the record and replays its catch-up itself "
                         "(default: the gather stashes the caught-up moments for it)")
    ap.add_argument("--adam", default="lazy", choices=["dense", "lazy"],
                    help="table Adam: dense sweep, or row records with lazy-exact catch-up (same result)")
    args = ap.parse_args()

    # --gpus N without a launcher: start the N ranks now, before anything touches the GPU
    world, need_launch = world_check(args.gpus, os.environ)
    if need_launch:
        sys.exit(relay_ranks(args.gpus, sys.argv[1:], json_fd))

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DLAMD_BENCH_BACKEND=gloo: rehearsal of the multi-rank flow with ranks sharing one GPU
    # (host-staged exchange); the measured configuration is nccl = RCCL, one GPU per rank.
    backend = os.environ.get("DLAMD_BENCH_BACKEND", "nccl")
    dev_index = local if backend == "nccl" else local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    sharded = world > 1 or args.sharded
    if sharded:
        if world == 1:   # --sharded at N=1: the multi-GPU code path on one rank (overhead measurement)
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(backend)

    def barrier():
        if world > 1:
            dist.barrier()

    wl = args.workload
    if wl == "c3" and sharded:
        raise SystemExit("--workload c3 is single-GPU here; the multi-GPU workloads are C4 (default) and C5")
    r = run_workload(wl, args, world, rank, sharded, args.steps, args.warmup, args.age_steps,
                     min(args.steps, 10), barrier)
    spec = r["spec"]
    B = args.batch
    # the other single-GPU BASELINE configurations, timed the same way with fewer steps, so the
    # driver's run covers every single-GPU config (BASELINE.json configs[2], configs[4])
    # (N > 1: the sharded Wide&Deep, C5 at N GPUs, after the sharded DeepFM C4)
    extra = {}
    others = ()
    if not args.no_extra:
        if world == 1 and not sharded:
            others = tuple((w2, None) for w2 in ("c2", "c3", "c5") if w2 != wl)
            if args.dist == "uniform":   # both id distributions for the training step
                others += (("c2", "zipf"), ("c5", "zipf"))
        elif world > 1 and wl == "c2":
            others = (("c5", None),)
    for w2, d2 in others:
        key = w2 + ("_" + d2 if d2 else "")
        try:
            e = run_workload(w2, args, world, rank, sharded, args.extra_steps, min(args.warmup, 3),
                             args.age_steps, 5, barrier, dist_ids=d2)
        except Exception as ex:   # reported, never fatal for the headline number
            if world > 1:         # a rank that failed alone would leave the others in a collective
                raise
            extra[key] = {"error": repr(ex)}
            continue
        extra[key] = {"id_dist": d2 or args.dist,
                      "workload": workload_name(w2, vocab_for(w2, args, sharded), e["spec"].n_rows, sharded),
                      "global_batch": B * world,
                      "ms_per_step": round(e["ms"], 4), "samples_per_s": round(e["value"], 1),
                      "steps": args.extra_steps, "roofline": e["roofline"], "gather_north_star": e["gather"],
                      "kernel_sum_us_per_step": round(e["kernel_sum"], 1), "loss": round(e["loss"], 6),
                      "host_submit_ms_per_step": round(e["host_ms"], 4),
                      "kernels": e["kernels"]}
    if "c5" in extra and "error" not in extra["c5"] and world == 1:
        try:
            extra["c5"]["dropin_fit"] = dropin_fit(args)
            extra["c5"]["dropin_fit"]["vs_engine_step"] = round(extra["c5"]["dropin_fit"]["ms_per_step"] /
                                                                extra["c5"]["ms_per_step"], 3)
        except Exception as ex:   # reported, never fatal
            extra["c5"]["dropin_fit"] = {"error": repr(ex)}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline (torch-CPU restatement)")
        torch.cuda.empty_cache()
        try:
            cpu = cpu_baseline(C2, B)
        except Exception as e:  # reported, never fatal for the GPU number
            cpu = {"value": None, "error": repr(e)}
        try:
            cpu["c1"] = c1_leg()
        except Exception as e:  # reported, never fatal
            cpu["c1"] = {"error": repr(e)}
    peak_meas = None
    if rank == 0:
        try:
            peak_meas = hbm_peak_measured()
            log("measured HBM copy peak %.1f GB/s" % peak_meas["GB/s"])
        except Exception as e:  # reported, never fatal
            peak_meas = {"error": repr(e)}
        if r["roofline"]["bound"] == "hbm" and "GB/s" in peak_meas:
            r["roofline"]["peak_measured"] = peak_meas["GB/s"]
            r["roofline"]["frac_of_measured"] = round(r["roofline"]["achieved"] / peak_meas["GB/s"], 3)

    if rank == 0:
        out = {
            "metric": "train samples/sec + achieved HBM GB/s, DeepFM Criteo-shape bsz=65536, 1/2/4/8 GPU",
            "value": round(r["value"], 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(r["ms"], 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16+f32" if wl == "c5" else "f32",
            "data": ("synthetic (seeded Criteo-shaped batches, uniform ids, a fresh batch drawn on the device for "
                     "every step, resident in HBM before the timed region)" if args.dist == "uniform" else
                     "synthetic (seeded Criteo-shaped batches, zipf ids, %d batches cycled, resident in HBM)"
                     % r["nb"]),
            "world": {"torch_distributed": dist.get_world_size() if sharded else 1,
                      "backend": dist.get_backend() if sharded else None,
                      "ranks": world, "device_per_rank": backend == "nccl"},
            "config": {"workload": workload_name(wl, vocab_for(wl, args, sharded), spec.n_rows, sharded),
                       "global_batch": B * world, "per_gpu_batch": B,
                       "parallelism": "dp%d" % world if not sharded else
                       "dp%d + row-sharded table (RCCL all-to-all lookup, all-reduce dense grads)" % world,
                       "id_dist": args.dist, "table_adam": args.adam},
            "roofline": r["roofline"],
            "cpu_baseline": cpu,
            "gather_north_star": r["gather"],
            "table_flush": r["flush"],
            "distinct_batches": r["nb"],
            "table_age_steps": args.age_steps,
            "gemm_peak_tflops": round(r["gemm_peak"], 1),
            "hbm_copy_measured": peak_meas,
            "kernels": r["kernels"],
            "kernel_sum_us_per_step": round(r["kernel_sum"], 1),
            "host_submit_ms_per_step": round(r["host_ms"], 4),
            **({"shard": r["shard"]} if r.get("shard") else {}),
            **({"step_events": r["step_events"]} if r.get("step_events") else {}),
            "loss": round(r["loss"], 6),
            "extra_workloads": extra or None,
        }
        os.write(json_fd, (json.dumps(out) + "\n").encode())
        # the headline's own summary once more, last on stderr (the extra workloads, the CPU
        # baseline and the C1 leg log after the headline's per-kernel line: a 4-KB tail drops it)
        k = r["kernels"]
        log("headline %s: %.4f ms/step, %.4g %s; per-kernel us/launch: %s" % (
            out["config"]["workload"].split(":")[0], r["ms"], out["value"], out["unit"], ", ".join(
                "%s %.0f%s" % (n, v["us"], "x%d" % v["launches"] if v["launches"] > 1 else "")
                for n, v in sorted(k.items(), key=lambda kv: -kv[1]["us"] * kv[1]["launches"]))))
    if sharded:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
