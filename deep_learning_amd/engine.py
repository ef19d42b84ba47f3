"""MI355X training engine for the reference's CTR models (DeepFM / DNN / Wide&Deep).

One ``CTREngine`` holds every device buffer of a model (parameters, TF1-Adam
state, activations, gradient tables, partial-sum slabs) and runs a training
step as a fixed sequence of HIP kernels from ``libdlamd.so`` on one stream —
so the whole step can be captured into a hipGraph and replayed.

Step (deepfm_pipeline, reference models/deepfm_pipeline.py:76-191):
  adam_begin_step                       alpha_t, beta powers, global_step
  embed_fwd                             gather + FM 1st/2nd order + x0 assembly
  gemm_f32 x L (ReLU)                   deep tower forward (bias = ones column)
  head_fwd_bwd                          logit, sigmoid, log-loss, dz, dh_L, dW_head partials
  for l = L-1..0: gemm dW (split-K) ; gemm dX (ReluGrad) ; adam_dense(W_l)
  embed_bwd + cont_reduce               FM/deep row gradients -> dense gradient table
  adam_dense(head) ; adam_rows(table) ; adam_rows(first-order)

Internal layouts (import/export map to the reference's):
  x0  = [cate embeddings (S*E) | pooled (M*E) | cont (C) | vector (V) | 1 | 0-pad]
  W_l = [in_ld, out_ld] row-major; row in_dim holds the bias, pads are zero
  head w = [first (F) | second (E) | deep (H) | bias]   (deepfm; dnn: [H | bias])
"""
import contextlib
import gc
import math
import os
import time

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr

F32 = torch.float32


def _ru(x, m):
    return (x + m - 1) // m * m


# Model families of the reference's pipeline-style model files:
#   fm     FM first/second order feeds the head (deepfm_*), else the deep_res head (dnn_*)
#   cont   dense features present; "first": FM cont rows 0..C-1, cate ids at +C
#          (deepfm_pipeline.py:58-61,89); "last": FM cont rows at cate_index_size + j,
#          ids unshifted (deepfm_multi.py:139); "deep": cont only in the deep input (dnn_*)
#   multi  nonzero-mean-pooled multi-hot slots after the S singles
FAMILIES = {
    "deepfm_pipeline": dict(fm=True, cont="first", multi=False),     # models/deepfm_pipeline.py:76-191
    "deepfm_cate": dict(fm=True, cont=None, multi=False),            # models/deepfm_cate.py:73-169
    "deepfm_multi_cate": dict(fm=True, cont=None, multi=True),       # models/deepfm_multi_cate.py:113-240
    "deepfm_multi": dict(fm=True, cont="last", multi=True),          # models/deepfm_multi.py:124-260
    "dnn_pipeline": dict(fm=False, cont="deep", multi=False),        # models/dnn_pipeline.py:68-137
    "dnn_cate": dict(fm=False, cont=None, multi=False),              # models/dnn_cate.py:62-131
    "dnn_multi": dict(fm=False, cont="deep", multi=True),            # models/dnn_multi.py:70-167
    "dnn_multi_cate": dict(fm=False, cont=None, multi=True),         # models/dnn_multi_cate.py:64-162
    "wdl": dict(fm=False, cont="deep", multi=False),                 # models/wdl.py:123-285
    # load-style models (int32 ids, no zero row):
    #   deepfm: FM fields [cate | cont] with cont rows at cate_field_size + j (deepfm.py:66-73)
    #   dnn:    xavier 'weight_mat' table, L1 on every hidden weight (dnn.py:49-52,88-90)
    "deepfm": dict(fm=True, cont="field", multi=False),              # models/deepfm.py:39-162
    "dnn": dict(fm=False, cont="deep", multi=False),                 # models/dnn.py:35-96
}


class ModelSpec:
    """Shape/hyper-parameter description of one reference model.

    model: a key of FAMILIES (the reference's pipeline-style model files + wdl)
    C cont fields, V vector size, S single cate fields, E embedding size,
    cate_index_size (reference `cate_feats_size`), hidden units, multi_ranges
    [[start, end, name], ...] (multi-hot slots, relative to the multi block), Fw wide
    ids (wdl), lr, l2, decay_steps/decay_rate (exponential_decay), Adam betas/eps.
    """

    def __init__(self, model, C=13, V=0, S=26, E=16, cate_index_size=1000, hidden=(400, 400, 400),
                 multi_ranges=(), Fw=0, lr=0.001, l2=1e-5, decay_steps=10000000, decay_rate=0.9,
                 beta1=0.9, beta2=0.999, eps=1e-8, logloss_eps=1e-7, tower="f32"):
        if model not in FAMILIES:
            raise ValueError("unsupported model %r" % model)
        fam = FAMILIES[model]
        self.model = model
        self.cont_mode = fam["cont"]
        self.C = C if fam["cont"] else 0          # cate algs have no cont_feats (data_loader.py:8)
        self.V = 0 if model == "wdl" else V
        self.S, self.E = S, E
        self.cate_index_size = cate_index_size
        self.hidden = list(hidden)
        self.multi_ranges = [list(r) for r in multi_ranges] if fam["multi"] else []
        self.Fw = Fw
        self.lr, self.l2 = lr, l2
        self.decay_steps, self.decay_rate = decay_steps, decay_rate
        self.beta1, self.beta2, self.eps, self.logloss_eps = beta1, beta2, eps, logloss_eps
        if tower not in ("f32", "bf16"):
            raise ValueError("tower must be 'f32' or 'bf16'")
        self.tower = tower      # bf16: the deep tower's GEMMs on bf16 MFMA (config C5), fp32 master weights

    @property
    def fm(self):
        return FAMILIES[self.model]["fm"]

    @property
    def fm_cont(self):
        """The cont fields are FM fields (deepfm_pipeline, deepfm_multi, deepfm)."""
        return self.fm and self.cont_mode in ("first", "last", "field") and self.C > 0

    @property
    def fm_cont_offset(self):
        """Table row of FM cont field 0."""
        return {"last": self.cate_index_size, "field": self.S}.get(self.cont_mode, 0)

    @property
    def zero_row0(self):
        """Row 0 is forced to zeros every step (deepfm_pipeline.py:83-86); wdl.py:44,
        deepfm.py:58-60 and dnn.py:49-52 have no zero row."""
        return self.model not in ("wdl", "deepfm", "dnn")

    @property
    def xavier_table(self):
        """glorot-uniform table named weight_mat (wdl.py:44-47, dnn.py:49-52)."""
        return self.model in ("wdl", "dnn")

    @property
    def table_key(self):
        return "weight_mat" if self.xavier_table else "feats_emb"

    @property
    def first_key(self):
        return "feats" if self.model == "deepfm" else "fm_first_order_emb"   # deepfm.py:60

    @property
    def sparse_table(self):
        """The table (and first-order) Variables are read by tf.nn.embedding_lookup directly,
        so TF updates them with Adam's sparse-apply form (Adam._apply_sparse_shared): wdl.py:44-47,
        132 weight_mat, deepfm.py:57-60,78,85,98 feats_emb / feats, dnn.py:49-54 weight_mat.  The
        pipeline models concat a zero row 0 first (deepfm_pipeline.py:83-86), which densifies the
        gradient: ApplyAdam."""
        return self.model in ("wdl", "deepfm", "dnn")

    @property
    def hidden_reg(self):
        """Regulariser on the hidden weight matrices: wdl.py:272-275 L2, dnn.py:88-90 L1."""
        return {"wdl": "l2", "dnn": "l1"}.get(self.model)

    @property
    def head_l2(self):
        """L2 on the output weights (deepfm_pipeline.py:183, dnn_pipeline.py:131); dnn.py has none."""
        return self.model != "dnn"

    def head_ref_index(self):
        """Reference index of each internal head weight (FM fields internally [cont | cate |
        pooled]; deepfm.py:70-71 orders its FM fields [cate | cont])."""
        n = self.fm_cols + self.hidden[-1] + 1
        idx = np.arange(n)
        if self.model == "deepfm" and self.C:
            C, S = self.C, self.S
            idx[:C] = S + np.arange(C)
            idx[C:C + S] = np.arange(S)
        return idx

    @property
    def fm_cate_offset(self):
        """Added to a cate id for its FM row (deepfm_pipeline.py:89); the deep row is the raw id."""
        return self.C if self.cont_mode == "first" and self.fm else 0

    @property
    def M(self):
        return len(self.multi_ranges)

    @property
    def multi_width(self):
        return sum(e - s for s, e, *_ in self.multi_ranges)

    @property
    def n_rows(self):
        if self.fm_cont:      # deepfm_pipeline.py:77 / deepfm_multi.py:125: cate_index_size + C
            return self.C + self.cate_index_size
        return self.cate_index_size

    @property
    def deep_in(self):
        return self.S * self.E + self.M * self.E + self.C + self.V

    @property
    def F(self):
        """FM fields: [cont (fm_cont) | single cate | pooled slots]."""
        if not self.fm:
            return 0
        return (self.C if self.fm_cont else 0) + self.S + self.M

    @property
    def fm_cols(self):
        return self.F + self.E if self.fm else 0

    @property
    def cate_ld(self):
        return self.S + self.multi_width

    def x0_ref_rows(self):
        """Reference row of W_0 for each internal x0 column < deep_in.  Every pipeline-style
        model concatenates its deep input as [cont, vector, single cate, pooled]
        (deepfm_pipeline.py:123, deepfm_multi.py:188, dnn_multi.py:106, deepfm_multi_cate.py:169,
        wdl.py:179); absent parts are empty."""
        S, E, M, C, V = self.S, self.E, self.M, self.C, self.V
        cat = np.arange(S * E) + C + V
        pool = np.arange(M * E) + C + V + S * E
        cont = np.arange(C)
        vec = np.arange(V) + C
        return np.concatenate([cat, pool, cont, vec])



def _root_to_v(s):
    """Device root state s = sqrt(v) (a tensor) -> TF's v, fl(s * s), as host numpy."""
    a = s.cpu().numpy().astype(np.float64)
    return (a * a).astype(np.float32)


def _v_to_root(v):
    """TF's v (array-like) -> the root state fl(sqrt(v)), host numpy f32."""
    return np.sqrt(np.ascontiguousarray(v, np.float64)).astype(np.float32)

class CTREngine:
    def __init__(self, spec, max_batch, device="cuda", seed=2019, init="device", bwd="atomic",
                 table_rows=None, adam="dense", hist_len=4096, rec_stash=True, fwd_rec=False, gemm="s3",
                 fwd_scatter=None):
        if not torch.cuda.is_available():
            raise _lib.DLError("CTREngine needs a HIP device (no CPU fallback)")
        _lib.lib()
        self.spec = sp = spec
        self.dev = torch.device(device)
        self.B = max_batch
        dev = self.dev
        z = lambda *s, dt=F32: torch.zeros(*s, dtype=dt, device=dev)
        E, S, M = sp.E, sp.S, sp.M
        N = sp.n_rows
        self.N = N
        # ---- layout
        self.cat_col = 0
        self.pool_col = S * E
        self.cont_col = (S + M) * E
        self.vec_col = self.cont_col + sp.C
        self.D0 = sp.deep_in
        dims = [self.D0] + sp.hidden
        self.in_ld = [_ru(d + 1, 16) for d in dims[:-1]]
        self.out_ld = [_ru(h, 16) for h in sp.hidden]
        self.h_ld = [_ru(h + 1, 16) for h in sp.hidden]
        self.fm_ld = _ru(max(sp.fm_cols, 1), 4)
        self.dx_cols = (S + M) * E
        self.dx_ld = _ru(max(self.dx_cols, 4), 4)
        # ---- parameters + Adam state
        rows_pad = _ru(table_rows if table_rows is not None else N, 16)
        self.rows_pad = rows_pad
        if adam not in ("dense", "lazy"):
            raise ValueError("adam must be 'dense' or 'lazy'")
        self.lazy = adam == "lazy"
        if self.lazy:
            # row records + lazy-exact Adam (rec.hip); needs the batch index (with multi-hot
            # slots it also indexes every multi-hot id position: pooling reads caught-up rows)
            bwd = "sorted"
            self.rec_ld = _ru(3 * E + 4, 32)
            self.rec = z(rows_pad, self.rec_ld)
            self.hist_len = hist_len
            self.hist = z(hist_len)
            self.n_rep = sp.C if sp.fm_cont else 0     # FM cont-field rows (replicated, hot)
            R = max(self.n_rep, 1)
            self.g_rep, self.g1_rep = z(_ru(R * E, 4)), z(_ru(R, 4))
            self.rep_touched = z(_ru(R, 16), dt=torch.uint8)
            self.since_flush = 0
            self.table = self.tm = self.tv = self.tg = self.touched = None
            self.first = self.fmm = self.fmv = self.fmg = None
        else:
            self.table = z(rows_pad, E)
            self.tm, self.tv, self.tg = z(rows_pad, E), z(rows_pad, E), z(rows_pad, E)
            self.touched = z(rows_pad, dt=torch.uint8)
            if sp.fm:
                self.first = z(rows_pad)
                self.fmm, self.fmv, self.fmg = z(rows_pad), z(rows_pad), z(rows_pad)
            else:
                self.first = self.fmm = self.fmv = self.fmg = None
        self.W = [z(self.in_ld[l], self.out_ld[l]) for l in range(len(sp.hidden))]
        self.Wm = [torch.zeros_like(w) for w in self.W]
        self.Wv = [torch.zeros_like(w) for w in self.W]
        self.Wt = z(max(o * i for o, i in zip(self.out_ld, self.in_ld)))   # W_l^T scratch for dX
        # fp32 tower products on the bf16 matrix cores through the exact three-plane split
        # (gemm_s3.hip, f32 accuracy): bf16 planes of W (the dX operand, [in][out]) and of W^T
        # (the forward operand, [out][in]), refreshed after every update of W
        if gemm not in ("s3", "f32"):
            raise ValueError("gemm must be 's3' or 'f32'")
        self.s3 = gemm == "s3" and sp.tower == "f32"
        if self.s3:
            zp = lambda n: torch.zeros(n, dtype=torch.int16, device=dev)
            self.Wp = [zp(3 * self.in_ld[l] * self.out_ld[l]) for l in range(len(sp.hidden))]
            self.WTp = [zp(3 * self.out_ld[l] * self.in_ld[l]) for l in range(len(sp.hidden))]
        H = sp.hidden[-1]
        self.head_n = sp.fm_cols + H + 1
        self.w_head = z(_ru(self.head_n, 4))
        self.hm, self.hv = torch.zeros_like(self.w_head), torch.zeros_like(self.w_head)
        self.w_head_prev = torch.zeros_like(self.w_head)
        self.opt = z(_lib.OPT_LEN)   # include/dlamd.h: Adam scalars, per-step sums, status word
        self.opt[:8].copy_(torch.tensor([sp.beta1, sp.beta2, sp.lr, 0.0, sp.beta1, sp.beta2, sp.eps, 0.0]))
        self.wdl = sp.model == "wdl"
        if self.wdl:   # wdl_weights [N + H] (deep-output rows alias wide ids, wdl.py:241-248) + bias
            self.w_rows = N + sp.hidden[-1]
            wr = _ru(self.w_rows, 16)
            self.ww, self.wm, self.wv = z(wr), z(wr), z(wr)
            # wide gradient: int64 fixed point (deterministic integer atomics, head.hip)
            self.wg = z(wr, dt=torch.int64)
            self.w_touched = z(wr, dt=torch.uint8)
            self.wb, self.wbm, self.wbv = z(4), z(4), z(4)
        # wide_lazy (single-GPU wdl with lazy tables): wdl_weights as {w, m, v, stamp} records
        # with lazy-exact Adam (wide.hip): the batch's unique wide ids indexed, gathered caught
        # up into the head's compact local table [— (Fw) | deep-output rows | unique rows], and
        # only those rows (and the H deep-output rows) updated — in place of the dense L2 sweep
        # over all N + H rows (wdl.py:270-271); bit-identical to it.  DLAMD_WIDE_LAZY=0: dense.
        self.wide_lazy = bool(self.wdl and self.lazy and type(self) is CTREngine
                              and os.environ.get("DLAMD_WIDE_LAZY", "1") != "0")
        if self.wide_lazy:
            Fw, Hh, Bm = sp.Fw, sp.hidden[-1], max_batch
            nw = Bm * Fw
            self.wrec = z(_ru(self.w_rows, 16), 4)    # {w, m, v, stamp} (wide.hip)
            self.wloc = z(_ru(Fw + Hh + nw, 4))
            self.wgloc = z(Fw + Hh + nw, dt=torch.int64)
            self.wstash = z(max(nw, 1), 4)
            self.wdmark = z(_ru(Hh, 16), dt=torch.uint8)
            self.wlong = z(nw + 1, dt=torch.int32)   # dl_wide_seg_grad's hot-row list
            # the update kernels' per-block partial sums of the touched rows' L2 term
            self.wsq_part = z(max(1, int(_lib.lib().dl_wide_update_blocks(nw, Hh))))
            self.wsq = z(2, dt=torch.int64)      # L2 term of the rows the last step left (a flush; fixed point)
            self._wsq_step = -1
            # the running loss's wide L2 term (loss_sum_begin / loss_sum_end): per-block slots the
            # update and flush kernels add to, and each unique row's replayed steps' w^2 (gather)
            self.wacc = z(_lib.LOSS_ACC_SLOTS, dt=torch.float64)
            self.wrep = z(max(nw, 1))
            self.in_wide_loc = z(Bm, Fw, dt=torch.int64)
            wsb = _lib.lib().dl_index_workspace_bytes(max(1, nw))
            self.widx_ws = z(wsb, dt=torch.uint8)
            self.widx_keys, self.widx_refs, self.widx_uniq = (z(max(nw, 1), dt=torch.int32) for _ in range(3))
            self.widx_off = z(nw + 1, dt=torch.int32)
            self.widx_n = z(4, dt=torch.int32)
            self.winv = z(max(nw, 1), dt=torch.int32)
            WL = _lib.EmbLayout()
            WL.n_rows = self.w_rows
            WL.batch = Bm
            WL.emb_dim = sp.E
            WL.cate_fields = Fw
            WL.cate_ld = max(Fw, 1)
            WL.use_fm = 0
            WL.zero_row0 = 0
            self.wlayout = WL
        self.err = z(4, dt=torch.int32)       # the batch's id-validation word (per buffer set)
        # batches prefetched ahead (train_step(next_batch=[...])): buffer sets = pf_depth + 1
        self.pf_depth = int(os.environ.get("DLAMD_PF_DEPTH", "1")) if type(self) is CTREngine else 1
        # running loss of a training loop (dl_loss_accumulate, every step inside its graph):
        # [sum of data terms, sum of regulariser terms, steps]
        self.loss_acc = z(4, dt=torch.float64)
        # table update form (TF: ApplyAdam, or the sparse-apply form for direct lookups)
        self.rec_flags = (_lib.REC_FIRST if sp.fm else 0) | (_lib.REC_SPARSE_ADAM if sp.sparse_table else 0)
        self.rows_sparse = _lib.ROWS_SPARSE_ADAM if sp.sparse_table else 0
        self._status_q = []
        self._status_host = None
        self.host_wait = 0.0
        # DLAMD_STATUS_RING=1: the step's last kernel writes its status into pinned host memory
        # (dl_loss_accumulate's ring) instead of a device-to-host copy after each step
        self._ring = None
        if os.environ.get("DLAMD_STATUS_RING", "1") == "1" and type(self) is CTREngine:
            self._ring = torch.zeros(8, dtype=torch.int32, pin_memory=True)
            self._ring_np = self._ring.numpy()
            self._ring_sent = None
        # ---- activations / workspaces
        B = max_batch
        self.x0 = z(B, self.in_ld[0])
        self.x0[:, self.D0] = 1.0
        self.h = []
        for l, hdim in enumerate(sp.hidden):
            t = z(B, self.h_ld[l])
            t[:, hdim] = 1.0
            self.h.append(t)
        self.dh = [z(B, self.h_ld[l]) for l in range(len(sp.hidden))]
        # the forward's ReLU sign bitmasks (s3 tower; dl_gemm_s3_nt_bits): the dX ReluGrad
        # epilogue reads 2 bytes per 16 columns instead of the f32 activations.
        # DLAMD_RELU_BITS=0 keeps the f32 mask.
        self.relu_bits = bool(self.s3 and os.environ.get("DLAMD_RELU_BITS", "1") != "0")
        self.hbits_ld = [_ru(-(-h // 16), 32) for h in sp.hidden]
        self.hbits = [z(B, self.hbits_ld[l], dt=torch.int16) for l in range(len(sp.hidden) - 1)] if self.relu_bits else []
        self.bf = sp.tower == "bf16"
        # bf16 tower without pooled fields: the embedding forward writes the bf16 x0 itself
        self.x0_direct = self.bf and not sp.M
        if self.bf:
            # bf16 tower operands: x0 and hidden activations (bias ones columns included),
            # gradients, and bf16 copies of the fp32 master weights (refreshed after each update)
            zb = lambda *sh: torch.zeros(*sh, dtype=torch.bfloat16, device=dev)
            self.x0b = zb(B, self.in_ld[0])
            self.x0b[:, self.D0] = 1.0
            self.hb = []
            for l, hdim in enumerate(sp.hidden[:-1]):
                t = zb(B, self.h_ld[l])
                t[:, hdim] = 1.0
                self.hb.append(t)
            self.dhb = [zb(B, self.h_ld[l]) for l in range(len(sp.hidden))]
            self.Wb = [zb(self.in_ld[l], self.out_ld[l]) for l in range(len(sp.hidden))]
            # W^T (k-contiguous) for the forward product; dW reads the batch-major X and dY
            # directly (transposing LDS reads in the kernel), so there are no X^T / dY^T copies
            self.WbT = [zb(self.out_ld[l], self.in_ld[l]) for l in range(len(sp.hidden))]
        self.dx0 = z(B, self.dx_ld)
        self.fm_out = z(B, self.fm_ld)
        self.fm_sum = z(B, E)
        self.score, self.z, self.dz = z(B), z(B), z(B)
        self.head_grid = "dl_wdl_head_grid" if self.wdl else "dl_head_grid"   # slab rows per batch size
        self.head_blocks = call_int(self.head_grid, B)
        self.head_slab = z(self.head_blocks, sp.fm_cols + H + 2)
        self.in_wide = z(B, max(sp.Fw, 1), dt=torch.int64)
        # split-K slabs of the weight gradients: the double-buffered s3 TN kernel (one block per
        # CU, 2 column tiles) runs best at 32 (scripts/s3_bench.py: 147 vs 152 us at 64)
        # (the bf16 tower's ring kernel, one 144 x 400 block per CU, takes up to 96: _bf16_dw_splits)
        dflt = 32 if self.s3 else 96 if self.bf else 64
        self.splits = max(1, min(int(os.environ.get("DLAMD_DW_SPLITS", dflt)), B // (512 if self.bf else 1024)))
        self.dw_splits = self._dw_splits(B, fixed="DLAMD_DW_SPLITS" in os.environ)
        # sized for the cap: a smaller batch may choose more splits than the largest one did
        # (one slab set per layer when the dense Adams run as one launch after the backward's
        # GEMMs, _adam_fused: each layer's slabs must survive until then)
        per = [self.splits * i * o for i, o in zip(self.in_ld, self.out_ld)]
        self.w_slab = z(sum(per) if self._adam_fused() else max(per))
        offs = np.cumsum([0] + per)
        self.w_slabs = [self.w_slab[offs[l]:offs[l + 1]] if self._adam_fused() else self.w_slab
                        for l in range(len(per))]
        self.layout = self._layout(B)
        self.bwd_blocks = _lib.lib().dl_embed_bwd_grid(C_ref(self.layout))
        self.cont_slab = z(max(1, self.bwd_blocks * sp.C * (E + 1)))
        self.fm_pool_col = sp.F - M      # head column of the first pooled first-order output
        if M:
            self.slot_start = torch.tensor([r[0] for r in sp.multi_ranges], dtype=torch.int32, device=dev)
            self.slot_end = torch.tensor([r[1] for r in sp.multi_ranges], dtype=torch.int32, device=dev)
            self.cnt_emb, self.cnt_first = z(B, M), z(B, M)
            if self.lazy:
                # per (sample, slot): the slot gradient (E floats) and the first-order one at
                # column E of a row padded to whole 128-B lines (one line fetch per multi-hot
                # reference in the backward instead of two: dl_pool_desc.g_pitch)
                gp = 0 if os.environ.get("DLAMD_GPOOL_PACKED") else _ru(E + 1, 32)   # env: A/B only
                self.g_pool = z(B, M, gp or E)
                self.g1_pool = self.g_pool.view(-1)[E:] if gp else z(B, M)
                self.pool_desc = _lib.PoolDesc(
                    slot_start=self.slot_start.data_ptr(), slot_end=self.slot_end.data_ptr(), n_slots=M,
                    fm_col=self.fm_pool_col, dx0_pool_col=S * E, g_pitch=gp, x0=self.x0.data_ptr(),
                    cnt_emb=self.cnt_emb.data_ptr(), cnt_first=self.cnt_first.data_ptr(),
                    g_pool=self.g_pool.data_ptr(), g1_pool=self.g1_pool.data_ptr())
        # batch reference index (deterministic backward)
        self.bwd = bwd
        self.n_slot = (S if sp.fm else 0) + S + (sp.multi_width if self.lazy else 0)
        self.n_refs = B * self.n_slot
        # wide_lazy: the table ids and the wide ids in ONE index build (dl_index_build_pair): the
        # table's index arrays hold both sets' sorted references and unique rows, the wide set's
        # own arrays (widx_*) are split out of them.  DLAMD_INDEX_PAIR=0: two builds.
        self.index_pair = bool(getattr(self, "wide_lazy", False) and bwd == "sorted"
                               and os.environ.get("DLAMD_INDEX_PAIR", "1") != "0")
        if bwd == "sorted":
            cap = self.n_refs + (B * sp.Fw if self.index_pair else 0)
            wsb = _lib.lib().dl_index_workspace_bytes(max(1, cap))
            self.idx_ws = z(wsb, dt=torch.uint8)
            self.idx_keys = z(cap, dt=torch.int32)
            self.idx_refs = z(cap, dt=torch.int32)
            self.idx_uniq = z(cap, dt=torch.int32)
            self.idx_off = z(cap + 1, dt=torch.int32)
            self.idx_n = z(4, dt=torch.int32)
            self.idx_inv = z(cap, dt=torch.int32) if self.lazy else None
            if self.index_pair:   # the second build's workspace and key array are not needed
                self.widx_ws = z(256, dt=torch.uint8)
                self.widx_keys = z(1, dt=torch.int32)
        if self.lazy:
            self.rows_u = z(self.n_rep + self.n_refs, E)
            self.rows_u1 = z(self.n_rep + self.n_refs)
            # rec_stash: the gather also stashes the caught-up moments for the backward's update.
            # Off by default — re-reading the record in the backward measured faster on both
            # kernels (gather 328 -> 232 us, backward 505 -> 447 us at C2; profiles/r01l).
            self.mv_u = z(self.n_rep + self.n_refs, int(_lib.lib().dl_rec_stash_floats(E))) if rec_stash else None
            # hot rows' chunked segment sums (dl_rec_bwd_adam: Zipf rows over many blocks)
            self.hot_ws = z(int(_lib.lib().dl_rec_bwd_workspace_bytes(self.n_refs, E)), dt=torch.uint8)
        # fwd_rec: the forward reads the cate rows straight from the records (dl_embed_fwd_rec)
        # instead of gathering the batch's unique rows and reading them back through the
        # inverse map; only the C replicated cont rows are gathered.  Single-valued fields.
        # Off by default: bit-identical, but at C2 it measured 444 us against 214 + 123 us for
        # the gather + indexed pair — the in-register catch-up of every reference at 2
        # waves/SIMD (169 VGPRs) costs ~190 us that the gather's catch-up hides (253 us with
        # no rows lagging; scripts/catchup_cost.py).
        self.fwd_rec = bool(fwd_rec and self.lazy and not M and not rec_stash)
        # fwd_scatter (opt-in, DLAMD_FWD_SCATTER=1): the gather writes each caught-up row
        # straight to the references reading it (dl_rec_gather_scatter: FM staging rows,
        # first-order outputs, x0's deep columns, multi-hot staging rows) and
        # dl_embed_fwd_staged sums the FM terms per sample from the staging rows — random
        # 64-B writes in place of the indexed forward's random 64-B reads through the inverse
        # map.  Measured slower end to end (profiles/r03d: C2 2.45 vs 2.32 ms, the gather
        # +170 us for the forward's -58 us; C3 gather +830 us for pooling's -95 us): the
        # per-reference segment walk serialises dependent loads in the gather's waves.
        if fwd_scatter is None:
            fwd_scatter = os.environ.get("DLAMD_FWD_SCATTER", "0") != "0"
        self.fwd_scatter = bool(fwd_scatter and self.lazy and not self.fwd_rec and type(self) is CTREngine)
        self.fmst = z(self.n_rep + B * S, E) if (self.fwd_scatter and sp.fm) else None
        # multi-hot staging (scatter form): position l of sample b at row b * multi_width + l
        mw = sp.multi_width
        self.mst = z(B * mw, E) if (self.fwd_scatter and M) else None
        self.mst1 = z(B * mw) if (self.fwd_scatter and M and sp.fm) else None
        # static input slots (graph capture reads from these)
        self.in_label = z(B)
        self.in_cont = z(B, max(sp.C, 1))
        self.in_vec = z(B, max(sp.V, 1))
        self.in_cate = z(B, max(sp.cate_ld, 1), dt=torch.int64)
        self.graphs = {}        # (buffer set, batch) -> captured step
        # predict on a flushed table reads dense p / first-order planes written by the flush
        # (DLAMD_FLAT_PLANES=0: each reference reads its record's first line instead)
        self.flat_planes = os.environ.get("DLAMD_FLAT_PLANES", "1") != "0"
        self.prof = None
        self.steps = 0
        if init == "device":
            self.init_device(seed)

    # ------------------------------------------------------------------ layout
    def _layout(self, B):
        sp = self.spec
        L = _lib.EmbLayout()
        L.n_rows = self.N
        L.fm_cont_offset = sp.fm_cont_offset                            # deepfm_multi.py:139
        L.fm_cate_offset = sp.fm_cate_offset                            # deepfm_pipeline.py:89
        L.deep_cate_offset = 0                                          # :120 raw ids
        L.batch = B
        L.emb_dim = sp.E
        L.cont_fields = sp.C
        L.vector_size = sp.V
        L.cate_fields = sp.S
        L.cate_ld = sp.cate_ld
        L.fm_cont = 1 if sp.fm_cont else 0
        L.use_fm = 1 if sp.fm else 0
        L.fm_extra = sp.M if sp.fm else 0
        L.zero_row0 = 1 if sp.zero_row0 else 0                         # :83-86 (wdl.py:49: none)
        L.x0_ld = self.in_ld[0]
        L.x0_cont_col = self.cont_col if sp.C else -1
        L.x0_vec_col = self.vec_col if sp.V else -1
        L.x0_cat_col = self.cat_col
        L.x0_pool_col = self.pool_col
        L.fm_ld = self.fm_ld
        L.dx0_ld = self.dx_ld
        L.dx0_cat_col = 0
        L.multi_width = sp.multi_width if self.lazy else 0
        L.cont_rows_compact = 1 if self.lazy else 0     # records: cont rows gathered first into rows_u
        L.x0_bf16 = 1 if self.x0_direct else 0           # bf16 tower: the forward writes x0 as bf16
        return L

    def _flat_layout(self, B):
        """The layout of the dense-table forward over the flushed planes (the replicated FM
        cont rows read from the planes in place, no batch index)."""
        L = self._layout(B)
        L.cont_rows_compact = 0
        L.multi_width = 0
        return L

    # ------------------------------------------------------------------ params
    def init_device(self, seed):
        """Reference initialisers (deepfm_pipeline.py:78-80,131-169): table ~ N(0, 0.01),
        first-order ~ U[0,1), dense weights/biases ~ N(0, glorot) (numpy, seeded)."""
        sp = self.spec
        s = _lib.stream_handle()
        if self.lazy:   # same values as the dense engine: initialise dense, then pack
            self.table = torch.zeros(self.rows_pad, sp.E, device=self.dev)
            self.first = torch.zeros(self.rows_pad, device=self.dev) if sp.fm else None
        if sp.xavier_table:   # xavier_initializer (wdl.py:44-47, dnn.py:49-52): U(-lim, lim), lim = sqrt(6/(N+E))
            lim = math.sqrt(6.0 / (self.N + sp.E))
            call("dl_init_random", ptr(self.table), self.table.numel(), 1, -lim, 2 * lim, seed, 0, s)
        if self.wdl:
            call("dl_init_random", ptr(self.ww), _ru(self.ww.numel(), 4), 0, 0.0,
                 math.sqrt(2.0 / self.w_rows), seed + 3, 0, s)                           # wdl.py:241-244
            self.ww[self.w_rows:].zero_()
            self.wb[0] = float(np.random.default_rng(seed).standard_normal())
        if not sp.xavier_table:
            call("dl_init_random", ptr(self.table), self.table.numel(), 0, 0.0, 0.01, seed, 0, s)
        if self.first is not None:
            call("dl_init_random", ptr(self.first), self.first.numel(), 1, 0.0, 1.0, seed + 1, 0, s)
        if self.lazy:
            self._pack(self.table, self.first)
            self.table = self.first = None
        rng = np.random.default_rng(seed)
        dims = [self.D0] + sp.hidden
        for l in range(len(sp.hidden)):
            g = math.sqrt(2.0 / (dims[l] + dims[l + 1]))
            self._set_layer(l, (rng.standard_normal((dims[l], dims[l + 1])) * g).astype(np.float32),
                            (rng.standard_normal((1, dims[l + 1])) * g).astype(np.float32), ref_order=False)
        H = sp.hidden[-1]
        g = math.sqrt(2.0 / (self.head_n))
        w = np.zeros(self.head_n, np.float32)
        w[:-1] = rng.standard_normal(self.head_n - 1) * g
        w[-1] = rng.standard_normal()
        self.w_head[: self.head_n].copy_(torch.from_numpy(w))
        if getattr(self, "wide_lazy", False):
            self._wide_pack()
        torch.cuda.synchronize()

    def _set_layer(self, l, W, b, ref_order=True):
        din = W.shape[0]
        Wi = np.zeros((self.in_ld[l], self.out_ld[l]), np.float32)
        if l == 0 and ref_order:
            Wi[:din, : W.shape[1]] = W[self.spec.x0_ref_rows()]
        else:
            Wi[:din, : W.shape[1]] = W
        Wi[din, : W.shape[1]] = b.reshape(-1)
        self.W[l].copy_(torch.from_numpy(Wi))
        self._refresh_wb(l)

    def _refresh_wb(self, l, s=None):
        """The tower's operand copies of the fp32 master weights W_l: bf16 tower, bf16 W and
        W^T; split (s3) GEMMs, the three bf16 planes of W and of W^T."""
        if getattr(self, "s3", False):
            s = s if s is not None else _lib.stream_handle()
            i, o = self.in_ld[l], self.out_ld[l]
            call("dl_split3", ptr(self.W[l]), i, o, o, 0, ptr(self.Wp[l]), o, i * o, s)
            call("dl_split3", ptr(self.W[l]), i, o, o, 1, ptr(self.WTp[l]), i, i * o, s)
        if self.bf:
            s = s if s is not None else _lib.stream_handle()
            call("dl_cast_bf16", ptr(self.W[l]), self.in_ld[l], self.out_ld[l], self.out_ld[l], ptr(self.Wb[l]),
                 self.out_ld[l], s)
            call("dl_transpose_bf16", ptr(self.W[l]), 1, self.in_ld[l], self.out_ld[l], self.out_ld[l],
                 ptr(self.WbT[l]), self.in_ld[l], s)

    def load_params(self, P):
        """Inject reference-layout parameters (dict of numpy arrays as in oracle/ctr_ref.py)."""
        sp = self.spec
        N = self.N
        tab = torch.from_numpy(np.ascontiguousarray(P[sp.table_key], np.float32))
        first = (torch.from_numpy(np.ascontiguousarray(P[sp.first_key][:, 0], np.float32))
                 if sp.fm else None)
        if self.lazy:
            self._pack(tab.to(self.dev), first.to(self.dev) if first is not None else None)
        else:
            self.table.zero_()
            self.table[:N].copy_(tab)
            if self.first is not None:
                self.first.zero_()
                self.first[:N].copy_(first)
        for l in range(len(sp.hidden)):
            self._set_layer(l, P["deep_%d" % l], P["deep_bias_%d" % l])
        if self.wdl:
            self.ww.zero_()
            self.ww[: self.w_rows].copy_(torch.from_numpy(np.ascontiguousarray(P["wdl_weights"][:, 0], np.float32)))
            self.wb.zero_()
            self.wb[:1].copy_(torch.from_numpy(np.asarray(P["wdl_bias"], np.float32).reshape(-1)))
            if self.wide_lazy:
                self.wm.zero_()
                self.wv.zero_()
                self._wide_pack()
            torch.cuda.synchronize()
            return
        if sp.fm:
            w = np.concatenate([P["deep_fm_weight"][:, 0], P["deep_fm_bias"].reshape(-1)]).astype(np.float32)
        else:
            w = np.concatenate([P["deep_res"][:, 0], P["deep_res_bias"].reshape(-1)]).astype(np.float32)
        w = w[sp.head_ref_index()]
        self.w_head.zero_()
        self.w_head[: self.head_n].copy_(torch.from_numpy(w))
        torch.cuda.synchronize()

    def params(self):
        """Export parameters in the reference layout (numpy)."""
        sp = self.spec
        N = self.N
        if self.lazy:
            self.flush()
            rec = self.rec[:N]
            P = {sp.table_key: rec[:, : sp.E].cpu().numpy()}
            if sp.fm:
                P[sp.first_key] = rec[:, sp.E: sp.E + 1].cpu().numpy()
        else:
            P = {sp.table_key: self.table[:N].cpu().numpy()}
            if self.first is not None:
                P[sp.first_key] = self.first[:N].cpu().numpy()[:, None]
        P.update(self.dense_params())
        return P

    def _dw_splits(self, B, fixed=False):
        """Per-layer split-K slab counts of the weight gradients (fixed: self.splits for all)."""
        base = max(1, min(self.splits, B // (512 if self.bf else 1024)))
        if fixed or not (self.s3 or self.bf):
            return [base] * len(self.spec.hidden)
        if self.bf:
            return [_bf16_dw_splits(i, B, base) for i in self.in_ld]
        return [_s3_dw_splits(i, o, B, base) for i, o in zip(self.in_ld, self.spec.hidden)]

    def dense_params(self):
        """The dense parameters (hidden layers, head or wdl weights + bias) in the reference
        layout (numpy); the wide records are caught up first."""
        return self._export_dense(self.W, self.w_head, self._wide_state()[0], getattr(self, "wb", None))

    def dense_state(self):
        """Adam moments of the dense parameters (hidden layers, head / wdl weights) in the
        reference layout: {"m": {key: array}, "v": {key: array}} (tests; the table's are in
        adam_state())."""
        _, wm, wv = self._wide_state()
        return {"m": self._export_dense(self.Wm, self.hm, wm, getattr(self, "wbm", None)),
                "v": self._export_dense(self.Wv, self.hv, wv, getattr(self, "wbv", None))}

    # ------------------------------------------------------------------ wide records (wdl)
    def _wide_pack(self):
        """Dense wdl_weights (+ moments) -> records {w, m, v, stamp = current step}."""
        n = self.ww.shape[0]
        self.wrec.zero_()
        self.wrec[:n, 0].copy_(self.ww)
        self.wrec[:n, 1].copy_(self.wm)
        self.wrec[:n, 2].copy_(self.wv)
        self.wrec.view(torch.int32)[:, 3] = int(self.opt[7].item())
        self._wsq_step = -1

    def _wide_state(self):
        """(w, m, v) of wdl_weights as device tensors (records: caught up first), or Nones."""
        if not getattr(self, "wdl", False):
            return None, None, None
        if not self.wide_lazy:
            return self.ww, self.wm, self.wv
        self._wide_flush()
        return self.wrec[:, 0], self.wrec[:, 1], self.wrec[:, 2]

    def _wide_flush(self):
        """Every wide record caught up to the current step; the L2 term of the rows the last
        step did not touch (their pre-update w^2) is left in wsq for loss()."""
        if self._wsq_step == self.steps:
            return
        self.wsq.zero_()
        call("dl_wide_rec_flush", ptr(self.wrec), self.w_rows, self.spec.l2, ptr(self.hist), self.hist_len,
             ptr(self.opt), ptr(self.wsq), ptr(self.wacc), _lib.stream_handle())
        self._wsq_step = self.steps

    def _export_dense(self, Ws, head, ww, wb):
        """Augmented hidden-layer matrices (bias row, x0 column order), the permuted head
        vector and the wdl weights -> reference keys and layouts."""
        sp = self.spec
        P = {}
        dims = [self.D0] + sp.hidden
        for l in range(len(sp.hidden)):
            Wi = Ws[l].cpu().numpy()
            W = Wi[: dims[l], : dims[l + 1]]
            if l == 0:
                Wr = np.zeros_like(W)
                Wr[sp.x0_ref_rows()] = W
                W = Wr
            P["deep_%d" % l] = W.copy()
            P["deep_bias_%d" % l] = Wi[dims[l], : dims[l + 1]][None, :].copy()
        if self.wdl:
            P["wdl_weights"] = ww[: self.w_rows].cpu().numpy()[:, None].copy()
            P["wdl_bias"] = wb[:1].cpu().numpy().copy()
            return P
        wi = head[: self.head_n].cpu().numpy()
        w = np.empty_like(wi)
        w[sp.head_ref_index()] = wi
        if sp.fm:
            P["deep_fm_weight"], P["deep_fm_bias"] = w[:-1, None].copy(), w[-1:].copy()
        else:
            P["deep_res"], P["deep_res_bias"] = w[:-1, None].copy(), w[-1:].reshape(1, 1).copy()
        return P

    # ------------------------------------------------------------------ row records
    def _pack(self, table, first):
        """Dense table (+ first-order) -> row records with zero Adam moments, stamped
        with the current step (a fully caught-up state)."""
        E = self.spec.E
        n = table.shape[0]
        self.rec.zero_()
        self.rec[:n, :E].copy_(table)
        if first is not None:
            self.rec[: first.shape[0], E].copy_(first)
        self.rec.view(torch.int32)[:, E + 3] = int(self.opt[7].item())
        self.since_flush = 0
        self.planes_step = -1   # the planes (if any) no longer match the records
        torch.cuda.synchronize()

    def flush(self, planes=False):
        """Catch every row record up to the current step (no-op for the dense engine).
        planes=True also writes every row's p and first-order weight out as dense planes
        (the table predict's plain lookup reads, _forward)."""
        if not self.lazy:
            return
        pp = w1 = None
        flags = self.rec_flags
        if planes and getattr(self, "p_plane", None) is None:
            # FM models: one slot plane, rows x 2E f32 (p, then the first-order weight in column E:
            # an FM reference's row and weight in one 128-B slot, one random request instead of
            # two — 3.3 GB at 26 M rows, E = 16); otherwise a rows x E p plane (1.7 GB).  Dropped
            # again when training resumes (train_step); without the memory, predict reads the
            # records instead
            try:
                self.p_plane = torch.empty(self.rec.shape[0], 2 * self.spec.E if self.spec.fm else self.spec.E,
                                           device=self.dev)
                self.w1_plane = None
            except torch.cuda.OutOfMemoryError:
                self.p_plane = self.w1_plane = None
                self.flat_planes = False
                planes = False
        if planes:
            pp, w1 = self.p_plane, self.w1_plane
            if self.spec.fm:
                flags |= _lib.REC_PLANE_SLOTS
        self._c("rec_flush", "dl_rec_flush", ptr(self.rec), self.rec_ld, self.spec.E, flags,
                self.rec.shape[0], ptr(self.hist), self.hist_len, ptr(self.opt), ptr(pp), ptr(w1),
                _lib.stream_handle())
        self.planes_step = self.steps if planes else getattr(self, "planes_step", -1)
        if getattr(self, "wide_lazy", False):
            self._wide_flush()
        self.since_flush = 0

    def plane_lookup(self, B, x0, s, deep=True, gtab=None):
        """The lookup over flush(planes=True)'s planes: FM models read the slot plane (row and
        first-order weight in one 128-B slot, dl_embed_fwd_slots), the others the p plane.
        deep=False: the deep embeddings are not written to x0 (x0_cat_col = -1): the first tower
        layer reads them from the plane itself (fused_gather_l0).  gtab: the deep rows' plane
        offsets go to gtab as well (dl_embed_fwd_gtab, fused_gather_tab) and fm_sum (backward
        only) is not written."""
        L = self._flat_layout(B)
        if not deep:
            L.x0_cat_col = -1
        if gtab is not None:
            self._c("embed_fwd", "dl_embed_fwd_gtab", C_ref(L), ptr(self.p_plane), 1 if self.spec.fm else 0,
                    ptr(self.in_cate), ptr(self.in_cont), ptr(self.in_vec), ptr(x0), ptr(self.fm_out), None,
                    ptr(gtab), ptr(self.err), s)
        elif self.spec.fm:
            self._c("embed_fwd", "dl_embed_fwd_slots", C_ref(L), ptr(self.p_plane),
                    ptr(self.in_cate), ptr(self.in_cont), ptr(self.in_vec), ptr(x0), ptr(self.fm_out),
                    ptr(self.fm_sum), ptr(self.err), s)
        else:
            self._c("embed_fwd", "dl_embed_fwd", C_ref(L), ptr(self.p_plane), None,
                    ptr(self.in_cate), ptr(self.in_cont), ptr(self.in_vec), ptr(x0), ptr(self.fm_out),
                    ptr(self.fm_sum), ptr(self.err), s)

    def fused_gather_rows(self):
        """Whether the lazy single-GPU forward (rec_gather + the indexed lookup) lets the first
        s3 tower layer gather the deep rows from the batch's compact rows itself
        (dl_gemm_s3_nt_gather_rows: the lookup writes the FM side and x0's cont / pooled columns,
        the layer reads rows_u through the inverse map and writes x0's deep columns for dw_l0 —
        bit-identical to the lookup writing them, tests/test_gpu_parity.py).  Same requirements
        as fused_gather_l0; DLAMD_FUSED_GATHER=0 turns both off."""
        sp = self.spec
        if (os.environ.get("DLAMD_FUSED_GATHER", "1") == "0" or not self.s3 or self.bf or not self.lazy
                or type(self) is not CTREngine or self.fwd_rec or self.fwd_scatter):
            return False
        return (self.cat_col == 0 and sp.E in (8, 16, 32, 64) and 0 < sp.S <= 40 and (sp.S * sp.E) % 32 == 0
                and sp.S * sp.E <= self.in_ld[0] and self.rows_u.numel() * 4 < 0xFFFFFF00
                and self.idx_inv is not None)

    def fused_gather_tab(self, B, force=False):
        """Whether predict's fused front takes the table form: the FM-side lookup writes the deep
        rows' plane offsets (dl_embed_fwd_gtab, which reads the same ids) and the first layer
        stages them as they stand instead of loading and range-checking the ids itself
        (dl_gemm_s3_nt_gather_tab) — bit-identical (tests/test_gpu_parity.py).  On top of
        fused_gather_l0: E = 8 / 16 with the FM slots in the lookup's short forms.  Off by
        default (DLAMD_GATHER_TAB=1 turns it on; force: the bench's A/B): measured alone the layer
        runs 7-17 us faster, but the lookup + layer pair moves 0-1 us (profiles/r06y/)."""
        sp = self.spec
        if (os.environ.get("DLAMD_GATHER_TAB", "0") != "1" and not force) or sp.M:
            return False
        if _lib.lib().dl_embed_fwd_gtab_ok(C_ref(self._flat_layout(B))) != 1:
            return False
        n = -(-B // 256) * sp.S * 272
        if getattr(self, "gtab", None) is None or self.gtab.numel() < n:
            self.gtab = torch.empty(n, dtype=torch.int32, device=self.dev)
        return True

    def fused_gather_l0(self):
        """Whether predict on current planes fuses the deep lookup into the first tower layer
        (dl_gemm_s3_nt_gather: the f32 tower's A stream reads each sample's embedding rows from
        the plane through its ids, x0's deep columns are never written or read — bit-identical
        to the lookup + GEMM pair, tests/test_gpu_parity.py).  The s3 tower only, the deep
        columns first in x0 and whole 32-deep chunks, a plane within one 32-bit buffer range;
        DLAMD_FUSED_GATHER=0 turns it off."""
        sp = self.spec
        if os.environ.get("DLAMD_FUSED_GATHER", "1") == "0" or not self.s3 or self.bf or sp.M:
            return False
        pl = getattr(self, "p_plane", None)
        return (pl is not None and self.cat_col == 0 and sp.E in (8, 16, 32, 64) and 0 < sp.S <= 40
                and (sp.S * sp.E) % 32 == 0 and sp.S * sp.E <= self.in_ld[0]
                and pl.shape[0] * pl.shape[1] * 4 < 0xFFFFFF00)

    def adam_state(self):
        """Table Adam state in the dense layout (tests, checkpoints): dict of m, v (+ m1, v1) as
        numpy.  The device keeps the root state s = sqrt(v) (csrc/common.h adam_elem_root);
        v is exported as fl(s * s)."""
        E, N = self.spec.E, self.N
        if not self.lazy:
            d = {"m": self.tm[:N].cpu().numpy(), "v": _root_to_v(self.tv[:N])}
            if self.first is not None:
                d["m1"], d["v1"] = self.fmm[:N].cpu().numpy(), _root_to_v(self.fmv[:N])
            return d
        self.flush()
        r = self.rec[:N]
        d = {"m": r[:, E + 4: 2 * E + 4].cpu().numpy(), "v": _root_to_v(r[:, 2 * E + 4: 3 * E + 4])}
        if self.spec.fm:
            d["m1"], d["v1"] = r[:, E + 1].cpu().numpy(), _root_to_v(r[:, E + 2])
        return d

    def set_adam_state(self, d):
        """Inverse of adam_state() (v imported as s = fl(sqrt(v))); for records, stamps the rows
        with the current step."""
        E, N = self.spec.E, self.N
        t = lambda k: torch.from_numpy(np.ascontiguousarray(d[k], np.float32)).to(self.dev)
        s = lambda k: torch.from_numpy(_v_to_root(d[k])).to(self.dev)
        if not self.lazy:
            self.tm[:N].copy_(t("m"))
            self.tv[:N].copy_(s("v"))
            if self.first is not None and "m1" in d:
                self.fmm[:N].copy_(t("m1"))
                self.fmv[:N].copy_(s("v1"))
            return
        self.rec[:N, E + 4: 2 * E + 4].copy_(t("m"))
        self.rec[:N, 2 * E + 4: 3 * E + 4].copy_(s("v"))
        if self.spec.fm and "m1" in d:
            self.rec[:N, E + 1].copy_(t("m1"))
            self.rec[:N, E + 2].copy_(s("v1"))
        self.rec.view(torch.int32)[:, E + 3] = int(self.opt[7].item())
        self.since_flush = 0
        self.planes_step = -1

    # ------------------------------------------------------------------ inputs
    def stage(self, batch):
        """Copy one batch (dict of tensors/arrays, reference keys) into the static slots."""
        sp = self.spec
        lab = batch["label"]
        B = int(np.prod(lab.shape))
        if B > self.B:
            raise ValueError("batch %d > engine max_batch %d" % (B, self.B))
        _copy_in(self.in_label[:B], lab, F32, self.dev)
        if sp.C:
            _copy_in(self.in_cont[:B, : sp.C], batch["cont_feats"], F32, self.dev)
        if sp.V:
            _copy_in(self.in_vec[:B, : sp.V], batch["vector_feats"], F32, self.dev)
        _copy_in(self.in_cate[:B, : sp.cate_ld], batch["cate_feats"], torch.int64, self.dev)
        if sp.Fw:
            _copy_in(self.in_wide[:B, : sp.Fw], batch["wide_feats"], torch.int64, self.dev)
        return B

    # ------------------------------------------------------------------ step
    def _cont(self):
        return self.in_cont if self.spec.C else None

    def _c(self, label, name, *args):
        """Launch one C-ABI entry point; with profiling on, bracket it with events
        on the launch stream (bench.py's live per-kernel timing)."""
        if self.prof is None:
            return call(name, *args)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        call(name, *args)
        e1.record()
        self.prof.append((label, e0, e1))

    def _forward(self, B, s, train=False):
        sp = self.spec
        L = self.layout
        L.batch = B
        x0 = self.x0b if self.x0_direct else self.x0
        fused = False   # the deep lookup inside the first tower layer (predict on planes only)
        if sp.M and not self.lazy:  # pooled vectors must be in x0 before the FM second order reads them
            self._c("pool_fwd", "dl_pool_fwd", C_ref(L), ptr(self.table), ptr(self.first) if sp.fm else None,
                 ptr(self.in_cate), sp.S, ptr(self.slot_start), ptr(self.slot_end), sp.M, self.fm_pool_col,
                 ptr(self.x0), ptr(self.fm_out), ptr(self.cnt_emb), ptr(self.cnt_first), ptr(self.err), s)
        if (not train and self.lazy and not sp.M and self.since_flush == 0 and type(self) is CTREngine
                and getattr(self, "planes_step", -1) == self.steps):
            # predict on a flushed table whose planes are current (flush(planes=True) at this
            # step): the plain lookup of the dense layout (dl_embed_fwd_slots / dl_embed_fwd),
            # its deep rows read by the first tower layer itself where it can (fused_gather_l0)
            fused = self.fused_gather_l0()
            if fused and self.fused_gather_tab(B):
                fused = "tab"
            self.plane_lookup(B, x0, s, deep=not fused, gtab=self.gtab if fused == "tab" else None)
        elif not train and self.lazy and not sp.M and self.since_flush == 0 and type(self) is CTREngine:
            # predict on a flushed table (every record caught up to the current step): the plain
            # lookup, each reference reading its record's first line (dl_embed_fwd_rec_flat)
            if self.n_rep:   # the replicated FM cont-field rows, compact
                self._c("rec_gather", "dl_rec_gather", C_ref(L), ptr(self.rec), self.rec_ld, self.rec_flags, self.n_rep,
                        ptr(self.idx_uniq), None, 0, 1, ptr(self.hist), self.hist_len, ptr(self.opt), 0,
                        ptr(self.rows_u), ptr(self.rows_u1), None, s)
            self._c("embed_fwd", "dl_embed_fwd_rec_flat", C_ref(L), ptr(self.rec), self.rec_ld, self.rec_flags,
                    ptr(self.rows_u), ptr(self.rows_u1) if sp.fm else None, ptr(self.in_cate), ptr(self.in_cont),
                    ptr(self.in_vec), ptr(self.opt), ptr(x0), ptr(self.fm_out), ptr(self.fm_sum), ptr(self.err), s)
        elif self.fwd_rec:
            if self.n_rep:   # the replicated FM cont-field rows, caught up, compact
                self._c("rec_gather", "dl_rec_gather", C_ref(L), ptr(self.rec), self.rec_ld, self.rec_flags, self.n_rep,
                        ptr(self.idx_uniq), None, 0, 1, ptr(self.hist), self.hist_len, ptr(self.opt),
                        1 if train else 0, ptr(self.rows_u), ptr(self.rows_u1), None, s)
            self._c("embed_fwd", "dl_embed_fwd_rec", C_ref(L), ptr(self.rec), self.rec_ld, self.rec_flags,
                    ptr(self.rows_u), ptr(self.rows_u1) if sp.fm else None, ptr(self.in_cate), ptr(self.in_cont),
                    ptr(self.in_vec), ptr(self.hist), self.hist_len, ptr(self.opt), 1 if train else 0,
                    ptr(x0), ptr(self.fm_out), ptr(self.fm_sum), ptr(self.err), s)
        elif self.fwd_scatter:
            # rows of the batch (index built by _pre), caught up to the step being taken and
            # scattered to the references reading them; then the FM sums per sample
            self._c("rec_gather", "dl_rec_gather_scatter", C_ref(L), ptr(self.rec), self.rec_ld, self.rec_flags,
                    self.n_rep, ptr(self.idx_uniq), ptr(self.idx_n), B * self.n_slot, ptr(self.idx_off),
                    ptr(self.idx_refs), ptr(self.hist), self.hist_len, ptr(self.opt), 1 if train else 0,
                    ptr(self.rows_u), ptr(self.rows_u1), ptr(self.mv_u) if (train and self.mv_u is not None) else None,
                    ptr(self.fmst), ptr(x0), ptr(self.fm_out), ptr(self.mst), ptr(self.mst1), s)
            if sp.M:
                self._c("pool_fwd", "dl_pool_fwd_staged", C_ref(L), ptr(self.mst), ptr(self.mst1), ptr(self.idx_inv),
                        ptr(self.slot_start), ptr(self.slot_end), sp.M, self.fm_pool_col, ptr(self.x0),
                        ptr(self.fm_out), ptr(self.cnt_emb), ptr(self.cnt_first), s)
            self._c("embed_fwd", "dl_embed_fwd_staged", C_ref(L), ptr(self.fmst), ptr(self.rows_u1) if sp.fm else None,
                    ptr(self.idx_inv), self.n_rep, ptr(self.in_cont), ptr(self.in_vec), ptr(x0), ptr(self.fm_out),
                    ptr(self.fm_sum), s)
        elif self.lazy:
            # rows of the batch (index built by _pre), caught up to the step being taken
            self._c("rec_gather", "dl_rec_gather", C_ref(L), ptr(self.rec), self.rec_ld, self.rec_flags, self.n_rep,
                    ptr(self.idx_uniq), ptr(self.idx_n), B * self.n_slot, 1, ptr(self.hist), self.hist_len,
                    ptr(self.opt), 1 if train else 0, ptr(self.rows_u), ptr(self.rows_u1),
                    ptr(self.mv_u) if (train and self.mv_u is not None) else None, s)
            if sp.M:
                self._c("pool_fwd", "dl_pool_fwd_indexed", C_ref(L), ptr(self.rows_u),
                        ptr(self.rows_u1) if sp.fm else None, ptr(self.idx_inv), self.n_rep, ptr(self.slot_start),
                        ptr(self.slot_end), sp.M, self.fm_pool_col, ptr(self.x0), ptr(self.fm_out), ptr(self.cnt_emb),
                        ptr(self.cnt_first), s)
            # the deep rows go to x0 through the first tower layer where it can gather them
            # (fused_gather_rows: dl_gemm_s3_nt_gather_rows writes x0's deep columns itself)
            fused = "rows" if self.fused_gather_rows() else False
            Lx = L
            if fused:
                Lx = type(L).from_buffer_copy(L)
                Lx.x0_cat_col = -1
            self._c("embed_fwd", "dl_embed_fwd_indexed", C_ref(Lx), ptr(self.rows_u),
                    ptr(self.rows_u1) if sp.fm else None, ptr(self.idx_inv), self.n_rep, ptr(self.in_cont),
                    ptr(self.in_vec), ptr(x0), ptr(self.fm_out), ptr(self.fm_sum), s)
        else:
            self._c("embed_fwd", "dl_embed_fwd", C_ref(L), ptr(self.table), ptr(self.first), ptr(self.in_cate),
                    ptr(self.in_cont), ptr(self.in_vec), ptr(x0), ptr(self.fm_out), ptr(self.fm_sum),
                    ptr(self.err), s)
        nl = len(sp.hidden)
        if self.bf:
            # bf16 tower: x0 -> bf16, ReLU layers on bf16 MFMA (fp32 accumulate), the last layer's
            # output kept fp32 for the fp32 head / wide cross logit (config C5)
            if not self.x0_direct:
                self._c("cast_x0", "dl_cast_bf16", ptr(self.x0), B, self.in_ld[0], self.in_ld[0], ptr(self.x0b),
                        self.in_ld[0], s)
            xb = self.x0b
            for l, hdim in enumerate(sp.hidden):
                last = l == nl - 1
                out = self.h[l] if last else self.hb[l]
                self._c("gemm_fwd_l%d" % l, "dl_gemm_bf16", 0, 1, B, hdim, self.in_ld[l], ptr(xb), self.in_ld[l],
                        ptr(self.WbT[l]), self.in_ld[l], ptr(out), self.h_ld[l], 0 if last else 1, 1, None, 0, 1,
                        0, s)
                if not last:
                    xb = self.hb[l]
        elif self.s3:
            x = self.x0
            for l, hdim in enumerate(sp.hidden):
                bits = (ptr(self.hbits[l]), self.hbits_ld[l]) if l < len(self.hbits) else (None, 0)
                if l == 0 and fused == "rows":
                    # the training form: rows_u through the inverse map (deep slots after the FM
                    # slots), x0's deep columns written for the weight gradient
                    off = sp.S if sp.fm else 0
                    self._c("gemm_fwd_l0", "dl_gemm_s3_nt_gather_rows", B, hdim, self.in_ld[0], ptr(x), self.in_ld[0],
                            ptr(self.rows_u), self.rows_u.shape[0], sp.E, ptr(self.idx_inv[off:]), self.n_slot,
                            self.n_rep, sp.S, sp.E, ptr(self.WTp[0]), self.in_ld[0], self.in_ld[0] * self.out_ld[0],
                            ptr(self.h[0]), self.h_ld[0], 1, *bits, s)
                elif l == 0 and fused == "tab":
                    # predict's table form: the rows' offsets staged from gtab
                    FL = self._flat_layout(B)
                    self._c("gemm_fwd_l0", "dl_gemm_s3_nt_gather_tab", B, hdim, self.in_ld[0], ptr(x), self.in_ld[0],
                            ptr(self.p_plane), FL.n_rows, self.p_plane.shape[1], ptr(self.gtab), sp.S, sp.E,
                            ptr(self.WTp[0]), self.in_ld[0], self.in_ld[0] * self.out_ld[0], ptr(self.h[0]),
                            self.h_ld[0], 1, *bits, s)
                elif l == 0 and fused:
                    FL = self._flat_layout(B)
                    self._c("gemm_fwd_l0", "dl_gemm_s3_nt_gather", B, hdim, self.in_ld[0], ptr(x), self.in_ld[0],
                            ptr(self.p_plane), FL.n_rows, self.p_plane.shape[1], ptr(self.in_cate), FL.cate_ld,
                            FL.deep_cate_offset, FL.zero_row0, sp.S, sp.E, ptr(self.WTp[0]), self.in_ld[0],
                            self.in_ld[0] * self.out_ld[0], ptr(self.h[0]), self.h_ld[0], 1, *bits, s)
                else:
                    self._c("gemm_fwd_l%d" % l, "dl_gemm_s3_nt_bits", B, hdim, self.in_ld[l], ptr(x), self.in_ld[l],
                            ptr(self.WTp[l]), self.in_ld[l], self.in_ld[l] * self.out_ld[l], ptr(self.h[l]),
                            self.h_ld[l], 1, None, 0, *bits, s)
                x = self.h[l]
        else:
            x = self.x0
            for l, hdim in enumerate(sp.hidden):
                self._c("gemm_fwd_l%d" % l, "dl_gemm_f32", 0, 0, B, hdim, self.in_ld[l], ptr(x), self.in_ld[l],
                        ptr(self.W[l]), self.out_ld[l], ptr(self.h[l]), self.h_ld[l], 1, None, 0, 1, 0, s)
                x = self.h[l]
        H = sp.hidden[-1]
        if self.wdl and self.wide_lazy:
            # the batch's wide rows caught up into the compact local table, the head on local ids
            fn, dh_last = ("dl_wdl_head_fwd_bwd_bf16", self.dhb[-1]) if self.bf else ("dl_wdl_head_fwd_bwd", self.dh[-1])
            nw = B * sp.Fw
            self._c("wide_gather", "dl_wide_rec_gather", ptr(self.wrec), self.w_rows, ptr(self.widx_uniq),
                    ptr(self.widx_n), nw, sp.Fw, H, ptr(self.hist), self.hist_len, ptr(self.opt), sp.l2,
                    1 if train else 0, ptr(self.wloc), ptr(self.wstash) if train else None,
                    ptr(self.wrep) if train else None, s)
            self._c("head", fn, B, sp.Fw, H, ptr(self.in_wide_loc), sp.Fw, ptr(self.h[-1]), self.h_ld[-1],
                    ptr(self.wloc), ptr(self.wb), sp.Fw + H + nw, ptr(self.in_label), sp.logloss_eps, 1.0 / B,
                    ptr(self.score), ptr(self.z), ptr(self.dz), ptr(dh_last), None, None,
                    ptr(self.head_slab), self.head_blocks, ptr(self.err), s)
            if train:   # the wide rows' gradient: segment sums over the wide index (no atomics)
                self._c("wide_grad", "dl_wide_seg_grad", ptr(self.dz), sp.Fw, ptr(self.widx_refs), ptr(self.widx_off),
                        ptr(self.widx_n), nw, nw, ptr(self.wgloc[sp.Fw + H:]), ptr(self.wlong), ptr(self.opt), s)
            return
        if self.wdl:
            # bf16 tower: dY of the last layer written as bf16 by the head itself (no cast pass)
            fn, dh_last = ("dl_wdl_head_fwd_bwd_bf16", self.dhb[-1]) if self.bf else ("dl_wdl_head_fwd_bwd", self.dh[-1])
            self._c("head", fn, B, sp.Fw, H, ptr(self.in_wide), self.in_wide.shape[1],
                    ptr(self.h[-1]), self.h_ld[-1], ptr(self.ww), ptr(self.wb), self.w_rows, ptr(self.in_label),
                    sp.logloss_eps, 1.0 / B, ptr(self.score), ptr(self.z), ptr(self.dz), ptr(dh_last),
                    ptr(self.wg) if train else None, ptr(self.w_touched) if train else None,
                    ptr(self.head_slab), self.head_blocks, ptr(self.err), s)
            return
        self._c("head", "dl_head_fwd_bwd", B, sp.fm_cols, H, ptr(self.fm_out), self.fm_ld, ptr(self.h[-1]),
             self.h_ld[-1], ptr(self.w_head), ptr(self.in_label), sp.logloss_eps, 1.0 / B,
             ptr(self.score), ptr(self.z), ptr(self.dz), ptr(self.dh[-1]), ptr(self.head_slab),
             self.head_blocks, s)

    def _pre(self, B):
        """The batch's validation and index build, before its step begins: the batch's
        validation word is reset, then set by dl_validate_batch for every id no index build
        checks (the dense-layout gathers' cate ids, wdl's wide ids) and by dl_index_build (the
        hand-written radix sort + segmented unique of index.hip, no host synchronisation).
        Runs on the current stream — inside the step's hipGraph (graph=True), or on the side
        stream when prefetched — so a bad batch is known before dl_step_begin opens its step."""
        s = _lib.stream_handle()
        L = self.layout
        L.batch = B
        sp = self.spec
        cate = self.in_cate if self.bwd != "sorted" else None
        wide = self.in_wide if self.wdl else None
        self._c("validate", "dl_validate_batch", C_ref(L), ptr(cate), ptr(wide), sp.Fw if wide is not None else 0,
                self.in_wide.shape[1], getattr(self, "w_rows", 0), 1, ptr(self.err), s)
        if self.bwd != "sorted":
            return
        if self.index_pair:
            WL = self.wlayout
            WL.batch = B
            self._c("index_build", "dl_index_build_pair", C_ref(L), ptr(self.in_cate), C_ref(WL), ptr(self.in_wide),
                    ptr(self.idx_ws), self.idx_ws.numel(), ptr(self.idx_keys), ptr(self.idx_refs),
                    ptr(self.idx_uniq), ptr(self.idx_off), ptr(self.idx_n), ptr(self.idx_inv), ptr(self.widx_uniq),
                    ptr(self.widx_refs), ptr(self.widx_off), ptr(self.widx_n), ptr(self.winv), ptr(self.err), s)
            call("dl_wide_local_ids", ptr(self.winv), B * sp.Fw, sp.Fw + sp.hidden[-1], ptr(self.in_wide_loc), s)
            return
        # single GPU: keys are the rows themselves (replicated rows need no owner group;
        # the record kernels recognise them by row < n_rep) — the narrowest sort range
        self._c("index_build", "dl_index_build", C_ref(L), ptr(self.in_cate), 1, 0, ptr(self.idx_ws),
                self.idx_ws.numel(), ptr(self.idx_keys), ptr(self.idx_refs), ptr(self.idx_uniq),
                ptr(self.idx_off), ptr(self.idx_n), ptr(self.idx_inv) if self.lazy else None, None,
                ptr(self.err), s)
        if getattr(self, "wide_lazy", False):
            # the wide ids' index (unique wdl_weights rows, inverse map) and the head's local ids
            WL = self.wlayout
            WL.batch = B
            Fw, H = sp.Fw, sp.hidden[-1]
            self._c("index_build_wide", "dl_index_build", C_ref(WL), ptr(self.in_wide), 1, 0, ptr(self.widx_ws),
                    self.widx_ws.numel(), ptr(self.widx_keys), ptr(self.widx_refs), ptr(self.widx_uniq),
                    ptr(self.widx_off), ptr(self.widx_n), ptr(self.winv), None, ptr(self.err), s)
            call("dl_wide_local_ids", ptr(self.winv), B * Fw, Fw + H, ptr(self.in_wide_loc), s)

    def _train(self, B, part="all"):
        """The step's launches; part "front" = through the tower's backward and dense Adam,
        "back" = the embedding backward onwards (train_step's DLAMD_PF_MID split)."""
        self._train_body(B, part)
        if part == "front":
            return
        # the step's loss into the running sum (read once per epoch: loss_sum_end)
        sp = self.spec
        width = self.head_slab.shape[1]
        coef = sp.l2 if sp.hidden_reg == "l1" else 0.5 * sp.l2
        self._c("loss_acc", "dl_loss_accumulate", ptr(self.head_slab), call_int(self.head_grid, B), width, width - 1,
                1.0 / B, ptr(self.opt), coef, ptr(self.loss_acc), ptr(self._ring), _lib.stream_handle())

    def _train_body(self, B, part="all"):
        sp = self.spec
        s = _lib.stream_handle()
        L = self.layout
        if part == "back":
            return self._train_back(B, s, L)
        # a batch whose ids failed validation (index build) poisons the step: nothing is applied
        # (dl_step_begin: the guard, the Adam step begin and the lazy tables' alpha ring entry)
        self._c("step_begin", "dl_step_begin", ptr(self.err), ptr(self.opt), sp.decay_rate, float(sp.decay_steps),
                ptr(self.hist) if self.lazy else None, self.hist_len if self.lazy else 0, s)
        self._forward(B, s, train=True)
        nl = len(sp.hidden)
        dws = self._dw_splits(B, fixed="DLAMD_DW_SPLITS" in os.environ)
        if self.bf and not self.wdl:      # the wdl head writes its bf16 dY itself
            self._c("cast_dh", "dl_cast_bf16", ptr(self.dh[-1]), B, self.h_ld[-1], self.h_ld[-1], ptr(self.dhb[-1]),
                    self.h_ld[-1], s)
        def dw(l):   # the weight gradient of layer l (split-K slabs into w_slab)
            hdim, stride = sp.hidden[l], self.in_ld[l] * self.out_ld[l]
            splits = dws[l]
            if self.bf:
                # dW = X^T dY straight from the batch-major bf16 activations and gradients
                # (transposing LDS reads inside the kernel: no X^T / dY^T copies)
                xl = self.x0b if l == 0 else self.hb[l - 1]
                self._c("gemm_dw_l%d" % l, "dl_gemm_bf16", 1, 0, self.in_ld[l], hdim, B, ptr(xl), self.in_ld[l],
                        ptr(self.dhb[l]), self.h_ld[l], ptr(self.w_slabs[l]), self.out_ld[l], 0, 3, None, 0, splits,
                        stride, s)
            elif self.s3:   # dW = X^T dY (split-K slabs over the batch)
                xin = self.x0 if l == 0 else self.h[l - 1]
                i, o = self.in_ld[l], self.out_ld[l]
                self._c("gemm_dw_l%d" % l, "dl_gemm_s3_tn", i, hdim, B, ptr(xin), i, ptr(self.dh[l]), self.h_ld[l],
                        ptr(self.w_slabs[l]), o, splits, stride, s)
            else:
                xin = self.x0 if l == 0 else self.h[l - 1]
                self._c("gemm_dw_l%d" % l, "dl_gemm_f32", 1, 0, self.in_ld[l], hdim, B, ptr(xin), self.in_ld[l],
                        ptr(self.dh[l]), self.h_ld[l], ptr(self.w_slab), self.out_ld[l], 3, None, 0, splits, stride, s)

        def dx(l):   # the input gradient of layer l (ReluGrad by the layer below; l = 0: dx0 in f32)
            if self.bf:
                if l > 0:   # dX = dY . W^T, ReluGrad by the bf16 activations, bf16 out
                    self._c("gemm_dx_l%d" % l, "dl_gemm_bf16", 0, 1, B, sp.hidden[l - 1], self.out_ld[l],
                            ptr(self.dhb[l]), self.h_ld[l], ptr(self.Wb[l]), self.out_ld[l], ptr(self.dhb[l - 1]),
                            self.h_ld[l - 1], 1, 2, ptr(self.hb[l - 1]), self.h_ld[l - 1], 1, 0, s)
                else:       # dx0 stays fp32 for the embedding backward
                    self._c("gemm_dx_l0", "dl_gemm_bf16", 0, 1, B, self.dx_cols, self.out_ld[0], ptr(self.dhb[0]),
                            self.h_ld[0], ptr(self.Wb[0]), self.out_ld[0], ptr(self.dx0), self.dx_ld, 0, 0, None, 0,
                            1, 0, s)
            elif self.s3:   # dX = dY W^T with ReluGrad
                i, o = self.in_ld[l], self.out_ld[l]
                if l > 0 and self.relu_bits:   # ReluGrad from the forward's sign bitmask
                    self._c("gemm_dx_l%d" % l, "dl_gemm_s3_nt_bits", B, sp.hidden[l - 1], o, ptr(self.dh[l]),
                            self.h_ld[l], ptr(self.Wp[l]), o, i * o, ptr(self.dh[l - 1]), self.h_ld[l - 1], 3,
                            None, 0, ptr(self.hbits[l - 1]), self.hbits_ld[l - 1], s)
                elif l > 0:
                    self._c("gemm_dx_l%d" % l, "dl_gemm_s3_nt", B, sp.hidden[l - 1], o, ptr(self.dh[l]),
                            self.h_ld[l], ptr(self.Wp[l]), o, i * o, ptr(self.dh[l - 1]), self.h_ld[l - 1], 2,
                            ptr(self.h[l - 1]), self.h_ld[l - 1], s)
                else:
                    self._c("gemm_dx_l0", "dl_gemm_s3_nt", B, self.dx_cols, o, ptr(self.dh[0]), self.h_ld[0],
                            ptr(self.Wp[0]), o, i * o, ptr(self.dx0), self.dx_ld, 0, None, 0, s)
            else:
                self._c("transpose_l%d" % l, "dl_transpose_f32", ptr(self.W[l]), self.in_ld[l], self.out_ld[l],
                        self.out_ld[l], ptr(self.Wt), self.in_ld[l], s)
                if l > 0:
                    self._c("gemm_dx_l%d" % l, "dl_gemm_f32", 0, 0, B, sp.hidden[l - 1], self.out_ld[l],
                            ptr(self.dh[l]), self.h_ld[l], ptr(self.Wt), self.in_ld[l], ptr(self.dh[l - 1]),
                            self.h_ld[l - 1], 2, ptr(self.h[l - 1]), self.h_ld[l - 1], 1, 0, s)
                else:
                    self._c("gemm_dx_l0", "dl_gemm_f32", 0, 0, B, self.dx_cols, self.out_ld[0], ptr(self.dh[0]),
                            self.h_ld[0], ptr(self.Wt), self.in_ld[0], ptr(self.dx0), self.dx_ld, 0, None, 0, 1, 0, s)

        def adam(l):
            # regulariser on every hidden weight matrix: wdl L2 (wdl.py:272-275), dnn L1 (dnn.py:88-90);
            # bias row excluded
            stride = self.in_ld[l] * self.out_ld[l]
            nsplit = _num_splits(B, dws[l], 64 if (self.bf or self.s3) else 16)
            reg = sp.hidden_reg
            l2, l2n = (sp.l2, ([self.D0] + sp.hidden)[l] * self.out_ld[l]) if reg else (0.0, 0)
            if self.s3 or self.bf:   # the update writes the GEMM operand copies of W and W^T itself
                self._c("adam_dense_l%d" % l, "dl_adam_dense_split3" if self.s3 else "dl_adam_dense_bf16", ptr(self.W[l]), ptr(self.Wm[l]), ptr(self.Wv[l]),
                        ptr(self.w_slabs[l]), nsplit, stride, self.in_ld[l], self.out_ld[l], l2, l2n,
                        1 if reg == "l1" else 0, ptr(self.opt), ptr(self.opt[8:]) if reg else None,
                        ptr(self.Wp[l] if self.s3 else self.Wb[l]), ptr(self.WTp[l] if self.s3 else self.WbT[l]), s)
                return
            self._c("adam_dense_l%d" % l, "dl_adam_dense_reg", ptr(self.W[l]), ptr(self.Wm[l]), ptr(self.Wv[l]),
                    ptr(self.w_slab), nsplit, stride, stride, l2, l2n, 1 if reg == "l1" else 0, ptr(self.opt),
                    None, ptr(self.opt[8:]) if reg else None, s)
            self._refresh_wb(l, s)

        if self._adam_fused():
            # every layer's weight and input gradients, then one launch for the dense Adams (each
            # layer's W planes are read by its dX first; nothing else reads W before the next step)
            for l in reversed(range(nl)):
                dw(l)
                dx(l)
            reg = sp.hidden_reg
            lay = (_lib.AdamLayer * nl)()
            for l in range(nl):
                stride = self.in_ld[l] * self.out_ld[l]
                l2, l2n = (sp.l2, ([self.D0] + sp.hidden)[l] * self.out_ld[l]) if reg else (0.0, 0)
                lay[l] = _lib.AdamLayer(ptr(self.W[l]), ptr(self.Wm[l]), ptr(self.Wv[l]), ptr(self.w_slabs[l]), stride,
                                        l2n, ptr(self.opt[8:]) if reg else None,
                                        ptr(self.Wp[l] if self.s3 else self.Wb[l]),
                                        ptr(self.WTp[l] if self.s3 else self.WbT[l]),
                                        _num_splits(B, dws[l], 64), self.in_ld[l], self.out_ld[l],
                                        1 if reg == "l1" else 0, l2, 0)
            self._adam_lay = lay   # kept alive: a captured graph's kernel arguments were copied at launch
            self._c("adam_dense", "dl_adam_dense_layers", nl, C_ref(lay), 3 if self.s3 else 1, ptr(self.opt), s)
        else:
            for l in reversed(range(nl)):
                dw(l)
                dx(l)
                adam(l)
        if part == "all":
            self._train_back(B, s, L)

    def _adam_fused(self):
        """The tower's dense Adams as one launch (dl_adam_dense_layers) after the backward's GEMMs
        (DLAMD_ADAM_FUSED=0: one launch per layer, after its input gradient)."""
        return ((self.s3 or self.bf) and len(self.spec.hidden) <= 4 and type(self) is CTREngine
                and os.environ.get("DLAMD_ADAM_FUSED", "1") != "0")

    def _train_back(self, B, s, L):
        sp = self.spec
        # embedding backward (uses pre-update table and head weights)
        bwd_blocks = call_int("dl_embed_bwd_grid", C_ref(L))
        if self.lazy:
            self._embed_bwd_lazy(B, L, s)
        elif self.bwd == "sorted":
            self._c("embed_bwd", "dl_embed_bwd_sorted", C_ref(L), ptr(self.table), None, ptr(self.idx_uniq),
                    ptr(self.idx_off), ptr(self.idx_n), ptr(self.idx_refs), 1, B * self.n_slot, ptr(self.dz),
                    ptr(self.w_head), ptr(self.fm_sum), ptr(self.dx0), ptr(self.tg), ptr(self.fmg),
                    ptr(self.touched), 0, None, s)
            self._c("cont_bwd", "dl_embed_cont_bwd", C_ref(L), ptr(self.table), ptr(self._cont()), ptr(self.dz),
                    ptr(self.w_head), ptr(self.fm_sum), ptr(self.cont_slab), self.bwd_blocks, s)
        else:
            self._c("embed_bwd", "dl_embed_bwd", C_ref(L), ptr(self.table), ptr(self.in_cate), ptr(self._cont()),
                    ptr(self.dz), ptr(self.w_head), ptr(self.fm_sum), ptr(self.dx0), ptr(self.tg), ptr(self.fmg),
                    ptr(self.touched), ptr(self.cont_slab), self.bwd_blocks, s)
        if not self.lazy:
            self._c("cont_reduce", "dl_embed_cont_reduce", C_ref(L), ptr(self.cont_slab), bwd_blocks, ptr(self.tg),
                    ptr(self.fmg), ptr(self.touched), s)
        if sp.M and not self.lazy:
            self._c("pool_bwd", "dl_pool_bwd", C_ref(L), ptr(self.in_cate), sp.S, ptr(self.slot_start), ptr(self.slot_end),
                 sp.M, self.fm_pool_col, ptr(self.x0), ptr(self.fm_sum), ptr(self.dz), ptr(self.w_head), ptr(self.dx0),
                 sp.S * sp.E, ptr(self.cnt_emb), ptr(self.cnt_first), ptr(self.tg), ptr(self.fmg),
                 ptr(self.touched), s)
        H = sp.hidden[-1]
        hb = call_int(self.head_grid, B)
        if self.wdl and self.wide_lazy:
            # wdl_weights, lazy: the deep-output rows' batch sums folded into the local gradient,
            # then TF1 Adam (L2 on every row, wdl.py:270-271) on the batch's unique wide rows and
            # the deep-output rows only; the untouched rows' L2 steps are replayed when read
            self._c("wdl_fold", "dl_slab_fold_rows", ptr(self.head_slab), hb, H + 2, 0, H, ptr(self.wgloc), sp.Fw,
                    None, s)
            self._c("adam_bias", "dl_adam_dense", ptr(self.wb), ptr(self.wbm), ptr(self.wbv),
                    ptr(self.head_slab[:, H:]), hb, H + 2, 1, 0.0, 0, ptr(self.opt), None, None, s)
            self._c("adam_wide", "dl_wide_rec_update", ptr(self.wrec), ptr(self.widx_n), B * sp.Fw, ptr(self.wstash),
                    ptr(self.wgloc), sp.Fw, H, sp.l2, ptr(self.hist), self.hist_len, ptr(self.opt), ptr(self.wdmark),
                    ptr(self.wsq_part), ptr(self.wrep), ptr(self.wacc), s)
            return
        if self.wdl:
            # wdl_weights: dense Adam with L2 on every row (wdl.py:270-271); the deep-output
            # rows get their batch sums folded in from the head slab first
            self._c("wdl_fold", "dl_slab_fold_rows", ptr(self.head_slab), hb, H + 2, 0, H, ptr(self.wg), sp.Fw,
                    ptr(self.w_touched), s)
            self._c("adam_bias", "dl_adam_dense", ptr(self.wb), ptr(self.wbm), ptr(self.wbv),
                    ptr(self.head_slab[:, H:]), hb, H + 2, 1, 0.0, 0, ptr(self.opt), None, None, s)
            self._c("adam_wide", "dl_adam_rows", ptr(self.ww), ptr(self.wm), ptr(self.wv), ptr(self.wg),
                    ptr(self.w_touched), self.ww.shape[0], 1, sp.l2, 1 | _lib.ROWS_GRAD_FIXED, ptr(self.opt),
                    ptr(self.opt[8:]), s)
            if self.lazy:
                return
            self._c("adam_table", "dl_adam_rows", ptr(self.table), ptr(self.tm), ptr(self.tv), ptr(self.tg),
                    ptr(self.touched), self.table.shape[0], sp.E, 0.0, 1 | self.rows_sparse, ptr(self.opt), None, s)
            return
        # head Adam: L2 on the output weights only (deepfm_pipeline.py:183 / dnn_pipeline.py:131)
        self._c("adam_head", "dl_adam_dense", ptr(self.w_head), ptr(self.hm), ptr(self.hv), ptr(self.head_slab),
                hb, sp.fm_cols + H + 2, self.head_n, sp.l2 if sp.head_l2 else 0.0,
                self.head_n - 1 if sp.head_l2 else 0, ptr(self.opt), ptr(self.w_head_prev), ptr(self.opt[8:]), s)
        if self.lazy:
            return
        if sp.fm:
            self._c("adam_table", "dl_adam_rows", ptr(self.table), ptr(self.tm), ptr(self.tv), ptr(self.tg),
                    ptr(self.touched), self.table.shape[0], sp.E, 0.0, self.rows_sparse, ptr(self.opt), None, s)
            self._c("adam_first", "dl_adam_rows", ptr(self.first), ptr(self.fmm), ptr(self.fmv), ptr(self.fmg),
                    ptr(self.touched), self.first.shape[0], 1, 0.0, 1 | self.rows_sparse, ptr(self.opt), None, s)
        else:
            self._c("adam_table", "dl_adam_rows", ptr(self.table), ptr(self.tm), ptr(self.tv), ptr(self.tg),
                    ptr(self.touched), self.table.shape[0], sp.E, 0.0, 1 | self.rows_sparse, ptr(self.opt), None, s)

    # per-batch buffers: inputs and the batch index.  With prefetching they are double
    # buffered — the next batch is staged and indexed into the other set on a side stream
    # while the current step runs.
    SLOT_ATTRS = ("in_label", "in_cont", "in_vec", "in_cate", "in_wide", "idx_ws", "idx_keys", "idx_refs",
                  "idx_uniq", "idx_off", "idx_n", "idx_inv", "err", "widx_ws", "widx_keys", "widx_refs", "widx_uniq",
                  "widx_off", "widx_n", "winv", "in_wide_loc")

    def _side_stream(self):
        if getattr(self, "side", None) is None:
            # high priority: a hardware queue of its own (a default-priority stream can share
            # the compute stream's queue, which serialises the two)
            self.side = torch.cuda.Stream(priority=int(os.environ.get("DLAMD_SIDE_PRIORITY", "-1")))
        return self.side

    def _use_slot(self, k):
        for n, t in self._slots[k].items():
            setattr(self, n, t)
        self._cur = k

    def _enable_slots(self):
        if getattr(self, "_slots", None) is not None:
            return
        a = {n: getattr(self, n) for n in self.SLOT_ATTRS if getattr(self, n, None) is not None}
        depth = max(1, getattr(self, "pf_depth", 1))
        self._slots = [a] + [{n: torch.zeros_like(t) for n, t in a.items()} for _ in range(depth)]
        self._cur = 0
        self._slot_free = [None] * len(self._slots)   # event: the compute stream is done with a set
        self._pfq = []                    # pending prefetches, oldest first: (set, B, ready event, batch)
        self._pf = None                   # the oldest pending prefetch (_pfq[0])

    def prefetch(self, batch, graph=False, after=None):
        """Stage `batch` and build its index into an idle buffer set on the side stream;
        train_step(batch) then starts from it.  Up to pf_depth batches may be pending (buffer
        sets: pf_depth + 1), consumed in order.  graph=True replays the index build as a
        captured hipGraph (one per buffer set and batch size).  after: an event on the compute
        stream recorded after every earlier step; the side stream starts from it (instead of
        from the moment the chosen buffer set is free)."""
        self._enable_slots()
        if any(p[3] is batch for p in self._pfq) or len(self._pfq) >= len(self._slots) - 1:
            return
        cur = self._cur
        used = {cur} | {p[0] for p in self._pfq}
        k = next(i for i in range(len(self._slots)) if i not in used)
        side = self._side_stream()
        if after is not None:
            side.wait_event(after)
        elif self._slot_free[k] is not None:
            side.wait_event(self._slot_free[k])
        else:
            side.wait_stream(torch.cuda.current_stream())
        self._use_slot(k)
        try:
            with torch.cuda.stream(side):
                B = self.stage(batch)
                if graph:
                    key = (k, B, "pre")
                    g = self.graphs.get(key)
                    if g is None:
                        g = self.graphs[key] = self._capture(B, pre_only=True)
                    g.replay()
                else:
                    self._pre(B)
                ev = torch.cuda.Event()
                ev.record(side)
        finally:
            self._use_slot(cur)
        self._pfq.append((k, B, ev, batch))
        self._pf = self._pfq[0]

    def _begin(self, batch):
        """Buffers of this step's batch: the prefetched set if `batch` is the oldest one
        prefetched, else (every pending prefetch dropped once it lands) staged and indexed now
        on the compute stream."""
        q = getattr(self, "_pfq", None) or []
        if q and batch is not None and batch is q[0][3]:
            k, B, ev, _ = q.pop(0)
            self._pf = q[0] if q else None
            self._use_slot(k)
            torch.cuda.current_stream().wait_event(ev)
            return B, True
        for p in q:      # other batches came: drop the prefetches (after they land)
            torch.cuda.current_stream().wait_event(p[2])
        if q:
            q.clear()
            self._pf = None
        return (self.stage(batch) if batch is not None else self.B), False

    def _step_mark(self, end):
        """bench.py (DLAMD_STEP_EVENTS=1): timing events on the compute stream around each step's
        launches — the step's own span, and the gap to the next step's start (waits included)."""
        ev = getattr(self, "step_events", None)
        if ev is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            ev.append((end, e))

    def _release(self):
        """Mark the current buffer set free once the compute stream's queued work is done."""
        if getattr(self, "_slots", None) is not None:
            ev = torch.cuda.Event()
            ev.record()
            self._slot_free[self._cur] = ev

    def train_step(self, batch=None, graph=False, next_batch=None):
        """One training step on `batch` (or on the already-staged slots if None).
        next_batch: prefetch it (stage + index build on the side stream) during this step."""
        B, indexed = self._begin(batch)
        if getattr(self, "p_plane", None) is not None:   # predict's planes go stale: free them
            self.p_plane = self.w1_plane = None
            self.planes_step = -1
        if self.lazy:
            # every row's lag must stay below the alpha ring (rec.hip)
            if self.since_flush >= self.hist_len - 2:
                self.flush()
            self.since_flush += 1
        if not indexed and not graph:
            self._pre(B)
        # next_batch: the batch after this one, or a list of the next ones (up to pf_depth are
        # kept in flight); prefetched before this step's graph is submitted, or after it
        # (DLAMD_PF_AFTER=1)
        ahead = [] if next_batch is None else list(next_batch) if isinstance(next_batch, (list, tuple)) else [next_batch]
        pf_after = os.environ.get("DLAMD_PF_AFTER", "0") == "1"
        pf_graph = graph and os.environ.get("DLAMD_PF_EAGER", "0") != "1"
        # DLAMD_PF_MID=1: the step in two launches, the prefetch's staging and index build
        # released between them — beside the embedding backward, not the tower GEMMs
        pf_mid = bool(ahead) and not pf_after and os.environ.get("DLAMD_PF_MID", "0") == "1"
        if pf_mid:
            self._step_mark(0)
            for part in ("front", "back"):
                if graph:
                    key = (getattr(self, "_cur", 0), B, not indexed, part)
                    g = self.graphs.get(key)
                    if g is None:
                        g = self.graphs[key] = self._capture(B, with_pre=not indexed, part=part)
                    g.replay()
                else:
                    self._train(B, part)
                if part == "front":
                    mid = torch.cuda.Event()
                    mid.record()
                    for nb in ahead:
                        self.prefetch(nb, graph=pf_graph, after=mid)
            self._step_mark(1)
            self._release()
            self._queue_status()
            self.steps += 1
            self.last_batch = B
            return B
        if not pf_after:
            for nb in ahead:
                self.prefetch(nb, graph=pf_graph)
        self._step_mark(0)
        if graph:
            # one graph per (buffer set, batch size, index built inside or prefetched)
            key = (getattr(self, "_cur", 0), B, not indexed)
            g = self.graphs.get(key)
            if g is None:
                g = self.graphs[key] = self._capture(B, with_pre=not indexed)
            g.replay()
        else:
            self._train(B)
        self._step_mark(1)
        self._release()
        if pf_after:
            for nb in ahead:
                self.prefetch(nb, graph=pf_graph)
        self._queue_status()
        self.steps += 1
        self.last_batch = B
        return B

    def _embed_bwd_lazy(self, B, L, s):
        """The lazy-record embedding backward on stream s: every unique row's ordered
        segment sum and TF1 Adam step (dl_rec_bwd_adam), then the FM cont-field rows."""
        sp = self.spec
        bwd_blocks = call_int("dl_embed_bwd_grid", C_ref(L))
        E, R = sp.E, self.n_rep
        self._c("embed_bwd", "dl_rec_bwd_adam", C_ref(L), ptr(self.rec), self.rec_ld, self.rec_flags, R,
                ptr(self.rows_u), ptr(self.rows_u1), ptr(self.mv_u), ptr(self.idx_uniq), ptr(self.idx_off),
                ptr(self.idx_n), ptr(self.idx_refs), 1, B * self.n_slot, ptr(self.dz), ptr(self.w_head),
                ptr(self.fm_sum), ptr(self.dx0), ptr(self.g_rep), ptr(self.g1_rep), ptr(self.hist),
                self.hist_len, ptr(self.opt), C_ref(self.pool_desc) if sp.M else None, ptr(self.hot_ws),
                self.hot_ws.numel(), s)
        if R:
            # FM cont-field rows: per-block register partials (on the blocks that hold samples),
            # folded into g_rep, then the rows updated
            cb = self._cont_blocks(B, bwd_blocks)
            self._c("cont_bwd", "dl_embed_cont_bwd", C_ref(L), ptr(self.rows_u), ptr(self._cont()),
                    ptr(self.dz), ptr(self.w_head), ptr(self.fm_sum), ptr(self.cont_slab), cb, s)
            self._c("cont_reduce", "dl_embed_cont_reduce", C_ref(L), ptr(self.cont_slab), cb,
                    ptr(self.g_rep), ptr(self.g1_rep), ptr(self.rep_touched), s)
            self._c("adam_rep", "dl_rec_apply_rows", ptr(self.rec), self.rec_ld, E, self.rec_flags, sp.fm_cont_offset, R,
                    ptr(self.g_rep), ptr(self.g1_rep), ptr(self.hist), self.hist_len, ptr(self.opt), s)

    def _cont_blocks(self, B, bwd_blocks):
        """dl_embed_cont_bwd's blocks that hold samples (embed.hip cont_bwd_kernel: 16 samples a
        lane group, 64 / (E / 4) per wave, four waves): the rest would write zero partials."""
        spw = 64 // (self.spec.E // 4)
        return max(1, min(bwd_blocks, (B + 16 * spw - 1) // (16 * spw)))

    def _capture(self, B, with_pre=False, pre_only=False, part="all"):
        """Capture the step (with its index build when `with_pre`), or only the index build
        (`pre_only`: the prefetch graph), on a capture stream; replayed on the caller's.
        part: the whole step, or its front / back half (see _train)."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with capture_guard(), torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            if (with_pre and part != "back") or pre_only:
                self._pre(B)
            if not pre_only:
                self._train(B, part)
        torch.cuda.current_stream().wait_stream(s)
        return g

    def predict(self, batch, logits=False, device=False):
        """Forward only: returns sigmoid scores [B] (or the logits) as host numpy, or as a
        device tensor (a copy) with device=True.  On a flushed table (no training step since
        the last flush) the first predict writes the p / first-order planes once (a flush
        that only copies: every row is caught up) and every later one reads them."""
        if (self.lazy and not self.spec.M and self.since_flush == 0 and type(self) is CTREngine
                and getattr(self, "planes_step", -1) != self.steps and self.flat_planes):
            self.flush(planes=True)
        B, indexed = self._begin(batch)
        s = _lib.stream_handle()
        if not indexed:
            self._pre(B)
        self._forward(B, s)
        self._release()
        self.check_error()
        out = (self.z if logits else self.score)[:B]
        return out.clone() if device else out.cpu().numpy()

    def loss(self):
        """Loss of the last training step: data term + the L2 terms on the pre-update
        weights (accumulated by the Adam kernels into opt[DL_OPT_REG], int64 fixed point)."""
        sp = self.spec
        H = sp.hidden[-1]
        B = self.last_batch
        width = self.head_slab.shape[1]
        rows = call_int(self.head_grid, B)
        data = self.head_slab[:rows, width - 1].double().sum().item() / B
        if sp.hidden_reg == "l1":   # l1_regularizer: scale * sum |W| (dnn.py:88-90)
            return data + sp.l2 * _lib.reg_sum(self.opt)
        reg = _lib.reg_sum(self.opt)
        if getattr(self, "wide_lazy", False):
            # the wide rows the step left untouched: their L2 term from a flush (wide.hip); the
            # touched rows' from the update's block partials — only the blocks this batch size
            # launched (a smaller last batch leaves an earlier batch's partials beyond them)
            self._wide_flush()
            nparts = int(_lib.lib().dl_wide_update_blocks(B * sp.Fw, H))
            reg += _lib.reg_sum(self.wsq) + float(self.wsq_part[:nparts].double().sum().item())
        return data + sp.l2 * 0.5 * reg

    def loss_sum_begin(self):
        """Start a running loss sum over the following training steps (the load-style fit's
        epoch loss, wdl.py:305-313): no host read per step — each step's graph adds its data and
        regulariser terms on the device (dl_loss_accumulate), and with lazy wide records their
        L2 term arrives as the records are applied (the wide table is flushed first, so every
        replayed step from here on belongs to the sum)."""
        if getattr(self, "wide_lazy", False):
            self._wide_flush()
            self.wacc.zero_()
        self.loss_acc.zero_()

    def loss_sum_end(self):
        """(sum of the per-step losses since loss_sum_begin, steps): every wide record is caught
        up first, which adds the L2 terms of the steps it left untouched."""
        sp = self.spec
        acc = self.loss_acc.tolist()
        total = acc[0] + acc[1]
        if getattr(self, "wide_lazy", False):
            self._wide_flush()
            total = (self.loss_acc[0] + self.loss_acc[1] + 0.5 * sp.l2 * self.wacc.sum()).item()
        return float(total), int(round(acc[2]))

    # ------------------------------------------------------------------ errors
    def _queue_status(self):
        """After each step: an asynchronous read-back of the status word into pinned host
        memory.  Completed read-backs are checked at the next steps without waiting; at most
        two may be outstanding, so a bad batch raises within two train_step calls (TF raises
        in the failing sess.run; here the failing step itself has applied nothing)."""
        if self._ring is not None:
            return self._ring_status()
        every = int(os.environ.get("DLAMD_STATUS_EVERY", "1"))   # A/B: read back every N steps
        if every > 1 and self.steps % every:
            return
        if self._status_host is None:
            self._status_host = torch.zeros(4, dtype=torch.int32, pin_memory=True)
        k = self.steps % 4
        self._status_host[k:k + 1].copy_(self.opt.view(torch.int32)[_lib.OPT_STATUS:_lib.OPT_STATUS + 1],
                                         non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._status_q.append((k, ev))
        while self._status_q:
            k0, e0 = self._status_q[0]
            if len(self._status_q) > 2:
                t0 = time.perf_counter()
                e0.synchronize()
                self.host_wait += time.perf_counter() - t0   # bench.py: host time spent ahead of the GPU
            elif not e0.query():
                break
            self._status_q.pop(0)
            if int(self._status_host[k0]) != 0:
                self._status_q.clear()
                self.check_error()

    def _ring_status(self):
        """_queue_status from the status ring the step's last kernel writes (slot k & 3: the
        step sequence k and its status word): reports already written are checked without
        waiting; with more than two steps outstanding the oldest is waited for."""
        r = self._ring_np
        if self._ring_sent is None:   # first step: the device's sequence (this read waits for it)
            self._ring_sent = int(self.opt.view(torch.int32)[_lib.OPT_SEQ].item())
            self._ring_checked = self._ring_sent - 1
        else:
            self._ring_sent += 1
        while self._ring_checked < self._ring_sent:
            k = self._ring_checked + 1
            j = 2 * (k & 3)
            if int(r[j]) != k:
                if self._ring_sent - self._ring_checked <= 2:
                    break
                t0 = time.perf_counter()
                spins = 0
                while int(r[j]) != k:
                    spins += 1
                    if spins > 1000:   # past ~1 ms: yield the core instead of spinning on it
                        time.sleep(2e-5)
                    if time.perf_counter() - t0 > 10.0:   # the sequence went out of step: resynchronise
                        torch.cuda.synchronize()
                        if int(r[j]) != k:
                            self._ring_sent = None
                            self.check_error()
                            return
                self.host_wait += time.perf_counter() - t0   # bench.py: host time spent ahead of the GPU
            self._ring_checked = k
            if int(r[j + 1]) != 0:
                self.check_error()

    def set_opt(self, values):
        """Restore the optimizer block (a checkpoint's opt array) mid-process.  The step sequence
        of the status ring (opt[DL_OPT_SEQ]) belongs to this process's timeline, not the
        checkpoint's: the device's current value is kept, and the host re-reads it at the next
        step (otherwise the ring numbers the host expects would never arrive)."""
        v = torch.as_tensor(values, dtype=torch.float32).to(self.dev).clone()
        v[_lib.OPT_SEQ] = self.opt[_lib.OPT_SEQ]
        self.opt.copy_(v)
        if self._ring is not None:
            self._ring_sent = None

    def _error_words(self):
        words = [self.err]
        for sl in (getattr(self, "_slots", None) or []):
            if sl.get("err") is not None and sl["err"] is not self.err:
                words.append(sl["err"])
        return words

    def check_error(self):
        """Raise (and clear) a pending device error: out-of-range ids of any batch buffer set
        or the optimizer's status word."""
        st = self.opt.view(torch.int32)[_lib.OPT_STATUS:_lib.OPT_STATUS + 1]
        status = int(st.item())
        # the current buffer set's validation word: a batch validated whose step has not begun
        # (predict); a trained batch's word is consumed by its step (dl_step_begin -> status),
        # and every batch's own validation resets its word (no other set's word is touched:
        # a prefetched bad batch must still be skipped by its own step)
        bad = int(self.err[0].item()) != 0 and not status
        if not status and not bad:
            return
        bad_step, n_bad = (int(x) for x in self.opt[_lib.OPT_BAD_STEP:_lib.OPT_BAD_COUNT + 1].tolist())
        if bad:
            self.err.zero_()
        self.opt[_lib.OPT_STATUS:_lib.OPT_BAD_COUNT + 1].zero_()   # status, skip, bad step, count
        self._status_q.clear()
        if status & _lib.STATUS_LAG:
            raise _lib.DLError("internal: a row record lagged past the alpha ring (flush schedule)")
        if status & _lib.STATUS_INDEX:
            raise _lib.DLError("internal: batch index entry out of range (corrupt index)")
        if not status:   # a validated batch whose step has not begun yet (predict, or queued)
            raise _lib.DLError("InvalidArgumentError: categorical id out of range [0, %d) in the current "
                               "batch — no update applied" % self.N)
        raise _lib.DLError("InvalidArgumentError: categorical id out of range [0, %d) — %d batch(es) skipped "
                           "with no update, the last at global_step %d; the batches around them applied "
                           "normally" % (self.N, n_bad, bad_step))


def default_adam(spec):
    """Table Adam used by the drop-in model classes: row records with lazy-exact
    catch-up (bit-identical to the dense sweep, rec.hip) wherever supported."""
    return "lazy"


def _s3_dw_splits(M, N, B, base, cus=256):
    """Split-K slab count of one s3 weight gradient (dl_gemm_s3_tn: one 128 x 224 block per CU,
    (M / 128) x (N / 224) tiles per slab).  The blocks run in ceil(tiles x s / cus) rounds of
    ceil(B / s) batch rows (rounded to 64) each; the s <= base minimising rounds x rows, the
    largest on ties.  C2's layers (8 tiles) keep 32; C3's layer 0 (M = 528: 10 tiles) takes 25
    — one round of 250 blocks instead of two rounds for 320."""
    tiles = -(-M // 128) * -(-N // 224)

    def cost(s):
        return -(-tiles * s // cus) * (-(-(-(-B // s)) // 64) * 64)
    return min(range(base, 0, -1), key=cost)


@contextlib.contextmanager
def capture_guard():
    """No Python garbage collection while a hipGraph is being captured: a collection that
    frees an unreachable object holding a HIP resource (a torch.cuda.Event of an engine a
    caller dropped) would call hipEventDestroy inside the capture, which HIP refuses (the
    process aborts).  Garbage is collected before the capture instead."""
    enabled = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        yield
    finally:
        if enabled:
            gc.enable()


def _bf16_dw_splits(M, B, base, cus=256):
    """Split-K slab count of one bf16 weight gradient.  With whole 32-row batch steps
    (B % 32 == 0) dl_gemm_bf16 runs the LDS-DMA ring kernel: one 144 x 400 block per CU,
    ceil(M / 144) tiles per slab; the s <= base minimising rounds x rows per block, the largest
    on ties (C5: M = 432 / 416 -> 3 tiles, 79 slabs of 832 rows, 237 blocks in one round).
    Otherwise the two-buffer kernel (64-row tiles, two blocks per CU) takes `base`."""
    if B % 32:
        return base
    tiles = -(-M // 144)

    def cost(s):
        return -(-tiles * s // cus) * (-(-(-(-B // s)) // 64) * 64)
    return min(range(base, 0, -1), key=cost)


def _num_splits(K, splits, align=16):
    """Split-K slabs the GEMM actually writes (K chunks rounded up to `align`: 16 for the f32
    kernel, 64 for the bf16 fast kernel)."""
    kps = -(-K // splits)
    kps = -(-kps // align) * align
    return -(-K // kps)


def call_int(name, *args):
    return getattr(_lib.lib(), name)(*args)


def C_ref(L):
    import ctypes
    return ctypes.byref(L)


def _copy_in(dst, x, dtype, dev):
    """One input array into its static device slot: a pinned host tensor of the slot's dtype is
    copied straight in, asynchronously on the current stream (no host wait); anything else goes
    through _as_dev."""
    if isinstance(x, torch.Tensor) and not x.is_cuda and x.dtype == dtype and x.is_pinned():
        dst.copy_(x.view(dst.shape), non_blocking=True)
    else:
        dst.copy_(_as_dev(x, dtype, dev).reshape(dst.shape))


def _as_dev(x, dtype, dev):
    if isinstance(x, torch.Tensor):
        return x.to(device=dev, dtype=dtype, non_blocking=True)
    return torch.from_numpy(np.ascontiguousarray(x)).to(device=dev, dtype=dtype, non_blocking=True)
