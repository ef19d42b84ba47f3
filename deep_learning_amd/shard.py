"""Row-sharded multi-GPU training (BASELINE configs C4 and C5 at N GPUs).

One process per GPU.  The embedding table (and its first-order column and TF1 Adam state) is
split by rows: row r lives on rank r % world at local row r // world (cyclic, so Zipf-hot low
ids spread over all ranks).  The rows below ``replicated`` (deepfm_pipeline's 13 cont-field
rows, hit by every sample) are replicated on every rank.  Dense parameters are replicated.
The loop this replaces is the reference's session loop, models/deepfm_pipeline.py:219-234
(and wdl.py:287-317), run at the global batch B * world.

A step is device-driven end to end, so it is one hipGraph: every exchange moves FIXED-SIZE
blocks (dl_shard_route / dl_shard_exchange, shard.hip's layout), the true row counts travel in a
header beside the data, and every decision that depends on them is taken on the device:

  prefetch (side stream, during the previous step): stage the batch; index it (sort/dedup, unique
      rows grouped by owner); route it — each owner's unique rows into a block of `cap` slots,
      the inverse map remapped to slots, a header per block {count, flags, rank, step}
  1. request exchange (ids + headers, one RCCL group)
  2. dl_shard_step_begin: from every rank's header, the same decision on every rank — a bad id
     anywhere skips the step everywhere; an overflowing block (more unique rows for an owner
     than `cap`), an internal fault or ranks at different steps poison it (and the next ones)
  3. owners gather the requested rows (caught up to step t-1) into their answer blocks; the
     owner sort that groups this step's arrivals by row runs on a branch meanwhile
  4. answer exchange (rows + first-order weights, one group); the forward reads them through
     the remapped inverse map
  5. MLP + head, the input-gradient chain, per-unique-row gradients written into slots
  6. gradient exchange to the owners (one group) on a branch, beside the weight gradients;
     the flat all-reduce of the dense + replicated gradients on a second communicator and
     stream, beside it
  7. TF1 Adam: dense + replicated parameters identically everywhere; owners apply each row's
     arrivals (at most one per sender, summed in rank order) once — lazy-exact row records
  8. the step's loss and status into the pinned status ring (no host read in the step)

The host waits only for the status report of the step submitted `lag` calls earlier.  A report
naming an overflow (every rank sees the same one) makes every rank synchronise, grow its blocks
and replay the skipped steps in order — the result is the same as if nothing had overflowed.

Collectives: backend "nccl" uses two RCCL communicators of our own (comm.cpp: one for the block
exchanges, one for the all-reduce), launched on our streams inside the step's graph; the torch
process group only ships their ids.  Backend "gloo" (CPU tests, several ranks sharing one GPU)
stages the same fixed blocks through host memory, eagerly.
"""
import ctypes
import os
import time

import numpy as np

import torch
import torch.distributed as dist

from . import _lib
from ._lib import call, ptr
from .engine import CTREngine, C_ref, _num_splits, _ru, call_int, capture_guard

_STICKY = _lib.STATUS_LAG | _lib.STATUS_INDEX | _lib.STATUS_OVERFLOW | _lib.STATUS_DESYNC


class Exchange:
    """The sharded step's collectives.  `blocks` moves whole blocks of 2W - 1-block arrays
    (dl_shard_exchange's layout); `all_reduce` sums in place.  RCCL: our own communicators on
    the caller's stream (capturable); gloo: staged through host memory."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = dist.get_backend(group)
        self.staged = self.backend != "nccl"
        self._comm = self._comm_ar = None

    def _comms(self):
        """Two RCCL communicators (the block exchanges; the all-reduce, so it can run beside
        them on its own stream), created collectively on first use; their ids travel over the
        torch process group."""
        if self._comm is None:
            nb = int(_lib.lib().dl_comm_unique_id_bytes())
            ids = torch.zeros(2 * nb, dtype=torch.uint8)
            if self.rank == 0:
                for k in range(2):
                    call("dl_comm_get_unique_id", ctypes.c_void_p(ids.data_ptr() + k * nb))
            d = ids.cuda()
            src = 0 if self.group is None else dist.get_global_rank(self.group, 0)
            dist.broadcast(d, src, group=self.group)
            ids = d.cpu()
            comms = []
            for k in range(2):
                c = ctypes.c_void_p()
                call("dl_comm_init", ctypes.c_void_p(ids.data_ptr() + k * nb), self.world, self.rank, ctypes.byref(c))
                comms.append(c)
            self._comm, self._comm_ar = comms
        return self._comm, self._comm_ar

    def block(self, p):
        """This rank's block of its traffic with peer p (p == rank: its own, never moved)."""
        return p if p == self.rank else self.world + p - (1 if p > self.rank else 0)

    def blocks(self, arrays, direction, stream=None):
        """arrays: [2W - 1, per-block elements] tensors.  direction 0 (to the owners): this rank's
        block for peer p goes to p, p's arrives in block p; 1 (back): block p goes to p, p's
        arrives in this rank's block for p."""
        W, me = self.world, self.rank
        if W == 1 or not arrays:
            return
        if not self.staged:
            comm, _ = self._comms()
            n = len(arrays)
            bases = (ctypes.c_void_p * n)(*[a.data_ptr() for a in arrays])
            bb = (ctypes.c_int64 * n)(*[a[0].numel() * a.element_size() for a in arrays])
            call("dl_shard_exchange", comm, n, ctypes.cast(bases, ctypes.c_void_p), ctypes.cast(bb, ctypes.c_void_p),
                 direction, _lib.stream_handle(stream))
            return
        for a in arrays:
            h = a.cpu()
            send = torch.zeros((W,) + tuple(h.shape[1:]), dtype=h.dtype)
            for p in range(W):
                if p != me:
                    send[p] = h[self.block(p) if direction == 0 else p]
            recv = torch.empty_like(send)
            dist.all_to_all_single(recv, send, group=self.group)
            for p in range(W):
                if p != me:
                    a[p if direction == 0 else self.block(p)].copy_(recv[p])

    def all_reduce(self, t, stream=None, serial=False):
        """Sum over the ranks, in place (inside the step: RCCL on `stream`; serial: on the block
        exchanges' communicator, else on the all-reduce's own)."""
        if self.world == 1:
            return t
        if self.staged:
            c = t.cpu()
            dist.all_reduce(c, group=self.group)
            t.copy_(c)
            return t
        comm, comm_ar = self._comms()
        call("dl_all_reduce_f32", comm if serial else comm_ar, ptr(t), ptr(t), t.numel(), _lib.stream_handle(stream))
        return t

    def host_sum(self, t):
        """A sum outside the step (loss read-out): the torch process group."""
        if self.world == 1:
            return t
        if self.staged and t.is_cuda:
            c = t.cpu()
            dist.all_reduce(c, group=self.group)
            t.copy_(c)
        else:
            dist.all_reduce(t, group=self.group)
        return t

    def close(self):
        """Release the RCCL communicators (after every rank's work is done)."""
        for c in (self._comm, self._comm_ar):
            if c is not None:
                torch.cuda.synchronize()
                call("dl_comm_destroy", c)
        self._comm = self._comm_ar = None


class ShardedCTREngine(CTREngine):
    """CTREngine whose embedding tables are row-sharded across the ranks of `exch`."""

    # slack of a block over an even split of the batch's references (DLAMD_SHARD_SLACK): at C4
    # (8 ranks, 3.4 M references a batch) a block holds 468 k rows against ~419 k unique rows per
    # owner for uniform ids (binomial spread ~0.7 k), fewer under Zipf; an overflow is replayed
    SLACK = 0.10

    def __init__(self, spec, max_batch, exch, device="cuda", seed=2019, adam="dense", hist_len=4096,
                 owner_update=None, slack=None, lag=2):
        if spec.model not in ("deepfm_pipeline", "dnn_pipeline", "wdl"):
            raise ValueError("sharded path supports deepfm_pipeline / dnn_pipeline / wdl")
        # the status ring holds 4 reports (slot k & 3) and the host reads report k only after
        # k + lag was submitted: lag <= 3, or report k + 4 overwrites k before it is read
        if not 0 <= int(lag) <= 3:
            raise ValueError("lag must be 0..3 (the status ring holds 4 reports), got %r" % (lag,))
        self.exch = exch
        self.world, self.rank = exch.world, exch.rank
        N = spec.n_rows
        self.rep = spec.C if spec.model == "deepfm_pipeline" else 0
        local_rows = -(-N // self.world)
        super().__init__(spec, max_batch, device=device, seed=seed, init="none", bwd="sorted",
                         table_rows=local_rows, adam=adam, hist_len=hist_len)
        z = lambda *sh, dt=torch.float32: torch.zeros(*sh, dtype=dt, device=self.dev)
        E, W = spec.E, self.world
        self.local_rows = local_rows
        self.side = None
        self.host_marks = [] if os.environ.get("DLAMD_HOST_TIMING") else None
        self.slack = float(os.environ.get("DLAMD_SHARD_SLACK", self.SLACK)) if slack is None else float(slack)
        self.lag = int(lag)
        # DLAMD_SHARD_AR_SERIAL (default 1): the flat all-reduce on the exchange communicator and
        # stream, after the gradient exchange — every RCCL kernel of the step on one communicator
        # in one order; 0: on a second communicator and stream, beside the gradient exchange
        # (why serial is the default)
        self.ar_serial = os.environ.get("DLAMD_SHARD_AR_SERIAL", "1") != "0"
        # the host's wait for a step's status report: past this many seconds the process exits
        # non-zero (a peer stuck in a collective cannot keep the job hanging silently)
        self.guard_s = float(os.environ.get("DLAMD_SHARD_GUARD_S", "60"))
        if self.lazy:
            # owners group a step's arrivals by row with a sort (dl_sort_unique + apply_segments) or
            # per-row arrival chains (dl_rec_chain_link + apply_chain); bit-identical records
            self.owner_update = owner_update or os.environ.get("DLAMD_OWNER_UPDATE", "sort")
            if self.owner_update not in ("sort", "chain"):
                raise ValueError("owner_update must be 'sort' or 'chain'")
            self.own_bits = max(1, int(self.rows_pad - 1).bit_length())
            if self.owner_update == "chain":
                self.own_head = torch.full((self.rows_pad,), -1, dtype=torch.int32, device=self.dev)
        # the single-GPU engine's batch buffers this engine replaces (blocks, slots, its own stash)
        self.mv_u = self.hot_ws = self.idx_inv = None
        R = max(self.rep, 1)
        rp = _ru(R, 16)
        self.rep_cap = rp if self.rep else 0
        self.rep_t, self.rep_m, self.rep_v = z(rp, E), z(rp, E), z(rp, E)
        self.rep_f, self.rep_fm, self.rep_fv = z(rp), z(rp), z(rp)
        self.rep_all = torch.ones(rp, dtype=torch.uint8, device=self.dev)    # every replicated row steps
        self.rep_scratch = z(rp, dt=torch.uint8)                               # touched flags nobody reads
        self.rep_iota = torch.arange(rp, dtype=torch.int32, device=self.dev)
        n = self.n_refs
        self.inv = z(n, dt=torch.int32)
        self.owner_counts = z(W + 1, dt=torch.int32)
        self.upos = z(n, dt=torch.int32)
        # flat dense-gradient buffer (one all-reduce): every layer's W_aug, the head, the replicated rows
        self.seg = []
        off = 0
        for l in range(len(spec.hidden)):
            sz = self.in_ld[l] * self.out_ld[l]
            self.seg.append(("W%d" % l, off, sz))
            off += sz
        H = spec.hidden[-1]
        self.head_w = spec.fm_cols + H + 2          # weights + bias + loss sum
        self.seg.append(("head", off, self.head_w))
        off += self.head_w
        off = _ru(off, 4)                           # the replicated rows' gradients 16-B aligned (dl_adam_rows)
        self.rep_off = off
        off += rp * E + rp
        self.flat = z(off)
        self.opt[_lib.OPT_BAD_RANKS] = 0.0
        if self.wdl:
            self._init_wide(max_batch)
        self.cap = self.wcap = 0
        self._alloc_blocks(self._cap_for(self.n_refs), self._cap_for(getattr(self, "n_wrefs", 0)))
        # the step's own streams: the gradient exchange and the owner sort (branches of the step
        # graph), the all-reduce (second communicator); the ring of per-step status reports
        self.x_stream = torch.cuda.Stream()
        self.ar_stream = torch.cuda.Stream()
        self.own_stream = torch.cuda.Stream()
        self._ring = torch.zeros(8, dtype=torch.int32, pin_memory=True)
        self._ring_np = self._ring.numpy()
        self._ring_sent = None
        self._hist_b = {}          # sequence -> batch of the steps not yet reported
        self._steps_eager = 0

    # ------------------------------------------------------------ block buffers
    def _cap_for(self, n):
        """Slots per block for n references a batch: all of them at one rank (no overflow
        possible), else an even split plus the slack, rounded to 64."""
        if n <= 0:
            return 0
        if self.world == 1:
            return n
        return min(n, _ru(int(np.ceil(n / self.world * (1.0 + self.slack))), 64))

    def _alloc_blocks(self, cap, wcap):
        """(Re)size everything whose shape follows the block capacity (first call, or growing
        after an overflow: the graphs and any prefetch are dropped with it)."""
        sp, E, W = self.spec, self.spec.E, self.world
        z = lambda *sh, dt=torch.float32: torch.zeros(*sh, dtype=dt, device=self.dev)
        nb = 2 * W - 1
        self.cap, self.wcap, self.nb = cap, wcap, nb
        rep, rc = self.rep, self.rep_cap
        # rows: [replicated cont rows | 2W - 1 blocks | replicated group], gradients likewise
        self.rows_u = z(rep + nb * cap + rc, E)
        self.rows_u1 = z(rep + nb * cap + rc)
        self.g_all = z(nb * cap + rc, E)
        self.g1_all = z(nb * cap + rc)
        per_batch = {"ids_all": z(nb * cap, dt=torch.int32), "hdr_all": z(nb * 4, dt=torch.int32),
                     "rep_ids": z(max(rc, 1), dt=torch.int32)}
        if self.wdl:
            Fw, H = sp.Fw, sp.hidden[-1]
            self.wloc_off = Fw + H
            old = getattr(self, "wloc", None)
            self.wloc = z(_ru(Fw + H + nb * wcap, 4))
            if old is not None:   # the replicated deep-output rows carry over
                self.wloc[Fw: Fw + H].copy_(old[Fw: Fw + H])
            self.wgloc = z(Fw + H + nb * wcap, dt=torch.int64)
            per_batch.update({"wids_all": z(nb * wcap, dt=torch.int32), "whdr_all": z(nb * 4, dt=torch.int32)})
        for k, t in per_batch.items():
            setattr(self, k, t)
        if getattr(self, "_slots", None) is not None:
            for sl in self._slots:
                for k, t in per_batch.items():
                    sl[k] = torch.zeros_like(t)
            self._use_slot(self._cur)
            self._pf = None
            self._pfq = []
            self._slot_free = [None] * len(self._slots)
        if self.lazy:
            self.own_mv = z(W * cap, int(_lib.lib().dl_rec_stash_floats(E))) if self.owner_update == "sort" else None
            if self.owner_update == "chain":
                self.own_next = z(W * cap, dt=torch.int32)
            elif W > 1:
                ws = _lib.lib().dl_index_workspace_bytes(W * cap)
                self.own_ws = z(ws, dt=torch.uint8)
                self.own_keys, self.own_pos, self.own_uniq = (z(W * cap, dt=torch.int32) for _ in range(3))
                self.own_off, self.own_n = z(W * cap + 1, dt=torch.int32), z(4, dt=torch.int32)
            else:   # one sender: its block is already grouped by row (sorted, unique) — no sort
                self.iota = torch.arange(cap + 1, dtype=torch.int32, device=self.dev)
        self.graphs = {}

    def _grow(self):
        """After an overflow: every block twice as large (at most every reference a batch)."""
        cap = min(self.n_refs, max(2 * self.cap, 64))
        wcap = min(getattr(self, "n_wrefs", 0), max(2 * self.wcap, 64)) if self.wdl else 0
        self._alloc_blocks(cap, wcap)

    def _init_wide(self, B):
        """wdl_weights sharded like the table (row r on rank r % world), plus the per-rank local
        wide table the cross logit reads: wloc = [unused (Fw) | deep-output rows Fw..Fw+H,
        replicated | the exchange blocks of this batch's wide rows].  The head
        (dl_wdl_head_fwd_bwd) runs unchanged on local ids and leaves each exchanged row's
        gradient in wgloc at the same slot."""
        sp = self.spec
        W = self.world
        z = lambda *sh, dt=torch.float32: torch.zeros(*sh, dtype=dt, device=self.dev)
        Fw = sp.Fw
        self.w_local = -(-self.w_rows // W)
        wl = _ru(self.w_local, 16)
        self.ww, self.wm, self.wv = z(wl), z(wl), z(wl)
        self.wg = z(wl, dt=torch.int64)
        self.w_touched = z(wl, dt=torch.uint8)
        self.wide_reg = z(2, dt=torch.int64)   # the shard's L2 sum (fixed point, DL_REG_SUM_SCALE)
        nw = B * Fw
        self.n_wrefs = nw
        self.in_wide_loc = z(B, Fw, dt=torch.int64)
        wsb = _lib.lib().dl_index_workspace_bytes(max(1, nw))
        self.widx_ws = z(wsb, dt=torch.uint8)
        self.widx_keys, self.widx_refs, self.widx_uniq = (z(nw, dt=torch.int32) for _ in range(3))
        self.widx_off = z(nw + 1, dt=torch.int32)
        self.widx_n = z(4, dt=torch.int32)
        self.winv = z(nw, dt=torch.int32)
        self.wowner_counts = z(W + 1, dt=torch.int32)
        WL = _lib.EmbLayout()
        WL.n_rows = self.w_rows
        WL.batch = B
        WL.emb_dim = sp.E
        WL.cate_fields = Fw
        WL.cate_ld = self.in_wide.shape[1]
        WL.use_fm = 0
        WL.zero_row0 = 0
        self.wlayout = WL

    # ------------------------------------------------------------ parameters
    def owned_rows(self):
        """Global rows stored locally (local row i <-> global rank + i*W)."""
        return np.arange(self.local_rows) * self.world + self.rank

    def load_params(self, P):
        """Inject reference-layout GLOBAL parameters; each rank keeps its rows."""
        sp = self.spec
        N = self.N
        rows = self.owned_rows()
        ok = rows < N
        t = np.zeros((self.rows_pad, sp.E), np.float32)
        t[: self.local_rows][ok] = P[sp.table_key][rows[ok]]
        if self.wdl:
            self._pack(torch.from_numpy(t).to(self.dev), None) if self.lazy else self.table.copy_(torch.from_numpy(t))
            for l in range(len(sp.hidden)):
                self._set_layer(l, P["deep_%d" % l], P["deep_bias_%d" % l])
            wrows = np.arange(self.w_local) * self.world + self.rank
            wok = wrows < self.w_rows
            w = np.zeros(self.ww.shape[0], np.float32)
            w[: self.w_local][wok] = np.asarray(P["wdl_weights"], np.float32)[wrows[wok], 0]
            self.ww.copy_(torch.from_numpy(w))
            self.wb.zero_()
            self.wb[:1].copy_(torch.from_numpy(np.asarray(P["wdl_bias"], np.float32).reshape(-1)))
            H = sp.hidden[-1]
            self.wloc[sp.Fw: sp.Fw + H].copy_(torch.from_numpy(np.asarray(P["wdl_weights"], np.float32)[sp.Fw: sp.Fw + H, 0]))
            torch.cuda.synchronize()
            return
        f = None
        if sp.fm:
            f = np.zeros(self.rows_pad, np.float32)
            f[: self.local_rows][ok] = P["fm_first_order_emb"][rows[ok], 0]
        if self.lazy:
            self._pack(torch.from_numpy(t).to(self.dev), torch.from_numpy(f).to(self.dev) if f is not None else None)
        else:
            self.table.copy_(torch.from_numpy(t))
            if f is not None:
                self.first.copy_(torch.from_numpy(f))
        if self.rep:
            self.rep_t[: self.rep].copy_(torch.from_numpy(np.ascontiguousarray(P["feats_emb"][: self.rep])))
            if sp.fm:
                self.rep_f[: self.rep].copy_(torch.from_numpy(np.ascontiguousarray(P["fm_first_order_emb"][: self.rep, 0])))
        for l in range(len(sp.hidden)):
            self._set_layer(l, P["deep_%d" % l], P["deep_bias_%d" % l])
        if sp.fm:
            w = np.concatenate([P["deep_fm_weight"][:, 0], P["deep_fm_bias"].reshape(-1)]).astype(np.float32)
        else:
            w = np.concatenate([P["deep_res"][:, 0], P["deep_res_bias"].reshape(-1)]).astype(np.float32)
        self.w_head.zero_()
        self.w_head[: self.head_n].copy_(torch.from_numpy(w))
        torch.cuda.synchronize()

    def init_device(self, seed):
        """Bench init: every rank draws its shard with a rank-distinct counter range."""
        sp = self.spec
        s = _lib.stream_handle()
        if self.lazy:
            self.table = torch.zeros(self.rows_pad, sp.E, device=self.dev)
            self.first = torch.zeros(self.rows_pad, device=self.dev) if sp.fm else None
        if sp.xavier_table:   # wdl.py:44-47: glorot-uniform weight_mat
            import math
            lim = math.sqrt(6.0 / (self.N + sp.E))
            call("dl_init_random", ptr(self.table), self.table.numel(), 1, -lim, 2 * lim, seed,
                 self.rank * self.table.numel() * 4, s)
        else:
            call("dl_init_random", ptr(self.table), self.table.numel(), 0, 0.0, 0.01, seed,
                 self.rank * self.table.numel() * 4, s)
        if self.wdl:   # wdl.py:241-244, the shard's rows; the deep-output rows from their owners
            import math
            call("dl_init_random", ptr(self.ww), _ru(self.ww.numel(), 4), 0, 0.0, math.sqrt(2.0 / self.w_rows),
                 seed + 3, self.rank * self.ww.numel(), s)
            self.ww[self.w_local:].zero_()
            self.wb[0] = float(np.random.default_rng(seed).standard_normal())
            self._wide_refresh(s)
        if self.first is not None:
            call("dl_init_random", ptr(self.first), _ru(self.first.numel(), 4), 1, 0.0, 1.0, seed + 1,
                 self.rank * _ru(self.first.numel(), 4), s)
        if self.lazy:
            self._pack(self.table, self.first)
            self.table = self.first = None
        if self.rep:
            call("dl_init_random", ptr(self.rep_t), self.rep_t.numel(), 0, 0.0, 0.01, seed + 7, 0, s)
            if sp.fm:
                call("dl_init_random", ptr(self.rep_f), _ru(self.rep_f.numel(), 4), 1, 0.0, 1.0, seed + 8, 0, s)
        rng = np.random.default_rng(seed)   # identical dense init on every rank
        import math
        dims = [self.D0] + sp.hidden
        for l in range(len(sp.hidden)):
            g = math.sqrt(2.0 / (dims[l] + dims[l + 1]))
            self._set_layer(l, (rng.standard_normal((dims[l], dims[l + 1])) * g).astype(np.float32),
                            (rng.standard_normal((1, dims[l + 1])) * g).astype(np.float32), ref_order=False)
        g = math.sqrt(2.0 / self.head_n)
        w = np.zeros(self.head_n, np.float32)
        w[:-1] = rng.standard_normal(self.head_n - 1) * g
        w[-1] = rng.standard_normal()
        self.w_head[: self.head_n].copy_(torch.from_numpy(w))
        torch.cuda.synchronize()

    def params(self):
        raise NotImplementedError("gather shards with gather_params()")

    def shard_state(self):
        """(global rows, table rows, first-order) of this rank's shard (host numpy)."""
        rows = self.owned_rows()
        ok = rows < self.N
        if self.lazy:
            self.flush()
            E = self.spec.E
            r = self.rec[: self.local_rows]
            t = r[:, :E].cpu().numpy()[ok]
            f = r[:, E].cpu().numpy()[ok] if self.spec.fm else None
            return rows[ok], t, f
        t = self.table[: self.local_rows].cpu().numpy()[ok]
        f = self.first[: self.local_rows].cpu().numpy()[ok] if self.first is not None else None
        return rows[ok], t, f

    def wide_state(self):
        """(global rows, wdl_weights values) of this rank's shard of wdl_weights (host numpy)."""
        rows = np.arange(self.w_local) * self.world + self.rank
        ok = rows < self.w_rows
        return rows[ok], self.ww[: self.w_local].cpu().numpy()[ok]

    @property
    def last_counts(self):
        """(unique rows this rank's batch needs from owners, replicated rows, rows it served as an
        owner) of the last step (bench.py prices the per-kernel work with them)."""
        W = self.world
        oc = self.owner_counts.tolist()
        h = self.hdr_all[: 4 * W].view(W, 4)[:, 0].tolist()
        return sum(oc[:W]), oc[W], sum(h)

    def exchange_bytes(self):
        """Bytes this rank SENDS over the interconnect per training step (its own block never
        moves; every exchange moves whole fixed-size blocks, so these are the step's sizes, not
        its counts): the requests (ids + 16-B headers), the answers (rows + first-order weights
        + wide values), the gradients back to the owners, and the flat all-reduce as a ring sends
        it (2 (W - 1) / W of the buffer)."""
        W, cap, E = self.world, self.cap, self.spec.E
        p = W - 1
        fm = 4 if self.spec.fm else 0
        out = {"requests": p * (cap * 4 + 16), "answers": p * cap * (E * 4 + fm),
               "gradients": p * cap * (E * 4 + fm)}
        if self.wdl:
            out["requests"] += p * (self.wcap * 4 + 16)
            out["answers"] += p * self.wcap * 4
            out["gradients"] += p * self.wcap * 8
        out["all_reduce"] = int(self.flat.numel() * 4 * 2 * p / W) if W > 1 else 0
        out["total"] = sum(out.values())
        out["block_slots"] = cap
        return out

    # ------------------------------------------------------------ the step's pieces
    def _mark(self, name):
        if self.host_marks is not None:
            self.host_marks.append((name, time.perf_counter()))

    def _own_layout(self):
        """The owner gather's layout: local rows (an empty slot's -1 decodes past them)."""
        L = self._layout(self.B)
        L.n_rows = self.local_rows
        return L

    # the per-batch buffers (double-buffered with prefetch): inputs, the index, the route
    SLOT_ATTRS = CTREngine.SLOT_ATTRS + ("inv", "owner_counts", "upos", "ids_all", "hdr_all", "rep_ids", "widx_ws",
                                         "widx_keys", "widx_refs", "widx_uniq", "widx_off", "widx_n", "winv",
                                         "wowner_counts", "wids_all", "whdr_all", "in_wide_loc")

    def _pre(self, B):
        """Index + route the staged batch on the current stream (the prefetch's work): the
        unique rows grouped by owner into this rank's blocks, the inverse map remapped to slots,
        the headers; for wdl the wide ids likewise and the head's local wide ids."""
        s = _lib.stream_handle()
        L = self.layout
        L.batch = B
        W = self.world
        # the batch's validation word starts clear (the index builds set it for a bad id)
        call("dl_validate_batch", C_ref(L), None, None, 0, 1, 0, 1, ptr(self.err), s)
        self._c("index_build", "dl_index_build", C_ref(L), ptr(self.in_cate), W, self.rep,
                ptr(self.idx_ws), self.idx_ws.numel(), ptr(self.idx_keys), ptr(self.idx_refs), ptr(self.idx_uniq),
                ptr(self.idx_off), ptr(self.idx_n), ptr(self.inv), ptr(self.owner_counts), ptr(self.err), s)
        n = B * self.n_slot
        self._c("route", "dl_shard_route", ptr(self.idx_uniq), ptr(self.idx_n), ptr(self.owner_counts), W, self.rank,
                self.cap, self.rep_cap, ptr(self.err), ptr(self.ids_all), ptr(self.hdr_all),
                ptr(self.rep_ids) if self.rep_cap else None, ptr(self.upos), ptr(self.inv), n, n, s)
        if self.wdl:   # the wide ids (dl_index_build range-checks them against w_rows)
            WL = self.wlayout
            WL.batch = B
            sp = self.spec
            self._c("index_build_wide", "dl_index_build", C_ref(WL), ptr(self.in_wide), W, 0,
                    ptr(self.widx_ws), self.widx_ws.numel(), ptr(self.widx_keys), ptr(self.widx_refs),
                    ptr(self.widx_uniq), ptr(self.widx_off), ptr(self.widx_n), ptr(self.winv),
                    ptr(self.wowner_counts), ptr(self.err), s)
            nw = B * sp.Fw
            self._c("route_wide", "dl_shard_route", ptr(self.widx_uniq), ptr(self.widx_n), ptr(self.wowner_counts), W,
                    self.rank, self.wcap, 0, ptr(self.err), ptr(self.wids_all), ptr(self.whdr_all), None, None,
                    ptr(self.winv), nw, 0, s)
            call("dl_wide_local_ids", ptr(self.winv), nw, self.wloc_off, ptr(self.in_wide_loc), s)

    def _requests(self, s):
        """Step 1: the requests (ids + headers) to their owners, stamped with this rank's sticky
        faults and step."""
        W, me = self.world, self.rank
        call("dl_shard_stamp", ptr(self.hdr_all), W, me, ptr(self.opt), s)
        arrs = [self.ids_all.view(self.nb, self.cap), self.hdr_all.view(self.nb, 4)]
        if self.wdl:
            arrs += [self.wids_all.view(self.nb, self.wcap), self.whdr_all.view(self.nb, 4)]
        self._c("x_requests", "exchange", lambda: self.exch.blocks(arrs, 0))

    def _c(self, label, name, *args):
        """_c of the engine; name 'exchange' runs a Python callable (a collective) timed alike."""
        if name != "exchange":
            return super()._c(label, name, *args)
        fn = args[0]
        if self.prof is None:
            return fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        self.prof.append((label, e0, e1))

    def _gather_owned(self, B, s, lag):
        """Step 3: the owner side — every requested row (blocks [0, W) of ids_all) caught up to
        step t - lag into this rank's answer blocks; the wide values likewise."""
        sp = self.spec
        E, W, rep, cap = sp.E, self.world, self.rep, self.cap
        rows, rows1 = self.rows_u[rep:], self.rows_u1[rep:]
        if self.lazy:
            stash = lag == 1 and self.own_mv is not None
            self._c("rec_gather", "dl_rec_gather", C_ref(self._own_layout()), ptr(self.rec), self.rec_ld,
                    self.rec_flags, 0, ptr(self.ids_all), None, W * cap, 1, ptr(self.hist), self.hist_len,
                    ptr(self.opt), lag, ptr(rows), ptr(rows1) if sp.fm else None, ptr(self.own_mv) if stash else None,
                    s)
        else:
            self._c("rec_gather", "dl_shard_gather", ptr(self.table), ptr(self.first), ptr(self.ids_all), W * cap, E,
                    ptr(rows), ptr(rows1) if self.first is not None else None, s)
        if self.wdl:
            self._c("wide_gather", "dl_shard_gather_scalar", ptr(self.ww), ptr(self.wids_all), W * self.wcap,
                    ptr(self.wloc[self.wloc_off:]), s)

    def _answers(self, s):
        """Step 4: the answers back to the senders (rows + first-order weights + wide values, one
        group), then the replicated rows (cont fields, and those cate ids reference) locally."""
        sp = self.spec
        E, rep, nb, cap = sp.E, self.rep, self.nb, self.cap
        arrs = [self.rows_u[rep: rep + nb * cap].view(nb, cap * E)]
        if sp.fm:
            arrs.append(self.rows_u1[rep: rep + nb * cap].view(nb, cap))
        if self.wdl:
            o = self.wloc_off
            arrs.append(self.wloc[o: o + nb * self.wcap].view(nb, self.wcap))
        self._c("x_answers", "exchange", lambda: self.exch.blocks(arrs, 1))
        if rep:
            f = self.rep_f if sp.fm else None
            call("dl_shard_gather", ptr(self.rep_t), ptr(f), ptr(self.rep_iota), rep, E, ptr(self.rows_u),
                 ptr(self.rows_u1) if sp.fm else None, s)
            o = rep + nb * cap
            call("dl_shard_gather", ptr(self.rep_t), ptr(f), ptr(self.rep_ids), self.rep_cap, E, ptr(self.rows_u[o:]),
                 ptr(self.rows_u1[o:]) if sp.fm else None, s)

    def _forward_local(self, B, s, train):
        """Step 5a: the forward on this rank's batch from the exchanged rows."""
        sp = self.spec
        L = self.layout
        L.batch = B
        self._c("embed_fwd", "dl_embed_fwd_indexed", C_ref(L), ptr(self.rows_u), ptr(self.rows_u1) if sp.fm else None,
                ptr(self.inv), self.rep, ptr(self.in_cont), ptr(self.in_vec),
                ptr(self.x0b if self.x0_direct else self.x0), ptr(self.fm_out), ptr(self.fm_sum), s)
        if self.bf and not self.x0_direct:
            self._c("cast_x0", "dl_cast_bf16", ptr(self.x0), B, self.in_ld[0], self.in_ld[0], ptr(self.x0b),
                    self.in_ld[0], s)
        self._tower_fwd(B, s)
        self._head(B, s, train)

    def _tower_fwd(self, B, s):
        """Deep tower forward from x0 (f32 / three-plane split on bf16 MFMA / bf16 tower)."""
        sp = self.spec
        nl = len(sp.hidden)
        if self.bf:
            xb = self.x0b
            for l, hdim in enumerate(sp.hidden):
                last = l == nl - 1
                out = self.h[l] if last else self.hb[l]
                self._c("gemm_fwd_l%d" % l, "dl_gemm_bf16", 0, 1, B, hdim, self.in_ld[l], ptr(xb), self.in_ld[l],
                        ptr(self.WbT[l]), self.in_ld[l], ptr(out), self.h_ld[l], 0 if last else 1, 1, None, 0, 1,
                        0, s)
                if not last:
                    xb = self.hb[l]
            return
        x = self.x0
        for l, hdim in enumerate(sp.hidden):
            if self.s3:
                bits = (ptr(self.hbits[l]), self.hbits_ld[l]) if l < len(self.hbits) else (None, 0)
                self._c("gemm_fwd_l%d" % l, "dl_gemm_s3_nt_bits", B, hdim, self.in_ld[l], ptr(x), self.in_ld[l],
                        ptr(self.WTp[l]), self.in_ld[l], self.in_ld[l] * self.out_ld[l], ptr(self.h[l]),
                        self.h_ld[l], 1, None, 0, *bits, s)
            else:
                self._c("gemm_fwd_l%d" % l, "dl_gemm_f32", 0, 0, B, hdim, self.in_ld[l], ptr(x), self.in_ld[l],
                        ptr(self.W[l]), self.out_ld[l], ptr(self.h[l]), self.h_ld[l], 1, None, 0, 1, 0, s)
            x = self.h[l]

    def _head(self, B, s, train=True):
        """Output layer + loss: the FM / deep_res head, or the wdl cross logit on the local
        wide table (gradients of the exchanged wide rows left in wgloc at their slots)."""
        sp = self.spec
        H = sp.hidden[-1]
        inv_b = 1.0 / (B * self.world)
        if self.wdl:
            if train:
                self.wgloc.zero_()
            fn, dh_last = ("dl_wdl_head_fwd_bwd_bf16", self.dhb[-1]) if self.bf else ("dl_wdl_head_fwd_bwd", self.dh[-1])
            self._c("head", fn, B, sp.Fw, H, ptr(self.in_wide_loc), sp.Fw, ptr(self.h[-1]), self.h_ld[-1],
                    ptr(self.wloc), ptr(self.wb), self.wgloc.numel(), ptr(self.in_label), sp.logloss_eps, inv_b,
                    ptr(self.score), ptr(self.z), ptr(self.dz), ptr(dh_last), ptr(self.wgloc) if train else None,
                    None, ptr(self.head_slab), self.head_blocks, ptr(self.err), s)
            return
        self._c("head", "dl_head_fwd_bwd", B, sp.fm_cols, H, ptr(self.fm_out), self.fm_ld, ptr(self.h[-1]),
                self.h_ld[-1], ptr(self.w_head), ptr(self.in_label), sp.logloss_eps, inv_b, ptr(self.score),
                ptr(self.z), ptr(self.dz), ptr(self.dh[-1]), ptr(self.head_slab), self.head_blocks, s)

    def _input_grads(self, B, s):
        """Step 5b: the input-gradient chain, top layer down to dx0, then every unique row's
        gradient into its slot (dl_embed_bwd_sorted with the route's slots)."""
        sp = self.spec
        L = self.layout
        nl = len(sp.hidden)
        if self.bf and not self.wdl:
            self._c("cast_dh", "dl_cast_bf16", ptr(self.dh[-1]), B, self.h_ld[-1], self.h_ld[-1], ptr(self.dhb[-1]),
                    self.h_ld[-1], s)
        for l in reversed(range(nl)):
            if self.bf:
                if l > 0:   # dX = dY . W^T, ReluGrad by the bf16 activations, bf16 out
                    self._c("gemm_dx_l%d" % l, "dl_gemm_bf16", 0, 1, B, sp.hidden[l - 1], self.out_ld[l],
                            ptr(self.dhb[l]), self.h_ld[l], ptr(self.Wb[l]), self.out_ld[l], ptr(self.dhb[l - 1]),
                            self.h_ld[l - 1], 1, 2, ptr(self.hb[l - 1]), self.h_ld[l - 1], 1, 0, s)
                else:       # dx0 stays fp32 for the embedding backward
                    self._c("gemm_dx_l0", "dl_gemm_bf16", 0, 1, B, self.dx_cols, self.out_ld[0], ptr(self.dhb[0]),
                            self.h_ld[0], ptr(self.Wb[0]), self.out_ld[0], ptr(self.dx0), self.dx_ld, 0, 0, None, 0,
                            1, 0, s)
                continue
            if self.s3:
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
                continue
            self._c("transpose_l%d" % l, "dl_transpose_f32", ptr(self.W[l]), self.in_ld[l], self.out_ld[l],
                    self.out_ld[l], ptr(self.Wt), self.in_ld[l], s)
            if l > 0:
                self._c("gemm_dx_l%d" % l, "dl_gemm_f32", 0, 0, B, sp.hidden[l - 1], self.out_ld[l], ptr(self.dh[l]),
                        self.h_ld[l], ptr(self.Wt), self.in_ld[l], ptr(self.dh[l - 1]), self.h_ld[l - 1], 2,
                        ptr(self.h[l - 1]), self.h_ld[l - 1], 1, 0, s)
            else:
                self._c("gemm_dx_l0", "dl_gemm_f32", 0, 0, B, self.dx_cols, self.out_ld[0], ptr(self.dh[0]),
                        self.h_ld[0], ptr(self.Wt), self.in_ld[0], ptr(self.dx0), self.dx_ld, 0, None, 0, 1, 0, s)
        self._c("embed_bwd", "dl_embed_bwd_sorted", C_ref(L), None, ptr(self.rows_u[self.rep:]), ptr(self.idx_uniq),
                ptr(self.idx_off), ptr(self.idx_n), ptr(self.idx_refs), self.world, B * self.n_slot, ptr(self.dz),
                ptr(self.w_head), ptr(self.fm_sum), ptr(self.dx0), ptr(self.g_all), ptr(self.g1_all), None, 1,
                ptr(self.upos), s)

    def _weight_grads(self, B, s):
        """Step 6 (main branch): weight gradients (split-K slabs summed into the flat buffer), the
        head's column sums, the replicated rows' gradients — beside the gradient exchange."""
        sp = self.spec
        E, L = sp.E, self.layout
        nl = len(sp.hidden)
        dws = self._dw_splits(B, fixed="DLAMD_DW_SPLITS" in os.environ)
        for l in reversed(range(nl)):
            splits = dws[l]
            xin = self.x0 if l == 0 else self.h[l - 1]
            hdim = sp.hidden[l]
            stride = self.in_ld[l] * self.out_ld[l]
            if self.bf:
                xl = self.x0b if l == 0 else self.hb[l - 1]
                self._c("gemm_dw_l%d" % l, "dl_gemm_bf16", 1, 0, self.in_ld[l], hdim, B, ptr(xl), self.in_ld[l],
                        ptr(self.dhb[l]), self.h_ld[l], ptr(self.w_slab), self.out_ld[l], 0, 3, None, 0, splits,
                        stride, s)
            elif self.s3:
                self._c("gemm_dw_l%d" % l, "dl_gemm_s3_tn", self.in_ld[l], hdim, B, ptr(xin), self.in_ld[l],
                        ptr(self.dh[l]), self.h_ld[l], ptr(self.w_slab), self.out_ld[l], splits, stride, s)
            else:
                self._c("gemm_dw_l%d" % l, "dl_gemm_f32", 1, 0, self.in_ld[l], hdim, B, ptr(xin), self.in_ld[l],
                        ptr(self.dh[l]), self.h_ld[l], ptr(self.w_slab), self.out_ld[l], 3, None, 0, splits, stride,
                        s)
            self._c("slab_sum_l%d" % l, "dl_slab_sum", ptr(self.w_slab),
                    _num_splits(B, splits, 64 if (self.s3 or self.bf) else 16), stride, stride,
                    ptr(self.flat[self.seg[l][1]:]), s)
        hoff = self.seg[nl][1]
        self._c("slab_sum_head", "dl_slab_sum", ptr(self.head_slab), call_int(self.head_grid, B), self.head_w,
                self.head_w, ptr(self.flat[hoff:]), s)
        if not self.rep:
            return
        # replicated rows: the cate-id references' gradients (the replicated group's slots) and
        # the FM cont fields', into the flat buffer (every rank adds its part; the all-reduce sums)
        rg = self.flat[self.rep_off: self.rep_off + self.rep_t.numel()].view(-1, E)
        rg1 = self.flat[self.rep_off + self.rep_t.numel():]
        rg.zero_()
        rg1.zero_()
        o = self.nb * self.cap
        call("dl_shard_scatter_add", ptr(self.g_all[o:]), ptr(self.g1_all[o:]) if sp.fm else None, ptr(self.rep_ids),
             self.rep_cap, E, ptr(rg), ptr(rg1) if sp.fm else None, ptr(self.rep_scratch), s)
        if sp.fm:
            bwd_blocks = call_int("dl_embed_bwd_grid", C_ref(L))
            cb = self._cont_blocks(B, bwd_blocks)
            self._c("cont_bwd", "dl_embed_cont_bwd", C_ref(L), ptr(self.rows_u), ptr(self.in_cont), ptr(self.dz),
                    ptr(self.w_head), ptr(self.fm_sum), ptr(self.cont_slab), cb, s)
            self._c("cont_reduce", "dl_embed_cont_reduce", C_ref(L), ptr(self.cont_slab), cb, ptr(rg), ptr(rg1),
                    ptr(self.rep_scratch), s)

    def _dense_adam(self, B, s):
        """Step 7a: TF1 Adam on the all-reduced dense and replicated gradients (identical on every
        rank); the tower updates write their GEMM operand copies themselves."""
        sp = self.spec
        E = sp.E
        nl = len(sp.hidden)
        hoff = self.seg[nl][1]
        reg = sp.hidden_reg   # wdl: L2 on every hidden weight matrix (wdl.py:272-275), bias row excluded
        for l in range(nl):
            off, sz = self.seg[l][1], self.seg[l][2]
            l2, l2n = (sp.l2, ([self.D0] + sp.hidden)[l] * self.out_ld[l]) if reg else (0.0, 0)
            if self.s3 or self.bf:
                self._c("adam_dense_l%d" % l, "dl_adam_dense_split3" if self.s3 else "dl_adam_dense_bf16",
                        ptr(self.W[l]), ptr(self.Wm[l]), ptr(self.Wv[l]), ptr(self.flat[off:]), 1, sz, self.in_ld[l],
                        self.out_ld[l], l2, l2n, 1 if reg == "l1" else 0, ptr(self.opt),
                        ptr(self.opt[8:]) if reg else None, ptr(self.Wp[l] if self.s3 else self.Wb[l]),
                        ptr(self.WTp[l] if self.s3 else self.WbT[l]), s)
            else:
                self._c("adam_dense_l%d" % l, "dl_adam_dense_reg", ptr(self.W[l]), ptr(self.Wm[l]), ptr(self.Wv[l]),
                        ptr(self.flat[off:]), 1, sz, sz, l2, l2n, 1 if reg == "l1" else 0, ptr(self.opt), None,
                        ptr(self.opt[8:]) if reg else None, s)
        if self.wdl:
            H = sp.hidden[-1]
            self._c("adam_bias", "dl_adam_dense", ptr(self.wb), ptr(self.wbm), ptr(self.wbv), ptr(self.flat[hoff + H:]),
                    1, 1, 1, 0.0, 0, ptr(self.opt), None, None, s)
        else:
            self._c("adam_head", "dl_adam_dense", ptr(self.w_head), ptr(self.hm), ptr(self.hv), ptr(self.flat[hoff:]),
                    1, self.head_w, self.head_n, sp.l2, self.head_n - 1, ptr(self.opt), ptr(self.w_head_prev), None,
                    s)
        if self.rep:
            rg = self.flat[self.rep_off: self.rep_off + self.rep_t.numel()]
            rg1 = self.flat[self.rep_off + self.rep_t.numel():]
            n = self.rep_t.shape[0]
            call("dl_adam_rows", ptr(self.rep_t), ptr(self.rep_m), ptr(self.rep_v), ptr(rg), ptr(self.rep_all), n, E,
                 0.0, 0, ptr(self.opt), None, s)
            if sp.fm:
                call("dl_adam_rows", ptr(self.rep_f), ptr(self.rep_fm), ptr(self.rep_fv), ptr(rg1), ptr(self.rep_all),
                     n, 1, 0.0, 0, ptr(self.opt), None, s)

    def _owner_apply(self, s):
        """Step 7b: the owners' update of every arriving row (blocks [0, W) of the gradients)."""
        sp = self.spec
        E, W, cap, rep = sp.E, self.world, self.cap, self.rep
        g1 = ptr(self.g1_all) if sp.fm else None
        if not self.lazy:
            self._c("rec_apply", "dl_shard_scatter_add", ptr(self.g_all), g1, ptr(self.ids_all), W * cap, E,
                    ptr(self.tg), ptr(self.fmg) if sp.fm else None, ptr(self.touched), s)
            if sp.fm:
                self._c("adam_table", "dl_adam_rows", ptr(self.table), ptr(self.tm), ptr(self.tv), ptr(self.tg),
                        ptr(self.touched), self.table.shape[0], E, 0.0, 0, ptr(self.opt), None, s)
                self._c("adam_first", "dl_adam_rows", ptr(self.first), ptr(self.fmm), ptr(self.fmv), ptr(self.fmg),
                        ptr(self.touched), self.first.shape[0], 1, 0.0, 1, ptr(self.opt), None, s)
            else:
                self._c("adam_table", "dl_adam_rows", ptr(self.table), ptr(self.tm), ptr(self.tv), ptr(self.tg),
                        ptr(self.touched), self.table.shape[0], E, 0.0, 1 | self.rows_sparse, ptr(self.opt), None, s)
            return
        if self.owner_update == "chain":
            self._c("rec_apply", "dl_rec_apply_chain", ptr(self.rec), self.rec_ld, E, self.rec_flags,
                    ptr(self.ids_all), W * cap, ptr(self.own_head), ptr(self.own_next), ptr(self.g_all), g1,
                    ptr(self.hist), self.hist_len, ptr(self.opt), s)
            return
        rows, rows1 = self.rows_u[rep:], (self.rows_u1[rep:] if sp.fm else None)
        if W == 1:   # one sender's block: rows already unique and in order — identity segments
            uniq, off, nu, pos = self.ids_all, self.iota, self.hdr_all, self.iota
        else:
            uniq, off, nu, pos = self.own_uniq, self.own_off, self.own_n, self.own_pos
        self._c("rec_apply", "dl_rec_apply_segments", ptr(self.rec), self.rec_ld, E, self.rec_flags, ptr(uniq),
                ptr(off), ptr(nu), W * cap, W * cap, ptr(pos), ptr(self.g_all), g1, ptr(rows), ptr(rows1),
                ptr(self.own_mv), ptr(self.hist), self.hist_len, ptr(self.opt), s)

    def _owner_group(self, s):
        """The owner's grouping of this step's arrivals by row (a branch: it needs only the
        received ids)."""
        W, cap = self.world, self.cap
        if not self.lazy:
            return
        if self.owner_update == "chain":
            call("dl_rec_chain_link", ptr(self.ids_all), W * cap, ptr(self.own_head), ptr(self.own_next), s)
        elif W > 1:
            self._c("owner_sort", "dl_sort_unique", ptr(self.ids_all), W * cap, self.own_bits, ptr(self.own_ws),
                    self.own_ws.numel(), ptr(self.own_keys), ptr(self.own_pos), ptr(self.own_uniq),
                    ptr(self.own_off), ptr(self.own_n), None, s)

    def _wide_update(self, s):
        """wdl_weights: the arrived wide gradients + the deep-output rows this rank owns, then the
        dense L2 Adam sweep over the shard (wdl.py:270-271), then every rank's copy of the
        deep-output rows from their owners (an in-place all-reduce)."""
        sp = self.spec
        H = sp.hidden[-1]
        hoff = self.seg[len(sp.hidden)][1]
        o = self.wloc_off
        call("dl_shard_add_fixed", ptr(self.wgloc[o:]), ptr(self.wids_all), self.world * self.wcap, ptr(self.wg),
             ptr(self.w_touched), s)
        call("dl_wide_fold_owned", ptr(self.flat[hoff:]), H, sp.Fw, self.world, self.rank, ptr(self.wg),
             ptr(self.w_touched), s)
        self.wide_reg.zero_()
        self._c("adam_wide", "dl_adam_rows", ptr(self.ww), ptr(self.wm), ptr(self.wv), ptr(self.wg),
                ptr(self.w_touched), self.ww.shape[0], 1, sp.l2, 1 | _lib.ROWS_GRAD_FIXED, ptr(self.opt),
                ptr(self.wide_reg), s)
        self._wide_refresh(s)

    def _wide_refresh(self, s):
        """Every rank's copy of the deep-output rows Fw..Fw+H of wdl_weights (read by the cross
        logit) from their owners: one [H] sum all-reduce, in place."""
        sp = self.spec
        H = sp.hidden[-1]
        d = self.wloc[sp.Fw: sp.Fw + H]
        call("dl_wide_owned_values", ptr(self.ww), H, sp.Fw, self.world, self.rank, ptr(d), s)
        self.exch.all_reduce(d, torch.cuda.current_stream())

    def _step(self, B):
        """One whole training step on the current stream (graph-captured, or eager), branches
        forked to the engine's streams and joined."""
        sp = self.spec
        s = _lib.stream_handle()
        main = torch.cuda.current_stream()
        L = self.layout
        L.batch = B
        self._requests(s)
        self._c("step_begin", "dl_shard_step_begin", ptr(self.hdr_all), ptr(self.whdr_all) if self.wdl else None,
                self.world, self.cap, self.wcap, ptr(self.opt), sp.decay_rate, float(sp.decay_steps),
                ptr(self.hist) if self.lazy else None, self.hist_len if self.lazy else 0, s)
        own = self.lazy and (self.owner_update == "chain" or self.world > 1)
        if own:   # the owner's grouping of the arrivals, beside the gather and the forward
            self.own_stream.wait_stream(main)
            with torch.cuda.stream(self.own_stream):
                self._owner_group(_lib.stream_handle(self.own_stream))
        self._gather_owned(B, s, 1)
        self._answers(s)
        self._forward_local(B, s, True)
        self._input_grads(B, s)
        # the gradients to their owners on a branch, beside the weight gradients
        x = self.x_stream
        x.wait_stream(main)
        garrs = [self.g_all[: self.nb * self.cap].view(self.nb, self.cap * sp.E)]
        if sp.fm:
            garrs.append(self.g1_all[: self.nb * self.cap].view(self.nb, self.cap))
        if self.wdl:
            o = self.wloc_off
            garrs.append(self.wgloc[o: o + self.nb * self.wcap].view(self.nb, self.wcap))
        with torch.cuda.stream(x):
            self._c("x_grads", "exchange", lambda: self.exch.blocks(garrs, 0, x))
        self._weight_grads(B, s)
        if self.ar_serial:
            # the dense all-reduce after the gradient exchange, on its communicator and stream:
            # one RCCL kernel at a time, in the same order on every rank
            x.wait_stream(main)
            with torch.cuda.stream(x):
                self._c("all_reduce", "exchange", lambda: self.exch.all_reduce(self.flat, x, serial=True))
            main.wait_stream(x)
        else:
            # the dense all-reduce on the second communicator's stream, beside the gradient exchange
            a = self.ar_stream
            a.wait_stream(main)
            with torch.cuda.stream(a):
                self._c("all_reduce", "exchange", lambda: self.exch.all_reduce(self.flat, a))
            main.wait_stream(a)
        self._dense_adam(B, s)
        main.wait_stream(x)
        if own:
            main.wait_stream(self.own_stream)
        if self.wdl:
            self._wide_update(s)
        self._owner_apply(s)
        hoff = self.seg[len(sp.hidden)][1]
        coef = sp.l2 if sp.hidden_reg == "l1" else 0.5 * sp.l2
        self._c("loss_acc", "dl_loss_accumulate", ptr(self.flat[hoff:]), 1, self.head_w, self.head_w - 1,
                1.0 / (B * self.world), ptr(self.opt), coef, ptr(self.loss_acc), ptr(self._ring), s)

    def _capture_step(self, B):
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with capture_guard(), torch.cuda.graph(g, stream=st, capture_error_mode="thread_local"):
            self._step(B)
        torch.cuda.current_stream().wait_stream(st)
        return g

    # ------------------------------------------------------------ step
    def prefetch(self, batch, graph=False, after=None):
        """Stage the next batch, index and route it on the side stream while this step runs."""
        super().prefetch(batch, graph=False, after=after)

    def train_step(self, batch=None, graph=False, next_batch=None):
        """One training step on this rank's batch (every rank calls it together).  Returns B.
        Raises (on every rank at the same call, `lag` calls after the step) when a step was
        skipped for a bad id on any rank; replays the steps an overflow skipped."""
        B = self._submit(batch, graph, next_batch)
        self._check_reports(self.lag)
        return B

    def _submit(self, batch, graph, next_batch):
        B, indexed = self._begin(batch)
        self._mark("start")
        if not indexed:
            self._pre(B)
        if self.lazy:
            if self.since_flush >= self.hist_len - 2:   # bound every row's lag below the alpha ring
                self.flush()
            self.since_flush += 1
        if next_batch is not None:   # the next batch's staging, index and route, beside this step
            self.prefetch(next_batch)
        self._mark("prefetch")
        if self._ring_sent is None:   # the device's step sequence (a read that waits, once)
            self._ring_sent = int(self.opt.view(torch.int32)[_lib.OPT_SEQ].item())
            self._ring_checked = self._ring_sent
        # the first steps run eagerly: RCCL connects its peers then, not inside a capture
        if (graph and self.prof is None and self._steps_eager >= 1 and not self.exch.staged
                and os.environ.get("DLAMD_SHARD_GRAPH", "1") != "0" and not getattr(self, "_graph_failed", False)):
            key = (getattr(self, "_cur", 0), B)
            g = self.graphs.get(key)
            if g is None:
                try:
                    g = self.graphs[key] = self._capture_step(B)
                except Exception as ex:   # a runtime that cannot capture the step's RCCL group: eager
                    import sys
                    print("[shard] step capture failed (%r): the step runs eagerly" % (ex,), file=sys.stderr)
                    self._graph_failed = True
                    g = None
            if g is not None:
                g.replay()
            else:
                self._step(B)
        else:
            self._step(B)
            self._steps_eager += 1
        self._mark("submitted")
        self._ring_sent += 1
        self._hist_b[self._ring_sent] = batch
        self._release()
        self.steps += 1
        self.last_batch = B
        self.last_loss_sum = None
        return B

    def _clear_status(self):
        """Status, skip, bad-step and bad-count words and the bad-rank mask (not the sequence)."""
        self.opt[_lib.OPT_STATUS: _lib.OPT_BAD_COUNT + 1].zero_()
        self.opt[_lib.OPT_BAD_RANKS] = 0.0

    def _check_reports(self, lag):
        """Read the status reports of every step submitted up to `lag` calls ago (waiting for the
        oldest if needed: every rank reads the same reports at the same call).  A skipped step is
        handled identically everywhere: bad ids raise, an overflow grows the blocks and replays."""
        if self._ring_sent is None:   # no step submitted since the last resynchronisation
            return
        r = self._ring_np
        bad = []
        while self._ring_checked < self._ring_sent - lag:
            k = self._ring_checked + 1
            j = 2 * (k & 3)
            t0 = time.perf_counter()
            spins = 0
            while int(r[j]) != k:
                spins += 1
                if spins > 1000:
                    time.sleep(2e-5)
                if time.perf_counter() - t0 > self.guard_s:
                    self._guard_exit(k)
            self.host_wait += time.perf_counter() - t0
            word = int(r[j + 1]) & 0xffffffff
            skip = word >> 16
            self._ring_checked = k
            batch = self._hist_b.pop(k, None)
            if skip & _lib.STATUS_OVERFLOW:
                return self._recover(k, batch)
            if skip & (_lib.STATUS_LAG | _lib.STATUS_INDEX | _lib.STATUS_DESYNC):
                self._hist_b.clear()
                raise _lib.DLError("internal: sharded step %d faulted (status bits %#x: lag / index / desync)"
                                   % (k, skip))
            if skip & _lib.STATUS_BAD_ID:
                bad.append(k)
        if bad:
            torch.cuda.synchronize()
            ranks = int(self.opt.view(torch.int32)[_lib.OPT_BAD_RANKS].item())
            step = int(self.opt[_lib.OPT_BAD_STEP].item())
            self._clear_status()
            for w in self._error_words():
                w.zero_()
            raise _lib.DLError("InvalidArgumentError: categorical id out of range [0, %d) in the batch of rank(s) %s "
                               "— %d step(s) skipped on every rank with no update, the last at global_step %d"
                               % (self.N, [p for p in range(self.world) if ranks >> p & 1], len(bad), step))

    def _guard_exit(self, k):
        """The status report of step k did not arrive within guard_s seconds: a peer stopped, or
        this rank's step is stuck in a collective.  Raising would leave the process (and the job)
        waiting on the device at its next synchronisation; instead say where it stopped, from host
        memory only (the device may be the thing that hangs), and exit non-zero — the launcher then
        stops the other ranks."""
        import sys
        r = self._ring_np
        last = [(int(r[2 * j]), int(r[2 * j + 1]) & 0xffffffff) for j in range(4)]
        sys.stderr.write("[shard] rank %d/%d: the status report of step %d (sequence) did not arrive within %.0f s; "
                         "submitted %d, reports read %d, train_step calls %d, cap %d; status ring (k, word) %s — "
                         "a peer stopped or a collective is stuck: exiting with status 75\n"
                         % (self.rank, self.world, k, self.guard_s, self._ring_sent, self._ring_checked,
                            self.steps, self.cap, last))
        sys.stderr.flush()
        os._exit(75)

    def _recover(self, k, batch):
        """Step k overflowed a block on some rank, so it and every step after it were skipped on
        every rank: wait for them, clear the fault, grow the blocks and replay them in order.
        The replay needs each skipped step's batch argument as it was submitted: a step submitted
        with batch None (its inputs staged by the caller) cannot be replayed, which raises."""
        torch.cuda.synchronize()
        replay = [batch] + [self._hist_b[q] for q in sorted(self._hist_b)]
        self._hist_b.clear()
        self._clear_status()
        self._grow()
        self.steps -= len(replay)
        self._ring_sent = None
        if any(b is None for b in replay):   # the engine goes on with grown blocks; these steps are lost
            raise _lib.DLError("sharded step %d overflowed a block and was skipped with the %d step(s) after it: "
                               "their replay needs each step's batch, but one was submitted as train_step(None) "
                               "(inputs already staged); pass the batch to train_step, unmodified for `lag` calls, "
                               "when blocks may overflow" % (k, len(replay) - 1))
        self.overflows = getattr(self, "overflows", 0) + 1
        for b in replay:
            self._submit(b, False, None)
            self._check_reports(0)

    # ------------------------------------------------------------ predict / eval
    def predict(self, batch, logits=False, device=False):
        """Forward only on this rank's batch (reference eval/predict, deepfm_pipeline.py:294-311):
        the same index, route, request and answer exchanges as a training step, rows caught up to
        the last completed step (records are only read), no gradients, no update.  Every rank
        must call it together.  Returns the sigmoid scores [B] (or logits) as host numpy, or a
        device tensor copy with device=True."""
        self._check_reports(0)
        q = getattr(self, "_pfq", None) or []
        for p in q:   # pending prefetches: let them land, drop them
            torch.cuda.current_stream().wait_event(p[2])
        if q:
            q.clear()
            self._pf = None
        B = self.stage(batch)
        s = _lib.stream_handle()
        W = self.world
        self._pre(B)
        call("dl_shard_stamp", ptr(self.hdr_all), W, self.rank, ptr(self.opt), s)
        arrs = [self.ids_all.view(self.nb, self.cap), self.hdr_all.view(self.nb, 4)]
        if self.wdl:
            arrs += [self.wids_all.view(self.nb, self.wcap), self.whdr_all.view(self.nb, 4)]
        self.exch.blocks(arrs, 0)
        # the same decision on every rank, from every rank's header
        fl = 0
        for h in (self.hdr_all, self.whdr_all if self.wdl else None):
            if h is not None:
                hv = h[: 4 * W].view(W, 4)
                bad_rows = hv[:, 1].tolist()
                for f in bad_rows:
                    fl |= int(f)
        if fl & _lib.STATUS_OVERFLOW:
            self._grow()
            return self.predict(batch, logits, device)
        if fl & _lib.STATUS_BAD_ID:
            for w in self._error_words():
                w.zero_()
            raise _lib.DLError("InvalidArgumentError: categorical id out of range [0, %d) in a predict batch" % self.N)
        self._gather_owned(B, s, 0)
        self._answers(s)
        self._forward_local(B, s, False)
        self._release()
        out = (self.z if logits else self.score)[:B]
        return out.clone() if device else out.cpu().numpy()

    def evaluate(self, batches):
        """Global ROC-AUC over every rank's batches (the reference's eval: sklearn roc_auc_score
        over the whole validation set): scores stay on the device, one all-gather, then the
        exact dl_auc on the concatenation — the same value on every rank."""
        from .metrics import ShardedAucAccumulator
        acc = ShardedAucAccumulator(self.exch)
        for b in batches:
            acc.add(b["label"], self.predict(b, device=True))
        return acc.result()

    def loss_sum_begin(self):
        raise NotImplementedError("the sharded engine reads the loss per step: loss()")

    loss_sum_end = loss_sum_begin

    def loss(self):
        """Global loss of the last step: the all-reduced loss column + L2 on the head weights
        (wdl: + L2 on every hidden weight matrix and on all of wdl_weights, whose shard sums are
        all-reduced here — every rank calls it)."""
        self._check_reports(0)
        sp = self.spec
        hoff = self.seg[len(sp.hidden)][1]
        if self.wdl:
            H = sp.hidden[-1]
            data = float(self.flat[hoff + H + 1].item())
            wr = self.wide_reg.clone()
            self.exch.host_sum(wr)
            return data / (self.last_batch * self.world) + sp.l2 * 0.5 * (_lib.reg_sum(self.opt) +
                                                                           _lib.reg_sum(wr))
        data = float(self.flat[hoff + self.head_w - 1].item())
        w = self.w_head_prev[: self.head_n - 1].double()
        return data / (self.last_batch * self.world) + sp.l2 * 0.5 * float((w * w).sum().item())

    def check_error(self):
        """Every report read (raising as train_step would), then the engine's own check."""
        self._check_reports(0)
        super().check_error()
