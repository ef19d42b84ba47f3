"""Row-sharded multi-GPU training (BASELINE config C4).

One process per GPU.  The embedding table (and its first-order column and TF1
Adam state) is split by rows: row r lives on rank r % world at local row
r // world (cyclic, so Zipf-hot low ids spread over all ranks).  The rows
below ``replicated`` (deepfm_pipeline's 13 cont-field rows, hit by every
sample) are replicated on every rank.  Dense parameters are replicated.

Step on every rank (local batch B, global batch B*world):
  1. index: sort/dedup this batch's row references; unique rows grouped by owner
  2. all-gather of the per-owner unique-row counts, all-to-all of the row ids
  3. owners gather the requested rows (E floats + first-order weight)
  4. all-to-all of the rows back; the forward expands them through the inverse map
  5. MLP + head forward, input gradients down to the embeddings
  6. per-unique-row gradient (deterministic segment sum), all-to-all to owners,
     overlapping the weight gradients
  7. one all-reduce (sum) of the dense gradients + replicated-row gradients
  8. TF1 Adam: dense + replicated parameters identically everywhere; the shard rows
     by their owners — row records with lazy-exact catch-up: each row's arrivals
     (at most one per sender) summed in a fixed order and applied once
The result equals single-GPU training on the concatenated global batch.

Off the critical path, on a second (high-priority) stream: the owners' arrival
chains and record update of a step, and — with train_step(next_batch=...) — the
next batch's staging, index build and count all-gather, so a step starts at its
id exchange with the counts already on the host.

Collectives go through torch.distributed: backend "nccl" is RCCL (xGMI) and
exchanges device tensors directly; backend "gloo" (CPU tests, and several ranks
sharing one GPU) stages them through host memory.
"""
import os
import time

import numpy as np

import torch
import torch.distributed as dist

from . import _lib
from ._lib import call, ptr
from .engine import CTREngine, C_ref, _num_splits, _ru, call_int, capture_guard


class _Works:
    """The works of one grouped point-to-point exchange, waited together, and the event
    after the rank's own segment's copy (queued on the issuing stream: a waiter on another
    stream must order after it too)."""

    def __init__(self, works, copied):
        self.works, self.copied = works, copied

    def wait(self):
        torch.cuda.current_stream().wait_event(self.copied)
        for w in self.works:
            w.wait()


class Exchange:
    """Thin wrapper over torch.distributed collectives for the sharded step."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = dist.get_backend(group)
        self.staged = self.backend != "nccl"

    def _dev(self, t):
        return t.cpu() if self.staged and t.is_cuda else t

    def counts(self, send_counts):
        """All-to-all of one int per peer -> list of received counts."""
        dev = "cpu" if self.staged else "cuda"
        s = torch.tensor(send_counts, dtype=torch.int64, device=dev)
        r = torch.empty_like(s)
        dist.all_to_all_single(r, s, group=self.group)
        return [int(x) for x in r.cpu().tolist()]

    def count_matrix(self, owner_counts):
        """All-gather of every rank's per-owner counts (device int32 [world+1]) -> host
        [world][world+1] list: row r = what rank r sends to each owner (+ its replicated
        count).  One collective and one device->host copy give both the send and the
        receive splits."""
        c = owner_counts.to(torch.int64)
        if self.staged:
            c = c.cpu()
        if self.staged:
            parts = [torch.empty_like(c) for _ in range(self.world)]
            dist.all_gather(parts, c, group=self.group)
            return torch.stack(parts).tolist()
        out = torch.empty(self.world * c.numel(), dtype=torch.int64, device=c.device)
        dist.all_gather_into_tensor(out, c, group=self.group)
        return out.view(self.world, -1).cpu().tolist()

    def count_matrix_async(self, owner_counts):
        """count_matrix without blocking the host: the all-gather and a copy into pinned host
        memory are queued behind the current stream's work; resolve_counts() waits only for
        that copy.  (Host-staged backends resolve immediately.)"""
        if self.staged:
            return self.count_matrix(owner_counts)
        c = owner_counts.to(torch.int64)
        out = torch.empty(self.world * c.numel(), dtype=torch.int64, device=c.device)
        dist.all_gather_into_tensor(out, c, group=self.group)
        host = torch.empty(out.numel(), dtype=torch.int64, pin_memory=True)
        host.copy_(out, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return (host, ev, c.numel())

    @staticmethod
    def resolve_counts(h):
        if isinstance(h, list):
            return h
        host, ev, n = h
        ev.synchronize()
        return host.view(-1, n).tolist()

    def _exchange_p2p(self, res, src, send_splits, recv_splits):
        """RCCL all-to-all as grouped point-to-point transfers with the rank's own segment
        copied on the current stream (a device copy at HBM speed instead of RCCL's few-CU
        self-transfer: all of the data at one rank, half of it at two).  Returns the works."""
        so = [0] * (self.world + 1)
        ro = [0] * (self.world + 1)
        for p in range(self.world):
            so[p + 1] = so[p] + send_splits[p]
            ro[p + 1] = ro[p] + recv_splits[p]
        me = self.rank
        if send_splits[me]:
            res[ro[me]: ro[me + 1]].copy_(src[so[me]: so[me + 1]])
        ops = []
        for p in range(self.world):
            if p == me:
                continue
            if send_splits[p]:
                ops.append(dist.P2POp(dist.isend, src[so[p]: so[p + 1]], p, self.group))
            if recv_splits[p]:
                ops.append(dist.P2POp(dist.irecv, res[ro[p]: ro[p + 1]], p, self.group))
        return dist.batch_isend_irecv(ops) if ops else []

    def all_to_all(self, send, send_splits, recv_splits, out=None, async_op=False):
        """Variable all-to-all along dim 0 (splits in rows).  `out` (device, contiguous,
        sum(recv_splits) rows) receives in place — RCCL writes straight into it.
        async_op (RCCL only): returns (result, work) with the collective running on
        RCCL's stream; work.wait() orders the current stream after it."""
        shape = (sum(recv_splits),) + tuple(send.shape[1:])
        src = self._dev(send.contiguous())
        direct = out is not None and not self.staged and out.is_contiguous()
        res = out if direct else torch.empty(shape, dtype=send.dtype, device=src.device)
        if not self.staged:
            works = self._exchange_p2p(res, src, list(send_splits), list(recv_splits))
            if async_op:
                copied = torch.cuda.Event()
                copied.record()
                return res, _Works(works, copied)
            for w in works:
                w.wait()
            if direct:
                return out
            if out is not None:
                out.copy_(res)
                return out
            return res
        dist.all_to_all_single(res, src, output_split_sizes=list(recv_splits),
                               input_split_sizes=list(send_splits), group=self.group)
        if async_op:
            res = res.to(send.device) if res.device != send.device else res
            return res, None
        if direct:
            return out
        res = res.to(send.device, non_blocking=False) if res.device != send.device else res
        if out is not None:
            out.copy_(res)
            return out
        return res

    def all_reduce(self, t):
        if self.world == 1:   # the sum over one rank is the input
            return t
        if self.staged and t.is_cuda:
            c = t.cpu()
            dist.all_reduce(c, group=self.group)
            t.copy_(c)
        else:
            dist.all_reduce(t, group=self.group)
        return t


class ShardedCTREngine(CTREngine):
    """CTREngine whose embedding tables are row-sharded across the ranks of `exch`."""

    def __init__(self, spec, max_batch, exch, device="cuda", seed=2019, adam="dense", hist_len=4096,
                 owner_update=None):
        if spec.model not in ("deepfm_pipeline", "dnn_pipeline", "wdl"):
            raise ValueError("sharded path supports deepfm_pipeline / dnn_pipeline / wdl")
        self.exch = exch
        self.world, self.rank = exch.world, exch.rank
        N = spec.n_rows
        self.rep = spec.C if spec.model == "deepfm_pipeline" else 0
        local_rows = -(-N // self.world)
        super().__init__(spec, max_batch, device=device, seed=seed, init="none", bwd="sorted",
                         table_rows=local_rows, adam=adam, hist_len=hist_len)
        dev = self.dev
        z = lambda *sh, dt=torch.float32: torch.zeros(*sh, dtype=dt, device=dev)
        E = spec.E
        self.local_rows = local_rows
        # side stream (own hardware queue): the owner arrival chains and the record update of
        # a step run there, the update overlapping the next step's start
        self.side = None
        self.apply_done = None
        # DLAMD_HOST_TIMING=1: host-side timestamps of the step's phases (diagnostics)
        self.host_marks = [] if os.environ.get("DLAMD_HOST_TIMING") else None
        self.opt_snap = z(2, _lib.OPT_LEN)
        if self.lazy:
            # shard rows as records (rec.hip).  Owners group the ids they receive by row (a sort,
            # or per-row arrival chains); the gradients come back in the same positions, so each
            # row's arrivals are summed in ascending position order and applied once —
            # deterministic, no dense gradient table.
            # owner_update: "sort" (dl_sort_unique + dl_rec_apply_segments) or "chain"
            # (dl_rec_chain_link + dl_rec_apply_chain: no sort; bit-identical records)
            self.owner_update = owner_update or os.environ.get("DLAMD_OWNER_UPDATE", "sort")
            if self.owner_update not in ("sort", "chain"):
                raise ValueError("owner_update must be 'sort' or 'chain'")
            self.mv_u = None
            self.own_cap = 0
            self.own_bits = max(1, int(self.rows_pad - 1).bit_length())
            if self.owner_update == "chain":
                # arrival chains (rec.hip dl_rec_chain_link): head per local row, -1 = no arrival
                self.own_head = torch.full((self.rows_pad,), -1, dtype=torch.int32, device=self.dev)
        R = max(self.rep, 1)
        rp = _ru(R, 16)
        self.rep_t, self.rep_m, self.rep_v, self.rep_g = z(rp, E), z(rp, E), z(rp, E), z(rp, E)
        self.rep_f, self.rep_fm, self.rep_fv, self.rep_fg = z(rp), z(rp), z(rp), z(rp)
        self.rep_touched = z(rp, dt=torch.uint8)
        n = self.n_refs
        self.inv = z(n, dt=torch.int32)
        self.owner_counts = z(self.world + 1, dt=torch.int32)
        self.send_ids = z(n, dt=torch.int32)
        self.gU = z(n, E)
        self.g1U = z(n)
        self.rows_u = z(self.rep + n, E)
        self.rows_u1 = z(self.rep + n)
        # flat dense-gradient buffer: every layer's W_aug, the head, replicated rows
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
        self.rep_off = off
        off += rp * E + rp
        self.flat = z(off)
        if self.rep:
            self.rep_touched[: self.rep] = 1
        if self.wdl:
            self._init_wide(max_batch)

    def _init_wide(self, B):
        """wdl_weights sharded like the table (row r on rank r % world), plus the per-rank local
        wide table the cross logit reads: wloc = [unused (Fw) | deep-output rows Fw..Fw+H,
        replicated | this batch's exchanged unique wide rows].  The head (dl_wdl_head_fwd_bwd)
        then runs unchanged on local ids and leaves each unique row's gradient in wgloc."""
        sp = self.spec
        W = self.world
        z = lambda *sh, dt=torch.float32: torch.zeros(*sh, dtype=dt, device=self.dev)
        Fw, H = sp.Fw, sp.hidden[-1]
        self.w_local = -(-self.w_rows // W)
        wl = _ru(self.w_local, 16)
        self.ww, self.wm, self.wv = z(wl), z(wl), z(wl)
        self.wg = z(wl, dt=torch.int64)
        self.w_touched = z(wl, dt=torch.uint8)
        self.wide_reg = z(4)
        nw = B * Fw
        self.n_wrefs = nw
        self.wloc_off = Fw + H
        self.wloc_rows = Fw + H + nw
        self.wloc = z(_ru(self.wloc_rows, 4))
        self.wgloc = z(self.wloc_rows, dt=torch.int64)
        self.in_wide_loc = z(B, Fw, dt=torch.int64)
        self.deep_buf = z(_ru(H, 4))
        # the wide ids' batch index (owner-grouped unique rows, inverse map), per buffer set
        wsb = _lib.lib().dl_index_workspace_bytes(max(1, nw))
        self.widx_ws = z(wsb, dt=torch.uint8)
        self.widx_keys, self.widx_refs, self.widx_uniq = (z(nw, dt=torch.int32) for _ in range(3))
        self.widx_off = z(nw + 1, dt=torch.int32)
        self.widx_n = z(4, dt=torch.int32)
        self.winv = z(nw, dt=torch.int32)
        self.wowner_counts = z(W + 1, dt=torch.int32)
        self.wsend_ids = z(nw, dt=torch.int32)
        WL = _lib.EmbLayout()
        WL.n_rows = self.w_rows
        WL.batch = B
        WL.emb_dim = sp.E
        WL.cate_fields = Fw
        WL.cate_ld = self.in_wide.shape[1]
        WL.use_fm = 0
        WL.zero_row0 = 0
        self.wlayout = WL

    def _owner_buffers(self, n):
        """(Re)size the owner-side arrival-chain buffer for n received ids."""
        if n > self.own_cap:
            self._join_side()   # the previous step's update on the side stream still reads them
        if n <= self.own_cap:
            return
        cap = max(n, int(self.own_cap * 1.25), 1 << 16)
        # empty, not zeros: a fill queued on the compute stream could land after the side
        # stream has written them (the sort / the link write every entry later read)
        e = lambda k, dt=torch.int32: torch.empty(k, dtype=dt, device=self.dev)
        if self.owner_update == "chain":
            self.own_next = e(cap)
        else:
            self.own_ws = e(_lib.lib().dl_index_workspace_bytes(cap), torch.uint8)
            self.own_keys, self.own_pos, self.own_uniq = e(cap), e(cap), e(cap)
            self.own_off, self.own_n = e(cap + 1), e(4)
            # the owner gather's moment stash [cap][2E+4], read back by the sorted update
            # (the arrival-chain update re-reads the record instead: no stash)
            self.own_mv = e(cap * (2 * self.spec.E + 4), torch.float32)
        self.own_cap = cap

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
            self._wide_refresh()
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

    def _owner_apply_args(self, recv_ids, nrecv, gb, g1b, opt, stream):
        """Entry point + arguments of the owners' record update (one per arriving row)."""
        sp = self.spec
        g1 = ptr(g1b) if sp.fm else None
        if self.owner_update == "chain":
            return ("dl_rec_apply_chain", ptr(self.rec), self.rec_ld, sp.E, self.rec_flags, ptr(recv_ids), nrecv,
                    ptr(self.own_head), ptr(self.own_next), ptr(gb), g1, ptr(self.hist), self.hist_len, ptr(opt),
                    stream)
        # the owner gather's outputs at every arrival: the caught-up state (no second replay)
        rows, rows1 = self.own_rows
        return ("dl_rec_apply_segments", ptr(self.rec), self.rec_ld, sp.E, self.rec_flags, ptr(self.own_uniq),
                ptr(self.own_off), ptr(self.own_n), nrecv, nrecv, ptr(self.own_pos), ptr(gb), g1, ptr(rows),
                ptr(rows1) if sp.fm else None, ptr(self.own_mv), ptr(self.hist), self.hist_len, ptr(opt), stream)

    def _mark(self, name):
        if self.host_marks is not None:
            self.host_marks.append((name, time.perf_counter()))

    def _join_side(self):
        """Order the compute stream after everything queued on the side stream."""
        if self.side is not None:
            torch.cuda.current_stream().wait_stream(self.side)

    def flush(self):
        self._join_side()
        super().flush()

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

    def _wide_exchange(self, B, cmw):
        """The wide lookup: unique wide rows' ids to their owners, the owners' current values
        back into the local wide table, local ids for the head.  Returns (send, recv, recv_ids)
        for the gradient return."""
        ex = self.exch
        W = self.world
        s = _lib.stream_handle()
        wsend = cmw[self.rank][:W]
        nwsend = sum(wsend)
        wrecv = [cmw[r][self.rank] for r in range(W)]
        nwrecv = sum(wrecv)
        wrecv_ids = ex.all_to_all(self.wsend_ids[:nwsend], wsend, wrecv)
        wout = torch.empty(max(nwrecv, 1), device=self.dev)
        if nwrecv:
            call("dl_shard_gather_scalar", ptr(self.ww), ptr(wrecv_ids), nwrecv, ptr(wout), s)
        off = self.wloc_off
        ex.all_to_all(wout[:nwrecv], wrecv, wsend, out=self.wloc[off: off + nwsend])
        call("dl_wide_local_ids", ptr(self.winv), B * self.spec.Fw, off, ptr(self.in_wide_loc), s)
        return wsend, wrecv, wrecv_ids

    def _wide_refresh(self):
        """Every rank's copy of the deep-output rows Fw..Fw+H of wdl_weights (read by the cross
        logit) from their owners: one [H] sum all-reduce."""
        sp = self.spec
        H = sp.hidden[-1]
        call("dl_wide_owned_values", ptr(self.ww), H, sp.Fw, self.world, self.rank, ptr(self.deep_buf),
             _lib.stream_handle())
        self.exch.all_reduce(self.deep_buf)
        self.wloc[sp.Fw: sp.Fw + H].copy_(self.deep_buf[:H])

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
        wide table (gradients of the exchanged wide rows left in wgloc)."""
        sp = self.spec
        H = sp.hidden[-1]
        inv_b = 1.0 / (B * self.world)
        if self.wdl:
            if train:
                self.wgloc.zero_()
            fn, dh_last = ("dl_wdl_head_fwd_bwd_bf16", self.dhb[-1]) if self.bf else ("dl_wdl_head_fwd_bwd", self.dh[-1])
            self._c("head", fn, B, sp.Fw, H, ptr(self.in_wide_loc), sp.Fw, ptr(self.h[-1]), self.h_ld[-1],
                    ptr(self.wloc), ptr(self.wb), self.wloc_rows, ptr(self.in_label), sp.logloss_eps, inv_b,
                    ptr(self.score), ptr(self.z), ptr(self.dz), ptr(dh_last), ptr(self.wgloc) if train else None,
                    None, ptr(self.head_slab), self.head_blocks, ptr(self.err), s)
            return
        self._c("head", "dl_head_fwd_bwd", B, sp.fm_cols, H, ptr(self.fm_out), self.fm_ld, ptr(self.h[-1]),
                self.h_ld[-1], ptr(self.w_head), ptr(self.in_label), sp.logloss_eps, inv_b, ptr(self.score),
                ptr(self.z), ptr(self.dz), ptr(self.dh[-1]), ptr(self.head_slab), self.head_blocks, s)

    def wide_state(self):
        """(global rows, wdl_weights values) of this rank's shard of wdl_weights (host numpy)."""
        rows = np.arange(self.w_local) * self.world + self.rank
        ok = rows < self.w_rows
        return rows[ok], self.ww[: self.w_local].cpu().numpy()[ok]

    def _mid_a(self, B):
        """Steps 5-6a: forward, head, the input-gradient chain down to dx0 and the per-row
        embedding gradients — fixed buffers and sizes for a batch size, so
        train_step(graph=True) replays it as one hipGraph (the exchanges around it need
        host-known sizes and stay eager).  The weight gradients are left to _mid_b, which
        runs while the embedding gradients are in flight to their owners."""
        sp = self.spec
        s = _lib.stream_handle()
        L = self.layout
        L.batch = B
        W = self.world
        rep = self.rep
        # 5. forward
        self._c("embed_fwd", "dl_embed_fwd_indexed", C_ref(L), ptr(self.rows_u), ptr(self.rows_u1) if sp.fm else None,
                ptr(self.inv), rep, ptr(self.in_cont), ptr(self.in_vec), ptr(self.x0b if self.x0_direct else self.x0),
                ptr(self.fm_out), ptr(self.fm_sum), s)
        if self.bf and not self.x0_direct:
            self._c("cast_x0", "dl_cast_bf16", ptr(self.x0), B, self.in_ld[0], self.in_ld[0], ptr(self.x0b),
                    self.in_ld[0], s)
        self._tower_fwd(B, s)
        self._head(B, s)
        # 6a. input gradients, top layer down
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
        # embedding gradients per unique row -> owners
        self._c("embed_bwd", "dl_embed_bwd_sorted", C_ref(L), None, ptr(self.rows_u[rep:]), ptr(self.idx_uniq),
                ptr(self.idx_off), ptr(self.idx_n), ptr(self.idx_refs), W, self.n_refs, ptr(self.dz),
                ptr(self.w_head), ptr(self.fm_sum), ptr(self.dx0), ptr(self.gU), ptr(self.g1U), None, 1, s)

    def _mid_b(self, B):
        """Step 6b: weight gradients (split-K slabs summed into the flat all-reduce buffer)
        and the head's column sums — overlaps the embedding-gradient all-to-all."""
        sp = self.spec
        s = _lib.stream_handle()
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
            call("dl_slab_sum", ptr(self.w_slab), _num_splits(B, splits, 64 if (self.s3 or self.bf) else 16), stride,
                 stride, ptr(self.flat[self.seg[l][1]:]), s)
        hoff = self.seg[nl][1]
        call("dl_slab_sum", ptr(self.head_slab), call_int(self.head_grid, B), self.head_w, self.head_w,
             ptr(self.flat[hoff:]), s)

    def _mid(self, B):
        self._mid_a(B)
        self._mid_b(B)

    def _replay(self, name, fn, B):
        """Capture fn(B) once per batch size as a hipGraph, then replay it."""
        g = getattr(self, name, None)
        if g is None or g[1] != B:
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            cg = torch.cuda.CUDAGraph()
            with capture_guard(), torch.cuda.graph(cg, stream=st, capture_error_mode="thread_local"):
                fn(B)
            torch.cuda.current_stream().wait_stream(st)
            g = (cg, B)
            setattr(self, name, g)
        g[0].replay()

    # ------------------------------------------------------------ step
    SLOT_ATTRS = CTREngine.SLOT_ATTRS + ("inv", "owner_counts", "send_ids", "widx_ws", "widx_keys", "widx_refs",
                                         "widx_uniq", "widx_off", "widx_n", "winv", "wowner_counts", "wsend_ids")

    def _index(self, B):
        """Step 1 on the current stream: the batch index (rows grouped by owner, replicated rows
        last) and the owner-local ids to send."""
        s = _lib.stream_handle()
        L = self.layout
        L.batch = B
        self._c("index_build", "dl_index_build", C_ref(L), ptr(self.in_cate), self.world, self.rep,
                ptr(self.idx_ws), self.idx_ws.numel(), ptr(self.idx_keys), ptr(self.idx_refs), ptr(self.idx_uniq),
                ptr(self.idx_off), ptr(self.idx_n), ptr(self.inv), ptr(self.owner_counts), ptr(self.err), s)
        call("dl_keys_to_local", ptr(self.idx_uniq), ptr(self.idx_n), self.n_refs, ptr(self.send_ids), s)
        if self.wdl:   # the wide ids: unique wdl_weights rows grouped by owner, inverse map
            WL = self.wlayout
            WL.batch = B
            self._c("index_build_wide", "dl_index_build", C_ref(WL), ptr(self.in_wide), self.world, 0,
                    ptr(self.widx_ws), self.widx_ws.numel(), ptr(self.widx_keys), ptr(self.widx_refs),
                    ptr(self.widx_uniq), ptr(self.widx_off), ptr(self.widx_n), ptr(self.winv),
                    ptr(self.wowner_counts), ptr(self.err), s)
            call("dl_keys_to_local", ptr(self.widx_uniq), ptr(self.widx_n), self.n_wrefs, ptr(self.wsend_ids), s)

    def _count_vec(self):
        """The per-owner counts every rank all-gathers: table rows (+ replicated), and for wdl
        the wide rows too (one collective for both), then the batch's id-validation word, so
        every rank learns from the same collective whether any rank's batch holds a bad id."""
        parts = [self.owner_counts] + ([self.wowner_counts] if self.wdl else []) + [self.err[:1]]
        return torch.cat(parts)

    def _split_counts(self, cm):
        """Strip the id-validation column off the all-gathered counts.  A bad id on any rank
        raises on every rank before the step begins (TF's InvalidArgumentError in the failing
        sess.run, deepfm_pipeline.py:219-221): nothing is exchanged or applied, the optimizer
        step does not advance, and the replicas stay identical."""
        bad = [r for r, row in enumerate(cm) if int(row[-1]) != 0]
        if bad:
            for w in self._error_words():
                w.zero_()
            raise _lib.DLError("InvalidArgumentError: categorical id out of range [0, %d) in the batch of rank(s) "
                               "%s — the step applied no update" % (self.N, bad))
        return [row[:-1] for row in cm]

    def _drop_prefetch(self, pf):
        """A prefetched batch that will not be trained: its counts are consumed and a bad id
        it carried is forgotten with it (its buffer set's validation word cleared)."""
        cm = self.exch.resolve_counts(pf[4])
        if any(int(row[-1]) != 0 for row in cm):
            self._slots[pf[0]]["err"].zero_()
        self._pf = None

    def prefetch(self, batch):
        """Stage the next batch, build its index and exchange its counts on the side stream
        while the current step runs; the next train_step(batch) starts at its id exchange with
        no host wait on the GPU (the counts are in pinned memory by then)."""
        self._enable_slots()
        if self._pf is not None:
            torch.cuda.current_stream().wait_event(self._pf[2])
        cur = self._cur
        k = 1 - cur
        side = self._side_stream()
        if self._slot_free[k] is not None:
            side.wait_event(self._slot_free[k])
        else:
            side.wait_stream(torch.cuda.current_stream())
        self._use_slot(k)
        try:
            with torch.cuda.stream(side):
                B = self.stage(batch)
                self._index(B)
                counts = self.exch.count_matrix_async(self._count_vec())
                ev = torch.cuda.Event()
                ev.record(side)
        finally:
            self._use_slot(cur)
        self._pf = (k, B, ev, batch, counts)

    def train_step(self, batch=None, graph=False, next_batch=None):
        sp = self.spec
        ex = self.exch
        E = sp.E
        pf = getattr(self, "_pf", None)
        counts = None
        if pf is not None and batch is not None and batch is pf[3]:
            self._pf = None
            self._use_slot(pf[0])
            torch.cuda.current_stream().wait_event(pf[2])
            B, counts = pf[1], pf[4]
        else:
            if pf is not None:   # a different batch came: drop the prefetch (after it lands)
                torch.cuda.current_stream().wait_event(pf[2])
                self._drop_prefetch(pf)
            B = self.stage(batch) if batch is not None else self.B
        s = _lib.stream_handle()
        L = self.layout
        L.batch = B
        W = self.world
        lazy = self.lazy
        self._mark("start")
        if lazy:
            if self.since_flush >= self.hist_len - 2:   # bound every row's lag below the alpha ring
                self.flush()
            self.since_flush += 1
        if counts is None:
            # 1. index + 2. counts: every rank's per-owner counts in one all-gather (host waits)
            self._index(B)
            cm = ex.count_matrix(self._count_vec())
        else:
            cm = ex.resolve_counts(counts)
        cm = self._split_counts(cm)   # raises on every rank if any rank's batch has a bad id
        # the step begins once every rank's ids are known to be valid
        call("dl_adam_begin_step", ptr(self.opt), sp.decay_rate, float(sp.decay_steps), s)
        if lazy:
            call("dl_adam_hist_record", ptr(self.opt), ptr(self.hist), self.hist_len, s)
        cmw = [row[W + 1:] for row in cm] if self.wdl else None
        self._mark("index_launched")
        send = cm[self.rank][:W]
        nsend, nrep = sum(send), cm[self.rank][W]
        U = nsend + nrep
        recv = [cm[r][self.rank] for r in range(W)]
        nrecv = sum(recv)
        self.last_counts = (nsend, nrep, nrecv)   # bench.py prices the per-kernel work with these
        self._mark("counts")
        recv_ids = ex.all_to_all(self.send_ids[:nsend], send, recv)
        self._mark("ids_a2a")
        # optimizer scalars of this step for the record update on the side stream (the next
        # step's adam_begin advances opt; two buffers: the update of step t-1 may still read one)
        snap = self.opt_snap[self.steps % 2]
        snap.copy_(self.opt)
        ids_ready = torch.cuda.Event()
        ids_ready.record()
        # 3. owners gather requested rows
        out_v = torch.empty(max(nrecv, 1), E, device=self.dev)
        out_1 = torch.empty(max(nrecv, 1), device=self.dev)
        if nrecv and lazy:   # rows caught up to the previous step (read only)
            if self.apply_done is not None:   # the previous step's record update (side stream)
                torch.cuda.current_stream().wait_event(self.apply_done)
            self._owner_buffers(nrecv)
            stash = self.owner_update == "sort"   # the update reads the caught-up state back
            self._c("rec_gather", "dl_rec_gather", C_ref(L), ptr(self.rec), self.rec_ld, self.rec_flags, 0,
                    ptr(recv_ids), None, nrecv, 1, ptr(self.hist), self.hist_len, ptr(self.opt), 1, ptr(out_v),
                    ptr(out_1) if sp.fm else None, ptr(self.own_mv) if stash else None, s)
            self.own_rows = (out_v, out_1)
        elif nrecv:
            call("dl_shard_gather", ptr(self.table), ptr(self.first), ptr(recv_ids), nrecv, E, ptr(out_v),
                 ptr(out_1) if self.first is not None else None, s)
        self._mark("gather")
        link_done = None
        if nrecv and lazy:
            # link this step's arrivals into per-row chains, for the update at the end of the
            # step: on the side stream, after the previous update reset the chain heads
            # (launched after the gather, so the host queues the critical path first)
            self._owner_buffers(nrecv)
            self._side_stream().wait_event(ids_ready)   # only the received ids, not the gather queued since
            with torch.cuda.stream(self.side):
                if self.owner_update == "chain":
                    call("dl_rec_chain_link", ptr(recv_ids), nrecv, ptr(self.own_head), ptr(self.own_next),
                         _lib.stream_handle(self.side))
                else:
                    call("dl_sort_unique", ptr(recv_ids), nrecv, self.own_bits, ptr(self.own_ws),
                         self.own_ws.numel(), ptr(self.own_keys), ptr(self.own_pos), ptr(self.own_uniq),
                         ptr(self.own_off), ptr(self.own_n), None, _lib.stream_handle(self.side))
                link_done = torch.cuda.Event()
                link_done.record(self.side)
            recv_ids.record_stream(self.side)
        self._mark("link")
        # 4. rows back, in unique-id order
        rep = self.rep
        ex.all_to_all(out_v[:nrecv], recv, send, out=self.rows_u[rep: rep + nsend])
        if sp.fm:
            ex.all_to_all(out_1[:nrecv], recv, send, out=self.rows_u1[rep: rep + nsend])
        if rep:
            self.rows_u[:rep].copy_(self.rep_t[:rep])
            if sp.fm:
                self.rows_u1[:rep].copy_(self.rep_f[:rep])
        if nrep:   # replicated rows referenced by cate ids: local rows of the replica
            call("dl_shard_gather", ptr(self.rep_t), ptr(self.rep_f) if sp.fm else None,
                 ptr(self.send_ids[nsend:U]), nrep, E, ptr(self.rows_u[rep + nsend:]),
                 ptr(self.rows_u1[rep + nsend:]) if sp.fm else None, s)
        wx = self._wide_exchange(B, cmw) if self.wdl else None
        self._mark("rows_a2a")
        if next_batch is not None:
            # after this step's row exchange is queued: the count all-gather it issues sits
            # behind it on RCCL's stream, and ahead of this step's gradient exchange
            self.prefetch(next_batch)
        replay = graph and self.prof is None
        slot = getattr(self, "_cur", 0)
        if replay:
            self._replay("graph_a%d" % slot, self._mid_a, B)
        else:
            self._mid_a(B)
        self._mark("mid_a")
        # embedding gradients to their owners, in flight while the weight gradients run
        gb, w_g = ex.all_to_all(self.gU[:nsend], send, recv, async_op=True)
        g1b, w_g1 = ex.all_to_all(self.g1U[:nsend], send, recv, async_op=True) if sp.fm else (None, None)
        if self.wdl:   # the exchanged wide rows' gradients (int64 fixed point) back to their owners
            off = self.wloc_off
            wg_in, w_gw = ex.all_to_all(self.wgloc[off: off + sum(wx[0])], wx[0], wx[1], async_op=True)
        if replay:
            self._replay("graph_b%d" % slot, self._mid_b, B)
        else:
            self._mid_b(B)
        self._mark("mid_b")
        side_apply = lazy and nrecv and self.prof is None
        if not side_apply:
            for w in (w_g, w_g1):
                if w is not None:
                    w.wait()
        nl = len(sp.hidden)
        hoff = self.seg[nl][1]
        if nrecv and not lazy:
            call("dl_shard_scatter_add", ptr(gb), ptr(g1b) if sp.fm else None, ptr(recv_ids), nrecv, E,
                 ptr(self.tg), ptr(self.fmg) if sp.fm else None, ptr(self.touched), s)
        # replicated rows: cate-id refs + the FM cont fields, into the flat buffer
        rg = self.flat[self.rep_off: self.rep_off + self.rep_g.numel()].view(-1, E)
        rg1 = self.flat[self.rep_off + self.rep_g.numel():]
        rg.zero_()
        rg1.zero_()
        tmp_touch = self.rep_touched.clone()
        if nrep:
            call("dl_shard_scatter_add", ptr(self.gU[nsend:U]), ptr(self.g1U[nsend:U]) if sp.fm else None,
                 ptr(self.send_ids[nsend:U]), nrep, E, ptr(rg), ptr(rg1) if sp.fm else None, ptr(tmp_touch), s)
        if rep and sp.fm:
            bwd_blocks = call_int("dl_embed_bwd_grid", C_ref(L))
            call("dl_embed_cont_bwd", C_ref(L), ptr(self.rows_u), ptr(self.in_cont), ptr(self.dz), ptr(self.w_head),
                 ptr(self.fm_sum), ptr(self.cont_slab), self.bwd_blocks, s)
            call("dl_embed_cont_reduce", C_ref(L), ptr(self.cont_slab), bwd_blocks, ptr(rg), ptr(rg1),
                 ptr(tmp_touch), s)
        # 7. one all-reduce of every replicated gradient
        self._mark("rep_grads")
        ex.all_reduce(self.flat)
        self._mark("all_reduce")
        # 8. TF1 Adam
        reg = sp.hidden_reg   # wdl: L2 on every hidden weight matrix (wdl.py:272-275), bias row excluded
        for l in range(nl):
            off, sz = self.seg[l][1], self.seg[l][2]
            l2, l2n = (sp.l2, ([self.D0] + sp.hidden)[l] * self.out_ld[l]) if reg else (0.0, 0)
            self._c("adam_dense_l%d" % l, "dl_adam_dense_reg", ptr(self.W[l]), ptr(self.Wm[l]), ptr(self.Wv[l]),
                    ptr(self.flat[off:]), 1, sz, sz, l2, l2n, 1 if reg == "l1" else 0, ptr(self.opt), None,
                    ptr(self.opt[8:]) if reg else None, s)
            self._refresh_wb(l, s)
        if self.wdl:
            H = sp.hidden[-1]
            self._c("adam_bias", "dl_adam_dense", ptr(self.wb), ptr(self.wbm), ptr(self.wbv), ptr(self.flat[hoff + H:]),
                    1, 1, 1, 0.0, 0, ptr(self.opt), None, None, s)
            # owners: arrived wide-row gradients + the deep-output rows they own, then the dense
            # L2 Adam sweep over the shard of wdl_weights (wdl.py:270-271)
            if w_gw is not None:
                w_gw.wait()
            nwrecv = sum(wx[1])
            call("dl_shard_add_fixed", ptr(wg_in), ptr(wx[2]), nwrecv, ptr(self.wg), ptr(self.w_touched), s)
            call("dl_wide_fold_owned", ptr(self.flat[hoff:]), H, sp.Fw, W, self.rank, ptr(self.wg),
                 ptr(self.w_touched), s)
            self.wide_reg.zero_()
            self._c("adam_wide", "dl_adam_rows", ptr(self.ww), ptr(self.wm), ptr(self.wv), ptr(self.wg),
                    ptr(self.w_touched), self.ww.shape[0], 1, sp.l2, 1 | _lib.ROWS_GRAD_FIXED, ptr(self.opt),
                    ptr(self.wide_reg), s)
            self._wide_refresh()
        else:
            self._c("adam_head", "dl_adam_dense", ptr(self.w_head), ptr(self.hm), ptr(self.hv), ptr(self.flat[hoff:]),
                    1, self.head_w, self.head_n, sp.l2, self.head_n - 1, ptr(self.opt), ptr(self.w_head_prev), None,
                    s)
        if rep:
            self.rep_g.view(-1)[: rg.numel()].copy_(rg.reshape(-1))
            self.rep_fg[: rg1.numel()].copy_(rg1)
            self.rep_touched[: self.rep] = 1
            call("dl_adam_rows", ptr(self.rep_t), ptr(self.rep_m), ptr(self.rep_v), ptr(self.rep_g),
                 ptr(self.rep_touched), self.rep_t.shape[0], E, 0.0, 0, ptr(self.opt), None, s)
            if sp.fm:
                call("dl_adam_rows", ptr(self.rep_f), ptr(self.rep_fm), ptr(self.rep_fv), ptr(self.rep_fg),
                     ptr(self.rep_touched), self.rep_f.shape[0], 1, 0.0, 0, ptr(self.opt), None, s)
        if lazy:
            if nrecv and self.prof is not None:   # bench's per-kernel pass: timed on the compute stream
                torch.cuda.current_stream().wait_event(link_done)
                self._c("rec_apply", *self._owner_apply_args(recv_ids, nrecv, gb, g1b, self.opt, s))
            elif nrecv:
                # on the side stream (after the chain link queued there): overlaps the next step's
                # start; that step's gather waits for it (apply_done).  The optimizer scalars
                # are snapshotted — the next adam_begin advances them.
                if ex.staged:   # host-staged exchange: the gradients were copied in on this stream
                    self.side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(self.side):
                    # the side stream waits for the arrived gradients themselves: the update
                    # starts as soon as they land, beside this step's weight gradients
                    for w in (w_g, w_g1):
                        if w is not None:
                            w.wait()
                    call(*self._owner_apply_args(recv_ids, nrecv, gb, g1b, snap, _lib.stream_handle(self.side)))
                    self.apply_done = torch.cuda.Event()
                    self.apply_done.record(self.side)
                gb.record_stream(self.side)
                if g1b is not None:
                    g1b.record_stream(self.side)
                out_v.record_stream(self.side)   # the update reads the gathered rows (stash form)
                out_1.record_stream(self.side)
        elif sp.fm:
            self._c("adam_table", "dl_adam_rows", ptr(self.table), ptr(self.tm), ptr(self.tv), ptr(self.tg),
                    ptr(self.touched), self.table.shape[0], E, 0.0, 0, ptr(self.opt), None, s)
            self._c("adam_first", "dl_adam_rows", ptr(self.first), ptr(self.fmm), ptr(self.fmv), ptr(self.fmg),
                    ptr(self.touched), self.first.shape[0], 1, 0.0, 1, ptr(self.opt), None, s)
        else:
            self._c("adam_table", "dl_adam_rows", ptr(self.table), ptr(self.tm), ptr(self.tv), ptr(self.tg),
                    ptr(self.touched), self.table.shape[0], E, 0.0, 1 | self.rows_sparse, ptr(self.opt), None, s)
        self._release()
        self._mark("end")
        self.steps += 1
        self.last_batch = B
        self.last_loss_sum = None
        return B

    # ------------------------------------------------------------ predict / eval
    def predict(self, batch, logits=False, device=False):
        """Forward only on this rank's batch (reference eval/predict, deepfm_pipeline.py:294-311):
        the same index, id exchange and owner gather as a training step, rows caught up to the
        last completed step (records are only read), no gradients, no update.  Every rank must
        call it together (collectives).  Returns the sigmoid scores [B] (or logits) as host
        numpy, or a device tensor copy with device=True."""
        sp = self.spec
        ex = self.exch
        E = sp.E
        pf = getattr(self, "_pf", None)
        if pf is not None:   # a pending prefetch: let it land, drop it
            torch.cuda.current_stream().wait_event(pf[2])
            self._drop_prefetch(pf)
        B = self.stage(batch)
        self._join_side()            # the last step's record update (side stream) has landed
        s = _lib.stream_handle()
        L = self.layout
        L.batch = B
        W = self.world
        self._index(B)
        cm = self._split_counts(ex.count_matrix(self._count_vec()))
        cmw = [row[W + 1:] for row in cm] if self.wdl else None
        send = cm[self.rank][:W]
        nsend, nrep = sum(send), cm[self.rank][W]
        recv = [cm[r][self.rank] for r in range(W)]
        nrecv = sum(recv)
        recv_ids = ex.all_to_all(self.send_ids[:nsend], send, recv)
        out_v = torch.empty(max(nrecv, 1), E, device=self.dev)
        out_1 = torch.empty(max(nrecv, 1), device=self.dev)
        if nrecv and self.lazy:   # lag 0: caught up to the last completed step, read only
            call("dl_rec_gather", C_ref(L), ptr(self.rec), self.rec_ld, self.rec_flags, 0, ptr(recv_ids), None,
                 nrecv, 1, ptr(self.hist), self.hist_len, ptr(self.opt), 0, ptr(out_v),
                 ptr(out_1) if sp.fm else None, None, s)
        elif nrecv:
            call("dl_shard_gather", ptr(self.table), ptr(self.first), ptr(recv_ids), nrecv, E, ptr(out_v),
                 ptr(out_1) if self.first is not None else None, s)
        rep = self.rep
        ex.all_to_all(out_v[:nrecv], recv, send, out=self.rows_u[rep: rep + nsend])
        if sp.fm:
            ex.all_to_all(out_1[:nrecv], recv, send, out=self.rows_u1[rep: rep + nsend])
        if rep:
            self.rows_u[:rep].copy_(self.rep_t[:rep])
            if sp.fm:
                self.rows_u1[:rep].copy_(self.rep_f[:rep])
        if nrep:
            call("dl_shard_gather", ptr(self.rep_t), ptr(self.rep_f) if sp.fm else None,
                 ptr(self.send_ids[nsend:nsend + nrep]), nrep, E, ptr(self.rows_u[rep + nsend:]),
                 ptr(self.rows_u1[rep + nsend:]) if sp.fm else None, s)
        if self.wdl:
            self._wide_exchange(B, cmw)
        call("dl_embed_fwd_indexed", C_ref(L), ptr(self.rows_u), ptr(self.rows_u1) if sp.fm else None, ptr(self.inv),
             rep, ptr(self.in_cont), ptr(self.in_vec), ptr(self.x0b if self.x0_direct else self.x0), ptr(self.fm_out),
             ptr(self.fm_sum), s)
        if self.bf and not self.x0_direct:
            call("dl_cast_bf16", ptr(self.x0), B, self.in_ld[0], self.in_ld[0], ptr(self.x0b), self.in_ld[0], s)
        self._tower_fwd(B, s)
        self._head(B, s, train=False)
        self._release()
        self.check_error()
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
        sp = self.spec
        hoff = self.seg[len(sp.hidden)][1]
        if self.wdl:
            H = sp.hidden[-1]
            data = float(self.flat[hoff + H + 1].item())
            wr = self.wide_reg.clone()
            self.exch.all_reduce(wr)
            return data / (self.last_batch * self.world) + sp.l2 * 0.5 * (float(self.opt[8].item()) +
                                                                           float(wr[0].item()))
        data = float(self.flat[hoff + self.head_w - 1].item())
        w = self.w_head_prev[: self.head_n - 1].double()
        return data / (self.last_batch * self.world) + sp.l2 * 0.5 * float((w * w).sum().item())
