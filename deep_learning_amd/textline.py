"""The multi-hot lookup of the textline DNN (models/dnn_multi_textline.py:69-103) on the device.

Every multi-hot slot is pooled as ``div_no_nan(sum_l value_l * V[id_l], count_nonzero(sum_E
V[id_l]))`` (:94-103) from the trainable table ``weight_mat`` with its row 0 zeroed (:37-42),
except the slot named ``tag``, which reads the frozen word2vec table (``tf.constant``,
:45-47,85-88: looked up directly, so no zero row, and no gradient).  The textline ingestion
itself is out of scope; this is the kernel-level surface of that forward and
backward: each run of consecutive slots on one table is one ``dl_pool_fwd_weighted`` /
``dl_pool_bwd_weighted`` call writing its pooled vectors at that run's columns.
"""
import ctypes

import torch

from . import _lib
from ._lib import call, ptr


class TextlinePooling:
    """ranges: [[start, end, name], ...] of the multi block (my_utils.get_mul_index_range);
    E: embedding size; n_rows: rows of the trainable table; w2v: the word2vec table [Nw, E]
    (device f32), read by the slot named 'tag' only."""

    def __init__(self, ranges, E, n_rows, w2v=None):
        self.ranges = [list(r) for r in ranges]
        self.E, self.n_rows = E, n_rows
        self.w2v = w2v
        if any(r[2] == "tag" for r in self.ranges) and w2v is None:
            raise ValueError("slot 'tag' needs the word2vec table")
        # runs of consecutive slots on the same table: (first slot, count, is_tag)
        self.runs = []
        for m, r in enumerate(self.ranges):
            tag = r[2] == "tag"
            if self.runs and self.runs[-1][2] == tag:
                self.runs[-1][1] += 1
            else:
                self.runs.append([m, 1, tag])
        dev = "cuda"
        self.s0 = torch.tensor([r[0] for r in self.ranges], dtype=torch.int32, device=dev)
        self.s1 = torch.tensor([r[1] for r in self.ranges], dtype=torch.int32, device=dev)

    def _layout(self, B, ids_ld, tag, out_ld, col):
        L = _lib.EmbLayout()
        L.n_rows = self.w2v.shape[0] if tag else self.n_rows
        L.batch = B
        L.emb_dim = self.E
        L.cate_fields = 0
        L.cate_ld = ids_ld
        L.use_fm = 0
        L.zero_row0 = 0 if tag else 1          # the constant table has no zero row
        L.x0_ld = out_ld
        L.x0_pool_col = col
        L.dx0_ld = out_ld
        return L

    def forward(self, table, ids, values):
        """table [n_rows, E] f32, ids [B, W] int64 (the multi block), values [B, W] f32 ->
        (pooled [B, M*E] f32, counts [B, M] f32), on the device."""
        B, W = ids.shape
        M, E = len(self.ranges), self.E
        out = torch.zeros(B, M * E, device="cuda")
        cnt = torch.zeros(B, M, device="cuda")
        err = torch.zeros(4, dtype=torch.int32, device="cuda")
        s = _lib.stream_handle()
        for m0, k, tag in self.runs:
            L = self._layout(B, W, tag, M * E, m0 * E)
            c = torch.empty(B, k, device="cuda")
            call("dl_pool_fwd_weighted", ctypes.byref(L), ptr(self.w2v if tag else table), ptr(ids), 0, ptr(values),
                 W, ptr(self.s0[m0:]), ptr(self.s1[m0:]), k, ptr(out), ptr(c), ptr(err), s)
            cnt[:, m0:m0 + k] = c
        if int(err[0].item()):
            raise _lib.DLError("InvalidArgumentError: multi-hot id out of range")
        self._last = (B, W, cnt)
        return out, cnt

    def backward(self, d_pooled, ids, values, g_table, touched):
        """d_pooled [B, M*E]: adds the trainable table's gradient into g_table [n_rows, E]
        (marks touched); the 'tag' slot's frozen table gets none."""
        B, W, cnt = self._last
        M, E = len(self.ranges), self.E
        s = _lib.stream_handle()
        for m0, k, tag in self.runs:
            if tag:
                continue
            L = self._layout(B, W, False, M * E, m0 * E)
            c = cnt[:, m0:m0 + k].contiguous()
            call("dl_pool_bwd_weighted", ctypes.byref(L), ptr(ids), 0, ptr(values), W, ptr(self.s0[m0:]),
                 ptr(self.s1[m0:]), k, ptr(d_pooled), m0 * E, ptr(c), ptr(g_table), ptr(touched), s)
