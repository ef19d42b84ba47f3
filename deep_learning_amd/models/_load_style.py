"""Shared implementation of the reference's load-style model surface (models/wdl.py,
models/deepfm.py, models/dnn.py): the models that train from lists of pickled batch
dicts (utils/data_loader_load.py:61-139) instead of the TFRecord iterator.

    DeepModel(args)                      (deepfm.py:15-37, dnn.py:15-33, wdl.py:19-51)
    .model_optimizer()                   (deepfm.py:146-162; dnn.py builds it in __init_graph)
    .fit(train_data, val_data)           (deepfm.py:164-214, dnn.py:98-145, wdl.py:287-341)
    .evaluate(sess, data_val) -> auc     (deepfm.py:216-232, dnn.py:147-161, wdl.py:343-358)
    .predict(data_val)                   (deepfm.py:234-255, dnn.py:163-185, wdl.py:360-384)

Per epoch the reference prints '[%s] valid-%s=%.5f\tloss=%.5f [%.1f s]' with the loss
averaged over the epoch's batches (each weighted by batch_size), then exports the model;
predict prints 'val of auc:%.5f'.  The engine runs the step as one hipGraph replay for
full batches.
"""
import concurrent.futures as cf
import os
import pickle
import sys
import threading
import time

import numpy as np
import torch

from ..engine import CTREngine, default_adam
from ..metrics import AucAccumulator
from ._ctr_model import _predict_batches, export_model, load_model


def unpickle(item):
    return pickle.loads(item) if isinstance(item, (bytes, bytearray)) else item


class PinnedFeed:
    """The load-style batches (pickled dicts, wdl.py:296) decoded on worker threads into a ring
    of pinned host buffers, in order, ahead of the training loop: libdlio's pickle decoder
    (dlio_unpickle_batch) writes each field straight into its pinned buffer with the GIL released
    (pickle.loads + a copy under the GIL for forms it does not take), and the engine stages each
    batch with an asynchronous host-to-device copy on its side stream (engine._copy_in) instead
    of the loop unpickling and copying 31 MB of pageable memory a C5 batch between steps.  A ring
    slot is refilled only after the step that consumed it has run (release(): an event on the
    compute stream after that step)."""

    def __init__(self, model, items, workers=None, depth=None):
        self.model = model
        self.items = iter(items)
        # one decoding worker (its copies on libdlio's own thread team), three slots: on two boxes
        # 1.79-1.88 ms a 24-batch C5 epoch step against 1.88-2.09 ms with two workers and four
        # slots — concurrent decodes slow each other down (0.5 -> 1.0-1.5 ms a batch; profiles/r05bk/)
        self.workers = workers or int(os.environ.get("DLAMD_FEED_WORKERS", "1"))
        self.depth = depth or int(os.environ.get("DLAMD_FEED_DEPTH", "0")) or self.workers + 2
        # the ring's pinned buffers (and each slot's last-use event) are the model's, kept across
        # epochs: pinning 124 MB afresh made each C5 epoch start 18-22 ms late (profiles/r05bi/)
        st = getattr(model, "_feed_ring", None)
        if st is None:
            st = model._feed_ring = ([], [])
        while len(st[0]) < self.depth:
            st[0].append(dict())
            st[1].append(None)
        self.bufs, self.events = st
        self.free = [threading.Event() for _ in range(self.depth)]
        for f in self.free:
            f.set()
        self.pool = cf.ThreadPoolExecutor(max_workers=self.workers)
        self.pending = []
        self.k = 0
        self.lock = threading.Lock()
        self.done = False
        self.aborted = False
        for _ in range(self.depth):
            self._submit()

    def _submit(self):
        with self.lock:
            if self.done:
                return
            item = next(self.items, None)
            if item is None:
                self.done = True
                return
            k = self.k
            self.k += 1
        self.pending.append(self.pool.submit(self._prepare, k, item))

    def _native(self, s, item):
        """The batch decoded by libdlio's pickle decoder straight into slot s's pinned buffers
        (GIL released, one host copy); None when the pickle is not a form it takes."""
        from ..utils.native_reader import unpickle_batch_into
        fields = self.model.native_fields()
        if fields is None or not isinstance(item, bytes):
            return None
        cap = self.model.batch_size
        outs = []
        for key, out_key, kind, size in fields:
            dt = torch.float32 if kind == 0 else torch.int64
            buf = self.bufs[s].get(out_key)
            if buf is None or buf.numel() < cap * size or buf.dtype != dt:
                buf = self.bufs[s][out_key] = torch.empty(max(cap * size, 1), dtype=dt).pin_memory()
            outs.append(buf)
        rows = unpickle_batch_into(item, [(key, kind, size) for key, _, kind, size in fields], outs, cap)
        if rows is None:
            return None
        out = {out_key: buf[: rows * size].view(rows, size) for (_, out_key, _, size), buf in zip(fields, outs)}
        out.update(self.model.native_extra(rows))
        return out

    def _prepare(self, k, item):
        s = k % self.depth
        self.free[s].wait()       # the slot's previous batch has been released (one claimant a slot:
        if self.aborted:          # batch k + depth is submitted only once batch k was taken), or the
            return None           # loop stopped on an exception (close(abort=True) sets every slot)
        self.free[s].clear()
        ev = self.events[s]
        if ev is not None:
            ev.synchronize()
        out = self._native(s, item)
        if out is not None:
            out["_slot"] = s
            return out
        d = self.model.batch(item)
        out = {}
        for key, a in d.items():
            a = np.ascontiguousarray(a)
            buf = self.bufs[s].get(key)
            if buf is None or buf.numel() < a.size or buf.dtype != torch.from_numpy(a[:0]).dtype:
                buf = self.bufs[s][key] = torch.empty(a.size, dtype=torch.from_numpy(a[:0]).dtype).pin_memory()
            v = buf[: a.size].view(a.shape)
            v.copy_(torch.from_numpy(a))
            out[key] = v
        out["_slot"] = s
        return out

    def __iter__(self):
        while self.pending:
            fut = self.pending.pop(0)
            b = fut.result()
            self._submit()
            yield b

    def release(self, b):
        """b's step has been submitted: its slot may be refilled once the compute stream is past it."""
        s = b["_slot"]
        ev = torch.cuda.Event()
        ev.record()
        self.events[s] = ev
        self.free[s].set()

    def close(self, abort=False):
        """Wait for the workers.  abort (the loop stopped on an exception — a bad-id DLError, an
        interrupt — with batches still held): every slot is released and the queued decodes are
        dropped first, so a worker waiting for a slot the loop will never release returns at
        once instead of hanging the shutdown."""
        if abort:
            with self.lock:
                self.aborted = self.done = True
            for f in self.free:
                f.set()
        self.pool.shutdown(wait=True, cancel_futures=abort)


class LoadStyleModel:
    # evaluate() scores: "score" (sigmoid) or "logit" (deepfm.py:229 evaluates the
    # pre-sigmoid self.out)
    EVAL_OUTPUT = "score"

    def __init__(self, args):
        self.hidden_units = [int(h) for h in args.hidden_units]
        self.epochs = int(args.epochs)
        self.batch_size = int(args.batch_size)
        self.learning_rate = args.learning_rate
        self.model_pb = args.model_pb
        self.l2_reg = args.l2_reg
        self.metric_type = "auc"
        self.random_seed = 2019
        self.spec = self.make_spec(args)
        self.engine = None

    def make_spec(self, args):
        raise NotImplementedError

    def native_fields(self):
        """(pickle key, batch key, 0 float32 / 1 int64, values per row) of the fields batch()
        reads, for libdlio's pickle decoder (PinnedFeed); None: always unpickle in Python."""
        return None

    def native_extra(self, rows):
        """Batch entries the decoder does not fill (empty fields)."""
        return {}

    def batch(self, item):
        """One pickled batch dict (data_loader_load.py:128-135 keys) -> engine batch."""
        raise NotImplementedError

    def model_optimizer(self):
        if self.engine is None:
            self.engine = CTREngine(self.spec, max_batch=self.batch_size, seed=self.random_seed,
                                    adam=default_adam(self.spec))
        return self.engine

    def train_epoch(self, train_data):
        """One pass over the pickled batches: sess.run([loss, optimizer]) per batch (wdl.py:
        305-309).  The step's loss is summed on the device (no host read per step, no wide-table
        flush) and read once at the end; the next batch is unpickled, staged and indexed while
        the current step runs.  Returns (sum of the per-step losses, steps)."""
        eng = self.model_optimizer()
        eng.loss_sum_begin()
        steps = 0
        if os.environ.get("DLAMD_PINNED_FEED", "1") == "0":
            # DLAMD_PINNED_FEED=0: the next batch unpickled (pickle.loads) and staged (pageable
            # host-to-device) on this thread while the current step runs.  The default is the
            # PinnedFeed below: worker threads decode each pickled batch with libdlio's decoder
            # (no GIL, one host copy) straight into pinned buffers (profiles/r05au/)
            items = iter(train_data)
            b = next(items, None)
            b = self.batch(b) if b is not None else None
            while b is not None:
                nxt = next(items, None)
                nxt = self.batch(nxt) if nxt is not None else None
                eng.train_step(b, graph=b["label"].shape[0] == eng.B, **({"next_batch": nxt} if nxt is not None else {}))
                steps += 1
                b = nxt
            loss_sum, counted = eng.loss_sum_end()
            if counted != steps:
                eng.check_error()
            return loss_sum, steps
        feed = PinnedFeed(self, train_data)
        ok = False
        try:
            items = iter(feed)
            b = next(items, None)
            while b is not None:
                nxt = next(items, None)
                eng.train_step(b, graph=b["label"].shape[0] == eng.B, **({"next_batch": nxt} if nxt is not None else {}))
                feed.release(b)
                steps += 1
                b = nxt
            ok = True
        finally:
            feed.close(abort=not ok)
        loss_sum, counted = eng.loss_sum_end()
        if counted != steps:
            eng.check_error()   # a skipped (bad) batch raises here, as its sess.run did
        return loss_sum, steps

    def fit(self, train_data, val_data):
        eng = self.model_optimizer()
        losses = []
        num_samples = 0
        for epoch in range(self.epochs):
            st = time.time()
            # the epoch's mean is the reference's sum(loss_t * batch_size) / num_samples
            # (num_samples counts batch_size per batch, the last partial batch included)
            loss_sum, steps = self.train_epoch(train_data)
            num_samples += self.batch_size * steps
            losses.append(loss_sum * self.batch_size)
            end_time = time.time()
            total_loss = float(np.sum(losses) / num_samples)
            valid_metric = self.evaluate(None, val_data)
            print('[%s] valid-%s=%.5f\tloss=%.5f [%.1f s]' % (epoch + 1, self.metric_type, valid_metric,
                                                               total_loss, end_time - st))
            sys.stdout.flush()
        eng.check_error()
        try:
            export_model(eng, self.model_pb)
        except Exception as e:
            print("Fail to export saved model, exception: {}".format(e))
            sys.stdout.flush()

    def evaluate(self, sess, data_val):
        eng = self.model_optimizer()
        acc = AucAccumulator()
        for item in data_val:
            b = self.batch(item)
            acc.add(b["label"], _predict_batches(eng, b, logits=self.EVAL_OUTPUT == "logit"))
        return acc.result()

    def predict(self, data_val):
        eng = load_model(self.model_pb, max_batch=self.batch_size)
        acc = AucAccumulator()
        for item in data_val:
            b = self.batch(item)
            acc.add(b["label"], _predict_batches(eng, b))
        auc = acc.result()
        print("val of auc:%.5f" % auc)
        sys.stdout.flush()
        print('---end---')
        return auc
