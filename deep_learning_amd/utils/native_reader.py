"""ctypes binding of the native TFRecord batch reader (``libdlio.so``, include/dlio.h).

The reader replaces the reference's tf.data input pipeline (utils/data_loader.py:29-40):
the records are framed, CRC-checked, shuffled, parsed against the FixedLenFeature spec
and batched in C++ threads; Python only receives finished batches as numpy arrays.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(HERE, "libdlio.so")

FLOAT, INT64 = 0, 1


class _Feature(C.Structure):
    _fields_ = [("name", C.c_char_p), ("kind", C.c_int32), ("size", C.c_int32)]


SIGNATURES = {
    "dlio_open": (C.c_void_p, [C.POINTER(C.c_char_p), C.c_int32, C.POINTER(_Feature), C.c_int32, C.c_int32,
                               C.c_int32, C.c_int64, C.c_int64, C.c_int32, C.c_int32]),
    "dlio_next": (C.c_int32, [C.c_void_p, C.POINTER(C.c_void_p)]),
    "dlio_records": (C.c_int64, [C.c_void_p]),
    "dlio_last_error": (C.c_char_p, [C.c_void_p]),
    "dlio_open_error": (C.c_char_p, []),
    "dlio_close": (None, [C.c_void_p]),
    "dlio_unpickle_batch": (C.c_int32, [C.c_char_p, C.c_int64, C.POINTER(_Feature), C.c_int32, C.c_int64,
                                        C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]),
    "dlio_crc32c": (C.c_uint32, [C.c_void_p, C.c_int64]),
    "dlio_masked_crc32c": (C.c_uint32, [C.c_void_p, C.c_int64]),
}

_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise OSError("libdlio.so not found at %s — build it with `python -m deep_learning_amd.build`"
                          % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def unpickle_batch_into(item, fields, outs, cap_rows):
    """Decode one pickled load-style batch (a dict of arrays or lists of rows,
    utils/data_loader_load.py:128-136) straight into `outs` (C-contiguous numpy arrays or CPU
    tensors, e.g. pinned, room for cap_rows rows each) without building Python objects — the
    native decoder runs with the GIL released.  fields: (key, FLOAT | INT64, values per row).
    Returns the batch's rows, or None when the pickle is not a form the decoder takes (the
    caller unpickles it in Python then; malformed data raises there, as pickle.loads does)."""
    if not isinstance(item, bytes):
        return None
    feats = (_Feature * len(fields))(*[_Feature(k.encode(), kind, size) for k, kind, size in fields])
    ptrs = (C.c_void_p * len(outs))(*[o.data_ptr() if hasattr(o, "data_ptr") else o.ctypes.data for o in outs])
    rows = C.c_int64(0)
    rc = lib().dlio_unpickle_batch(item, len(item), feats, len(fields), int(cap_rows), ptrs, C.byref(rows))
    return int(rows.value) if rc == 0 else None


def crc32c(data):
    b = bytes(data)
    return lib().dlio_crc32c(b, len(b))


class PinnedFeed:
    """Host-to-device double buffering for a NativeReader: the reader's
    decoder threads write each batch straight into one of `depth` pinned host buffer sets,
    so the engine's staging copy (CTREngine.stage / prefetch, non_blocking) is an async DMA
    that overlaps the running step.  A set is reused only after the event recorded behind
    its copy has completed (`mark`)."""

    def __init__(self, reader, depth=4):
        import torch
        self.reader, self.depth, self.n = reader, depth, 0
        self.sets = [{name: torch.empty((reader.batch, max(sz, 0)), dtype=torch.int64 if k == "int64" else torch.float32,
                                        pin_memory=True) for name, k, sz in reader.spec} for _ in range(depth)]
        self.events = [None] * depth

    def next(self):
        """The next batch as a dict of pinned CPU tensors (None at the end of the data)."""
        k = self.n % self.depth
        if self.events[k] is not None:
            self.events[k].synchronize()        # its previous batch's copy has landed
            self.events[k] = None
        try:
            b = self.reader.next_into(self.sets[k])
        except StopIteration:
            return None
        self.n += 1
        b = dict(b)
        b["_slot"] = k
        return b

    def mark(self, batch, event):
        """`event` completes after every read of `batch`'s host buffers."""
        if batch is not None:
            self.events[batch["_slot"]] = event


class DeviceBatches:
    """Iterator of batches as DEVICE tensors (the reference's loader hands its graph
    `get_next()` tensors, utils/data_loader.py:29-46): the native reader decodes into pinned
    host buffers (PinnedFeed), each batch is uploaded on a copy stream of its own one batch
    ahead of the consumer, and a yielded batch is ordered after its upload on the consumer's
    current stream (keys, dtypes and shapes as the host batches: label [B,1] f32, cont_feats
    [B,C] f32, vector_feats [B,V] f32, cate_feats [B,S+M] int64)."""

    def __init__(self, reader, device="cuda", depth=4):
        import torch
        self.torch = torch
        self.device = torch.device(device)
        self.feed = PinnedFeed(reader, depth)
        self.stream = torch.cuda.Stream(self.device)
        self.pending = self._upload(self.feed.next())

    def _upload(self, hb):
        if hb is None:
            return None
        torch = self.torch
        with torch.cuda.stream(self.stream):
            d = {k: v.to(self.device, non_blocking=True) for k, v in hb.items() if k != "_slot"}
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self.feed.mark(hb, ev)          # the pinned set is reused once this copy has landed
        return d, ev

    def __iter__(self):
        return self

    def __next__(self):
        if self.pending is None:
            raise StopIteration
        d, ev = self.pending
        self.pending = self._upload(self.feed.next())   # the next upload overlaps this batch's use
        cur = self.torch.cuda.current_stream(self.device)
        cur.wait_event(ev)
        for t in d.values():
            t.record_stream(cur)        # allocated on the copy stream, used on the consumer's
        return d


class NativeReader:
    """Iterator of batches: dict name -> array [batch, size] (float32 / int64).

    spec: list of (name, 'float'|'int64', size); shuffle_buf <= 0 keeps file order;
    seed None = OS-seeded (the reference's shuffle is unseeded)."""

    def __init__(self, files, spec, batch, repeat=1, shuffle_buf=0, seed=None, threads=10, depth=4):
        self.spec = [(n, k, int(s)) for n, k, s in spec]
        self.batch = int(batch)
        L = lib()
        names = [f.encode() for f in files]
        farr = (C.c_char_p * max(1, len(names)))(*names)
        self._keep = [n.encode() for n, _, _ in self.spec]
        feats = (_Feature * len(self.spec))(*[
            _Feature(self._keep[i], INT64 if k == "int64" else FLOAT, s) for i, (_, k, s) in enumerate(self.spec)])
        self.h = L.dlio_open(farr, len(names), feats, len(self.spec), self.batch, int(repeat), int(shuffle_buf),
                             -1 if seed is None else int(seed), int(threads), int(depth))
        if not self.h:
            raise IOError(L.dlio_open_error().decode())

    def __iter__(self):
        return self

    def __next__(self):
        return self.next_into(None)

    def next_into(self, out):
        """Next batch into `out` (dict name -> preallocated contiguous host buffers with a
        ``data_ptr()`` or numpy ``ctypes.data``, e.g. pinned torch tensors) or fresh arrays."""
        if self.h is None:
            raise StopIteration
        if out is None:
            out = {n: np.empty((self.batch, s), np.int64 if k == "int64" else np.float32) for n, k, s in self.spec}
        addr = lambda a: a.data_ptr() if hasattr(a, "data_ptr") else a.ctypes.data
        ptrs = (C.c_void_p * len(self.spec))(*[addr(out[n]) for n, _, _ in self.spec])
        rc = lib().dlio_next(self.h, ptrs)
        if rc == 1:
            return out
        if rc == 0:
            self.close()
            raise StopIteration
        msg = lib().dlio_last_error(self.h).decode()
        self.close()
        raise ValueError(msg) if msg.startswith("Key:") or msg.startswith("malformed") else IOError(msg)

    def records(self):
        return lib().dlio_records(self.h) if self.h else 0

    def close(self):
        if self.h is not None:
            lib().dlio_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
