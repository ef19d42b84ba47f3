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


def crc32c(data):
    b = bytes(data)
    return lib().dlio_crc32c(b, len(b))


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
        if self.h is None:
            raise StopIteration
        out = {n: np.empty((self.batch, s), np.int64 if k == "int64" else np.float32) for n, k, s in self.spec}
        ptrs = (C.c_void_p * len(self.spec))(*[out[n].ctypes.data for n, _, _ in self.spec])
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
