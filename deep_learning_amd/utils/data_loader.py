"""TFRecord batch iterator with the reference loader's contract
(utils/data_loader.py:7-58).

    data = load_input_file(mp, input_path, action_type)   # 'train' repeats mp.epochs times
    for batch in data: ...   # dict: label [B,1] f32, cont_feats [B,C] f32 (non-cate algs),
                             #       vector_feats [B,V] f32, cate_feats [B,S+M] int64

Semantics kept from the reference:
  * files = entries of `input_path` whose name starts with "part", path = input_path + name
    (string concatenation, so a trailing slash is required), in directory-listing order;
  * FixedLenFeature: every record must carry exactly the configured sizes, else ValueError
    (TF raises InvalidArgumentError);
  * cate algorithms (deepfm_cate, dnn_cate, dnn_multi_cate, deepfm_multi_cate) parse no
    cont_feats;
  * shuffle buffer of batch_size*10 records, batch(drop_remainder=True), repeat(epochs) for 'train'.
Differences: end of data is StopIteration (the reference raises tf.errors.OutOfRangeError);
the iterator is re-iterable (each `iter()` starts over, like a fresh tf.Session); the
shuffle is seeded by ``mp.shuffle_seed`` (None = unseeded like the reference) and can be
disabled with ``mp.shuffle = 0`` so parity runs see identical batches.
The reading itself is native (``NativeReader`` over libdlio.so, include/dlio.h).
"""
import os

import numpy as np

from . import tfrecord
from .native_reader import DeviceBatches, NativeReader

CATE_ALGS = ("deepfm_cate", "dnn_cate", "dnn_multi_cate", "deepfm_multi_cate")


def _spec(mp):
    if mp.alg_name in CATE_ALGS:
        print("-----------tf_cate-----------")
        return {"cate_feats": ("int64", mp.cate_field_size + mp.multi_feats_size),
                "label": ("float", 1), "vector_feats": ("float", mp.vector_feats_size)}
    print("-----------tf_pipeline-----------")
    return {"label": ("float", 1), "cont_feats": ("float", mp.cont_field_size),
            "vector_feats": ("float", mp.vector_feats_size),
            "cate_feats": ("int64", mp.cate_field_size + mp.multi_feats_size)}


def parse_example(data, spec):
    ex = tfrecord.decode_example(data)
    out = {}
    for key, (kind, size) in spec.items():
        k, vals = ex.get(key, (kind, []))
        if len(vals) != size:
            raise ValueError("Key: %s. Can't parse serialized Example: expected %d values, got %d"
                             % (key, size, len(vals)))
        out[key] = vals
    return out


class BatchStream:
    """Re-iterable stream of batches (dicts of numpy arrays; with ``device`` set — or
    ``mp.device_batches`` — dicts of device tensors with the same keys, dtypes and shapes,
    uploaded one batch ahead through pinned buffers: DeviceBatches).  Each ``iter()`` opens
    the native reader (libdlio.so: framing + CRC-32C, shuffle buffer, FixedLenFeature parse on
    ``threads`` C++ threads — num_parallel_calls=10 at data_loader.py:31 — and batching)."""

    def __init__(self, mp, files, action_type, threads=10, depth=4, device=None):
        self.mp = mp
        self.files = list(files)
        self.repeat = int(mp.epochs) if action_type == "train" else 1
        self.spec = _spec(mp)
        self.bsz = int(mp.batch_size)
        self.shuffle = int(getattr(mp, "shuffle", 1))
        self.seed = getattr(mp, "shuffle_seed", None)
        self.threads = int(getattr(mp, "reader_threads", threads))
        self.depth = depth
        self.device = device if device is not None else getattr(mp, "device_batches", None)

    def __iter__(self):
        spec = [(k, kind, size) for k, (kind, size) in self.spec.items()]
        r = NativeReader(self.files, spec, self.bsz, repeat=self.repeat,
                         shuffle_buf=self.bsz * 10 if self.shuffle else 0,   # shuffle(bsz*10), :34
                         seed=self.seed, threads=self.threads, depth=self.depth)
        return DeviceBatches(r, self.device, self.depth) if self.device else r


def get_file_list(input_path):
    files = os.listdir(input_path)
    print("file_list_len:", len(files))
    return [input_path + f for f in files if f[:4] == "part"]


def pipeline_process(mp, file_dir_list, action_type, device=None):
    return BatchStream(mp, file_dir_list, action_type, device=device)


def load_input_file(mp, input_path, action_type, device=None):
    """device="cuda": batches as device tensors (the reference's get_next() tensors,
    data_loader.py:43-46); default host numpy batches (the model stages them itself)."""
    return pipeline_process(mp, get_file_list(input_path), action_type, device=device)


def write_tfrecord_part(path, batch):
    """Writes a batch dict (reference keys) as one TFRecord part file (test/fixture helper)."""
    n = batch["label"].shape[0]
    recs = []
    for i in range(n):
        feats = {"label": ("float", batch["label"][i].reshape(-1).tolist()),
                 "cate_feats": ("int64", batch["cate_feats"][i].reshape(-1).tolist()),
                 "vector_feats": ("float", batch.get("vector_feats", np.zeros((n, 0)))[i].reshape(-1).tolist())}
        if "cont_feats" in batch:
            feats["cont_feats"] = ("float", batch["cont_feats"][i].reshape(-1).tolist())
        recs.append(tfrecord.encode_example(feats))
    tfrecord.write_records(path, recs)
