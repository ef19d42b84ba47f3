"""Throughput of the native TFRecord reader (libdlio.so) on C2-shaped records
(13 cont + 26 cate + label), as records/s per decoder thread count.
Usage: python scripts/reader_bench.py [n_records] [dir]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from deep_learning_amd.synthetic import make_batch  # noqa: E402
from deep_learning_amd.utils import data_loader  # noqa: E402
from deep_learning_amd.utils.native_reader import NativeReader  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
d = sys.argv[2] if len(sys.argv) > 2 else "/tmp/dlio_bench"
os.makedirs(d, exist_ok=True)
per = 65536
files = []
for i in range(n // per):
    f = os.path.join(d, "part-%05d" % i)
    if not os.path.exists(f):
        data_loader.write_tfrecord_part(f, make_batch(per, cate_index_size=26_000_000, seed=i))
    files.append(f)
mb = sum(os.path.getsize(f) for f in files) / 1e6
spec = [("label", "float", 1), ("cont_feats", "float", 13), ("vector_feats", "float", 0), ("cate_feats", "int64", 26)]
for th in (1, 2, 4, 8, 16):
    for shuffle in (0, 1):
        t = time.perf_counter()
        nb = 0
        for b in NativeReader(files, spec, 65536, repeat=2, shuffle_buf=655360 if shuffle else 0, seed=1, threads=th):
            nb += 1
        dt = time.perf_counter() - t
        print("threads=%2d shuffle=%d  %.2f M records/s  %.0f MB/s  (%d batches of 65536, %.1f MB x 2 epochs)"
              % (th, shuffle, nb * 65536 / dt / 1e6, 2 * mb / dt, nb, mb), flush=True)
