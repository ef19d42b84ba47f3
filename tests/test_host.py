"""CPU tests of the host-side mirror of the reference interface: my_utils against
goldens captured from the reference's own utils/my_utils.py, the TFRecord codec
(CRC-32C known answers), the batch iterator, AUC against sklearn goldens, and the
oracle against its committed fixtures."""
import json
import os
import struct
import tempfile

import numpy as np
import pytest

from deep_learning_amd.synthetic import make_batch
from deep_learning_amd.utils import data_loader, my_utils, tfrecord

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


# ------------------------------------------------------------------ my_utils
def test_feat_size_matches_reference_goldens():
    d = json.load(open(os.path.join(GOLD, "my_utils_golden.json")))
    for case in d["feat_size"]:
        with tempfile.TemporaryDirectory() as tmp:
            with open(os.path.join(tmp, "dnn.conf"), "w") as f:
                f.write("\n".join(case["lines"]) + "\n")
            with open(os.path.join(tmp, "ignored.conf"), "w") as f:
                f.write("zz\tx\tfloat\n")
            got = list(my_utils.feat_size(tmp, case["alg"]))
        exp = case["result"]
        if case["alg"] in ("deepfm_multi_cate", "dnn_multi_cate"):
            # documented deviation: the reference misspells these in its pooling list
            # (utils/my_utils.py:27) and then crashes (deepfm_multi_cate.py:136); the
            # intended pooling behaviour equals its *_multi algorithms'.
            twin = [c for c in d["feat_size"] if c["conf"] == case["conf"]
                    and c["alg"] == case["alg"].replace("_multi_cate", "_multi")][0]
            exp = twin["result"]
        assert [got[0], got[1], got[2], got[3], got[4], [list(r) for r in got[5]]] == exp, case


def test_arg_parse_matches_reference_goldens():
    d = json.load(open(os.path.join(GOLD, "my_utils_golden.json")))
    for case in d["arg_parse"]:
        assert my_utils.arg_parse(case["argv"]) == case["result"]


# ------------------------------------------------------------------ TFRecord
def test_crc32c_known_answers():
    assert tfrecord.crc32c(b"123456789") == 0xE3069283
    assert tfrecord.crc32c(b"") == 0
    assert tfrecord.crc32c(bytes(32)) == 0x8A9136AA        # RFC 3720 B.4: 32 zero bytes
    assert tfrecord.crc32c(b"\xff" * 32) == 0x62A8AB43     # RFC 3720 B.4: 32 0xff bytes


def test_example_roundtrip_and_record_crc(tmp_path):
    feats = {"label": ("float", [1.0]), "cont_feats": ("float", [0.5, -2.25, 3.0]),
             "cate_feats": ("int64", [0, 7, 2 ** 40, -3]), "vector_feats": ("float", [])}
    data = tfrecord.encode_example(feats)
    back = tfrecord.decode_example(data)
    assert back["cate_feats"] == ("int64", [0, 7, 2 ** 40, -3])
    assert back["cont_feats"][1] == [0.5, -2.25, 3.0]
    p = tmp_path / "part-0"
    tfrecord.write_records(str(p), [data, data])
    assert list(tfrecord.read_records(str(p))) == [data, data]
    raw = bytearray(p.read_bytes())
    raw[20] ^= 0xFF                                         # corrupt the first payload
    p.write_bytes(bytes(raw))
    with pytest.raises(IOError):
        list(tfrecord.read_records(str(p)))
    # frame layout: u64 length, masked crc of the length
    ln = struct.unpack("<Q", bytes(raw[:8]))[0]
    assert ln == len(data)


class _MP:
    def __init__(self, **kw):
        self.__dict__.update(dict(alg_name="deepfm_pipeline", epochs=2, batch_size=32, cont_field_size=13,
                                  vector_feats_size=2, cate_field_size=26, multi_feats_size=0, shuffle=0,
                                  shuffle_seed=None))
        self.__dict__.update(kw)


def _write_parts(d, n_parts=2, per=50, **mk):
    batches = []
    for i in range(n_parts):
        b = make_batch(per, vector=2, cate_index_size=5000, seed=i, **mk)
        data_loader.write_tfrecord_part(os.path.join(d, "part-%05d" % i), b)
        batches.append(b)
    with open(os.path.join(d, "_SUCCESS"), "w"):
        pass
    return batches


def test_loader_batches_drop_remainder_and_repeat(tmp_path):
    src = _write_parts(str(tmp_path))
    mp = _MP()
    files = data_loader.get_file_list(str(tmp_path) + "/")
    assert sorted(os.path.basename(f) for f in files) == ["part-00000", "part-00001"]
    stream = data_loader.pipeline_process(mp, sorted(files), "train")
    got = list(stream)
    assert len(got) == 2 * (100 // 32)              # per epoch: batch(drop_remainder) then repeat
    flat = {k: np.concatenate([b[k] for b in src]) for k in src[0]}
    np.testing.assert_array_equal(got[0]["cate_feats"], flat["cate_feats"][:32])
    np.testing.assert_array_equal(got[0]["cont_feats"], flat["cont_feats"][:32])
    assert got[0]["label"].shape == (32, 1) and got[0]["cate_feats"].dtype == np.int64
    # re-iterable: a second pass starts over (a fresh session in the reference)
    assert np.array_equal(next(iter(stream))["cate_feats"], got[0]["cate_feats"])
    pred = list(data_loader.pipeline_process(mp, sorted(files), "pred"))
    assert len(pred) == 100 // 32


def test_loader_fixed_len_and_cate_algs(tmp_path):
    _write_parts(str(tmp_path), n_parts=1)
    files = data_loader.get_file_list(str(tmp_path) + "/")
    with pytest.raises(ValueError):
        list(data_loader.pipeline_process(_MP(cont_field_size=12), files, "pred"))
    got = list(data_loader.pipeline_process(_MP(alg_name="deepfm_multi_cate"), files, "pred"))
    assert "cont_feats" not in got[0]
    plain = list(data_loader.pipeline_process(_MP(), files, "pred"))[0]["cate_feats"]
    sh = list(data_loader.pipeline_process(_MP(shuffle=1, shuffle_seed=3), files, "pred"))[0]["cate_feats"]
    src = {tuple(r) for r in make_batch(50, vector=2, cate_index_size=5000, seed=0)["cate_feats"]}
    assert all(tuple(r) in src for r in sh) and not np.array_equal(sh, plain)


# ------------------------------------------------------------------ AUC
def test_oracle_auc_matches_sklearn_goldens():
    """The oracle AUC (the checker of the GPU dl_auc, tests/test_gpu_kernels.py) against
    the sklearn goldens."""
    from oracle import ctr_ref as R
    d = np.load(os.path.join(GOLD, "auc_golden.npz"))
    for case in ("ties", "random", "all_tied"):
        assert abs(R.auc(d[case + "_y"], d[case + "_s"]) - d[case + "_auc"][0]) < 1e-12


# ------------------------------------------------------------------ oracle fixtures
@pytest.mark.parametrize("name", ["deepfm_pipeline", "dnn_pipeline", "deepfm_multi_cate"])
def test_oracle_reproduces_fixtures(name):
    from oracle import ctr_ref as R
    from tests.golden.make_golden import MODEL_CASES
    d = np.load(os.path.join(GOLD, "model_%s.npz" % name))
    cfg = R.make_cfg(name, **MODEL_CASES[name])
    P = {k[5:]: d[k].copy() for k in d.files if k.startswith("init/")}
    opt = R.AdamTF1(cfg, P)
    for i in range(3):
        b = {k.split("/", 1)[1]: d[k] for k in d.files if k.startswith("batch%d/" % i)}
        fw = R.train_step(cfg, P, opt, b)
        np.testing.assert_array_equal(fw["z"], d["z%d" % i])
    for k in P:
        np.testing.assert_array_equal(P[k], d["final/" + k])


def test_load_style_loader(tmp_path):
    from deep_learning_amd.utils import data_loader_load as dll
    import pickle

    class MP:
        alg_name, cont_field_size, cate_field_size, wide_field_size, batch_size, vector_field_size = \
            "wdl", 13, 26, 26, 40, 0
    b = make_batch(100, cate_index_size=5000, seed=3, wide_fields=26)
    dll.write_lines(str(tmp_path / "part-0"), b)
    out = dll.load_input_file(MP, str(tmp_path))
    assert len(out) == 3                                  # last partial batch kept (40, 40, 20)
    d0 = pickle.loads(out[0])
    np.testing.assert_array_equal(d0["cate_feats"], b["cate_feats"][:40])
    np.testing.assert_array_equal(d0["wide_feats"], b["wide_feats"][:40])
    np.testing.assert_allclose(d0["cont_feats"], b["cont_feats"][:40])
    assert pickle.loads(out[2])["labels"].shape == (20, 1)


# ------------------------------------------------------------------ native reader (libdlio.so)
def test_native_crc32c_known_answers():
    from deep_learning_amd.utils import native_reader as nr
    assert nr.crc32c(b"123456789") == 0xE3069283                 # CRC-32C check value
    assert nr.crc32c(bytes(32)) == 0x8A9136AA                    # RFC 3720 B.4: 32 zero bytes
    assert nr.crc32c(b"\xff" * 32) == 0x62A8AB43                 # RFC 3720 B.4: 32 0xff bytes
    rng = np.random.default_rng(0)
    for n in (0, 1, 7, 8, 9, 63, 1000):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert nr.crc32c(b) == tfrecord.crc32c(b)


@pytest.mark.parametrize("threads", [1, 3, 10])
def test_native_reader_matches_python_decoder(tmp_path, threads):
    """Unshuffled batches of the native reader equal the pure-Python decode of the same
    files (file order, drop_remainder, repeat), for any decoder thread count."""
    src = _write_parts(str(tmp_path), n_parts=3, per=70)
    files = sorted(data_loader.get_file_list(str(tmp_path) + "/"))
    spec = data_loader._spec(_MP())
    exs = [data_loader.parse_example(r, spec) for _ in range(2) for f in files for r in tfrecord.read_records(f)]
    from deep_learning_amd.utils.native_reader import NativeReader
    got = list(NativeReader(files, [(k, kd, s) for k, (kd, s) in spec.items()], 32, repeat=2, threads=threads))
    # utils/data_loader.py:30-37: batch(drop_remainder) inside each epoch, then repeat:
    # 2 x floor(210 / 32) = 12 batches, epoch 2 starts again at record 0 (records 192..209
    # of epoch 1 are dropped, never mixed into a batch with epoch 2's)
    assert len(got) == 2 * (210 // 32)
    per_epoch = 210 // 32
    for i, b in enumerate(got):
        ep, j = divmod(i, per_epoch)
        r0 = ep * 210 + j * 32
        for k, (kind, size) in spec.items():
            want = np.asarray([e[k] for e in exs[r0:r0 + 32]],
                              np.int64 if kind == "int64" else np.float32).reshape(32, size)
            np.testing.assert_array_equal(b[k], want, err_msg=k)
    flat = np.concatenate([s["cate_feats"] for s in src])
    np.testing.assert_array_equal(got[0]["cate_feats"], flat[:32])


def test_native_reader_seeded_shuffle(tmp_path):
    _write_parts(str(tmp_path), n_parts=2, per=100)
    files = sorted(data_loader.get_file_list(str(tmp_path) + "/"))
    run = lambda seed: np.concatenate([b["cate_feats"] for b in data_loader.pipeline_process(
        _MP(shuffle=1, shuffle_seed=seed, batch_size=20), files, "pred")])
    plain = np.concatenate([b["cate_feats"] for b in data_loader.pipeline_process(_MP(batch_size=20), files, "pred")])
    a, a2, b = run(5), run(5), run(6)
    np.testing.assert_array_equal(a, a2)                         # deterministic for a seed
    assert not np.array_equal(a, plain) and not np.array_equal(a, b)
    key = lambda m: sorted(map(tuple, m))
    assert key(a) == key(plain)                                  # a permutation of the records


def test_native_reader_shuffled_epochs_do_not_mix(tmp_path):
    """shuffle -> batch(drop_remainder) -> repeat (utils/data_loader.py:30-37) with a shuffle
    buffer: every epoch is its own shuffled permutation cut into floor(N/B) batches; the
    records a batch holds all come from one epoch, and each epoch drops its own remainder."""
    from deep_learning_amd.utils.native_reader import NativeReader
    src = _write_parts(str(tmp_path), n_parts=1, per=70)           # 70 records, B = 16 -> 4 per epoch
    files = sorted(data_loader.get_file_list(str(tmp_path) + "/"))
    spec = [(k, kd, s) for k, (kd, s) in data_loader._spec(_MP()).items()]
    got = list(NativeReader(files, spec, 16, repeat=3, shuffle_buf=40, seed=11, threads=2))
    assert len(got) == 3 * (70 // 16)
    rec_id = {tuple(r): i for i, r in enumerate(src[0]["cate_feats"])}
    for ep in range(3):
        ids = [rec_id[tuple(r)] for b in got[4 * ep:4 * ep + 4] for r in b["cate_feats"]]
        assert len(set(ids)) == 64                                 # no record twice within an epoch
    first = [rec_id[tuple(r)] for b in got[:4] for r in b["cate_feats"]]
    second = [rec_id[tuple(r)] for b in got[4:8] for r in b["cate_feats"]]
    assert first != second                                         # reshuffled each iteration


def test_native_reader_errors(tmp_path):
    from deep_learning_amd.utils.native_reader import NativeReader
    _write_parts(str(tmp_path), n_parts=1, per=40)
    f = str(tmp_path / "part-00000")
    spec = [(k, kd, s) for k, (kd, s) in data_loader._spec(_MP()).items()]
    with pytest.raises(ValueError, match="Key: cont_feats. Can't parse serialized Example: expected 12"):
        list(NativeReader([f], [(k, kd, 12 if k == "cont_feats" else s) for k, kd, s in spec], 8))
    with pytest.raises(ValueError, match="Data types don't match"):
        list(NativeReader([f], [(k, "float" if k == "cate_feats" else kd, s) for k, kd, s in spec], 8))
    with pytest.raises(IOError, match="No such file"):
        NativeReader([f + "x"], spec, 8)
    raw = bytearray(open(f, "rb").read())
    bad = tmp_path / "part-bad"
    raw2 = bytearray(raw)
    raw2[30] ^= 0x01                                             # payload byte of record 0
    bad.write_bytes(bytes(raw2))
    with pytest.raises(IOError, match="corrupted record data"):
        list(NativeReader([str(bad)], spec, 8))
    raw3 = bytearray(raw)
    raw3[0] ^= 0x01                                              # length field of record 0
    bad.write_bytes(bytes(raw3))
    with pytest.raises(IOError, match="corrupted record length"):
        list(NativeReader([str(bad)], spec, 8))
    bad.write_bytes(bytes(raw[:-3]))                             # truncated last record
    with pytest.raises(IOError, match="truncated"):
        list(NativeReader([str(bad)], spec, 8))


def test_native_reader_wire_variants(tmp_path):
    """Unpacked float/int64 lists, a feature outside the spec, a repeated key (map
    semantics: the last entry wins) and negative int64 varints decode like the spec says."""
    from deep_learning_amd.utils.native_reader import NativeReader
    v = tfrecord._varint
    ld = tfrecord._len_field

    def entry(name, feat):
        return ld(1, ld(1, name.encode()) + ld(2, feat))

    unpacked_f = ld(2, b"".join(v((1 << 3) | 5) + struct.pack("<f", x) for x in (1.5, -2.0)))
    unpacked_i = ld(3, b"".join(v((1 << 3) | 0) + v(x) for x in (7, -3)))
    stale = ld(3, ld(1, v(99) + v(98)))
    label = ld(2, ld(1, struct.pack("<f", 1.0)))
    extra = ld(1, ld(1, b"abc"))
    ex = ld(1, entry("cont", unpacked_f) + entry("ids", stale) + entry("junk", extra) + entry("ids", unpacked_i)
            + entry("label", label))
    p = str(tmp_path / "part-w")
    tfrecord.write_records(p, [ex] * 3)
    b = next(NativeReader([p], [("label", "float", 1), ("cont", "float", 2), ("ids", "int64", 2)], 3))
    np.testing.assert_array_equal(b["cont"], [[1.5, -2.0]] * 3)
    np.testing.assert_array_equal(b["ids"], [[7, -3]] * 3)
    np.testing.assert_array_equal(b["label"], [[1.0]] * 3)


@pytest.mark.parametrize("proto", [3, 4, 5, "lists"])
def test_native_unpickle_batch_matches_pickle(proto):
    """dlio_unpickle_batch (the load-style feed's decoder): a batch dict pickled with protocols
    3-5 (numpy arrays of several dtypes, converted to float32 / int64) or as the reference's
    lists of rows decodes to exactly what pickle.loads + np.asarray give; forms it does not take
    (a missing key, an object array, protocols 0 and 2, another global, Fortran or big-endian
    arrays, truncated data, more rows than the buffers hold) return None, so the caller falls back
    to pickle.loads."""
    import collections
    import pickle
    from deep_learning_amd.utils import native_reader as nr
    rng = np.random.default_rng(0)
    B, C, S = 777, 13, 26
    d = {"labels": rng.integers(0, 2, (B, 1)).astype(np.float32), "cont_feats": rng.random((B, C)),
         "cate_feats": rng.integers(0, 1 << 40, (B, S)), "wide_feats": rng.integers(0, 1000, (B, S)).astype(np.int32),
         "other": np.arange(3)}
    fields = [("labels", nr.FLOAT, 1), ("cont_feats", nr.FLOAT, C), ("cate_feats", nr.INT64, S),
              ("wide_feats", nr.INT64, S)]
    item = pickle.dumps({k: v.tolist() for k, v in d.items()}) if proto == "lists" else pickle.dumps(d, protocol=proto)
    outs = [np.full((B + 3, sz), 7, np.float32 if k == nr.FLOAT else np.int64) for _, k, sz in fields]
    assert nr.unpickle_batch_into(item, fields, outs, B + 3) == B
    ref = pickle.loads(item)
    for (key, k, sz), o in zip(fields, outs):
        np.testing.assert_array_equal(o[:B], np.asarray(ref[key], o.dtype).reshape(B, sz), err_msg=key)
        assert (o[B:] == 7).all()
    if proto != 4:
        return
    bad = [pickle.dumps({"labels": d["labels"]}), pickle.dumps(dict(d, cont_feats=d["cont_feats"].astype(object))),
           pickle.dumps(d, protocol=0), pickle.dumps(d, protocol=2), pickle.dumps(collections.OrderedDict(d)),
           pickle.dumps(dict(d, cont_feats=np.asfortranarray(d["cont_feats"]))),
           pickle.dumps(dict(d, cont_feats=d["cont_feats"].astype(">f8"))), item[:-40]]
    for b in bad:
        assert nr.unpickle_batch_into(b, fields, outs, B) is None
    assert nr.unpickle_batch_into(item, fields, outs, B - 1) is None
    # 8-byte length opcodes (BINUNICODE8, BINBYTES8, BYTEARRAY8) whose length is near INT64_MAX:
    # the bounds check must not overflow into a pass (a read far past the buffer)
    import struct
    for op in (b"\x8d", b"\x8e", b"\x96"):
        for ln in (0x7FFFFFFFFFFFFFF0, 0x7FFFFFFFFFFFFFFF, 1 << 62):
            evil = b"\x80\x05\x95" + struct.pack("<Q", 11 + 4) + op + struct.pack("<Q", ln) + b"abcd."
            assert nr.unpickle_batch_into(evil, fields, outs, B) is None


def test_native_unpickle_large_batch_in_row_pieces():
    """A batch of 4 MB or more is copied as row pieces on a team of threads: a C5-sized dict
    (arrays that are copied, and arrays converted from float64 / int32) and a lists-of-rows
    batch decode exactly as pickle.loads gives them; a bad row deep inside the lists (its piece
    on some helper thread) still makes the whole decode decline."""
    import pickle
    from deep_learning_amd.utils import native_reader as nr
    rng = np.random.default_rng(5)
    B, C, S = 60000, 13, 26
    d = {"labels": rng.integers(0, 2, B).astype(np.float32), "cont_feats": rng.random((B, C)),
         "cate_feats": rng.integers(0, 1 << 40, (B, S)), "wide_feats": rng.integers(0, 1 << 30, (B, S)).astype(np.int32)}
    fields = [("labels", nr.FLOAT, 1), ("cont_feats", nr.FLOAT, C), ("cate_feats", nr.INT64, S),
              ("wide_feats", nr.INT64, S)]
    outs = [np.full((B, sz), 7, np.float32 if k == nr.FLOAT else np.int64) for _, k, sz in fields]
    for item in (pickle.dumps(d, protocol=5), pickle.dumps({"labels": d["labels"].tolist(),
                                                           "cont_feats": d["cont_feats"].tolist(),
                                                           "cate_feats": d["cate_feats"].tolist(),
                                                           "wide_feats": d["wide_feats"].tolist()})):
        assert len(item) >= 4 << 20
        for o in outs:
            o.fill(7)
        assert nr.unpickle_batch_into(item, fields, outs, B) == B
        for (key, k, sz), o in zip(fields, outs):
            np.testing.assert_array_equal(o, np.asarray(d[key], o.dtype).reshape(B, sz), err_msg=key)
    rows = d["cate_feats"].tolist()
    rows[B - 123] = rows[B - 123][:-1]          # one short row, far from the first piece
    bad = pickle.dumps(dict(d, cate_feats=rows))
    assert nr.unpickle_batch_into(bad, fields, outs, B) is None


def test_s3_dw_split_counts():
    """engine._s3_dw_splits: the split-K count of an s3 weight gradient fills the CUs in as few
    rounds of 128 x 224 blocks as possible (C2's 8-tile layers keep 32 slabs; C3's layer 0,
    M = 528 = 10 tiles, takes 25 — one round of 250 blocks, not two of 320), never more than
    the cap, at least one."""
    from deep_learning_amd.engine import _s3_dw_splits
    assert _s3_dw_splits(432, 400, 65536, 32) == 32
    assert _s3_dw_splits(416, 400, 65536, 32) == 32
    assert _s3_dw_splits(528, 400, 65536, 32) == 25
    assert _s3_dw_splits(432, 400, 1536, 1) == 1
    for M in (16, 100, 432, 528, 1000):
        for base in (1, 7, 32, 64):
            s = _s3_dw_splits(M, 400, 65536, base)
            assert 1 <= s <= base


def test_bf16_dw_split_counts():
    """engine._bf16_dw_splits: the bf16 ring kernel's split count (144 x 400 blocks, one per CU):
    C5's layers (M = 432 / 416: 3 tiles) take 85 requested = 79 slabs of 832 rows in one round
    of 237 blocks; a batch without whole 32-row steps keeps the cap (two-buffer kernel)."""
    from deep_learning_amd.engine import _bf16_dw_splits, _num_splits
    assert _bf16_dw_splits(432, 65536, 96) == 85
    assert _bf16_dw_splits(416, 65536, 96) == 85
    assert _num_splits(65536, 85, 64) == 79
    assert _bf16_dw_splits(432, 1000, 1) == 1
    assert _bf16_dw_splits(432, 65540, 96) == 96
    for M in (16, 144, 432, 1000):
        for base in (1, 7, 64, 96):
            s = _bf16_dw_splits(M, 65536, base)
            assert 1 <= s <= base and -(-M // 144) * s <= max(256, -(-M // 144))
