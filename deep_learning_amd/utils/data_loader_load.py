"""In-memory batch loader of the load-style models (reference utils/data_loader_load.py:61-139).

Input lines: ``label,cont values,cate ids[,multi|wide ids]`` — space-separated
inside each comma field.  Output: a list of pickled batch dicts with the
reference's keys (cont_feats, vector_feats, cate_feats, mul_cate_feats,
mul_cate_feats_value, wide_feats, labels), batches of mp.batch_size with the
last partial batch kept.  The vector part is the last ``vector_field_size``
values of the cont field (:113-117).

Deviations: values are numeric arrays (the reference keeps strings and lets
TF's feed cast them); ``wide_feats`` is filled for alg ``wdl`` as well (the
reference fills it only for "wide_deep"/"wdl_textline", :125, so its own wdl
runner could not train — SURVEY.md §3.4).
"""
import os
import pickle

import numpy as np

WIDE_ALGS = ("wdl", "wide_deep", "wdl_textline")


def read_data(mp, file_dir_list):
    lines = []
    for f in file_dir_list:
        with open(f) as fh:
            lines.extend(l for l in fh if l.strip())
    print("size of read data = ", len(lines))
    return lines


def _vals(field, dtype):
    return np.asarray(field.split(" ") if field else [], dtype=dtype)


def load_process(mp, file_dir_list):
    data = read_data(mp, file_dir_list)
    first = data[0].strip("\n").split(",")
    cont_n, cate_n = len(first[1].split(" ")), len(first[2].split(" "))
    print("data_cont_field_size = ", cont_n)
    print("data_cate_field_size = ", cate_n)
    if cont_n != mp.cont_field_size or cate_n != mp.cate_field_size:
        print("feature size is error!!!")
        raise SystemExit(-1)
    wide = mp.alg_name in WIDE_ALGS
    if wide:
        wn = len(first[3].split(" "))
        print("data_wide_field_size = ", wn)
        if wn != mp.wide_field_size:
            print("feature size is error!!!")
            raise SystemExit(-1)
    vec_n = int(getattr(mp, "vector_field_size", 0) or 0)
    out = []
    for i in range(0, len(data), mp.batch_size):
        batch = data[i:i + mp.batch_size]
        labels, cont, vec, cate, widef = [], [], [], [], []
        for line in batch:
            sp = line.strip("\n").split(",")
            labels.append([float(sp[0])])
            c = _vals(sp[1], np.float32)
            cut = mp.cont_field_size - vec_n
            cont.append(c[:cut])
            vec.append(c[cut:])
            cate.append(_vals(sp[2], np.int64))
            if wide:
                widef.append(_vals(sp[3], np.int64))
        d = {"cont_feats": np.stack(cont), "vector_feats": np.stack(vec), "cate_feats": np.stack(cate),
             "mul_cate_feats": [], "mul_cate_feats_value": [],
             "wide_feats": np.stack(widef) if wide else [], "labels": np.asarray(labels, np.float32)}
        out.append(pickle.dumps(d))
    return out


def load_input_file(mp, input_path, action_type=""):
    files = sorted(os.path.join(input_path, f) for f in os.listdir(input_path) if f[:4] == "part")
    return load_process(mp, files)


def write_lines(path, batch):
    """Writes a batch dict (cont_feats, cate_feats, wide_feats, label) as load-style text lines."""
    with open(path, "w") as f:
        for i in range(batch["label"].shape[0]):
            parts = [repr(float(batch["label"][i, 0])),
                     " ".join(repr(float(x)) for x in batch["cont_feats"][i]),
                     " ".join(str(int(x)) for x in batch["cate_feats"][i])]
            if "wide_feats" in batch:
                parts.append(" ".join(str(int(x)) for x in batch["wide_feats"][i]))
            f.write(",".join(parts) + "\n")
