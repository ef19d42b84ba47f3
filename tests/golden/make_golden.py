"""Regenerates the committed golden fixtures in tests/golden/ (run in the build
container, where /root/reference exists; the GPU box never runs this).

  my_utils_golden.json : outputs of the REFERENCE's own utils/my_utils.py
                         (feat_size, arg_parse) on synthetic conf files — imported
                         from /root/reference (pure Python, no TF needed).
  auc_golden.npz       : sklearn.metrics.roc_auc_score (the reference's AUC call,
                         models/deepfm_pipeline.py:311) on tie-heavy and random cases.
  model_<name>.npz     : oracle (oracle/ctr_ref.py) fixtures — inputs, injected initial
                         parameters, logits/loss per step and parameters after 3 TF1-Adam
                         steps.  These pin the oracle against regressions; the model math
                         itself is parity-unpinned against TF (not installable).
"""
import importlib.util
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
REF = "/root/reference/utils/my_utils.py"

CONFS = {
    "pipeline_mix": ["f%d\tx\tfloat" % i for i in range(13)] + ["c%d\tx\tstring" % i for i in range(26)]
    + ["user_vec\tx\tvector", "item_midv\tx\tvec", "other_vec\tx\tvec",
       "tags\tx\tarr\t_\t_\t_\t_\tk=30\ttags", "cats\tx\tarr\t_\t_\t_\t_\tk=20\tcats"],
    "with_blank_and_unknown": ["", "a\tx\tfloat", "b\tx\tbogus", "c\tx\tstring", ""],
}
ALGS = ["deepfm_pipeline", "deepfm_multi", "deepfm_multi_cate", "dnn_multi", "dnn_multi_cate", "dnn_pipeline",
        "deepfm_cate"]


def my_utils_goldens():
    spec = importlib.util.spec_from_file_location("ref_my_utils", REF)
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    out = {"feat_size": [], "arg_parse": []}
    for cname, lines in CONFS.items():
        with tempfile.TemporaryDirectory() as d:
            with open(os.path.join(d, "dnn.conf"), "w") as f:
                f.write("\n".join(lines) + "\n")
            with open(os.path.join(d, "ignored.conf"), "w") as f:
                f.write("zz\tx\tfloat\n")
            for alg in ALGS:
                res = ref.feat_size(d, alg)
                out["feat_size"].append({"conf": cname, "lines": lines, "alg": alg,
                                         "result": [res[0], res[1], res[2], res[3], res[4], res[5]]})
    for argv in (["x", "alg_name=deepfm_pipeline", "batch_size=256"], ["prog", " a = b ", "k=v"]):
        out["arg_parse"].append({"argv": argv, "result": ref.arg_parse(argv)})
    out["has_venus_set_environ"] = hasattr(ref, "venus_set_environ")
    with open(os.path.join(HERE, "my_utils_golden.json"), "w") as f:
        json.dump(out, f, indent=1)


def auc_goldens():
    from sklearn.metrics import roc_auc_score
    rng = np.random.default_rng(0)
    cases = {}
    y = (rng.random(3000) < 0.3).astype(np.float32)
    s = np.round(rng.random(3000) * 10) / 10
    cases["ties"] = (y, s)
    s2 = rng.random(1001).astype(np.float32)
    cases["random"] = ((rng.random(1001) < s2).astype(np.float32), s2)
    cases["all_tied"] = (np.array([0, 1, 0, 1, 1], np.float32), np.full(5, 0.5, np.float32))
    arrs = {}
    for k, (yy, ss) in cases.items():
        arrs[k + "_y"], arrs[k + "_s"] = yy, ss
        arrs[k + "_auc"] = np.array([roc_auc_score(yy, ss)])
    np.savez(os.path.join(HERE, "auc_golden.npz"), **arrs)


MODEL_CASES = {
    "deepfm_pipeline": dict(C=13, V=0, S=26, E=8, cate_index_size=600, hidden=[16, 12]),
    "dnn_pipeline": dict(C=13, V=3, S=26, E=8, cate_index_size=600, hidden=[16, 12]),
    "deepfm_multi_cate": dict(V=2, S=6, E=8, cate_index_size=900, hidden=[16, 12],
                              multi_ranges=[[0, 10, "a"], [10, 16, "b"]]),
}


def model_batches(name, kw, B=64, n=3):
    from deep_learning_amd.synthetic import make_batch
    out = []
    for i in range(n):
        if name == "deepfm_multi_cate":
            b = make_batch(B, cont=0, vector=kw["V"], cate_fields=kw["S"], cate_index_size=kw["cate_index_size"],
                           seed=50 + i, cate_only=True)
            rng = np.random.default_rng(70 + i)
            multi = rng.integers(1, kw["cate_index_size"], size=(B, 16))
            multi[rng.random((B, 16)) < 0.5] = 0
            b["cate_feats"] = np.concatenate([b["cate_feats"], multi], 1)
        else:
            b = make_batch(B, cont=kw["C"], vector=kw["V"], cate_fields=kw["S"],
                           cate_index_size=kw["cate_index_size"], seed=50 + i)
            b["cate_feats"][0, :3] = [0, 1, 12]
        out.append(b)
    return out


def model_goldens():
    from oracle import ctr_ref as R
    for name, kw in MODEL_CASES.items():
        cfg = R.make_cfg(name, **kw)
        P = R.init_params(cfg, np.random.default_rng(3))
        arrs = {"init/" + k: v.copy() for k, v in P.items()}
        opt = R.AdamTF1(cfg, P)
        for i, b in enumerate(model_batches(name, kw)):
            for k, v in b.items():
                arrs["batch%d/%s" % (i, k)] = v
            fw = R.train_step(cfg, P, opt, b)
            arrs["z%d" % i] = fw["z"]
            arrs["loss%d" % i] = np.array([fw["loss"]])
        for k, v in P.items():
            arrs["final/" + k] = v
        np.savez(os.path.join(HERE, "model_%s.npz" % name), **arrs)


if __name__ == "__main__":
    if os.path.exists(REF):
        my_utils_goldens()
    auc_goldens()
    model_goldens()
    print("goldens written to", HERE)
