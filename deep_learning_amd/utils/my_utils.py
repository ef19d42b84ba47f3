"""Config helpers with the reference's contract (utils/my_utils.py:7-78).

arg_parse : "key=value" argv items -> dict of strings (argv[0] skipped).
feat_size : scans ``dnn.conf`` / ``lr.conf`` in a directory (TSV: col0 name,
            col2 type, col7 "k=N" for arr) and returns
            (cont_size, vector_size, cate_size, multi_size, multi_fields, multi_ranges).

Documented deviation (SURVEY.md ledger item 10): the reference's pooling list
misspells the *_multi_cate algorithm names, so those algorithms get no multi-hot
ranges and then crash (deepfm_multi_cate.py:136).  Here the intended names are
recognised as pooling algorithms as well.  Every other behaviour — the vector
widths (200 for user/item vectors, 100 for mid vectors), ranges as
[start, end, feature_name], the exit(-1) on a malformed line — is the reference's.
"""
import os
import sys

VEC_200 = ("user_vec", "ruUserVec", "item_vec", "user_kgv", "item_kgv")
VEC_100 = ("item_midv", "user_midv")
# reference list (incl. its typos) + the intended multi_cate names
POOLING_ALGS = ("deepfm_multi_cat", "deepfm_multi", "dnn_multi_cat", "dnn_multi",
                "deepfm_multi_cate", "dnn_multi_cate")


def arg_parse(argv):
    out = {}
    for item in argv[1:]:
        parts = item.split("=")
        out[parts[0].strip()] = parts[1].strip()
    return out


def feat_size(path, alg_name):
    cont = vector = cate = multi = multi_fields = 0
    ranges = []
    for fname in os.listdir(path):
        if fname not in ("dnn.conf", "lr.conf"):
            continue
        print("----read %s----" % (path + "/" + fname))
        with open(os.path.join(path, fname)) as fh:
            start = 0                      # slot offsets restart per conf file
            for raw in fh:
                line = raw.strip()
                if not line:
                    continue
                try:
                    cols = line.split("\t")
                    name, kind = cols[0], cols[2]
                    if kind in ("vector", "vec"):
                        if name in VEC_200:
                            vector += 200
                        elif name in VEC_100:
                            vector += 100
                    elif kind == "arr":
                        top_n = int(cols[7].strip().split("=")[1])
                        if alg_name in POOLING_ALGS:
                            multi += top_n
                            multi_fields += 1
                            ranges.append([start, start + top_n, cols[-1]])
                            start += top_n
                        else:
                            cate += top_n
                    elif kind == "string":
                        cate += 1
                    elif kind == "float":
                        cont += 1
                    else:
                        print("%s is error!!!" % line)
                except Exception:
                    print("-----------feat_conf is Error!!!!-----------")
                    print(line)
                    sys.exit(-1)
    return cont, vector, cate, multi, multi_fields, ranges
