"""bench.py's bookkeeping (CPU): the PMC traffic it quotes comes only from a summary of the
same workload and id distribution, the calibrated backward bytes only for the case they were
measured on, and the vocab per workload follows BASELINE's configs (C4 = 100 M rows sharded)."""
import argparse
import json
import os

import bench


def test_pmc_traffic_matches_workload_and_id_dist():
    got = bench.pmc_traffic("embed_bwd", 1, lazy=True, workload="c2", id_dist="uniform")
    assert got is not None
    d = json.load(open(os.path.join(bench.ROOT, got["source"])))
    assert d.get("workload", "c2") == "c2" and d.get("id_dist", "uniform") == "uniform"
    # no committed Zipf summary of C2's backward: nothing is quoted rather than uniform bytes
    z = bench.pmc_traffic("embed_bwd", 1, lazy=True, workload="c2", id_dist="zipf")
    if z is not None:
        assert json.load(open(os.path.join(bench.ROOT, z["source"]))).get("id_dist") == "zipf"
    assert bench.pmc_traffic("embed_bwd", 2, lazy=True) is None        # per-rank figures only at N = 1


def test_calibrated_backward_bytes_only_where_measured():
    cal = bench.bwd_calibrated("embed_bwd", 1, lazy=True, workload="c2", id_dist="uniform")
    assert cal is not None and cal["traffic_calibrated"] > 0
    d = json.load(open(os.path.join(bench.ROOT, cal["traffic_calibrated_source"])))
    # the calibration never exceeds the x2-everywhere figure and keeps every write
    assert d["write_bytes"] <= d["hbm_bytes_calibrated"] <= d["hbm_bytes_x2_everywhere"]
    for other in (dict(workload="c3"), dict(id_dist="zipf"), dict(lazy=False)):
        kw = dict(lazy=True, workload="c2", id_dist="uniform")
        kw.update(other)
        assert bench.bwd_calibrated("embed_bwd", 1, **kw) is None
    assert bench.bwd_calibrated("rec_gather", 1, lazy=True) is None


def test_vocab_per_workload():
    a = argparse.Namespace(vocab=None)
    assert bench.vocab_for("c2", a, sharded=False) == 1_000_000
    assert bench.vocab_for("c5", a, sharded=True) == 1_000_000
    v = bench.vocab_for("c2", a, sharded=True)          # C4: 100 M rows over the 26 fields
    assert v * 26 >= 100_000_000 > (v - 1) * 26
    assert bench.vocab_for("c2", argparse.Namespace(vocab=7), sharded=True) == 7
