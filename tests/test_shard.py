"""Multi-rank (world_size 2, 4 and 8) tests of the row-sharded path.

CPU (gloo): the sharded algorithm restated in numpy over the real Exchange
collectives equals single-process training on the global batch.
GPU: the real ShardedCTREngine, two ranks sharing cuda:0 (gloo-staged
exchange), equals the oracle on the global batch."""
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ctr_ref as R  # noqa: E402
from tests.shard_worker import KW, WKW, global_batches, wdl_batches  # noqa: E402

STEPS, BL, WORLD = 5, 96, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(mode, tmp_path, world=WORLD):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "shard_worker.py"), mode, str(STEPS), str(BL), str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def _oracle(world=WORLD):
    cfg = R.make_cfg("deepfm_pipeline", **KW)
    P = R.init_params(cfg, np.random.default_rng(42))
    opt = R.AdamTF1(cfg, P)
    zs = []
    for b in global_batches(BL * world, STEPS):
        zs.append(R.train_step(cfg, P, opt, b)["z"])
    return P, zs


@pytest.mark.parametrize("world", [2, 4])
def test_shard_sim_gloo_equals_global_batch(tmp_path, world):
    _launch("sim", tmp_path, world)
    P, zs = _oracle(world)
    for step in range(STEPS):
        z = np.concatenate([np.load(tmp_path / ("rank%d_step%d.npz" % (r, step)))["z"] for r in range(world)])
        np.testing.assert_allclose(z, zs[step], atol=1e-5, rtol=0, err_msg="step %d" % step)
    got = np.load(tmp_path / "rank0.npz")
    for k in P:
        np.testing.assert_allclose(got[k], P[k], atol=1e-5, rtol=0, err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["gpu", "gpu_lazy", "gpu_lazy_pf", "gpu_lazy_chain_pf", "gpu_lazy_ovf_pf"])
def test_sharded_engine_two_ranks_equals_global_batch(tmp_path, mode):
    """gpu_lazy: shard rows as records with lazy-exact Adam and a 4-entry alpha ring
    (flushes inside the 5 steps); _pf: each step prefetches the next batch's index and route
    on the side stream; _chain: owners group arrivals by chains instead of a sort; _ovf: blocks
    sized below these batches' unique rows per owner, so the first step overflows on the device,
    every rank skips it and those after it, grows its blocks and replays them in order — the
    result must still be the oracle's."""
    _check_engine(tmp_path, mode, WORLD)


@pytest.mark.gpu
@pytest.mark.parametrize("world,mode", [(4, "gpu_lazy_pf"), (8, "gpu_lazy_pf"), (8, "gpu_lazy_ovf_pf")])
def test_sharded_engine_many_ranks_equals_global_batch(tmp_path, world, mode):
    """BASELINE C4's world (8 ranks, owner r % 8, 15 exchange blocks a rank, one header
    consensus over 8 ranks), here 4 and 8 ranks sharing cuda:0 over the gloo-staged exchange:
    every step's logits, the sharded table, the replicated state on every rank and the
    all-gathered eval AUC equal the oracle trained on the global batch (8 x 96 samples); the
    overflow case replays its skipped steps with grown blocks on all 8 ranks."""
    _check_engine(tmp_path, mode, world)


def _check_engine(tmp_path, mode, world):
    _launch(mode, tmp_path, world)
    if "_ovf" in mode:
        for r in range(world):
            d = np.load(tmp_path / ("rank%d.npz" % r))
            assert int(d["overflows"]) >= 1 and d["cap"][1] > d["cap"][0], (int(d["overflows"]), d["cap"])
    P, zs = _oracle(world)
    for step in range(STEPS):
        if "_ovf" in mode and step < 2:   # skipped, then replayed by the call that read its report
            continue
        z = np.concatenate([np.load(tmp_path / ("rank%d_step%d.npz" % (r, step)))["z"] for r in range(world)])
        np.testing.assert_allclose(z, zs[step], atol=1e-5, rtol=0, err_msg="logits step %d" % step)
    table = np.zeros_like(P["feats_emb"])
    first = np.zeros_like(P["fm_first_order_emb"][:, 0])
    for r in range(world):
        d = np.load(tmp_path / ("rank%d.npz" % r), allow_pickle=False)
        table[d["rows"]] = d["table"]
        first[d["rows"]] = d["first"]
    C = KW["C"]
    rep = np.load(tmp_path / "rank0.npz")["rep"]
    np.testing.assert_allclose(rep, P["feats_emb"][:C], atol=1e-5, rtol=0)
    np.testing.assert_allclose(table[C:], P["feats_emb"][C:], atol=1e-5, rtol=0)
    np.testing.assert_allclose(first[C:], P["fm_first_order_emb"][C:, 0], atol=1e-5, rtol=0)
    d0 = np.load(tmp_path / "rank0.npz")
    for r in range(1, world):                                    # replicated dense state identical
        np.testing.assert_array_equal(np.load(tmp_path / ("rank%d.npz" % r))["head"], d0["head"])
    # sharded eval: every rank's predictions of two unseen global batches equal the oracle's
    # forward on the trained parameters; the all-gathered AUC equals the oracle AUC of the
    # whole set (north star: AUC within 1e-4), identically on both ranks
    cfg = R.make_cfg("deepfm_pipeline", **KW)
    ev = [np.load(tmp_path / ("rank%d_eval.npz" % r)) for r in range(world)]
    evb = global_batches(BL * world, STEPS + 2)[STEPS:]
    all_s, all_y = [], []
    for j, b in enumerate(evb):
        want = 1.0 / (1.0 + np.exp(-R.forward(cfg, P, b)["z"].astype(np.float64)))
        got = np.concatenate([e["s%d" % j] for e in ev])
        np.testing.assert_allclose(got, want, atol=1e-5, rtol=0, err_msg="eval batch %d" % j)
        all_s.append(want)
        all_y.append(b["label"].reshape(-1))
    want_auc = R.auc(np.concatenate(all_y), np.concatenate(all_s))
    assert all(float(e["auc"]) == float(ev[0]["auc"]) for e in ev)
    assert abs(float(ev[0]["auc"]) - want_auc) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("serial", ["0", "1"])
def test_sharded_all_reduce_placement_equals_global_batch(tmp_path, serial, monkeypatch):
    """DLAMD_SHARD_AR_SERIAL: the flat all-reduce after the gradient exchange on its stream
    (1, the default) or on a stream of its own beside it (0) — the same global-batch result."""
    monkeypatch.setenv("DLAMD_SHARD_AR_SERIAL", serial)
    _check_engine(tmp_path, "gpu_lazy_pf", WORLD)


def test_sharded_report_lag_bounded_by_the_status_ring():
    """The status ring holds 4 reports, so a report lag past 3 would let report k + 4 overwrite
    report k before the host reads it: refused up front (CPU: before any device work)."""
    import types
    from deep_learning_amd.engine import ModelSpec
    from deep_learning_amd.shard import ShardedCTREngine
    ex = types.SimpleNamespace(world=2, rank=0)
    spec = ModelSpec("deepfm_pipeline", **KW)
    for lag in (-1, 4, 8):
        with pytest.raises(ValueError, match="lag must be 0..3"):
            ShardedCTREngine(spec, 64, ex, lag=lag)


@pytest.mark.gpu
def test_sharded_bad_id_on_one_rank_raises_everywhere(tmp_path):
    """A bad id in one rank's batch (here rank 1's half of global batch 1, prefetched during
    step 0): its validation bit travels in the request headers, so every rank's step-begin node
    skips that step (nothing applied anywhere) and every rank raises TF's InvalidArgumentError
    (deepfm_pipeline.py:219-221) at the same call — the engine's report lag (2) after it, naming
    rank 1 — and training continues: equal to the oracle trained on the global batches without
    batch 1, with the replicated state identical on both ranks."""
    _launch("gpu_badid", tmp_path)
    cfg = R.make_cfg("deepfm_pipeline", **KW)
    P = R.init_params(cfg, np.random.default_rng(42))
    opt = R.AdamTF1(cfg, P)
    good = [b for i, b in enumerate(global_batches(BL * WORLD, STEPS)) if i != 1]
    for step, b in enumerate(good):
        z = np.concatenate([np.load(tmp_path / ("rank%d_step%d.npz" % (r, step)))["z"] for r in range(WORLD)])
        np.testing.assert_allclose(z, R.train_step(cfg, P, opt, b)["z"], atol=1e-5, rtol=0,
                                   err_msg="logits step %d" % step)
    d = [np.load(tmp_path / ("rank%d.npz" % r)) for r in range(WORLD)]
    for e in d:
        assert e["raised"].tolist() == [3]
    table = np.zeros_like(P["feats_emb"])
    for e in d:
        table[e["rows"]] = e["table"]
    C = KW["C"]
    np.testing.assert_allclose(table[C:], P["feats_emb"][C:], atol=1e-5, rtol=0)
    np.testing.assert_array_equal(d[0]["head"], d[1]["head"])


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["gpu_wdl", "gpu_wdl_lazy_pf", "gpu_wdl_bf16_lazy"])
def test_sharded_wdl_two_ranks_equals_global_batch(tmp_path, mode):
    """Wide&Deep row-sharded (BASELINE C5 at N GPUs): weight_mat and wdl_weights split by rows
    (r % world), the wide lookup and its fixed-point gradients exchanged, the deep-output rows
    of wdl_weights (aliasing wide ids Fw..Fw+H) updated by their owners and re-broadcast.
    Against the fp32 oracle on the global batch: 1e-5 for the fp32 tower, the bf16 tower's
    stated tolerance (test_gpu_parity.py::test_wdl_bf16_tower_tracks_oracle) for bf16."""
    _check_wdl(tmp_path, mode, WORLD)


@pytest.mark.gpu
def test_sharded_wdl_eight_ranks_equals_global_batch(tmp_path):
    """C5 at BASELINE's 8 ranks (sharing cuda:0, gloo-staged): the lazy fp32 Wide&Deep step with
    prefetch against the oracle on the global batch, as the two-rank test."""
    _check_wdl(tmp_path, "gpu_wdl_lazy_pf", 8)


def _check_wdl(tmp_path, mode, world):
    _launch(mode, tmp_path, world)
    bf = "bf16" in mode
    ztol, ptol = (3e-2, 5e-3) if bf else (1e-5, 1e-5)
    cfg = R.make_cfg("wdl", **WKW)
    P = R.init_params(cfg, np.random.default_rng(42))
    opt = R.AdamTF1(cfg, P)
    for step, b in enumerate(wdl_batches(BL * world, STEPS)):
        fw = R.train_step(cfg, P, opt, b)
        z = np.concatenate([np.load(tmp_path / ("rank%d_step%d.npz" % (r, step)))["z"] for r in range(world)])
        np.testing.assert_allclose(z, fw["z"], atol=ztol, rtol=0, err_msg="logits step %d" % step)
        loss = float(np.load(tmp_path / ("rank0_step%d.npz" % step))["loss"])
        assert abs(loss - fw["loss"]) < (5e-3 if bf else 1e-5), (step, loss, fw["loss"])
    d = [np.load(tmp_path / ("rank%d.npz" % r)) for r in range(world)]
    table = np.zeros_like(P["weight_mat"])
    ww = np.zeros_like(P["wdl_weights"][:, 0])
    for e in d:
        table[e["rows"]] = e["table"]
        ww[e["wrows"]] = e["ww"]
    np.testing.assert_allclose(table, P["weight_mat"], atol=ptol, rtol=0)
    np.testing.assert_allclose(ww, P["wdl_weights"][:, 0], atol=ptol, rtol=0)
    np.testing.assert_allclose(d[0]["wb"], P["wdl_bias"], atol=ptol, rtol=0)
    for e in d[1:]:                                             # replicated dense state identical
        np.testing.assert_array_equal(e["W0"], d[0]["W0"])
    # sharded eval on two unseen global batches
    evb = wdl_batches(BL * world, STEPS + 2)[STEPS:]
    all_s, all_y = [], []
    for j, b in enumerate(evb):
        want = 1.0 / (1.0 + np.exp(-R.forward(cfg, P, b)["z"].astype(np.float64)))
        got = np.concatenate([e["s%d" % j] for e in d])
        np.testing.assert_allclose(got, want, atol=ztol, rtol=0, err_msg="eval batch %d" % j)
        all_s.append(want)
        all_y.append(b["label"].reshape(-1))
    assert all(float(e["auc"]) == float(d[0]["auc"]) for e in d)
    assert abs(float(d[0]["auc"]) - R.auc(np.concatenate(all_y), np.concatenate(all_s))) < (2e-3 if bf else 1e-4)


@pytest.mark.parametrize("world", [2, 3])
def test_block_exchange_moves_every_block(world):
    """Exchange.blocks (the sharded step's fixed-capacity exchange, host-staged over gloo here —
    the same block layout dl_shard_exchange moves over RCCL): both directions deliver every
    peer's block to its place and never move a rank's own block."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "exchange_worker.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_status_guard_exits_when_a_peer_is_stuck():
    """The sharded step's status guard (ShardedCTREngine._guard_exit): a rank whose step report
    does not arrive within DLAMD_SHARD_GUARD_S exits non-zero naming its rank, the step and its
    status ring, while its peer sits in a collective it will never complete (a peer stuck in
    RCCL); the launcher then stops the peer, so the job ends within the guard's time instead of
    hanging.  gloo, 2 ranks, CPU."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1", DLAMD_SHARD_GUARD_S="3")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "guard_worker.py")]
    t0 = time.time()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120, cwd=ROOT)
    out = r.stdout + r.stderr
    assert r.returncode != 0 and "guard did not fire" not in out, out[-3000:]
    assert "rank 0/2: the status report of step 3" in out and "exiting with status 75" in out, out[-3000:]
    assert time.time() - t0 < 90, "the stuck peer kept the job alive"
