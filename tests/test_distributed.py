"""Data-parallel correctness on CPU with gloo (world_size 2): the RCCL path by construction."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(seed=3):
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.store import DeviceStore
    from gnnqc.data.synthetic import make_cml_raw
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    pc.timestep_before, pc.timestep_after = 30, 15
    ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=8, n_minutes=4 * 1440, seed=seed))
    st = DeviceStore(ws, "rolling_median", pc.graph)
    mc = C.default("model_cml")
    mc.baseline_model.filter_1_size = 8
    return pc, mc, st


def _worker(rank, world, port, out_dir, ids):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    from gnnqc.models import BaselineClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.parallel import dist as D
    from gnnqc.train.engine import Trainer
    D.init_distributed(device="cpu")
    pc, mc, st = _setup()
    torch.manual_seed(rank + 100)            # different init per rank: broadcast must fix it
    m = BaselineClassifier(mc, pc)
    opt = make_optimizer("adam", m.parameters(), 1e-3)
    D.broadcast_module(m)
    t = Trainer(m, st, opt, {0: 1.0, 1: 5.0}, baseline=True, use_graph=False, batch_size=len(ids[rank]))
    t._body(torch.tensor(ids[rank]), with_opt=False)
    D.all_reduce_(opt.flat_g)
    g = (opt.flat_g / world).numpy()
    np.save(os.path.join(out_dir, f"g{rank}.npy"), g)
    np.save(os.path.join(out_dir, f"p{rank}.npy"), opt.flat_p.detach().numpy())
    D.destroy()


def test_dp_gradients_equal_single_process_large_batch(tmp_path):
    ids = [list(range(0, 16)), list(range(16, 32))]
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path), ids), nprocs=2, join=True)
    g0, g1 = np.load(tmp_path / "g0.npy"), np.load(tmp_path / "g1.npy")
    p0, p1 = np.load(tmp_path / "p0.npy"), np.load(tmp_path / "p1.npy")
    assert np.array_equal(p0, p1)            # broadcast made ranks identical
    assert np.allclose(g0, g1)
    # single process on the union batch, same weights
    from gnnqc.models import BaselineClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    pc, mc, st = _setup()
    m = BaselineClassifier(mc, pc)
    opt = make_optimizer("adam", m.parameters(), 1e-3)
    opt.flat_p.copy_(torch.from_numpy(p0))
    t = Trainer(m, st, opt, {0: 1.0, 1: 5.0}, baseline=True, use_graph=False, batch_size=32)
    t._body(torch.tensor(ids[0] + ids[1]), with_opt=False)
    ref = opt.flat_g.numpy()
    assert np.allclose(g0, ref, rtol=1e-4, atol=1e-6), np.abs(g0 - ref).max()


@pytest.mark.slow
def test_bench_runs_with_two_gloo_ranks():
    port = _free_port()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--sensors", "8", "--days", "3", "--no-soil-line"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 256 and out["value"] > 0


def _gcn_setup(ds="cml"):
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.store import DeviceStore
    from gnnqc.data.synthetic import make_cml_raw, make_soilnet_raw
    if ds == "soilnet":          # network-wide SoilNet: one prediction per node (BASELINE config iii)
        pc = C.normalize_preproc(C.default("preprocessing_soilnet"))
        pc.timestep_before, pc.timestep_after = 24 * 60, 6 * 60
        raw = make_soilnet_raw(n_boxes=3, n_time=8 * 96, seed=6)
        pc["min_date"], pc["max_date"] = str(raw.time[0]), str(raw.time[-1])
        ws = create_windows_dataset(pc, raw=raw)
        st = DeviceStore(ws, "scale_range", pc.graph)
        mc = C.default("model_soilnet")
        mc.sequence_layer.filter_1_size = 4
        return pc, mc, st
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    pc.timestep_before, pc.timestep_after = 30, 15
    ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=8, n_minutes=4 * 1440, seed=5))
    st = DeviceStore(ws, "rolling_median", pc.graph)
    mc = C.default("model_cml")
    mc.sequence_layer.filter_1_size = 4          # small TimeLayer: fast on CPU, same structure
    mc.dense.units = 64
    return pc, mc, st


def _gcn_worker(rank, world, port, out_dir, ids, n_epoch_batches, ds="cml"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    from gnnqc.data.store import DeviceLoader
    from gnnqc.models import GCNClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.parallel import dist as D
    from gnnqc.train.engine import Trainer
    D.init_distributed(device="cpu")
    pc, mc, st = _gcn_setup(ds)
    torch.manual_seed(rank + 200)             # different init per rank: broadcast must fix it
    m = GCNClassifier(mc, pc)
    opt = make_optimizer("adam", m.parameters(), 1e-3)
    D.broadcast_module(m)
    np.save(os.path.join(out_dir, f"p0_{rank}.npy"), opt.flat_p.detach().numpy().copy())
    t = Trainer(m, st, opt, {0: 1.0, 1: 5.0}, baseline=False, use_graph=False, batch_size=len(ids[rank]))
    # one gradient: this rank's shard, all-reduced mean
    t._body(torch.tensor(ids[rank]), with_opt=False)
    D.all_reduce_(opt.flat_g)
    np.save(os.path.join(out_dir, f"g{rank}.npy"), (opt.flat_g / world).numpy())
    opt.zero_grad()
    # an epoch of DP training: parameters and BN statistics must agree on every rank
    loader = DeviceLoader(st, list(range(n_epoch_batches * 8 * world)), 8, shuffle=True, seed=3, rank=rank,
                          world_size=world, drop_last=True)
    t.batch_size = 8
    t.train_epoch(loader, 0)
    np.save(os.path.join(out_dir, f"p{rank}.npy"), opt.flat_p.detach().numpy())
    bufs = torch.cat([b.reshape(-1).double() for b in m.buffers() if b.is_floating_point()])
    np.save(os.path.join(out_dir, f"b{rank}.npy"), bufs.numpy())
    D.destroy()


@pytest.mark.parametrize("world,ds", [(2, "cml"), (4, "cml"), (2, "soilnet"), (4, "soilnet")])
def test_gcn_dp_gradients_and_bn_statistics(tmp_path, world, ds):
    """GCNClassifier under data parallelism (gloo, the RCCL path by construction): the all-reduced
    gradient equals the mean of single-process per-shard gradients (BatchNorm batch statistics are
    per replica, as in Keras MirroredStrategy), and after an epoch parameters and BN moving
    statistics are identical on every rank (the epoch-end BN average, gnnqc.parallel.dist)."""
    per = 6
    ids = [list(range(r * per, (r + 1) * per)) for r in range(world)]
    port = _free_port()
    mp.spawn(_gcn_worker, args=(world, port, str(tmp_path), ids, 2, ds), nprocs=world, join=True)
    p0 = [np.load(tmp_path / f"p0_{r}.npy") for r in range(world)]
    for r in range(1, world):
        assert np.array_equal(p0[r], p0[0])
    gs = [np.load(tmp_path / f"g{r}.npy") for r in range(world)]
    for r in range(1, world):
        assert np.allclose(gs[r], gs[0])
    # reference: one process, the same weights, each shard's gradient, averaged
    from gnnqc.models import GCNClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    pc, mc, st = _gcn_setup(ds)
    m = GCNClassifier(mc, pc)
    opt = make_optimizer("adam", m.parameters(), 1e-3)
    opt.flat_p.copy_(torch.from_numpy(p0[0]))
    t = Trainer(m, st, opt, {0: 1.0, 1: 5.0}, baseline=False, use_graph=False, batch_size=per)
    ref = np.zeros_like(gs[0])
    for r in range(world):
        t._body(torch.tensor(ids[r]), with_opt=False)
        ref += opt.flat_g.numpy() / world
    assert np.allclose(gs[0], ref, rtol=1e-4, atol=1e-6), np.abs(gs[0] - ref).max()
    ps = [np.load(tmp_path / f"p{r}.npy") for r in range(world)]
    bs = [np.load(tmp_path / f"b{r}.npy") for r in range(world)]
    for r in range(1, world):
        assert np.array_equal(ps[r], ps[0])
        assert np.allclose(bs[r], bs[0], rtol=0, atol=1e-12)
    assert not np.array_equal(ps[0], p0[0])


def _cv_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import json
    from gnnqc.parallel import dist as D
    from gnnqc.train.cv import run_cv
    D.init_distributed(device="cpu")
    pc, mc, st = _gcn_setup()
    mc["epochs"] = 1
    s = run_cv(pc, mc, st.windows, folds=3, store=st, seed=5, verbose=0, fold_per_rank=True)
    with open(os.path.join(out_dir, f"cv{rank}.json"), "w") as f:
        json.dump({"folds_run": s["folds_run"], "auc": [r["auc"] for r in s["per_fold"]],
                   "loss": [r["final_train_loss"] for r in s["per_fold"]]}, f)
    D.destroy()


def test_cv_fold_per_rank(tmp_path):
    """``cv --fold-per-gpu``: 2 ranks train 3 folds between them (rank 0: folds 0, 2; rank 1: fold 1)
    without any collective in the steps; every rank ends with all folds, identical to running the
    folds one by one in a single process."""
    import json
    port = _free_port()
    mp.spawn(_cv_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    a = json.load(open(tmp_path / "cv0.json"))
    b = json.load(open(tmp_path / "cv1.json"))
    assert a == b and a["folds_run"] == [0, 1, 2]
    from gnnqc.train.cv import run_cv
    pc, mc, st = _gcn_setup()
    mc["epochs"] = 1
    ref = run_cv(pc, mc, st.windows, folds=3, store=st, seed=5, verbose=0)
    assert np.allclose([r["final_train_loss"] for r in ref["per_fold"]], a["loss"], rtol=1e-5)
    assert np.allclose([r["auc"] for r in ref["per_fold"]], a["auc"], rtol=1e-6, equal_nan=True)
