#!/usr/bin/env python3
"""Flagship benchmark: CML GCN training throughput (windows/s) on N MI355X.

    python bench.py --gpus N --steps K --warmup W          (N > 1: spawns the N rank processes itself)
    torchrun --nproc-per-node N bench.py --gpus N ...      (or one rank per GPU from a launcher)

One process per GPU, data parallel over RCCL (backend "nccl"). Without a launcher (no WORLD_SIZE in the
environment) ``--gpus N > 1`` starts N child processes of this script with RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set; the parent never touches HIP, forwards rank 0's
JSON line (the children inherit stdout) and exits non-zero if any child fails. Under a launcher,
WORLD_SIZE must equal ``--gpus``. Per-GPU batch is the
reference's ``batch_size`` 128 windows (weak scaling: global batch = 128 * N).
Model = the reference CML GCN architecture (GeneralConv 2->16 + mean pooling +
7-layer LSTM TimeLayer 16/16/32/32/64/64/128 + dense head, 188,193 trainables),
random init; data = synthetic CML neighbourhood (23 links, 28 days at 1 min, the
shape of ``cml_raw_example.nc``) windowed with T = 181. Every timed step is a full
training step: on-device window gather, forward, weighted BCE, backward, gradient
all-reduce (N > 1), Adam update.

After the timed region the same line carries the quality half of BASELINE.json's headline metric
("ROC-AUC (5-fold CV)"): the paper's 5-fold CV of the CML GCN and of the graph-less baseline LSTM
(``cv``; folds dealt over the ranks under --gpus N, CML data in which only the neighbourhood tells
rain-shaped anomalies from rain), the integrated-gradients throughput (``ig``), and the second dataset
of the headline (``soilnet``: SoilNet GCN training throughput, B=32 x T=337, same timed-step
contract, and its 5-fold CV against the baseline on the generator with neighbour-only faults).
``--no-cv-line`` / ``--no-ig-line`` / ``--no-soil-line`` skip them. ``--time-layer cnn`` measures the
CNN TimeLayer branch instead (diagnostic line, no side records).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

import torch

REF_GCN_WINDOWS_PER_S = 350.0   # reference GCN predict() on V100 (training not published)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpu_count():
    """GPUs this job may use, counted WITHOUT touching HIP (no ``torch.cuda`` call: on ROCm
    ``torch.cuda.device_count`` falls back to ``hipGetDeviceCount`` when amdsmi is unavailable, which
    would initialise the runtime in a parent that then forks its ranks). Reads the KFD topology
    (``/sys/class/kfd/kfd/topology/nodes/*/properties``: GPU nodes have ``simd_count > 0``) and
    honours ``ROCR_VISIBLE_DEVICES`` / ``HIP_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES``. Returns
    None when the topology is not readable (every rank then checks its own device count)."""
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        nodes = sorted(os.listdir(root), key=lambda s: int(s) if s.isdigit() else 1 << 30)
    except OSError:
        return None
    n = 0
    for nd in nodes:
        try:
            with open(os.path.join(root, nd, "properties")) as f:
                props = dict(ln.split(None, 1) for ln in f.read().splitlines() if len(ln.split(None, 1)) == 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0").strip() or 0) > 0:
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([s for s in v.split(",") if s.strip()]))
    return n


def launch_ranks(n: int, argv) -> int:
    """Run this script as ``n`` rank processes (one per GPU) and wait for all of them. The parent
    never calls into HIP (GPUs are counted from sysfs, :func:`visible_gpu_count`); a child that
    fails takes the others down (exact Popen handles, no pattern kills) and its exit code becomes
    this process's. A SIGTERM / SIGINT of the parent (e.g. a driver timeout) stops every rank too."""
    ndev = visible_gpu_count()
    if ndev and n > ndev:
        print(f"bench.py: --gpus {n} but only {ndev} GPUs are visible", file=sys.stderr)
        return 2
    port = _free_port()
    procs = []

    def _raise(signum, _frame):
        raise KeyboardInterrupt(f"signal {signum}")

    prev = {s: signal.signal(s, _raise) for s in (signal.SIGTERM, signal.SIGINT)}
    rc = 0
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            if not ndev:                  # CPU (gloo) rehearsal: do not oversubscribe the cores
                env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // n)))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 1
                    print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                          file=sys.stderr)
                    for q in live:
                        q.terminate()
            time.sleep(0.05)
    except KeyboardInterrupt as e:
        print(f"bench.py: interrupted ({e}); stopping every rank", file=sys.stderr)
        rc = rc or 130
    finally:
        for p in procs:                   # terminate, then kill, whatever is still running
            if p.poll() is None:
                p.terminate()
        deadline = time.time() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for s, h in prev.items():
            signal.signal(s, h)
    return rc


def measure_ig(args, trainer, dev, world, rank, D):
    """BASELINE.json config (v): integrated-gradients attribution of the CML GCN (m_steps = 100: 101
    forward + backward passes per explained window) on the trained-for-a-few-steps model. Batches are
    dealt round-robin over the ranks (batch i on rank i % world, as the reference deals them over
    workers, ``xai/libs/integrated_gradients.py:180-187,432-448``); every rank explains ``calls`` of
    them. Aggregate explained windows/s over the max-over-ranks time."""
    from gnnqc.xai.ig import IntegratedGradients
    gpu = dev.type == "cuda"
    max_rows = 32768
    # windows per call: one full path chunk (max_rows // (m_steps + 1) = 324 windows x 101 points = 2,046
    # sixteen-sequence tiles, whole rounds of the recurrence grids; 256 windows leave a 16 % tail round,
    # profiles/r6_ig_windows_per_call.txt)
    B = args.ig_windows or (max_rows // 101 if gpu else 4)
    nb = args.ig_calls or (6 if gpu else 1)
    store, model = trainer.store, trainer.model
    expl = IntegratedGradients(model, "cml", m_steps=100, max_rows=max_rows)
    span = max(1, store.n_windows - B)

    def ig_batch(j):                  # this rank's j-th batch = global batch rank + world * j
        s0 = ((rank + world * j) * B) % span
        return store.gather(torch.arange(s0, s0 + B, device=dev))

    warm = 2 if gpu else 0            # graph capture + one replay outside the timed region
    for j in range(warm):
        expl.attribute(ig_batch(j))
    D.barrier()
    if gpu:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(nb):
        expl.attribute(ig_batch(warm + j))
    if gpu:
        torch.cuda.synchronize()
    D.barrier()
    dti = D.max_over_ranks(time.perf_counter() - t0)
    return {"metric": "integrated-gradients explained windows/s (CML GCN, m_steps=100, 101 passes per window)",
            "value": round(world * nb * B / dti, 2), "windows_per_call": B, "calls_per_rank": nb,
            "n_ranks": world, "ms_per_call": round(1e3 * dti / nb, 3),
            "sharding": "round-robin batches over ranks" if world > 1 else "one rank"}


# 5-fold CV mean ROC-AUC on the paper's data (README.md:10)
REF_CV_AUC = {"cml": {"gcn": 0.941, "baseline": 0.885}, "soilnet": {"gcn": 0.858, "baseline": 0.816}}


def cv_data(args, ds: str, gpu: bool):
    """(pc, ws, description) of the CV data. CML: the reference example shape (23 links x 28 days @1 min,
    4 flagged links) from ``make_cml_raw`` with rain-shaped wet-antenna anomalies (``--cv-rainlike`` of
    the anomaly events; the flagged link alone cannot tell them from rain, its neighbours can: SURVEY
    §7.4 item 4) and ``--cv-rain-fraction`` rain. SoilNet: 40 boxes x 365 days @15 min from
    ``make_soilnet_raw(spatial_fault_frac=0.5)`` (half of the faults only visible against the
    neighbours; the data of ``profiles/r2_cv_soilnet_spatial.json``)."""
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.synthetic import make_cml_raw, make_soilnet_raw
    pc = C.normalize_preproc(C.default(f"preprocessing_{ds}"))
    if ds == "cml":
        sensors = args.cv_sensors or (23 if gpu else args.sensors)
        days = args.cv_days or (28 if gpu else min(args.days, 3))
        flagged = args.cv_flagged or (4 if gpu else 1)
        raw = make_cml_raw(n_sensors=sensors, n_flagged=flagged, n_minutes=int(days * 1440), seed=0,
                           rainlike_frac=args.cv_rainlike, rain_fraction=args.cv_rain_fraction)
        desc = ("synthetic CML: %d links x %g days @1min, %d flagged links, %.0f%% of the anomaly events rain-shaped "
                "(seen by the flagged link only), rain_fraction %.2f" % (sensors, days, flagged,
                                                                      100 * args.cv_rainlike, args.cv_rain_fraction))
    else:
        boxes = args.soil_cv_boxes or (40 if gpu else 3)
        days = args.soil_cv_days or (365 if gpu else 5)
        raw = make_soilnet_raw(n_boxes=boxes, n_time=int(days * 96), seed=0, spatial_fault_frac=0.5)
        desc = ("synthetic SoilNet: %d boxes x %g days @15min, make_soilnet_raw(spatial_fault_frac=0.5): half of "
                "the faults only visible against the neighbours" % (boxes, days))
    pc["min_date"], pc["max_date"] = str(raw.time[0]), str(raw.time[-1])
    ws = create_windows_dataset(pc, raw=raw)
    return pc, ws, desc + ", T=%d, %d windows" % (ws.seq_len, ws.n_windows)


def measure_cv(args, dev, world, D, ds: str = "cml"):
    """The quality half of BASELINE.json's headline metric: the paper's 5-fold cross-validation
    protocol (contiguous folds of ``load_dataset_CV``, ``xai/libs/preprocessing_functions.py:804-836``;
    CV training monitors ``loss``, ``xai/libs/fit_model.py:94-99``) for the GCN AND the graph-less
    baseline LSTM, each fold a fresh random-init model trained for the config's epochs at the bench
    dtype and scored by exact ROC-AUC on its held-out fold (``gnnqc.train.cv.run_cv``). Runs after the
    timed region (data: :func:`cv_data`). Under ``--gpus N`` the folds are dealt over the ranks (fold f
    on rank f % N, no collective inside a fold) and gathered. The GCN - baseline difference is
    reported per fold (paired: both models see the same folds)."""
    from gnnqc import config as C
    from gnnqc.data.store import DeviceStore
    from gnnqc.train.cv import run_cv
    gpu = dev.type == "cuda"
    folds = args.cv_folds or (5 if gpu else 2)
    pc, ws, desc = cv_data(args, ds, gpu)
    mc = C.default(f"model_{ds}")
    mc.runtime.compute_dtype = args.dtype
    if args.cv_epochs or not gpu:
        mc.epochs = int(args.cv_epochs or 1)
    store = DeviceStore(ws, "rolling_median" if ds == "cml" else "scale_range", pc.graph, device=dev)
    D.barrier()
    t0 = time.perf_counter()
    out = {"protocol": "%d-fold CV (contiguous folds, load_dataset_CV), fresh random-init model per fold, "
                       "exact ROC-AUC on the held-out fold" % folds,
           "data": desc, "folds": folds, "epochs": int(mc.epochs), "dtype": args.dtype,
           "fold_per_rank": world > 1}
    for name, baseline in (("gcn", False), ("baseline", True)):
        def progress(r, name=name):       # (stderr: stdout carries the one JSON line)
            print("bench.py: cv %s %s fold %d auc %.4f (%.1f s)" % (ds, name, r["fold"], r["auc"], r["seconds"]),
                  file=sys.stderr, flush=True)
        s = run_cv(pc, mc, ws, folds=folds, baseline=baseline, store=store, seed=0, verbose=0,
                   fold_per_rank=world > 1, progress=progress)
        out[f"{name}_mean_auc"] = round(s["mean_auc"], 5)
        out[f"{name}_std"] = round(s["std_auc"], 5)
        out[f"{name}_fold_auc"] = [round(r["auc"], 5) for r in s["per_fold"]]
        out[f"{name}_folds_run"] = s["folds_run"]
        out[f"{name}_mean_mcc"] = round(s["mean_mcc"], 5)
    if gpu:
        torch.cuda.synchronize()
    D.barrier()
    out["seconds"] = round(D.max_over_ranks(time.perf_counter() - t0), 2)
    diff = [round(g - b, 5) for g, b in zip(out["gcn_fold_auc"], out["baseline_fold_auc"])]
    out["gcn_minus_baseline_auc"] = round(out["gcn_mean_auc"] - out["baseline_mean_auc"], 5)
    out["gcn_minus_baseline_fold_auc"] = diff
    out["gcn_wins_folds"] = "%d/%d" % (sum(d > 0 for d in diff), len(diff))
    out["paper_mean_auc"] = dict(REF_CV_AUC[ds])
    out["paper_parity"] = ("unpinned: synthetic data here, the paper's numbers are on its real %s data"
                           % ("CML" if ds == "cml" else "SoilNet"))
    return out


def safe_cv(args, dev, world, D, ds):
    """:func:`measure_cv`, with a failure reported inside the JSON line on one rank (a multi-rank
    failure is raised: the other ranks would otherwise wait in the fold gather)."""
    try:
        return measure_cv(args, dev, world, D, ds)
    except Exception as e:            # noqa: BLE001
        if world > 1:
            raise
        import traceback
        traceback.print_exc()
        return {"error": f"{type(e).__name__}: {e}"}


def train_data(args, ds: str, sensors: int, days: int):
    """(pc, mc, ws) of a throughput measurement: synthetic data of the reference example shapes
    (CML 23 links x 28 days @1 min; SoilNet 40 boxes x 89 days @15 min), config batch size."""
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.synthetic import make_cml_raw, make_soilnet_raw
    pc = C.normalize_preproc(C.default(f"preprocessing_{ds}"))
    mc = C.default(f"model_{ds}")
    mc.runtime.compute_dtype = args.dtype
    if args.time_layer == "cnn":
        # CNN TimeLayer branch (create_model.py:80-101): Conv1D(same)+LeakyReLU stacks, GAP
        mc.sequence_layer.algorithm = "cnn"
        mc.sequence_layer.kernel_size = 5
    if ds == "soilnet":
        raw = make_soilnet_raw(n_boxes=sensors, n_time=days * 96, seed=7)
        pc["min_date"], pc["max_date"] = str(raw.time[0]), str(raw.time[-1])
    else:
        raw = make_cml_raw(n_sensors=sensors, n_minutes=days * 1440, seed=7)
    return pc, mc, create_windows_dataset(pc, raw=raw)


def measure_train(args, ds, pc, mc, ws, graph_cfg, batch, dev, world, rank, D, baseline=False):
    """Build store / model / trainer for one dataset and adjacency rule, warm up, time args.steps full
    training steps (max over ranks). Returns (seconds, trainer, loss, trainable params)."""
    from gnnqc.data.store import DeviceLoader, DeviceStore
    from gnnqc.models import BaselineClassifier, GCNClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    from gnnqc.train.loss import calculate_weights
    tr = list(range(ws.n_windows))          # throughput: every window is a training window
    store = DeviceStore(ws, "scale_range" if ds == "soilnet" else "rolling_median", graph_cfg, device=dev)
    loader = DeviceLoader(store, tr, batch, shuffle=True, seed=44, rank=rank, world_size=world, drop_last=True)
    torch.manual_seed(1234)
    model = (BaselineClassifier if baseline else GCNClassifier)(mc, pc).to(dev)
    n_params = sum(p.numel() for p in model.parameters() if p.requires_grad)
    opt = make_optimizer("adam", model.parameters(), mc.learning_rate)
    D.broadcast_module(model)
    trainer = Trainer(model, store, opt, calculate_weights(mc), baseline, use_graph=not args.no_graph,
                      batch_size=batch)
    rows = loader.batch_ids()                 # [n_batches, B] device tensor, no host sync while stepping
    # every one of the steps is a full training step (gather, forward, backward, guarded Adam); chunks of
    # trainer.graph_steps of them replay one multi-step HIP graph
    trainer.prepare_graphs(rows)              # graph captures happen here, never inside the timed steps
    trainer.train_steps(rows, 0, args.warmup)
    trainer._comm_events = []
    D.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    trainer.train_steps(rows, args.warmup, args.steps)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    D.barrier()
    dt = D.max_over_ranks(time.perf_counter() - t0)
    return dt, trainer, float(trainer.last_loss.item()), n_params


def _release(dev):
    import gc
    gc.collect()
    if dev.type == "cuda":
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


def model_desc(ds, baseline, time_layer):
    if baseline:
        return ("SoilNet" if ds == "soilnet" else "CML") + " baseline LSTM"
    tl = "Conv1D TimeLayer k5 f16 n_stacks2" if time_layer == "cnn" else "LSTM TimeLayer f16 n_stacks2"
    return "%s GCN (GeneralConv16+%s+%s+dense64)" % ("SoilNet" if ds == "soilnet" else "CML",
                                                   "per-node sequences" if ds == "soilnet" else "mean pool", tl)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None, help="windows per GPU per step (default: config batch_size,"
                    " CML 128 / SoilNet 32)")
    ap.add_argument("--model", choices=["gcn", "baseline"], default="gcn")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--no-graph", action="store_true", help="disable HIP-graph capture of the step")
    ap.add_argument("--ds", choices=["cml", "soilnet"], default="cml",
                    help="cml = the headline config; soilnet = SoilNet only (T=337, per-node sequences)")
    ap.add_argument("--time-layer", choices=["lstm", "cnn"], default="lstm",
                    help="cnn = diagnostic: the CNN TimeLayer branch (Conv1D k=5 + LeakyReLU stacks + GAP); not the "
                         "headline config, no side records")
    ap.add_argument("--sensors", type=int, default=None, help="default: 23 CML links / 40 SoilNet boxes")
    ap.add_argument("--days", type=int, default=None, help="default: 28 (CML) / 89 (SoilNet)")
    ap.add_argument("--adjacency", choices=["radius", "knn"], default="radius",
                    help="radius = the reference's rule (max_sample_distance, SURVEY 5.11.4); knn = symmetrised "
                         "k-nearest-neighbour graph (BASELINE.json's 'k=5')")
    ap.add_argument("--k", type=int, default=5, help="neighbours per node for --adjacency knn")
    ap.add_argument("--no-knn-line", dest="knn_line", action="store_false",
                    help="skip the second measurement on the k=5 graph (reported as 'knn5' in the JSON line)")
    ap.add_argument("--no-ig-line", dest="ig_line", action="store_false",
                    help="skip the integrated-gradients throughput (BASELINE.json config v; reported as 'ig' in "
                         "the JSON line; under DP every rank explains its own shard of the batches)")
    ap.add_argument("--ig-windows", type=int, default=None,
                    help="windows per attribute() call (default 324 = one 32768-row path chunk on a GPU, 4 on the CPU)")
    ap.add_argument("--ig-calls", type=int, default=None,
                    help="timed attribute() calls per rank (default 6 on a GPU, 1 on the CPU)")
    ap.add_argument("--no-cv-line", dest="cv_line", action="store_false",
                    help="skip the 5-fold CV ROC-AUC of the GCN and baseline (reported as 'cv' in the JSON line, and "
                         "inside 'soilnet')")
    ap.add_argument("--cv-folds", type=int, default=None, help="CV folds (default 5 on a GPU, 2 on the CPU)")
    ap.add_argument("--cv-epochs", type=int, default=None, help="epochs per fold (default: the model config's, "
                    "1 on the CPU)")
    ap.add_argument("--cv-sensors", type=int, default=None, help="CML CV data: links (default 23)")
    ap.add_argument("--cv-days", type=float, default=None, help="CML CV data: days (default 28)")
    ap.add_argument("--cv-flagged", type=int, default=None, help="CML CV data: flagged links (default 4)")
    ap.add_argument("--cv-rainlike", type=float, default=0.85,
                    help="CML CV data: fraction of the anomaly events that are rain-shaped (flagged link only)")
    ap.add_argument("--cv-rain-fraction", type=float, default=0.15, help="CML CV data: rain_fraction")
    ap.add_argument("--no-soil-line", dest="soil_line", action="store_false",
                    help="skip the SoilNet sub-record of the CML line (training throughput B=32 T=337 and its 5-fold "
                         "CV, reported as 'soilnet')")
    ap.add_argument("--soil-sensors", type=int, default=None, help="SoilNet throughput data: boxes (default 40; "
                    "3 on the CPU)")
    ap.add_argument("--soil-days", type=int, default=None, help="SoilNet throughput data: days (default 89; 5 on "
                    "the CPU)")
    ap.add_argument("--soil-cv-boxes", type=int, default=None, help="SoilNet CV data: boxes (default 40; 3 on the CPU)")
    ap.add_argument("--soil-cv-days", type=float, default=None, help="SoilNet CV data: days (default 365; 5 on the CPU)")
    args = ap.parse_args(argv)

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: WORLD_SIZE={env_world} from the launcher but --gpus {args.gpus}", file=sys.stderr)
        return 2
    if env_world is None and args.gpus > 1:
        return launch_ranks(args.gpus, argv)
    if args.gpus > 1 and torch.cuda.is_available() and torch.cuda.device_count() < args.gpus:
        # (a rank process may initialise HIP; the spawning parent never does)
        print(f"bench.py: --gpus {args.gpus} but only {torch.cuda.device_count()} GPUs are visible", file=sys.stderr)
        return 2

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from gnnqc.parallel import dist as D

    dev = D.init_distributed()
    world, rank = D.world_size(), D.rank()
    if os.environ.get("GNNQC_BENCH_FAIL_RANK") == str(rank):    # fault injection (tests/test_bench_launch.py)
        print(f"bench.py: rank {rank} failing on request", file=sys.stderr)
        return 3
    gpu = dev.type == "cuda"
    torch.manual_seed(1234)
    soil = args.ds == "soilnet"
    cnn = args.time_layer == "cnn"
    baseline = args.model == "baseline"
    args.sensors = args.sensors or (40 if soil else 23)
    args.days = args.days or (89 if soil else 28)
    pc, mc, ws = train_data(args, args.ds, args.sensors, args.days)
    args.batch = args.batch or int(pc.batch_size)
    pc.batch_size = args.batch
    pc.graph["adjacency"] = args.adjacency
    pc.graph["k"] = int(args.k)
    adj_desc = (f"knn(k={args.k})" if args.adjacency == "knn" else
                f"radius(max_sample_distance={pc.graph['max_sample_distance']})")

    dt, trainer, loss, n_params = measure_train(args, args.ds, pc, mc, ws, pc.graph, args.batch, dev, world, rank, D,
                                                baseline)
    comm_us = None
    if trainer._comm_events:             # N > 1, eager layout: HIP events around the timed all-reduces
        comm_us = 1e3 * sum(a.elapsed_time(b) for a, b in trainer._comm_events) / len(trainer._comm_events)
    elif trainer.collective:             # in-graph all-reduce: the same collective timed on its own, after
        comm_us = trainer.measure_allreduce()
    if comm_us is not None:
        comm_us = D.max_over_ranks(comm_us)
    graph_steps = trainer.graph_steps if trainer._multi_ok() else 1
    use_graph, peer, peer_fused = trainer.use_graph, trainer.peer is not None, trainer.peer_fused()
    dp_graph = trainer.dp_graph and trainer._multi_ok()
    windows = args.steps * args.batch * world
    value = windows / dt
    side = not soil and not cnn            # the side records ride on the headline (CML, LSTM) line
    knn = ig = cv = soil_rec = None
    if side and args.knn_line and args.adjacency == "radius":
        # BASELINE.json names the CML graph "k=5": the same measurement on the symmetrised
        # 5-nearest-neighbour graph, reported inside the one JSON line
        g5 = dict(pc.graph)
        g5["adjacency"], g5["k"] = "knn", 5
        dt5, _, loss5, _ = measure_train(args, "cml", pc, mc, ws, g5, args.batch, dev, world, rank, D, baseline)
        knn = {"adjacency": "knn(k=5)", "value": round(windows / dt5, 2),
               "ms_per_step": round(1000.0 * dt5 / args.steps, 4), "final_loss": round(loss5, 5)}
        _release(dev)
    if side and args.ig_line and not baseline:
        ig = measure_ig(args, trainer, dev, world, rank, D)
    del trainer
    _release(dev)
    if side and args.cv_line:
        cv = safe_cv(args, dev, world, D, "cml")
        _release(dev)
    if side and args.soil_line:
        # BASELINE.json's headline names both datasets (CML 0.941 / SoilNet 0.858): the SoilNet GCN's
        # training throughput (same timed-step contract) and its 5-fold CV against the baseline
        soil_shape = (args.soil_sensors or (40 if gpu else 3), args.soil_days or (89 if gpu else 5))
        spc, smc, sws = train_data(args, "soilnet", *soil_shape)
        sb = int(spc.batch_size)
        sdt, strainer, sloss, snp = measure_train(args, "soilnet", spc, smc, sws, spc.graph, sb, dev, world, rank, D,
                                                  baseline)
        sgs = strainer.graph_steps if strainer._multi_ok() else 1
        del strainer
        _release(dev)
        soil_rec = {"metric": "train windows/s, SoilNet GCN (B=%d windows x node sequences, T=%d)" % (sb, sws.seq_len),
                    "value": round(args.steps * sb * world / sdt, 2), "unit": "train windows/s (whole job)",
                    "ms_per_step": round(1000.0 * sdt / args.steps, 4), "steps": args.steps, "warmup": args.warmup,
                    "global_batch": sb * world, "seq_len": sws.seq_len, "graph_steps": sgs,
                    "model": model_desc("soilnet", baseline, args.time_layer), "trainable_params": snp,
                    "final_loss": round(sloss, 5),
                    "data": "synthetic (SoilNet example shape: %d boxes x %d days @15min), random-init weights"
                            % soil_shape}
        if args.cv_line:
            soil_rec["cv"] = safe_cv(args, dev, world, D, "soilnet")
            _release(dev)
    if rank == 0:
        out = {
            "metric": ("train windows/sec, SoilNet GCN (diagnostic; not the headline metric)" if soil else
                       "train windows/sec, CML GCN with the CNN TimeLayer (diagnostic; not the headline metric)"
                       if cnn else "ROC-AUC (5-fold CV) + train windows/sec, CML GCN at 1/2/4/8 MI355X"),
            "value": round(value, 2),
            "unit": "train windows/s (whole job)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * dt / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            # BASELINE.json publishes no training throughput; the only reference speed is GCN predict()
            # incl. tf.data parsing on a V100 (BASELINE.md nb:321), which is not the same metric
            "vs_baseline": None,
            "vs_baseline_basis": "no published reference training windows/s (BASELINE.json 'published' is "
                                 "empty); context only: reference GCN predict() %.0f windows/s on V100"
                                 % REF_GCN_WINDOWS_PER_S,
            "dtype": args.dtype,
            "data": ("synthetic (SoilNet: %d boxes x %d days @15min, T=%d), random-init weights" if soil else
                     "synthetic (CML example shape: %d links x %d days @1min, T=%d), random-init weights")
                    % (args.sensors, args.days, ws.seq_len),
            "config": {
                "model": model_desc(args.ds, baseline, args.time_layer),
                "global_batch": args.batch * world,
                "seq_len": ws.seq_len,
                "parallelism": f"dp{world}",
                "adjacency": adj_desc,
                "graph_steps": graph_steps,
                "trainable_params": n_params,
                "hip_graph": use_graph,
                "final_loss": round(loss, 5),
            },
        }
        if knn is not None:
            out["knn5"] = knn
        if ig is not None:
            out["ig"] = ig
        if cv is not None:
            out["cv"] = cv
        if soil_rec is not None:
            out["soilnet"] = soil_rec
        if comm_us is not None:
            # the collective of the timed steps, run on its own (in-graph collectives cannot be timed one
            # by one), plus the setup-time comparison of both modes when the peer kernel was considered
            from gnnqc.parallel.peer import LAST_SELECTION
            out["allreduce_us"] = round(comm_us, 2)
            out["allreduce_mode"] = (("peer one-shot xGMI" if peer else "RCCL") +
                                     (" fused into the Adam launch" if peer_fused else "") +
                                     (" in-graph (timed standalone)" if dp_graph else " eager"))
            if LAST_SELECTION:
                out["allreduce_selection"] = {k: (round(v, 2) if isinstance(v, float) else v)
                                              for k, v in LAST_SELECTION.items()}
        print(json.dumps(out), flush=True)
    D.destroy()


if __name__ == "__main__":
    sys.exit(main() or 0)
