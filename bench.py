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
(``cv``; folds dealt over the ranks under --gpus N), and the integrated-gradients throughput
(``ig``). ``--no-cv-line`` / ``--no-ig-line`` skip them.

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
    B = args.ig_windows or (256 if gpu else 4)
    nb = args.ig_calls or (6 if gpu else 1)
    store, model = trainer.store, trainer.model
    expl = IntegratedGradients(model, "cml", m_steps=100, max_rows=32768)
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


REF_CV_AUC = {"gcn": 0.941, "baseline": 0.885}   # CML 5-fold CV mean ROC-AUC (README.md:10)


def measure_cv(args, dev, world, D):
    """The quality half of BASELINE.json's headline metric: the paper's 5-fold cross-validation
    protocol (contiguous folds of ``load_dataset_CV``, ``xai/libs/preprocessing_functions.py:804-836``;
    CV training monitors ``loss``, ``xai/libs/fit_model.py:94-99``) for the CML GCN AND the graph-less
    baseline LSTM, each fold a fresh random-init model trained for the config's epochs at the bench
    dtype and scored by exact ROC-AUC on its held-out fold (``gnnqc.train.cv.run_cv``). Runs after the
    timed region, on the CV data shape of ``scripts/cv_headline.sh`` (synthetic CML, 23 links x 28
    days, 4 flagged links). Under ``--gpus N`` the folds are dealt over the ranks (fold f on rank
    f % N, no collective inside a fold) and gathered."""
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.store import DeviceStore
    from gnnqc.data.synthetic import make_cml_raw
    from gnnqc.train.cv import run_cv
    gpu = dev.type == "cuda"
    folds = args.cv_folds or (5 if gpu else 2)
    sensors = args.cv_sensors or (23 if gpu else args.sensors)
    days = args.cv_days or (28 if gpu else min(args.days, 3))
    flagged = args.cv_flagged or (4 if gpu else 1)
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    mc = C.default("model_cml")
    mc.runtime.compute_dtype = args.dtype
    if args.cv_epochs or not gpu:
        mc.epochs = int(args.cv_epochs or 1)
    raw = make_cml_raw(n_sensors=sensors, n_flagged=flagged, n_minutes=int(days * 1440), seed=0)
    pc["min_date"], pc["max_date"] = str(raw.time[0]), str(raw.time[-1])
    ws = create_windows_dataset(pc, raw=raw)
    store = DeviceStore(ws, "rolling_median", pc.graph, device=dev)
    D.barrier()
    t0 = time.perf_counter()
    out = {"protocol": "%d-fold CV (contiguous folds, load_dataset_CV), fresh random-init model per fold, "
                       "exact ROC-AUC on the held-out fold" % folds,
           "data": "synthetic CML: %d links x %g days @1min, %d flagged links, T=%d, %d windows"
                   % (sensors, days, flagged, ws.seq_len, ws.n_windows),
           "folds": folds, "epochs": int(mc.epochs), "dtype": args.dtype,
           "fold_per_rank": world > 1}
    for name, baseline in (("gcn", False), ("baseline", True)):
        s = run_cv(pc, mc, ws, folds=folds, baseline=baseline, store=store, seed=0, verbose=0,
                   fold_per_rank=world > 1)
        out[f"{name}_mean_auc"] = round(s["mean_auc"], 5)
        out[f"{name}_std"] = round(s["std_auc"], 5)
        out[f"{name}_fold_auc"] = [round(r["auc"], 5) for r in s["per_fold"]]
        out[f"{name}_folds_run"] = s["folds_run"]
        out[f"{name}_mean_mcc"] = round(s["mean_mcc"], 5)
    if gpu:
        torch.cuda.synchronize()
    D.barrier()
    out["seconds"] = round(D.max_over_ranks(time.perf_counter() - t0), 2)
    out["gcn_minus_baseline_auc"] = round(out["gcn_mean_auc"] - out["baseline_mean_auc"], 5)
    out["reference_mean_auc"] = dict(REF_CV_AUC)
    out["vs_reference_gcn_auc"] = round(out["gcn_mean_auc"] / REF_CV_AUC["gcn"], 4)
    return out


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
                    help="cml = the headline config; soilnet = diagnostic (T=337, per-node sequences)")
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
                    help="windows per attribute() call (default 256 on a GPU, 4 on the CPU)")
    ap.add_argument("--ig-calls", type=int, default=None,
                    help="timed attribute() calls per rank (default 6 on a GPU, 1 on the CPU)")
    ap.add_argument("--no-cv-line", dest="cv_line", action="store_false",
                    help="skip the 5-fold CV ROC-AUC of the CML GCN and baseline (reported as 'cv' in the JSON line)")
    ap.add_argument("--cv-folds", type=int, default=None, help="CV folds (default 5 on a GPU, 2 on the CPU)")
    ap.add_argument("--cv-epochs", type=int, default=None, help="epochs per fold (default: the model config's, "
                    "1 on the CPU)")
    ap.add_argument("--cv-sensors", type=int, default=None, help="CV data: CML links (default 23)")
    ap.add_argument("--cv-days", type=float, default=None, help="CV data: days (default 28)")
    ap.add_argument("--cv-flagged", type=int, default=None, help="CV data: flagged links (default 4)")
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
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.store import DeviceLoader, DeviceStore
    from gnnqc.data.synthetic import make_cml_raw, make_soilnet_raw
    from gnnqc.models import BaselineClassifier, GCNClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.parallel import dist as D
    from gnnqc.train.engine import Trainer
    from gnnqc.train.loss import calculate_weights

    dev = D.init_distributed()
    world, rank = D.world_size(), D.rank()
    if os.environ.get("GNNQC_BENCH_FAIL_RANK") == str(rank):    # fault injection (tests/test_bench_launch.py)
        print(f"bench.py: rank {rank} failing on request", file=sys.stderr)
        return 3
    torch.manual_seed(1234)
    soil = args.ds == "soilnet"
    args.sensors = args.sensors or (40 if soil else 23)
    args.days = args.days or (89 if soil else 28)
    pc = C.normalize_preproc(C.default(f"preprocessing_{args.ds}"))
    args.batch = args.batch or int(pc.batch_size)
    pc.batch_size = args.batch
    pc.graph["adjacency"] = args.adjacency
    pc.graph["k"] = int(args.k)
    adj_desc = (f"knn(k={args.k})" if args.adjacency == "knn" else
                f"radius(max_sample_distance={pc.graph['max_sample_distance']})")
    mc = C.default(f"model_{args.ds}")
    mc.runtime.compute_dtype = args.dtype
    if soil:
        raw = make_soilnet_raw(n_boxes=args.sensors, n_time=args.days * 96, seed=7)
    else:
        raw = make_cml_raw(n_sensors=args.sensors, n_minutes=args.days * 1440, seed=7)
    if soil:
        pc["min_date"], pc["max_date"] = str(raw.time[0]), str(raw.time[-1])
    ws = create_windows_dataset(pc, raw=raw)
    tr = list(range(ws.n_windows))          # throughput: every window is a training window
    baseline = args.model == "baseline"

    def measure(graph_cfg):
        """Build store / model / trainer for one adjacency rule, warm up, time args.steps full
        training steps (max over ranks). Returns (seconds, trainer, loss, trainable params)."""
        store = DeviceStore(ws, "scale_range" if soil else "rolling_median", graph_cfg, device=dev)
        loader = DeviceLoader(store, tr, args.batch, shuffle=True, seed=44, rank=rank, world_size=world,
                              drop_last=True)
        torch.manual_seed(1234)
        model = (BaselineClassifier if baseline else GCNClassifier)(mc, pc).to(dev)
        n_params = sum(p.numel() for p in model.parameters() if p.requires_grad)
        opt = make_optimizer("adam", model.parameters(), mc.learning_rate)
        D.broadcast_module(model)
        trainer = Trainer(model, store, opt, calculate_weights(mc), baseline,
                          use_graph=not args.no_graph, batch_size=args.batch)
        rows = loader.batch_ids()                 # [n_batches, B] device tensor, no host sync while stepping

        def run(k, start):
            # every one of the k steps is a full training step (gather, forward, backward, guarded
            # Adam); chunks of trainer.graph_steps of them replay one multi-step HIP graph
            trainer.train_steps(rows, start, k)

        trainer.prepare_graphs(rows)              # graph captures happen here, never inside the timed steps
        run(args.warmup, 0)
        trainer._comm_events = []
        D.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(args.steps, args.warmup)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        D.barrier()
        dt = D.max_over_ranks(time.perf_counter() - t0)
        return dt, trainer, float(trainer.last_loss.item()), n_params

    dt, trainer, loss, n_params = measure(pc.graph)
    comm_us = None
    if trainer._comm_events:             # N > 1, eager layout: HIP events around the timed all-reduces
        comm_us = 1e3 * sum(a.elapsed_time(b) for a, b in trainer._comm_events) / len(trainer._comm_events)
    elif trainer.collective:             # in-graph all-reduce: the same collective timed on its own, after
        comm_us = trainer.measure_allreduce()
    if comm_us is not None:
        comm_us = D.max_over_ranks(comm_us)
    windows = args.steps * args.batch * world
    value = windows / dt
    knn = None
    if args.knn_line and args.adjacency == "radius" and not soil:
        # BASELINE.json names the CML graph "k=5": the same measurement on the symmetrised
        # 5-nearest-neighbour graph, reported inside the one JSON line
        g5 = dict(pc.graph)
        g5["adjacency"], g5["k"] = "knn", 5
        dt5, _, loss5, _ = measure(g5)
        knn = {"adjacency": "knn(k=5)", "value": round(windows / dt5, 2),
               "ms_per_step": round(1000.0 * dt5 / args.steps, 4), "final_loss": round(loss5, 5)}
    ig = None
    if args.ig_line and not soil and not baseline:
        ig = measure_ig(args, trainer, dev, world, rank, D)
    cv = None
    if args.cv_line and not soil:
        cv = measure_cv(args, dev, world, D)
    if rank == 0:
        out = {
            "metric": ("train windows/sec, SoilNet GCN (diagnostic; not the headline metric)" if soil else
                       "ROC-AUC (5-fold CV) + train windows/sec, CML GCN at 1/2/4/8 MI355X"),
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
                "model": ("%s GCN (GeneralConv16+%s+LSTM TimeLayer f16 n_stacks2+dense64)"
                          % ("SoilNet" if soil else "CML", "per-node sequences" if soil else "mean pool"))
                if not baseline else ("SoilNet" if soil else "CML") + " baseline LSTM",
                "global_batch": args.batch * world,
                "seq_len": ws.seq_len,
                "parallelism": f"dp{world}",
                "adjacency": adj_desc,
                "graph_steps": trainer.graph_steps if trainer._multi_ok() else 1,
                "trainable_params": n_params,
                "hip_graph": trainer.use_graph,
                "final_loss": round(loss, 5),
            },
        }
        if knn is not None:
            out["knn5"] = knn
        if ig is not None:
            out["ig"] = ig
        if cv is not None:
            out["cv"] = cv
        if comm_us is not None:
            # the collective of the timed steps, run on its own (in-graph collectives cannot be timed one
            # by one), plus the setup-time comparison of both modes when the peer kernel was considered
            from gnnqc.parallel.peer import LAST_SELECTION
            out["allreduce_us"] = round(comm_us, 2)
            out["allreduce_mode"] = (("peer one-shot xGMI" if trainer.peer is not None else "RCCL") +
                                     (" fused into the Adam launch" if trainer.peer_fused() else "") +
                                     (" in-graph (timed standalone)" if trainer.dp_graph and trainer._multi_ok()
                                      else " eager"))
            if LAST_SELECTION:
                out["allreduce_selection"] = {k: (round(v, 2) if isinstance(v, float) else v)
                                              for k, v in LAST_SELECTION.items()}
        print(json.dumps(out), flush=True)
    D.destroy()


if __name__ == "__main__":
    sys.exit(main() or 0)
