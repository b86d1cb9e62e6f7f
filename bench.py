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

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
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


def launch_ranks(n: int, argv) -> int:
    """Run this script as ``n`` rank processes (one per GPU) and wait for all of them. The parent
    only counts devices (``torch.cuda.device_count`` does not initialise HIP) and never calls into
    the GPU; a child that fails takes the others down (exact Popen handles, no pattern kills) and
    its exit code becomes this process's."""
    ndev = torch.cuda.device_count()
    if ndev and n > ndev:
        print(f"bench.py: --gpus {n} but only {ndev} GPUs are visible", file=sys.stderr)
        return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if not ndev:                  # CPU (gloo) rehearsal: do not oversubscribe the cores
            env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // n)))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
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
    for p in procs:
        p.wait()
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
    args = ap.parse_args(argv)

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: WORLD_SIZE={env_world} from the launcher but --gpus {args.gpus}", file=sys.stderr)
        return 2
    if env_world is None and args.gpus > 1:
        return launch_ranks(args.gpus, argv)

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
