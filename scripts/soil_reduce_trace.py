"""Attribute the aten reductions / fills / copies of one GCN training step (eager, no graph).

Usage: python scripts/soil_reduce_trace.py [soilnet|cml]

Prints the top aten ops by device time with their input shapes and Python stacks,
so a stray PyTorch reduction in the SoilNet path can be traced to its call site.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.store import DeviceLoader, DeviceStore
    from gnnqc.data.synthetic import make_soilnet_raw
    from gnnqc.models import GCNClassifier
    from gnnqc.ops.optim import make_optimizer
    from gnnqc.train.engine import Trainer
    from gnnqc.train.loss import calculate_weights

    from gnnqc.data.synthetic import make_cml_raw
    ds = sys.argv[1] if len(sys.argv) > 1 else "soilnet"
    dev = torch.device("cuda:0")
    pc = C.normalize_preproc(C.default(f"preprocessing_{ds}"))
    mc = C.default(f"model_{ds}")
    if ds == "soilnet":
        raw = make_soilnet_raw(n_boxes=40, n_time=89 * 96, seed=7)
        pc["min_date"], pc["max_date"] = str(raw.time[0]), str(raw.time[-1])
    else:
        raw = make_cml_raw(n_sensors=23, n_minutes=28 * 1440, seed=7)
    ws = create_windows_dataset(pc, raw=raw)
    store = DeviceStore(ws, "scale_range" if ds == "soilnet" else "rolling_median", pc.graph, device=dev)
    loader = DeviceLoader(store, list(range(ws.n_windows)), int(pc.batch_size), shuffle=True, seed=44,
                          drop_last=True)
    model = GCNClassifier(mc, pc).to(dev)
    opt = make_optimizer("adam", model.parameters(), mc.learning_rate)
    tr = Trainer(model, store, opt, calculate_weights(mc), False, use_graph=False, batch_size=int(pc.batch_size))
    rows = loader.batch_ids()
    for i in range(3):
        tr.train_step(rows[i])
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                 with_stack=True) as prof:
        tr.train_step(rows[3])
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=25,
                                                            max_name_column_width=40,
                                                            max_shapes_column_width=90))
    for ev in prof.events():
        if ev.name in ("aten::sum", "aten::mean", "aten::amax", "aten::max", "aten::all", "aten::any",
                       "aten::norm", "aten::linalg_vector_norm"):
            print("==", ev.name, ev.input_shapes)
            for fr in (ev.stack or [])[:8]:
                print("   ", fr)
        if ev.name in ("aten::fill_", "aten::zero_", "aten::copy_", "aten::clone", "aten::zeros", "aten::contiguous"):
            chain, p = [], ev.cpu_parent
            while p is not None and len(chain) < 6:
                chain.append(p.name)
                p = p.cpu_parent
            print("==", ev.name, ev.input_shapes, "<-", " <- ".join(chain))


if __name__ == "__main__":
    main()
