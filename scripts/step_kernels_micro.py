"""Per-kernel timings of the small kernels of the CML step, each replayed on its own in a HIP graph
(back to back, 50 launches per replay), to separate a kernel's own cost from its place in the
step (scripts/gpu_r3.sh profiles the whole step). Prints one JSON line per kernel."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, n=50, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    best = 1e9
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / n)
    return best


def main():
    from gnnqc import config as C
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.store import CursorIds, DeviceStore
    from gnnqc.data.synthetic import make_cml_raw
    from gnnqc.models import GCNClassifier
    from gnnqc.ops.lstm import chain_ctl
    from gnnqc.ops.optim import FlatAdam
    from gnnqc.utils.native import hip_ops
    dev = torch.device("cuda:0")
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=23, n_minutes=28 * 1440, seed=7))
    st = DeviceStore(ws, "rolling_median", pc.graph, device=dev)
    model = GCNClassifier(C.default("model_cml"), pc).to(dev)
    g = model.gcn_layer
    ops = hip_ops()
    data = st.gcn_fused_data(True, 0)
    table = torch.randint(0, st.n_windows, (64, 128), device=dev)
    cur = torch.zeros(1, dtype=torch.long, device=dev)
    e = torch.zeros(0, dtype=torch.long, device=dev)
    out = {}

    def fwd():
        return ops.gcn_fused_fwd(*data["fwd"], e, table, cur, *data["dims"], g.kernel, g.bias, g.bn_gamma, g.bn_beta,
                                 g.prelu_alpha, g.bn_moving_mean, g.bn_moving_variance, True, 0.99, 1e-3, 128, 20)

    h, S, stt, _, _, _ = fwd()
    out["gcn_fused_fwd"] = timed(fwd)
    dh = torch.randn_like(h)
    gW, gg, gb_, ga = (torch.zeros_like(p) for p in (g.kernel, g.bn_gamma, g.bn_beta, g.prelu_alpha))

    def bwd():
        ops.gcn_fused_bwd(dh, 2, *data["bwd"], e, table, cur, *data["dims"], S, stt, g.kernel, g.bias, g.prelu_alpha,
                          gW, gg, gb_, ga)

    out["gcn_fused_bwd"] = timed(bwd)
    opt = FlatAdam(model.parameters(), 1e-3)
    opt.flagged_producers = True
    out["adam_flagged"] = timed(lambda: opt.step(1.0))
    opt.flagged_producers = False
    out["adam_guarded"] = timed(lambda: opt.step(1.0))
    chain_ctl(dev)
    x = torch.zeros(1, device=dev)
    out["empty_fill"] = timed(lambda: x.fill_(1.0))
    for k, v in out.items():
        print(json.dumps({"kernel": k, "us_per_launch": round(v, 2)}))


if __name__ == "__main__":
    main()
