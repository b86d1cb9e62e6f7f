#!/usr/bin/env python3
"""Time-major LSTM backward on the SoilNet layer shapes (T = 337, 6,688 sequences): the recurrence
with weight gradients inside it (lstm_tm_bwd_wg_kernel) vs recurrence + separate weight-gradient
pass, per (H, Din). Mean of REPS launches after a warmup; one JSON line per config and path.
Select a compile-time variant library with GNNQC_HIP_LIB."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from gnnqc.utils.native import hip_ops
    ops = hip_ops()
    dev = torch.device("cuda:0")
    Mp = int(os.environ.get("MP", "6688"))
    reps = int(os.environ.get("REPS", "20"))
    torch.manual_seed(0)
    # CONFIGS: "H:Din:T,..." (default: the SoilNet layers' shapes; H = 64 has no in-recurrence path)
    cfgs = [tuple(int(v) for v in c.split(":")) for c in
            os.environ.get("CONFIGS", "16:16:337,32:16:112,32:32:112,64:32:37,64:64:37").split(",")]
    for H, Din, T in cfgs:
        x = torch.randn(T, Mp, Din, device=dev) * 0.5
        W = torch.randn(Din, 4 * H, device=dev) * 0.2
        U = torch.randn(H, 4 * H, device=dev) * 0.2
        b = torch.zeros(4 * H, device=dev)
        h, g, c = ops.lstm_tm_fwd(x, W, U, b, True)
        dh = torch.randn(T, Mp, H, device=dev) * 0.1
        for path in (("in_rec", "pass", "dx_only") if H <= 32 else ("pass", "dx_only")):
            os.environ["GNNQC_TM_FUSED_WGRAD"] = "1" if path == "in_rec" else "0"
            if path == "dx_only":            # the recurrence alone (frozen weights: dx, no dz stream)
                dW = dU = db = torch.zeros(0, device=dev)
            else:
                dW, dU, db = torch.zeros_like(W), torch.zeros_like(U), torch.zeros_like(b)
            for _ in range(3):
                ops.lstm_tm_bwd(dh, g, c, x, h, W, U, b, dW, dU, db, True)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                ops.lstm_tm_bwd(dh, g, c, x, h, W, U, b, dW, dU, db, True)
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"H": H, "Din": Din, "T": T, "path": path, "us": round(e0.elapsed_time(e1) * 1e3 / reps, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
