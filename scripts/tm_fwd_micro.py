#!/usr/bin/env python3
"""Time-major LSTM forward kernels vs the number of 16-sequence tiles (one workgroup each): the layer
pair (lstm_tm2_fwd, H = 16 / 32) and the single layer (lstm_tm_fwd), T steps, train mode (gates and c
saved). us per launch and ns per step; one JSON line per (kernel, H, tiles). Shows whether a step is
bound by its own latency (flat in tiles until the CUs fill) or by the CU's shared resources."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from gnnqc.utils.native import hip_ops
    ops = hip_ops()
    dev = torch.device("cuda:0")
    T = int(os.environ.get("T", "337"))
    reps = int(os.environ.get("REPS", "10"))
    torch.manual_seed(0)
    for H, Din in ((16, 16), (32, 16)):
        for tiles in (64, 128, 256, 418, 512, 1024):
            Mp = 16 * tiles
            x = torch.randn(T, Mp, Din, device=dev) * 0.5
            WA, UA = torch.randn(Din, 4 * H, device=dev) * 0.2, torch.randn(H, 4 * H, device=dev) * 0.2
            WB, UB = torch.randn(H, 4 * H, device=dev) * 0.2, torch.randn(H, 4 * H, device=dev) * 0.2
            b = torch.zeros(4 * H, device=dev)
            for name, fn in (("pair", lambda: ops.lstm_tm2_fwd(x, WA, UA, b, WB, UB, b, True)[:6]),
                             ("single", lambda: ops.lstm_tm_fwd(x, WA, UA, b, True))):
                for _ in range(2):
                    fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / reps
                print(json.dumps({"kernel": name, "H": H, "tiles": tiles, "T": T, "us": round(us, 1),
                                  "ns_per_step": round(us * 1e3 / T, 1)}), flush=True)
            del x


if __name__ == "__main__":
    main()
