"""Chain backward with producer-side un-pooling (GNNQC_CHAINB_PUNPOOL) vs the per-layer backward:
gradient agreement and the chain status words (timeout diagnostics ctl[7/8/11])."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gnnqc.models.timelayer import TimeLayer  # noqa: E402
from gnnqc.utils.native import hip_ops  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 16
dev = torch.device("cuda:0")
torch.manual_seed(0)
tl = TimeLayer(18, 16, 2, "lstm", pool_size=3).to(dev)
x = torch.randn(M, 181, 18, device=dev)
os.environ["GNNQC_NO_PAIR"] = "1"
os.environ["GNNQC_CHAIN"] = "1"


def run(bwd):
    os.environ["GNNQC_CHAIN_BWD"] = bwd
    xi = x.clone().requires_grad_(True)
    for p in tl.parameters():
        p.grad = None
    out = tl(xi)
    out.pow(2).sum().backward()
    torch.cuda.synchronize()
    return [xi.grad.clone()] + [p.grad.clone() for p in tl.parameters()]


g0 = run("0")
print("status after per-layer", hip_ops().lstm_chain_status(x).cpu().tolist(), flush=True)
g1 = run("1")
st = hip_ops().lstm_chain_status(x).cpu().tolist()
print("status after chain bwd", st, flush=True)
names = ["x"] + [n for n, _ in tl.named_parameters()]
for n, a, b in zip(names, g1, g0):
    print(f"{n:40s} rel {((a - b).norm() / (b.norm() + 1e-6)).item():.3e} |a| {a.norm().item():.4e} |b| {b.norm().item():.4e}")
