"""Device-dispatching operators.

Every hot op has two implementations:

* the HIP/CDNA4 kernel in ``csrc/kernels`` (``torch.ops.gnnqc.*``) - used for every
  tensor that lives on a GPU; a missing extension is a hard error there;
* an eager PyTorch implementation - used on CPU (unit tests, gloo CI) and as the
  fp32 numerics oracle the kernel tests compare against.

``GNNQC_FORCE_EAGER=1`` forces the eager path on GPU (debugging only).
``GNNQC_DETERMINISTIC=1`` / :func:`set_deterministic` selects bitwise-reproducible
kernel launches (single-workgroup float reductions, slower).
"""
from __future__ import annotations

import os

import torch

from ..utils.native import hip_available, hip_ops


def use_hip(t: torch.Tensor) -> bool:
    if not t.is_cuda:
        return False
    if os.environ.get("GNNQC_FORCE_EAGER", "0") == "1":
        return False
    hip_ops()   # raises if the library is missing
    return True


def set_deterministic(flag: bool = True) -> bool:
    """Bitwise-reproducible mode for the HIP kernels (and torch's own ops). Returns the
    previous setting. The flag is process-wide; HIP graphs captured before the switch
    keep their launch configuration (re-create the Trainer)."""
    prev = deterministic()
    os.environ["GNNQC_DETERMINISTIC"] = "1" if flag else "0"
    torch.use_deterministic_algorithms(bool(flag), warn_only=True)
    if hip_available():
        hip_ops().set_deterministic(bool(flag))
    return prev


def deterministic() -> bool:
    return os.environ.get("GNNQC_DETERMINISTIC", "0") == "1"


from .lstm import lstm_layer, lstm_eager  # noqa: E402
from .gcn import gcn_pool, node_pool_weights, masked_batchnorm  # noqa: E402
from .optim import FlatAdam  # noqa: E402
from .metrics import score_histogram  # noqa: E402

__all__ = ["set_deterministic", "deterministic", "use_hip", "hip_available", "hip_ops", "lstm_layer", "lstm_eager", "gcn_pool",
           "node_pool_weights", "masked_batchnorm", "FlatAdam", "score_histogram"]
