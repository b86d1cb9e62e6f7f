"""The HIP extension's operator schemas register without error. A bad schema (e.g. a default on a
Tensor list) aborts the process when the library is loaded, which on the GPU box looks like a crash
of the first GPU test; loading the library needs no GPU, so it is checked here, in a subprocess."""
import os
import subprocess
import sys

import pytest

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gnnqc", "_lib", "libgnnqc_hip.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="HIP extension not built")
def test_hip_library_registers_its_ops():
    code = ("import torch; torch.ops.load_library(%r); "
            "import sys; ops = torch.ops.gnnqc; "
            "names = ['lstm_chain_head_fwd', 'lstm_chain_head_bwd', 'lstm_grads_multi', 'gcn_fused_bwd', "
            "'adam_flagged', 'time4_head_bwd', 'lstm_defer_reduce', 'lstm_reduce_flush', 'gcn_fused_fwd', "
            "'gcn_prod_flush', 'gcn_coef_flush', 'gcn_coef_bwd', 'head_prob_fwd', 'head_prob_bwd']; "
            "[getattr(ops, n) for n in names]; print('ok')" % LIB)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.returncode, r.stderr[-2000:])
