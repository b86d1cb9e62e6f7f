"""Tiny CPU training job for the kill / resume tests (tests/test_resilience.py).

    python tests/helpers/resume_job.py <work_dir> <out.pt> [--resume]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from gnnqc import config as C  # noqa: E402
from gnnqc.data.preprocessing import create_windows_dataset  # noqa: E402
from gnnqc.data.store import DeviceLoader, DeviceStore  # noqa: E402
from gnnqc.data.synthetic import make_cml_raw  # noqa: E402
from gnnqc.models import BaselineClassifier  # noqa: E402
from gnnqc.train import train_model  # noqa: E402


def main():
    work, out = sys.argv[1], sys.argv[2]
    resume = "--resume" in sys.argv
    torch.set_num_threads(2)
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    pc.timestep_before, pc.timestep_after = 30, 15
    ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=8, n_minutes=10 * 1440, seed=5))
    st = DeviceStore(ws, "rolling_median", pc.graph)
    mc = C.default("model_cml")
    mc.baseline_model.filter_1_size = 8
    mc.epochs = 3
    mc.es_patience = 10
    torch.manual_seed(0)
    m = BaselineClassifier(mc, pc)
    L = DeviceLoader(st, np.arange(min(st.n_windows, 640)), 64)
    hist, m = train_model(m, mc, pc, L, None, baseline=True, store=st, classes_weights={0: 1.0, 1: 5.0},
                          use_graph=False, verbose=0, resume_dir=os.path.join(work, "resume"), resume=resume)
    torch.save({"state": {k: v.clone() for k, v in m.state_dict().items()}, "loss": hist.history["loss"]}, out)


if __name__ == "__main__":
    main()
