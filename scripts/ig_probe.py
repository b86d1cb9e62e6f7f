import os, sys, time, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from gnnqc import config as C
from gnnqc.data.preprocessing import create_windows_dataset
from gnnqc.data.store import DeviceStore
from gnnqc.data.synthetic import make_cml_raw
from gnnqc.models import GCNClassifier
from gnnqc.xai.ig import IntegratedGradients
dev = torch.device("cuda:0")
torch.manual_seed(0)
pc = C.normalize_preproc(C.default("preprocessing_cml"))
mc = C.default("model_cml")
ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=23, n_minutes=28 * 1440, seed=7))
store = DeviceStore(ws, "rolling_median", pc.graph, device=dev)
model = GCNClassifier(mc, pc).to(dev)
for flag in ("1", "0", "1"):
    os.environ["GNNQC_IG_HEAD_HIP"] = flag
    for graph in (True, False):
        ig = IntegratedGradients(model, "cml", m_steps=100, max_rows=32768, use_graph=graph)
        b = store.gather(torch.arange(0, 256, device=dev))
        for _ in range(2):
            ig.attribute(b)
        torch.cuda.synchronize()
        ts = []
        for _ in range(4):
            t0 = time.perf_counter(); ig.attribute(b); torch.cuda.synchronize(); ts.append(1e3 * (time.perf_counter() - t0))
        print(json.dumps({"hip_head": flag, "graph": graph, "ms": [round(t, 3) for t in ts]}), flush=True)
