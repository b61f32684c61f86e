import os, sys, time, tempfile, json
sys.path.insert(0, os.getcwd())
import torch
from fed_tgan_amd.data.schema import intrusion_spec
from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime
from fed_tgan_amd.parallel.comm import Comm
dev = torch.device("cuda:0")
out = tempfile.mkdtemp()
cfg = FedConfig(spec=intrusion_spec(), epochs=20, synthetic_rows=40000, out_dir=out, n_sample=40000,
                gmm_backend="torch", seed=0, verbose=False)
rt = FedRuntime(cfg, Comm(0, 1, [0], "gloo", device=dev), dev)
rt.initialize()
for ep in range(4):
    rt.run_round(ep)
rt.flush_writes()
torch.cuda.synchronize()
rt.timer.reset()
t0 = time.perf_counter()
n = 12
for ep in range(4, 4 + n):
    rt.run_round(ep)
t1 = time.perf_counter()
rt.flush_writes()
torch.cuda.synchronize()
t2 = time.perf_counter()
tot = rt.timer.totals
print(json.dumps({"rounds_ms": (t1 - t0) / n * 1e3, "with_flush_ms": (t2 - t0) / n * 1e3,
                  **{k: v / n * 1e3 for k, v in tot.items()}}))
