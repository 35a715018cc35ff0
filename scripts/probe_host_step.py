"""Host-side cost of one HipTrainer.step call (batch staging + graph launch) vs the device step time:
if the median host call approaches the wall time per step, the loop is host-bound."""
import sys, time, json
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import torch
from gru_mpi_cuda_amd.config import preset
from gru_mpi_cuda_amd.parallel import dist as gdist
from gru_mpi_cuda_amd.utils.data import NameStream
from gru_mpi_cuda_amd.engine.trainer import make_trainer
ctx = gdist.init(use_gpu=True)
cfg = preset("h512")
st = NameStream(cfg.batch, cfg.seq, cfg.sos, cfg.eos, seed=1000, max_len=cfg.max_len)
pool = [st.next() for _ in range(8)]
tr = make_trainer(cfg, ctx)
for i in range(20): tr.step(*pool[i % 8])
torch.cuda.synchronize()
host = []
t0 = time.perf_counter()
for i in range(200):
    a = time.perf_counter(); tr.step(*pool[i % 8]); host.append(time.perf_counter() - a)
torch.cuda.synchronize()
el = time.perf_counter() - t0
host.sort()
print(json.dumps({"wall_ms_per_step": 1000 * el / 200, "host_call_ms_median": 1000 * host[100], "host_call_ms_p90": 1000 * host[180], "host_call_ms_max": 1000 * host[-1]}))
