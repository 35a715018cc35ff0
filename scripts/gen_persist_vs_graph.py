"""Where the persistent fp32 launch (gen_persist.hip) beats the bf16 per-char graph: microseconds per
char of generate_device at several batch sizes on the reference model, both paths on the same box.
Sets the bf16 mode's persistent cap (Generator::persist_max_bf16_).  One JSON line per N.
    python scripts/gen_persist_vs_graph.py [N,N,...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gru_mpi_cuda_amd.config import preset
from gru_mpi_cuda_amd.models.params import init_params
from gru_mpi_cuda_amd.engine.generator import HipGenerator
from gru_mpi_cuda_amd.utils.data import random_floats

Ns = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "8,16,24,32,40,48,64").split(",")]
cfg = preset("ref")
params = init_params(cfg)
ML = cfg.max_len


def us_per_char(gen, rf, n, reps=20):
    gen.generate_device(rf, n)   # warm (graph capture, first launch)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        gen.generate_device(rf, n)
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) * 1e3 / reps / ML


for n in Ns:
    rf = torch.from_numpy(random_floats(n, ML, seed=3).reshape(n, ML)).cuda()
    pers = HipGenerator(cfg, params, max_batch=64, precision="fp32")
    assert pers.g.uses_persist(n)
    fast = HipGenerator(cfg, params, max_batch=64, precision="bf16")
    fast.g.set_persist(False)
    row = {"N": n, "persistent_fp32_us_per_char": round(us_per_char(pers, rf, n), 2),
           "bf16_graph_us_per_char": round(us_per_char(fast, rf, n), 2)}
    print(json.dumps(row), flush=True)
