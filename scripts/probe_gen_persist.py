"""Phase timing of the persistent fp32 generator (gen_persist.hip stamps): per char, the mean
microseconds between consecutive stamps of workgroup 0 -- logits wait, sampling, layer 0 gates +
publish, each product's input wait, its MFMA / reduce / gates + publish.
    python scripts/probe_gen_persist.py [N] [preset]"""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from gru_mpi_cuda_amd.config import preset
from gru_mpi_cuda_amd.models.params import init_params
from gru_mpi_cuda_amd.engine.generator import HipGenerator
from gru_mpi_cuda_amd.utils.data import random_floats

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1
cfg = preset(sys.argv[2] if len(sys.argv) > 2 else "ref")
g = HipGenerator(cfg, init_params(cfg), max_batch=max(N, 64), precision="fp32")
assert g.g.uses_persist(N)
ML = cfg.max_len
dbg = torch.zeros(2 * (ML + 1) * 16, dtype=torch.int64, device="cuda")
rf = torch.from_numpy(random_floats(N, ML, seed=3).reshape(N, ML)).cuda()
g.generate_device(rf, N)
torch.cuda.synchronize()
# end to end (no stamps): one generate_device per batch, launch and slot fills included
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(20):
    g.generate_device(rf, N)
ev1.record()
torch.cuda.synchronize()
e2e = ev0.elapsed_time(ev1) * 1e3 / 20
g.g.set_persist_dbg(dbg.data_ptr())
g.generate_device(rf, N)
torch.cuda.synchronize()
d = dbg.view(2, ML + 1, 16).cpu().numpy().astype(np.float64) / 100.0   # 100 MHz -> us
names = ["char start", "logits seen", "sampled", "L0 published", "L1 input seen", "L1 published",
         "FC input seen", "logits published"]
w0 = d[0]
steps = [w0[t] for t in range(1, ML)]   # chars 1..ML-1 (char 0 has no sampling)
diffs = np.array([[s[k] - s[k - 1] for k in range(1, 8)] for s in steps])
per_char = np.array([w0[t + 1][0] - w0[t][0] for t in range(1, ML - 1)])
out = {"N": N, "model": f"L={cfg.layers} H={cfg.hidden}", "us_per_char": round(float(per_char.mean()), 2),
       "phase_us": {f"{names[k - 1]} -> {names[k]}": round(float(diffs[:, k - 1].mean()), 2) for k in range(1, 8)},
       "tail_us (logits published -> next char start)": round(float(np.mean([w0[t + 1][0] - w0[t][7] for t in range(1, ML - 1)])), 2),
       "sampling_us": ({"logits seen -> staged": round(float(np.mean([w0[t][8] - w0[t][1] for t in range(1, ML)])), 2),
                        "staged -> first name": round(float(np.mean([w0[t][9] - w0[t][8] for t in range(1, ML)])), 2),
                        "first name -> wave 0 done": round(float(np.mean([w0[t][10] - w0[t][9] for t in range(1, ML)])), 2),
                        "wave 0 done -> sampled (barrier)": round(float(np.mean([w0[t][2] - w0[t][10] for t in range(1, ML)])), 2)}
                       if N <= 16 else   # distributed sampling: workgroup 0 samples name 0, then reads all ids
                       {"logits seen -> own name sampled": round(float(np.mean([w0[t][9] - w0[t][1] for t in range(1, ML)])), 2),
                        "own name sampled -> all ids seen": round(float(np.mean([w0[t][10] - w0[t][9] for t in range(1, ML)])), 2),
                        "ids seen -> sampled (barrier)": round(float(np.mean([w0[t][2] - w0[t][10] for t in range(1, ML)])), 2)}),
       "L1_phase_us": {"input seen -> x in": round(float(np.mean([w0[t][11] - w0[t][4] for t in range(1, ML)])), 2),
                       "x in -> MFMAs stashed": round(float(np.mean([w0[t][12] - w0[t][11] for t in range(1, ML)])), 2),
                       "stashed -> reduced": round(float(np.mean([w0[t][13] - w0[t][12] for t in range(1, ML)])), 2),
                       "reduced -> gates": round(float(np.mean([w0[t][14] - w0[t][13] for t in range(1, ML)])), 2),
                       "gates -> barrier (<= 16 names: stored)": round(float(np.mean([w0[t][15] - w0[t][14] for t in range(1, ML)])), 2),
                       "barrier (stored) -> published": round(float(np.mean([w0[t][5] - w0[t][15] for t in range(1, ML)])), 2)}
       if cfg.layers >= 2 else {},
       "sclk_ghz": round(float(np.mean([(dbg.view(2, ML + 1, 16)[1, t + 1, 15] - dbg.view(2, ML + 1, 16)[1, t, 15]).item()
                                         / ((d[1][t + 1][0] - d[1][t][0]) * 1e3) for t in range(1, ML - 1)])), 3),
       "launch_us": {"entry -> char 0 start (weights to VGPRs / LDS)": round(float(w0[0][0] - w0[ML][14]), 2),
                     "char 0 (no sampling)": round(float(w0[1][0] - w0[0][0]), 2),
                     "char ML start -> loop end (last sampling)": round(float(w0[ML][13] - w0[ML][0]), 2),
                     "entry -> loop end": round(float(w0[ML][13] - w0[ML][14]), 2)},
       "end_to_end_us_per_generate": round(e2e, 2), "end_to_end_us_per_char": round(e2e / ML, 2),
       "error_word": int(g.g.read_error())}
print(json.dumps(out))
