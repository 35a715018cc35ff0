"""C-API generation default on evidence.  Fraction of names identical to the
fp64 oracle (models/cpu_ref.generate in float64) for fp32, bf16x3 and bf16 generation over three
weight seeds x two reference-shaped presets (ref: L2 E512 H1024; h1024_l2: L2 E1024 H1024), 400
names each, unsharpened random-init fp32 weights.  One JSON line per (preset, seed)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gru_mpi_cuda_amd.config import preset
from gru_mpi_cuda_amd.models import cpu_ref
from gru_mpi_cuda_amd.models.params import init_params
from gru_mpi_cuda_amd.engine.generator import HipGenerator
from gru_mpi_cuda_amd.utils.data import random_floats

N = int(os.environ.get("N", 400))
for name in ("ref", "h1024_l2"):
    for seed in (4, 11, 23):
        cfg = preset(name, max_len=10, sos=0, eos=0, seed=seed)
        params = init_params(cfg)
        rf = random_floats(N, cfg.max_len, seed=seed + 100)
        t0 = time.time()
        ref = cpu_ref.generate({k: v.double() for k, v in params.items()}, cfg, rf)
        row = {"preset": name, "seed": seed, "names": N, "oracle_s": round(time.time() - t0, 1)}
        for prec in ("fp32", "bf16x3", "bf16"):
            got = HipGenerator(cfg, params, precision=prec).generate(rf)
            row[prec] = round(float((got == ref).all(1).mean()), 4)
        print(json.dumps(row), flush=True)
