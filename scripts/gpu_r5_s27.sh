#!/bin/bash
# session 27: loss trajectories with dW_fc on gemm256p (32 K-slices) vs 128 x 128 (8 K-slices)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u - <<'PY' > gpurun_out/s27.log 2>&1
import os, torch
from gru_mpi_cuda_amd.config import GRUConfig, preset
from gru_mpi_cuda_amd.models.params import init_params
from gru_mpi_cuda_amd.engine.trainer import HipTrainer
from gru_mpi_cuda_amd.utils.data import NameStream
for name, cfg in [("h256", GRUConfig(vocab=256, embed=64, hidden=256, layers=1, batch=512, seq=128, seed=4)),
                  ("h2048", preset("h2048", batch=512))]:
    params = init_params(cfg)
    st = NameStream(cfg.batch, cfg.seq, cfg.sos, cfg.eos, seed=7, max_len=cfg.max_len)
    pool = [st.next() for _ in range(8)]
    traj = {}
    for eng in ("0", "1"):
        os.environ["GK_FC256"] = eng
        tr = HipTrainer(cfg, params={k: v.clone() for k, v in params.items()})
        out = []
        for i in range(300):
            tr.step(*pool[i % 8])
            if i in (0, 1, 2, 5, 10, 30, 100, 200, 299):
                torch.cuda.synchronize(); out.append((i, round(tr.loss(), 6)))
        traj[eng] = out
        del tr
    print(name, "fc128", traj["0"], flush=True)
    print(name, "fc256", traj["1"], flush=True)
PY
rc=$?; cat gpurun_out/s27.log; exit $rc
