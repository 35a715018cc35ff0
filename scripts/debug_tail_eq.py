"""Which tensors differ between the fused-tail step, the phased step and the 1-rank RCCL step."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from gru_mpi_cuda_amd.config import GRUConfig
from gru_mpi_cuda_amd.models.params import init_params, from_flat
from gru_mpi_cuda_amd.engine.trainer import HipTrainer
from gru_mpi_cuda_amd.utils.data import NameStream
from gru_mpi_cuda_amd.ops import load_ext
C = load_ext()
for (L, E, H, B) in [(1, 512, 512, 64), (1, 256, 256, 64), (1, 512, 512, 256)]:
    cfg = GRUConfig(vocab=256, embed=E, hidden=H, layers=L, batch=B, seq=8, seed=3, bucket_mb=1.0)
    x, y = NameStream(cfg.batch, cfg.seq, seed=4).next()
    comm = C.RcclComm(C.RcclComm.unique_id(), 0, 1)
    tr = {"dp": HipTrainer(cfg, params=init_params(cfg), comm=comm), "fused": HipTrainer(cfg, params=init_params(cfg)),
          "phased": HipTrainer(cfg, params=init_params(cfg))}
    print(L, E, H, B, tr["fused"].t.plan(), tr["fused"].t.tail_plan())
    for step in range(2):
        tr["dp"].step(x, y); tr["fused"].step(x, y)
        tr["phased"].forward_backward(x, y); tr["phased"].optimizer_step()
        torch.cuda.synchronize()
        for what in ("grads", "params"):
            ref = from_flat(tr["phased"].icfg, getattr(tr["phased"], what))
            for name in ("dp", "fused"):
                got = from_flat(tr[name].icfg, getattr(tr[name], what))
                bad = [k for k in ref if not torch.equal(ref[k], got[k])]
                if bad:
                    print(f"  step {step} {what} {name} != phased: " + ", ".join(
                        f"{k} (max {float((ref[k] - got[k]).abs().max()):.3g})" for k in bad))
        print(f"  step {step} err fused={tr['fused'].t.read_error()} dp={tr['dp'].t.read_error()} "
              f"steps {tr['fused'].t.get_step()} {tr['phased'].t.get_step()}")
