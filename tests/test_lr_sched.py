"""Learning-rate schedule: host formula (models/cpu_ref.lr_at) and the CPU trainer using it.
The device twin (csrc/kernels/misc.hip sched_lr) is pinned against this oracle in
tests/test_engine_gpu.py::test_trainer_lr_schedule_matches_cpu."""
import math

import numpy as np
import pytest
import torch

from gru_mpi_cuda_amd.config import GRUConfig
from gru_mpi_cuda_amd.models import cpu_ref
from gru_mpi_cuda_amd.models.params import init_params


def test_lr_at_values():
    c = GRUConfig(lr=1e-2, lr_sched="cosine", warmup_steps=4, total_steps=14, lr_min=1e-3)
    assert cpu_ref.lr_at(c, 1) == pytest.approx(2.5e-3)
    assert cpu_ref.lr_at(c, 4) == pytest.approx(1e-2)
    assert cpu_ref.lr_at(c, 9) == pytest.approx(1e-3 + 9e-3 * 0.5 * (1 + math.cos(math.pi * 0.5)))
    assert cpu_ref.lr_at(c, 14) == pytest.approx(1e-3)
    assert cpu_ref.lr_at(c, 100) == pytest.approx(1e-3)   # clamped after total_steps
    lin = c.replace(lr_sched="linear")
    assert cpu_ref.lr_at(lin, 9) == pytest.approx(1e-3 + 9e-3 * 0.5)
    const = c.replace(lr_sched="const", warmup_steps=0)
    assert all(cpu_ref.lr_at(const, t) == 1e-2 for t in (1, 7, 1000))
    with pytest.raises(ValueError):
        cpu_ref.lr_at(c.replace(lr_sched="step"), 1)


def test_cpu_adam_uses_schedule():
    """Warm-up step 1 of 4 moves every weight by a quarter of the constant-lr step (the first
    bias-corrected Adam step is lr * sign(g) for each element)."""
    cfg = GRUConfig(vocab=16, embed=8, hidden=8, layers=1, batch=4, seq=4, lr=1e-2)
    params = init_params(cfg)
    grads = {k: torch.randn_like(v) for k, v in params.items()}
    out = {}
    for name, c in (("const", cfg), ("warm", cfg.replace(lr_sched="linear", warmup_steps=4, total_steps=10))):
        p = {k: v.clone() for k, v in params.items()}
        cpu_ref.Adam(c, p).step(p, {k: g.clone() for k, g in grads.items()})
        out[name] = {k: p[k] - params[k] for k in p}
    for k in params:
        torch.testing.assert_close(out["warm"][k], out["const"][k] / 4, rtol=1e-4, atol=1e-7)


def test_cli_accepts_schedule_flags():
    import argparse
    from gru_mpi_cuda_amd import cli
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="cpu_tiny")
    cli._add_model_args(ap)
    args = ap.parse_args(["--lr-sched", "cosine", "--warmup-steps", "5", "--total-steps", "50", "--lr-min", "1e-5"])
    cfg = cli._cfg_from(args)
    assert (cfg.lr_sched, cfg.warmup_steps, cfg.total_steps, cfg.lr_min) == ("cosine", 5, 50, 1e-5)
