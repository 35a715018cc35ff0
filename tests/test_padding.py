"""The HIP engine runs V, E, H that are not multiples of 64 on a zero-padded model
(models/params.py pad_config / pad_params).  This checks on the CPU oracle that the padding is
exact: same loss, the real gradient entries unchanged, every padded gradient entry zero (so Adam
never moves a padded weight), for hidden-state carry too."""
import numpy as np
import torch

from gru_mpi_cuda_amd.config import GRUConfig
from gru_mpi_cuda_amd.models import cpu_ref
from gru_mpi_cuda_amd.models.params import init_params, pad_config, pad_params, unpad_params


def test_zero_padding_is_exact():
    cfg = GRUConfig(vocab=100, embed=40, hidden=72, layers=2, batch=6, seq=5, seed=3)
    pcfg = pad_config(cfg)
    assert (pcfg.vocab, pcfg.embed, pcfg.hidden) == (128, 64, 128)
    p = {k: v.double() for k, v in init_params(cfg).items()}
    pp = pad_params(p, cfg, pcfg)
    rng = np.random.default_rng(0)
    x = torch.from_numpy(rng.integers(0, cfg.vocab, size=(cfg.batch, cfg.seq)))
    y = torch.from_numpy(rng.integers(0, cfg.vocab, size=(cfg.batch, cfg.seq)))
    y[0, -1] = -1
    h0 = [torch.randn(cfg.batch, cfg.hidden, dtype=torch.float64) for _ in range(cfg.layers)]
    h0p = [torch.nn.functional.pad(h, (0, pcfg.hidden - cfg.hidden)) for h in h0]
    loss, g = cpu_ref.manual_backward(p, cfg, x, y, h0=h0)
    lossp, gp = cpu_ref.manual_backward(pp, pcfg, x, y, h0=h0p)
    assert abs(float(loss) - float(lossp)) < 1e-12
    gu = unpad_params(gp, cfg, pcfg)
    for k in g:
        torch.testing.assert_close(gu[k], g[k], atol=1e-12, rtol=1e-10)
        # every padded entry of the gradient is zero
        total = gp[k].abs().sum()
        real = gu[k].abs().sum()
        assert abs(float(total - real)) < 1e-12, k


def test_pad_unpad_roundtrip():
    cfg = GRUConfig(vocab=77, embed=50, hidden=100, layers=3)
    pcfg = pad_config(cfg)
    p = init_params(cfg)
    u = unpad_params(pad_params(p, cfg, pcfg), cfg, pcfg)
    assert all(torch.equal(u[k], p[k]) for k in p)
