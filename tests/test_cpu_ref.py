"""CPU reference path: GRU math (= torch.nn.GRU), manual BPTT (= autograd, fp64),
finite differences, the reference's sampler and generation semantics."""
import numpy as np
import pytest
import torch
from hypothesis import given, settings, strategies as st

from gru_mpi_cuda_amd.config import GRUConfig, PRESETS
from gru_mpi_cuda_amd.models import cpu_ref
from gru_mpi_cuda_amd.models.params import init_params
from gru_mpi_cuda_amd.utils.data import NameStream, make_padded_batch, synthetic_names, random_floats


def p64(cfg, seed=0):
    return {k: v.double() for k, v in init_params(cfg, seed).items()}


@pytest.mark.parametrize("layers", [1, 2])
def test_forward_matches_torch_gru(layers):
    cfg = GRUConfig(vocab=50, embed=12, hidden=9, layers=layers)
    p = p64(cfg)
    x = torch.randint(0, 50, (3, 7))
    gru = torch.nn.GRU(12, 9, layers, batch_first=True).double()
    with torch.no_grad():
        for l in range(layers):
            for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
                getattr(gru, f"{n}_l{l}").copy_(p[f"{n}_l{l}"])
    h, _ = gru(p["embedding"][x])
    ref = h @ p["fc.weight"].T + p["fc.bias"]
    torch.testing.assert_close(cpu_ref.forward(p, cfg, x), ref, atol=1e-12, rtol=1e-10)


@pytest.mark.parametrize("layers", [1, 2, 3])
def test_manual_bptt_matches_autograd(layers):
    cfg = GRUConfig(vocab=40, embed=10, hidden=8, layers=layers)
    p = p64(cfg, 3)
    x, y = NameStream(4, 9, seed=2).next()
    x, y = np.clip(x, 0, 39), np.clip(y, 0, 39)
    y[1, 4:] = -1
    l1, g1 = cpu_ref.manual_backward(p, cfg, torch.from_numpy(x), torch.from_numpy(y))
    l2, g2 = cpu_ref.autograd_grads(p, cfg, torch.from_numpy(x), torch.from_numpy(y))
    assert abs(float(l1 - l2)) < 1e-12
    for k in g2:
        torch.testing.assert_close(g1[k], g2[k], atol=1e-12, rtol=1e-9)


def test_finite_differences():
    cfg = GRUConfig(vocab=20, embed=4, hidden=3, layers=2)
    p = p64(cfg, 1)
    x = torch.randint(0, 20, (2, 5))
    y = torch.randint(0, 20, (2, 5))
    _, g = cpu_ref.manual_backward(p, cfg, x, y)
    rng = np.random.default_rng(0)
    for name in ("weight_hh_l0", "bias_ih_l1", "embedding", "fc.weight"):
        for _ in range(3):
            idx = tuple(int(rng.integers(s)) for s in p[name].shape)
            eps = 1e-6
            q = {k: v.clone() for k, v in p.items()}
            q[name][idx] += eps
            lp = cpu_ref.xent(cpu_ref.forward(q, cfg, x), y)
            q[name][idx] -= 2 * eps
            lm = cpu_ref.xent(cpu_ref.forward(q, cfg, x), y)
            fd = float(lp - lm) / (2 * eps)
            assert abs(fd - float(g[name][idx])) < 1e-6 + 1e-5 * abs(fd), (name, idx)


@settings(max_examples=200, deadline=None)
@given(st.lists(st.floats(0.0, 1.0), min_size=1, max_size=40), st.floats(0.0, 1.0))
def test_sampler_is_first_index_with_running_sum_above_r(ws, r):
    """namegensf.cu:322-333: first i with fp32 psum > r, in index order; else n-1."""
    p = torch.tensor(ws, dtype=torch.float32)
    got = int(cpu_ref.sample_inverse_cdf(p[None], torch.tensor([r], dtype=torch.float32))[0])
    psum, exp = np.float32(0.0), len(ws) - 1
    for i, v in enumerate(p.numpy()):
        psum = np.float32(psum + v)
        if psum > np.float32(r):
            exp = i
            break
    assert got == exp


def test_generation_semantics_eos_written_then_nul():
    cfg = GRUConfig(vocab=64, embed=8, hidden=16, layers=2, max_len=12, sos=0, eos=0)
    p = p64(cfg, 2)
    rf = random_floats(50, cfg.max_len, seed=1)
    out = cpu_ref.generate(p, cfg, rf)
    assert out.shape == (50, 13)
    for row in out:
        z = np.flatnonzero(row == 0)
        first = z[0]
        assert np.all(row[first:] == 0)      # EOS (== NUL here) written, then nothing
    cfg2 = cfg.replace(eos=5)
    out2 = cpu_ref.generate(p, cfg2, rf)
    for row in out2:
        hit = np.flatnonzero(row[:cfg.max_len] == 5)
        if hit.size:
            assert np.all(row[hit[0] + 1:] == 0)   # stopped right after writing EOS
    assert np.all(out2[:, -1] == 0)               # MAX_LEN+1-th byte always NUL


def test_generation_uses_global_random_index():
    """name n at step l consumes random_floats[n*MAX_LEN + l] -> any split of the
    name range into slices produces the same names."""
    cfg = GRUConfig(vocab=64, embed=8, hidden=16, layers=2, max_len=8, eos=3)
    p = p64(cfg, 4)
    rf = random_floats(37, cfg.max_len, seed=9)
    full = cpu_ref.generate(p, cfg, rf)
    parts = [cpu_ref.generate(p, cfg, rf, s, c) for s, c in ((0, 10), (10, 14), (24, 13))]
    np.testing.assert_array_equal(np.concatenate(parts), full)


def test_adam_and_training_reduce_loss():
    from gru_mpi_cuda_amd.engine.trainer import CpuTrainer
    cfg = PRESETS["cpu_tiny"].replace(lr=1e-2)
    tr = CpuTrainer(cfg)
    ds = NameStream(cfg.batch, cfg.seq, seed=0)
    losses = []
    for _ in range(40):
        tr.step(*ds.next())
        losses.append(tr.loss())
    assert np.mean(losses[-5:]) < np.mean(losses[:5]) - 0.5


def test_clip_norm_and_sgd():
    cfg = GRUConfig(vocab=20, embed=4, hidden=3, layers=1, clip_norm=0.1, optimizer="sgd", lr=0.5)
    p = {k: v.clone() for k, v in init_params(cfg).items()}
    g = {k: torch.ones_like(v) for k, v in p.items()}
    n = float(torch.sqrt(sum((v ** 2).sum() for v in g.values())))
    q = {k: v.clone() for k, v in p.items()}
    cpu_ref.Adam(cfg, q).step(q, g)
    for k in p:
        torch.testing.assert_close(p[k] - q[k], 0.5 * g[k] * (0.1 / (n + 1e-6)))


def test_config_param_counts_match_survey():
    # SURVEY §6.2 parameter counts (E = H, V = 256)
    assert PRESETS["cpu_tiny"].num_params() == 57_984
    assert PRESETS["h512"].num_params() == 1_838_336
    assert PRESETS["h1024_l2"].num_params() == 13_119_744
    assert PRESETS["h2048"].num_params() == 26_226_944


def test_data_streams():
    a = NameStream(8, 12, seed=3).next()
    b = NameStream(8, 12, seed=3).next()
    np.testing.assert_array_equal(a[0], b[0])
    x, y = a
    assert x.shape == y.shape == (8, 12)
    np.testing.assert_array_equal(x[:, 1:], y[:, :-1])     # next-char targets
    xp, yp = make_padded_batch(synthetic_names(5, seed=1), 16)
    assert (yp == -1).any() and (xp[:, 0] == 0).all()


@pytest.mark.parametrize("layers", [1, 2])
def test_truncated_bptt_carried_state(layers):
    """carry_hidden: h0 is a constant of the step -- manual BPTT with h0 equals
    autograd with a detached h0, and CpuTrainer carries each step's final state into the next."""
    from gru_mpi_cuda_amd.engine.trainer import CpuTrainer
    cfg = GRUConfig(vocab=256, embed=24, hidden=16, layers=layers, batch=6, seq=5, seed=3, carry_hidden=True)
    p = {k: v.double() for k, v in init_params(cfg).items()}
    ds = NameStream(cfg.batch, cfg.seq, seed=9)
    x, y = (torch.from_numpy(a) for a in ds.next())
    h0 = [torch.randn(cfg.batch, cfg.hidden, dtype=torch.float64) * 0.5 for _ in range(layers)]
    out = []
    loss, g = cpu_ref.manual_backward(p, cfg, x, y, h0=h0, state_out=out)
    loss_a, g_a = cpu_ref.autograd_grads(p, cfg, x, y, h0=h0)
    assert abs(float(loss) - float(loss_a)) < 1e-10
    for k in g:
        torch.testing.assert_close(g[k], g_a[k], atol=1e-10, rtol=1e-8)
    logits, caches = cpu_ref.forward(p, cfg, x, h0=h0, keep_cache=True)
    for l in range(layers):
        torch.testing.assert_close(out[l], caches[l]["out"][:, -1])
    # the trainer: step 2 starts from step 1's final state; reset_state goes back to zeros
    ct = CpuTrainer(cfg.replace(lr=0.0), params={k: v.float() for k, v in p.items()})
    b1, b2 = ds.next(), ds.next()
    ct.forward_backward(*b1)
    s1 = [h.clone() for h in ct._state]
    ct.forward_backward(*b2)
    pf = {k: v.float() for k, v in p.items()}
    ref_loss, _ = cpu_ref.manual_backward(pf, cfg, torch.from_numpy(b2[0]), torch.from_numpy(b2[1]), h0=s1)
    assert abs(ct.loss() - float(ref_loss)) < 1e-5
    ct.reset_state()
    ct.forward_backward(*b2)
    ref0, _ = cpu_ref.manual_backward(pf, cfg, torch.from_numpy(b2[0]), torch.from_numpy(b2[1]))
    assert abs(ct.loss() - float(ref0)) < 1e-5
