"""Checkpoint I/O: the reference's headerless OFFSET0..26 layout (SURVEY Appendix A,
/root/reference/namegensf.cu:375-407) and the generalised self-describing format."""
import numpy as np
import pytest
import torch

from gru_mpi_cuda_amd.config import GRUConfig, preset
from gru_mpi_cuda_amd.models.params import init_params, flat_layout, to_flat, from_flat
from gru_mpi_cuda_amd.utils import ckpt


def test_reference_offsets_match_appendix_a():
    cfg = preset("ref")            # V=256, E=512, H=1024, L=2
    offs = {name: off for name, off, _ in ckpt.ref_offsets(cfg)}
    H = 1024
    # Appendix A, in floats
    assert offs["embedding"] == 0
    assert offs["weight_ih_l0"] == 131_072            # W_ir0 (W_iz0 at +H*E, W_in0 at +2H*E)
    assert offs["weight_ih_l0"] + H * 512 == 655_360
    assert offs["weight_ih_l1"] == 1_703_936
    assert offs["weight_hh_l0"] == 4_849_664
    assert offs["bias_ih_l0"] == 11_141_120
    assert offs["bias_hh_l0"] == 11_147_264
    assert offs["fc.weight"] == 11_153_408
    assert offs["fc.bias"] == 11_415_552
    assert ckpt.blob_floats(cfg) == 11_415_808        # 45,663,232 bytes


def test_reference_split_names():
    cfg = GRUConfig(vocab=64, embed=8, hidden=4, layers=2)
    p = init_params(cfg)
    parts = ckpt.reference_split(cfg, p)
    assert len(parts) == 27
    assert torch.equal(parts["W_iz1"], p["weight_ih_l1"][4:8])
    assert torch.equal(parts["b_hn0"], p["bias_hh_l0"][8:12])


@pytest.mark.parametrize("fmt", ["gen", "ref"])
@pytest.mark.parametrize("layers", [1, 2, 3])
def test_round_trip(tmp_path, fmt, layers):
    cfg = GRUConfig(vocab=64, embed=16, hidden=8, layers=layers, max_len=7, sos=1, eos=2)
    p = init_params(cfg, seed=5)
    path = str(tmp_path / "m.bin")
    ckpt.save(path, cfg, p, fmt=fmt)
    cfg2, q = ckpt.load(path, cfg if fmt == "ref" else None)
    assert (cfg2.vocab, cfg2.embed, cfg2.hidden, cfg2.layers) == (64, 16, 8, layers)
    if fmt == "gen":
        assert (cfg2.max_len, cfg2.sos, cfg2.eos) == (7, 1, 2)
    for k in p:
        assert torch.equal(p[k], q[k]), k


def test_blob_is_plain_little_endian_fp32_in_reference_order(tmp_path):
    cfg = GRUConfig(vocab=4, embed=2, hidden=1, layers=2)
    p = init_params(cfg)
    path = str(tmp_path / "r.bin")
    ckpt.save(path, cfg, p, fmt="ref")
    blob = np.fromfile(path, dtype="<f4")
    exp = np.concatenate([p[n].numpy().ravel() for n in
                          ["embedding", "weight_ih_l0", "weight_ih_l1", "weight_hh_l0", "weight_hh_l1",
                           "bias_ih_l0", "bias_ih_l1", "bias_hh_l0", "bias_hh_l1", "fc.weight", "fc.bias"]])
    np.testing.assert_array_equal(blob, exp)


def test_size_mismatch_is_rejected(tmp_path):
    cfg = GRUConfig(vocab=64, embed=16, hidden=8, layers=2)
    path = str(tmp_path / "r.bin")
    ckpt.save(path, cfg, init_params(cfg), fmt="ref")
    with pytest.raises(ValueError, match="floats"):
        ckpt.load(path, cfg.replace(hidden=16), fmt="ref")
    with pytest.raises(ValueError, match="headerless"):
        ckpt.load(path, None, fmt="ref")


def test_optimizer_state_round_trip(tmp_path):
    cfg = GRUConfig(vocab=64, embed=16, hidden=8, layers=1)
    p = init_params(cfg)
    st = {"m": torch.randn(10), "v": torch.rand(10), "step": torch.tensor([3])}
    path = str(tmp_path / "m.bin")
    ckpt.save(path, cfg, p, opt_state=st)
    st2 = ckpt.load_opt_state(path)
    for k in st:
        assert torch.equal(st[k], st2[k])


def test_flat_layout_aligned_and_readiness_ordered():
    cfg = GRUConfig(vocab=256, embed=64, hidden=64, layers=2)
    lay = flat_layout(cfg)
    assert all(s.offset % 64 == 0 for s in lay.segments)
    names = [s.name for s in lay.segments]
    assert names[:2] == ["fc.weight", "fc.bias"] and names[-1] == "embedding"
    assert names.index("weight_hh_l1") < names.index("weight_hh_l0")
    p = init_params(cfg)
    q = from_flat(cfg, to_flat(cfg, p))
    for k in p:
        assert torch.equal(p[k], q[k])
