"""Native 3-call C API + driver binary (no Python in the generation path) vs the Python-driven
HIP generator on the same checkpoint and the same uniforms."""
import os
import subprocess

import numpy as np
import pytest
import torch

from gru_mpi_cuda_amd.config import GRUConfig
from gru_mpi_cuda_amd.models.params import init_params
from gru_mpi_cuda_amd.utils import ckpt

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "gru_mpi_cuda_amd", "bin", "namegen")

M64 = (1 << 64) - 1


def splitmix_uniforms(n, seed):
    out = np.empty(n, dtype=np.float32)
    s = seed & M64
    for i in range(n):
        s = (s + 0x9E3779B97F4A7C15) & M64
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        z ^= z >> 31
        out[i] = np.float32((z >> 40) * (1.0 / 16777216.0))
    return out


def test_native_driver_matches_python_generator(tmp_path):
    from gru_mpi_cuda_amd.engine.generator import HipGenerator
    assert os.path.exists(BIN), "build the extension first (python -m gru_mpi_cuda_amd.build_ext)"
    cfg = GRUConfig(vocab=256, embed=256, hidden=256, layers=2, max_len=10, sos=0, eos=0)
    params = init_params(cfg, seed=3)
    params["fc.weight"] = params["fc.weight"] * 6
    path = str(tmp_path / "model.bin")
    ckpt.save(path, cfg, params, fmt="gen")
    N, seed = 200, 5
    out = str(tmp_path / "names.txt")
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([BIN, path, out, str(N), str(seed)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Hello world, rank 0 out of 1" in r.stdout
    native = open(out, "rb").read()
    rf = splitmix_uniforms(N * cfg.max_len, seed)
    py = HipGenerator(cfg, params).generate(rf)
    pyn = [bytes(row).split(b"\0", 1)[0] for row in py]
    # names of an untrained model may contain '\n' bytes: compare the whole file image
    assert native == b"".join(n + b"\n" for n in pyn)
