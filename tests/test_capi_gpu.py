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


def test_capi_repeated_calls_reuse_device_buffers(tmp_path):
    """C-API hygiene: namegen() keeps its uniform / output device buffers across
    calls (no hipMalloc per call once the largest N has been seen), and repeated calls with the same
    uniforms give the same names as the Python-driven generator."""
    lib = os.path.join(ROOT, "gru_mpi_cuda_amd", "bin", "libnamegen.so")
    assert os.path.exists(lib), "build the extension first"
    cfg = GRUConfig(vocab=256, embed=256, hidden=256, layers=2, max_len=10, sos=0, eos=0)
    params = init_params(cfg, seed=5)
    path = str(tmp_path / "model.bin")
    ckpt.save(path, cfg, params, fmt="gen")
    script = tmp_path / "run.py"
    script.write_text(f'''
import ctypes, sys
import numpy as np
lib = ctypes.CDLL({lib!r})
lib.namegen_device_allocs.restype = ctypes.c_long
N, ML = 300, {cfg.max_len}
rf = np.random.default_rng(7).random(N * ML, dtype=np.float32)
lib.namegen_initialize(N, 0, {path!r}.encode())
outs, allocs = [], []
for n in (N, N, 120, N):
    out = ctypes.create_string_buffer(n * (ML + 1))
    lib.namegen(n, rf.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), out)
    outs.append(out.raw)
    allocs.append(lib.namegen_device_allocs())
lib.namegen_finalize()
np.save(sys.argv[1], np.frombuffer(b"".join(outs), dtype=np.uint8))
print("allocs", allocs)
''')
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    res = str(tmp_path / "out.npy")
    r = subprocess.run(["python3", str(script), res], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    allocs = eval(r.stdout.strip().split("allocs", 1)[1])
    assert allocs[0] == allocs[-1] == 2, allocs      # uniforms + output rows, allocated once
    raw = np.load(res).tobytes()
    row = cfg.max_len + 1
    a, b, c, d = raw[:300 * row], raw[300 * row:600 * row], raw[600 * row:720 * row], raw[720 * row:]
    assert a == b == d and c == a[:120 * row]
    from gru_mpi_cuda_amd.engine.generator import HipGenerator
    rf = np.random.default_rng(7).random(300 * cfg.max_len, dtype=np.float32)
    py = HipGenerator(cfg, params).generate(rf)
    assert a == bytes(np.asarray(py, dtype=np.uint8).tobytes())
