"""Host-side sanitizer tier: the native checkpoint reader that the C API uses
(csrc/capi/ckpt_reader.cpp) runs under AddressSanitizer + UBSan (bin/ckpt_check_asan, built by
build_ext with g++).  GPU sanitizers are not available on the target pool, so the device side is
covered by the numerics tests instead."""
import json
import os
import subprocess

import numpy as np
import pytest

from gru_mpi_cuda_amd.build_ext import build_host_tools
from gru_mpi_cuda_amd.config import GRUConfig
from gru_mpi_cuda_amd.models.params import init_params
from gru_mpi_cuda_amd.utils import ckpt


@pytest.fixture(scope="module")
def tools():
    return dict(zip(("plain", "asan"), build_host_tools()))


def _run(exe, path, env=None):
    e = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", **(env or {}))
    return subprocess.run([exe, path], capture_output=True, text=True, env=e, timeout=60)


@pytest.mark.parametrize("fmt,layers", [("gen", 1), ("gen", 2), ("ref", 2)])
def test_reader_under_asan_matches_python(tools, tmp_path, fmt, layers):
    cfg = GRUConfig(vocab=256, embed=64, hidden=96, layers=layers)
    p = init_params(cfg, seed=5)
    path = str(tmp_path / "m.bin")
    ckpt.save(path, cfg, p, fmt=fmt)
    env = {} if fmt == "gen" else {"GK_VOCAB": "256", "GK_EMBED": "64", "GK_HIDDEN": "96", "GK_LAYERS": str(layers)}
    r = _run(tools["asan"], path, env)
    assert r.returncode == 0, r.stderr
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
    out = json.loads(r.stdout)
    assert out["total"] == ckpt.blob_floats(cfg)
    for name, t in p.items():
        off, n, s = out["tensors"][name]
        assert n == t.numel()
        assert abs(s - float(t.double().sum())) <= 1e-6 * max(1.0, float(t.double().abs().sum()))
    # the plain build agrees byte for byte
    assert _run(tools["plain"], path, env).stdout == r.stdout


@pytest.mark.parametrize("delta", [-4, 4, -4096])
def test_wrong_size_blob_is_rejected_cleanly(tools, tmp_path, delta):
    cfg = GRUConfig(vocab=256, embed=64, hidden=96, layers=1)
    path = str(tmp_path / "m.bin")
    ckpt.save(path, cfg, init_params(cfg), fmt="gen")
    raw = open(path, "rb").read()
    open(path, "wb").write(raw[:delta] if delta < 0 else raw + b"\0" * delta)
    r = _run(tools["asan"], path)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "need" in r.stderr and "AddressSanitizer" not in r.stderr


def test_missing_file(tools, tmp_path):
    r = _run(tools["asan"], str(tmp_path / "nope.bin"))
    assert r.returncode == 3 and "cannot open" in r.stderr
