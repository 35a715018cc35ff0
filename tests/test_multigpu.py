"""Multi-GPU tier (SURVEY §4.2 'Distributed on GPU'): the same checks as tests/test_dist_cpu.py, on
the HIP engine with the native RCCL communicator, one process per GPU over xGMI.

    (a) data-parallel training: P ranks x B/P sequences == 1 GPU x B, step for step (bf16 engine,
        in-graph RCCL all-reduce of the readiness-ordered gradient groups);
    (b) the bench's data-parallel step runs and reports one JSON line.

Needs >= 2 visible GPUs; skipped otherwise (the 1-GPU test boxes run tests/test_engine_gpu.py's
1-rank-communicator test of the same graph structure instead).  Launched through
torch.distributed.run with 127.0.0.1 rendezvous, each worker a separate process (no GPU state
in the pytest process)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gpus() -> int:
    try:
        return torch.cuda.device_count()
    except Exception:
        return 0


needs2 = pytest.mark.skipif(_gpus() < 2, reason="needs >= 2 GPUs")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


WORKER = r'''
import json, os, sys, torch
sys.path.insert(0, os.environ["GK_ROOT"])
from gru_mpi_cuda_amd.config import GRUConfig, preset
from gru_mpi_cuda_amd.models.params import init_params
from gru_mpi_cuda_amd.parallel import dist as gdist
from gru_mpi_cuda_amd.parallel.rccl import make_comm
from gru_mpi_cuda_amd.engine.trainer import HipTrainer
from gru_mpi_cuda_amd.utils.data import NameStream
ctx = gdist.init(use_gpu=True)
cfg = GRUConfig(**json.loads(os.environ["GK_CFG"]))
stream = NameStream(cfg.batch, cfg.seq, seed=21)
batches = [stream.next() for _ in range(3)]
per = cfg.batch // ctx.world
comm = make_comm(ctx)
assert comm is None or comm.count() == ctx.world
tr = HipTrainer(cfg, ctx, params=init_params(cfg), comm=comm)
for x, y in batches:   # every rank takes its contiguous slice of the same global batch
    tr.step(x[ctx.rank * per:(ctx.rank + 1) * per], y[ctx.rank * per:(ctx.rank + 1) * per])
torch.cuda.synchronize()
if ctx.rank == 0:
    torch.save({k: v for k, v in tr.state_dict().items()}, os.environ["GK_OUT"])
gdist.shutdown()
'''


def _run(n, script_path, out, timeout=240, cfg=None):
    env = dict(os.environ, GK_ROOT=ROOT, GK_OUT=out, HSA_ENABLE_IPC_MODE_LEGACY="0",
               GK_CFG=json.dumps(cfg or BASE_CFG))
    if n == 1:
        cmd = [sys.executable, script_path]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), script_path]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    return p


BASE_CFG = dict(vocab=256, embed=256, hidden=256, layers=1, batch=128, seq=8, seed=5, lr=0.5, optimizer="sgd")
# the headline h512 shape at 256 sequences per rank, and the 2-layer readiness-ordered flush path
# (bucket_mb 0.25: the top layer's group goes out while layer 0 is still in its backward)
H512_CFG = dict(vocab=256, embed=512, hidden=512, layers=1, batch=256, seq=32, seed=5, lr=0.2, optimizer="sgd")
L2_CFG = dict(vocab=256, embed=256, hidden=256, layers=2, batch=128, seq=8, seed=5, lr=0.5, optimizer="sgd",
              bucket_mb=0.25)


def _world_sizes():
    return [n for n in (2, 4, 8) if n <= _gpus()]


def _compare_dp(tmp_path, n, cfg, tol):
    a, b = str(tmp_path / "p1.pt"), str(tmp_path / f"p{n}.pt")
    worker = tmp_path / "worker.py"
    worker.write_text(WORKER)
    _run(1, str(worker), a, cfg=cfg)      # same global batch: each rank takes its slice
    _run(n, str(worker), b, cfg=cfg)
    pa = torch.load(a, weights_only=True)
    pb = torch.load(b, weights_only=True)
    # SGD (an update proportional to the gradient, unlike Adam's sign-like steps on near-zero
    # gradients); the mean over ranks differs from the 1-GPU sum only in fp32 summation order
    for k in pa:
        d = (pa[k] - pb[k]).abs().max().item()
        assert d < tol, f"{k}: max |diff| {d}"


@needs2
def test_dp_training_on_gpus_equals_one_gpu(tmp_path):
    n = 2 if _gpus() < 4 else 4
    _compare_dp(tmp_path, n, BASE_CFG, 1e-4)


@needs2
@pytest.mark.parametrize("n", [2, 4, 8])
def test_dp_h512_on_gpus_equals_one_gpu(tmp_path, n):
    """SURVEY §4.2 'Distributed on GPU' at the headline shape: P ranks x 256/P sequences of the
    h512 model (persistent kernels, fused dW_hh + dP, dP all-reduced in the W_ih0 slot) equal one
    GPU x 256 sequences after 3 SGD steps."""
    if n > _gpus():
        pytest.skip(f"needs {n} GPUs")
    _compare_dp(tmp_path, n, H512_CFG, 2e-4)


@needs2
def test_dp_two_layer_flush_path_equals_one_gpu(tmp_path):
    _compare_dp(tmp_path, 2, L2_CFG, 1e-4)


@needs2
def test_dp_sharded_optimizer_equals_one_gpu(tmp_path):
    """ZeRO-1 step at world 2 (reduce-scatter, SGD on the owned half, all-gather of the fp32
    masters) equals one GPU on the whole batch."""
    _compare_dp(tmp_path, 2, dict(H512_CFG, shard_optim=True), 2e-4)


@needs2
def test_bench_dp_step_reports():
    n = 2
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py",
                        "--gpus", str(n), "--steps", "10", "--warmup", "3"],
                       env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    r = json.loads(line)
    assert r["n_gpus"] == n and r["config"]["global_batch"] == 256 * n and r["value"] > 0
    assert r["config"]["collectives"] >= 1


CAPI_WORKER_N = 203   # N % P != 0 for P = 2, 4, 8 (the reference drops those names, cu:628-630)


@needs2
@pytest.mark.parametrize("n", [2, 4, 8])
def test_capi_namegen_identical_across_world_sizes(tmp_path, n):
    """SURVEY §3.2 invariant on the native C API (no Python in the path): bin/namegen under the
    one-process-per-GPU launcher writes byte-identical names at world 1 and world n, including
    N % n != 0 (RCCL broadcast of the uniforms + all-gather of the name slabs)."""
    if n > _gpus():
        pytest.skip(f"needs {n} GPUs")
    from gru_mpi_cuda_amd.config import GRUConfig
    from gru_mpi_cuda_amd.models.params import init_params
    from gru_mpi_cuda_amd.utils import ckpt
    binp = os.path.join(ROOT, "gru_mpi_cuda_amd", "bin", "namegen")
    cfg = GRUConfig(vocab=256, embed=256, hidden=256, layers=2, max_len=10, sos=0, eos=0)
    params = init_params(cfg, seed=3)
    params["fc.weight"] = params["fc.weight"] * 6
    path = str(tmp_path / "model.bin")
    ckpt.save(path, cfg, params, fmt="gen")
    outs = {}
    for w in (1, n):
        out = str(tmp_path / f"names_{w}.txt")
        cmd = [sys.executable, "-m", "gru_mpi_cuda_amd.parallel.launch", "--nproc", str(w), "--timeout", "240",
               "--no-python", "--", binp, path, out, str(CAPI_WORKER_N), "5"]
        p = subprocess.run(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"), capture_output=True,
                           text=True, timeout=300, cwd=ROOT)
        assert p.returncode == 0, p.stderr[-3000:]
        outs[w] = open(out, "rb").read()
    assert outs[1] == outs[n] and outs[1].count(b"\n") == CAPI_WORKER_N
