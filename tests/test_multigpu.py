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
steps = int(os.environ.get("GK_STEPS", "3"))
inject = int(os.environ.get("GK_INJECT", "-1"))     # rank that raises the error word before step 2
stream = NameStream(cfg.batch, cfg.seq, seed=21)
batches = [stream.next() for _ in range(steps)]
per = cfg.batch // ctx.world
comm = make_comm(ctx)
if comm is None and os.environ.get("GK_FORCE_COMM") == "1":   # 1-rank communicator (twin runs)
    from gru_mpi_cuda_amd.ops import load_ext
    C = load_ext()
    comm = C.RcclComm(C.RcclComm.unique_id(), 0, 1)
assert comm is None or comm.count() == ctx.world
tr = HipTrainer(cfg, ctx, params=init_params(cfg), comm=comm)
after1 = None
for i, (x, y) in enumerate(batches):   # every rank takes its contiguous slice of the same global batch
    if i == 1 and ctx.rank == inject:
        tr.t.inject_error(1)
    tr.step(x[ctx.rank * per:(ctx.rank + 1) * per], y[ctx.rank * per:(ctx.rank + 1) * per])
    if i == 0:
        torch.cuda.synchronize()
        after1 = {k: v.clone() for k, v in tr.state_dict().items()}
torch.cuda.synchronize()
out = {"p": {k: v for k, v in tr.state_dict().items()}, "after1": after1, "err": int(tr.t.read_error()),
       "plan": tr.t.plan()}
if ctx.rank == 0 or os.environ.get("GK_SAVE_ALL") == "1":
    torch.save(out, os.environ["GK_OUT"].replace(".pt", f"_r{ctx.rank}.pt") if ctx.rank else os.environ["GK_OUT"])
gdist.shutdown()
'''


def _run(n, script_path, out, timeout=240, cfg=None, **extra):
    env = dict(os.environ, GK_ROOT=ROOT, GK_OUT=out, HSA_ENABLE_IPC_MODE_LEGACY="0",
               GK_CFG=json.dumps(cfg or BASE_CFG), **{k: str(v) for k, v in extra.items()})
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


def _dp_pair(tmp_path, n, cfg, **extra):
    a, b = str(tmp_path / "p1.pt"), str(tmp_path / f"p{n}.pt")
    worker = tmp_path / "worker.py"
    worker.write_text(WORKER)
    _run(1, str(worker), a, cfg=cfg, **extra)      # same global batch: each rank takes its slice
    _run(n, str(worker), b, cfg=cfg, **extra)
    return torch.load(a, weights_only=True), torch.load(b, weights_only=True)


def _compare_dp(tmp_path, n, cfg, tol):
    pa, pb = (r["p"] for r in _dp_pair(tmp_path, n, cfg))
    # SGD (an update proportional to the gradient, unlike Adam's sign-like steps on near-zero
    # gradients); the mean over ranks differs from the 1-GPU sum only in fp32 summation order
    for k in pa:
        d = (pa[k] - pb[k]).abs().max().item()
        assert d < tol, f"{k}: max |diff| {d}"


def _adam_close(pa, pb, lr, steps):
    """Adam's first steps are sign-like (m / sqrt(v) = +-1 at step 1), so an element whose gradient
    is at fp32 rounding level may step the other way under another summation order: bound the
    worst element by 2 lr per step and require all but a handful to agree to 1e-6."""
    for k in pa:
        d = (pa[k] - pb[k]).abs()
        assert d.max().item() <= 2 * lr * steps + 1e-6, (k, d.max().item())
        assert (d > 1e-6).float().mean().item() < 1e-3, (k, (d > 1e-6).float().mean().item())


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
@pytest.mark.parametrize("pipe", [1, 0])
def test_dp_h512_tail_modes_equal_one_gpu(tmp_path, pipe):
    """Both one-layer data-parallel tails at world 2: the bucketed, pipelined one (readiness buckets on a
    comm stream, opt-in; Trainer::record_dp_tail_l1) and the single collective after the backward (the
    default), each equal to one GPU on the whole batch."""
    _compare_dp(tmp_path, 2, dict(H512_CFG, dp_pipeline=pipe), 2e-4)


@needs2
def test_dp_two_layer_flush_path_equals_one_gpu(tmp_path):
    _compare_dp(tmp_path, 2, L2_CFG, 1e-4)


@needs2
@pytest.mark.parametrize("mode", [1, 2])
def test_dp_sharded_optimizer_equals_one_gpu(tmp_path, mode):
    """ZeRO-1 step at world 2 (reduce-scatter, SGD on the owned half, all-gather of the fp32
    masters (1) or of the bf16 working copies with the fp32 biases exchanged (2)) equals one GPU on
    the whole batch."""
    _compare_dp(tmp_path, 2, dict(H512_CFG, shard_optim=mode), 2e-4)


ADAM_CFG = dict(H512_CFG, optimizer="adam", lr=1e-3)
# BASELINE config #4 (2-layer H=1024, 1024 sequences, T=64) as the default plan runs it per rank:
# wavefront forward (both layers in one persistent launch), persistent backward per layer,
# readiness-ordered gradient groups flushed while the lower layer's backward runs
L2H1024_CFG = dict(vocab=256, embed=1024, hidden=1024, layers=2, batch=1024, seq=64, seed=5, lr=0.05,
                   optimizer="sgd")


@needs2
@pytest.mark.parametrize("n", [2, 4, 8])
def test_dp_adam_five_steps_equals_one_gpu(tmp_path, n):
    """Adam, the default optimizer, across ranks: P ranks x 256/P sequences of
    the headline model equal one GPU x 256 after 5 steps (gloo twin:
    tests/test_dist_cpu.py::test_dp_training_equals_single_rank; 1-rank twin below)."""
    if n > _gpus():
        pytest.skip(f"needs {n} GPUs")
    pa, pb = (r["p"] for r in _dp_pair(tmp_path, n, ADAM_CFG, GK_STEPS=5))
    _adam_close(pa, pb, ADAM_CFG["lr"], 5)


def test_dp_adam_five_steps_one_rank_twin(tmp_path):
    """1-GPU twin of the Adam DP test: the same worker with a 1-rank RCCL communicator (the
    data-parallel graph: grouped collectives + error word, slab sums materialised before the
    collective) against no communicator (the slab sums inside the fused Adam launch: another fp32
    summation order for dW_fc), 5 Adam steps."""
    worker = tmp_path / "worker.py"
    worker.write_text(WORKER)
    a, b = str(tmp_path / "nocomm.pt"), str(tmp_path / "comm1.pt")
    _run(1, str(worker), a, cfg=ADAM_CFG, GK_STEPS=5)
    _run(1, str(worker), b, cfg=ADAM_CFG, GK_STEPS=5, GK_FORCE_COMM=1)
    pa, pb = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    assert pa["err"] == 0 and pb["err"] == 0
    _adam_close(pa["p"], pb["p"], ADAM_CFG["lr"], 5)


@needs2
@pytest.mark.parametrize("n", [4, 8])
def test_dp_l2_h1024_default_plan_equals_one_gpu(tmp_path, n):
    """BASELINE config #4 with the default plan at 4 and 8 ranks (1024/P
    sequences each) equals one GPU on all 1024 sequences after 2 SGD steps; every rank runs the
    wavefront forward."""
    if n > _gpus():
        pytest.skip(f"needs {n} GPUs")
    ra, rb = _dp_pair(tmp_path, n, L2H1024_CFG, GK_STEPS=2)
    assert "fwd=persistent+wave" in rb["plan"], rb["plan"]
    for k in ra["p"]:
        d = (ra["p"][k] - rb["p"][k]).abs().max().item()
        assert d < 2e-4, f"{k}: max |diff| {d}"


def test_l2_h1024_default_plan_one_rank_twin(tmp_path):
    """1-GPU twin: the per-rank shard of the 8-rank run (128 sequences, L=2 H=1024, T=64) with a
    1-rank communicator equals the same shard without one and runs the wavefront forward."""
    worker = tmp_path / "worker.py"
    worker.write_text(WORKER)
    cfg = dict(L2H1024_CFG, batch=128)
    a, b = str(tmp_path / "nocomm.pt"), str(tmp_path / "comm1.pt")
    _run(1, str(worker), a, cfg=cfg, GK_STEPS=2)
    _run(1, str(worker), b, cfg=cfg, GK_STEPS=2, GK_FORCE_COMM=1)
    pa, pb = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    assert "fwd=persistent+wave" in pb["plan"], pb["plan"]
    for k in pa["p"]:
        d = (pa["p"][k] - pb["p"][k]).abs().max().item()
        assert d < 2e-4, f"{k}: max |diff| {d}"


@needs2
@pytest.mark.parametrize("n", [2, 8])
def test_error_word_agreement_across_gpus(tmp_path, n):
    """an error raised on ONE rank (the last one) before step 2 rides the
    last gradient collective as a max, so every rank skips that update and keeps its step-1 weights
    (gloo twin: tests/test_dist_cpu.py::test_error_word_is_global_across_ranks; 1-rank twin:
    tests/test_engine_gpu.py::test_error_word_rides_the_last_collective)."""
    if n > _gpus():
        pytest.skip(f"needs {n} GPUs")
    worker = tmp_path / "worker.py"
    worker.write_text(WORKER)
    out = str(tmp_path / "e.pt")
    _run(n, str(worker), out, cfg=ADAM_CFG, GK_STEPS=3, GK_INJECT=n - 1, GK_SAVE_ALL=1)
    res = [torch.load(out if r == 0 else out.replace(".pt", f"_r{r}.pt"), weights_only=True) for r in range(n)]
    for r, q in enumerate(res):
        assert q["err"] == 1, (r, q["err"])
        for k in q["p"]:
            assert torch.equal(q["p"][k], q["after1"][k]), (r, k)
            assert torch.equal(q["p"][k], res[0]["p"][k]), (r, k)


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
    N % n != 0 (RcclComm::scatterv_f32 of each rank's uniforms, gatherv_u8 of its name rows:
    grouped ncclSend / ncclRecv with the uneven remainder counts)."""
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
