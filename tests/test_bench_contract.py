"""bench.py's output contract (one JSON line from rank 0, K timed steps, whole-job value, max over
ranks), rehearsed on the CPU path: world 1 directly, worlds 2 and 8 under torch.distributed.run with
gloo and 127.0.0.1 rendezvous -- the same launcher line the driver uses for N GPUs."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _lines(cmd, n, env=None):
    env = dict(env if env is not None else os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout   # rank 0 only
    r = json.loads(lines[0])
    assert KEYS <= set(r), set(r) ^ KEYS
    assert r["n_gpus"] == n and r["steps"] == 3 and r["warmup"] == 1
    assert r["higher_is_better"] is True and r["scaling"] == "weak"
    cfg = r["config"]
    assert cfg["parallelism"] == f"dp{n}" and cfg["global_batch"] == 4 * n and cfg["seq_len"] == 16
    # value is the whole-job aggregate: global tokens over the (max-over-ranks) timed span
    tok = cfg["global_batch"] * cfg["seq_len"] * r["steps"]
    assert abs(r["value"] - tok / (r["ms_per_step"] * r["steps"] / 1000)) / r["value"] < 0.01
    return r


def test_bench_contract_world1():
    _lines([sys.executable, "bench.py", "--preset", "cpu_tiny", "--steps", "3", "--warmup", "1"], 1)


@pytest.mark.parametrize("world", [2, 8])
def test_bench_contract_torchrun_gloo(world):
    """The driver's multi-GPU form (torchrun, one rank per device, up to a whole 8-GPU node),
    rehearsed on CPU with gloo: one JSON line from rank 0 with n_gpus == world."""
    r = _lines([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
                "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py",
                "--gpus", str(world), "--preset", "cpu_tiny", "--steps", "3", "--warmup", "1"], world)
    assert r["rccl_ranks"] == world


def test_bench_self_launches_world2():
    """``bench.py --gpus 2`` with no launcher starts its own 2 ranks (parallel/launch.py) and still
    prints exactly one JSON line with n_gpus 2 (--gpus must not be a no-op)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = _lines([sys.executable, "bench.py", "--gpus", "2", "--preset", "cpu_tiny", "--steps", "3",
                "--warmup", "1"], 2, env=env)
    assert r["rccl_ranks"] == 2 and r["comm_backend"] == "gloo"


def test_bench_sharded_optimizer_world2():
    """``--shard-optim`` through the self-launched 2-rank job: same contract, flag reported, and the
    same final loss as the replicated optimiser (the CPU twin is bitwise equal)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    args = [sys.executable, "bench.py", "--gpus", "2", "--preset", "cpu_tiny", "--steps", "3", "--warmup", "1"]
    a = _lines(args, 2, env=env)
    b = _lines(args + ["--shard-optim"], 2, env=env)
    assert b["config"]["shard_optim"] == 1 and a["config"]["shard_optim"] == 0
    assert a["final_loss"] == b["final_loss"]
    assert b["extra_warmup_steps"] == 0     # the GPU clock-ramp warm-up only runs on GPUs
    c = _lines(args + ["--shard-optim", "2"], 2, env=env)   # bf16 working copies gathered
    assert c["config"]["shard_optim"] == 2 and abs(c["final_loss"] - a["final_loss"]) < 0.05 * a["final_loss"]


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--preset", "cpu_tiny", "--steps", "1",
                        "--warmup", "0"], env=env, capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert p.returncode == 2 and "WORLD_SIZE=1" in p.stderr
