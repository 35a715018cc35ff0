"""Multi-process (gloo, CPU) tests of the distributed layer (SURVEY §4.2 'Distributed w/o GPUs').

(a) namegen over P ranks == namegen on 1 rank, including N % P != 0 (the reference drops
    those names, namegensf.cu:628-630; here the remainder is spread over the first ranks);
(b) data-parallel training of P ranks x B/P == 1 rank x B, step for step.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from gru_mpi_cuda_amd.config import GRUConfig
from gru_mpi_cuda_amd.models.params import init_params
from gru_mpi_cuda_amd.utils import ckpt
from gru_mpi_cuda_amd.utils.data import NameStream, random_floats


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))


def _namegen_worker(rank, world, port, path, N, outdir):
    _env(rank, world, port)
    from gru_mpi_cuda_amd.parallel import dist as gdist
    from gru_mpi_cuda_amd.engine import generator as G
    ctx = gdist.init(use_gpu=False)
    cfg = GRUConfig(max_len=9)
    rf = random_floats(N, 9, seed=7)
    G.namegen_initialize(N, 0, path, None, "gen", ctx=ctx)
    out = np.zeros(N * 10, dtype=np.uint8)
    G.namegen(N, rf, out)
    G.namegen_finalize()
    if rank == 0:
        np.save(os.path.join(outdir, f"names_{world}.npy"), out)
    gdist.shutdown()


@pytest.mark.parametrize("world,N", [(2, 37), (3, 20), (8, 29)])
def test_namegen_independent_of_world_size(tmp_path, world, N):
    cfg = GRUConfig(vocab=64, embed=8, hidden=16, layers=2, max_len=9, eos=3)
    path = str(tmp_path / "m.bin")
    ckpt.save(path, cfg, init_params(cfg, seed=11))
    ctx = mp.get_context("spawn")
    for w in (1, world):
        port = _free_port()
        procs = [ctx.Process(target=_namegen_worker, args=(r, w, port, path, N, str(tmp_path))) for r in range(w)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
            assert p.exitcode == 0
    a = np.load(tmp_path / "names_1.npy")
    b = np.load(tmp_path / f"names_{world}.npy")
    np.testing.assert_array_equal(a, b)
    assert (a.reshape(N, 10)[:, 0] != 0).any()


def _train_worker(rank, world, port, outdir, steps):
    _env(rank, world, port)
    from gru_mpi_cuda_amd.parallel import dist as gdist
    from gru_mpi_cuda_amd.engine.trainer import CpuTrainer
    ctx = gdist.init(use_gpu=False)
    cfg = GRUConfig(vocab=256, embed=16, hidden=16, layers=2, batch=8, seq=6, bucket_mb=0.001, lr=1e-2)
    tr = CpuTrainer(cfg, ctx, params=init_params(cfg, seed=1) if rank == 0 else init_params(cfg, seed=99))
    ds = NameStream(cfg.batch, cfg.seq, seed=5)
    per = cfg.batch // world
    for _ in range(steps):
        x, y = ds.next()
        tr.step(x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per])
    if rank == 0:
        torch.save({k: v for k, v in tr.state_dict().items()}, os.path.join(outdir, f"p_{world}.pt"))
    gdist.shutdown()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_training_equals_single_rank(tmp_path, world):
    ctx = mp.get_context("spawn")
    for w in (1, world):
        port = _free_port()
        procs = [ctx.Process(target=_train_worker, args=(r, w, port, str(tmp_path), 5)) for r in range(w)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(180)
            assert p.exitcode == 0
    a = torch.load(tmp_path / "p_1.pt", weights_only=True)
    b = torch.load(tmp_path / f"p_{world}.pt", weights_only=True)
    # fp32 sums in a different order; Adam (lr 1e-2) normalises tiny gradients, so compare at
    # 1 % of one update step
    for k in a:
        torch.testing.assert_close(a[k], b[k], atol=1e-4, rtol=1e-4)


def _pipe_worker(rank, world, port, outdir, steps, pipe):
    _env(rank, world, port)
    from gru_mpi_cuda_amd.parallel import dist as gdist
    from gru_mpi_cuda_amd.engine.trainer import CpuTrainer
    ctx = gdist.init(use_gpu=False)
    cfg = GRUConfig(vocab=256, embed=16, hidden=24, layers=1, batch=8, seq=6, lr=1e-2, dp_pipeline=pipe)
    tr = CpuTrainer(cfg, ctx, params=init_params(cfg, seed=1))
    assert tr._pipelined() == (world > 1 and pipe == 1)
    ds = NameStream(cfg.batch, cfg.seq, seed=5)
    per = cfg.batch // world
    for _ in range(steps):
        x, y = ds.next()
        tr.step(x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per])
    if rank == 0:
        m, v, n = tr.opt_state()
        torch.save({"p": tr.state_dict(), "m": m, "v": v, "n": n}, os.path.join(outdir, f"pipe{pipe}_{world}.pt"))
    gdist.shutdown()


@pytest.mark.parametrize("world", [2, 4])
def test_dp_pipelined_tail_equals_single_bucket(tmp_path, world):
    """CPU twin of the one-layer pipelined data-parallel tail (Trainer::record_dp_tail_l1): two
    readiness buckets (W_hh0 .. end with the error word, then the FC pair) and Adam in two parts of
    ONE step equal the single-bucket step at the same world size -- bitwise at world 2, where a
    two-rank sum has one order; at 4 gloo's ring order follows the buffer's chunking, so to fp32
    rounding -- and one rank with the whole batch."""
    ctx = mp.get_context("spawn")
    for w, pipe in ((world, 1), (world, 0), (1, 1)):
        port = _free_port()
        procs = [ctx.Process(target=_pipe_worker, args=(r, w, port, str(tmp_path), 4, pipe)) for r in range(w)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(180)
            assert p.exitcode == 0
    a = torch.load(tmp_path / f"pipe1_{world}.pt", weights_only=True)
    b = torch.load(tmp_path / f"pipe0_{world}.pt", weights_only=True)
    one = torch.load(tmp_path / "pipe1_1.pt", weights_only=True)
    assert a["n"] == b["n"] == one["n"] == 4
    tol = dict(atol=0, rtol=0) if world == 2 else dict(atol=1e-6, rtol=1e-4)
    for k in a["p"]:
        torch.testing.assert_close(a["p"][k], b["p"][k], **tol)
        torch.testing.assert_close(a["p"][k], one["p"][k], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(a["m"], b["m"], **tol)
    torch.testing.assert_close(a["v"], b["v"], **(tol if world == 2 else dict(atol=1e-9, rtol=1e-3)))


def _shard_worker(rank, world, port, outdir, steps, shard):
    _env(rank, world, port)
    from gru_mpi_cuda_amd.parallel import dist as gdist
    from gru_mpi_cuda_amd.engine.trainer import CpuTrainer
    ctx = gdist.init(use_gpu=False)
    cfg = GRUConfig(vocab=256, embed=12, hidden=20, layers=2, batch=12, seq=5, lr=1e-2, shard_optim=shard)
    tr = CpuTrainer(cfg, ctx, params=init_params(cfg, seed=1))
    if shard:
        c = tr.shard[0]
        assert c % 4 == 0 and c * world <= tr.layout.total < (c + 4) * world
    ds = NameStream(cfg.batch, cfg.seq, seed=5)
    per = cfg.batch // world
    for _ in range(steps):
        x, y = ds.next()
        tr.step(x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per])
    torch.save(tr.state_dict(), os.path.join(outdir, f"s{int(shard)}_{world}_r{rank}.pt"))
    gdist.shutdown()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_optimizer_equals_replicated(tmp_path, world):
    """ZeRO-1 step (cfg.shard_optim; the CPU twin of Trainer::set_shard_optim): Adam on the owned
    1/world slice + tail, then an all-gather of the masters, is bitwise the replicated step, and every
    rank ends with the same weights.  world 3 leaves a non-empty tail."""
    ctx = mp.get_context("spawn")
    for shard in (False, True):
        port = _free_port()
        procs = [ctx.Process(target=_shard_worker, args=(r, world, port, str(tmp_path), 3, shard))
                 for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(180)
            assert p.exitcode == 0
    ref = torch.load(tmp_path / f"s0_{world}_r0.pt", weights_only=True)
    for r in range(world):
        got = torch.load(tmp_path / f"s1_{world}_r{r}.pt", weights_only=True)
        for k in ref:
            assert torch.equal(ref[k], got[k]), (r, k)


def _shard_bf16_worker(rank, world, port, outdir, steps, mode):
    """mode 'rep': replicated step computing with bf16-rounded weight matrices (the device's working
    copies); 'zero2': ZeRO-1 with the bf16 working copies gathered (cfg.shard_optim = 2)."""
    _env(rank, world, port)
    from gru_mpi_cuda_amd.parallel import dist as gdist
    from gru_mpi_cuda_amd.engine.trainer import CpuTrainer
    ctx = gdist.init(use_gpu=False)
    cfg = GRUConfig(vocab=256, embed=12, hidden=20, layers=2, batch=16, seq=5, lr=1e-2,
                    shard_optim=2 if mode == "zero2" else 0)
    tr = CpuTrainer(cfg, ctx, params=init_params(cfg, seed=1), bf16_weights=True)
    ds = NameStream(cfg.batch, cfg.seq, seed=5)
    per = cfg.batch // world
    for _ in range(steps):
        x, y = ds.next()
        tr.step(x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per])
    cp = tr.compute_params()
    torch.save({"compute": {k: v.clone() for k, v in cp.items()}, "masters": tr.state_dict(), "loss": tr.loss()},
               os.path.join(outdir, f"b{mode}_{world}_r{rank}.pt"))
    gdist.shutdown()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_bf16_gather_equals_replicated(tmp_path, world):
    """ZeRO-1 with the bf16 working copies gathered (shard_optim = 2; CPU twin of Trainer::record_sharded_opt
    mode 2: Adam on the owned slice, its bf16 copy all-gathered, the owned fp32 biases exchanged as an
    integer sum) against the replicated step on bf16 working copies: after 3 steps every rank holds
    bitwise the same bf16 weights, fp32 biases and (after gather_params) fp32 masters."""
    ctx = mp.get_context("spawn")
    for mode in ("rep", "zero2"):
        port = _free_port()
        procs = [ctx.Process(target=_shard_bf16_worker, args=(r, world, port, str(tmp_path), 3, mode))
                 for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(240)
            assert p.exitcode == 0
    ref0 = torch.load(tmp_path / f"brep_{world}_r0.pt", weights_only=True)
    for r in range(world):
        ref = torch.load(tmp_path / f"brep_{world}_r{r}.pt", weights_only=True)
        got = torch.load(tmp_path / f"bzero2_{world}_r{r}.pt", weights_only=True)
        assert got["loss"] == ref["loss"]   # (the loss is the rank's own shard of the batch)
        for k in ref0["compute"]:           # every rank: the same weights
            assert torch.equal(ref0["compute"][k], ref["compute"][k]), (r, k)
        for part in ("compute", "masters"):
            for k in ref[part]:
                assert torch.equal(ref[part][k], got[part][k]), (r, part, k)


def test_shard_and_buckets():
    from gru_mpi_cuda_amd.parallel.dist import shard, bucket_bounds
    for n in (0, 1, 7, 37, 64):
        for w in (1, 2, 3, 8):
            parts = [shard(n, r, w) for r in range(w)]
            assert sum(c for _, c in parts) == n
            assert all(parts[i][0] + parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            assert max(c for _, c in parts) - min(c for _, c in parts) <= 1
    b = bucket_bounds(1000, 300, [0, 100, 350, 900])
    assert b[0][0] == 0 and b[-1][1] == 1000
    assert all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))


def _resume_worker(rank, world, port, path, outdir):
    _env(rank, world, port)
    from gru_mpi_cuda_amd.parallel import dist as gdist
    from gru_mpi_cuda_amd.engine.trainer import CpuTrainer
    from gru_mpi_cuda_amd.cli import load_checkpoint
    ctx = gdist.init(use_gpu=False)
    cfg = GRUConfig(vocab=256, embed=16, hidden=16, layers=2, batch=6, seq=6)
    tr = CpuTrainer(cfg, ctx, params=init_params(cfg, seed=50 + rank))
    # only rank 0 is given (and may open) the checkpoint; the others get it by broadcast
    step = load_checkpoint(tr, path if rank == 0 else None)
    torch.save({"p": tr.state_dict(), "m": dict(tr.opt.m), "step": step},
               os.path.join(outdir, f"resume_{rank}.pt"))
    gdist.shutdown()


def test_dp_resume_rank0_reads_and_broadcasts(tmp_path):
    """DP resume: rank 0 reads the checkpoint, weights + Adam moments + step
    reach every rank by broadcast; ranks > 0 never touch the file."""
    from gru_mpi_cuda_amd.engine.trainer import CpuTrainer
    from gru_mpi_cuda_amd.cli import save_checkpoint
    cfg = GRUConfig(vocab=256, embed=16, hidden=16, layers=2, batch=6, seq=6)
    src = CpuTrainer(cfg, params=init_params(cfg, seed=3))
    ds = NameStream(cfg.batch, cfg.seq, seed=2)
    for _ in range(2):
        src.step(*ds.next())
    path = str(tmp_path / "ck.bin")
    save_checkpoint(src, path)
    world = 3
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_resume_worker, args=(r, world, port, path, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    want = src.state_dict()
    for r in range(world):
        got = torch.load(tmp_path / f"resume_{r}.pt", weights_only=True)
        assert got["step"] == 2
        for k in want:
            torch.testing.assert_close(got["p"][k], want[k], atol=0, rtol=0)
            torch.testing.assert_close(got["m"][k], src.opt.m[k], atol=0, rtol=0)


def _shard_ckpt_worker(rank, world, port, outdir, mode):
    """mode 'straight': 4 steps.  'save': 2 steps, then save_checkpoint on EVERY rank (a collective
    with a sharded optimiser).  'resume': load that checkpoint, 2 more steps."""
    _env(rank, world, port)
    from gru_mpi_cuda_amd.parallel import dist as gdist
    from gru_mpi_cuda_amd.engine.trainer import CpuTrainer
    from gru_mpi_cuda_amd.cli import load_checkpoint, save_checkpoint
    ctx = gdist.init(use_gpu=False)
    cfg = GRUConfig(vocab=256, embed=12, hidden=20, layers=2, batch=12, seq=5, lr=1e-2, shard_optim=True)
    tr = CpuTrainer(cfg, ctx, params=init_params(cfg, seed=1))
    path = os.path.join(outdir, "shard_ck.bin")
    ds = NameStream(cfg.batch, cfg.seq, seed=5)
    batches = [ds.next() for _ in range(4)]
    per = cfg.batch // world
    todo = range(4) if mode == "straight" else (range(2) if mode == "save" else range(2, 4))
    if mode == "resume":
        assert load_checkpoint(tr, path if rank == 0 else None) == 2
    for i in todo:
        x, y = batches[i]
        tr.step(x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per])
    if mode == "save":
        save_checkpoint(tr, path)
    else:
        torch.save(tr.state_dict(), os.path.join(outdir, f"shard_{mode}_r{rank}.pt"))
    gdist.shutdown()


def test_sharded_optimizer_checkpoint_resume(tmp_path):
    """with --shard-optim the moments live in 1/world slices.  save_checkpoint gathers
    them on every rank (only rank 0 writes), load_checkpoint scatters them back into the slices:
    save after 2 steps + resume for 2 more is bitwise the uninterrupted 4-step run on every rank."""
    world = 3
    ctx = mp.get_context("spawn")
    for mode in ("straight", "save", "resume"):
        port = _free_port()
        procs = [ctx.Process(target=_shard_ckpt_worker, args=(r, world, port, str(tmp_path), mode))
                 for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(180)
            assert p.exitcode == 0, mode
    for r in range(world):
        a = torch.load(tmp_path / f"shard_straight_r{r}.pt", weights_only=True)
        b = torch.load(tmp_path / f"shard_resume_r{r}.pt", weights_only=True)
        for k in a:
            assert torch.equal(a[k], b[k]), (r, k)


def _err_worker(rank, world, port, outdir, inject):
    _env(rank, world, port)
    from gru_mpi_cuda_amd.parallel import dist as gdist
    from gru_mpi_cuda_amd.engine.trainer import CpuTrainer
    ctx = gdist.init(use_gpu=False)
    cfg = GRUConfig(vocab=256, embed=16, hidden=16, layers=1, batch=12, seq=5, lr=1e-2)
    tr = CpuTrainer(cfg, ctx, params=init_params(cfg, seed=1))
    ds = NameStream(cfg.batch, cfg.seq, seed=5)
    per = cfg.batch // world
    for i in range(3):
        x, y = ds.next()
        if inject and i == 1 and rank == world - 1:
            tr.inject_error(1)        # e.g. a persistent kernel's spin limit on the last rank only
        tr.step(x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per])
        if i == 0:
            after1 = tr.state_dict()
    torch.save({"p": tr.state_dict(), "after1": after1, "err": tr.error_word()},
               os.path.join(outdir, f"err{int(inject)}_r{rank}.pt"))
    gdist.shutdown()


def test_error_word_is_global_across_ranks(tmp_path):
    """the step error word rides the last gradient collective as a max over
    ranks, so an error raised on ONE rank skips the update on EVERY rank (the replicas never
    diverge).  gloo twin of the device path (RcclComm::allreduce_avg_f32_err)."""
    world = 3
    ctx = mp.get_context("spawn")
    for inject in (False, True):
        port = _free_port()
        procs = [ctx.Process(target=_err_worker, args=(r, world, port, str(tmp_path), inject)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
            assert p.exitcode == 0
    for r in range(world):
        ok = torch.load(tmp_path / f"err0_r{r}.pt", weights_only=True)
        bad = torch.load(tmp_path / f"err1_r{r}.pt", weights_only=True)
        assert ok["err"] == 0 and bad["err"] == 1
        for k in bad["p"]:
            # the failed step and every later one left the weights at their step-1 values, on every rank
            assert torch.equal(bad["p"][k], bad["after1"][k]), (r, k)
            assert not torch.equal(ok["p"][k], ok["after1"][k]) or k.startswith("bias"), (r, k)
        ref = torch.load(tmp_path / "err1_r0.pt", weights_only=True)
        for k in bad["p"]:
            assert torch.equal(bad["p"][k], ref["p"][k])
