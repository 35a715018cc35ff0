"""Command-line entry point.

    python -m gru_mpi_cuda_amd.cli train    --preset h512 --steps 200 --ckpt out/model.bin
    python -m gru_mpi_cuda_amd.cli generate --ckpt out/model.bin -n 20 --seed 1
    python -m gru_mpi_cuda_amd.cli info
    python -m gru_mpi_cuda_amd.cli bench    [bench.py args]

Multi-GPU: launch with ``python -m torch.distributed.run --nproc-per-node N ...`` (one process
per GPU; RANK / WORLD_SIZE / LOCAL_RANK from the launcher).  The reference's own driver
(main.cpp, missing from the repo) called namegen_initialize / namegen /
namegen_finalize -- ``generate`` does exactly that; the native equivalent without Python is
``gru_mpi_cuda_amd/bin/namegen``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import Optional

import numpy as np


def _add_model_args(ap: argparse.ArgumentParser) -> None:
    for name, typ in (("vocab", int), ("embed", int), ("hidden", int), ("layers", int), ("batch", int),
                      ("seq", int), ("lr", float), ("max_len", int), ("sos", int), ("eos", int),
                      ("clip_norm", float), ("seed", int), ("bucket_mb", float), ("time_chunks", int),
                      ("warmup_steps", int), ("total_steps", int), ("lr_min", float)):
        ap.add_argument("--" + name.replace("_", "-"), dest=name, type=typ, default=None)
    ap.add_argument("--optimizer", choices=["adam", "sgd"], default=None)
    ap.add_argument("--lr-sched", dest="lr_sched", choices=["const", "cosine", "linear"], default=None,
                    help="learning-rate decay after --warmup-steps, down to --lr-min at --total-steps")
    ap.add_argument("--shard-optim", dest="shard_optim", type=int, nargs="?", const=1, default=None, choices=[0, 1, 2],
                    help="data-parallel: sharded optimiser step (reduce-scatter, Adam on 1/world, all-gather of "
                         "the fp32 masters (1) or of the bf16 working copies (2))")
    ap.add_argument("--carry-hidden", dest="carry_hidden", action="store_const", const=True, default=None,
                    help="truncated BPTT: carry each step's final hidden state into the next step")


def _cfg_from(args):
    from .config import preset
    cfg = preset(args.preset)
    over = {k: v for k, v in vars(args).items()
            if k in cfg.__dataclass_fields__ and v is not None}
    return cfg.replace(**over)


def save_checkpoint(tr, path: str, fmt: str = "gen") -> None:
    """Weights (reference or generalised layout) + Adam state + step counter (rank 0 writes)."""
    import torch
    from .utils import ckpt
    # optimiser state first, on EVERY rank: with a sharded optimiser it is a collective (the moment
    # slices other ranks own are all-gathered); only then do the non-writing ranks leave
    if hasattr(tr, "t"):                    # HipTrainer
        (m, v), step = tr.opt_state(), tr.t.get_step()
    else:
        m, v, step = tr.opt_state()
    if getattr(tr, "ctx", None) is not None and not tr.ctx.is_main:
        return
    cfg = tr.cfg
    params = tr.state_dict()
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    ckpt.save(path, cfg, params, fmt=fmt,
              opt_state={"m": m, "v": v, "step": torch.tensor([step], dtype=torch.int64)})


def _read_checkpoint(tr, path: Optional[str]):
    """(params dict, opt-state dict or None).  Data-parallel: only rank 0 opens the file; the
    flat weights, Adam moments and step go to the other ranks by broadcast (SURVEY §5.4 -- the
    reference has every rank read the blob, namegensf.cu:368-372, §2.7 item 4), so ranks > 0
    need neither the file nor a shared filesystem."""
    import torch
    from .models.params import flat_layout, from_flat, to_flat
    from .utils import ckpt
    ctx = getattr(tr, "ctx", None)
    if ctx is None or ctx.world <= 1:
        _, params = ckpt.load(path, tr.cfg)
        return params, ckpt.load_opt_state(path)
    import torch.distributed as dist
    dev = ctx.device if ctx.backend == "nccl" else torch.device("cpu")
    n = flat_layout(tr.cfg).total
    hdr = torch.zeros(2, dtype=torch.int64, device=dev)   # [has optimiser state, step]
    flat = torch.zeros(3 * n, dtype=torch.float32, device=dev)
    if ctx.is_main:
        _, params = ckpt.load(path, tr.cfg)
        st = ckpt.load_opt_state(path)
        flat[:n] = to_flat(tr.cfg, params).to(dev)
        if st is not None:
            flat[n:2 * n] = st["m"].float().to(dev)
            flat[2 * n:] = st["v"].float().to(dev)
            hdr[0], hdr[1] = 1, int(st["step"][0])
    dist.broadcast(hdr, 0)
    dist.broadcast(flat, 0)
    flat, hdr = flat.cpu(), hdr.cpu()
    params = from_flat(tr.cfg, flat[:n])
    st = None
    if int(hdr[0]):
        st = {"m": flat[n:2 * n].clone(), "v": flat[2 * n:].clone(),
              "step": torch.tensor([int(hdr[1])], dtype=torch.int64)}
    return params, st


def load_checkpoint(tr, path: Optional[str]) -> int:
    """Restore weights (+ optimiser state when present) into a trainer; returns the step.
    ``path`` is only read on rank 0 (may be None elsewhere)."""
    params, st = _read_checkpoint(tr, path)
    if hasattr(tr, "t"):
        tr.load_state(params)
        if st is not None:
            tr.load_opt_state(st["m"], st["v"])
            tr.t.set_step(int(st["step"][0]))
    else:
        for k in tr.params:
            tr.params[k].copy_(params[k])
        if st is not None:
            tr.load_opt_state(st["m"], st["v"], int(st["step"][0]))
    return int(st["step"][0]) if st is not None else 0


def cmd_train(args) -> int:
    import torch
    from .parallel import dist as gdist
    from .parallel.rccl import make_comm
    from .engine.trainer import make_trainer
    from .utils.data import make_stream
    from .utils.metrics import MetricsWriter, StepTimer, log
    ctx = gdist.init(use_gpu=torch.cuda.is_available() and not args.cpu, verbose=True)
    cfg = _cfg_from(args)
    if cfg.lr_sched != "const" and cfg.total_steps <= 0:
        if args.resume:
            # the resumed run restores the step counter: a default of --steps would put the whole run
            # past the end of the schedule (at lr_min, warm-up skipped)
            raise SystemExit("--resume with --lr-sched cosine/linear needs --total-steps (the schedule's "
                             "length across restarts)")
        cfg = cfg.replace(total_steps=args.steps)   # decay over this run
    comm = make_comm(ctx) if ctx.device.type == "cuda" else None
    tr = make_trainer(cfg, ctx, comm=comm)
    start = load_checkpoint(tr, args.resume) if args.resume else 0
    if hasattr(tr, "t"):
        log(f"plan: {tr.t.plan()}, workspace {tr.t.workspace_bytes() / 2**20:.1f} MiB")
    data = make_stream(cfg.batch // ctx.world, cfg.seq, cfg.sos, cfg.eos, seed=cfg.seed * 1000 + ctx.rank + start,
                       max_len=cfg.max_len, path=args.data)
    mw = MetricsWriter(args.metrics)
    timer = StepTimer()
    for it in range(start, start + args.steps):
        tr.step(*data.next())
        timer.tick()
        if (it + 1) % args.log_every == 0 or it + 1 == start + args.steps:
            loss = tr.loss()                # synchronises
            r = timer.rate()
            tok_s = r["steps_per_s"] * cfg.batch * cfg.seq
            rec = dict(step=it + 1, loss=loss, tokens_per_s=tok_s, world=ctx.world,
                       ms_per_step=1e3 / r["steps_per_s"] if r["steps_per_s"] else None)
            if ctx.device.type == "cuda":
                free, total = torch.cuda.mem_get_info(ctx.device)
                rec["hbm_used_gb"] = (total - free) / 2 ** 30
                if hasattr(tr, "t"):
                    rec["workspace_mb"] = tr.t.workspace_bytes() / 2 ** 20
                if hasattr(tr, "comm_stats"):
                    cs = tr.comm_stats()
                    rec.update(cs)
                    if cs and rec["ms_per_step"]:
                        # upper bound of the step share the collectives take if none of it overlaps
                        rec["allreduce_step_fraction_max"] = cs["allreduce_ms_standalone"] / rec["ms_per_step"]
                timer.rate()                # the probe above is not training time
            log(f"step {it + 1} loss {loss:.4f} {tok_s / 1e6:.2f} M char-tokens/s")
            mw.write(**rec)
        if args.ckpt and args.save_every and (it + 1) % args.save_every == 0:
            save_checkpoint(tr, args.ckpt, args.fmt)
    if args.ckpt:
        save_checkpoint(tr, args.ckpt, args.fmt)
        log(f"saved {args.ckpt} ({args.fmt})")
    mw.close()
    gdist.shutdown()
    return 0


def cmd_generate(args) -> int:
    from .engine import generator as G
    from .utils.data import random_floats
    from .utils import ckpt
    fmt = args.fmt
    if fmt == "auto":
        fmt = "gen" if os.path.exists(args.ckpt + ".json") else "ref"
    cfg = _cfg_from(args) if fmt == "ref" else None
    N = args.n
    ml = args.max_len if args.max_len is not None else (
        cfg.max_len if fmt == "ref" else ckpt.load(args.ckpt, None, "gen")[0].max_len)
    rf = random_floats(N, ml, seed=args.seed)
    t0 = time.perf_counter()
    G.namegen_initialize(N, args.seed, args.ckpt, cfg, fmt, precision=args.precision)
    out = np.zeros(N * (ml + 1), dtype=np.uint8)
    t1 = time.perf_counter()
    G.namegen(N, rf, out)
    t2 = time.perf_counter()
    rank = int(os.environ.get("RANK", "0"))
    if rank == 0:
        # raw bytes of an untrained model can be control chars: escape them for text output
        names = ["".join(c if c.isprintable() else f"\\x{ord(c):02x}" for c in nm)
                 for nm in G.decode_names(out, N, ml)]
        if args.raw_out:
            out.tofile(args.raw_out)        # the reference's N x (MAX_LEN+1) byte layout
        if args.out:
            with open(args.out, "w") as f:
                f.write("\n".join(names) + "\n")
        else:
            print("\n".join(names))
        print(json.dumps({"names": N, "init_s": round(t1 - t0, 4), "generate_s": round(t2 - t1, 4),
                          "names_per_s": round(N / max(t2 - t1, 1e-9), 1)}), file=sys.stderr)
    G.namegen_finalize()
    return 0


def cmd_info(args) -> int:
    import torch
    info = {"torch": torch.__version__, "hip": torch.version.hip, "gpu": torch.cuda.is_available()}
    if torch.cuda.is_available():
        from .ops import load_ext
        info["device"] = load_ext().device_info()
    print(json.dumps(info, indent=1))
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="gru_mpi_cuda_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    t = sub.add_parser("train", help="train on synthetic names (one process per GPU)")
    t.add_argument("--preset", default="h512")
    t.add_argument("--steps", type=int, default=100)
    t.add_argument("--log-every", type=int, default=10)
    t.add_argument("--ckpt", default=None)
    t.add_argument("--fmt", choices=["gen", "ref"], default="gen")
    t.add_argument("--save-every", type=int, default=0)
    t.add_argument("--resume", default=None)
    t.add_argument("--metrics", default=None, help="JSONL metrics file (rank 0)")
    t.add_argument("--cpu", action="store_true", help="force the CPU reference path")
    t.add_argument("--data", default=None,
                   help="names file, one per line (default: synthetic names); read by the native loader")
    _add_model_args(t)
    g = sub.add_parser("generate", help="namegen_initialize / namegen / namegen_finalize")
    g.add_argument("--ckpt", required=True)
    g.add_argument("--fmt", choices=["auto", "gen", "ref"], default="auto")
    g.add_argument("-n", type=int, default=10)
    g.add_argument("--out", default=None, help="names, one per line (non-printables escaped)")
    g.add_argument("--raw-out", default=None, help="raw N x (MAX_LEN+1) output bytes")
    g.add_argument("--precision", choices=["fp32", "bf16", "bf16x3"], default="fp32",
                   help="fp32 (default): the reference's fp32 arithmetic (fp32 MFMA products); "
                        "bf16x3: fp32 arithmetic on split-bf16 MFMA products (~2^-16 relative error per "
                        "product, ~2x faster; parity with fp32 unpinned on near-tie samples); "
                        "bf16: MFMA fast mode")
    g.add_argument("--preset", default="ref", help="dims for --fmt ref (headerless blob)")
    _add_model_args(g)
    g.set_defaults(seed=0)
    sub.add_parser("info", help="device / build info")
    b = sub.add_parser("bench", help="run bench.py", add_help=False)
    args, rest = ap.parse_known_args(argv)
    if args.cmd == "bench":
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        sys.argv = ["bench.py"] + rest
        return bench.main()
    if rest:
        ap.error(f"unrecognized arguments: {rest}")
    return {"train": cmd_train, "generate": cmd_generate, "info": cmd_info}[args.cmd](args)


if __name__ == "__main__":
    sys.exit(main())
