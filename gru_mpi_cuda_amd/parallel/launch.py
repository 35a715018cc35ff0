"""One-process-per-GPU launcher: the ``mpirun -np P`` of this framework.

The reference is started under MPI: ``MPI_Init`` lives in its (missing) ``main.cpp`` and every
rank queries ``MPI_Comm_rank/size`` (/root/reference/namegensf.cu:360-366), with no device
selection (all ranks land on GPU 0).  Here a rank is a plain child process
with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in its environment; the children
bind ``hipSetDevice(LOCAL_RANK)`` themselves (``parallel.dist.init``) and build their RCCL
communicator from the torch.distributed store.

Failure handling: the launcher polls its children, and the first rank that exits
non-zero (or a wall-clock ``--timeout``) ends the job -- the remaining ranks get SIGTERM, then
SIGKILL after ``--grace`` seconds, each addressed by the exact process group this launcher
created -- and the launcher exits with that rank's code.  A rank blocked in a collective whose
peer died therefore does not hang the job.  The launcher itself never touches the GPU, so it can
start ranks without the exec-after-GPU-init hazard.

    python -m gru_mpi_cuda_amd.parallel.launch --nproc 8 -- -m gru_mpi_cuda_amd.cli train --preset h512_dp8
    python -m gru_mpi_cuda_amd.parallel.launch --nproc 2 --log-dir run/logs -- bench.py --gpus 2

Arguments after ``--`` go to ``python`` (a script path or ``-m module``), or with ``--no-python``
form the command itself (``--no-python -- gru_mpi_cuda_amd/bin/namegen model.bin out.txt 1000``).
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence


def free_port(addr: str = "127.0.0.1") -> int:
    s = socket.socket()
    s.bind((addr, 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env(rank: int, world: int, addr: str, port: int, base: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
               LOCAL_WORLD_SIZE=str(world), MASTER_ADDR=addr, MASTER_PORT=str(port))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC for RCCL peer buffers
    env.setdefault("GK_RUN_ID", f"{os.getpid()}-{port}")   # job key of the C API's id exchange
    return env


def _stop(procs: List[subprocess.Popen], grace: float) -> None:
    """SIGTERM every live rank's process group, SIGKILL what is still there after ``grace`` s."""
    live = [p for p in procs if p.poll() is None]
    for p in live:
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
    end = time.monotonic() + grace
    while time.monotonic() < end and any(p.poll() is None for p in live):
        time.sleep(0.05)
    for p in live:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def run(nproc: int, argv: Sequence[str], addr: str = "127.0.0.1", port: Optional[int] = None,
        timeout: float = 0.0, grace: float = 10.0, log_dir: Optional[str] = None,
        poll_s: float = 0.1, python: bool = True) -> int:
    """Start ``nproc`` ranks of ``python argv...`` (``argv...`` itself with python=False, e.g. the
    native bin/namegen driver); return 0 or the first failing rank's code.

    A rank killed by a signal reports 128 + signal number; a ``timeout`` ends the job with 124.
    """
    if nproc < 1:
        raise ValueError("nproc must be >= 1")
    port = port or free_port(addr)
    procs: List[subprocess.Popen] = []
    logs = []
    try:
        for r in range(nproc):
            out = None
            if log_dir:
                os.makedirs(log_dir, exist_ok=True)
                out = open(os.path.join(log_dir, f"rank{r}.log"), "wb")
                logs.append(out)
            procs.append(subprocess.Popen([sys.executable, *argv] if python else list(argv),
                                          env=rank_env(r, nproc, addr, port),
                                          stdout=out, stderr=subprocess.STDOUT if out else None,
                                          start_new_session=True))
        t0 = time.monotonic()
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                print(f"[launch] rank {r} exited with {c}; stopping the other ranks", file=sys.stderr, flush=True)
                _stop(procs, grace)
                return 128 - c if c < 0 else c
            if all(c == 0 for c in codes):
                return 0
            if timeout > 0 and time.monotonic() - t0 > timeout:
                print(f"[launch] job exceeded {timeout:.0f} s; stopping all ranks", file=sys.stderr, flush=True)
                _stop(procs, grace)
                return 124
            time.sleep(poll_s)
    except KeyboardInterrupt:
        _stop(procs, grace)
        return 130
    finally:
        for f in logs:
            f.close()


def main(argv: Optional[Sequence[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if "--" in argv:
        i = argv.index("--")
        own, child = argv[:i], argv[i + 1:]
    else:
        own, child = argv, []
    ap = argparse.ArgumentParser(prog="python -m gru_mpi_cuda_amd.parallel.launch")
    ap.add_argument("--nproc", type=int, default=None,
                    help="ranks to start (default: visible GPUs, 1 without any)")
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=None)
    ap.add_argument("--timeout", type=float, default=0.0, help="wall-clock limit for the job in s (0 = none)")
    ap.add_argument("--grace", type=float, default=10.0, help="SIGTERM -> SIGKILL delay in s")
    ap.add_argument("--log-dir", default=None, help="per-rank logs rank<r>.log instead of the terminal")
    ap.add_argument("--no-python", action="store_true",
                    help="the program after -- is an executable (e.g. gru_mpi_cuda_amd/bin/namegen), not python args")
    a = ap.parse_args(own)
    if not child:
        ap.error("nothing to run: give the program after --")
    n = a.nproc
    if n is None:
        import torch   # device_count() does not initialise the GPU on this image
        n = max(1, torch.cuda.device_count())
    return run(n, child, a.master_addr, a.master_port, a.timeout, a.grace, a.log_dir, python=not a.no_python)


if __name__ == "__main__":
    sys.exit(main())
