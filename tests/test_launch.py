"""The one-process-per-rank launcher (parallel/launch.py) on the CPU / gloo path.

(a) ranks get RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* and can form a gloo group;
(b) one failing rank ends the job with its exit code while its peer is blocked in a collective
    (the MPI job-abort behaviour the reference relied on);
(c) a wall-clock timeout ends a hung job with 124;
(d) the train CLI runs data-parallel under the launcher (gloo, world 2).
"""
import os
import sys
import textwrap
import time

import pytest

from gru_mpi_cuda_amd.parallel import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_WORKER = textwrap.dedent("""
    import os, sys, time
    import torch, torch.distributed as dist
    mode, outdir = sys.argv[1], sys.argv[2]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["LOCAL_RANK"] == str(rank) and os.environ["MASTER_ADDR"] == "127.0.0.1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t)
    open(os.path.join(outdir, f"r{rank}.txt"), "w").write(str(int(t.item())))
    if mode == "fail" and rank == world - 1:
        sys.exit(3)
    if mode == "fail":
        dist.barrier()          # the failed peer never arrives: blocks until the launcher stops us
    if mode == "hang":
        time.sleep(600)
    dist.destroy_process_group()
""")


@pytest.fixture
def worker(tmp_path):
    p = tmp_path / "worker.py"
    p.write_text(_WORKER)
    return str(p)


def test_ranks_form_a_group(tmp_path, worker):
    assert launch.run(3, [worker, "ok", str(tmp_path)], timeout=120) == 0
    got = [int((tmp_path / f"r{r}.txt").read_text()) for r in range(3)]
    assert got == [6, 6, 6]


def test_failing_rank_stops_the_job(tmp_path, worker):
    t0 = time.monotonic()
    rc = launch.run(2, [worker, "fail", str(tmp_path)], timeout=120, grace=2.0)
    assert rc == 3
    assert time.monotonic() - t0 < 60


def test_timeout_ends_hung_job(tmp_path, worker):
    rc = launch.run(2, [worker, "hang", str(tmp_path)], timeout=8, grace=1.0,
                    log_dir=str(tmp_path / "logs"))
    assert rc == 124
    assert sorted(os.listdir(tmp_path / "logs")) == ["rank0.log", "rank1.log"]


def test_cli_train_under_launcher(tmp_path):
    env_py = os.environ.get("PYTHONPATH", "")
    os.environ["PYTHONPATH"] = ROOT + (os.pathsep + env_py if env_py else "")
    try:
        rc = launch.main(["--nproc", "2", "--timeout", "300", "--log-dir", str(tmp_path / "logs"), "--",
                          "-m", "gru_mpi_cuda_amd.cli", "train", "--preset", "cpu_tiny", "--steps", "3",
                          "--metrics", str(tmp_path / "m.jsonl")])
    finally:
        if env_py:
            os.environ["PYTHONPATH"] = env_py
        else:
            os.environ.pop("PYTHONPATH", None)
    logs = "".join((tmp_path / "logs" / f"rank{r}.log").read_text() for r in range(2))
    assert rc == 0, logs
    assert (tmp_path / "m.jsonl").exists()


def test_no_python_runs_an_executable(tmp_path):
    """--no-python starts the command itself once per rank (the native bin/namegen driver's way
    in), each with its own RANK / WORLD_SIZE."""
    import subprocess
    import sys
    out = tmp_path / "ranks"
    out.mkdir()
    cmd = [sys.executable, "-m", "gru_mpi_cuda_amd.parallel.launch", "--nproc", "3", "--no-python", "--",
           "/bin/sh", "-c", f'echo "$WORLD_SIZE $GK_RUN_ID" > {out}/r$RANK']
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    got = sorted(f.read_text().split()[0] for f in out.iterdir())
    assert got == ["3", "3", "3"]
    assert len({f.read_text().split()[1] for f in out.iterdir()}) == 1   # one job key for all ranks
