"""Launcher-agnostic rank discovery of the native C API (comm/bootstrap.cpp launch_env,
bootstrap_key): torchrun, Open MPI and MPICH mpirun, Slurm srun -- so `mpirun -np P bin/namegen ...`
works like the reference's MPI launch (namegensf.cu:360-366).  CPU only: each case runs in a fresh
interpreter with exactly that launcher's variables."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STRIP = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE",
         "OMPI_COMM_WORLD_LOCAL_RANK", "PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID", "SLURM_PROCID",
         "SLURM_NTASKS", "SLURM_LOCALID", "GK_RUN_ID", "TORCHELASTIC_RUN_ID", "PMIX_NAMESPACE",
         "OMPI_MCA_ess_base_jobid", "SLURM_JOB_ID", "SLURM_STEP_ID", "MASTER_PORT")


def _probe(extra):
    env = {k: v for k, v in os.environ.items() if k not in STRIP}
    env.update(extra)
    code = ("import json; from gru_mpi_cuda_amd.ops import load_ext; C = load_ext(); "
            "print(json.dumps(dict(C.launch_env(), key=C.bootstrap_key())))")
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120, cwd=ROOT)
    if p.returncode:
        return {"error": p.stderr}
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("env,want", [
    ({}, (0, 1, 0, "none")),
    ({"RANK": "3", "WORLD_SIZE": "8", "LOCAL_RANK": "3"}, (3, 8, 3, "torchrun")),
    ({"OMPI_COMM_WORLD_RANK": "5", "OMPI_COMM_WORLD_SIZE": "8", "OMPI_COMM_WORLD_LOCAL_RANK": "1"},
     (5, 8, 1, "openmpi")),
    ({"PMI_RANK": "2", "PMI_SIZE": "4", "MPI_LOCALRANKID": "2"}, (2, 4, 2, "hydra")),
    ({"SLURM_PROCID": "6", "SLURM_NTASKS": "8", "SLURM_LOCALID": "6"}, (6, 8, 6, "slurm")),
    ({"PMI_RANK": "1", "PMI_SIZE": "2"}, (1, 2, 1, "hydra")),   # no local rank: the global one
])
def test_launch_env(env, want):
    r = _probe(env)
    assert (r["rank"], r["world"], r["local"], r["launcher"]) == want, r


def test_launch_env_rejects_inconsistent():
    r = _probe({"OMPI_COMM_WORLD_RANK": "4", "OMPI_COMM_WORLD_SIZE": "4"})
    assert "inconsistent" in r.get("error", ""), r


@pytest.mark.parametrize("env,prefix", [
    ({"PMIX_NAMESPACE": "prterun-host-123@1"}, "pmix:prterun-host-123@1"),
    ({"OMPI_MCA_ess_base_jobid": "4242"}, "ompi:4242"),
    ({"SLURM_JOB_ID": "77", "SLURM_STEP_ID": "3"}, "slurm:77.3"),
    ({"GK_RUN_ID": "abc", "SLURM_JOB_ID": "77"}, "run:abc"),
])
def test_bootstrap_key_per_launcher(env, prefix):
    assert _probe(env)["key"] == prefix
