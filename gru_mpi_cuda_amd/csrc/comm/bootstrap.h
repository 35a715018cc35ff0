// File-based ncclUniqueId exchange for the native C API, which has no TCP store (the Python
// side ships the id through torch.distributed's store instead: parallel/rccl.py).
//
// The file is job-unique: its name and its payload carry a job key every rank of one job derives
// identically -- GK_RUN_ID (set by parallel/launch.py), else torchrun's TORCHELASTIC_RUN_ID, else an
// MPI / Slurm job id (PMIX_NAMESPACE, OMPI_MCA_ess_base_jobid, SLURM_JOB_ID.SLURM_STEP_ID), else the
// launcher's pid (all ranks of one node are its children) plus MASTER_PORT.  Rank 0
// removes any old file before publishing; the others accept only a file whose payload names
// their key, so a file left by a crashed or concurrent job is never taken for this job's id.
#pragma once
#include <string>

namespace gk {

// This process's place in the job, from whichever launcher started it: torchrun / the in-tree
// launcher (RANK, WORLD_SIZE, LOCAL_RANK), Open MPI's mpirun (OMPI_COMM_WORLD_*), MPICH / Intel MPI
// Hydra (PMI_RANK, PMI_SIZE, MPI_LOCALRANKID) or Slurm's srun (SLURM_PROCID, SLURM_NTASKS,
// SLURM_LOCALID) -- so the C API and its driver run under `mpirun -np P` like the reference
// (namegensf.cu:360-366).  Single process when none is set.
struct LaunchEnv { int rank = 0, world = 1, local = 0; std::string launcher = "none"; };
LaunchEnv launch_env();

std::string bootstrap_key();
std::string bootstrap_path(const std::string& key);   // GK_BOOTSTRAP_FILE overrides
// rank 0 publishes `uid`; every rank returns the id of this job (throws after timeout_ms)
std::string file_exchange_uid(int rank, const std::string& path, const std::string& key, const std::string& uid,
                              int timeout_ms = 120000);

}  // namespace gk
