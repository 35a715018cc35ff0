"""gru_mpi_cuda_amd — MI355X-native GRU name-generation / training engine.

Capabilities of junyongeom/gru-mpi-cuda (reference: /root/reference/namegensf.cu) rebuilt for
CDNA4: the reference's 3-call generation API and checkpoint layout, plus the training half
(softmax-xent, BPTT, Adam, RCCL data parallelism) that the benchmark measures.

Layout:
  config.py        GRUConfig + BASELINE presets
  models/          parameter layout/init, CPU reference path (oracle + BASELINE config #1)
  ops/             loader for the native extension (_C) + thin Python wrappers of the kernels
  engine/          GPU trainer / generator (native executors driven from Python)
  parallel/        torch.distributed bootstrap, RCCL communicator, gradient bucketing, name sharding
  utils/           checkpoint I/O, synthetic data, metrics/logging
  csrc/            HIP kernels (gfx950), C++ runtime/engine, RCCL comm, C API
"""
from .config import GRUConfig, PRESETS, preset  # noqa: F401

__version__ = "0.1.0"
