"""Loads the in-tree native extension ``gru_mpi_cuda_amd/_C``.

torch is imported first so the extension binds to torch's already-loaded HIP runtime
(same soname ``libamdhip64.so.7``).  On a machine with a GPU a missing or broken extension
is an ERROR, never a silent fallback to eager PyTorch: the HIP path is the product.
"""
from __future__ import annotations

import importlib
import os

_EXT = None


def ext_available() -> bool:
    from ..build_ext import ext_path
    return os.path.exists(ext_path())


class StaleExtensionError(ImportError):
    """The built extension does not match the native sources in the tree."""


def check_fresh() -> str:
    """Source hash of the tree if the built extension was built from it; raises StaleExtensionError
    otherwise (missing sidecar = unknown provenance = stale)."""
    from ..build_ext import built_hash, source_hash, hash_path
    want, have = source_hash(), built_hash()
    if want != have:
        raise StaleExtensionError(
            f"native extension is STALE: csrc/ hashes to {want[:16]} but {hash_path()} records "
            f"{(have or 'nothing')[:16]}; rebuild with `python -m gru_mpi_cuda_amd.build_ext` "
            "(GK_EXT_REBUILD=1 rebuilds on load)")
    return want


def load_ext(build_if_missing: bool = True):
    """Import ``_C``.  A missing extension is built when ``build_if_missing``; a stale one (sources
    changed since the build) is rebuilt only where that is safe and asked for -- no GPU visible
    (this build container) or GK_EXT_REBUILD=1 -- and otherwise refused loudly: a GPU run never
    exercises an older binary than the sources it claims to test."""
    global _EXT
    if _EXT is not None:
        return _EXT
    import torch  # noqa: F401  (load torch's libamdhip64 first)
    from ..build_ext import build, ext_path
    if not os.path.exists(ext_path()):
        if not build_if_missing:
            raise ImportError(f"native extension missing at {ext_path()}; run "
                              "`python -m gru_mpi_cuda_amd.build_ext`")
        build()
    try:
        check_fresh()
    except StaleExtensionError:
        rebuild = os.environ.get("GK_EXT_REBUILD")
        if rebuild == "1" or (rebuild != "0" and build_if_missing and not torch.cuda.is_available()):
            build()
            check_fresh()
        else:
            raise
    try:
        _EXT = importlib.import_module("gru_mpi_cuda_amd._C")
    except ImportError as e:
        raise ImportError(f"failed to load native extension {ext_path()}: {e}. "
                          "Rebuild with `python -m gru_mpi_cuda_amd.build_ext --force`") from e
    return _EXT


def ft_layout(t):
    """FT (fragment-tiled) copy of a K-contiguous [R][K] tensor (kernels.h ``ft_offset``):
    every 16x32 MFMA operand fragment becomes 1 KB contiguous in lane order."""
    R, K = t.shape
    assert R % 16 == 0 and K % 32 == 0
    # [R/16][16 rows][K/32][4 k-groups][8] -> [R/16][K/32][4 k-groups][16 rows][8]
    return t.reshape(R // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous().reshape(-1)
