"""In-tree build of the native engine with hipcc for gfx950 only.

No torch.utils.cpp_extension (its ROCm path hipifies sources; this code is written for
CDNA4 directly) and no torch headers: the extension is pybind11 + HIP, linked into
``gru_mpi_cuda_amd/_C.<abi>.so`` next to this file, so it ships with the repo snapshot to
the GPU box.  Also builds ``libnamegen.so`` (the reference's 3-call C API, no Python) and
the ``namegen`` driver executable under ``gru_mpi_cuda_amd/bin``.

    python -m gru_mpi_cuda_amd.build_ext [--force] [--jobs N]
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build", "obj")
ARCH = os.environ.get("GK_OFFLOAD_ARCH", "gfx950")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

KERNELS = ["kernels/gru_step.hip", "kernels/gru_seq.hip", "kernels/fc.hip", "kernels/gemm.hip",
           "kernels/gemm_lds.hip", "kernels/gemm_small.hip", "kernels/gru_step_lds.hip", "kernels/misc.hip",
           "kernels/gen_f32.hip", "kernels/gemm256.hip", "kernels/gen_persist.hip", "kernels/gru_seq_big.hip",
           "kernels/gru_seq16.hip", "kernels/onehot.hip"]
ENGINE = ["runtime/blaslt.cpp", "engine/trainer.cpp", "engine/trainer_seq.cpp", "engine/generator.cpp", "comm/rccl_comm.cpp",
          "comm/watchdog.cpp", "comm/bootstrap.cpp", "data/name_loader.cpp"]
PYBIND = ["bindings.cpp"]
CAPI = ["capi/namegen_api.cpp", "capi/ckpt_reader.cpp"]
DRIVER = ["capi/namegen_main.cpp"]


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(HERE, "_C" + suffix)


def hash_path() -> str:
    """Sidecar written next to the extension by every build: the source hash it was built from."""
    return ext_path() + ".srchash"


def source_hash() -> str:
    """sha256 over every native source under csrc/ (path + bytes, sorted) plus the build target and
    flags.  A built ``_C`` / ``libnamegen.so`` is only trusted when its sidecar carries this value, so a
    test, the smoke check or the bench can never silently run an older build than the tree."""
    import hashlib
    h = hashlib.sha256()
    h.update(("arch=%s;flags=%s" % (ARCH, " ".join(_FLAG_BASE))).encode())
    for root, dirs, files in os.walk(CSRC):
        dirs.sort()
        for f in sorted(files):
            if f.endswith((".h", ".hpp", ".hip", ".cpp", ".cc")):
                path = os.path.join(root, f)
                h.update(os.path.relpath(path, CSRC).encode() + b"\0")
                with open(path, "rb") as fh:
                    h.update(fh.read())
                h.update(b"\0")
    return h.hexdigest()


def built_hash() -> str | None:
    try:
        with open(hash_path()) as fh:
            return fh.read().strip() or None
    except OSError:
        return None


def _headers():
    for root, _, files in os.walk(CSRC):
        for f in files:
            if f.endswith((".h", ".hpp")):
                yield os.path.join(root, f)


_FLAG_BASE = ["-O3", "-fPIC", "-std=c++17", "-Wno-unused-result"]


def _flags(extra=()):
    import pybind11
    return [f"--offload-arch={ARCH}", *_FLAG_BASE,
            f"-I{CSRC}", f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
            "-I/opt/rocm/include", *extra]


def _headers_digest() -> str:
    import hashlib
    h = hashlib.sha256()
    for p in sorted(_headers()):
        h.update(os.path.relpath(p, CSRC).encode() + b"\0")
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _compile(src: str, force: bool, hdr_digest: str) -> str:
    """Compile one source unless its object was built from exactly these bytes: the object's stamp
    file holds sha256(source + every header + flags) -- content, not mtimes, so a checkout, a copy or
    a clock skew can never leave an object older than its source looking current."""
    import hashlib
    out = os.path.join(OBJ, src.replace("/", "_") + ".o")
    path = os.path.join(CSRC, src)
    with open(path, "rb") as fh:
        digest = hashlib.sha256(fh.read() + hdr_digest.encode() + " ".join(_FLAG_BASE + [ARCH]).encode()).hexdigest()
    stamp = out + ".src"
    if not force and os.path.exists(out) and os.path.exists(stamp):
        with open(stamp) as fh:
            if fh.read().strip() == digest:
                return out
    cmd = [HIPCC, *_flags(), "-c", path, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    with open(stamp, "w") as fh:
        fh.write(digest + "\n")
    return out


def _link(objs, out, shared=True, libs=()):
    newest = max(os.path.getmtime(o) for o in objs)
    if os.path.exists(out) and os.path.getmtime(out) >= newest:
        return
    # link to a temporary name, then rename: a reader (a tree snapshot, a running process loading the
    # library) sees the old file or the new one, never a partly written one
    tmp = out + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", *(["-shared"] if shared else []), "-fPIC", *objs, "-o", tmp,
           "-L/opt/rocm/lib", *libs, "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)


HOST_TOOL = ["capi/ckpt_check.cpp", "capi/ckpt_reader.cpp"]


def build_host_tools(force: bool = False) -> list:
    """Host-only tools (g++, no device code): bin/ckpt_check and bin/ckpt_check_asan, the latter
    with AddressSanitizer + UBSan (sanitizers on host code; GPU sanitizers are not
    available on the target pool)."""
    gxx = shutil.which("g++") or "g++"
    srcs = [os.path.join(CSRC, s) for s in HOST_TOOL]
    newest = max(os.path.getmtime(p) for p in srcs + list(_headers()))
    outs = []
    for name, extra in (("ckpt_check", ["-O2"]),
                        ("ckpt_check_asan", ["-O1", "-g", "-fsanitize=address,undefined",
                                             "-fno-omit-frame-pointer", "-fno-sanitize-recover=all"])):
        out = os.path.join(HERE, "bin", name)
        outs.append(out)
        if not force and os.path.exists(out) and os.path.getmtime(out) >= newest:
            continue
        cmd = [gxx, "-std=c++17", *extra, f"-I{CSRC}", *srcs, "-o", out]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"host tool build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return outs


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.join(HERE, "bin"), exist_ok=True)
    # the sidecar must describe the bytes the objects are compiled FROM: hash before compiling, and
    # refuse to stamp a build whose sources changed while it ran (an edit mid-build would otherwise
    # label an old-source binary with the new tree's hash and defeat the stale-binary guard)
    src_hash = source_hash()
    hdr = _headers_digest()
    srcs = KERNELS + ENGINE + PYBIND + [s for s in CAPI + DRIVER if os.path.exists(os.path.join(CSRC, s))]
    jobs = jobs or min(8, os.cpu_count() or 4, 16)
    with ThreadPoolExecutor(jobs) as ex:
        objs = dict(zip(srcs, ex.map(lambda s: _compile(s, force, hdr), srcs)))
    core = [objs[s] for s in KERNELS + ENGINE]
    _link(core + [objs[s] for s in PYBIND], ext_path(), libs=["-lrccl", "-lhipblaslt", "-lrocprofiler-sdk-roctx"])
    capi_objs = [objs[s] for s in CAPI if s in objs]
    if capi_objs:
        lib = os.path.join(HERE, "bin", "libnamegen.so")
        _link(core + capi_objs, lib, libs=["-lrccl", "-lhipblaslt", "-lrocprofiler-sdk-roctx"])
        drv = [objs[s] for s in DRIVER if s in objs]
        if drv:
            _link(drv, os.path.join(HERE, "bin", "namegen"), shared=False,
                  libs=[f"-L{os.path.join(HERE, 'bin')}", "-lnamegen", "-lrccl", "-lhipblaslt", "-lrocprofiler-sdk-roctx",
                        f"-Wl,-rpath,{os.path.join(HERE, 'bin')}", "-Wl,-rpath,$ORIGIN"])
    build_host_tools(force)
    if source_hash() != src_hash:
        raise RuntimeError("build_ext: csrc/ changed while building; run the build again")
    tmp = hash_path() + ".tmp"
    with open(tmp, "w") as fh:
        fh.write(src_hash + "\n")
    os.replace(tmp, hash_path())
    if verbose:
        print(f"[build_ext] {ext_path()} ({len(srcs)} sources, arch {ARCH}, src {built_hash()[:16]})")
    return ext_path()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    a = ap.parse_args()
    build(force=a.force, jobs=a.jobs)


if __name__ == "__main__":
    sys.exit(main())
