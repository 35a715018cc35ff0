"""Stale-native-binary guard: the extension is only trusted when the source hash
recorded next to it at build time equals the hash of the csrc/ tree being tested."""
import os
import shutil

import pytest

from gru_mpi_cuda_amd import build_ext
from gru_mpi_cuda_amd.ops import _ext


def test_source_hash_tracks_every_native_source(tmp_path, monkeypatch):
    root = tmp_path / "csrc"
    shutil.copytree(build_ext.CSRC, root)
    monkeypatch.setattr(build_ext, "CSRC", str(root))
    h0 = build_ext.source_hash()
    assert h0 == build_ext.source_hash()   # deterministic
    for rel in ("kernels/misc.hip", "kernels/seq_sync.h", "engine/trainer.cpp"):
        p = root / rel
        orig = p.read_bytes()
        p.write_bytes(orig + b"\n// touched\n")
        assert build_ext.source_hash() != h0, rel
        p.write_bytes(orig)
        assert build_ext.source_hash() == h0, rel


def test_load_ext_refuses_a_stale_build(tmp_path, monkeypatch):
    side = tmp_path / "stale.srchash"
    side.write_text("0" * 64 + "\n")
    monkeypatch.setattr(build_ext, "hash_path", lambda: str(side))
    monkeypatch.setattr(build_ext, "ext_path", lambda: str(tmp_path / "present.so"))
    (tmp_path / "present.so").write_bytes(b"")
    monkeypatch.setattr(_ext, "_EXT", None)
    monkeypatch.setenv("GK_EXT_REBUILD", "0")
    called = []
    monkeypatch.setattr(build_ext, "build", lambda *a, **k: called.append(1))
    with pytest.raises(_ext.StaleExtensionError, match="STALE"):
        _ext.load_ext()
    assert not called   # refused, not silently rebuilt
    with pytest.raises(_ext.StaleExtensionError):
        _ext.check_fresh()


def test_load_ext_rebuilds_a_stale_build_when_allowed(tmp_path, monkeypatch):
    side = tmp_path / "stale.srchash"
    side.write_text("missing\n")
    monkeypatch.setattr(build_ext, "hash_path", lambda: str(side))
    monkeypatch.setattr(build_ext, "ext_path", lambda: str(tmp_path / "present.so"))
    (tmp_path / "present.so").write_bytes(b"")
    monkeypatch.setattr(_ext, "_EXT", None)
    monkeypatch.setenv("GK_EXT_REBUILD", "1")
    calls = []

    def fake_build(*a, **k):   # a rebuild writes the tree's hash
        calls.append(1)
        side.write_text(build_ext.source_hash() + "\n")
    monkeypatch.setattr(build_ext, "build", fake_build)
    sentinel = object()
    monkeypatch.setattr(_ext.importlib, "import_module", lambda name: sentinel)
    assert _ext.load_ext() is sentinel
    assert calls == [1]


@pytest.mark.skipif(not _ext.ext_available(), reason="native extension not built")
def test_tree_extension_is_fresh():
    """The in-tree build matches the sources (what the GPU tiers will load)."""
    assert _ext.check_fresh() == build_ext.source_hash()
