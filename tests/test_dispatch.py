"""Host-side kernel dispatch checks that need the built extension but no GPU: an unmatched
variant must raise instead of silently launching nothing (gru_seq.hip dispatch)."""
import pytest

from gru_mpi_cuda_amd.ops import ext_available


@pytest.mark.skipif(not ext_available(), reason="native extension not built")
@pytest.mark.parametrize("H,fuse_w,fuse_p", [(1024, True, False), (2048, False, False), (512, False, True)])
def test_bwd_seq_unmatched_variant_raises(H, fuse_w, fuse_p):
    from gru_mpi_cuda_amd.ops import load_ext
    C = load_ext()
    d = dict(H=H, Bp=256, T=8, unchecked=1)
    if fuse_w:
        d["dWhh_part"] = 64        # non-null marks the fused-dW_hh variant; never dereferenced
    if fuse_p:
        d["dP_part"] = 64
        d["V"] = 256
    with pytest.raises(RuntimeError, match="no kernel variant"):
        C.bwd_seq(d, 0)


@pytest.mark.skipif(not ext_available(), reason="native extension not built")
def test_capi_bootstrap_ignores_stale_file(tmp_path, monkeypatch):
    """the C API's file exchange of the ncclUniqueId is job-unique.  A file left by
    another job at the same path is never accepted: rank 1 waits until rank 0 of ITS job
    publishes (here 0.3 s later), and rank 0 replaces the stale file."""
    import threading
    import time
    from gru_mpi_cuda_amd.ops import load_ext
    C = load_ext()
    path = str(tmp_path / "uid.bin")
    monkeypatch.setenv("GK_RUN_ID", "job-A")
    key = C.bootstrap_key()
    assert key == "run:job-A" and C.bootstrap_path(key) != C.bootstrap_path("run:job-B")
    stale = b"S" * 128
    # the other job's complete, well-formed publication
    C.file_exchange_uid(0, path, "run:job-B", stale, 1000)
    fresh = bytes(range(128))
    got = {}
    t = threading.Thread(target=lambda: got.setdefault("r1", C.file_exchange_uid(1, path, key, b"", 5000)))
    t.start()
    time.sleep(0.3)
    assert "r1" not in got          # the stale file was not taken
    assert C.file_exchange_uid(0, path, key, fresh, 1000) == fresh
    t.join(10)
    assert got["r1"] == fresh
    with pytest.raises(RuntimeError, match="timed out"):
        C.file_exchange_uid(1, path, "run:job-C", b"", 200)
