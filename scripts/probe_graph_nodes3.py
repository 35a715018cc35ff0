"""Graph replay probe, pass 3: the failing case (mode 9: memset-first graph + 71-kernel chain, copy-in
and memset before / copy-out after each replay, NULL stream) -- which kernel of the chain saw a stale
buffer, per sync cadence; mode 10 (mode 9 with a memcpy node), and mode 7 (mode 9 on a created stream) for contrast."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gru_mpi_cuda_amd.ops import load_ext
C = load_ext()
for mode in (9, 10, 7):
    for sync in (0, 1, 2, 3, 4, 5, 8):
        r = C.graph_node_probe(4096, 40, sync, mode)
        d = C.graph_node_probe_detail()
        print(json.dumps({"mode": mode, "sync_every": sync, "kernel_stale_words": r & 0xFFFFFFFF,
                          "copied_bad_words": r >> 32,
                          "stale_buffers_by_kernel": {k: v // 4096 for k, v in enumerate(d) if v}}), flush=True)
