"""Graph replay probe, pass 2: modes 6-9 over sync cadences; kernel-seen vs copied-out stale words
and which replays went wrong."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gru_mpi_cuda_amd.ops import load_ext
C = load_ext()
for words in (64, 4096, 1 << 20):
    for mode in (6, 7, 8, 9):
        for sync in (0, 1, 2, 3, 5):
            r = C.graph_node_probe(words, 40, sync, mode)
            print(json.dumps({"words": words, "mode": mode, "sync_every": sync,
                              "kernel_stale_words": r & 0xFFFFFFFF, "copied_bad_words": r >> 32}), flush=True)
