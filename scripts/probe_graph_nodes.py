"""Graph-node ordering probe: failures per node kind, sizes and sync cadence."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gru_mpi_cuda_amd.ops import load_ext
C = load_ext()
names = {0: "memset", 1: "memcpy", 2: "memcpy2d", 3: "memsetD32", 4: "5 memsets", 5: "odd byte memset",
         6: "memset first + copy-out after each replay",
         7: "memset + 71-kernel chain, copy-in/memset before and copy-out after each replay",
         8: "mode 6 on the NULL stream", 9: "mode 7 on the NULL stream"}
for words in (64, 176, 4096, 1 << 20):
    for mode in range(10):
        for sync in (0, 1):
            bad = C.graph_node_probe(words, 40, sync, mode)
            print(json.dumps({"words": words, "node": names[mode], "sync_every": sync, "bad_words": bad}))
