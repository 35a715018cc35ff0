"""Per-kernel launch floor: eager vs torch-captured hipGraph, trivial vs GRU step kernel."""
import sys, os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time, torch, json
from gru_mpi_cuda_amd.ops import load_ext
C = load_ext()
dev = torch.device("cuda", 0)
s = lambda: torch.cuda.current_stream().cuda_stream
src = torch.zeros(1024, device=dev); dst = torch.zeros(256, device=dev)
def tiny(): C.reduce_slabs(src.data_ptr(), 4, 256, dst.data_ptr(), s())
H, Bp = 512, 256
hb = torch.zeros(Bp, H, device=dev, dtype=torch.bfloat16); hf = torch.zeros(Bp, H, device=dev)
W = torch.randn(3 * H, H, device=dev).bfloat16(); b = torch.zeros(3 * H, device=dev)
Gi = torch.zeros(Bp, 3 * H, device=dev); of = torch.zeros(Bp, H, device=dev); ob = torch.zeros_like(hb)
d = dict(hprev_bf=hb.data_ptr(), hprev_f=hf.data_ptr(), Whh=W.data_ptr(), bhh=b.data_ptr(), Gi=Gi.data_ptr(),
         h_f=of.data_ptr(), h_bf=ob.data_ptr(), Bp=Bp, H=H)
def step(): C.fwd_step(d, s())
res = {}
for name, fn in (("tiny", tiny), ("fwd_step", step)):
    for _ in range(50): fn()
    torch.cuda.synchronize()
    n = 2000
    t = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize()
    res[name + "_eager_us"] = (time.perf_counter() - t) / n * 1e6
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(200): fn()
    g.replay(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10): g.replay()
    torch.cuda.synchronize()
    res[name + "_graph_us"] = (time.perf_counter() - t) / 2000 * 1e6
print(json.dumps({k: round(v, 2) for k, v in res.items()}))
