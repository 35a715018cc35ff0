#!/usr/bin/env python3
"""Scaling curve for the headline metric: runs ``bench.py`` at N = 1, 2, 4, 8 GPUs of one node
(one process per GPU via torch.distributed.run, RCCL over xGMI), then prints one JSON line per N
plus a BASELINE.md-style table with weak-scaling efficiency = value(N) / (N * value(1)).

    python bench/bench_scaling.py [--gpus 1,2,4,8] [--steps 50] [--warmup 10] [-- extra bench.py args]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(n: int, steps: int, warmup: int, extra, port: int) -> dict:
    bench = os.path.join(ROOT, "bench.py")
    args = ["--gpus", str(n), "--steps", str(steps), "--warmup", str(warmup)] + list(extra)
    if n == 1:
        cmd = [sys.executable, bench] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), bench] + args
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run(cmd, capture_output=True, text=True, env=env, cwd=ROOT)
    for line in p.stdout.splitlines():
        if line.startswith("{"):
            return json.loads(line)
    raise RuntimeError(f"bench at N={n} failed (rc={p.returncode}):\n{p.stderr[-2000:]}")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--port", type=int, default=29511)
    args, extra = ap.parse_known_args()
    extra = [a for a in extra if a != "--"]
    rows = []
    for i, n in enumerate(int(x) for x in args.gpus.split(",")):
        r = run(n, args.steps, args.warmup, extra, args.port + i)
        print(json.dumps(r), flush=True)
        rows.append(r)
    base = next((r for r in rows if r["n_gpus"] == 1), None)
    print("\n| GPUs | global batch | ms/step | char-tokens/s | weak-scaling eff. |")
    print("|---|---|---|---|---|")
    for r in rows:
        eff = r["value"] / (r["n_gpus"] * base["value"]) if base else float("nan")
        print(f"| {r['n_gpus']} | {r['config']['global_batch']} | {r['ms_per_step']} | "
              f"{r['value']:,.0f} | {eff:.3f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
