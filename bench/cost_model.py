#!/usr/bin/env python3
"""World-aware plan for the data-parallel step: which optimiser / collective structure to record at
world size W, from MEASURED 1-GPU costs plus an explicit xGMI collective model.

No 8-GPU node was ever available to this build (every SCALE_rNN.json so far is "skipped"), so the
collective times at W > 1 are modelled, not measured:

    t_AR(S)  = alpha + 2 (W-1)/W * S / B        (ring all-reduce, fp32 gradient of S bytes)
    t_RS(S)  = alpha +   (W-1)/W * S / B        (reduce-scatter)
    t_AG(S)  = alpha +   (W-1)/W * S / B        (all-gather)

B is the effective bus bandwidth of one collective over the 7 xGMI links (153 GB/s per
link; a single ring is per-link bound, RCCL's multi-channel rings reach several links) and alpha the
per-collective latency of a graph-captured RCCL launch; the defaults (B = 300 GB/s, alpha = 10 us)
are assumptions, printed with every prediction together with the B = 153 / 600 GB/s bounds.

Plans (Trainer::record_step_body / record_sharded_opt / record_dp_tail_l1):
  replicated  one in-graph all-reduce of the fp32 gradient after the backward (one-layer models
              cannot overlap it: every gradient is ready only when the persistent backward ends)
  zero1_fp32  reduce-scatter, Adam on 1/W, all-gather of the fp32 masters, bf16 refresh (shard 1)
  zero1_bf16  reduce-scatter, Adam on 1/W, all-gather of the bf16 working copies + exact bias
              exchange, every bf16 layout re-derived locally (shard 2)
  pipelined   two readiness buckets on a comm stream (one-layer models; --dp-pipeline 1)
Each plan's time at W is its measured time on a 1-rank communicator (bench.py --rccl-self, same box)
minus the 1-rank collective nodes and the (W-1)/W part of the optimiser it shards, plus the modelled
collectives at W.  `plan()` picks the cheapest; bench.py --shard-optim -1 and --dp-pipeline -1 use it.

    python bench/cost_model.py [--world 8] [--bus-gbs 300] [--alpha-us 10]
"""
from __future__ import annotations

import argparse
import json

# Measured on one MI355X (round 6, same box, the tree of this commit): step times of each plan on a
# 1-rank RCCL communicator (bench.py --rccl-self --shard-optim M --steps 20 --warmup 5) and the kernel
# times that change with W (rocprofv3 traces profiles/r6_rccl_self_shard{0,1,2}_summary.txt,
# r5_c4_step_summary_final.txt, r6_c5_save16_0_step_summary.txt).  Per config: gradient bytes all-reduced
# per step (Trainer::allreduce_log), parameter count, the fused Adam launch (full model), the 1-rank
# collective node(s), the re-layout pass of plan zero1_bf16 (bf16-source cast of every layout: 12.1 us
# at 1.84 M parameters, scaled by parameter count elsewhere) and the pipelined tail's extra graph
# edges (+46 us at one rank in round 5, profiles/r5_tag_dp_ab.jsonl).
MEASURED = {
    "h512": dict(layers=1, params=1_838_336, grad_mb=5.25, step_ms={"replicated": 0.2317, "zero1_fp32": 0.2515,
                 "zero1_bf16": 0.2539, "pipelined": 0.2524 + (0.2317 - 0.2215)},
                 adam_us=14.1, coll1_us={"replicated": 7.0, "zero1_fp32": 8.6, "zero1_bf16": 9.0, "pipelined": 14.0},
                 hideable_us={"pipelined": 10.6}),
    # config-4 shard (L = 2, H = 1024, 128 sequences / GPU) and config 5 (H = 2048, 512 / GPU): 1-GPU step
    # without a communicator (round-6 final tree, profiles/r6_final_benches.jsonl; Adam from the final
    # traces) + the 1-rank collective node estimated as at h512 per MB
    "h1024_l2": dict(layers=2, params=13_119_744, grad_mb=52.5, step_ms={"replicated": 1.3225},
                     adam_us=75.2, coll1_us={"replicated": 7.0 + 52.5 / 5.25 * 1.0}, hideable_us={}),
    "h2048": dict(layers=1, params=26_226_944, grad_mb=104.9, step_ms={"replicated": 7.92},
                  adam_us=155.6, coll1_us={"replicated": 7.0 + 104.9 / 5.25 * 1.0}, hideable_us={}),
}
RELAYOUT_US_PER_MPARAM = 12.1 / 1.838336     # cast_multi from the bf16 mirror (h512 trace)
REFRESH_US_PER_MPARAM = 12.6 / 1.838336      # cast_multi from the fp32 masters (h512 trace)
PACK_US = 9.8                                # the two bias pack / unpack launches (h512 trace)


def coll_us(kind: str, nbytes: float, world: int, bus_gbs: float, alpha_us: float) -> float:
    if world <= 1:
        return 0.0
    f = (world - 1) / world * (2.0 if kind == "ar" else 1.0)
    return alpha_us + f * nbytes / (bus_gbs * 1e3)   # bytes / (GB/s) -> us with bus_gbs * 1e3 bytes per us


def predict(cfg: str, world: int, bus_gbs: float = 300.0, alpha_us: float = 10.0) -> dict:
    m = MEASURED[cfg]
    S = m["grad_mb"] * 2 ** 20                # the replicated step's all-reduced fp32 gradient
    P = 4.0 * m["params"]                     # the sharded steps reduce-scatter the whole flat gradient
    mp = m["params"] / 1e6
    adam_saved = m["adam_us"] * (1 - 1 / world)
    out = {}
    base = m["step_ms"]["replicated"] * 1e3 - m["coll1_us"]["replicated"]
    out["replicated"] = base + coll_us("ar", S, world, bus_gbs, alpha_us)
    # sharded: measured at one rank where available, else the replicated step + the refresh / re-layout
    for name, gathered, extra in (("zero1_fp32", P, REFRESH_US_PER_MPARAM * mp),
                                  ("zero1_bf16", P / 2, RELAYOUT_US_PER_MPARAM * mp + PACK_US)):
        if name in m["step_ms"]:
            t1 = m["step_ms"][name] * 1e3 - m["coll1_us"][name]
        else:
            t1 = base + extra
        out[name] = (t1 - adam_saved + coll_us("rs", P, world, bus_gbs, alpha_us)
                     + coll_us("ag", gathered, world, bus_gbs, alpha_us))
    if m["layers"] == 1 and "pipelined" in m["step_ms"]:
        # two collectives (the second one's latency added), the first hidden behind the dW_fc K-slices
        t1 = m["step_ms"]["pipelined"] * 1e3 - m["coll1_us"]["pipelined"]
        ar = coll_us("ar", S, world, bus_gbs, alpha_us)
        out["pipelined"] = t1 + max(0.0, ar + alpha_us - m["hideable_us"]["pipelined"])
    return {k: round(v / 1e3, 4) for k, v in out.items()}


def plan(cfg: str, world: int, bus_gbs: float = 300.0, alpha_us: float = 10.0) -> str:
    """The cheapest plan at this world size (1 GPU: replicated -- nothing to shard or overlap)."""
    if world <= 1 or cfg not in MEASURED:
        return "replicated"
    p = predict(cfg, world, bus_gbs, alpha_us)
    return min(p, key=p.get)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--bus-gbs", type=float, default=300.0)
    ap.add_argument("--alpha-us", type=float, default=10.0)
    a = ap.parse_args()
    for cfg in MEASURED:
        row = {"config": cfg, "world": a.world, "bus_gbs": a.bus_gbs, "alpha_us": a.alpha_us,
               "predicted_ms_per_step": predict(cfg, a.world, a.bus_gbs, a.alpha_us),
               "plan": plan(cfg, a.world, a.bus_gbs, a.alpha_us),
               "bounds_ms": {f"B={b:g}": predict(cfg, a.world, b, a.alpha_us) for b in (153.0, 600.0)}}
        print(json.dumps(row))


if __name__ == "__main__":
    main()
