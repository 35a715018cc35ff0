#!/usr/bin/env python3
"""Generation benchmark: the reference's workload (namegen, /root/reference/namegensf.cu:627-890)
on the reference's own model (preset ``ref``: L=2, H=1024, V=256, E=512 assumed), three ways:

* ``engine``       -- this framework's device-resident batched generator (csrc/engine/generator.cpp:
                      all N names as one batch, fused GRU/FC/softmax/inverse-CDF kernels, one
                      hipGraph per generation, no host round trip per char);
* ``torch``        -- torch eager on the GPU, batched, same semantics (cumsum inverse CDF on device);
* ``ref-schedule`` -- the reference's execution schedule re-enacted with torch eager fp32 ops on the
                      GPU: batch 1 per name, one op per launch, probabilities copied to the host and
                      sampled there every char, the sampled char copied back (namegensf.cu:649-882,
                      BASELINE.md comparator (b)).  It is slow, so it runs --ref-names names and the
                      rate is per generated char.

Metric: generated chars/s (every emitted char incl. the EOS, as namegen writes them).  Random-init
weights (no checkpoints are available offline), uniform randoms from a fixed seed.

    python bench/bench_generate.py [--names 4096] [--preset ref] [--modes engine,torch,ref-schedule]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch


def _emitted(out: np.ndarray) -> int:
    return int((out != 0).sum())


def _gates(gi, gh, h):
    H = h.shape[-1]
    r = torch.sigmoid(gi[:, :H] + gh[:, :H])
    z = torch.sigmoid(gi[:, H:2 * H] + gh[:, H:2 * H])
    n = torch.tanh(gi[:, 2 * H:] + r * gh[:, 2 * H:])
    return n + z * (h - n)


def torch_batched(params, cfg, rf: torch.Tensor) -> torch.Tensor:
    N, ML = rf.shape
    dev = rf.device
    hs = [torch.zeros(N, cfg.hidden, device=dev) for _ in range(cfg.layers)]
    cur = torch.full((N,), cfg.sos, dtype=torch.int64, device=dev)
    alive = torch.ones(N, dtype=torch.bool, device=dev)
    out = torch.zeros(N, ML + 1, dtype=torch.uint8, device=dev)
    for l in range(ML):
        x = params["embedding"][cur]
        for k in range(cfg.layers):
            gi = torch.addmm(params[f"bias_ih_l{k}"], x, params[f"weight_ih_l{k}"].T)
            gh = torch.addmm(params[f"bias_hh_l{k}"], hs[k], params[f"weight_hh_l{k}"].T)
            hs[k] = _gates(gi, gh, hs[k])
            x = hs[k]
        p = torch.softmax(torch.addmm(params["fc.bias"], x, params["fc.weight"].T), -1)
        cs = torch.cumsum(p, -1)
        hit = cs > rf[:, l:l + 1]
        idx = torch.where(hit.any(-1), hit.to(torch.int8).argmax(-1), torch.full_like(cur, cfg.vocab - 1))
        out[:, l] = torch.where(alive, idx, torch.zeros_like(idx)).to(torch.uint8)
        alive = alive & (idx != cfg.eos)
        cur = idx
    return out


def ref_schedule(params, cfg, rf_host: np.ndarray, dev) -> np.ndarray:
    """One name at a time, one small op per launch, host-side sampling every char."""
    N, ML = rf_host.shape
    H = cfg.hidden
    out = np.zeros((N, ML + 1), dtype=np.uint8)
    W = {k: v for k, v in params.items()}
    for n in range(N):
        hs = [torch.zeros(H, device=dev) for _ in range(cfg.layers)]
        c = cfg.sos
        for l in range(ML):
            x = W["embedding"][torch.tensor(c, device=dev)]          # H2D of the char id (cu:668)
            for k in range(cfg.layers):
                Wi, Wh = W[f"weight_ih_l{k}"], W[f"weight_hh_l{k}"]
                bi, bh = W[f"bias_ih_l{k}"], W[f"bias_hh_l{k}"]
                g = []
                for q in range(3):                                  # per-gate matvecs (cu:676-749)
                    gi = torch.mv(Wi[q * H:(q + 1) * H], x) + bi[q * H:(q + 1) * H]
                    gh = torch.mv(Wh[q * H:(q + 1) * H], hs[k]) + bh[q * H:(q + 1) * H]
                    g.append((gi, gh))
                r = torch.sigmoid(g[0][0] + g[0][1])
                z = torch.sigmoid(g[1][0] + g[1][1])
                nn_ = torch.tanh(g[2][0] + r * g[2][1])
                hs[k] = nn_ + z * (hs[k] - nn_)
                x = hs[k]
            p = torch.softmax(torch.mv(W["fc.weight"], x) + W["fc.bias"], 0).cpu().numpy()  # D2H (cu:873)
            ps, sel = np.float32(0), cfg.vocab - 1
            for i in range(cfg.vocab):                               # host random_select (cu:322-333)
                ps = np.float32(ps + p[i])
                if ps > rf_host[n, l]:
                    sel = i
                    break
            out[n, l] = sel
            if sel == cfg.eos:
                break
            c = sel
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="ref")
    ap.add_argument("--names", default="4096", help="comma list: one JSON line per batch size")
    ap.add_argument("--ref-names", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", default="engine,engine_fp32,torch,ref-schedule",
                    help="engine (bf16), engine_fp32 (fp32, persistent kernel at <= 64 names), "
                         "engine_fp32_batched (fp32, per-char graph), engine_bf16x3 (split-bf16 products), "
                         "torch, ref-schedule")
    args = ap.parse_args()
    for n in [int(x) for x in str(args.names).split(",")]:
        args.n = n
        run(args)
    return 0


def run(args) -> None:

    from gru_mpi_cuda_amd.config import preset
    from gru_mpi_cuda_amd.models.params import init_params

    cfg = preset(args.preset)
    dev = torch.device("cuda", 0)
    params = init_params(cfg)
    gparams = {k: v.to(dev) for k, v in params.items()}
    ML = cfg.max_len
    rng = np.random.default_rng(7)
    rf = rng.random((args.n, ML), dtype=np.float32)
    rf_dev = torch.from_numpy(rf).to(dev)
    res = {"preset": args.preset, "model": f"GRU L={cfg.layers} H={cfg.hidden} E={cfg.embed} V={cfg.vocab}",
           "max_len": ML, "names": args.n, "data": "random-init weights, seeded uniforms"}

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            o = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps, o

    modes = args.modes.split(",")
    from gru_mpi_cuda_amd.engine.generator import HipGenerator
    # engine = bf16 MFMA fast mode; engine_fp32 = fp32-faithful mode (the C API default: one
    # persistent launch at <= 64 names); engine_fp32_batched = fp32 with the per-char graph forced
    for key, prec, persist in (("engine", "bf16", True), ("engine_fp32", "fp32", True),
                               ("engine_fp32_batched", "fp32", False), ("engine_bf16x3", "bf16x3", True)):
        if key not in modes:
            continue
        g = HipGenerator(cfg, params, max_batch=args.n, device=dev, precision=prec)
        g.g.set_persist(persist)
        dt, o = timed(lambda: g.generate_device(rf_dev, args.n), args.reps)
        o = o.cpu().numpy()
        res[key] = {"precision": prec, "s": round(dt, 5), "chars_per_s": round(_emitted(o) / dt, 1),
                    "names_per_s": round(args.n / dt, 1), "us_per_char_step": round(dt / ML * 1e6, 2),
                    "persistent": bool(g.g.uses_persist(args.n)), "error_word": int(g.g.read_error())}
        del g
    if "torch" in modes:
        dt, o = timed(lambda: torch_batched(gparams, cfg, rf_dev), args.reps)
        o = o.cpu().numpy()
        res["torch"] = {"s": round(dt, 5), "chars_per_s": round(_emitted(o) / dt, 1),
                        "names_per_s": round(args.n / dt, 1)}
        if "engine" in res:
            res["engine"]["speedup_vs_torch"] = round(res["torch"]["s"] / res["engine"]["s"], 2)
    if "ref-schedule" in modes:
        nr = min(args.ref_names, args.n)
        ref_schedule(gparams, cfg, rf[:1], dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        o = ref_schedule(gparams, cfg, rf[:nr], dev)
        dt = time.perf_counter() - t0
        res["ref_schedule"] = {"names": nr, "s": round(dt, 4), "chars_per_s": round(_emitted(o) / dt, 1)}
        if "engine" in res:
            res["engine"]["speedup_vs_ref_schedule"] = round(
                res["engine"]["chars_per_s"] / res["ref_schedule"]["chars_per_s"], 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    sys.exit(main())
