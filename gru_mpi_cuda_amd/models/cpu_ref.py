"""CPU reference path (BASELINE config #1) and the numerical oracle for the HIP engine.

Math is the reference's forward step (/root/reference/namegensf.cu:664-872,
SURVEY §3.3), in PyTorch gate convention:

    r = σ(W_ir x + b_ir + W_hr h + b_hr)          namegensf.cu:676-695
    z = σ(W_iz x + b_iz + W_hz h + b_hz)          namegensf.cu:702-721
    n = tanh(W_in x + b_in + r ⊙ (W_hn h + b_hn)) namegensf.cu:729-749
    h' = (1 − z) ⊙ n + z ⊙ h = n + z ⊙ (h − n)    namegensf.cu:754-763
    p = softmax(W_fc h_top + b_fc)                namegensf.cu:861-872

with a *correct* (max-subtracted, race-free) softmax -- the reference's K9 kernel
races on its atomic sum (namegensf.cu:294-300).

The training half (loss, BPTT, optimiser) has no reference counterpart;
``manual_backward`` is the exact formula set the HIP backward kernels implement and
is checked against ``torch.autograd`` in tests/test_cpu_ref.py.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..config import GRUConfig

Params = Dict[str, torch.Tensor]


def _gates(gi: torch.Tensor, gh: torch.Tensor, h: torch.Tensor):
    H = h.shape[-1]
    r = torch.sigmoid(gi[..., :H] + gh[..., :H])
    z = torch.sigmoid(gi[..., H:2 * H] + gh[..., H:2 * H])
    ghn = gh[..., 2 * H:]
    n = torch.tanh(gi[..., 2 * H:] + r * ghn)
    hn = n + z * (h - n)
    return hn, (r, z, n, ghn)


def forward(params: Params, cfg: GRUConfig, x: torch.Tensor, h0: Optional[List[torch.Tensor]] = None,
            keep_cache: bool = False):
    """x: [B, T] int ids.  Returns logits [B, T, V] (and per-layer caches if asked)."""
    B, T = x.shape
    H = cfg.hidden
    dt = params["fc.weight"].dtype
    inp = params["embedding"][x.long()]                       # [B, T, E]
    caches = []
    for l in range(cfg.layers):
        W_ih, W_hh = params[f"weight_ih_l{l}"], params[f"weight_hh_l{l}"]
        b_ih, b_hh = params[f"bias_ih_l{l}"], params[f"bias_hh_l{l}"]
        gi_all = inp @ W_ih.T + b_ih                          # hoisted input projection [B,T,3H]
        h = torch.zeros(B, H, dtype=dt) if h0 is None else h0[l]
        hs, rs, zs, ns, ghns, hprev = [], [], [], [], [], []
        for t in range(T):
            gh = h @ W_hh.T + b_hh
            hprev.append(h)
            h, (r, z, n, ghn) = _gates(gi_all[:, t], gh, h)
            hs.append(h); rs.append(r); zs.append(z); ns.append(n); ghns.append(ghn)
        out = torch.stack(hs, 1)                              # [B, T, H]
        if keep_cache:
            caches.append(dict(inp=inp, hprev=torch.stack(hprev, 1), r=torch.stack(rs, 1),
                               z=torch.stack(zs, 1), n=torch.stack(ns, 1), ghn=torch.stack(ghns, 1),
                               out=out))
        inp = out
    logits = inp @ params["fc.weight"].T + params["fc.bias"]
    return (logits, caches) if keep_cache else logits


def xent(logits: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """Mean next-char cross-entropy over valid (label >= 0) positions."""
    valid = y >= 0
    lp = torch.log_softmax(logits, -1)
    nll = -lp.gather(-1, y.clamp_min(0).long().unsqueeze(-1)).squeeze(-1)
    return (nll * valid).sum() / valid.sum().clamp_min(1)


def manual_backward(params: Params, cfg: GRUConfig, x: torch.Tensor, y: torch.Tensor,
                    h0: Optional[List[torch.Tensor]] = None, state_out: Optional[list] = None
                    ) -> Tuple[torch.Tensor, Params]:
    """Explicit BPTT. Returns (loss, grads) with grads keyed like params.

    h0: optional per-layer initial states (truncated BPTT: treated as constants, no gradient
    flows into them).  state_out: if a list, receives the per-layer final states h_{T-1}."""
    logits, caches = forward(params, cfg, x, h0=h0, keep_cache=True)
    if state_out is not None:
        state_out[:] = [c["out"][:, -1].detach().clone() for c in caches]
    B, T, V = logits.shape
    H = cfg.hidden
    valid = (y >= 0)
    cnt = valid.sum().clamp_min(1)
    p = torch.softmax(logits, -1)
    onehot = torch.zeros_like(p).scatter_(-1, y.clamp_min(0).long().unsqueeze(-1), 1.0)
    dlog = (p - onehot) * (valid.unsqueeze(-1).to(p.dtype) / cnt.to(p.dtype))
    loss = xent(logits, y)
    g: Params = {}
    top = caches[-1]["out"]
    g["fc.weight"] = dlog.reshape(-1, V).T @ top.reshape(-1, H)
    g["fc.bias"] = dlog.sum((0, 1))
    dy = dlog @ params["fc.weight"]                           # [B, T, H]
    for l in reversed(range(cfg.layers)):
        c = caches[l]
        W_hh = params[f"weight_hh_l{l}"]
        dgi = torch.zeros(B, T, 3 * H, dtype=dy.dtype)
        dgh = torch.zeros_like(dgi)
        dh_carry = torch.zeros(B, H, dtype=dy.dtype)          # z_{t+1}⊙dh_{t+1} + dGh_{t+1} W_hh
        for t in reversed(range(T)):
            dh = dy[:, t] + dh_carry
            r, z, n, ghn, hp = c["r"][:, t], c["z"][:, t], c["n"][:, t], c["ghn"][:, t], c["hprev"][:, t]
            dn = dh * (1 - z)
            dz = dh * (hp - n)
            dan = dn * (1 - n * n)
            dr = dan * ghn
            dar = dr * r * (1 - r)
            daz = dz * z * (1 - z)
            dgi[:, t] = torch.cat([dar, daz, dan], -1)
            dgh[:, t] = torch.cat([dar, daz, dan * r], -1)
            dh_carry = z * dh + dgh[:, t] @ W_hh
        g[f"weight_hh_l{l}"] = dgh.reshape(-1, 3 * H).T @ c["hprev"].reshape(-1, H)
        g[f"bias_hh_l{l}"] = dgh.sum((0, 1))
        g[f"weight_ih_l{l}"] = dgi.reshape(-1, 3 * H).T @ c["inp"].reshape(-1, c["inp"].shape[-1])
        g[f"bias_ih_l{l}"] = dgi.sum((0, 1))
        dy = dgi @ params[f"weight_ih_l{l}"]                  # grad wrt this layer's input
    demb = torch.zeros_like(params["embedding"])
    demb.index_add_(0, x.reshape(-1).long(), dy.reshape(-1, dy.shape[-1]))
    g["embedding"] = demb
    return loss, g


def autograd_grads(params: Params, cfg: GRUConfig, x: torch.Tensor, y: torch.Tensor,
                   h0: Optional[List[torch.Tensor]] = None):
    ps = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
    h0 = None if h0 is None else [h.detach() for h in h0]
    loss = xent(forward(ps, cfg, x, h0=h0), y)
    loss.backward()
    return loss.detach(), {k: v.grad for k, v in ps.items()}


# --------------------------------------------------------------------------- optimiser
LR_SCHEDS = ("const", "cosine", "linear")


def lr_at(cfg: GRUConfig, t: int) -> float:
    """Learning rate of update t (1-based): linear warm-up over ``warmup_steps``, then constant,
    cosine or linear decay from ``lr`` to ``lr_min`` at ``total_steps`` -- the host twin of the
    device schedule in the Adam kernels (csrc/kernels/misc.hip sched_lr)."""
    if cfg.lr_sched not in LR_SCHEDS:
        raise ValueError(f"lr_sched must be one of {LR_SCHEDS}, got {cfg.lr_sched!r}")
    if cfg.warmup_steps > 0 and t <= cfg.warmup_steps:
        return cfg.lr * t / cfg.warmup_steps
    if cfg.lr_sched == "const" or cfg.total_steps <= cfg.warmup_steps:
        return cfg.lr
    p = min(1.0, (t - cfg.warmup_steps) / (cfg.total_steps - cfg.warmup_steps))
    f = 0.5 * (1.0 + math.cos(math.pi * p)) if cfg.lr_sched == "cosine" else 1.0 - p
    return cfg.lr_min + (cfg.lr - cfg.lr_min) * f


class Adam:
    """Functional Adam/SGD on a dict of fp32 tensors -- same update rule as the HIP
    ``optim`` kernel (bias-corrected Adam, decoupled weight decay, optional global
    norm clipping)."""

    def __init__(self, cfg: GRUConfig, params: Params):
        self.cfg = cfg
        self.step_n = 0
        self.m = {k: torch.zeros_like(v) for k, v in params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in params.items()}

    def step(self, params: Params, grads: Params, advance: bool = True) -> None:
        """advance=False: a further part of the SAME step (the pipelined data-parallel tail updates
        the FC pair in a second launch with the step counter of the first)."""
        c = self.cfg
        scale = 1.0
        if c.clip_norm > 0:
            if not advance:
                raise ValueError("a split optimiser step cannot clip (needs the global norm)")
            norm = torch.sqrt(sum((g.double() ** 2).sum() for g in grads.values())).item()
            scale = min(1.0, c.clip_norm / (norm + 1e-6))
        if advance:
            self.step_n += 1
        lr = lr_at(c, self.step_n)
        if c.optimizer == "sgd":
            for k in params:
                params[k] -= lr * (grads[k] * scale + c.weight_decay * params[k])
            return
        b1, b2 = c.beta1, c.beta2
        bc1 = 1 - b1 ** self.step_n
        bc2 = 1 - b2 ** self.step_n
        for k in params:
            gk = grads[k] * scale
            self.m[k].mul_(b1).add_(gk, alpha=1 - b1)
            self.v[k].mul_(b2).addcmul_(gk, gk, value=1 - b2)
            upd = (self.m[k] / bc1) / (torch.sqrt(self.v[k] / bc2) + c.eps)
            if c.weight_decay:
                upd = upd + c.weight_decay * params[k]
            params[k] -= lr * upd


# --------------------------------------------------------------------------- generation
def sample_inverse_cdf(prob: torch.Tensor, r: torch.Tensor) -> torch.Tensor:
    """The reference's ``random_select`` (namegensf.cu:322-333): first i with an fp32
    running sum ``psum > r`` in index order, else n-1.  prob [N, V], r [N]."""
    # sequential prefix on CPU: fp32 like the reference, or fp64 for the exact-math oracle.  An explicit
    # loop over the vocabulary (vectorised over the names): torch.cumsum does not promise the strictly
    # left-to-right fp32 rounding of the reference's loop (a hypothesis case: 0.25 + 8.2e-9 + 8.2e-9
    # stays 0.25 sequentially but not in cumsum)
    p = prob if prob.dtype == torch.float64 else prob.to(torch.float32)
    cs = torch.empty_like(p)
    acc = torch.zeros_like(p[..., 0])
    for i in range(p.shape[-1]):
        acc = acc + p[..., i]
        cs[..., i] = acc
    hit = cs > r.unsqueeze(-1)
    idx = hit.to(torch.int64).argmax(-1)
    return torch.where(hit.any(-1), idx, torch.full_like(idx, prob.shape[-1] - 1))


def generate(params: Params, cfg: GRUConfig, rfloats: np.ndarray, start: int = 0,
             count: Optional[int] = None) -> np.ndarray:
    """Batched version of the reference's per-name loop (namegensf.cu:649-884).

    Names ``start .. start+count-1`` of the global job; name n at step l consumes
    ``rfloats[n*MAX_LEN + l]`` (SURVEY §3.2 invariant) -- the global index, so the
    result is independent of how names are split across ranks.  Returns uint8
    [count, MAX_LEN+1]; the EOS char *is* written before stopping
    (namegensf.cu:877-882) and the rest stays NUL."""
    ML = cfg.max_len
    N = (rfloats.size // ML - start) if count is None else count
    out = np.zeros((N, ML + 1), dtype=np.uint8)
    if N <= 0:
        return out
    H = cfg.hidden
    dt = params["fc.weight"].dtype
    rf = torch.from_numpy(np.asarray(rfloats, dtype=np.float32)[start * ML:(start + N) * ML]).view(N, ML)
    hs = [torch.zeros(N, H, dtype=dt) for _ in range(cfg.layers)]
    cur = torch.full((N,), cfg.sos, dtype=torch.int64)
    alive = torch.ones(N, dtype=torch.bool)
    for l in range(ML):
        inp = params["embedding"][cur]
        for k in range(cfg.layers):
            gi = inp @ params[f"weight_ih_l{k}"].T + params[f"bias_ih_l{k}"]
            gh = hs[k] @ params[f"weight_hh_l{k}"].T + params[f"bias_hh_l{k}"]
            hs[k], _ = _gates(gi, gh, hs[k])
            inp = hs[k]
        logits = inp @ params["fc.weight"].T + params["fc.bias"]
        prob = torch.softmax(logits if dt == torch.float64 else logits.to(torch.float32), -1)
        sel = sample_inverse_cdf(prob, rf[:, l].to(prob.dtype))
        out[alive.numpy(), l] = sel[alive].numpy().astype(np.uint8)
        alive &= sel != cfg.eos
        cur = sel
        if not alive.any():
            break
    return out
