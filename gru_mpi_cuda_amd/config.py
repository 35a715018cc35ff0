"""Model / run configuration.

The reference hard-codes its model constants as compile-time ``#define``s in a
``namegen.h`` that is not even in the repo (evidence for
HIDDEN_DIM=1024 at /root/reference/namegensf.cu:694,760,789 and NUM_CHAR=256 at
namegensf.cu:862).  Here every one of them is a runtime field, and the five
BASELINE.json configurations are named presets.
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field
from typing import Dict


@dataclass
class GRUConfig:
    # ---- model -----------------------------------------------------------------
    vocab: int = 256            # NUM_CHAR (namegensf.cu:862 "f 256")
    embed: int = 512            # EMBEDDING_DIM (not determinable from the reference)
    hidden: int = 1024          # HIDDEN_DIM (namegensf.cu:694)
    layers: int = 2             # the reference is a 2-layer GRU (namegensf.cu:669-854)
    # ---- generation (reference semantics) --------------------------------------
    max_len: int = 10           # MAX_LEN (unknown in the reference; config field)
    sos: int = 0                # SOS char id (unknown in the reference; config field)
    eos: int = 0                # EOS char id (unknown in the reference; config field)
    # ---- training ----------------------------------------------------------------
    batch: int = 256            # GLOBAL batch (split over ranks)
    seq: int = 32               # BPTT length T
    lr: float = 1e-3
    optimizer: str = "adam"     # "adam" | "sgd"
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-8
    weight_decay: float = 0.0
    clip_norm: float = 0.0      # 0 = off; global-norm gradient clipping otherwise
    # learning-rate schedule (applied on the device from the step counter, so graph replay keeps
    # it): linear warm-up over warmup_steps, then "const", "cosine" or "linear" decay to lr_min at
    # total_steps (models/cpu_ref.lr_at)
    lr_sched: str = "const"
    warmup_steps: int = 0
    total_steps: int = 0
    lr_min: float = 0.0
    dtype: str = "bf16"         # compute dtype of the HIP engine (fp32 master weights)
    seed: int = 1234
    carry_hidden: bool = False  # truncated BPTT over a continuous stream: each step starts from the
                                # previous step's final (detached) hidden state
    keep_grads: bool = False    # after a one-graph step(), leave the step's full gradient in the grad
                                # buffer (grad_dict); off, the fused optimiser sums the split-K /
                                # row-block partials of a tensor in registers and does not write them
                                # back (7 MB fewer bytes per headline step).  forward_backward() always
                                # leaves the gradient.
    # ---- distributed -------------------------------------------------------------
    bucket_mb: float = 8.0      # gradient all-reduce bucket size (MiB of fp32)
    shard_optim: int = 0        # data-parallel ZeRO-1 step: reduce-scatter the gradient, Adam on the
                                # owned 1/world slice, then all-gather (Trainer::set_shard_optim):
                                # 1 (or True) the fp32 masters; 2 the bf16 working copies (half the
                                # bytes; every bf16 layout re-derived locally, fp32 biases exchanged
                                # exactly, other ranks' fp32 master slices gathered only for checkpoints)
    dp_pipeline: int = -1       # one-layer data-parallel step: the bucketed, pipelined tail (two
                                # collectives on a comm stream beside the dW_fc / embedding GEMMs and
                                # a split Adam; Trainer::record_dp_tail_l1).  1 on; 0 and -1 (auto) one
                                # collective after the backward -- the pipelined form measured slower
                                # (graph cross-stream edges, profiles/r5_rccl_self_dp_pipeline1_timeline.txt)
    time_chunks: int = 4        # time-chunked side-stream pipelining inside one step
    overlap: bool = False       # True: chunked side-stream schedule; False: single stream built on
                                # the persistent sequence kernels (faster on MI355X, profiles/)
    watchdog_ms: int = -1       # host watchdog thread per trainer: >0 aborts the RCCL
                                # communicator when a step is not done in time; 0 only watches the
                                # communicator's async errors and the step error word; -1 = auto
                                # (120 s deadline when data-parallel, 0 at one rank); < -1 = off

    def __post_init__(self):
        if self.layers < 1:
            raise ValueError("layers must be >= 1")
        for name in ("vocab", "embed", "hidden", "batch", "seq", "max_len"):
            if getattr(self, name) <= 0:
                raise ValueError(f"{name} must be positive")

    # -- sizes -------------------------------------------------------------------
    def layer_in(self, l: int) -> int:
        return self.embed if l == 0 else self.hidden

    def num_params(self) -> int:
        V, E, H, L = self.vocab, self.embed, self.hidden, self.layers
        n = V * E + V * H + V
        for l in range(L):
            n += 3 * H * self.layer_in(l) + 3 * H * H + 6 * H
        return n

    def to_json(self) -> str:
        return json.dumps(dataclasses.asdict(self), indent=1, sort_keys=True)

    @staticmethod
    def from_dict(d: Dict) -> "GRUConfig":
        names = {f.name for f in dataclasses.fields(GRUConfig)}
        return GRUConfig(**{k: v for k, v in d.items() if k in names})

    def replace(self, **kw) -> "GRUConfig":
        return dataclasses.replace(self, **kw)


# BASELINE.json "configs" (batch is the GLOBAL batch; E = H assumed as in SURVEY §6.2)
PRESETS: Dict[str, GRUConfig] = {
    # 1) plumbing config, CPU reference path, world_size=1
    "cpu_tiny": GRUConfig(vocab=256, embed=64, hidden=64, layers=1, batch=4, seq=16),
    # 2) headline: 1-layer H=512, B=256, T=32 bf16 on 1 GPU (weak-scaled: 256 per GPU)
    "h512": GRUConfig(vocab=256, embed=512, hidden=512, layers=1, batch=256, seq=32),
    # 3) same model, global batch 2048 on 8 GPUs
    "h512_dp8": GRUConfig(vocab=256, embed=512, hidden=512, layers=1, batch=2048, seq=32),
    # 4) 2-layer stacked H=1024, B=1024, T=64 on 8 GPUs
    "h1024_l2": GRUConfig(vocab=256, embed=1024, hidden=1024, layers=2, batch=1024, seq=64),
    # 5) large hidden
    "h2048": GRUConfig(vocab=256, embed=2048, hidden=2048, layers=1, batch=4096, seq=128),
    # the reference's own inference model (namegensf.cu; E assumed 512)
    "ref": GRUConfig(vocab=256, embed=512, hidden=1024, layers=2),
}


def preset(name: str, **overrides) -> GRUConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown preset {name!r}; choose from {sorted(PRESETS)}")
    return PRESETS[name].replace(**overrides)
