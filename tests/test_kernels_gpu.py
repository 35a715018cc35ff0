"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op.

Operands are rounded to bf16 first (the kernels' input precision) so the comparison
isolates the kernel: fp32-accumulated MFMA vs fp32 torch matmul of the same bf16 values.
Asymmetric operands everywhere (an A = I / symmetric-B test would hide a transposed C-write,
cdna_hip_programming.md §3).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def S():
    return torch.cuda.current_stream().cuda_stream


def bf(t):
    return t.to(torch.bfloat16).contiguous()


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(DEV)


@pytest.mark.parametrize("algo", [1, 2, 3])   # 3: one-shot 64x64 small GEMM (K-slice <= 512, or n x 512 chunks)
@pytest.mark.parametrize("M,N,K,splits", [(64, 64, 32, 1), (128, 192, 256, 1), (256, 512, 1024, 4), (192, 128, 512, 2),
                                          (384, 256, 768, 3), (128, 128, 128, 1), (256, 1536, 512, 1),
                                          (256, 512, 8192, 16), (256, 3072, 1024, 1), (128, 256, 3072, 2)])
def test_gemm_nt(ext, algo, M, N, K, splits):
    if algo == 2 and (M % 128 or N % 128 or (K // splits) % 64 or K // splits < 128):
        pytest.skip("shape not supported by the LDS kernel")
    if algo == 3 and (M % 64 or N % 64 or K % splits or K // splits not in (128, 192, 256, 512, 1024, 1536)):
        pytest.skip("shape not supported by the one-shot kernel")
    A, B = bf(rnd(M, K, seed=1)), bf(rnd(N, K, seed=2) + 0.1 * torch.arange(K, device=DEV) / K)
    bias = rnd(N, seed=3) if splits == 1 else None
    C = torch.full((splits, M, N), float("nan"), device=DEV)
    rs = torch.full((splits, M), float("nan"), device=DEV)
    d = dict(A=A.data_ptr(), lda=K, B=B.data_ptr(), ldb=K, C=C.data_ptr(), ldc=N, M=M, N=N, K=K,
             splits=splits, rowsumA=rs.data_ptr(), algo=algo)
    if bias is not None:
        d["bias"] = bias.data_ptr()
    ext.gemm_nt(d, S())
    torch.cuda.synchronize()
    ref = A.float() @ B.float().T + (bias if bias is not None else 0)
    got = C.sum(0)
    torch.testing.assert_close(got, ref, atol=2e-3 * K ** 0.5, rtol=1e-3)
    torch.testing.assert_close(rs.sum(0), A.float().sum(1), atol=1e-2, rtol=1e-3)


@pytest.mark.parametrize("M,N,K,lda_pad,accumulate", [(256, 512, 1024, 0, 0), (6144 // 4, 512, 4096, 64, 0),
                                                      (512, 384, 2048, 0, 1), (1024, 2048, 256, 0, 0)])
def test_gemm_library(ext, M, N, K, lda_pad, accumulate):
    """algo 4: hipBLASLt (bf16 in, fp32 out, TN) + the bf16 row-sum kernel for the bias gradient,
    against fp32 torch; lda_pad exercises a strided A view (the engine's HT + B operand)."""
    lda = K + lda_pad
    A_full = bf(rnd(M, lda, seed=11))
    A = A_full[:, lda_pad:]
    B = bf(rnd(N, K, seed=12))
    C0 = rnd(M, N, seed=13)
    C = C0.clone() if accumulate else torch.full((M, N), float("nan"), device=DEV)
    rs = torch.full((M,), float("nan"), device=DEV)
    ext.gemm_nt(dict(A=A.data_ptr(), lda=lda, B=B.data_ptr(), ldb=K, C=C.data_ptr(), ldc=N, M=M, N=N, K=K,
                     rowsumA=rs.data_ptr(), accumulate=accumulate, algo=4), S())
    torch.cuda.synchronize()
    ref = A.float() @ B.float().T + (C0 if accumulate else 0)
    torch.testing.assert_close(C, ref, atol=2e-3 * K ** 0.5, rtol=1e-3)
    torch.testing.assert_close(rs, A.float().sum(1), atol=1e-3 * K ** 0.5, rtol=1e-4)


@pytest.mark.parametrize("stream", [0, 1])
@pytest.mark.parametrize("N,K,splits,algo", [(192, 512, 1, 1), (384, 1024, 1, 2), (256, 2048, 4, 2)])
def test_gemm_onehot(ext, N, K, splits, algo, stream):
    """algo 2: the one-hot A tile synthesised into the swizzled LDS image of the LDS GEMM (stream = 0)
    or, N % 128 == 0, the streaming one-hot kernel (onehot.hip, GemmVariants.onehot = 1)."""
    V = 256
    ids = torch.randint(0, V, (K,), device=DEV, dtype=torch.int32)
    ids[:64] = 7                                                   # a heavy bucket
    B = bf(rnd(N, K, seed=5))
    C = torch.full((splits, V, N), float("nan"), device=DEV)
    saved = ext.gemm_variants()
    try:
        ext.set_gemm_variants(dict(onehot=stream))
        ext.gemm_nt(dict(onehot_ids=ids.data_ptr(), B=B.data_ptr(), ldb=K, C=C.data_ptr(), ldc=N, M=V, N=N, K=K,
                         splits=splits, algo=algo), S())
        torch.cuda.synchronize()
    finally:
        ext.set_gemm_variants(saved)
    oh = torch.nn.functional.one_hot(ids.long(), V).float()      # [K][V]
    ref = oh.T @ B.float().T
    torch.testing.assert_close(C.sum(0), ref, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("geo", [1, 2, 3])
@pytest.mark.parametrize("K,splits,dist", [(65536, 8, "names"), (16384, 2, "uniform"), (8192, 16, "names"),
                                          (4096, 1, "invalid"), (24576, 4, "one")])
def test_onehot_dp_stream(ext, K, splits, dist, geo):
    """The streaming one-hot kernel at its real shape family (N = 3H, B2 = the n-gate rows, 8192-deep
    K-slices) against the fp32 product: char-like ids (a few 16-row vocabulary tiles active: most
    waves skip most k-tiles), uniform ids (every tile active), ids outside [0, 256) that must match
    nothing, and a single id.  Bitwise equal to the one-hot gemm_lds product per slab: the same MFMA
    chains over the same exact one-hot x bf16 products, in the same k order (skipped tiles add zeros)."""
    V, H = 256, 512
    N = 3 * H
    g = torch.Generator(device="cpu").manual_seed(K + splits)
    if dist == "names":
        ids = torch.randint(97, 123, (K,), generator=g, dtype=torch.int32)
        ids[::17] = 0                                               # end-of-name / padding id
    elif dist == "uniform":
        ids = torch.randint(0, V, (K,), generator=g, dtype=torch.int32)
    elif dist == "invalid":
        ids = torch.randint(-300, 600, (K,), generator=g, dtype=torch.int32)
    else:
        ids = torch.full((K,), 101, dtype=torch.int32)
    ids = ids.to(DEV)
    B = bf(rnd(N, K, seed=7))
    B2 = bf(rnd(N, K, seed=8))
    B2[:2 * H] = float("nan")
    B1 = B.clone()
    B1[2 * H:] = float("nan")
    merged = torch.cat([B[:2 * H], B2[2 * H:]])
    out = []
    saved = ext.gemm_variants()
    try:
        for stream in (geo, 0):   # GemmVariants.onehot: the streaming kernel's tile geometry, 0 = gemm_lds
            ext.set_gemm_variants(dict(onehot=stream))
            C = torch.full((splits, V, N), float("nan"), device=DEV)
            ext.gemm_nt(dict(onehot_ids=ids.data_ptr(), B=B1.data_ptr(), B2=B2.data_ptr(), b2_row=2 * H, ldb=K,
                             C=C.data_ptr(), ldc=N, M=V, N=N, K=K, splits=splits, algo=2), S())
            torch.cuda.synchronize()
            out.append(C)
    finally:
        ext.set_gemm_variants(saved)
    valid = (ids >= 0) & (ids < V)
    oh = torch.nn.functional.one_hot(torch.where(valid, ids, 0).long(), V).float() * valid[:, None].float()
    ref = (oh.T @ merged.float().T)
    torch.testing.assert_close(out[0].sum(0), ref, atol=1e-3, rtol=1e-4)
    assert torch.equal(out[0], out[1])


def _gates_ref(gi, gh, hp):
    H = hp.shape[1]
    r = torch.sigmoid(gi[:, :H] + gh[:, :H])
    z = torch.sigmoid(gi[:, H:2 * H] + gh[:, H:2 * H])
    n = torch.tanh(gi[:, 2 * H:] + r * gh[:, 2 * H:])
    return n + z * (hp - n), r, z, n, gh[:, 2 * H:]


# algo 1 = register-direct 32x16 tile, 2 = LDS-staged 128-row big tile (gru_step_lds.hip)
@pytest.mark.parametrize("mode", ["table", "gi", "fused"])
@pytest.mark.parametrize("H,Bp,algo", [(128, 64, 1), (512, 64, 1), (1024, 128, 1), (1024, 128, 2), (1024, 256, 2),
                                      (512, 256, 2), (256, 128, 2), (1024, 2048, 2), (1024, 4096, 2)])
def test_fwd_step(ext, mode, H, Bp, algo):
    """algo 2, fused, (H/64)*(Bp/256) >= 256 (H=1024, Bp=4096): the 256 x 64 x 3 big-batch tile."""
    V, Kin = 256, 256   # fused mode, algo 2: input phase of 4 k-tiles ahead of the recurrent phase
    hp = rnd(Bp, H, scale=0.5, seed=1).clamp(-1, 1)
    hpb = bf(hp)
    Whh = bf(rnd(3 * H, H, scale=H ** -0.5, seed=2))
    bhh = rnd(3 * H, scale=0.1, seed=3)
    d = dict(hprev_bf=hpb.data_ptr(), hprev_f=hp.data_ptr(), Whh=Whh.data_ptr(), bhh=bhh.data_ptr(), Bp=Bp, H=H,
             algo=algo)
    keep = []
    if mode == "table":
        P = rnd(V, 3 * H, seed=4)
        ids = torch.randint(0, V, (Bp,), device=DEV, dtype=torch.int32)
        d.update(P=P.data_ptr(), ids=ids.data_ptr())
        gi = P[ids.long()]
        keep += [P, ids]
    elif mode == "gi":
        Gi = rnd(Bp, 3 * H, seed=5)
        d.update(Gi=Gi.data_ptr())
        gi = Gi
        keep.append(Gi)
    else:
        x = bf(rnd(Bp, Kin, seed=6))
        Wih = bf(rnd(3 * H, Kin, scale=Kin ** -0.5, seed=7))
        bih = rnd(3 * H, scale=0.1, seed=8)
        d.update(x_bf=x.data_ptr(), Wih=Wih.data_ptr(), bih=bih.data_ptr(), Kin=Kin)
        gi = x.float() @ Wih.float().T + bih
        keep += [x, Wih, bih]
    T = 3
    h_f = torch.empty(Bp, H, device=DEV)
    h_b = torch.empty(Bp, H, device=DEV, dtype=torch.bfloat16)
    hT = torch.zeros(H, (T + 1) * Bp, device=DEV, dtype=torch.bfloat16)
    sv = [torch.empty(Bp, H, device=DEV) for _ in range(4)]
    d.update(h_f=h_f.data_ptr(), h_bf=h_b.data_ptr(), hT=hT.data_ptr(), ldT=(T + 1) * Bp, colT=2 * Bp,
             sr=sv[0].data_ptr(), sz=sv[1].data_ptr(), sn=sv[2].data_ptr(), sghn=sv[3].data_ptr())
    ext.fwd_step(d, S())
    torch.cuda.synchronize()
    gh = hpb.float() @ Whh.float().T + bhh
    h, r, z, n, ghn = _gates_ref(gi, gh, hp)
    tol = dict(atol=2e-3, rtol=2e-3)
    torch.testing.assert_close(h_f, h, **tol)
    torch.testing.assert_close(h_b.float(), h, atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(hT[:, 2 * Bp:3 * Bp].T.float(), h_b.float(), atol=0, rtol=0)
    for got, ref in zip(sv, (r, z, n, ghn)):
        torch.testing.assert_close(got, ref, **tol)


def test_gemm_onehot_split_b(ext):
    """B2: rows >= b2_row of the B operand read from a second buffer (layer 0's dP reads the r/z gate
    rows of dGi^T from dGh^T); equals the one-hot product with the merged operand."""
    V, H, K, splits = 256, 256, 1024, 2
    N = 3 * H
    ids = torch.randint(0, V, (K,), device=DEV, dtype=torch.int32)
    B = bf(rnd(N, K, seed=5))
    B2 = bf(rnd(N, K, seed=6))
    B2[:2 * H] = float("nan")          # rows the kernel must not read from B2
    B1 = B.clone()
    B1[2 * H:] = float("nan")          # rows the kernel must not read from B
    C = torch.zeros(splits, V, N, device=DEV)
    ext.gemm_nt(dict(onehot_ids=ids.data_ptr(), B=B1.data_ptr(), B2=B2.data_ptr(), b2_row=2 * H, ldb=K,
                     C=C.data_ptr(), ldc=N, M=V, N=N, K=K, splits=splits, algo=2), S())
    torch.cuda.synchronize()
    merged = torch.cat([B[:2 * H], B2[2 * H:]]).float()
    ref = torch.nn.functional.one_hot(ids.long(), V).float().T @ merged.T
    torch.testing.assert_close(C.sum(0), ref, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("first", [False, True])
@pytest.mark.parametrize("H,Bp,algo,sk", [(128, 64, 1, 0), (1024, 128, 1, 0), (1024, 128, 2, 0), (1024, 256, 2, 0),
                                          (512, 128, 2, 0), (2048, 512, 2, 0), (2048, 512, 2, 1),
                                          (2048, 1024, 2, 1)])
def test_bwd_step(ext, first, H, Bp, algo, sk, n_only=False):
    """sk = 1: the split-K LDS kernel (128 x 128 tiles, S workgroups per tile meeting through
    fp32 partials and monotonic arrival counters), launched three times on one workspace."""
    T = 4
    t = 1
    dgn = bf(rnd(Bp, 3 * H, scale=0.1, seed=1))
    Whh = rnd(3 * H, H, scale=H ** -0.5, seed=2)
    WhhT = bf(Whh.T)
    carry = rnd(Bp, H, scale=0.1, seed=3)
    dy = rnd(Bp, H, scale=0.1, seed=4)
    r, z, n = torch.sigmoid(rnd(Bp, H, seed=5)), torch.sigmoid(rnd(Bp, H, seed=6)), torch.tanh(rnd(Bp, H, seed=7))
    ghn, hp = rnd(Bp, H, seed=8), torch.tanh(rnd(Bp, H, seed=9))
    cout = torch.empty(Bp, H, device=DEV)
    dgh = torch.empty(Bp, 3 * H, device=DEV, dtype=torch.bfloat16)
    dgi = torch.empty(Bp, 3 * H, device=DEV, dtype=torch.bfloat16)
    dghT = torch.zeros(3 * H, T * Bp, device=DEV, dtype=torch.bfloat16)
    dgiT = torch.zeros(3 * H, T * Bp, device=DEV, dtype=torch.bfloat16)
    d = dict(WhhT=WhhT.data_ptr(), dy=dy.data_ptr(), r=r.data_ptr(), z=z.data_ptr(), n=n.data_ptr(),
             ghn=ghn.data_ptr(), hprev=hp.data_ptr(), carry_out=cout.data_ptr(), dgh=dgh.data_ptr(),
             dghT=dghT.data_ptr(), dgiT=dgiT.data_ptr(), dgi=dgi.data_ptr(), ldT=T * Bp, colT=t * Bp, Bp=Bp, H=H, algo=algo)
    if not first:
        d.update(dgh_next=dgn.data_ptr(), carry_in=carry.data_ptr())
    if n_only:
        d["dgiT_n_only"] = 1
    launches = 1
    if sk:
        S_ = ext.bwd_step_sk_splits(H, Bp)
        assert S_ in (2, 4), S_
        part = torch.empty(H * Bp * S_, device=DEV)
        cnt = torch.zeros((H // 128) * (Bp // 64) * 16, device=DEV, dtype=torch.int32)
        err = torch.zeros(1, device=DEV, dtype=torch.int32)
        d.update(sk_part=part.data_ptr(), sk_part_floats=part.numel(), sk_cnt=cnt.data_ptr(),
                 sk_cnt_words=cnt.numel(), err=err.data_ptr())
        launches = 3
    outs = []
    for _ in range(launches):
        ext.bwd_step(d, S())
        torch.cuda.synchronize()
        outs.append((cout.clone(), dgh.clone()))
    if sk:
        assert int(err.item()) == 0
        if not first:
            assert int(cnt[0].item()) == 3 * S_   # monotonic: every launch adds S per tile
        for c2, g2 in outs[1:]:
            assert torch.equal(c2, outs[0][0]) and torch.equal(g2, outs[0][1])   # deterministic
    dh = dy.clone()
    if not first:
        dh += dgn.float() @ WhhT.float().T + carry
    dn = dh * (1 - z)
    dz = dh * (hp - n)
    dan = dn * (1 - n * n)
    dar = dan * ghn * r * (1 - r)
    daz = dz * z * (1 - z)
    ref_h = torch.cat([dar, daz, dan * r], 1)
    ref_i = torch.cat([dar, daz, dan], 1)
    torch.testing.assert_close(cout, z * dh, atol=1e-4, rtol=1e-3)
    torch.testing.assert_close(dgh.float(), ref_h, atol=2e-3, rtol=1e-2)
    torch.testing.assert_close(dgi.float(), ref_i, atol=2e-3, rtol=1e-2)
    torch.testing.assert_close(dghT[:, t * Bp:(t + 1) * Bp].T, dgh, atol=0, rtol=0)
    if n_only:   # r/z rows untouched (zeros), n rows = dgi's n block
        assert not dgiT[:2 * H].any()
        torch.testing.assert_close(dgiT[2 * H:, t * Bp:(t + 1) * Bp].T, dgi[:, 2 * H:], atol=0, rtol=0)
    else:
        torch.testing.assert_close(dgiT[:, t * Bp:(t + 1) * Bp].T, dgi, atol=0, rtol=0)


@pytest.fixture
def step_variants(ext):
    saved = ext.step_lds_variants()
    yield ext
    ext.set_step_lds_variants(saved)


# large-H step-kernel variants (StepLdsVariants in kernels.h): each against the same fp32 reference
@pytest.mark.parametrize("var", [dict(fwd64=1), dict(fwd64=0)])
@pytest.mark.parametrize("H,Bp", [(1024, 256), (2048, 512)])
@pytest.mark.parametrize("mode", ["table", "gi"])
def test_fwd_step_variants(step_variants, mode, H, Bp, var):
    step_variants.set_step_lds_variants(var)
    test_fwd_step(step_variants, mode, H, Bp, 2)


@pytest.mark.parametrize("H,Bp", [(1024, 256), (1024, 1024), (512, 128)])
def test_fwd_step_fused_64row(step_variants, H, Bp):
    """The 64-row forward tile with the fused input phase (layers >= 1 of batched generation)."""
    step_variants.set_step_lds_variants(dict(fwd64=1))
    test_fwd_step(step_variants, "fused", H, Bp, 2)


@pytest.mark.parametrize("first", [False, True])
def test_bwd_step_sk_variants(step_variants, first):
    test_bwd_step(step_variants, first, 2048, 512, 2, 1)


def test_bwd_step_sk_at_h1024(step_variants):
    step_variants.set_step_lds_variants(dict(bwd_sk_min_h=1024))
    test_bwd_step(step_variants, False, 1024, 1024, 2, 1)


# dgiT_n_only: every backward step kernel family writes only the n-gate rows of dGi^T
@pytest.mark.parametrize("H,Bp,algo,sk", [(128, 64, 1, 0), (1024, 128, 2, 0), (2048, 512, 2, 1)])
def test_bwd_step_dgit_n_only(ext, H, Bp, algo, sk):
    test_bwd_step(ext, False, H, Bp, algo, sk, n_only=True)


@pytest.mark.parametrize("mode", ["plain", "fused_dh", "fused_dh_2s", "dl_v256"])
@pytest.mark.parametrize("H", [256, 320, 512, 1024])
def test_fc_xent(ext, mode, H):
    """fused_dh at H = 512 takes fc_xent_fl (W_fc read once, online softmax over vocabulary chunks,
    dy = scale (sum_v bf16(e_v) W_v / s - W_y)): checked against the fp32 (softmax - onehot) · W_fc;
    fused_dh_2s runs the same call on the 8-wave two-stream kernel (StepLdsVariants fc_flash = 0),
    whose dy is exactly dl(bf16) · W_fc."""
    fused_dh = mode.startswith("fused_dh")
    if mode in ("dl_v256", "fused_dh_2s") and H % 512:
        pytest.skip("the 8-wave kernel is for H in (512, 1024)")
    saved = ext.step_lds_variants()
    ext.set_step_lds_variants(dict(fc_flash=0 if mode == "fused_dh_2s" else 1))
    try:
        _fc_xent_case(ext, mode, H, fused_dh)
    finally:
        ext.set_step_lds_variants(saved)


def _fc_xent_case(ext, mode, H, fused_dh):
    flash = mode == "fused_dh" and H == 512
    M, V = 128, 256
    X = bf(rnd(M, H, seed=1))
    W = bf(rnd(V, H, scale=H ** -0.5, seed=2))
    b = rnd(V, scale=0.5, seed=3)
    y = torch.randint(0, V, (M,), device=DEV, dtype=torch.int32)
    y[::7] = -1
    inv = torch.tensor([1.0 / int((y >= 0).sum())], device=DEV)
    dl = torch.empty(M, V, device=DEV, dtype=torch.bfloat16)
    dlT = torch.zeros(V, 2 * M, device=DEV, dtype=torch.bfloat16)
    lp = torch.empty(M // 32, device=DEV)
    d = dict(X=X.data_ptr(), W=W.data_ptr(), b=b.data_ptr(), labels=y.data_ptr(), inv_count=inv.data_ptr(),
             dl=dl.data_ptr(), dlT=dlT.data_ptr(), loss_part=lp.data_ptr(), M=M, H=H, V=V, ldT=2 * M, colT=M)
    WT = W.T.contiguous()
    dy = torch.full((M, H), float("nan"), device=DEV)
    if fused_dh:   # the training path: no row-major dl; with the FT copies and H % 512 == 0 it
        # takes the 8-wave V = 256 kernel
        from gru_mpi_cuda_amd.ops import ft_layout
        Wf, WTf = ft_layout(W), ft_layout(WT)
        d.update(WT=WT.data_ptr(), dy=dy.data_ptr(), Wf=Wf.data_ptr(), WTf=WTf.data_ptr())
        del d["dl"]
    if mode == "dl_v256":   # persistent-backward path: 8-wave kernel, row-major dl, no dH
        from gru_mpi_cuda_amd.ops import ft_layout
        Wf = ft_layout(W)
        d.update(Wf=Wf.data_ptr())
    ext.fc_xent(d, S())
    torch.cuda.synchronize()
    if fused_dh:
        dl = dlT[:, M:].T.contiguous()
    logits = X.float() @ W.float().T + b
    valid = y >= 0
    loss = torch.nn.functional.cross_entropy(logits[valid], y[valid].long())
    p = torch.softmax(logits, -1)
    oh = torch.nn.functional.one_hot(y.clamp_min(0).long(), V).float()
    ref = (p - oh) * valid[:, None] * inv
    torch.testing.assert_close(lp.sum(), loss, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(dl.float(), ref, atol=1e-4, rtol=1e-2)
    torch.testing.assert_close(dlT[:, M:].T, dl, atol=0, rtol=0)
    if flash:   # dH from bf16 exp(logit - running max) products, normalised at the end
        torch.testing.assert_close(dy, ref @ W.float(), atol=1e-5, rtol=1e-2)
    elif fused_dh:   # dH = dlogits(bf16) · W_fc, fp32 accumulate
        torch.testing.assert_close(dy, dl.float() @ W.float(), atol=1e-5, rtol=1e-3)


@pytest.mark.parametrize("H", [128, 512, 1024])   # 512/1024: 8-wave kernel on the FT copy of W_fc
def test_fc_sample(ext, H):
    from gru_mpi_cuda_amd.models.cpu_ref import sample_inverse_cdf
    from gru_mpi_cuda_amd.ops import ft_layout
    N, Bp, V, ML = 50, 64, 256, 6
    X = bf(rnd(Bp, H, seed=1))
    W = bf(rnd(V, H, scale=3 * H ** -0.5, seed=2))
    b = rnd(V, seed=3)
    rf = torch.rand(N, ML, device=DEV)
    ids = torch.zeros(Bp, device=DEV, dtype=torch.int32)
    alive = torch.ones(Bp, device=DEV, dtype=torch.int32)
    alive[3] = 0
    out = torch.zeros(N, ML + 1, device=DEV, dtype=torch.uint8)
    probs = torch.zeros(Bp, V, device=DEV)
    step = 2
    d = dict(X=X.data_ptr(), W=W.data_ptr(), b=b.data_ptr(), rf=rf.data_ptr(), ids=ids.data_ptr(),
             out=out.data_ptr(), alive=alive.data_ptr(), probs=probs.data_ptr(), N=N, Bp=Bp, H=H, V=V,
             step=step, max_len=ML, eos=0)
    if H >= 512:
        Wf = ft_layout(W)
        d["Wf"] = Wf.data_ptr()
    ext.fc_sample(d, S())
    torch.cuda.synchronize()
    ref_p = torch.softmax(X.float() @ W.float().T + b, -1)
    torch.testing.assert_close(probs, ref_p, atol=1e-5, rtol=1e-4)
    sel = sample_inverse_cdf(probs[:N].double().cpu(), rf[:, step].double().cpu())
    got = ids[:N].long().cpu()
    assert (got == sel).float().mean() >= 0.98
    o = out.cpu()
    assert o[3, step] == 0                       # dead row untouched
    live = [i for i in range(N) if i != 3]
    assert torch.equal(o[live, step].long(), got[live])


@pytest.mark.parametrize("R,C,ft", [(256, 1536, False), (100, 72, False), (64, 128, True), (192, 256, True)])
def test_cast_multi(ext, R, C, ft):
    """fp32 -> bf16 / bf16 transposed (/ FT copies): 16-row tiles without FT outputs, 64-row with."""
    from gru_mpi_cuda_amd.ops import ft_layout
    src = rnd(R, C, seed=R + C)
    dst = torch.empty(R, C, device=DEV, dtype=torch.bfloat16)
    dT = torch.empty(C, R, device=DEV, dtype=torch.bfloat16)
    job = dict(src=src.data_ptr(), R=R, C=C, dst=dst.data_ptr(), dstT=dT.data_ptr())
    if ft:
        dF = torch.empty(R * C, device=DEV, dtype=torch.bfloat16)
        dTF = torch.empty(R * C, device=DEV, dtype=torch.bfloat16)
        job.update(dstF=dF.data_ptr(), dstTF=dTF.data_ptr())
    ext.cast_multi([job, dict(job)], S())   # two jobs: the block prefix sum
    torch.cuda.synchronize()
    ref = src.bfloat16()
    assert torch.equal(dst, ref) and torch.equal(dT, ref.T.contiguous())
    if ft:
        assert torch.equal(dF, ft_layout(ref)) and torch.equal(dTF, ft_layout(ref.T.contiguous()))


@pytest.mark.parametrize("R,C,splits", [(256, 1536, 8), (16, 64, 1), (48, 192, 3)])
def test_reduce_slabs_cast(ext, R, C, splits):
    """Slab sum (slab order 0, 1, 2, ...) -> fp32 + bf16 + bf16 transposed, on 16 x 64 tiles."""
    src = rnd(splits, R, C, seed=splits)
    dst = torch.empty(R, C, device=DEV)
    bf = torch.empty(R, C, device=DEV, dtype=torch.bfloat16)
    bT = torch.empty(C, R, device=DEV, dtype=torch.bfloat16)
    ext.reduce_slabs_cast(dict(src=src.data_ptr(), splits=splits, R=R, C=C, dst=dst.data_ptr(),
                               bf=bf.data_ptr(), bfT=bT.data_ptr()), S())
    torch.cuda.synchronize()
    ref = src[0].clone()
    for k in range(1, splits):
        ref += src[k]
    assert torch.equal(dst, ref)
    assert torch.equal(bf, ref.bfloat16()) and torch.equal(bT, ref.bfloat16().T.contiguous())


@pytest.mark.parametrize("M,N,K,splits,bias,accumulate,lda_pad,rowsum", [
    (256, 256, 64, 1, True, False, 0, False), (512, 768, 1024, 1, True, False, 0, False),
    (768, 512, 2048, 4, False, False, 0, True), (1024, 1024, 3072, 1, False, True, 0, False),
    (512, 256, 4096, 8, False, False, 64, True), (2304, 1280, 576, 1, True, True, 32, False),
    (1536, 512, 8192, 4, False, False, 0, True), (512, 768, 1024, 1, False, False, 0, True),
    (256, 512, 128, 1, False, False, 0, True), (512, 512, 192, 1, True, False, 0, False)])
@pytest.mark.parametrize("mfma", ["16", "16auto", "16legacy", "16sc0", "32"])
def test_gemm256(ext, monkeypatch, M, N, K, splits, bias, accumulate, lda_pad, rowsum, mfma):
    """algo 5: 256 x 256 x 64 LDS-staged MFMA GEMM (gemm256.hip) against fp32 torch on bf16-rounded
    operands -- bias, accumulate, split-K slabs, a strided A view and the fused row sums of A (the
    bias gradient of a weight-gradient product, one partial per split); on v_mfma_f32_16x16x32_bf16
    (the phased pipeline, and the one-vmcnt(0)-per-k-tile kernel with GemmVariants phased = 0) and on
    v_mfma_f32_32x32x16_bf16 (mfma = 32).  K = 64 and odd k-tile counts cover the phased
    pipeline's prologue / drain paths; BM = 192 tiles (M = 768, 1536, 2304) its 3-piece A staging;
    16sc0 the staging schedule of the long-K products (sched = 0, all A pieces in R4)."""
    saved = ext.gemm_variants()
    ext.set_gemm_variants(dict(mfma=int(mfma[:2]), sched=0 if mfma == "16sc0" else -1,
                               phased=-1 if mfma == "16auto" else (0 if mfma == "16legacy" else 1)))
    try:
        _gemm256_case(ext, M, N, K, splits, bias, accumulate, lda_pad, rowsum)
    finally:
        ext.set_gemm_variants(saved)


def _gemm256_case(ext, M, N, K, splits, bias, accumulate, lda_pad, rowsum):
    lda = K + lda_pad
    Af = bf(rnd(M, lda, seed=4))
    A, B = Af[:, :K], bf(rnd(N, K, seed=5) + 0.1 * torch.arange(K, device=DEV) / K)
    bv = rnd(N, seed=6) if bias else None
    C0 = rnd(M, N, seed=7)
    C = torch.full((splits, M, N), float("nan"), device=DEV)
    if accumulate:
        C[0] = C0
    d = dict(A=Af.data_ptr(), lda=lda, B=B.data_ptr(), ldb=K, C=C.data_ptr(), ldc=N, M=M, N=N, K=K,
             splits=splits, algo=5, accumulate=int(accumulate))
    if bv is not None:
        d["bias"] = bv.data_ptr()
    rs = torch.full((splits, M), float("nan"), device=DEV)
    if rowsum:
        d["rowsumA"] = rs.data_ptr()
    ext.gemm_nt(d, S())
    torch.cuda.synchronize()
    ref = A.float() @ B.float().T + (bv if bv is not None else 0) + (C0 if accumulate else 0)
    torch.testing.assert_close(C.sum(0), ref, atol=2e-3 * K ** 0.5, rtol=1e-3)
    if rowsum:
        torch.testing.assert_close(rs.sum(0), A.float().sum(1), atol=1e-2, rtol=1e-3)


@pytest.mark.parametrize("M,N,K,splits", [(4096, 3072, 1024, 1), (2048, 2048, 512, 1), (64, 3072, 1024, 8),
                                          (128, 256, 1024, 4), (256, 256, 512, 1)])
def test_gemm_f32(ext, M, N, K, splits):
    """fp32 generation GEMM (gen_f32.hip: v_mfma_f32_16x16x4_f32, exact fp32 products): the 128 x 128
    kernel (>= 256 tiles, unsplit) and the 64 x 64 split-K kernel against an fp64 torch product;
    split-K slabs summed here, the bias in slab 0 only."""
    A, B, bv = rnd(M, K, seed=4), rnd(N, K, seed=5), rnd(N, seed=6)
    C = torch.full((splits, M, N), float("nan"), device=DEV)
    ext.gemm_f32(dict(A=A.data_ptr(), lda=K, B=B.data_ptr(), ldb=K, C=C.data_ptr(), ldc=N, bias=bv.data_ptr(),
                      M=M, N=N, K=K, splits=splits, slab=M * N), S())
    torch.cuda.synchronize()
    ref = A.double() @ B.double().T + bv.double()
    torch.testing.assert_close(C.double().sum(0), ref, atol=1e-5 * K ** 0.5, rtol=1e-5)


def _gru2_ref(P, ids, Whh0, bhh0, Wih1, bih1, Whh1, bhh1, h00, h01):
    """Two stacked GRU layers in fp32 with the kernels' bf16 rounding of every MFMA operand (h is
    exchanged as bf16; the gate math and the carried state stay fp32)."""
    T, B = ids.shape
    f = lambda t: t.to(torch.bfloat16).float()
    h0, h1 = h00.clone(), h01.clone()
    H0, H1, S1 = [], [], []
    for t in range(T):
        gi = P[ids[t].long()]
        gh = f(h0) @ Whh0.float().t() + bhh0
        gi_r, gi_z, gi_n = torch.chunk(gi, 3, dim=1)
        gh_r, gh_z, gh_n = torch.chunk(gh, 3, dim=1)
        r = torch.sigmoid(gi_r + gh_r); z = torch.sigmoid(gi_z + gh_z); n = torch.tanh(gi_n + r * gh_n)
        h0 = n + z * (h0 - n)
        gi1 = f(h0) @ Wih1.float().t() + bih1
        gh1 = f(h1) @ Whh1.float().t() + bhh1
        gi_r, gi_z, gi_n = torch.chunk(gi1, 3, dim=1)
        gh_r, gh_z, gh_n = torch.chunk(gh1, 3, dim=1)
        r = torch.sigmoid(gi_r + gh_r); z = torch.sigmoid(gi_z + gh_z); n = torch.tanh(gi_n + r * gh_n)
        h1 = n + z * (h1 - n)
        H0.append(h0); H1.append(h1); S1.append(gh_n)
    return torch.stack(H0), torch.stack(H1), torch.stack(S1)


@pytest.mark.parametrize("H,B,T", [(256, 64, 8), (512, 64, 8), (1024, 128, 8), (256, 32, 1), (512, 96, 2)])
@pytest.mark.parametrize("carry", [False, True])
def test_fwd_seq2_two_layer_wavefront(ext, H, B, T, carry):
    """gru_fwd_seq2 (layer 0 at step s, layer 1 at step s-1, layer 1's input projection in-kernel)
    against a torch fp32 two-layer recurrence on the same bf16 operands."""
    if not ext.fwd_seq2_supported(H, B):
        pytest.skip("shape not co-resident")
    V = 256
    g = torch.Generator(device="cpu").manual_seed(3)
    R = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).to(DEV)
    Whh0, Wih1, Whh1 = (bf(R(3 * H, H, sc=H ** -0.5)) for _ in range(3))
    bhh0, bih1, bhh1 = (R(3 * H, sc=0.1) for _ in range(3))
    P = R(V, 3 * H, sc=0.5)
    ids = torch.randint(0, V, (T, B), generator=g, dtype=torch.int32).to(DEV)
    h00 = R(B, H, sc=0.5) if carry else torch.zeros(B, H, device=DEV)
    h01 = R(B, H, sc=0.5) if carry else torch.zeros(B, H, device=DEV)
    err = torch.zeros(16, device=DEV, dtype=torch.int32)
    bufs, dicts = [], []
    for Whh, bhh, h0 in ((Whh0, bhh0, h00), (Whh1, bhh1, h01)):
        b = dict(HSb=torch.zeros(T + 1, B, H, device=DEV, dtype=torch.bfloat16),
                 xch=torch.zeros(T, B, H, device=DEV, dtype=torch.bfloat16),
                 HSf=torch.zeros(T + 1, B, H, device=DEV),
                 HT=torch.zeros(H, (T + 1) * B, device=DEV, dtype=torch.bfloat16),
                 sv=[torch.zeros(T, B, H, device=DEV) for _ in range(4)],
                 cnt=torch.zeros(B // 32 * H // 16 * 16 + 64, device=DEV, dtype=torch.int32), h0=h0.contiguous())
        b["HSb"][0] = h0.to(torch.bfloat16)
        b["HSf"][0] = h0
        d = dict(HSb=b["HSb"].data_ptr(), xch=b["xch"].data_ptr(), HSf=b["HSf"].data_ptr(), HT=b["HT"].data_ptr(),
                 ldT=(T + 1) * B, sr=b["sv"][0].data_ptr(), sz=b["sv"][1].data_ptr(), sn=b["sv"][2].data_ptr(),
                 sghn=b["sv"][3].data_ptr(), Whh=Whh.data_ptr(), bhh=bhh.data_ptr(), cnt=b["cnt"].data_ptr(),
                 err=err.data_ptr(), T=T, Bp=B, H=H)
        if carry:
            d["h0"] = b["h0"].data_ptr()
        bufs.append(b); dicts.append(d)
    dicts[0].update(P=P.data_ptr(), ids=ids.data_ptr())
    ext.fwd_seq2(dicts[0], dicts[1], Wih1.data_ptr(), bih1.data_ptr(), S())
    torch.cuda.synchronize()
    assert int(err[0]) == 0
    H0, H1, GHN1 = _gru2_ref(P, ids, Whh0, bhh0, Wih1, bih1, Whh1, bhh1, h00, h01)
    torch.testing.assert_close(bufs[0]["HSf"][1:], H0, atol=5e-3, rtol=0)
    torch.testing.assert_close(bufs[1]["HSf"][1:], H1, atol=5e-3, rtol=0)
    torch.testing.assert_close(bufs[1]["sv"][3], GHN1, atol=5e-3, rtol=0)
    # bf16 copies: row-major HS and the transposed HT of layer 1 (the weight-gradient operands)
    torch.testing.assert_close(bufs[1]["HSb"][1:].float(), H1, atol=2e-2, rtol=0)
    HT1 = bufs[1]["HT"].view(H, T + 1, B)[:, 1:].permute(1, 2, 0).float()
    torch.testing.assert_close(HT1, H1, atol=2e-2, rtol=0)
