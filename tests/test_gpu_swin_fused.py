"""Fused Swin stage (irads/swin_fused.py, csrc/swinblock.hip) on the GPU.

The fused stage must reproduce the module-by-module autocast path (itself checked against
the reference in test_gpu_swin.py), which is the reference's own arithmetic under bf16 AMP.
Kernel-level checks compare each row/element kernel with the torch ops it replaces, in
the rounding the autocast reference applies.  Tolerances: bit-exact where the arithmetic
is the same formula (GELU, ReLU, dropout scaling, casts, DropPath); LayerNorm differs from
torch's Welford reduction in summation order only (1 bf16 ulp on a few elements); the
whole stage at bf16 GEMM scale (relative L2 1e-2, stated per test)."""
import pytest
import torch
import torch.nn.functional as F

from fill import fill_module

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _N():
    from irads import native as N
    return N


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("C", [128, 192, 512, 1024])
def test_resln_fwd_matches_torch(C):
    from irads import swin_fused as SF
    torch.manual_seed(C)
    S, L = 4, 37
    M = S * L
    x = torch.randn(M, C, device=DEV)
    o = torch.randn(M, C, device=DEV).bfloat16()
    f = torch.randn(M, C, device=DEV).bfloat16()
    d = torch.randn(M, C, device=DEV).bfloat16()
    norm = torch.nn.LayerNorm(C).to(DEV)
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
        norm.bias.uniform_(-0.2, 0.2)
    s = torch.tensor([0.0, 1.0 / 0.7, 1.0, 1.0 / 0.7], device=DEV)  # per-sample DropPath factors
    # X1 = x + DP(o); LN; bf16 copy
    X1, h, xb, mean, rstd = SF._resln_fwd(x, M, C, L, add1=o, add1_scale=s, norm=norm, x_out=True, xb_out=True)
    dp = (o.view(S, L, C) * s.view(S, 1, 1)).bfloat16().float().view(M, C)  # bf16(v * s); s = 0 drops
    ref = x + dp
    assert torch.equal(X1, ref)
    assert torch.equal(xb, ref.bfloat16())
    href = F.layer_norm(ref, (C,), norm.weight, norm.bias, 1e-5)
    err = (h.float() - href).abs() / href.abs().clamp_min(1e-2)
    assert err.max().item() < 2 ** -7, err.max().item()
    torch.testing.assert_close(mean, ref.mean(-1), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rstd, torch.rsqrt(ref.var(-1, unbiased=False) + 1e-5), rtol=1e-4, atol=1e-6)
    # Xout = (X1 + f) + bf16(0.5 d), no LN
    xo, _, _, _, _ = SF._resln_fwd(X1, M, C, L, add1=f, add2=d, add2_mult=0.5, x_out=True)
    assert torch.equal(xo, (X1 + f.float()) + (0.5 * d.float()).bfloat16().float())


@pytest.mark.parametrize("C", [128, 384, 1024])
def test_resln_bwd_matches_autograd(C):
    from irads import swin_fused as SF
    torch.manual_seed(C + 1)
    S, L = 2, 50
    M = S * L
    x = torch.randn(M, C, device=DEV, requires_grad=True)
    norm = torch.nn.LayerNorm(C).to(DEV)
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
    _, _, _, mean, rstd = SF._resln_fwd(x.detach(), M, C, L, norm=norm)
    dy = torch.randn(M, C, device=DEV).bfloat16()
    gres = torch.randn(M, C, device=DEV)
    gadd = torch.randn(M, C, device=DEV).bfloat16()
    s = torch.tensor([1.0 / 0.8, 0.0], device=DEV)
    dx, b1, b2 = SF._resln_bwd(M, C, L, dy=dy, x=x.detach(), mean=mean, rstd=rstd, norm=norm, g_res=gres,
                               g_add=gadd, b1=True, b1_scale=s, b2=True, b2_mult=0.5)
    y = F.layer_norm(x, (C,), norm.weight, norm.bias, 1e-5)
    (gx,) = torch.autograd.grad(y, x, dy.float())
    ref = gx + gres + gadd.float()
    torch.testing.assert_close(dx, ref, rtol=1e-4, atol=1e-4)
    gb = dx.bfloat16().float()
    assert torch.equal(b1.float(), (gb.view(S, L, C) * s.view(S, 1, 1)).bfloat16().float().view(M, C))
    assert torch.equal(b2.float(), (0.5 * gb).bfloat16().float())


def test_gelu_and_relu_dropout_kernels():
    N = _N()
    torch.manual_seed(3)
    n = 8 * 1000 + 5  # ragged tail
    u = (torch.randn(n, device=DEV) * 3).bfloat16()
    g = torch.empty_like(u)
    N.call("irads_gelu_fwd", N.ptr(u), N.ptr(g), n, N.stream())
    ref = F.gelu(u)  # torch bf16 GELU: fp32 erf, rounded
    assert (g.float() - ref.float()).abs().max().item() <= 2 ** -8 * ref.float().abs().max().item()
    assert (g != ref).float().mean().item() < 0.01
    dg = torch.randn(n, device=DEV).bfloat16()
    du = torch.empty_like(u)
    N.call("irads_gelu_bwd", N.ptr(u), N.ptr(dg), N.ptr(du), n, N.stream())
    uu = u.float().requires_grad_()
    (ref,) = torch.autograd.grad(F.gelu(uu), uu, dg.float())
    torch.testing.assert_close(du.float(), ref.bfloat16().float(), rtol=2 ** -7, atol=1e-3)
    # ReLU (p = 0) and ReLU + dropout(0.1)
    r = torch.empty_like(u)
    N.call("irads_relu_dropout_fwd", N.ptr(u), N.ptr(r), n, 0.0, 1234, None, N.stream())
    assert torch.equal(r, F.relu(u))
    N.call("irads_relu_dropout_fwd", N.ptr(u), N.ptr(r), n, 0.1, 1234, None, N.stream())
    pos = u.float() > 0
    kept = pos & (r.float() != 0)
    frac = kept.sum().item() / pos.sum().item()
    assert 0.87 < frac < 0.93, frac
    scale = torch.tensor(1.0 / (1.0 - 0.1), dtype=torch.float32)
    assert torch.equal(r[kept].float(), (u[kept].float() * scale.item()).bfloat16().float())
    assert torch.all(r[~kept] == 0)
    r2 = torch.empty_like(u)
    N.call("irads_relu_dropout_fwd", N.ptr(u), N.ptr(r2), n, 0.1, 1234, None, N.stream())
    assert torch.equal(r, r2)  # counter-based: same seed, same mask
    sd = torch.tensor([1234 ^ 77], device=DEV, dtype=torch.int64)  # device seed: salt ^ *seed_dev
    N.call("irads_relu_dropout_fwd", N.ptr(u), N.ptr(r2), n, 0.1, 77, N.ptr(sd), N.stream())
    assert torch.equal(r, r2)
    da = torch.empty_like(u)
    N.call("irads_relu_dropout_bwd", N.ptr(r), N.ptr(dg), N.ptr(da), n, 0.1, N.stream())
    ref = torch.where(kept, (dg.float() * scale.item()), torch.zeros_like(dg.float())).bfloat16()
    assert torch.equal(da, ref)


def _stage(C=128, heads=4, depth=2, dpr=0.0, seed=5):
    from semseg.models.backbones import swin
    seq = swin.SwinBlockSequence(C, heads, 4 * C, depth, 12, drop_path_rate=dpr).to(DEV)
    fill_module(seq, seed=seed)
    for n, p in seq.named_parameters():
        p.requires_grad_("Adapter" in n)
    return seq


def _run(seq, x, hw, fused, g):
    seq.fused = fused
    xx = x.clone().requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = seq.forward_pair(xx, hw, x.shape[0] // 2)[2]
    params = [p for n, p in seq.named_parameters() if p.requires_grad]
    grads = torch.autograd.grad((y.float() * g).sum(), [xx] + params)
    return y.float(), grads


@pytest.mark.parametrize("C,heads,H,W", [(128, 4, 28, 28), (256, 8, 24, 20), (512, 16, 16, 16)])
def test_fused_stage_matches_module_path(C, heads, H, W):
    """Eval mode (no randomness): the fused stage against the op-by-op autocast path.
    Tolerance: relative L2 5e-3 on the output; on the gradients 2e-2 over all of them and 5e-2
    per tensor (bf16 operand rounding of the GEMMs; the only differences are LayerNorm
    summation order flipping a bf16 rounding here and there — and, through that, now and then
    an Adapter ReLU whose input sits at zero, which moves one entry of an 8-wide D_fc1 bias
    gradient by a few percent)."""
    from irads import swin_fused as SF
    torch.manual_seed(0)
    seq = _stage(C, heads)
    seq.eval()
    x = torch.randn(4, H * W, C, device=DEV)
    assert SF.usable(seq, x) is False  # autocast is off here
    g = torch.randn(4, H * W, C, device=DEV)
    y0, g0 = _run(seq, x, (H, W), False, g)
    calls = {"n": 0}
    orig = SF.SwinStageFn.forward

    def spy(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)
    SF.SwinStageFn.forward = staticmethod(spy)
    try:
        y1, g1 = _run(seq, x, (H, W), True, g)
    finally:
        SF.SwinStageFn.forward = staticmethod(orig)
    assert calls["n"] == 1, "fused stage was not taken"
    assert _rel(y1, y0) < 5e-3, _rel(y1, y0)
    for a, b in zip(g1, g0):
        assert _rel(a, b) < 5e-2, _rel(a, b)
    flat1 = torch.cat([a.flatten() for a in g1[1:]])
    flat0 = torch.cat([b.flatten() for b in g0[1:]])
    assert _rel(flat1, flat0) < 2e-2, _rel(flat1, flat0)


def test_fused_stage_training_deterministic_parts():
    """Training mode with DropPath and adapter dropout switched off equals eval mode;
    with them on, the output stays finite, the dropout mask differs per call and the
    gradient matches a finite-difference check along the input direction."""
    from irads import swin_fused as SF
    torch.manual_seed(1)
    seq = _stage(128, 4, dpr=0.0)
    x = torch.randn(4, 24 * 24, 128, device=DEV)
    g = torch.randn_like(x)
    seq.eval()
    ye, ge = _run(seq, x, (24, 24), True, g)
    seq.train()
    old = SF.ADAPTER_DROPOUT
    SF.ADAPTER_DROPOUT = 0.0
    try:
        yt, gt = _run(seq, x, (24, 24), True, g)
    finally:
        SF.ADAPTER_DROPOUT = old
    assert torch.equal(ye, yt)
    for a, b in zip(ge, gt):
        assert torch.equal(a, b)
    y1, _ = _run(seq, x, (24, 24), True, g)
    y2, _ = _run(seq, x, (24, 24), True, g)
    assert torch.isfinite(y1).all() and not torch.equal(y1, y2)


def test_fused_stage_droppath_semantics():
    """DropPath (drop_path_rate 0.3 over 2 blocks): per-sample factors are either 0 or
    1/keep, and a dropped sample's branch contributes nothing: with every branch dropped
    the stage output equals its input plus the adapter terms only."""
    from irads import swin_fused as SF
    seq = _stage(128, 4, depth=2, dpr=[0.2, 0.3])
    seq.train()
    s = SF._droppath_scales(seq, 64, torch.device(DEV))
    assert s.shape == (2, 2, 64)
    keep = torch.tensor([[0.8, 0.8], [0.7, 0.7]], device=DEV)[..., None]
    inv = (1.0 / keep.float())
    ok = (s == 0) | (s == inv)
    assert ok.all()
    frac = (s != 0).float().mean(-1)
    assert ((frac - keep[..., 0]).abs() < 0.25).all()
    # one launch per stage (irads_droppath_scales): keep + U, U on the 2^-8 grid, rounded to bf16 ->
    # P(kept) = P(bf16(keep + U) >= 1), counted over the 256 values of U; fresh factors per seed
    big = torch.stack([SF._droppath_scales(seq, 8192, torch.device(DEV)) for _ in range(4)])
    for k, (kp, slot) in enumerate([(0.8, 0), (0.7, 1)]):
        u = torch.arange(256, dtype=torch.float64) / 256
        p_keep = ((u + kp).float().bfloat16().float().floor() >= 1).double().mean().item()
        got = (big[:, slot] != 0).double().mean().item()
        assert abs(got - p_keep) < 0.01, (kp, got, p_keep)
    assert not torch.equal(big[0], big[1])
    seq.blocks[0].attn.drop.p = 0.0  # a branch without DropPath: factor 1
    s1 = SF._droppath_scales(seq, 64, torch.device(DEV))
    assert torch.equal(s1[0, 0], torch.ones(64, device=DEV))


@pytest.mark.parametrize("K,m,n", [(131072, 8, 128), (8192, 512, 32), (1000, 16, 24), (300, 64, 256), (77, 128, 136),
                                   (4096, 1024, 64), (2048, 256, 512)])
def test_wgrad_split_k(K, m, n):
    """irads_wgrad against fp32 torch on the same bf16 operands: the products are exact in
    fp32 and only the summation order differs (relative error ~1e-6)."""
    from irads import ops
    torch.manual_seed(K + m + n)
    Aw = torch.randn(K, m + 8, device=DEV).bfloat16()
    A = Aw[:, 8:]  # row stride m + 8: a column slice, as the fused stage passes
    B = torch.randn(K, n, device=DEV).bfloat16()
    D = torch.empty(m, n, device=DEV)
    ca, cb = torch.empty(m, device=DEV), torch.zeros(n, device=DEV)
    ops.wgrad(A, B, D, colsum_a=ca)
    ref = A.float().t() @ B.float()
    assert _rel(D, ref) < 1e-5, _rel(D, ref)
    torch.testing.assert_close(ca, A.float().sum(0), rtol=1e-4, atol=1e-3)
    # accumulate + alpha + the other operand's column sums
    D2 = D.clone()
    ops.wgrad(A, B, D2, colsum_b=cb, alpha=0.5, accumulate=True)
    assert _rel(D2, 1.5 * ref) < 1e-5
    torch.testing.assert_close(cb, 0.5 * B.float().sum(0), rtol=1e-4, atol=1e-3)
    # deterministic: fixed-order reduction
    D3 = torch.empty_like(D)
    ops.wgrad(A, B, D3)
    assert torch.equal(D, D3)


@pytest.mark.parametrize("out_features", [16, 2, 5])
@pytest.mark.parametrize("x_dtype", [torch.bfloat16, torch.float32])
def test_linear_fn_matches_autocast_linear(out_features, x_dtype):
    """ops.linear (trainable weight, bf16 autocast): forward is the autocast GEMM bit for bit;
    dX equals autocast's (bf16 GEMM output, cast to an fp32 input's dtype by autograd as for
    F.linear); dW / db are the fp32 sums autocast rounds to bf16 (tolerance: one bf16 rounding,
    2^-8 relative).  out_features < 8 takes the zero-padded weight-gradient path."""
    from irads import ops
    from semseg.models.layers.common import TrainLinear
    torch.manual_seed(2)
    lin = torch.nn.Linear(128, out_features).to(DEV)
    tl = TrainLinear(128, out_features).to(DEV)
    tl.load_state_dict(lin.state_dict())
    x = torch.randn(2, 300, 128, device=DEV).to(x_dtype)
    g = torch.randn(2, 300, out_features, device=DEV).bfloat16()
    assert ops.wgrad_ok(128, out_features)
    outs = []
    for mod in (lin, tl):
        xx = x.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = mod(xx)
        gx, gw, gb = torch.autograd.grad(y, [xx, mod.weight, mod.bias], g)
        outs.append((y, gx, gw, gb))
    (y0, gx0, gw0, gb0), (y1, gx1, gw1, gb1) = outs
    assert y1.dtype == torch.bfloat16 and torch.equal(y0, y1)
    assert gx1.dtype == x_dtype
    assert torch.equal(gx0, gx1)
    assert _rel(gw1, gw0) < 4e-3 and _rel(gb1, gb0) < 4e-3


@pytest.mark.parametrize("in_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C", [128, 512, 1024, 2048, 3072])
def test_layer_norm_bf16_matches_autocast(C, in_dtype):
    """ops.layer_norm_bf16 (frozen affine LN feeding a Linear): the bf16 output is autocast's
    fp32 LayerNorm rounded to bf16 (1 ulp on a few elements: reduction order), and dX is
    autograd's through that cast (relative L2 1e-3).  A bf16 input (DeformMPG's fuse_norm
    on the U_fc1 output) takes the bf16-in / bf16-out kernels where C / 64 allows."""
    from irads import ops
    torch.manual_seed(C)
    norm = torch.nn.LayerNorm(C).to(DEV)
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
        norm.bias.uniform_(-0.2, 0.2)
    norm.requires_grad_(False)
    x = (torch.randn(2, 333, C, device=DEV) * 2 + 0.3).to(in_dtype)
    g = torch.randn(2, 333, C, device=DEV).bfloat16()
    outs = []
    for fused in (False, True):
        xx = x.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            assert ops.ln_bf16_ok(xx, norm)
            y = ops.layer_norm_bf16(xx, norm) if fused else norm(xx).to(torch.bfloat16)
        (gx,) = torch.autograd.grad(y, [xx], g)
        outs.append((y, gx))
    (y0, gx0), (y1, gx1) = outs
    assert y1.dtype == torch.bfloat16 and y1.shape == y0.shape
    d = (y1.float() - y0.float()).abs()
    assert (d <= y0.float().abs() * 2 ** -7 + 1e-6).all()
    assert gx1.dtype == in_dtype and _rel(gx1.float(), gx0.float()) < 1e-3


@pytest.mark.parametrize("C", [128, 1024])
def test_layer_norm_bf16_pair_matches_two_norms(C):
    """ops.layer_norm_bf16_pair (the two streams' output norms on one batched tensor) gives
    exactly the two separate layer_norm_bf16 calls on x[:B] and x[B:]: same kernels on the
    same rows, so outputs and dX are bit-identical, including with one half's grad unused."""
    from irads import ops
    torch.manual_seed(C + 1)
    norms = [torch.nn.LayerNorm(C).to(DEV) for _ in range(2)]
    for n in norms:
        with torch.no_grad():
            n.weight.uniform_(0.5, 1.5)
            n.bias.uniform_(-0.2, 0.2)
        n.requires_grad_(False)
    x = torch.randn(4, 257, C, device=DEV) * 2 + 0.3
    g = torch.randn(4, 257, C, device=DEV).bfloat16()
    for use_second in (True, False):
        outs = []
        for pair in (False, True):
            xx = x.clone().requires_grad_()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                if pair:
                    y1, y2 = ops.layer_norm_bf16_pair(xx, *norms)
                else:
                    y1, y2 = ops.layer_norm_bf16(xx[:2], norms[0]), ops.layer_norm_bf16(xx[2:], norms[1])
            ys, gs = ([y1, y2], [g[:2], g[2:]]) if use_second else ([y1], [g[:2]])
            (gx,) = torch.autograd.grad(ys, [xx], gs)
            outs.append((y1, y2, gx))
        for a, b in zip(*outs):
            assert a.dtype == b.dtype and torch.equal(a, b)


def test_patch_merging_reshape_matches_unfold():
    """PatchMerging's permute-reshape equals nn.Unfold's 2x2 sampling (same channel order),
    and under AMP the block output matches the unfold + LayerNorm + Linear path."""
    from semseg.models.backbones.embed import PatchMerging
    torch.manual_seed(4)
    pm = PatchMerging(128, 256).to(DEV)
    fill_module(pm)
    pm.requires_grad_(False)
    B, H, W = 2, 32, 48
    x = torch.randn(B, H * W, 128, device=DEV)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y, hw = pm(x, (H, W))
        ref_cols = pm.sampler(x.view(B, H, W, 128).permute(0, 3, 1, 2)).transpose(1, 2)
        ref = pm.reduction(pm.norm(ref_cols))
    assert hw == (H // 2, W // 2) and y.shape == ref.shape
    assert _rel(y, ref) < 5e-3


@pytest.mark.parametrize("C,Mh", [(128, 4096), (256, 1024), (512, 512), (1024, 256), (192, 240)])
def test_adapter_kernels_match_linear_path(C, Mh):
    """irads_adapter_down / _up (both modality halves per launch) against the per-half
    F.linear + relu_dropout element path they replace, in autocast rounding.  The GEMM
    accumulation order differs (hipBLASLt vs one MFMA chain), so a bf16 GEMM output may
    differ by one ulp; the dropout mask is the same draw (same seed, salt, index)."""
    N = _N()
    torch.manual_seed(C)
    R, M, p = C // 16, 2 * Mh, 0.1
    x = (torch.randn(M, C, device=DEV) * 0.5).bfloat16()
    W1 = (torch.randn(2, R, C, device=DEV) * C ** -0.5).bfloat16()
    B1 = (torch.randn(2, R, device=DEV) * 0.1).bfloat16()
    W2 = (torch.randn(2, C, R, device=DEV) * R ** -0.5).bfloat16()
    B2 = (torch.randn(2, C, device=DEV) * 0.1).bfloat16()
    seed = torch.tensor([123456789], device=DEV, dtype=torch.int64)
    salts = (0x1234567, 0x7654321)
    st = N.stream()
    r = torch.empty(M, R, device=DEV, dtype=torch.bfloat16)
    N.call("irads_adapter_down", 0, N.ptr(x), N.ptr(W1[0]), N.ptr(W1[1]), N.ptr(B1[0]), N.ptr(B1[1]), None, M, Mh,
           C, R, p, salts[0], salts[1], N.ptr(seed), N.ptr(r), st)
    d = torch.empty(M, C, device=DEV, dtype=torch.bfloat16)
    N.call("irads_adapter_up", N.ptr(r), N.ptr(W2[0]), N.ptr(W2[1]), N.ptr(B2[0]), N.ptr(B2[1]), M, Mh, C, R,
           N.ptr(d), st)
    dd = (torch.randn(M, C, device=DEV) * 0.1).bfloat16()
    W2t, W1t = W2.transpose(1, 2).contiguous(), W1.transpose(1, 2).contiguous()
    dA = torch.empty(M, R, device=DEV, dtype=torch.bfloat16)
    N.call("irads_adapter_down", 1, N.ptr(dd), N.ptr(W2t[0]), N.ptr(W2t[1]), None, None, N.ptr(r), M, Mh, C, R, p,
           0, 0, None, N.ptr(dA), st)
    dx = torch.empty(M, C, device=DEV, dtype=torch.bfloat16)
    N.call("irads_adapter_up", N.ptr(dA), N.ptr(W1t[0]), N.ptr(W1t[1]), None, None, M, Mh, C, R, N.ptr(dx), st)
    for h in (0, 1):
        rows = slice(h * Mh, (h + 1) * Mh)
        lin = F.linear(x[rows], W1[h], B1[h])
        r_ref = torch.empty_like(lin)
        N.call("irads_relu_dropout_fwd", N.ptr(lin), N.ptr(r_ref), r_ref.numel(), p, salts[h], N.ptr(seed), st)
        # same mask: where the reference kept a positive value the kernel did too
        keep_ref, keep = r_ref != 0, r[rows] != 0
        assert (keep_ref != keep).float().mean().item() < 1e-3  # only ulp-level flips at lin ~ 0
        assert _rel(r[rows], r_ref) < 4e-3
        d_ref = torch.addmm(B2[h], r[rows], W2[h].t())
        assert _rel(d[rows], d_ref) < 4e-3
        dr = torch.mm(dd[rows], W2[h])
        dA_ref = torch.empty_like(dr)
        N.call("irads_relu_dropout_bwd", N.ptr(r[rows].contiguous()), N.ptr(dr), N.ptr(dA_ref), dr.numel(), p, st)
        assert torch.equal(dA[rows] != 0, dA_ref != 0) or (dA[rows] != 0).ne(dA_ref != 0).float().mean() < 1e-3
        assert _rel(dA[rows], dA_ref) < 4e-3
        assert _rel(dx[rows], torch.mm(dA[rows], W1[h])) < 4e-3


def test_wgrad_batched_matches_single():
    """irads_wgrad_batched: four problems of one shape (the Adapter layout: two transposed
    stores with column sums of B, two plain with column sums of A) against the fp32 A^T B
    and column sums of the same bf16 operands (fp32 accumulation order: rtol 1e-5)."""
    from irads import ops
    torch.manual_seed(5)
    K, m, n = 8192, 32, 512
    probs, refs = [], []
    for q in range(4):
        A = (torch.randn(K, m, device=DEV) * 0.3).bfloat16()
        B = (torch.randn(K, n, device=DEV) * 0.3).bfloat16()
        tr = q % 2 == 0
        D = torch.empty((n, m) if tr else (m, n), device=DEV)
        sa = None if tr else torch.empty(m, device=DEV)
        sb = torch.empty(n, device=DEV) if tr else None
        probs.append((A, B, D, sa, sb, tr))
        ref = A.float().t() @ B.float()
        refs.append((ref.t() if tr else ref, A.float().sum(0), B.float().sum(0)))
    ops.wgrad_batched(probs)
    for (A, B, D, sa, sb, tr), (ref, ca, cb) in zip(probs, refs):
        torch.testing.assert_close(D, ref, rtol=1e-5, atol=1e-3)
        if sa is not None:
            torch.testing.assert_close(sa, ca, rtol=1e-5, atol=1e-3)
        if sb is not None:
            torch.testing.assert_close(sb, cb, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("sdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C,L", [(128, 4096), (256, 1024), (512, 256), (1024, 64), (192, 300)])
def test_mpg_residual_matches_module_math(C, L, sdt):
    """irads_mpg_fwd/bwd against MPGBlock's prompt arithmetic + the stage loop's residual adds
    + torch.cat under autocast.  Forward: the same fp32 ops in the same order, bit-exact.
    Backward: dx_rgb / dx_dte are the halves of the incoming gradient (exact); the tfts
    gradients are fp32 sums in another order (rtol 1e-5); dx is the exact sum rounded to bf16
    once (one bf16 rounding + the fp32 rounding of its terms, against fp64)."""
    from irads import ops
    from semseg.models.backbones.swin import apply_tfts
    torch.manual_seed(C)
    B = 2
    x = (torch.randn(B, L, C, device=DEV)).bfloat16().requires_grad_()
    # stream inputs fp32 (stage 0) or bf16 (stages 1-3: PatchMerging's GEMM output)
    xr = torch.randn(B, L, C, device=DEV).to(sdt).requires_grad_()
    xd = torch.randn(B, L, C, device=DEV).to(sdt).requires_grad_()
    prm = [(torch.randn(C, device=DEV) * 0.1 + (1.0 if i % 2 == 0 else 0.0)).requires_grad_() for i in range(4)]
    g = torch.randn(2 * B, L, C, device=DEV)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ref = torch.cat([xr + (x + apply_tfts(x, prm[0], prm[1])), xd + (x + apply_tfts(x, prm[2], prm[3]))], 0)
        out = ops.MPGResidualFn.apply(x, xr, xd, *prm)
    assert out.dtype == ref.dtype == torch.float32 and torch.equal(out, ref)
    g_ref = torch.autograd.grad(ref, [x, xr, xd] + prm, g)
    g_out = torch.autograd.grad(out, [x, xr, xd] + prm, g)
    assert torch.equal(g_out[1], g_ref[1]) and torch.equal(g_out[2], g_ref[2])
    # dx: one rounding of the exact sum (autograd's four bf16-rounded partial terms can be
    # several ulps off it under cancellation, so the check is against fp64, not against autograd)
    gd = g.double()
    exact = (gd[:B] + gd[:B] * prm[0].double() + gd[B:] + gd[B:] * prm[2].double())
    # one bf16 rounding of the result + the fp32 rounding of the four terms it sums
    terms = gd[:B].abs() * (1 + prm[0].double().abs()) + gd[B:].abs() * (1 + prm[2].double().abs())
    tol = torch.finfo(torch.bfloat16).eps * exact.abs() + 4 * torch.finfo(torch.float32).eps * terms
    assert ((g_out[0].double() - exact).abs() <= tol).all()
    for a, b in zip(g_out[3:], g_ref[3:]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-3)


def test_patch_embed_gemm_matches_conv():
    """PatchEmbed under bf16 autocast: non-overlapping patches as one gather + GEMM (token-major
    output, contiguous LayerNorm input) against the Conv2d + flatten/transpose path.  Same bf16
    operands; the conv adds its bias in a second rounding and sums in another order: output and
    gradients within relative L2 1e-2."""
    from semseg.models.backbones.embed import PatchEmbed
    torch.manual_seed(9)
    pe = PatchEmbed(3, 128, 'Conv2d', 4, 4, 'corner', norm_cfg=dict(type='LN')).to(DEV)
    fill_module(pe, seed=2)
    x = torch.randn(2, 3, 64, 96, device=DEV)
    g = torch.randn(2, 16 * 24, 128, device=DEV)
    res = []
    for fast in (True, False):
        if not fast:
            pe._patchify_ok = lambda *a, **k: False
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y, hw = pe(x)
        grads = torch.autograd.grad(y, list(pe.parameters()), g)
        res.append((y, hw, grads))
    del pe._patchify_ok
    (y1, hw1, g1), (y0, hw0, g0) = res
    assert hw1 == hw0 == (16, 24) and y1.shape == y0.shape and y1.dtype == y0.dtype
    assert _rel(y1, y0) < 1e-2
    for a, b in zip(g1, g0):
        assert _rel(a, b) < 1e-2


@pytest.mark.parametrize("C,M", [(128, 131072), (192, 3000), (64, 77), (256, 1000)])
def test_layer_norm_from_bf16_matches_autocast(C, M):
    """irads_ln_bf16_fwd/bwd (PatchEmbed's trainable norm on the bf16 projection output)
    against nn.LayerNorm under bf16 autocast (fp32 math on the upcast input).  Forward and
    the gamma / beta gradients are fp32 sums in another order (rtol 1e-5 / 1e-4); dx is one
    bf16 rounding of the fp32 result."""
    from irads import ops
    torch.manual_seed(C + M)
    norm = torch.nn.LayerNorm(C).to(DEV)
    with torch.no_grad():
        norm.weight.copy_(torch.randn(C) * 0.2 + 1)
        norm.bias.copy_(torch.randn(C) * 0.1)
    x = (torch.randn(2, M // 2 if M % 2 == 0 else M, C, device=DEV) * 3 + 0.5).bfloat16()
    g = torch.randn(x.shape, device=DEV)
    outs = []
    for fn in (lambda t: norm(t), lambda t: ops.layer_norm_from_bf16(t, norm)):
        xx = x.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = fn(xx)
        outs.append((y,) + torch.autograd.grad(y, [xx, norm.weight, norm.bias], g))
    (y0, dx0, dw0, db0), (y1, dx1, dw1, db1) = outs
    assert y1.dtype == y0.dtype == torch.float32 and dx1.dtype == torch.bfloat16
    torch.testing.assert_close(y1, y0, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dx1.float(), dx0.float(), rtol=2 ** -7, atol=1e-3)
    torch.testing.assert_close(dw1, dw0, rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(db1, db0, rtol=1e-4, atol=1e-2)
    with torch.autocast("cuda", dtype=torch.bfloat16):  # the output may be modified in place (apply_mask)
        y = ops.layer_norm_from_bf16(x.clone().requires_grad_(), norm)
    y[0].zero_()


@pytest.mark.parametrize("C,H,W", [(128, 64, 64), (256, 32, 32), (512, 16, 16), (192, 12, 20)])
def test_patch_merge_norm_matches_unfold_path(C, H, W):
    """irads_merge_ln_fwd/bwd (PatchMerging's 2x2 unfold as the frozen LayerNorm's gather)
    against nn.Unfold + LayerNorm(4C) under autocast (fp32 math, bf16 operand of the
    reduction): one bf16 rounding apart in the forward; dx fp32 within the rounding of the
    bf16 incoming gradient's fp32 LayerNorm backward (rtol 1e-4)."""
    from irads import ops
    torch.manual_seed(C + H)
    B = 3
    norm = torch.nn.LayerNorm(4 * C).to(DEV).requires_grad_(False)
    with torch.no_grad():
        norm.weight.copy_(torch.randn(4 * C) * 0.2 + 1)
        norm.bias.copy_(torch.randn(4 * C) * 0.1)
    x = torch.randn(B, H * W, C, device=DEV) * 2 + 0.3
    g = torch.randn(B, H * W // 4, 4 * C, device=DEV).bfloat16()
    xa = x.clone().requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        unf = torch.nn.functional.unfold(xa.view(B, H, W, C).permute(0, 3, 1, 2), 2, stride=2).transpose(1, 2)
        ya = norm(unf).to(torch.bfloat16)
    (dxa,) = torch.autograd.grad(ya, xa, g)
    xb = x.clone().requires_grad_()
    yb = ops.PatchMergeNormFn.apply(xb, H, W, norm.weight, norm.bias, norm.eps)
    (dxb,) = torch.autograd.grad(yb, xb, g)
    assert yb.dtype == torch.bfloat16 and yb.shape == ya.shape
    torch.testing.assert_close(yb.float(), ya.float(), rtol=2 ** -7, atol=1e-2)
    torch.testing.assert_close(dxb, dxa, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("C,H,W", [(128, 32, 32), (256, 16, 24)])
def test_stage_tail_matches_separate_norms(C, H, W):
    """ops.stage_tail (output norms of both streams + PatchMerging's gather-norm on the batched
    stage output, one node) against the two separate ops: same kernels forward (bit-exact);
    backward writes the norms' gradient and adds the PatchMerging gradient in place: the fp32
    sum autograd forms from the two nodes, to one rounding (the kernels are built without FMA
    contraction, so in practice bit-exact)."""
    from irads import ops
    torch.manual_seed(C + W)
    B = 2
    norms = [torch.nn.LayerNorm(n).to(DEV).requires_grad_(False) for n in (4 * C, C, C)]
    with torch.no_grad():
        for nm in norms:
            nm.weight.uniform_(0.5, 1.5)
            nm.bias.uniform_(-0.2, 0.2)
    x = torch.randn(2 * B, H * W, C, device=DEV) * 2 + 0.3
    gm = torch.randn(2 * B, H * W // 4, 4 * C, device=DEV).bfloat16()
    g1, g2 = (torch.randn(B, H * W, C, device=DEV).bfloat16() for _ in range(2))
    xa = x.clone().requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert ops.stage_tail_ok(xa, H, W, norms[0], norms[1], norms[2])
        ya = ops.stage_tail(xa, H, W, *norms)
    xb = x.clone().requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ymb = ops.PatchMergeNormFn.apply(xb, H, W, norms[0].weight, norms[0].bias, norms[0].eps)
        y1b, y2b = ops.layer_norm_bf16_pair(xb, norms[1], norms[2])
    for a, b in zip(ya, (ymb, y1b, y2b)):
        assert torch.equal(a, b)
    (da,) = torch.autograd.grad(ya, xa, (gm, g1, g2))
    (db,) = torch.autograd.grad((ymb, y1b, y2b), xb, (gm, g1, g2))
    torch.testing.assert_close(da, db, rtol=2e-7, atol=1e-7)  # one fp32 rounding of the same two terms


@pytest.mark.parametrize("count", [1, 2, 3, 4])
@pytest.mark.parametrize("sums", ["none", "a", "b", "both"])
@pytest.mark.parametrize("K,m,n", [(8192, 32, 512), (1000, 16, 128), (64, 128, 256)])
def test_wgrad_batched_stays_in_its_workspace(count, sums, K, m, n):
    """Regression for the round-1 illegal-address fault ("Scratch memory"): every
    batched launch, with and without column-sum pointers, writes only inside the workspace
    irads_wgrad_batched_workspace() sizes (a NaN-filled guard region behind it stays intact) and
    gives the fp32 A^T B and column sums of each problem."""
    from irads import native as N
    from irads.ops import _WgradProblem
    torch.manual_seed(count * 7 + K)
    arr = (_WgradProblem * count)()
    keep = []
    for q in range(count):
        A = (torch.randn(K, m, device=DEV) * 0.3).bfloat16()
        B = (torch.randn(K, n, device=DEV) * 0.3).bfloat16()
        D = torch.full((m, n), float("nan"), device=DEV)
        sa = torch.full((m,), float("nan"), device=DEV) if sums in ("a", "both") else None
        sb = torch.full((n,), float("nan"), device=DEV) if sums in ("b", "both") else None
        arr[q] = _WgradProblem(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), D.data_ptr(),
                               None if sa is None else sa.data_ptr(), None if sb is None else sb.data_ptr(), 0)
        keep.append((A, B, D, sa, sb))
    need = N.load().irads_wgrad_batched_workspace(count, K, m, n)
    guard = 1 << 16
    ws = torch.full((need + guard,), float("nan"), device=DEV)
    N.call("irads_wgrad_batched", count, arr, K, m, n, 1.0, 0, N.ptr(ws), N.stream())
    torch.cuda.synchronize()
    assert torch.isnan(ws[need:]).all(), "irads_wgrad_batched wrote past its workspace"
    for A, B, D, sa, sb in keep:
        torch.testing.assert_close(D, A.float().t() @ B.float(), rtol=1e-5, atol=1e-3)
        if sa is not None:
            torch.testing.assert_close(sa, A.float().sum(0), rtol=1e-5, atol=1e-3)
        if sb is not None:
            torch.testing.assert_close(sb, B.float().sum(0), rtol=1e-5, atol=1e-3)


def test_bias_quads_cache_lives_with_its_table():
    """ops.bias_quads caches the re-laid bias table on its owner Parameter: a hit while the
    table is unchanged, a recompute after an in-place update (new version), the entry dropped
    when the table dies (so a graph that read cached quads holds valid memory exactly as long
    as its model), and a trainable table being captured recomputes inside the graph."""
    from irads import ops
    table = torch.nn.Parameter(torch.randn(529, 4, device=DEV), requires_grad=False)
    q1 = ops.bias_quads(table.detach(), 4, 32 ** -0.5, owner=table)
    q2 = ops.bias_quads(table.detach(), 4, 32 ** -0.5, owner=table)
    assert q1 is q2
    ref = q1.clone()
    with torch.no_grad():
        table.mul_(2.0)
    q3 = ops.bias_quads(table.detach(), 4, 32 ** -0.5, owner=table)
    assert q3 is not q1 and not torch.equal(q3, ref)
    assert ops.bias_quads(table.detach(), 4, 32 ** -0.5) is not q3  # no owner: no caching
    k = id(table)
    assert k in ops._QUADS
    del table
    import gc
    gc.collect()
    assert k not in ops._QUADS
    tr = torch.nn.Parameter(torch.randn(529, 4, device=DEV))
    eager = ops.bias_quads(tr.detach(), 4, 1.0, owner=tr)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            inside = ops.bias_quads(tr.detach(), 4, 1.0, owner=tr)
    torch.cuda.synchronize()
    assert inside is not eager
    with torch.no_grad():
        tr.add_(1.0)
    g.replay()
    torch.cuda.synchronize()
    fresh = ops.bias_quads(tr.detach(), 4, 1.0)
    assert torch.equal(inside, fresh)
