"""Segmentation-head tail on the HIP path: bilinear resize (segformer.py:44,
cmnext.py:30-32) and the fused softmax cross-entropy / MMST objective (losses.py:6-19,
train_mm.py:137-148).

Oracle: the reference calls these as plain PyTorch ops, so the checker is the same call
on the CPU in fp32/fp64 (F.interpolate, nn.CrossEntropyLoss and autograd through them),
plus the MMST golden fixture generated from the reference's formula
(tests/golden/metrics_loss.npz, oracle/gen_golden.py:394-413).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from golden_util import Fixture, close

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ops():
    from irads import ops
    return ops


def _rand(shape, seed, dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g, dtype=torch.float64).to(dtype)


def _fmt(x, cl):
    return x.contiguous(memory_format=torch.channels_last) if cl else x.contiguous()


RESIZE_CASES = [
    # (B, C, h, w, H, W)
    (2, 40, 32, 32, 128, 128),   # x4: CMNeXt logits -> image size (scaled down)
    (2, 64, 16, 16, 32, 32),     # x2: SegFormer c2 -> c1 grid
    (1, 16, 8, 8, 64, 64),       # x8: c4 -> c1
    (2, 5, 13, 17, 50, 61),      # non-integer ratios
    (1, 3, 37, 29, 30, 20),      # downscale
    (1, 1, 1, 1, 7, 5),          # single source pixel
    (3, 8, 9, 9, 9, 9),          # identity size
]


@pytest.mark.parametrize("cl", [False, True])
@pytest.mark.parametrize("case", RESIZE_CASES)
def test_resize_fp32_vs_interpolate(case, cl):
    ops = _ops()
    B, C, h, w, H, W = case
    x = _fmt(_rand((B, C, h, w), 1), cl)
    ref = F.interpolate(x, size=(H, W), mode="bilinear", align_corners=False)
    xg = x.to(DEV).requires_grad_(True)
    out = ops.resize(xg, (H, W))
    assert out.is_contiguous(memory_format=torch.channels_last if (cl and C > 1) else torch.contiguous_format)
    close(out, ref, 2e-6, 2e-6, f"resize fwd {case}")
    # backward = adjoint, vs autograd through F.interpolate in fp64
    go = _rand((B, C, H, W), 2)
    xd = x.double().requires_grad_(True)
    F.interpolate(xd, size=(H, W), mode="bilinear", align_corners=False).backward(go.double())
    out.backward(_fmt(go, cl).to(DEV))
    close(xg.grad, xd.grad, 2e-5, 1e-5, f"resize bwd {case}")


@pytest.mark.parametrize("cl", [False, True])
def test_resize_bf16(cl):
    """bf16 storage, fp32 arithmetic: within one bf16 rounding of the exact value."""
    ops = _ops()
    B, C, h, w, H, W = 2, 40, 32, 32, 128, 128
    x = _fmt(_rand((B, C, h, w), 3).to(torch.bfloat16), cl)
    exact = F.interpolate(x.double(), size=(H, W), mode="bilinear", align_corners=False)
    xg = x.to(DEV).requires_grad_(True)
    out = ops.resize(xg, (H, W))
    close(out.float(), exact, 1e-6, 2 ** -8, "resize bf16 fwd")
    go = _rand((B, C, H, W), 4).to(torch.bfloat16)
    xd = x.double().requires_grad_(True)
    F.interpolate(xd, size=(H, W), mode="bilinear", align_corners=False).backward(go.double())
    out.backward(_fmt(go, cl).to(DEV))
    close(xg.grad.float(), xd.grad, 1e-5, 2 ** -7, "resize bf16 bwd")


def test_resize_full_size_c2():
    """C2 shapes: 8 x 40 x 128² logits to 512² (cmnext.py:30) — forward exact vs CPU fp32,
    backward checked through <gin, x> = <gout, resize(x)> (adjointness, size-independent)."""
    ops = _ops()
    x = _rand((8, 40, 128, 128), 5)
    out = ops.resize(x.to(DEV), (512, 512))
    ref = F.interpolate(x, size=(512, 512), mode="bilinear", align_corners=False)
    close(out, ref, 2e-6, 2e-6, "resize C2 fwd")
    go = _rand((8, 40, 512, 512), 6).to(DEV)
    xg = x.to(DEV).requires_grad_(True)
    ops.resize(xg, (512, 512)).backward(go)
    lhs = (xg.grad.double() * x.to(DEV).double()).sum()
    rhs = (go.double() * out.double()).sum()
    assert abs(float(lhs - rhs)) <= 1e-4 * abs(float(rhs)) + 1e-3


def _targets(B, H, W, C, seed, ignore=255, p_ignore=0.1):
    g = torch.Generator().manual_seed(seed)
    t = torch.randint(0, C, (B, H, W), generator=g)
    t[torch.rand((B, H, W), generator=g) < p_ignore] = ignore
    return t


@pytest.mark.parametrize("cl", [False, True])
@pytest.mark.parametrize("C", [1, 7, 19, 40, 64, 100, 128])
def test_cross_entropy_fp32(C, cl):
    ops = _ops()
    B, H, W = 2, 24, 31
    x = _fmt(_rand((B, C, H, W), 10 + C) * 3, cl)
    t = _targets(B, H, W, C, 20 + C)
    xd = x.double().requires_grad_(True)
    ref = F.cross_entropy(xd, t, ignore_index=255)
    ref.backward()
    xg = x.to(DEV).requires_grad_(True)
    loss = ops.cross_entropy(xg, t.to(DEV), 255)
    close(loss, ref, 1e-6, 1e-6, f"CE fwd C={C}")
    loss.backward()
    close(xg.grad, xd.grad, 1e-7, 1e-5, f"CE bwd C={C}")


def test_cross_entropy_weights_and_grad_scale():
    ops = _ops()
    B, C, H, W = 2, 9, 16, 20
    x = _rand((B, C, H, W), 30) * 2
    t = _targets(B, H, W, C, 31)
    wt = torch.rand(C, generator=torch.Generator().manual_seed(32)) + 0.5
    xd = x.double().requires_grad_(True)
    ref = F.cross_entropy(xd, t, weight=wt.double(), ignore_index=255)
    (3.5 * ref).backward()
    xg = x.to(DEV).requires_grad_(True)
    loss = ops.cross_entropy(xg, t.to(DEV), 255, wt.to(DEV))
    close(loss, ref, 1e-6, 1e-6, "weighted CE fwd")
    (3.5 * loss).backward()
    close(xg.grad, xd.grad, 1e-7, 1e-5, "weighted CE bwd")


@pytest.mark.parametrize("cl", [False, True])
def test_cross_entropy_bf16(cl):
    """bf16 logits (the reference's AMP path casts them to fp32 before the loss)."""
    ops = _ops()
    B, C, H, W = 2, 40, 32, 48
    x = _fmt((_rand((B, C, H, W), 40) * 4).to(torch.bfloat16), cl)
    t = _targets(B, H, W, C, 41)
    xd = x.double().requires_grad_(True)
    ref = F.cross_entropy(xd, t, ignore_index=255)
    ref.backward()
    xg = x.to(DEV).requires_grad_(True)
    loss = ops.cross_entropy(xg, t.to(DEV), 255)
    close(loss, ref, 1e-6, 1e-5, "CE bf16 fwd")
    loss.backward()
    assert xg.grad.dtype == torch.bfloat16
    close(xg.grad.float(), xd.grad, 1e-9, 2 ** -8, "CE bf16 bwd")


def test_cross_entropy_edges():
    ops = _ops()
    # every pixel ignored: nan, as nn.CrossEntropyLoss
    x = _rand((1, 4, 3, 3), 50).to(DEV)
    t = torch.full((1, 3, 3), 255, dtype=torch.int64, device=DEV)
    assert torch.isnan(ops.cross_entropy(x, t, 255))
    # a 1x1 image, custom ignore index
    x = _rand((3, 6, 1, 1), 51)
    t = torch.tensor([[[2]], [[-100]], [[5]]])
    ref = F.cross_entropy(x, t, ignore_index=-100)
    close(ops.cross_entropy(x.to(DEV), t.to(DEV), -100), ref, 1e-6, 1e-6, "1x1 CE")
    with pytest.raises(RuntimeError):
        ops.cross_entropy(_rand((1, 129, 2, 2), 52).to(DEV), torch.zeros(1, 2, 2, dtype=torch.int64, device=DEV))
    with pytest.raises(RuntimeError):
        ops.cross_entropy(_rand((1, 3, 2, 2), 53).to(DEV), torch.zeros(1, 2, 3, dtype=torch.int64, device=DEV))
    # documented deviation: a target outside [0, C) that is not ignore_index counts as
    # an ignored pixel (no loss, zero gradient, MMST target = ignore) where nn.CrossEntropyLoss raises
    # a device-side assert; the loss equals the reference's on the same pixels marked ignored
    x = _rand((2, 5, 4, 4), 54).to(DEV).requires_grad_()
    t = torch.randint(0, 5, (2, 4, 4), device=DEV)
    t[0, 1, 2], t[1, 3, 0] = 7, -3
    loss, match = ops.cross_entropy(x, t, 255, return_match=True)
    t_ref = t.clone()
    t_ref[(t_ref < 0) | (t_ref >= 5)] = 255
    xr = x.detach().clone().requires_grad_()
    ref = F.cross_entropy(xr, t_ref, ignore_index=255)
    close(loss, ref, 1e-6, 1e-6, "CE with out-of-range targets")
    (gx,) = torch.autograd.grad(loss, x)
    (gr,) = torch.autograd.grad(ref, xr)
    close(gx, gr, 1e-7, 1e-6, "CE grad with out-of-range targets")
    assert gx[0, :, 1, 2].abs().max() == 0 and gx[1, :, 3, 0].abs().max() == 0
    assert match[0, 1, 2] == 255 and match[1, 3, 0] == 255


def test_mmst_target_and_loss_golden():
    """MMST (train_mm.py:137-148) against the fixture made from the reference formula."""
    from semseg.losses import get_loss, mmst_loss
    ops = _ops()
    fx = Fixture("metrics_loss.npz")
    logits, gt = fx.t("logits", device=DEV), fx.t("gt", device=DEV)
    loss = mmst_loss(get_loss("CrossEntropy", 255), logits, fx.t("logits_rgb", device=DEV),
                     fx.t("logits_dte", device=DEV), gt)
    close(loss, fx["mmst_loss"], 1e-6, 1e-6, "MMST loss")
    _, match = ops.cross_entropy(logits, gt, 255, return_match=True)
    pred = fx.t("logits").softmax(dim=1).argmax(dim=1)
    want = fx.t("gt").clone()
    want[pred != want] = 255
    assert torch.equal(match.cpu(), want)


def test_mmst_full_size_c2_bf16():
    """C2 sizes (8 x 40 x 512², bf16 logits): loss vs the CPU restatement on the same
    bf16 values, gradients of all three heads vs autograd in fp64."""
    from semseg.losses import get_loss, mmst_loss
    import irads_ref as R
    B, C, H, W = 8, 40, 512, 512
    xs = [(_rand((B, C, H, W), 60 + i) * 3).to(torch.bfloat16) for i in range(3)]
    t = _targets(B, H, W, C, 63)
    xd = [x.double().requires_grad_(True) for x in xs]
    ref = R.mmst_loss(*xd, t)
    ref.backward()
    xg = [x.to(DEV).requires_grad_(True) for x in xs]
    loss = mmst_loss(get_loss("CrossEntropy", 255), *xg, t.to(DEV))
    close(loss, ref, 1e-5, 1e-5, "MMST C2 loss")
    loss.backward()
    for i in range(3):
        scale = float(xd[i].grad.abs().max())
        close(xg[i].grad.float(), xd[i].grad, 1e-3 * scale, 2 ** -7, f"MMST C2 grad head {i}")


@pytest.mark.parametrize("E", [256, 512])
def test_head_bnact_tail_matches_module_path(E):
    """SegFormerHead in training mode under bf16 autocast: the fused BN (batch statistics) +
    ReLU + Dropout2d kernels + token-major linear_pred against the module path (nn.BatchNorm2d
    on MIOpen, in-place ReLU, Dropout2d, 1x1 Conv2d).  With Dropout2d at p = 0 the two are the
    same arithmetic up to the BN normalisation's fp32 formula and GEMM summation order: output
    and every gradient within relative L2 1e-2 (the MLP biases, whose gradient BatchNorm
    cancels, only need to be noise-sized), running statistics within 1e-5.  A second pass
    at p = 0.5 checks the Dropout2d semantics: each (image, channel) of the fused map is either
    zeroed or scaled by 1 / (1 - p)."""
    from semseg.models.heads import SegFormerHead
    from fill import fill_module
    torch.manual_seed(E)
    dims = [128, 256, 512, 1024]
    heads = []
    for _ in range(2):
        h = SegFormerHead(dims, E, 40).to(DEV)
        heads.append(h)
    fill_module(heads[0], seed=3)
    heads[1].load_state_dict(heads[0].state_dict())
    B, sizes = 2, [(64, 64), (32, 32), (16, 16), (8, 8)]
    feats = [torch.randn(B, c, *hw, device=DEV).contiguous(memory_format=torch.channels_last)
             for c, hw in zip(dims, sizes)]
    res = []
    for k, h in enumerate(heads):
        h.train()
        h.dropout.p = 0.0
        fs = [f.clone().requires_grad_() for f in feats]
        from irads import ops
        orig = ops.bnact_ok
        if k == 1:
            ops.bnact_ok = lambda *a, **kw: False
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = h(fs)
        finally:
            ops.bnact_ok = orig
        torch.manual_seed(7)
        go = torch.randn(out.shape, device=DEV)
        params = [p for p in h.parameters() if p.requires_grad]
        grads = torch.autograd.grad(out, fs + params, go)
        res.append((out, grads, h.linear_fuse.bn.running_mean.clone(), h.linear_fuse.bn.running_var.clone()))
    (o1, g1, rm1, rv1), (o0, g0, rm0, rv0) = res

    def rel(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()
    assert o1.shape == o0.shape and rel(o1, o0) < 1e-2
    names = [f"feat{i}" for i in range(4)] + [n for n, p in heads[0].named_parameters() if p.requires_grad]
    for n, a, b in zip(names, g1, g0):
        if n.startswith("linear_c") and n.endswith("proj.bias"):
            # a per-channel constant ahead of train-mode BatchNorm: the gradient vanishes
            # analytically and is rounding noise in both paths
            assert a.abs().max() < 1e-2 * g0[names.index(n[:-4] + "weight")].abs().max() + 1e-3, n
            continue
        assert rel(a, b) < 1e-2, (n, rel(a, b))
    torch.testing.assert_close(rm1, rm0, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(rv1, rv0, rtol=1e-5, atol=1e-5)
    # Dropout2d semantics on the fused kernels
    from irads import ops
    bn = heads[0].linear_fuse.bn
    x = torch.randn(B, 100, E, device=DEV).bfloat16()
    with torch.no_grad():
        torch.manual_seed(1)
        y0 = ops.bn_relu_dropout2d(x, bn, 0.0).float()
        y1 = ops.bn_relu_dropout2d(x, bn, 0.5).float()
    ratio = torch.where(y0 != 0, y1 / y0.where(y0 != 0, torch.ones_like(y0)), torch.zeros_like(y0))
    per_chan = ratio.abs().amax(1)  # (B, E): 0 (dropped) or 2 (kept)
    assert ((per_chan == 0) | ((per_chan - 2).abs() < 1e-2)).all()
    assert 0.2 < (per_chan > 0).float().mean().item() < 0.8


@pytest.mark.parametrize("E,M", [(256, 2 * 64 * 64), (512, 2 * 128 * 128), (768, 77)])
def test_bnact_finalize_and_sums_pass_match_torch_expressions(E, M):
    """irads_bnact_finalize (batch mean / invstd + running-statistics update in one launch) and
    irads_bnact_bwd_sums (pass 2 from the raw sums) bit for bit (invstd within 1 ulp) against the
    torch expressions they replace: m1 = S1 / M, mean = x[0] + m1, var = (S2 / M - m1²).clamp_min(0), rsqrt(var + eps),
    running_*.mul_(1 - mom).add_(.., alpha=mom), num_batches_tracked += 1; md, mdx = S / M."""
    from irads import native as N
    torch.manual_seed(E + M)
    x = torch.randn(M, E, device=DEV).bfloat16()
    sums = torch.randn(2 * E, device=DEV) * 50
    sums[E:] = sums[E:].abs() * 20
    sums[E + 3] = 0.0  # a channel whose variance formula goes negative -> clamped to 0
    bn = torch.nn.BatchNorm2d(E).to(DEV)
    bn.running_mean.normal_()
    bn.running_var.uniform_(0.5, 2.0)
    rm, rv, nbt = bn.running_mean.clone(), bn.running_var.clone(), bn.num_batches_tracked.clone()
    s = sums.view(2, E)
    m1 = s[0] / M
    mean_ref = x[0].float() + m1
    var = (s[1] / M - m1 * m1).clamp_min(0.)
    inv_ref = torch.rsqrt(var + bn.eps)
    mom = bn.momentum
    rm.mul_(1 - mom).add_(mean_ref, alpha=mom)
    rv.mul_(1 - mom).add_(var * (M / (M - 1)), alpha=mom)
    nbt.add_(1)
    mean = torch.empty(E, device=DEV)
    inv = torch.empty(E, device=DEV)
    N.call("irads_bnact_finalize", N.ptr(sums), N.ptr(x), M, E, float(bn.eps), float(mom), N.ptr(mean), N.ptr(inv),
           N.ptr(bn.running_mean), N.ptr(bn.running_var), N.ptr(bn.num_batches_tracked), N.stream())
    assert torch.equal(mean, mean_ref)
    # the variance is bit-exact (running_var carries it); rsqrt is the device library's, within an ulp
    # of torch's rsqrt kernel (the two builds lower it differently)
    ulp = (inv_ref.view(torch.int32) - inv.view(torch.int32)).abs()
    assert int(ulp.max()) <= 1, int(ulp.max())
    assert torch.equal(bn.running_mean, rm) and torch.equal(bn.running_var, rv)
    assert int(bn.num_batches_tracked) == int(nbt)
    # pass 2 from the raw sums against pass 2 from torch's S / M
    L = M // 2 if M % 2 == 0 else M
    w = torch.randn(E, device=DEV)
    b = torch.randn(E, device=DEV)
    dy = torch.randn(M, E, device=DEV).bfloat16()
    dsum = torch.randn(2 * E, device=DEV) * 30
    md, mdx = dsum[:E] / M, dsum[E:] / M
    dx0, dx1 = torch.empty_like(x), torch.empty_like(x)
    N.call("irads_bnact_bwd", N.ptr(dy), N.ptr(x), M, E, L, N.ptr(mean), N.ptr(inv), N.ptr(w), N.ptr(b), None, None,
           N.ptr(md), N.ptr(mdx), N.ptr(dx0), N.stream())
    N.call("irads_bnact_bwd_sums", N.ptr(dy), N.ptr(x), M, E, L, N.ptr(mean), N.ptr(inv), N.ptr(w), N.ptr(b), None,
           N.ptr(dsum), N.ptr(dx1), N.stream())
    assert torch.equal(dx0, dx1)


RESIZE_CE_CASES = [
    # (B, C, h, w, H, W): x4 like the CMNeXt heads, ragged widths (segments of 32 low-res columns
    # with a partial last one), non-integer ratios, one-column / one-row maps
    (2, 40, 32, 32, 128, 128), (2, 16, 24, 70, 96, 280), (1, 8, 13, 17, 50, 61), (2, 24, 1, 9, 4, 36),
    (1, 16, 7, 1, 28, 4)]


def _spy_calls():
    from irads import native as N
    calls, orig = [], N.call

    def spy(name, *a):
        calls.append(name)
        return orig(name, *a)
    return calls, orig, spy


@pytest.mark.parametrize("case", RESIZE_CE_CASES)
def test_ce_through_resize_fused_fp32(case):
    """cross_entropy(resize(low)) takes its gradient to `low` in one irads_ce_resize_bwd pass:
    loss and gradient vs autograd through F.interpolate + F.cross_entropy in fp64, with class
    weights, ignored and out-of-range targets and a scaled loss."""
    from irads import native as N
    ops = _ops()
    B, C, h, w, H, W = case
    low = (_rand((B, C, h, w), 70 + C) * 2).contiguous(memory_format=torch.channels_last)
    t = _targets(B, H, W, C, 71 + C)
    t[0, 0, :2] = C + 3  # out of range: treated as ignored
    t_ref = t.clone()
    t_ref[t_ref == C + 3] = 255
    wt = torch.rand(C, generator=torch.Generator().manual_seed(72)) + 0.5
    ld = low.double().requires_grad_(True)
    ref = F.cross_entropy(F.interpolate(ld, (H, W), mode="bilinear", align_corners=False), t_ref,
                          weight=wt.double(), ignore_index=255)
    (2.5 * ref).backward()
    calls, orig, spy = _spy_calls()
    N.call = spy
    try:
        lg = low.to(DEV).requires_grad_(True)
        y = ops.resize(lg, (H, W))
        loss = ops.cross_entropy(y, t.to(DEV), 255, wt.to(DEV))
        (2.5 * loss).backward()
    finally:
        N.call = orig
    assert "irads_ce_resize_bwd" in calls and "irads_resize_bwd" not in calls and "irads_ce_bwd" not in calls
    close(loss, ref, 1e-6, 1e-6, f"CE(resize) fwd {case}")
    assert lg.grad.is_contiguous(memory_format=torch.channels_last)
    close(lg.grad, ld.grad, 1e-7, 1e-5, f"CE(resize) bwd {case}")


def test_ce_through_resize_fused_bf16_and_fallbacks():
    """bf16 (the AMP path): the fused gradient against fp64 autograd is at least as close as the
    unfused one (which rounds the full-resolution gradient to bf16 first); the unfused path still
    serves NCHW logits, a modified output and no-grad inputs."""
    from irads import native as N
    ops = _ops()
    B, C, h, w, H, W = 2, 40, 32, 40, 128, 160
    low = (_rand((B, C, h, w), 80) * 3).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    t = _targets(B, H, W, C, 81)
    ld = low.double().requires_grad_(True)
    F.cross_entropy(F.interpolate(ld, (H, W), mode="bilinear", align_corners=False), t, ignore_index=255).backward()
    grads = {}
    for fused in (True, False):
        lg = low.to(DEV).requires_grad_(True)
        y = ops.resize(lg, (H, W))
        if not fused:
            y = y * 1  # a new tensor: not ops.resize's output, so the unfused path runs
        ops.cross_entropy(y, t.to(DEV), 255).backward()
        assert lg.grad.dtype == torch.bfloat16
        grads[fused] = lg.grad.double().cpu()
    ref = ld.grad
    err = {k: float((g - ref).norm() / ref.norm()) for k, g in grads.items()}
    assert err[True] <= 4e-3 and err[True] <= err[False] * 1.05, err
    # fallbacks: NCHW logits, an in-place-modified output, a source that wants no gradient
    calls, orig, spy = _spy_calls()
    N.call = spy
    try:
        lg = low.float().contiguous().to(DEV).requires_grad_(True)
        ops.cross_entropy(ops.resize(lg, (H, W)), t.to(DEV), 255).backward()
        lg2 = low.to(DEV).requires_grad_(True)
        y2 = ops.resize(lg2, (H, W))
        y2.mul_(1.0)
        ops.cross_entropy(y2, t.to(DEV), 255).backward()
        ops.cross_entropy(ops.resize(low.to(DEV), (H, W)).requires_grad_(), t.to(DEV), 255).backward()
    finally:
        N.call = orig
    assert "irads_ce_resize_bwd" not in calls and calls.count("irads_ce_bwd") == 3


@pytest.mark.parametrize("C,h,H", [(512, 64, 128), (256, 32, 128), (512, 16, 128), (40, 13, 50), (24, 9, 36)])
def test_resize_adjoint_one_pass_vs_two_pass(C, h, H):
    """Channels-last resize gradients take irads_resize_bwd_cl (rows reduced in LDS, one pass;
    the SegFormer upsample_sum sources and the CMNeXt logits): against the NCHW two-pass adjoint
    (irads_resize_bwd) on the same gradient, fp32 to 1e-5 relative and bf16 to one rounding,
    and fp32 against F.interpolate's autograd in fp64."""
    from irads import native as N
    ops = _ops()
    B = 2
    assert N.load().irads_resize_bwd_cl_fits(C, h, H)
    x = _rand((B, C, h, h + 3), 90 + C)
    go = _rand((B, C, H, H + 12), 91 + C)
    xd = x.double().requires_grad_(True)
    F.interpolate(xd, (H, H + 12), mode="bilinear", align_corners=False).backward(go.double())
    for dt, rtol in ((torch.float32, 1e-5), (torch.bfloat16, 2 ** -7)):
        grads = []
        for cl in (True, False):
            xg = _fmt(x.to(dt), cl).to(DEV).requires_grad_(True)
            y = ops.resize(xg, (H, H + 12))
            y.backward(_fmt(go.to(dt), cl).to(DEV))
            grads.append(xg.grad.float().cpu())
        scale = float(grads[1].abs().max())
        close(grads[0], grads[1], rtol * scale, rtol, f"one-pass vs two-pass adjoint C={C} {dt}")
        if dt == torch.float32:
            close(grads[0], xd.grad, 1e-5 * scale, 1e-5, f"one-pass adjoint vs fp64 C={C}")
