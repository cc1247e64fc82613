"""The two bf16 window-attention forward kernels (irads_winattn_fwd_variant: 0 = one workgroup per
(window, head), 1 = persistent LDS-DMA pipelined) perform the same arithmetic: outputs and LSE
must be bit-identical on every geometry the C1-C4 configs produce (padding, shifted windows, the
explicit-mask path), on chunkings that leave workgroups with one window or none, and the
backward must accept either forward's LSE."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(variant, qkv, bias, table, mask, H, W, nH, shift, scale):
    from irads import native as N, ops
    lib = N.load()
    prev = lib.irads_winattn_fwd_variant(variant)
    try:
        out, lse = ops.winattn_fwd(qkv, bias, table, mask, H, W, nH, shift, scale)
        torch.cuda.synchronize()
    finally:
        lib.irads_winattn_fwd_variant(prev)
    return out, lse


@pytest.mark.parametrize("B,side_h,side_w,C,shift,explicit_mask", [
    (4, 128, 128, 128, 0, False), (4, 128, 128, 128, 6, False),   # C2 stage 0 (pad 132)
    (4, 32, 32, 512, 6, False), (2, 16, 16, 1024, 0, False),     # C2 stages 2 / 3
    (2, 30, 40, 384, 6, False), (3, 60, 80, 192, 6, False),      # Swin-L 480x640 stages
    (1, 12, 12, 128, 0, False), (1, 13, 25, 128, 6, False),      # one window; ragged pads
    (2, 24, 24, 128, 6, True)])                                   # explicit WindowMSA mask
def test_pipelined_forward_bitexact(B, side_h, side_w, C, shift, explicit_mask):
    torch.manual_seed(B * 1000 + C + shift)
    nH = C // 32
    qkv = (torch.randn(B, side_h * side_w, 3 * C, device=DEV) * 0.7).bfloat16()
    bias = torch.randn(3 * C, device=DEV) * 0.1
    table = torch.randn(23 * 23, nH, device=DEV) * 0.5
    mask = None
    if explicit_mask:
        nW = (-(-side_h // 12)) * (-(-side_w // 12))
        mask = torch.where(torch.rand(nW, 144, 144, device=DEV) < 0.2, -100.0, 0.0)
    scale = 32 ** -0.5
    o0, l0 = _run(0, qkv, bias, table, mask, side_h, side_w, nH, shift, scale)
    o1, l1 = _run(1, qkv, bias, table, mask, side_h, side_w, nH, shift, scale)
    assert torch.equal(o0, o1), (o0.float() - o1.float()).abs().max().item()
    assert torch.equal(l0, l1)


def test_pipelined_forward_through_backward():
    """The shifted-window op end to end with the pipelined forward: gradients equal the per-item
    forward's (the backward reads the forward's out and LSE)."""
    from irads import native as N, ops
    torch.manual_seed(7)
    B, H, W, C, nH = 4, 32, 32, 256, 8
    qkv = (torch.randn(B, H * W, 3 * C, device=DEV) * 0.7).bfloat16()
    bias = torch.randn(3 * C, device=DEV) * 0.1
    table = torch.randn(23 * 23, nH, device=DEV) * 0.5
    gout = torch.randn(B, H * W, C, device=DEV).bfloat16()
    lib = N.load()
    res = []
    for v in (0, 1):
        prev = lib.irads_winattn_fwd_variant(v)
        try:
            x = qkv.clone().requires_grad_()
            y = ops.window_attention(x, bias, table, None, H, W, nH, 6, 32 ** -0.5)
            (g,) = torch.autograd.grad(y, x, gout)
            torch.cuda.synchronize()
        finally:
            lib.irads_winattn_fwd_variant(prev)
        res.append((y, g))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
