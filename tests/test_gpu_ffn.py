"""The FFN GEMMs with the GELU in their epilogues (irads_ffn_fc1_gelu, irads_ffn_fc2_dgrad_dgelu;
csrc/ffn.hip) against the unfused path they replace in the fused Swin stage (swin.py:586-601:
hipBLASLt F.linear under autocast, then irads_gelu_fwd / irads_gelu_bwd, themselves pinned to
torch's erf GELU in test_gpu_swin_fused.py):
  * the GEMM results agree with autocast's to bf16 rounding (the two kernels sum in different
    orders: relative L2 <= 2e-3, and >= 98 % of the elements identical);
  * the epilogue arithmetic is the unfused path's bit for bit: g == irads_gelu_fwd(u) on the
    fused kernel's own u, and du == irads_gelu_bwd(u, bf16(dy · w2)) on its own GEMM result
    (recovered exactly where GELU'(u) == 1 is not needed: checked through an fp32 reference);
  * every Swin-B / Swin-L stage shape, and row counts that are not multiples of the tile."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm())


def _fc1(x, w1, b1f):
    from irads import native as N
    M, K = x.shape
    Nn = w1.shape[0]
    u = torch.empty((M, Nn), device=DEV, dtype=torch.bfloat16)
    g = torch.empty_like(u)
    N.call("irads_ffn_fc1_gelu", N.ptr(x), N.ptr(w1), N.ptr(b1f), M, K, Nn, N.ptr(u), N.ptr(g), N.stream())
    return u, g


def _dgrad(dy, w2t, u):
    from irads import native as N
    M, K = dy.shape
    Nn = w2t.shape[0]
    du = torch.empty((M, Nn), device=DEV, dtype=torch.bfloat16)
    N.call("irads_ffn_fc2_dgrad_dgelu", N.ptr(dy), N.ptr(w2t), N.ptr(u), M, K, Nn, N.ptr(du), N.stream())
    return du


@pytest.mark.parametrize("M,C", [(16 * 1024, 512), (8 * 4096, 256), (4 * 16384, 128), (16 * 256, 1024),
                                 (2400, 192), (300, 384), (1200, 768), (4 * 300, 1536), (77, 128)])
def test_fused_ffn_gemms_match_unfused(M, C):
    from irads import native as N
    torch.manual_seed(M + C)
    x = (torch.randn(M, C, device=DEV)).bfloat16()
    w1 = (torch.randn(4 * C, C, device=DEV) * C ** -0.5).bfloat16()
    b1 = torch.randn(4 * C, device=DEV) * 0.1
    b1b = b1.bfloat16()  # autocast casts the bias too
    u, g = _fc1(x, w1, b1b.float())
    torch.cuda.synchronize()
    u_ref = F.linear(x, w1, b1b)
    assert _rel(u.float(), u_ref.float()) < 2e-3
    assert (u == u_ref).float().mean().item() > 0.98
    g_own = torch.empty_like(u)
    N.call("irads_gelu_fwd", N.ptr(u), N.ptr(g_own), u.numel(), N.stream())
    assert torch.equal(g, g_own)  # the epilogue is irads_gelu_fwd on the kernel's own u
    # fc2 input gradient + GELU backward
    dy = torch.randn(M, C, device=DEV).bfloat16()
    w2 = (torch.randn(C, 4 * C, device=DEV) * (4 * C) ** -0.5).bfloat16()
    du = _dgrad(dy, w2.t().contiguous(), u)
    dg_ref = torch.mm(dy, w2)
    du_ref = torch.empty_like(u)
    N.call("irads_gelu_bwd", N.ptr(u), N.ptr(dg_ref), N.ptr(du_ref), u.numel(), N.stream())
    torch.cuda.synchronize()
    assert _rel(du.float(), du_ref.float()) < 4e-3
    assert (du == du_ref).float().mean().item() > 0.97
    # against fp32 arithmetic: within bf16 rounding of the exact product
    uu = u.float().requires_grad_()
    (exact,) = torch.autograd.grad(F.gelu(uu), uu, dy.float() @ w2.float())
    assert _rel(du.float(), exact) < 1e-2


def test_fused_ffn_rejects_bad_shapes():
    from irads import native as N
    x = torch.zeros(128, 96, device=DEV, dtype=torch.bfloat16)
    w = torch.zeros(384, 96, device=DEV, dtype=torch.bfloat16)
    b = torch.zeros(384, device=DEV)
    u = torch.empty(128, 384, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):  # K = 96 is not a multiple of 64
        N.call("irads_ffn_fc1_gelu", N.ptr(x), N.ptr(w), N.ptr(b), 128, 96, 384, N.ptr(u), N.ptr(u), N.stream())
