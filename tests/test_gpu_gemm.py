"""irads_gemm_nt (csrc/gemm.hip) and its dispatch (irads/gemm.py) on the GPU.

The kernel replaces hipBLASLt for some of the frozen Swin trunk's projections (swin.py:81-119,
:586-601 under bf16 autocast): C = bf16(A·Bᵀ (+ bias)) with fp32 accumulation.  Its summation
order differs from hipBLASLt's, so the bar is the library's own: relative L2 error against the
fp32 product within 1.5x hipBLASLt's on the same operands (both ≈ 2^-9, bf16 output rounding).
The GELU / dGELU epilogues are checked bit for bit against the element kernels applied to the
same GEMM's plain output; every tile variant bit for bit against the shipped one."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _N():
    from irads import native as N
    return N


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _gemm(epi, A, B, bias=None, U=None, C1=None, variant=None):
    N = _N()
    M, K = A.shape
    C0 = torch.empty((M, B.shape[0]), device=A.device, dtype=torch.bfloat16)
    args = (epi, N.ptr(A), A.stride(0), N.ptr(B), B.stride(0), N.ptr(bias), N.ptr(U), 0 if U is None else U.stride(0),
            N.ptr(C0), N.ptr(C1), C0.stride(0), M, B.shape[0], K, N.stream())
    if variant is None:
        N.call("irads_gemm_nt", *args)
    else:
        N.call("irads_gemm_nt_variant", variant, *args)
    return C0


N_VARIANTS = 5  # irads_gemm_nt_variant tilings 0-4 (4: 256 x 256, N % 256 == 0)

# (M, N, K): trunk shapes, a ragged M (tiles past M clamped / masked), a single k-step, a long K
SHAPES = [(16384, 512, 512), (4096, 1024, 4096), (1000, 384, 128), (77, 128, 64), (2048, 2048, 1536)]


@pytest.mark.parametrize("M,Nn,K", SHAPES)
def test_gemm_nt_bias_vs_fp32_and_hipblaslt(M, Nn, K):
    torch.manual_seed(M + Nn + K)
    A = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(Nn, K, device=DEV) * K ** -0.5).bfloat16()
    b16 = (torch.randn(Nn, device=DEV) * 0.1).bfloat16()
    ref = torch.addmm(b16.float(), A.float(), W.float().t())
    lib = F.linear(A, W, b16)
    mine = _gemm(0, A, W, b16.float())
    assert _rel(mine, ref) <= 1.5 * _rel(lib, ref) + 1e-4, (_rel(mine, ref), _rel(lib, ref))
    # no bias, and every tile variant bit for bit
    nob = _gemm(0, A, W)
    assert _rel(nob, A.float() @ W.float().t()) <= 1.5 * _rel(lib, ref) + 1e-4
    for v in range(N_VARIANTS):
        if v >= 4 and Nn % 256:
            continue
        assert torch.equal(_gemm(0, A, W, b16.float(), variant=v), mine), v


@pytest.mark.parametrize("M,Nn,K", [(16384, 2048, 512), (1000, 384, 128), (4096, 512, 256)])
def test_gemm_nt_gelu_epilogues_bit_exact(M, Nn, K):
    """EPI_GELU / EPI_DGELU on EVERY tiling (variant 4 where N % 256 == 0): U, G and dU bit for bit
    those of the plain GEMM + irads_gelu_fwd / irads_gelu_bwd (the same accumulators: every variant
    sums the k-steps in the same order)."""
    N = _N()
    torch.manual_seed(7)
    A = torch.randn(M, K, device=DEV).bfloat16()
    W = (torch.randn(Nn, K, device=DEV) * K ** -0.5).bfloat16()
    b32 = (torch.randn(Nn, device=DEV) * 0.1).bfloat16().float()
    plain = _gemm(0, A, W, b32)
    g_ref = torch.empty_like(plain)
    N.call("irads_gelu_fwd", N.ptr(plain), N.ptr(g_ref), plain.numel(), N.stream())
    # dGELU: dU = bf16(bf16(dY·W) * GELU'(U)), U of the GEMM's output shape
    Wt = W.t().contiguous()  # (K, Nn): B operand of dX = dY W
    dY = torch.randn(M, Nn, device=DEV).bfloat16()
    U = (torch.randn(M, K, device=DEV) * 1.5).bfloat16()
    dx = _gemm(0, dY, Wt)
    du_ref = torch.empty_like(dx)
    N.call("irads_gelu_bwd", N.ptr(U), N.ptr(dx), N.ptr(du_ref), dx.numel(), N.stream())
    for v in range(N_VARIANTS):
        if not (v >= 4 and Nn % 256):
            g = torch.empty_like(plain)
            u = _gemm(1, A, W, b32, C1=g, variant=v)
            assert torch.equal(u, plain), v
            assert torch.equal(g, g_ref), v
        if not (v >= 4 and K % 256):
            du = _gemm(2, dY, Wt, U=U, variant=v)
            assert torch.equal(du, du_ref), v


def test_gelu_table_covers_every_bf16_u():
    """The 256 x 256 tiling's GELU' table (gemm.hip gemm_gelu_table_kernel, staged in LDS) against the
    formula path, bit for bit, on EVERY bf16 value of U (65 536 patterns as a 256 x 256 U: zeros,
    denormals, the table's exponent range, the values beyond it, Inf and NaN), through EPI_DGELU
    against the plain GEMM + irads_gelu_bwd."""
    N = _N()
    torch.manual_seed(11)
    dY = torch.randn(256, 64, device=DEV).bfloat16()
    Wt = (torch.randn(256, 64, device=DEV) * 0.125).bfloat16()
    U = torch.arange(65536, dtype=torch.int32, device=DEV).to(torch.int16).view(torch.bfloat16).reshape(256, 256)
    U = U.contiguous()
    dx = _gemm(0, dY, Wt, variant=4)
    ref = torch.empty_like(dx)
    N.call("irads_gelu_bwd", N.ptr(U), N.ptr(dx), N.ptr(ref), dx.numel(), N.stream())
    du = _gemm(2, dY, Wt, U=U, variant=4)
    assert torch.equal(du.view(torch.int16), ref.view(torch.int16))


def _entry_id(e):
    (d, M, Nn, K), v = e
    return f"{d}-{M}x{Nn}x{K}-v{v}"


def _shipped_entries():
    # read at collection time without touching the GPU (irads.gemm imports only json / torch)
    import json
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    path = os.path.join(here, "..", "ir-ads_amd", "irads", "tuned", "irads_gemm_select_mi355x.json")
    with open(path) as fh:
        return [((k[0], k[1], k[2], k[3]), k[4] if len(k) > 4 else 2) for k in json.load(fh)["irads"]]


@pytest.mark.parametrize("entry", _shipped_entries(), ids=_entry_id)
def test_shipped_table_entry(entry):
    """Every (direction, M, N, K) -> tiling entry of irads/tuned/irads_gemm_select_mi355x.json, launched
    exactly as irads.gemm launches it (the listed variant and epilogue), at its full shape:
      * against the fp32 product (addmm), relative L2 <= 1.5x hipBLASLt's own on the same operands;
      * bit for bit against the plain variant-2 GEMM (+ irads_gelu_fwd / _bwd for the fused pairs)."""
    from irads import gemm as G
    N = _N()
    (d, M, Nn, K), v = entry
    assert G.kernel_fits(Nn, K, v), entry
    torch.manual_seed(M % 9973 + Nn + K)
    A = torch.randn(M, K, device=DEV).bfloat16()
    B = (torch.randn(Nn, K, device=DEV) * K ** -0.5).bfloat16()
    bias = (torch.randn(Nn, device=DEV) * 0.1).bfloat16() if d in ("fwd", "fwd_gelu") else None
    b32 = None if bias is None else bias.float()
    ref = A.float() @ B.float().t()
    if bias is not None:
        ref += b32
    lib = F.linear(A, B, bias)
    lib_err = _rel(lib, ref)
    del lib
    plain = _gemm(0, A, B, b32, variant=2)
    if d in ("fwd", "bwd"):
        out = _gemm(0, A, B, b32, variant=v)
        assert torch.equal(out, plain), entry
        e = _rel(out, ref)
        assert e <= 1.5 * lib_err + 1e-4, (entry, e, lib_err)
    elif d == "fwd_gelu":
        g = torch.empty_like(plain)
        u = _gemm(1, A, B, b32, C1=g, variant=v)
        assert torch.equal(u, plain), entry
        g_ref = torch.empty_like(u)
        N.call("irads_gelu_fwd", N.ptr(plain), N.ptr(g_ref), plain.numel(), N.stream())
        assert torch.equal(g, g_ref), entry
        e = _rel(u, ref)
        assert e <= 1.5 * lib_err + 1e-4, (entry, e, lib_err)
        assert _rel(g, F.gelu(ref)) < 6e-3, entry
    else:  # bwd_dgelu: dU = bf16(bf16(dY W) GELU'(U)), U of the output's shape
        U = (torch.randn(M, Nn, device=DEV) * 1.5).bfloat16()
        du = _gemm(2, A, B, U=U, variant=v)
        du_ref = torch.empty_like(du)
        N.call("irads_gelu_bwd", N.ptr(U), N.ptr(plain), N.ptr(du_ref), du.numel(), N.stream())
        assert torch.equal(du, du_ref), entry
        e = _rel(plain, ref)
        assert e <= 1.5 * lib_err + 1e-4, (entry, e, lib_err)
        u = U.float()
        dgelu = 0.5 * (1 + torch.erf(u * 0.7071067811865476)) + u * torch.exp(-0.5 * u * u) * 0.3989422804014327
        assert _rel(du, ref * dgelu) < 6e-3, entry


def test_dispatch_falls_back_on_misaligned_views(monkeypatch):
    """A contiguous view at an offset that is not 16-byte aligned goes to hipBLASLt instead of
    raising in the C entry point (irads.gemm._aligned)."""
    from irads import gemm as G
    from semseg.models.layers.common import Linear
    monkeypatch.setenv("IRADS_GEMM", "all")
    torch.manual_seed(5)
    lin = Linear(256, 512).to(DEV).requires_grad_(False)
    lw = G.weights(lin)
    w16, b16 = lin.amp_weights(torch.bfloat16)
    buf = torch.randn(1024 * 256 + 1, device=DEV).bfloat16()
    x = buf[1:].view(1024, 256)  # 2-byte offset
    assert x.is_contiguous() and x.data_ptr() % 16
    y = G.linear(x, lw)
    assert torch.equal(y, F.linear(x, w16, b16))
    dy = torch.randn(1024 * 512 + 1, device=DEV).bfloat16()[1:].view(1024, 512)
    assert torch.equal(G.dgrad(dy, lw), torch.mm(dy, w16))


def test_gemm_nt_rejects_unsupported_shapes():
    N = _N()
    A = torch.zeros(256, 192, device=DEV, dtype=torch.bfloat16)
    W = torch.zeros(192, 192, device=DEV, dtype=torch.bfloat16)
    C0 = torch.empty(256, 192, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="N % 128"):  # N = 192
        N.call("irads_gemm_nt", 0, N.ptr(A), 192, N.ptr(W), 192, None, None, 0, N.ptr(C0), None, 192, 256, 192, 192,
               N.stream())
    W2 = torch.zeros(256, 96, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="K % 64"):  # K = 96
        N.call("irads_gemm_nt", 0, N.ptr(A), 192, N.ptr(W2), 96, None, None, 0, N.ptr(C0), None, 192, 256, 256, 96,
               N.stream())


@pytest.mark.parametrize("mode", ["all", "off", "table"])
def test_dispatch_linear_and_dgrad(mode, monkeypatch):
    """irads.gemm.linear / dgrad against F.linear / torch.mm on a frozen Linear, every dispatch mode."""
    from irads import gemm as G
    from semseg.models.layers.common import Linear
    monkeypatch.setenv("IRADS_GEMM", mode)
    torch.manual_seed(11)
    lin = Linear(512, 2048).to(DEV).requires_grad_(False)
    x = torch.randn(16384, 512, device=DEV).bfloat16()
    lw = G.weights(lin)
    w16, b16 = lin.amp_weights(torch.bfloat16)
    ref = torch.addmm(b16.float(), x.float(), w16.float().t())
    lib = F.linear(x, w16, b16)
    y = G.linear(x, lw)
    assert _rel(y, ref) <= 1.5 * _rel(lib, ref) + 1e-4
    if mode == "off":
        assert torch.equal(y, lib)
    dy = torch.randn(16384, 2048, device=DEV).bfloat16()
    ref = dy.float() @ w16.float()
    lib = torch.mm(dy, w16)
    dx = G.dgrad(dy, lw)
    assert _rel(dx, ref) <= 1.5 * _rel(lib, ref) + 1e-4
    if mode == "off":
        assert torch.equal(dx, lib)
    # the cached transpose follows a weight update
    with torch.no_grad():
        lin.weight.mul_(2)
    lw2 = G.weights(lin)
    assert torch.equal(lw2[2], lin.amp_weights(torch.bfloat16)[0].t())


@pytest.mark.parametrize("mode", ["all", "all4", "off"])
def test_ffn_fused_gelu_paths(mode, monkeypatch):
    """irads.gemm.ffn_up / ffn_down_dgrad_gelu (GELU and GELU' in irads_gemm_nt's epilogue) against the
    unfused GEMM + element passes: bit for bit given the same GEMM (mode all: both arms irads_gemm_nt),
    and within hipBLASLt's own rounding of the fp32 result (mode off: the hipBLASLt arm)."""
    from irads import gemm as G
    from semseg.models.layers.common import Linear
    N = _N()
    torch.manual_seed(13)
    C, M = 256, 4096
    fc1 = Linear(C, 4 * C).to(DEV).requires_grad_(False)
    fc2 = Linear(4 * C, C).to(DEV).requires_grad_(False)
    l1, l2 = G.weights(fc1), G.weights(fc2)
    h = torch.randn(M, C, device=DEV).bfloat16()
    df = torch.randn(M, C, device=DEV).bfloat16()
    monkeypatch.setenv("IRADS_GEMM", mode[:3])
    if mode == "all4":  # the 256 x 256 tiling (two 64-row epilogue halves) for every fitting shape
        monkeypatch.setenv("IRADS_GEMM_VARIANT", "4")
        assert G.use_irads("fwd_gelu", M, 4 * C, C) == 4 and G.use_irads("bwd_dgelu", M, 4 * C, C) == 4
    u, g = G.ffn_up(h, l1)
    du = G.ffn_down_dgrad_gelu(df, l2, u)
    # unfused arms with the same GEMM kernel
    u2 = G.linear(h, l1)
    g2 = torch.empty_like(u2)
    N.call("irads_gelu_fwd", N.ptr(u2), N.ptr(g2), u2.numel(), N.stream())
    dg2 = G.dgrad(df, l2)
    du2 = torch.empty_like(dg2)
    N.call("irads_gelu_bwd", N.ptr(u), N.ptr(dg2), N.ptr(du2), du2.numel(), N.stream())
    assert torch.equal(u, u2) and torch.equal(g, g2) and torch.equal(du, du2)
    # and against fp32 math on the same operands
    w1, b1 = fc1.amp_weights(torch.bfloat16)
    ref_u = torch.addmm(b1.float(), h.float(), w1.float().t())
    assert _rel(u, ref_u) < 4e-3
    assert _rel(g, F.gelu(ref_u)) < 4e-3
