"""The frozen Swin trunk's projection GEMMs: irads_gemm_nt (csrc/gemm.hip) where it measured faster
than hipBLASLt, F.linear / torch.mm elsewhere.

Reference: the Linear layers of ShiftWindowMSA (qkv, proj; swin.py:81-119) and the mmcv FFN
(swin.py:586-601) under bf16 autocast.  The trunk is frozen (TRAIN_TYPE Adapter), so a layer is
used as  y = x Wᵀ + b  forward and  dX = dY W  backward, both "NT" products of K-contiguous
operands once Wᵀ is kept beside W (made once per weight version).

Which kernel serves a shape is a table, not a heuristic: scripts/gemm_tune.py times both on the
shapes of BASELINE.json's C2 and C4 steps (interleaved rounds in one process) and writes
tuned/irads_gemm_select_mi355x.json, the (direction, M, N, K) keys where irads_gemm_nt measured
within 5 % of hipBLASLt or faster for the C2 shapes (in that step it gains on the library: 0.1 ms per
step better than a "5 % faster" rule), at least 5 % faster for the C3 / C4 shapes (there the looser
rule measured slower), each with the tiling that won (variant 2: 128 x 128 tiles, 2 workgroups per CU; 4: 256 x 256
tiles on 8 waves, N % 256 == 0).  Directions: "fwd" (y = x Wᵀ + b), "bwd" (dX = dY W), and the FFN's fused pairs
"fwd_gelu" (fc1 with the erf GELU in the epilogue, against the better GEMM + gelu pass) and
"bwd_dgelu" (fc2's dX with GELU' applied in the epilogue, against GEMM + gelu_bwd pass).  A
shape not in the table, or one the kernel cannot take (N % 128, K % 64, an operand not 16-byte aligned
or with a leading dimension not a multiple of 8), goes to hipBLASLt.  IRADS_GEMM=off sends every shape
to hipBLASLt, IRADS_GEMM=all every shape the kernel takes to irads_gemm_nt (A/B and tests), on the
tiling IRADS_GEMM_VARIANT names (default 2; variant 4 where N % 256 == 0, else 2); IRADS_GEMM_SELECT
names another table file (A/B of a re-tune).
"""
import json
import os

import torch
import torch.nn.functional as F

from . import native as N
from .stamps import STAMPS

_BF16 = torch.bfloat16
_TABLE_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned", "irads_gemm_select_mi355x.json")
_table = None


DEFAULT_VARIANT = 2  # 128 x 128 tiles, 2 workgroups per CU (csrc/gemm.hip)


def _selected():
    """{(direction, M, N, K): tiling variant} of the shipped table (entries [dir, M, N, K, variant])."""
    global _table
    if _table is None:
        try:
            with open(os.environ.get("IRADS_GEMM_SELECT", _TABLE_PATH)) as fh:
                _table = {tuple(k[:4]): (k[4] if len(k) > 4 else DEFAULT_VARIANT) for k in json.load(fh)["irads"]}
        except FileNotFoundError:
            _table = {}
    return _table


def kernel_fits(N_out, K, variant=DEFAULT_VARIANT):
    return N_out % (256 if variant == 4 else 128) == 0 and K % 64 == 0


def use_irads(direction, M, N_out, K):
    """The irads_gemm_nt tiling variant serving this shape, or None for hipBLASLt."""
    mode = os.environ.get("IRADS_GEMM", "table")
    if mode == "off" or not kernel_fits(N_out, K):
        return None
    if mode == "all":
        v = int(os.environ.get("IRADS_GEMM_VARIANT", DEFAULT_VARIANT))
        return v if kernel_fits(N_out, K, v) else DEFAULT_VARIANT
    v = _selected().get((direction, M, N_out, K))
    return v if v is not None and kernel_fits(N_out, K, v) else None


def _aligned(*ts):
    """Every operand as the C entry point takes it: rows contiguous, 16-byte aligned base, leading
    dimension a multiple of 8 elements (a contiguous view at an odd offset goes to hipBLASLt)."""
    return all(t.stride(-1) == 1 and t.data_ptr() % 16 == 0 and t.stride(0) % 8 == 0 for t in ts)


def weights(lin):
    """(W bf16 [N, K], b bf16 [N] or None, Wᵀ bf16 [K, N], b fp32 or None) of a frozen Linear, cached
    on the module until a parameter's version moves (the fp32 bias is the bf16 one widened: the
    epilogue adds exactly what hipBLASLt's bias epilogue adds)."""
    w, b = lin.weight, lin.bias
    key = (w.data_ptr(), w._version, None if b is None else b._version)
    cache = lin.__dict__.get("_irads_gemm_cache")
    if cache is None or cache[0] != key:
        w16, b16 = lin.amp_weights(_BF16)
        with torch.no_grad():
            cache = (key, w16, b16, w16.t().contiguous(), None if b16 is None else b16.float())
        lin.__dict__["_irads_gemm_cache"] = cache
    return cache[1:]


def _nt(A, B, bias32, M, N_out, K, variant):
    out = torch.empty((M, N_out), device=A.device, dtype=_BF16)
    N.call("irads_gemm_nt_variant", variant, 0, N.ptr(A), A.stride(0), N.ptr(B), B.stride(0), N.ptr(bias32), None, 0,
           N.ptr(out), None, out.stride(0), M, N_out, K, N.stream())
    return out


def linear(x, lw):
    """y = x Wᵀ + b for x (M, K) bf16 contiguous and lw = weights(lin)."""
    w16, b16, _, b32 = lw
    M, K = x.shape
    N_out = w16.shape[0]
    v = use_irads("fwd", M, N_out, K)
    ok = v is not None and x.is_contiguous() and _aligned(x, w16)
    STAMPS.follow(ok)
    if ok:
        return _nt(x, w16, b32, M, N_out, K, v)
    return F.linear(x, w16, b16)


def ffn_up(h, lw):
    """(U, G) = (h W1ᵀ + b1, GELU(U)) of the FFN's first Linear: one irads_gemm_nt launch with the GELU
    in its epilogue where the table says so ("fwd_gelu"), else the GEMM and the element pass."""
    w16, _, _, b32 = lw
    M, K = h.shape
    N_out = w16.shape[0]
    v = use_irads("fwd_gelu", M, N_out, K)
    if v is not None and h.is_contiguous() and _aligned(h, w16):
        u = torch.empty((M, N_out), device=h.device, dtype=_BF16)
        g = torch.empty_like(u)
        N.call("irads_gemm_nt_variant", v, 1, N.ptr(h), h.stride(0), N.ptr(w16), w16.stride(0), N.ptr(b32), None, 0,
               N.ptr(u), N.ptr(g), u.stride(0), M, N_out, K, N.stream())
        return u, g
    u = linear(h, lw)
    g = torch.empty_like(u)
    N.call("irads_gelu_fwd", N.ptr(u), N.ptr(g), u.numel(), N.stream())
    return u, g


def ffn_down_dgrad_gelu(df, lw, u):
    """dU = GELU'(U) ⊙ (dF W2) through the FFN's second Linear and the GELU: one irads_gemm_nt launch
    with the dGELU in its epilogue where the table says so ("bwd_dgelu"; dG never reaches HBM), else
    the input-gradient GEMM and the element pass."""
    w16, _, wt, _ = lw
    M, N_in = df.shape
    K_out = w16.shape[1]
    v = use_irads("bwd_dgelu", M, K_out, N_in)
    if v is not None and df.is_contiguous() and u.is_contiguous() and _aligned(df, wt, u):
        du = torch.empty((M, K_out), device=df.device, dtype=_BF16)
        N.call("irads_gemm_nt_variant", v, 2, N.ptr(df), df.stride(0), N.ptr(wt), wt.stride(0), None, N.ptr(u), u.stride(0),
               N.ptr(du), None, du.stride(0), M, K_out, N_in, N.stream())
        return du
    dg = dgrad(df, lw)
    du = torch.empty_like(dg)
    N.call("irads_gelu_bwd", N.ptr(u), N.ptr(dg), N.ptr(du), du.numel(), N.stream())
    return du


def dgrad(dy, lw):
    """dX = dY W for dY (M, N) bf16 contiguous (the input gradient of a frozen Linear)."""
    w16, _, wt, _ = lw
    M, N_in = dy.shape
    K_out = w16.shape[1]
    v = use_irads("bwd", M, K_out, N_in)
    ok = v is not None and dy.is_contiguous() and _aligned(dy, wt)
    STAMPS.follow(ok)
    if ok:
        return _nt(dy, wt, None, M, K_out, N_in, v)
    return torch.mm(dy, w16)
