"""Fused Swin stage: one autograd node per SwinBlockSequence under bf16 autocast.

Reference: SwinBlockAdapter.forward (semseg/models/backbones/swin.py:584-610) with
ShiftWindowMSA (:180-254), mmcv FFN and the MAPA Adapter (:472-502), iterated by
SwinBlockSequence.forward (:683-697), in TRAIN_TYPE Adapter (optimizers.py:7-30: the Swin
trunk is frozen, only the Adapters train).

Run op by op under autocast, a block is ~25 elementwise launches each way around its 9
GEMMs (LayerNorm in fp32, a cast to bf16 before every Linear, DropPath div/mul, residual
adds, GELU, ReLU/dropout, and the fp32 gradient sums of the residual stream).  Here a
stage is a single torch.autograd.Function whose forward and backward are hand-scheduled:

  forward, per block (M = 2B*H*W rows of the rgb+dte batch, C channels)
    h1            = LN1(x)                                 [resln_fwd, fused into the
                                                            previous block's output pass]
    qkv           = h1 Wqkvᵀ + b                          [irads_gemm_nt | hipBLASLt, irads.gemm]
    a             = shifted-window attention(qkv)         [irads_winattn_fwd]
    o             = a Wpᵀ + b                             [irads_gemm_nt | hipBLASLt]
    X1, h2, X1b   = x + DP(o), LN2(.), bf16(.)            [resln_fwd]
    g             = GELU(h2 W1ᵀ + b1)                      [irads_gemm_nt GELU epilogue | GEMM + gelu_fwd]
    f             = g W2ᵀ + b2                             [irads_gemm_nt | hipBLASLt]
    d[rgb|dte]    = Adapter_{rgb|dte}(X1b[rgb|dte])        [adapter_down + adapter_up]
    x'            = (X1 + DP(f)) + 0.5 d ; h1' = LN1'(x')  [resln_fwd]
  backward mirrors it with resln_bwd producing, in one pass, the fp32 residual gradient
  and the bf16 operands of the branches (DropPath-backward, 0.5 * for the adapter).

Rounding is the autocast reference's op by op (see csrc/swinblock.hip); each projection GEMM
is either the hipBLASLt call F.linear makes under autocast or irads_gemm_nt (bf16 operands,
fp32 accumulate, bf16(acc + bias)), per the measured selection table of irads.gemm.  Used only when the stage is frozen
(no trunk parameter requires grad) and autocast runs in bf16; any other configuration takes
the module-by-module path.  Gradient checkpointing (with_cp, Swin-L) is numerically neutral
and is not re-enacted: the fused stage keeps its activations.
"""
import torch
import torch.nn.functional as F

from . import gemm as G
from . import native as N
from . import ops

_BF16 = torch.bfloat16
ADAPTER_DROPOUT = 0.1  # hard-coded in the reference Adapter (swin.py:496)
_UNBATCHED = bool(__import__("os").environ.get("IRADS_WGRAD_UNBATCHED"))


def _frozen_trunk(block):
    for name, p in block.named_parameters():
        if "Adapter" not in name and p.requires_grad:
            return False
    return True


def usable(seq, x):
    """Whether the fused stage applies to this call (else the module path runs)."""
    if not (x.is_cuda and x.dtype == torch.float32 and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == _BF16):
        return False
    for blk in seq.blocks:
        # with_cp (Swin-L, base.py:43-50) only trades memory for recompute: the fused stage keeps
        # its activations (a few GB at Swin-L 480x640, B=4, well inside 288 GB) and serves it
        if not _frozen_trunk(blk):
            return False
        w = blk.attn.w_msa
        if w.attn_drop.p > 0 and blk.training:
            return False
        if blk.ffn.layers[0][2].p > 0 and blk.training or blk.ffn.layers[2].p > 0 and blk.training:
            return False
        if w.proj_drop.p > 0 and blk.training:
            return False
        if not isinstance(blk.ffn.layers[0][1], torch.nn.GELU) or blk.ffn.layers[0][1].approximate != "none":
            return False
        if not blk.ffn.add_identity:
            return False
        if blk.MLP_RGB_Adapter.prompt_add or blk.MLP_DTE_Adapter.prompt_add:
            return False
    C = x.shape[-1]
    return C % 64 == 0 and (C // 64) in (2, 3, 4, 6, 8, 12, 16, 24)


def adapter_params(seq):
    ps = []
    for blk in seq.blocks:
        for ad in (blk.MLP_RGB_Adapter, blk.MLP_DTE_Adapter):
            ps += [ad.D_fc1.weight, ad.D_fc1.bias, ad.D_fc2.weight, ad.D_fc2.bias]
    return ps


_DP_SALT = 0xD1B54A32D192ED03  # the DropPath stream of a stage's seed (the Adapters' use _salt)


def _droppath_scales(seq, S, device, seed=None):
    """(n_blocks, 2, S) fp32 per-sample factors s = mask ? fp32(1/keep) : 0 for the attention
    and FFN DropPaths (common.py DropPath: x.div(keep) * floor(keep + U), U in x.dtype), 1 for a
    branch without one, or None when no DropPath is active.  `seed`: int64 device tensor (the
    stage's Adapter-dropout seed), drawn here when None."""
    ps = []
    for blk in seq.blocks:
        pa = blk.attn.drop.p if (blk.training and getattr(blk.attn.drop, "p", 0)) else 0.
        pf = blk.ffn.dropout_layer.p if (blk.training and getattr(blk.ffn.dropout_layer, "p", 0)) else 0.
        ps.append((pa or 0., pf or 0.))
    if all(a == 0 and b == 0 for a, b in ps):
        return None
    cache = seq.__dict__.get("_dp_cache")
    if cache is None or cache[0] != (tuple(ps), device):
        keep = torch.tensor([[1. - a, 1. - b] for a, b in ps], dtype=torch.float64)
        inv = (1.0 / keep.float()).float()  # the fp32 reciprocal torch's div-by-scalar multiplies by
        cache = ((tuple(ps), device), keep.to(device).contiguous(), inv.to(device).contiguous())
        seq.__dict__["_dp_cache"] = cache
    _, keep, inv = cache
    if seed is None:
        seed = torch.randint(0, 2 ** 62, (1,), device=device, dtype=torch.int64)
    # floor(bf16(keep + U)) / keep per (block, branch, sample), 1 where the branch has no DropPath:
    # one launch (irads_droppath_scales) for what torch ran as rand, casts, add, floor, mul, where
    out = torch.empty((len(ps), 2, S), device=device, dtype=torch.float32)
    N.call("irads_droppath_scales", N.ptr(seed), _DP_SALT, N.ptr(keep), N.ptr(inv), 2 * len(ps), S, N.ptr(out),
           N.stream())
    return out


def _resln_fwd(x, M, C, rps, add1=None, add1_scale=None, add2=None, add2_mult=0.5, norm=None, x_out=False,
               xb_out=False):
    dev = x.device
    xo = torch.empty((M, C), device=dev, dtype=torch.float32) if x_out else None
    xb = torch.empty((M, C), device=dev, dtype=_BF16) if xb_out else None
    lo = mean = rstd = None
    g = b = None
    eps = 1e-5
    if norm is not None:
        lo = torch.empty((M, C), device=dev, dtype=_BF16)
        mean = torch.empty((M,), device=dev, dtype=torch.float32)
        rstd = torch.empty((M,), device=dev, dtype=torch.float32)
        g, b, eps = norm.weight, norm.bias, norm.eps
    N.call("irads_resln_fwd", N.ptr(x), N.ptr(add1), N.ptr(add1_scale), N.ptr(add2), float(add2_mult), M, C, rps,
           N.ptr(g), N.ptr(b), float(eps), N.ptr(xo), N.ptr(lo), N.ptr(xb), N.ptr(mean), N.ptr(rstd), N.stream())
    return xo, lo, xb, mean, rstd


def _resln_bwd(M, C, rps, dy=None, x=None, mean=None, rstd=None, norm=None, g_res=None, g_add=None, dx_out=True,
               b1_scale=None, b1=False, b2=False, b2_mult=0.5):
    dev = (g_res if g_res is not None else dy).device
    dx = torch.empty((M, C), device=dev, dtype=torch.float32) if dx_out else None
    o1 = torch.empty((M, C), device=dev, dtype=_BF16) if b1 else None
    o2 = torch.empty((M, C), device=dev, dtype=_BF16) if b2 else None
    gamma = None if norm is None else norm.weight
    N.call("irads_resln_bwd", N.ptr(dy), N.ptr(x), N.ptr(mean), N.ptr(rstd), N.ptr(gamma), N.ptr(g_res),
           N.ptr(g_add), M, C, rps, N.ptr(dx), N.ptr(o1), N.ptr(b1_scale), N.ptr(o2), float(b2_mult), N.stream())
    return dx, o1, o2


def _salt(block, half):
    """Dropout stream of one Adapter (block, modality half): the seed is *seed_dev ^ salt."""
    return (0x9E3779B97F4A7C15 * (2 * block + half + 1)) & 0xFFFFFFFFFFFFFFFF


def _adapter_kernels_ok(M, Mh, C, R):
    return M == 2 * Mh and Mh % 16 == 0 and C % 32 == 0 and 1 <= R <= 128


def _adapter_weights(aparams, nb):
    """bf16 copies of a stage's Adapter parameters (aparams in adapter_params order: per block
    rgb then dte, each D_fc1.weight, D_fc1.bias, D_fc2.weight, D_fc2.bias) in one cast,
    grouped: W1 (2nb, R, C), W2 (2nb, C, R), B1 (2nb, R), B2 (2nb, C), index 2*block + half.
    `abf` lists the same storage in aparams order."""
    order = [8 * b + 4 * h + j for j in (0, 2, 1, 3) for b in range(nb) for h in (0, 1)]
    flat = torch.cat([aparams[k].detach().reshape(-1) for k in order]).to(_BF16)
    R, C = aparams[0].shape
    n_w, n = 2 * nb * R * C, 2 * nb
    W1 = flat[:n_w].view(n, R, C)
    W2 = flat[n_w:2 * n_w].view(n, C, R)
    B1 = flat[2 * n_w:2 * n_w + n * R].view(n, R)
    B2 = flat[2 * n_w + n * R:].view(n, C)
    abf = []
    for b in range(nb):
        for h in (0, 1):
            abf += [W1[2 * b + h], B1[2 * b + h], W2[2 * b + h], B2[2 * b + h]]
    return {"W1": W1, "W2": W2, "B1": B1, "B2": B2, "abf": abf, "R": R}


def _elem(name, *tensors, out_like, extra=()):
    out = torch.empty_like(out_like)
    N.call(name, *[N.ptr(t) for t in tensors], N.ptr(out), out.numel(), *extra, N.stream())
    return out


class SwinStageFn(torch.autograd.Function):
    """x (S, L, C) fp32 -> stage output (S, L, C) fp32, S = 2B (rgb samples first)."""

    @staticmethod
    def forward(ctx, x, seq, hw, *aparams):
        with torch.autocast("cuda", enabled=False):
            return SwinStageFn._forward(ctx, x, seq, hw, aparams)

    @staticmethod
    def _forward(ctx, x, seq, hw, aparams):
        S, L, C = x.shape
        H, W = hw
        M, Mh = S * L, (S // 2) * L
        blocks = list(seq.blocks)
        nb = len(blocks)
        dev = x.device
        x = x.contiguous().view(M, C)
        # the Adapter's F.dropout(p=0.1, training=self.training) (swin.py:496)
        p_drop = ADAPTER_DROPOUT if blocks[0].MLP_RGB_Adapter.training else 0.
        # dropout seed drawn on the device by torch's generator: graph-capturable, fresh per replay;
        # the stage's DropPath factors draw from the same seed (another salt)
        seed = torch.randint(0, 2 ** 62, (1,), device=dev, dtype=torch.int64) if p_drop > 0 else None
        dp = _droppath_scales(seq, S, dev, seed)
        # all adapter weights of the stage cast to bf16 in two launches (autocast casts each per
        # call), grouped as (2nb, R, C) D_fc1 weights, (2nb, C, R) D_fc2 weights and the biases
        aw = _adapter_weights(aparams, nb)
        abf = aw["abf"]
        R = aw["R"]
        fast = _adapter_kernels_ok(M, Mh, C, R)
        _, h1, _, mean1, rstd1 = _resln_fwd(x, M, C, L, norm=blocks[0].norm1)
        saved = []
        cur = x
        for i, blk in enumerate(blocks):
            w_msa = blk.attn.w_msa
            lq, lp = G.weights(w_msa.qkv), G.weights(w_msa.proj)
            l1, l2 = G.weights(blk.ffn.layers[0][0]), G.weights(blk.ffn.layers[1])
            qkv = G.linear(h1, lq).view(S, L, 3 * C)
            bias_f = None if w_msa.qkv.bias is None else w_msa.qkv.bias.detach()
            table_f = w_msa.relative_position_bias_table.detach()
            a, lse = ops.winattn_fwd(qkv, bias_f, table_f, None, H, W, w_msa.num_heads, blk.attn.shift_size,
                                     w_msa.scale, table_owner=w_msa.relative_position_bias_table)
            o = G.linear(a.view(M, C), lp)
            X1, h2, X1b, mean2, rstd2 = _resln_fwd(cur, M, C, L, add1=o, add1_scale=None if dp is None else dp[i, 0],
                                                  norm=blk.norm2, x_out=True, xb_out=True)
            u, g = G.ffn_up(h2, l1)
            f = G.linear(g, l2)
            d = torch.empty((M, C), device=dev, dtype=_BF16)
            if fast:
                # both Adapters in two launches: D_fc1 + ReLU + dropout, then D_fc2 (+ bias)
                W1, B1, W2, B2 = aw["W1"], aw["B1"], aw["W2"], aw["B2"]
                rs = torch.empty((M, R), device=dev, dtype=_BF16)
                N.call("irads_adapter_down", 0, N.ptr(X1b), N.ptr(W1[2 * i]), N.ptr(W1[2 * i + 1]),
                       N.ptr(B1[2 * i]), N.ptr(B1[2 * i + 1]), None, M, Mh, C, R, float(p_drop),
                       _salt(i, 0), _salt(i, 1), N.ptr(seed), N.ptr(rs), N.stream())
                N.call("irads_adapter_up", N.ptr(rs), N.ptr(W2[2 * i]), N.ptr(W2[2 * i + 1]), N.ptr(B2[2 * i]),
                       N.ptr(B2[2 * i + 1]), M, Mh, C, R, N.ptr(d), N.stream())
            else:
                rs = []
                for half in (0, 1):
                    wa1, ba1, wa2, ba2 = abf[8 * i + 4 * half: 8 * i + 4 * half + 4]
                    rows = slice(half * Mh, (half + 1) * Mh)
                    a1 = F.linear(X1b[rows], wa1, ba1)
                    r = torch.empty_like(a1)
                    N.call("irads_relu_dropout_fwd", N.ptr(a1), N.ptr(r), r.numel(), float(p_drop), _salt(i, half),
                           N.ptr(seed), N.stream())
                    torch.addmm(ba2, r, wa2.t(), out=d[rows])
                    rs.append(r)
            nxt = blocks[i + 1].norm1 if i + 1 < nb else None
            xn, h1, _, mean1n, rstd1n = _resln_fwd(X1, M, C, L, add1=f, add1_scale=None if dp is None else dp[i, 1],
                                                  add2=d, add2_mult=0.5, norm=nxt, x_out=True)
            saved.append((cur, mean1, rstd1, qkv, a, lse, X1, mean2, rstd2, u, X1b, rs))
            cur, mean1, rstd1 = xn, mean1n, rstd1n
        ctx.saved = saved
        ctx.cfg = (S, L, C, H, W, M, Mh, p_drop)
        ctx.seq, ctx.dp, ctx.aw, ctx.fast = seq, dp, aw, fast
        ctx.nparams = len(aparams)
        return cur.view(S, L, C)

    @staticmethod
    def backward(ctx, gy):
        with torch.autocast("cuda", enabled=False):
            return SwinStageFn._backward(ctx, gy)

    @staticmethod
    def _backward(ctx, gy):
        S, L, C, H, W, M, Mh, p_drop = ctx.cfg
        blocks = list(ctx.seq.blocks)
        nb = len(blocks)
        dp, aw, fast = ctx.dp, ctx.aw, ctx.fast
        abf, R = aw["abf"], aw["R"]
        if fast:  # operands of the input-gradient GEMMs: D_fc2.weightᵀ (R, C), D_fc1.weightᵀ (C, R)
            W2t = aw["W2"].transpose(1, 2).contiguous()
            W1t = aw["W1"].transpose(1, 2).contiguous()
        need = ctx.needs_input_grad[3:]
        gflat = torch.empty((sum(t.numel() for t in abf),), device=gy.device, dtype=torch.float32)
        gparts = [t.view(p.shape) for t, p in zip(torch.split(gflat, [t.numel() for t in abf]), abf)]
        g = gy.contiguous().view(M, C).float()
        _, df, dd = _resln_bwd(M, C, L, g_res=g, dx_out=False, b1=True, b2=True,
                               b1_scale=None if dp is None else dp[nb - 1, 1])
        for i in range(nb - 1, -1, -1):
            blk = blocks[i]
            x, mean1, rstd1, qkv, a, lse, X1, mean2, rstd2, u, X1b, rs = ctx.saved[i]
            w_msa = blk.attn.w_msa
            lq, lp = G.weights(w_msa.qkv), G.weights(w_msa.proj)
            l1, l2 = G.weights(blk.ffn.layers[0][0]), G.weights(blk.ffn.layers[1])
            # Adapters (per modality half): D_fc2, ReLU+dropout, D_fc1
            dX1b = torch.empty((M, C), device=g.device, dtype=_BF16)
            if fast:
                dA = torch.empty((M, R), device=g.device, dtype=_BF16)  # grad of the D_fc1 output
                N.call("irads_adapter_down", 1, N.ptr(dd), N.ptr(W2t[2 * i]), N.ptr(W2t[2 * i + 1]), None, None,
                       N.ptr(rs), M, Mh, C, R, float(p_drop), 0, 0, None, N.ptr(dA), N.stream())
                # the four weight gradients of the block (D_fc2, D_fc1 x rgb, dte) in one batched
                # split-K launch pair, all as (R, C) products: D_fc2's stored transposed
                probs = []
                for half in (0, 1):
                    k = 8 * i + 4 * half
                    gwa1, gba1, gwa2, gba2 = gparts[k: k + 4]
                    rows = slice(half * Mh, (half + 1) * Mh)
                    probs.append((rs[rows], dd[rows], gwa2, None, gba2, True))
                    probs.append((dA[rows], X1b[rows], gwa1, gba1, None, False))
                if R % 8:
                    # Swin-L (C = 192: R = 12): the split-K kernel takes 16-B rows (R % 8 == 0);
                    # these four skinny products go to hipBLASLt in bf16 with fp32 column sums
                    # (autocast's own rounding of a bf16 Linear's weight gradient)
                    for A_, B_, D_, sa_, sb_, tr_ in probs:
                        if tr_:
                            D_.copy_(torch.mm(B_.t(), A_))
                        else:
                            D_.copy_(torch.mm(A_.t(), B_))
                        if sa_ is not None:
                            torch.sum(A_, 0, dtype=torch.float32, out=sa_)
                        if sb_ is not None:
                            torch.sum(B_, 0, dtype=torch.float32, out=sb_)
                elif _UNBATCHED:
                    for A_, B_, D_, sa_, sb_, tr_ in probs:
                        if tr_:
                            ops.wgrad(B_, A_, D_, colsum_a=sb_)
                        else:
                            ops.wgrad(A_, B_, D_, colsum_a=sa_)
                else:
                    ops.wgrad_batched(probs)
                N.call("irads_adapter_up", N.ptr(dA), N.ptr(W1t[2 * i]), N.ptr(W1t[2 * i + 1]), None, None, M, Mh,
                       C, R, N.ptr(dX1b), N.stream())
            for half in (() if fast else (0, 1)):
                k = 8 * i + 4 * half
                wa1, _, wa2, _ = abf[k: k + 4]
                gwa1, gba1, gwa2, gba2 = gparts[k: k + 4]
                rows = slice(half * Mh, (half + 1) * Mh)
                ddh, r = dd[rows], rs[half]
                ops.wgrad(ddh, r, gwa2, colsum_a=gba2)  # dW, db of D_fc2 in fp32 (split-K)
                dr = torch.mm(ddh, wa2)
                da1 = torch.empty_like(dr)
                N.call("irads_relu_dropout_bwd", N.ptr(r), N.ptr(dr), N.ptr(da1), da1.numel(), float(p_drop),
                       N.stream())
                ops.wgrad(da1, X1b[rows], gwa1, colsum_a=gba1)
                torch.mm(da1, wa1, out=dX1b[rows])
            # FFN
            du = G.ffn_down_dgrad_gelu(df, l2, u)
            dh2 = G.dgrad(du, l1)
            dX1, do, _ = _resln_bwd(M, C, L, dy=dh2, x=X1, mean=mean2, rstd=rstd2, norm=blk.norm2, g_res=g,
                                    g_add=dX1b, b1=True, b1_scale=None if dp is None else dp[i, 0])
            # attention
            da = G.dgrad(do, lp).view(S, L, C)
            bias_f = None if w_msa.qkv.bias is None else w_msa.qkv.bias.detach()
            gqkv, _, _ = ops.winattn_bwd(qkv, bias_f, w_msa.relative_position_bias_table.detach(), None, H, W,
                                         w_msa.num_heads, blk.attn.shift_size, w_msa.scale, a, lse, da,
                                         table_owner=w_msa.relative_position_bias_table)
            dh1 = G.dgrad(gqkv.view(M, 3 * C), lq)
            if i > 0:
                g, df, dd = _resln_bwd(M, C, L, dy=dh1, x=x, mean=mean1, rstd=rstd1, norm=blk.norm1, g_res=dX1,
                                       b1=True, b2=True, b1_scale=None if dp is None else dp[i - 1, 1])
            else:
                g, _, _ = _resln_bwd(M, C, L, dy=dh1, x=x, mean=mean1, rstd=rstd1, norm=blk.norm1, g_res=dX1)
            ctx.saved[i] = None
        grads = gflat
        out = []
        off = 0
        for j, t in enumerate(abf):
            n = t.numel()
            out.append(grads[off: off + n].view(t.shape) if need[j] else None)
            off += n
        return (g.view(S, L, C) if ctx.needs_input_grad[0] else None, None, None, *out)


def stage_forward(seq, x, hw):
    return SwinStageFn.apply(x, seq, tuple(hw), *adapter_params(seq))
