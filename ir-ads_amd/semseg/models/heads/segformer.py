"""SegFormer decode head (reference semseg/models/heads/segformer.py:7-48)."""
from typing import Tuple

import torch
from torch import nn, Tensor
from torch.nn import functional as F

from irads import ops
from semseg.models.layers.common import TrainLinear


class MLP(nn.Module):
    def __init__(self, dim, embed_dim):
        super().__init__()
        self.proj = TrainLinear(dim, embed_dim)

    def forward(self, x: Tensor) -> Tensor:
        return self.proj(x.flatten(2).transpose(1, 2))


class _ComposeFn(torch.autograd.Function):
    """The branch weights of SegFormerHead.forward: A_i = W_i M_i and c_i = W_i b_i, W_i the column
    block of linear_fuse's weight that branch i's MLP feeds (blocks in [c4 | c3 | c2 | c1] order),
    all in fp32 in one autograd node.  As separate autocast ops each branch cost a weight cast each
    way, a bf16 product, a slice backward (zero fill + copy) and a gradient add on the shared fuse
    weight; here the fuse weight's gradient is the concatenation of its blocks', written once."""

    @staticmethod
    def forward(ctx, Wf, E, *mb):
        n = len(mb) // 2
        outs = []
        for i in range(n):
            Wi = Wf[:, (n - 1 - i) * E:(n - i) * E]
            outs += [Wi @ mb[2 * i], Wi @ mb[2 * i + 1]]
        ctx.save_for_backward(Wf, *mb)
        ctx.E = E
        return tuple(outs)

    @staticmethod
    def backward(ctx, *g):
        Wf, *mb = ctx.saved_tensors
        E, n = ctx.E, len(mb) // 2
        blocks, dmb = [None] * n, []
        for i in range(n):
            Wi = Wf[:, (n - 1 - i) * E:(n - i) * E]
            M, b = mb[2 * i], mb[2 * i + 1]
            gA = g[2 * i] if g[2 * i] is not None else torch.zeros((E, M.shape[1]), device=Wf.device)
            gc = g[2 * i + 1] if g[2 * i + 1] is not None else torch.zeros((E,), device=Wf.device)
            blocks[n - 1 - i] = torch.addr(gA @ M.t(), gc, b)
            dmb += [Wi.t() @ gA, Wi.t() @ gc]
        dWf = torch.cat(blocks, dim=1) if ctx.needs_input_grad[0] else None
        return (dWf, None, *dmb)


class ConvModule(nn.Module):
    def __init__(self, c1, c2):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, 1, bias=False)
        self.bn = nn.BatchNorm2d(c2)  # per-GPU BN, as the reference (no SyncBN)
        self.activate = nn.ReLU(True)

    def forward(self, x: Tensor) -> Tensor:
        return self.activate(self.bn(self.conv(x)))


class SegFormerHead(nn.Module):
    def __init__(self, dims: list, embed_dim: int = 256, num_classes: int = 19):
        super().__init__()
        for i, dim in enumerate(dims):
            self.add_module(f"linear_c{i + 1}", MLP(dim, embed_dim))
        self.linear_fuse = ConvModule(embed_dim * 4, embed_dim)
        self.linear_pred = nn.Conv2d(embed_dim, num_classes, 1)
        self.dropout = nn.Dropout2d(0.1)
        self.keep_feature = False  # CMNeXt's SB hook reads the fused E-dim feature (tokens) of the last call
        self.feature, self.feature_hw = None, None

    def forward(self, features: Tuple[Tensor, Tensor, Tensor, Tensor]) -> Tensor:
        """Reference (segformer.py:37-48):
            c_i = resize(MLP_i(f_i))  (i = 2..4; c_1 = MLP_1(f_1));  seg = BN-ReLU(W · cat[c4, c3, c2, c1])
        Computed here as the algebraically identical
            seg = BN-ReLU(z_1 + Σ_{i>1} resize(z_i)),  z_i = (W_i M_i) f_i + W_i b_i
        where W_i is linear_fuse's column block for branch i and (M_i, b_i) the MLP: resize and a
        1x1 projection commute, so each branch is ONE GEMM at its own resolution (1/4 ... 1/32)
        into E channels, and the 4E-channel concatenation at 1/4 resolution never exists.  The
        composed weights W_i M_i are formed each call in fp32 (E x E x dim_i flops, _ComposeFn), so
        gradients reach linear_fuse.conv.weight and every MLP through autograd.  Parameters and
        keys unchanged."""
        B, _, H, W = features[0].shape
        E = self.linear_fuse.conv.weight.shape[0]
        Wf = self.linear_fuse.conv.weight.view(E, -1)  # column blocks: [c4 | c3 | c2 | c1]
        n = len(features)
        mlps = [getattr(self, f"linear_c{i + 1}").proj for i in range(n)]
        if mlps[0].bias is not None and Wf.dtype == torch.float32:
            # the branch weights (E, dim_i) and biases in fp32, one node (ops.linear casts A to bf16)
            with torch.autocast("cuda", enabled=False):
                Ac = _ComposeFn.apply(Wf, E, *[t for m in mlps for t in (m.weight, m.bias)])
        else:
            Ac = []
            for i, mlp in enumerate(mlps):
                Wi = Wf[:, (n - 1 - i) * E:(n - i) * E]
                Ac += [Wi @ mlp.weight, None if mlp.bias is None else Wi @ mlp.bias]
        zs = []
        for i, f in enumerate(features):
            z = ops.linear(f.flatten(2).transpose(1, 2), Ac[2 * i], Ac[2 * i + 1])  # (B, h*w, E)
            zs.append(z.transpose(1, 2).reshape(B, E, *f.shape[-2:]))  # channels-last (B, E, h, w) view
        seg = ops.upsample_sum(zs[0], zs[1:])
        if self.training and seg.dtype == torch.bfloat16 and seg.is_cuda:
            tok = seg.permute(0, 2, 3, 1).reshape(B, H * W, E)  # channels-last memory: a view
            if ops.bnact_ok(tok, self.linear_fuse.bn):
                # BN (batch statistics) + ReLU + Dropout2d in one pass each way (csrc/bnact.hip),
                # then linear_pred as a token-major Linear: logits stay channels-last
                z = ops.bn_relu_dropout2d(tok, self.linear_fuse.bn, self.dropout.p)
                if self.keep_feature:
                    self.feature, self.feature_hw = z, (H, W)
                pred = self.linear_pred
                out = ops.linear(z, pred.weight.view(pred.out_channels, E), pred.bias)
                return out.view(B, H, W, -1).permute(0, 3, 1, 2)
        seg = self.linear_fuse.activate(self.linear_fuse.bn(seg))
        if self.keep_feature:
            self.feature, self.feature_hw = seg.permute(0, 2, 3, 1).reshape(B, H * W, E), (H, W)
        return self.linear_pred(self.dropout(seg))
