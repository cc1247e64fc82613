"""Patch embedding / merging of the Swin backbone (reference semseg/models/backbones/embed.py).

Conv and Linear go to MIOpen / hipBLASLt.  PatchMerging's non-overlapping unfold is one
permute copy, and its LayerNorm writes the bf16 operand of `reduction` directly under AMP
(ops.layer_norm_bf16).  State-dict keys as the reference (``projection``, ``norm``, ``reduction``).
"""
import math
from typing import Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F
from irads import ops

from ..layers.common import Linear


def _pair(x):
    return tuple(x) if isinstance(x, (tuple, list)) else (x, x)


class AdaptivePadding(nn.Module):
    """Pad so the filter covers the input: 'corner' pads bottom/right, 'same' both sides."""

    def __init__(self, kernel_size=1, stride=1, dilation=1, padding='corner'):
        super().__init__()
        assert padding in ('same', 'corner')
        self.padding = padding
        self.kernel_size, self.stride, self.dilation = _pair(kernel_size), _pair(stride), _pair(dilation)

    def get_pad_shape(self, input_shape):
        pads = []
        for size, k, s, d in zip(input_shape, self.kernel_size, self.stride, self.dilation):
            out = math.ceil(size / s)
            pads.append(max((out - 1) * s + (k - 1) * d + 1 - size, 0))
        return tuple(pads)

    def forward(self, x):
        ph, pw = self.get_pad_shape(x.size()[-2:])
        if ph > 0 or pw > 0:
            if self.padding == 'corner':
                x = F.pad(x, [0, pw, 0, ph])
            else:
                x = F.pad(x, [pw // 2, pw - pw // 2, ph // 2, ph - ph // 2])
        return x


class PatchEmbed(nn.Module):
    """Conv patch embedding + LayerNorm; returns (B, h*w, C) and (h, w)."""

    def __init__(self, in_channels=3, embed_dims=768, conv_type='Conv2d', kernel_size=16, stride=None,
                 padding='corner', dilation=1, bias=True, norm_cfg=None, input_size=None, init_cfg=None):
        super().__init__()
        assert conv_type == 'Conv2d'
        self.embed_dims = embed_dims
        stride = kernel_size if stride is None else stride
        kernel_size, stride, dilation = _pair(kernel_size), _pair(stride), _pair(dilation)
        if isinstance(padding, str):
            self.adap_padding = AdaptivePadding(kernel_size, stride, dilation, padding)
            padding = 0
        else:
            self.adap_padding = None
        padding = _pair(padding)
        self.projection = nn.Conv2d(in_channels, embed_dims, kernel_size, stride, padding, dilation, bias=bias)
        self.norm = nn.LayerNorm(embed_dims) if norm_cfg is not None else None
        self.init_input_size = self.init_out_size = None
        if input_size:
            input_size = _pair(input_size)
            self.init_input_size = input_size
            if self.adap_padding:
                ph, pw = self.adap_padding.get_pad_shape(input_size)
                input_size = (input_size[0] + ph, input_size[1] + pw)
            self.init_out_size = tuple(
                (input_size[i] + 2 * padding[i] - dilation[i] * (kernel_size[i] - 1) - 1) // stride[i] + 1
                for i in range(2))

    def _patchify_ok(self, x):
        c = self.projection
        return (x.is_cuda and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16
                and c.kernel_size == c.stride and c.padding == (0, 0) and c.dilation == (1, 1) and c.groups == 1
                and x.shape[2] % c.kernel_size[0] == 0 and x.shape[3] % c.kernel_size[1] == 0)

    def forward(self, x):
        if self.adap_padding:
            x = self.adap_padding(x)
        if self._patchify_ok(x):
            # non-overlapping patches: the convolution is a GEMM over the (c, ky, kx) patch
            # vectors, gathered and cast in one copy; its output is token-major, so the
            # LayerNorm reads contiguous rows (no NCHW -> (B, HW, C) transpose)
            c = self.projection
            B, Cin, H, W = x.shape
            kh, kw = c.kernel_size
            h, w = H // kh, W // kw
            tok = torch.empty((B, h * w, Cin * kh * kw), device=x.device, dtype=torch.bfloat16)
            tok.view(B, h, w, Cin, kh, kw).copy_(x.view(B, Cin, h, kh, w, kw).permute(0, 2, 4, 1, 3, 5))
            x = ops.linear(tok, c.weight.view(c.out_channels, -1), c.bias)
            out_size = (h, w)
        else:
            x = self.projection(x)
            out_size = (x.shape[2], x.shape[3])
            x = x.flatten(2).transpose(1, 2)
        if self.norm is not None:
            x = ops.layer_norm_from_bf16(x, self.norm)  # = self.norm(x) under autocast, one kernel
        return x, out_size


class PatchMerging(nn.Module):
    """2x2 unfold -> LayerNorm(4C) -> Linear(4C, out, bias=False)."""

    def __init__(self, in_channels, out_channels, kernel_size=2, stride=None, padding='corner', dilation=1,
                 bias=False, norm_cfg=dict(type='LN'), init_cfg=None):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        stride = stride if stride else kernel_size
        kernel_size, stride, dilation = _pair(kernel_size), _pair(stride), _pair(dilation)
        if isinstance(padding, str):
            self.adap_padding = AdaptivePadding(kernel_size, stride, dilation, padding)
            padding = 0
        else:
            self.adap_padding = None
        padding = _pair(padding)
        self.sampler = nn.Unfold(kernel_size=kernel_size, dilation=dilation, padding=padding, stride=stride)
        sample_dim = kernel_size[0] * kernel_size[1] * in_channels
        self.norm = nn.LayerNorm(sample_dim) if norm_cfg is not None else None
        self.reduction = Linear(sample_dim, out_channels, bias=bias)

    def gather_shape_ok(self, H, W):
        """The 2x2 / stride-2 unfold with a norm and no padding: the gather-norm kernels apply."""
        s = self.sampler
        no_pad = not self.adap_padding or tuple(self.adap_padding.get_pad_shape((H, W))) == (0, 0)
        return (self.norm is not None and no_pad and s.kernel_size == s.stride == (2, 2) and s.padding == (0, 0)
                and s.dilation == (1, 1))

    def forward(self, x, input_size, sub_mode=None):
        B, L, C = x.shape
        assert isinstance(input_size, Sequence), f'Expect input_size is `Sequence` but get {input_size}'
        H, W = input_size
        assert L == H * W, 'input feature has wrong size'
        s = self.sampler
        if self.gather_shape_ok(H, W) and ops.patch_merge_norm_ok(x, H, W, self.norm):
            # the 2x2 unfold as the LayerNorm's gather (one HIP pass each way, no permuted copy)
            with torch.autocast("cuda", enabled=False):
                xm = ops.PatchMergeNormFn.apply(x, H, W, self.norm.weight, self.norm.bias, self.norm.eps)
            return self.reduction(xm), (H // 2, W // 2)
        x = x.view(B, H, W, C).permute([0, 3, 1, 2])
        if self.adap_padding:
            x = self.adap_padding(x)
            H, W = x.shape[-2:]
        s = self.sampler
        out_hw = tuple((size + 2 * s.padding[i] - s.dilation[i] * (s.kernel_size[i] - 1) - 1) // s.stride[i] + 1
                       for i, size in enumerate((H, W)))
        if (s.kernel_size == s.stride and s.padding == (0, 0) and s.dilation == (1, 1)
                and H % s.kernel_size[0] == 0 and W % s.kernel_size[1] == 0):
            # non-overlapping 2x2 unfold == a reshape: channel index c*kh*kw + i*kw + j, as
            # nn.Unfold orders it, gathered by one permute copy (no im2col / col2im)
            kh, kw = s.kernel_size
            x = x.reshape(B, C, H // kh, kh, W // kw, kw).permute(0, 2, 4, 1, 3, 5).reshape(B, -1, C * kh * kw)
        else:
            x = self.sampler(x).transpose(1, 2)
        x = ops.layer_norm_bf16(x, self.norm) if self.norm else x  # the bf16 operand of `reduction`
        return self.reduction(x), out_hw
