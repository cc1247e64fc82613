"""CPU restatement (oracle) of IR-ADS's multimodal-segmentation hot path, in PyTorch fp32.

TEST INFRASTRUCTURE ONLY.  Imported exclusively by tests/, __graft_entry__.smoke() and
bench.py's ``cpu_baseline`` leg, and only as the checker / the timed CPU baseline —
never by the product package (``ir-ads_amd/``), which fails loudly without its HIP
library.  Pinned by tests/test_oracle_golden.py against the golden fixtures produced
from the reference itself (oracle/gen_golden.py).

Module names, constructor arguments and state-dict keys follow the reference so a
reference (or product) state dict loads unchanged.  Each class cites the reference
file:line it restates.  mmcv/mmengine/timm building blocks are restated per
SURVEY.md Appendix B (their arithmetic is plain PyTorch: parity unpinned beyond that).
"""
import math

import numpy as np
from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F


# ----------------------------------------------------------------- building blocks
class DropPath(nn.Module):
    """timm DropPath as mmcv build_dropout(DropPath) constructs it."""

    def __init__(self, drop_prob=0.0):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x):
        if self.drop_prob == 0.0 or not self.training:
            return x
        kp = 1 - self.drop_prob
        r = (kp + torch.rand((x.shape[0],) + (1,) * (x.ndim - 1), dtype=x.dtype, device=x.device)).floor_()
        return x.div(kp) * r


class FFN(nn.Module):
    """mmcv FFN(num_fcs=2, GELU, add_identity=True) — keys layers.0.0 / layers.1."""

    def __init__(self, embed_dims, feedforward_channels, ffn_drop=0.0, drop_path=0.0):
        super().__init__()
        self.layers = nn.Sequential(
            nn.Sequential(nn.Linear(embed_dims, feedforward_channels), nn.GELU(), nn.Dropout(ffn_drop)),
            nn.Linear(feedforward_channels, embed_dims), nn.Dropout(ffn_drop))
        self.dropout_layer = DropPath(drop_path)

    def forward(self, x, identity=None):
        return (x if identity is None else identity) + self.dropout_layer(self.layers(x))


# ----------------------------------------------------------------- Swin window attention
class WindowMSA(nn.Module):
    """swin.py:23-125."""

    def __init__(self, embed_dims, num_heads, window_size, qkv_bias=True, qk_scale=None,
                 attn_drop_rate=0.0, proj_drop_rate=0.0, init_cfg=None):
        super().__init__()
        self.embed_dims, self.window_size, self.num_heads = embed_dims, window_size, num_heads
        self.scale = qk_scale or (embed_dims // num_heads) ** -0.5
        Wh, Ww = window_size
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * Wh - 1) * (2 * Ww - 1), num_heads))
        # idx[i, j] = (hi - hj + Wh-1) * (2Ww-1) + (wi - wj + Ww-1)   (swin.py:64-69)
        hh, ww = torch.meshgrid(torch.arange(Wh), torch.arange(Ww), indexing="ij")
        hh, ww = hh.flatten(), ww.flatten()
        idx = (hh[:, None] - hh[None, :] + Wh - 1) * (2 * Ww - 1) + (ww[:, None] - ww[None, :] + Ww - 1)
        self.register_buffer("relative_position_index", idx.contiguous())
        self.qkv = nn.Linear(embed_dims, embed_dims * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop_rate)
        self.proj = nn.Linear(embed_dims, embed_dims)
        self.proj_drop = nn.Dropout(proj_drop_rate)

    def forward(self, x, mask=None):
        B, N, C = x.shape
        qkv = self.qkv(x).reshape(B, N, 3, self.num_heads, C // self.num_heads).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0] * self.scale, qkv[1], qkv[2]
        attn = q @ k.transpose(-2, -1)
        bias = self.relative_position_bias_table[self.relative_position_index.view(-1)].view(N, N, -1)
        attn = attn + bias.permute(2, 0, 1).unsqueeze(0)
        if mask is not None:
            nW = mask.shape[0]
            attn = (attn.view(B // nW, nW, self.num_heads, N, N) + mask[None, :, None]).view(-1, self.num_heads, N, N)
        attn = self.attn_drop(attn.softmax(-1))
        return self.proj_drop(self.proj((attn @ v).transpose(1, 2).reshape(B, N, C)))


def shift_mask(Hp, Wp, ws, shift, device=None):
    """Region mask of swin.py:199-220: 0 inside a region, -100 across regions."""
    img = torch.zeros((Hp, Wp), device=device)
    cnt = 0
    for h in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
        for w in (slice(0, -ws), slice(-ws, -shift), slice(-shift, None)):
            img[h, w] = cnt
            cnt += 1
    win = img.view(Hp // ws, ws, Wp // ws, ws).permute(0, 2, 1, 3).reshape(-1, ws * ws)
    m = win[:, None, :] - win[:, :, None]
    return m.masked_fill(m != 0, -100.0).masked_fill(m == 0, 0.0)


class ShiftWindowMSA(nn.Module):
    """swin.py:128-285."""

    def __init__(self, embed_dims, num_heads, window_size, shift_size=0, qkv_bias=True, qk_scale=None,
                 attn_drop_rate=0, proj_drop_rate=0, drop_path=0.0, init_cfg=None):
        super().__init__()
        self.window_size, self.shift_size = window_size, shift_size
        self.w_msa = WindowMSA(embed_dims, num_heads, (window_size, window_size), qkv_bias, qk_scale,
                               attn_drop_rate, proj_drop_rate)
        self.drop = DropPath(drop_path)

    def forward(self, query, hw_shape):
        B, L, C = query.shape
        H, W = hw_shape
        ws, s = self.window_size, self.shift_size
        x = F.pad(query.view(B, H, W, C), (0, 0, 0, (ws - W % ws) % ws, 0, (ws - H % ws) % ws))
        Hp, Wp = x.shape[1], x.shape[2]
        mask = None
        if s > 0:
            x = torch.roll(x, (-s, -s), (1, 2))
            mask = shift_mask(Hp, Wp, ws, s, x.device)
        win = x.view(B, Hp // ws, ws, Wp // ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(-1, ws * ws, C)
        o = self.w_msa(win, mask=mask)
        o = o.view(B, Hp // ws, Wp // ws, ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B, Hp, Wp, C)
        if s > 0:
            o = torch.roll(o, (s, s), (1, 2))
        return self.drop(o[:, :H, :W, :].reshape(B, H * W, C))


class Adapter(nn.Module):
    """swin.py:472-502 (skip_connect=False, prompt_add=False as SwinBlockAdapter builds it)."""

    def __init__(self, D_features, mlp_ratio=0.0625, act_layer=nn.ReLU, skip_connect=True):
        super().__init__()
        self.skip_connect = skip_connect
        self.act = act_layer()
        hid = int(D_features * mlp_ratio)
        self.D_fc1 = nn.Linear(D_features, hid)
        self.D_fc2 = nn.Linear(hid, D_features)

    def forward(self, x):
        xs = self.D_fc2(F.dropout(self.act(self.D_fc1(x)), p=0.1, training=self.training))
        return x + xs if self.skip_connect else xs


class SwinBlockAdapter(nn.Module):
    """swin.py:505-610."""

    def __init__(self, embed_dims, num_heads, feedforward_channels, window_size=7, shift=False,
                 drop_path_rate=0.0, adapter_ratio=0.0625, with_cp=False):
        super().__init__()
        self.with_cp = with_cp
        self.norm1 = nn.LayerNorm(embed_dims)
        self.attn = ShiftWindowMSA(embed_dims, num_heads, window_size, window_size // 2 if shift else 0,
                                   drop_path=drop_path_rate)
        self.norm2 = nn.LayerNorm(embed_dims)
        self.ffn = FFN(embed_dims, feedforward_channels, drop_path=drop_path_rate)
        self.MLP_RGB_Adapter = Adapter(embed_dims, adapter_ratio, skip_connect=False)
        self.MLP_DTE_Adapter = Adapter(embed_dims, adapter_ratio, skip_connect=False)
        self.scale = 0.5

    def forward(self, x, hw_shape, sub_mode):
        x = self.attn(self.norm1(x), hw_shape) + x
        ad = self.MLP_RGB_Adapter if sub_mode == "rgb" else self.MLP_DTE_Adapter
        a = self.scale * ad(x)
        return self.ffn(self.norm2(x), identity=x) + a


class PatchEmbed(nn.Module):
    """embed.py PatchEmbed with padding='corner', LN."""

    def __init__(self, in_channels=3, embed_dims=128, kernel_size=4, stride=4):
        super().__init__()
        self.k, self.s = kernel_size, stride
        self.projection = nn.Conv2d(in_channels, embed_dims, kernel_size, stride)
        self.norm = nn.LayerNorm(embed_dims)

    def forward(self, x):
        H, W = x.shape[-2:]
        ph = max((math.ceil(H / self.s) - 1) * self.s + self.k - H, 0)
        pw = max((math.ceil(W / self.s) - 1) * self.s + self.k - W, 0)
        if ph or pw:
            x = F.pad(x, [0, pw, 0, ph])
        x = self.projection(x)
        hw = (x.shape[2], x.shape[3])
        return self.norm(x.flatten(2).transpose(1, 2)), hw


class PatchMerging(nn.Module):
    """embed.py:207-329 (nn.Unfold 2x2 -> LN(4C) -> Linear(4C, 2C, bias=False))."""

    def __init__(self, in_channels, out_channels, stride=2):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.sampler = nn.Unfold(kernel_size=2, stride=stride)
        self.norm = nn.LayerNorm(4 * in_channels)
        self.reduction = nn.Linear(4 * in_channels, out_channels, bias=False)

    def forward(self, x, hw, sub_mode=None):
        B, L, C = x.shape
        H, W = hw
        x = x.view(B, H, W, C).permute(0, 3, 1, 2)
        if H % 2 or W % 2:
            x = F.pad(x, [0, W % 2, 0, H % 2])
            H, W = x.shape[-2:]
        x = self.sampler(x).transpose(1, 2)
        return self.reduction(self.norm(x)), (H // 2, W // 2)


class SwinBlockSequence(nn.Module):
    """swin.py:613-697."""

    def __init__(self, embed_dims, num_heads, feedforward_channels, depth, window_size=12,
                 drop_path_rate=0.0, downsample=None, adapter_ratio=0.0625, with_cp=False):
        super().__init__()
        dpr = drop_path_rate if isinstance(drop_path_rate, list) else [drop_path_rate] * depth
        self.blocks = nn.ModuleList([
            SwinBlockAdapter(embed_dims, num_heads, feedforward_channels, window_size, i % 2 == 1, dpr[i],
                             adapter_ratio, with_cp) for i in range(depth)])
        self.downsample = downsample

    def forward(self, x, hw_shape, sub_mode):
        for b in self.blocks:
            x = b(x, hw_shape, sub_mode)
        if self.downsample:
            xd, hwd = self.downsample(x, hw_shape, sub_mode)
            return xd, hwd, x, hw_shape
        return x, hw_shape, x, hw_shape


# ----------------------------------------------------------------- fusion blocks
class LayerNormProxy(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.norm = nn.LayerNorm(dim)

    def forward(self, x):
        return self.norm(x.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)


class conv_bn_relu(nn.Module):  # noqa: N801  (reference name, swin.py:713-723)
    def __init__(self, cin, cout):
        super().__init__()
        self.conv = nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1), nn.BatchNorm2d(cout), nn.GELU())

    def forward(self, x):
        return self.conv(x)


class DAttentionMM(nn.Module):
    """swin.py:726-1025 (default config: use_pe, no dwc_pe/fixed_pe/log_cpb, offset_range_factor=-1)."""

    def __init__(self, dims, q_size=(60, 80), kv_size=56, n_heads=2, n_groups=1, attn_drop=0, proj_drop=0,
                 stride=8, ksize=9, dpr=0, level=None):
        super().__init__()
        self.n_head_channels = dims // n_heads
        self.scale = self.n_head_channels ** -0.5
        self.n_heads, self.n_groups = n_heads, n_groups
        self.q_h, self.q_w = q_size
        self.nc = dims
        self.n_group_channels = dims // n_groups
        self.n_group_heads = n_heads // n_groups
        self.stride = stride
        pad = ksize // 2 if ksize != stride else 0
        gc = self.n_group_channels

        def off():
            return nn.Sequential(nn.Conv2d(gc, gc, ksize, stride, pad, groups=gc), LayerNormProxy(gc), nn.GELU(),
                                 nn.Conv2d(gc, 2, 1, 1, 0, bias=False))
        self.conv_offset_x = off()
        self.conv_offset_y = off()
        self.fuse_q = conv_bn_relu(2 * dims, dims)
        self.proj_q = nn.Conv2d(dims, dims, 1)
        self.get_sample_weight = nn.Sequential(nn.Conv2d(dims, dims, 1), nn.ReLU(), nn.Conv2d(dims, 2, 1))
        self.proj_k = nn.Conv2d(dims, dims, 1)
        self.proj_v = nn.Conv2d(dims, dims, 1)
        self.proj_out = nn.Conv2d(dims, dims, 1)
        self.deform_weight = nn.Parameter([1e-3, 1e-3, 1e-3, 1][level] * torch.ones(dims))
        self.identity_weight = nn.Parameter(torch.ones(dims))
        self.rpe_table = nn.Parameter(torch.zeros(n_heads, self.q_h * 2 - 1, self.q_w * 2 - 1))

    def forward(self, x, y):
        B, C, H, W = x.shape
        g, gc, nh, hc = self.n_groups, self.n_group_channels, self.n_heads, self.n_head_channels
        xy = self.fuse_q(torch.cat([x, y], 1))
        q = self.proj_q(xy)
        xo = self.conv_offset_x(x.reshape(B * g, gc, H, W)).permute(0, 2, 3, 1)
        yo = self.conv_offset_y(y.reshape(B * g, gc, H, W)).permute(0, 2, 3, 1)
        Hk, Wk = xo.shape[1], xo.shape[2]
        n = Hk * Wk
        ry, rx = torch.meshgrid(torch.linspace(0.5, Hk - 0.5, Hk), torch.linspace(0.5, Wk - 0.5, Wk), indexing="ij")
        ref = torch.stack((ry, rx), -1)
        ref[..., 1].div_(Wk - 1.0).mul_(2.0).sub_(1.0)
        ref[..., 0].div_(Hk - 1.0).mul_(2.0).sub_(1.0)
        ref = ref.to(x.dtype)[None]
        pos_x = (xo + ref).clamp(-1.0, 1.0)
        pos_y = (yo + ref).clamp(-1.0, 1.0)

        def samp(t, pos):
            return F.grid_sample(t.reshape(B * g, gc, H, W), pos[..., (1, 0)], mode="bilinear",
                                 align_corners=True).reshape(B, C, 1, n)
        xs = torch.cat([samp(x, pos_x), samp(x, pos_y)], -1)
        ys = torch.cat([samp(y, pos_x), samp(y, pos_y)], -1)
        qs = torch.cat([samp(q, pos_x), samp(q, pos_y)], -1)
        w = self.get_sample_weight(qs).softmax(1).squeeze(2).unsqueeze(1)
        sampled = (w * torch.cat([xs, ys], -2)).sum(-2, keepdim=True)
        qh = q.reshape(B * nh, hc, H * W)
        k = self.proj_k(sampled).reshape(B * nh, hc, 2 * n)
        v = self.proj_v(sampled).reshape(B * nh, hc, 2 * n)
        attn = torch.einsum("bcm,bcn->bmn", qh, k).mul(self.scale)
        qy, qx = torch.meshgrid(torch.arange(H, dtype=x.dtype), torch.arange(W, dtype=x.dtype), indexing="ij")
        qg = torch.stack((qy, qx), -1)
        qg[..., 1].div_(W - 1.0).mul_(2.0).sub_(1.0)
        qg[..., 0].div_(H - 1.0).mul_(2.0).sub_(1.0)
        qg = qg.reshape(1, H * W, 1, 2)
        table = self.rpe_table[None].expand(B, -1, -1, -1).reshape(B * g, self.n_group_heads,
                                                                  2 * self.q_h - 1, 2 * self.q_w - 1)
        bias = []
        for pos in (pos_x, pos_y):
            disp = (qg - pos.reshape(B * g, 1, n, 2)).mul(0.5)
            bias.append(F.grid_sample(table, disp[..., (1, 0)], mode="bilinear", align_corners=True))
        attn = attn + torch.cat(bias, -1).reshape(B * nh, H * W, 2 * n)
        out = torch.einsum("bmn,bcn->bcm", attn.softmax(2), v).reshape(B, C, H, W)
        out = self.proj_out(out)
        return self.deform_weight[None, :, None, None] * out + self.identity_weight[None, :, None, None] * xy


class MPGBlock(nn.Module):
    """swin.py:1045-1068."""

    def __init__(self, dim, ratio):
        super().__init__()
        d = int(dim * ratio)
        self.D_fc1, self.D_fc2 = nn.Linear(dim, d), nn.Linear(dim, d)
        self.P_fc2, self.U_fc1 = nn.Linear(2 * d, d), nn.Linear(d, dim)
        self.act = nn.GELU()
        self.tfts_gamma_rgb = nn.Parameter(torch.ones(dim))
        self.tfts_beta_rgb = nn.Parameter(torch.zeros(dim))
        self.tfts_gamma_dte = nn.Parameter(torch.ones(dim))
        self.tfts_beta_dte = nn.Parameter(torch.zeros(dim))

    def forward(self, x_rgb, x_dte, H, W):
        x = self.U_fc1(self.P_fc2(torch.cat([self.D_fc1(x_rgb), self.D_fc2(x_dte)], -1)))
        return x + (x * self.tfts_gamma_rgb + self.tfts_beta_rgb), x + (x * self.tfts_gamma_dte + self.tfts_beta_dte)


class DeformMPGBlock(nn.Module):
    """swin.py:1071-1091."""

    def __init__(self, dims, stride, n_groups, n_heads, dpr, level, ratio):
        super().__init__()
        d = int(dims * ratio)
        self.D_fc1, self.D_fc2, self.U_fc1 = nn.Linear(dims, d), nn.Linear(dims, d), nn.Linear(d, dims)
        self.act = nn.GELU()
        self.deform_atten = DAttentionMM(d, stride=stride, n_groups=n_groups, n_heads=n_heads, dpr=dpr, level=level)

    def forward(self, x_rgb, x_dte, H, W, level):
        xr, xd = self.D_fc1(x_rgb), self.D_fc2(x_dte)
        B, N, c = xr.shape
        f = self.deform_atten(xr.reshape(B, H, W, c).permute(0, 3, 1, 2), xd.reshape(B, H, W, c).permute(0, 3, 1, 2))
        return self.U_fc1(f.reshape(B, c, -1).permute(0, 2, 1))


class SwinTransformer(nn.Module):
    """swin.py:1110-1479 (eval-mode semantics for parity; training adds apply_mask)."""

    def __init__(self, embed_dims=128, depths=(2, 2, 18, 2), num_heads=(4, 8, 16, 32), window_size=12,
                 mlp_ratio=4, drop_path_rate=0.3, with_cp=False, mapa_ratio=0.125, adapter_ratio=0.0625,
                 dscf_ratio=0.125, init_cfg=None, **unused):
        super().__init__()
        self.patch_embed = PatchEmbed(3, embed_dims)
        self.extra_patch_embed = PatchEmbed(3, embed_dims)
        dpr = [x.item() for x in torch.linspace(0, drop_path_rate, sum(depths))]
        self.stages, self.MPGBlocks, self.DeformMPGBlocks = nn.ModuleList(), nn.ModuleList(), nn.ModuleList()
        stride, n_groups, n_heads = [8, 4, 2, 1], [1, 2, 4, 8], [2, 4, 8, 16]
        c = embed_dims
        for i in range(len(depths)):
            ds = PatchMerging(c, 2 * c) if i < len(depths) - 1 else None
            stage = SwinBlockSequence(c, num_heads[i], int(mlp_ratio * c), depths[i], window_size,
                                      dpr[sum(depths[:i]):sum(depths[:i + 1])], ds, adapter_ratio, with_cp)
            self.MPGBlocks.append(MPGBlock(c, mapa_ratio))
            self.stages.append(stage)
            self.DeformMPGBlocks.append(DeformMPGBlock(c, stride[i], n_groups[i], n_heads[i], 0, i, dscf_ratio))
            if ds:
                c = ds.out_channels
        self.num_features = [int(embed_dims * 2 ** i) for i in range(len(depths))]
        for i in range(len(depths)):
            self.add_module(f"norm{i}", nn.LayerNorm(self.num_features[i]))
            self.add_module(f"extra_norm{i}", nn.LayerNorm(self.num_features[i]))
            self.add_module(f"fuse_norm{i}", nn.LayerNorm(self.num_features[i]))

    def forward(self, x):
        xr, hw = self.patch_embed(x[0])
        xd, hwd = self.extra_patch_embed(x[1])
        if self.training:  # MMST apply_mask (swin.py:1094-1105, 1433-1434)
            import random
            idx = random.sample(range(xr.size(0)), xr.size(0) // 2)
            xr, xd = xr.clone(), xd.clone()
            xr[idx[0]] = 0
            xd[idx[1]] = 0
        outs, outs_r, outs_d = [], [], []
        for i, stage in enumerate(self.stages):
            fr, fd = self.MPGBlocks[i](xr, xd, hw[0], hw[1])
            xr, xd = xr + fr, xd + fd
            xr, hw, xro, ohw = stage(xr, hw, "rgb")
            xd, hwd, xdo, _ = stage(xd, hwd, "dte")
            xro = getattr(self, f"norm{i}")(xro)
            xdo = getattr(self, f"extra_norm{i}")(xdo)
            o = getattr(self, f"fuse_norm{i}")(self.DeformMPGBlocks[i](xro, xdo, *ohw, i))
            c = self.num_features[i]
            outs.append(o.view(-1, *ohw, c).permute(0, 3, 1, 2).contiguous())
            outs_r.append(xro.view(-1, *ohw, c).permute(0, 3, 1, 2).contiguous())
            outs_d.append(xdo.view(-1, *ohw, c).permute(0, 3, 1, 2).contiguous())
        return outs, outs_r, outs_d


class _MLP(nn.Module):
    def __init__(self, dim, embed_dim):
        super().__init__()
        self.proj = nn.Linear(dim, embed_dim)

    def forward(self, x):
        return self.proj(x.flatten(2).transpose(1, 2))


class _ConvModule(nn.Module):
    def __init__(self, c1, c2):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, 1, bias=False)
        self.bn = nn.BatchNorm2d(c2)
        self.activate = nn.ReLU(True)

    def forward(self, x):
        return self.activate(self.bn(self.conv(x)))


class SegFormerHead(nn.Module):
    """semseg/models/heads/segformer.py:29-48."""

    def __init__(self, dims: List[int], embed_dim=256, num_classes=19):
        super().__init__()
        for i, d in enumerate(dims):
            self.add_module(f"linear_c{i + 1}", _MLP(d, embed_dim))
        self.linear_fuse = _ConvModule(embed_dim * 4, embed_dim)
        self.linear_pred = nn.Conv2d(embed_dim, num_classes, 1)
        self.dropout = nn.Dropout2d(0.1)

    def forward(self, feats):
        B, _, H, W = feats[0].shape
        outs = [self.linear_c1(feats[0]).permute(0, 2, 1).reshape(B, -1, H, W)]
        for i, f in enumerate(feats[1:]):
            cf = getattr(self, f"linear_c{i + 2}")(f).permute(0, 2, 1).reshape(B, -1, *f.shape[-2:])
            outs.append(F.interpolate(cf, size=(H, W), mode="bilinear", align_corners=False))
        return self.linear_pred(self.dropout(self.linear_fuse(torch.cat(outs[::-1], 1))))


class CMNeXt(nn.Module):
    """cmnext.py:11-33 + base.py:37-53 (Swin-B / Swin-L)."""

    def __init__(self, backbone="SwinTransformer-B", num_classes=25, modals=("img", "depth"), _tiny=False):
        super().__init__()
        if _tiny:
            self.backbone = SwinTransformer(embed_dims=32, depths=(2, 2, 2, 2), num_heads=(1, 2, 4, 8))
            ch, e = [32, 64, 128, 256], (64, 32)
        elif backbone == "SwinTransformer-B":
            self.backbone = SwinTransformer(with_cp="event" in modals)
            ch, e = [128, 256, 512, 1024], (512, 256)
        elif backbone == "SwinTransformer-L":
            self.backbone = SwinTransformer(embed_dims=192, num_heads=(6, 12, 24, 48), with_cp=True)
            ch, e = [192, 384, 768, 1536], (512, 256)
        else:
            raise ValueError("The backbone does not exist.")
        self.modals = list(modals)
        self.decode_head = SegFormerHead(ch, e[0], num_classes)
        self.decode_head_rgb = SegFormerHead(ch, e[1], num_classes)
        self.decode_head_dte = SegFormerHead(ch, e[1], num_classes)

    def forward(self, x):
        y, yr, yd = self.backbone(x)
        size = x[0].shape[2:]
        return tuple(F.interpolate(h(f), size=size, mode="bilinear", align_corners=False)
                     for h, f in ((self.decode_head, y), (self.decode_head_rgb, yr), (self.decode_head_dte, yd)))


# ----------------------------------------------------------------- MSDA
def multi_scale_deformable_attn_pytorch(value, value_spatial_shapes, sampling_locations, attention_weights):
    """multi_scale_deform_attn.py:96-136."""
    bs, _, M, D = value.shape
    _, Q, _, L, P, _ = sampling_locations.shape
    vl = value.split([int(h) * int(w) for h, w in value_spatial_shapes], dim=1)
    grids = 2 * sampling_locations - 1
    outs = []
    for lvl, (h, w) in enumerate(value_spatial_shapes):
        v = vl[lvl].flatten(2).transpose(1, 2).reshape(bs * M, D, int(h), int(w))
        g = grids[:, :, :, lvl].transpose(1, 2).flatten(0, 1)
        outs.append(F.grid_sample(v, g, mode="bilinear", padding_mode="zeros", align_corners=False))
    aw = attention_weights.transpose(1, 2).reshape(bs * M, 1, Q, L * P)
    out = (torch.stack(outs, dim=-2).flatten(-2) * aw).sum(-1).view(bs, M * D, Q)
    return out.transpose(1, 2).contiguous()


class MultiScaleDeformableAttention(nn.Module):
    """multi_scale_deform_attn.py:139-363 (CPU path)."""

    def __init__(self, embed_dim=256, num_heads=8, num_levels=4, num_points=4, img2col_step=64, dropout=0.1,
                 batch_first=False):
        super().__init__()
        self.dropout = nn.Dropout(dropout)
        self.batch_first = batch_first
        self.im2col_step = img2col_step
        self.embed_dim, self.num_heads, self.num_levels, self.num_points = embed_dim, num_heads, num_levels, num_points
        self.sampling_offsets = nn.Linear(embed_dim, num_heads * num_levels * num_points * 2)
        self.attention_weights = nn.Linear(embed_dim, num_heads * num_levels * num_points)
        self.value_proj = nn.Linear(embed_dim, embed_dim)
        self.output_proj = nn.Linear(embed_dim, embed_dim)

    def forward(self, query, key=None, value=None, identity=None, query_pos=None, key_padding_mask=None,
                reference_points=None, spatial_shapes=None, level_start_index=None, **kw):
        value = query if value is None else value
        identity = query if identity is None else identity
        if query_pos is not None:
            query = query + query_pos
        if not self.batch_first:
            query, value = query.permute(1, 0, 2), value.permute(1, 0, 2)
        bs, Q, _ = query.shape
        _, S, _ = value.shape
        M, L, P = self.num_heads, self.num_levels, self.num_points
        value = self.value_proj(value)
        if key_padding_mask is not None:
            value = value.masked_fill(key_padding_mask[..., None], 0.0)
        value = value.view(bs, S, M, -1)
        off = self.sampling_offsets(query).view(bs, Q, M, L, P, 2)
        aw = self.attention_weights(query).view(bs, Q, M, L * P).softmax(-1).view(bs, Q, M, L, P)
        if reference_points.shape[-1] == 2:
            norm = torch.stack([spatial_shapes[..., 1], spatial_shapes[..., 0]], -1)
            loc = reference_points[:, :, None, :, None, :] + off / norm[None, None, None, :, None, :]
        else:
            loc = (reference_points[:, :, None, :, None, :2]
                   + off / P * reference_points[:, :, None, :, None, 2:] * 0.5)
        out = self.output_proj(multi_scale_deformable_attn_pytorch(value, spatial_shapes, loc, aw))
        if not self.batch_first:
            out = out.permute(1, 0, 2)
        return self.dropout(out) + identity


# ----------------------------------------------------------------- LightSB (diagonal)
def lightsb_drift(x, t, r, S_log_diag, log_alpha_raw, epsilon):
    """Closed form of sb.py:106-161 get_drift (diagonal): the gradient of the logsumexp is
    sum_k softmax_k * c_k / A_k / (eps (1-t)), so drift = (sum_k w_k c_k / A_k - x) / (1-t)."""
    eps = epsilon
    S = torch.exp(S_log_diag)                                        # K, D
    tt = t[:, None, None]
    A = tt / (eps * (1 - tt)) + 1.0 / (eps * S)[None]               # R, K, D
    c = (x / (eps * (1 - t[:, None])))[:, None, :] + (r / (eps * S))[None]
    arg = (log_alpha_raw / eps)[None] - 0.5 * S_log_diag.sum(-1)[None] - 0.5 * torch.log(A).sum(-1) \
        - 0.5 * (r * r / S / eps).sum(-1)[None] + 0.5 * (c * c / A).sum(-1)
    w = arg.softmax(-1)                                              # R, K
    return ((w[:, :, None] * c / A).sum(1) - x) / (1 - t[:, None])


def lightsb_log_C(x, r, S_log_diag, log_alpha_raw, epsilon):
    """sb.py:206-224 (diagonal)."""
    S = torch.exp(S_log_diag)
    arg = ((x[:, None] * S[None] * x[:, None]).sum(-1) + 2 * (x @ r.T)) / (2 * epsilon) + (log_alpha_raw / epsilon)[None]
    return torch.logsumexp(arg, -1)


def lightsb_em(x, n_steps, noise, r, S_log_diag, log_alpha_raw, epsilon):
    """sb.py:163-175 with the per-step N(0,1) draws supplied."""
    t = torch.zeros(x.shape[0], dtype=x.dtype)
    dt = 1.0 / n_steps
    traj = [x]
    for i in range(n_steps):
        x = x + lightsb_drift(x, t, r, S_log_diag, log_alpha_raw, epsilon) * dt \
            + math.sqrt(dt) * math.sqrt(float(epsilon)) * noise[i]
        t = t + dt
        traj.append(x)
    return torch.stack(traj, 1)


def lightsb_full_S(U, S_log_diag):
    """sb.py:47-48: S = (U * exp(s)[:, None, :]) @ Uᵀ (U orthogonal, however parametrised)."""
    return (U * torch.exp(S_log_diag)[:, None, :]) @ U.permute(0, 2, 1)


def lightsb_full_log_C(x, r, S_log_diag, U, log_alpha_raw, epsilon):
    """sb.py:206-224, is_diagonal=False, dense: xᵀSx by matrix products."""
    S = lightsb_full_S(U, S_log_diag)
    x_S_x = (x[:, None, None, :] @ (S[None, :, :, :] @ x[:, None, :, None]))[:, :, 0, 0]
    x_r = (x[:, None, :] * r[None, :, :]).sum(dim=-1)
    return torch.logsumexp((x_S_x + 2 * x_r) / (2 * epsilon) + log_alpha_raw[None, :] / epsilon, dim=-1)


def lightsb_full_drift(x, t, r, S_log_diag, U, log_alpha_raw, epsilon):
    """sb.py:106-161, is_diagonal=False, as written: dense S, A (rows x K x D x D), their inverses
    through the rotation, the log-partition and its gradient by autograd."""
    x = x.clone().requires_grad_(True)
    S_diagonal = torch.exp(S_log_diag)
    A_diagonal = (t / (epsilon * (1 - t)))[:, None, None] + 1 / (epsilon * S_diagonal)[None, :, :]
    S_log_det = torch.sum(S_log_diag, dim=-1)
    A_log_det = torch.sum(torch.log(A_diagonal), dim=-1)
    log_alpha = log_alpha_raw / epsilon
    S_inv = (U * (1 / S_diagonal[:, None, :])) @ U.permute(0, 2, 1)
    A_inv = (U[None] * (1 / A_diagonal[:, :, None, :])) @ U.permute(0, 2, 1)[None]
    c = ((1 / (epsilon * (1 - t)))[:, None] * x)[:, None, :] + (S_inv @ (r[:, :, None]))[None, :, :, 0] / epsilon
    c_A_inv_c = (c[:, :, None, :] @ A_inv @ c[:, :, :, None])[:, :, 0, 0]
    r_S_inv_r = (r[:, None, :] @ S_inv @ r[:, :, None])[None, :, 0, 0]
    exp_arg = log_alpha[None, :] - 0.5 * S_log_det[None, :] - 0.5 * A_log_det - 0.5 * r_S_inv_r / epsilon + 0.5 * c_A_inv_c
    lse = torch.logsumexp(exp_arg, dim=-1)
    g = torch.autograd.grad(lse, x, grad_outputs=torch.ones_like(lse))[0]
    return (-x / (1 - t[:, None]) + epsilon * g).detach()


def lightsb_full_log_potential(x, r, S_log_diag, U, log_alpha_raw, epsilon):
    """sb.py:183-204, is_diagonal=False: the MultivariateNormal mixture's log-density + logsumexp(log α)."""
    from torch.distributions import Categorical, MixtureSameFamily, MultivariateNormal
    log_alpha = log_alpha_raw / epsilon
    S = lightsb_full_S(U, S_log_diag)
    gmm = MixtureSameFamily(Categorical(logits=log_alpha), MultivariateNormal(loc=r, covariance_matrix=epsilon * S))
    return gmm.log_prob(x) + torch.logsumexp(log_alpha, dim=-1)


# ----------------------------------------------------------------- detection post-processing
def nms_ref(boxes, scores, iou_threshold):
    """Greedy NMS as torchvision.ops.nms computes it on the CPU (torchvision is a third-party
    dependency of detectron2, absent here; vCLR calls it through detectron2 batched_nms,
    projects/vCLR_deformable_mask/modeling/dino.py:1245): boxes in decreasing score order (stable
    here), box j suppressed when a kept earlier box i has IoU(i, j) > threshold, IoU = inter /
    (area_i + area_j - inter) in fp32 without fused multiply-adds.  Returns kept indices."""
    b = np.asarray(boxes, dtype=np.float32)
    order = np.argsort(-np.asarray(scores, dtype=np.float64), kind="stable")
    b = b[order]
    n = len(b)
    area = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    supp = np.zeros(n, dtype=bool)
    keep = []
    for i in range(n):
        if supp[i]:
            continue
        keep.append(order[i])
        w = np.maximum(np.minimum(b[i, 2], b[i + 1:, 2]) - np.maximum(b[i, 0], b[i + 1:, 0]), np.float32(0))
        h = np.maximum(np.minimum(b[i, 3], b[i + 1:, 3]) - np.maximum(b[i, 1], b[i + 1:, 1]), np.float32(0))
        inter = (w * h).astype(np.float32)
        iou = inter / ((area[i] + area[i + 1:]).astype(np.float32) - inter)
        supp[i + 1:] |= iou > np.float32(iou_threshold)
    return np.asarray(keep, dtype=np.int64)


def batched_nms_ref(boxes, scores, idxs, iou_threshold):
    """torchvision batched_nms's coordinate trick (offset = label x (max coordinate + 1), fp32) then nms_ref."""
    b = np.asarray(boxes, dtype=np.float32)
    if len(b) == 0:
        return np.zeros((0,), dtype=np.int64)
    off = np.asarray(idxs).astype(np.float32) * (b.max() + np.float32(1))
    return nms_ref(b + off[:, None], scores, iou_threshold)


# ----------------------------------------------------------------- metrics
def metrics_tp_fp_fn(pred_logits, gt, n_classes, ignore=255):
    """semseg/metrics.py:57-69 (one update)."""
    pred = pred_logits.argmax(1)
    valid = gt != ignore
    tp, fp, fn = [], [], []
    for c in range(n_classes):
        g, p = gt == c, pred == c
        tp.append(int((g & p & valid).sum()))
        fp.append(int((~g & p & valid).sum()))
        fn.append(int((g & ~p & valid).sum()))
    return tp, fp, fn


def metrics_iou(tp, fp, fn):
    """semseg/metrics.py:85-96 compute_iou: per-class Jaccard tp / max(tp + fp + fn, 1e-8) as
    fractions (the reference's rounding loop rebinds a loop variable and changes nothing), and
    round(mean * 100, 2)."""
    jac = [float(a) / max(float(a + b + c), 1e-8) for a, b, c in zip(tp, fp, fn)]
    return jac, round(sum(jac) / len(jac) * 100, 2)


def evaluate_msf(model, batches, n_classes, scales, flip, ignore=255):
    """val_mm.py:87-120: for each batch, the softmax probabilities of the model at every scale
    (sizes int(scale * H) rounded UP to a multiple of 32, align_corners=True bilinear resizes of
    every modality, and the logits resized back the same way), plus the horizontally flipped
    input's (logits flipped back), summed; Metrics (semseg/metrics.py) on the sums.  Returns the
    per-batch summed probabilities and (ious, miou)."""
    import math
    import torch.nn.functional as F
    model.eval()
    sums, tp, fp, fn = [], [0] * n_classes, [0] * n_classes, [0] * n_classes
    with torch.no_grad():
        for images, labels in batches:
            B, H, W = labels.shape
            acc = torch.zeros(B, n_classes, H, W)
            for scale in scales:
                nH, nW = int(scale * H), int(scale * W)
                nH, nW = int(math.ceil(nH / 32)) * 32, int(math.ceil(nW / 32)) * 32
                xs = [F.interpolate(img, size=(nH, nW), mode="bilinear", align_corners=True) for img in images]
                for flipped in ([False, True] if flip else [False]):
                    inp = [torch.flip(x, dims=(3,)) for x in xs] if flipped else xs
                    logits = model(inp)[0]
                    if flipped:
                        logits = torch.flip(logits, dims=(3,))
                    logits = F.interpolate(logits, size=(H, W), mode="bilinear", align_corners=True)
                    acc += logits.softmax(dim=1)
            sums.append(acc)
            a, b, c = metrics_tp_fp_fn(acc, labels, n_classes, ignore)
            tp, fp, fn = [x + y for x, y in zip(tp, a)], [x + y for x, y in zip(fp, b)], [x + y for x, y in zip(fn, c)]
    return sums, metrics_iou(tp, fp, fn)


# ====================================================================== training objective
def mmst_loss(logits, logits_rgb, logits_dte, lbl, ignore_label=255, weight=None):
    """train_mm.py:137-148 with CrossEntropy (semseg/losses.py:6-19): the two modality
    heads are trained only on pixels the fused head classifies correctly."""
    lf = nn.CrossEntropyLoss(weight=weight, ignore_index=ignore_label)
    pred = logits.softmax(dim=1).argmax(dim=1)
    mask_lbl = lbl.clone()
    mask_lbl[pred != lbl] = ignore_label
    return lf(logits, lbl) + 0.01 * lf(logits_rgb, mask_lbl) + 0.01 * lf(logits_dte, mask_lbl)
