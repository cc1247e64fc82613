"""ChannelMapper neck (reference detrex/modeling/neck/channel_mapper.py:87-170, ConvNormAct of
detrex/layers/conv.py): one conv + norm per backbone level to ``out_channels``, extra stride-2
3x3 convs for levels past the backbone's (the first reads the last backbone feature)."""
import copy

import torch.nn as nn


class ConvNormAct(nn.Module):
    """``conv`` -> optional ``norm`` -> optional ``activation`` (same keys as the reference)."""

    def __init__(self, in_channels, out_channels, kernel_size=1, stride=1, padding=0, dilation=1, groups=1,
                 bias=True, norm_layer=None, activation=None):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias)
        self.norm = norm_layer
        self.activation = activation

    def forward(self, x):
        x = self.conv(x)
        if self.norm is not None:
            x = self.norm(x)
        if self.activation is not None:
            x = self.activation(x)
        return x


class ChannelMapper(nn.Module):
    """input_shapes: {name: channels} (or detectron2 ShapeSpec-like objects with ``.channels``)."""

    def __init__(self, input_shapes, in_features, out_channels, kernel_size=3, stride=1, bias=True, groups=1,
                 dilation=1, norm_layer=None, activation=None, num_outs=None, **kwargs):
        super().__init__()
        chans = [getattr(input_shapes[f], "channels", input_shapes[f]) for f in in_features]
        num_outs = len(input_shapes) if num_outs is None else num_outs
        self.convs = nn.ModuleList(
            ConvNormAct(c, out_channels, kernel_size, stride, (kernel_size - 1) // 2, dilation, groups, bias,
                        copy.deepcopy(norm_layer), copy.deepcopy(activation)) for c in chans)
        self.extra_convs = None
        if num_outs > len(chans):
            self.extra_convs = nn.ModuleList(
                ConvNormAct(chans[-1] if i == len(chans) else out_channels, out_channels, 3, 2, 1, dilation, groups,
                            bias, copy.deepcopy(norm_layer), copy.deepcopy(activation))
                for i in range(len(chans), num_outs))
        self.input_shapes, self.in_features, self.out_channels = input_shapes, in_features, out_channels

    def forward(self, inputs):
        assert len(inputs) == len(self.convs)
        outs = [self.convs[i](inputs[self.in_features[i]]) for i in range(len(inputs))]
        if self.extra_convs:
            for i, conv in enumerate(self.extra_convs):
                outs.append(conv(inputs[self.in_features[-1]] if i == 0 else outs[-1]))
        return tuple(outs)
