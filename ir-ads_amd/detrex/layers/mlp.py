"""MLP and FFN blocks (reference detrex/layers/mlp.py:28-132), same keys (``layers.*``)."""
import torch
import torch.nn as nn
import torch.nn.functional as F


class MLP(nn.Module):
    """``Linear -> ReLU -> ... -> Linear`` without dropout or identity (reference mlp.py:28-63)."""

    def __init__(self, input_dim: int, hidden_dim: int, output_dim: int, num_layers: int):
        super().__init__()
        self.num_layers = num_layers
        dims = [input_dim] + [hidden_dim] * (num_layers - 1) + [output_dim]
        self.layers = nn.ModuleList(nn.Linear(a, b) for a, b in zip(dims[:-1], dims[1:]))

    def forward(self, x):
        last = self.num_layers - 1
        for i, layer in enumerate(self.layers):
            x = layer(x) if i == last else F.relu(layer(x))
        return x


class FFN(nn.Module):
    """``(Linear, act, Dropout) x (num_fcs-1), Linear, Dropout`` plus identity (reference mlp.py:66-132)."""

    def __init__(self, embed_dim=256, feedforward_dim=1024, output_dim=None, num_fcs=2,
                 activation=nn.ReLU(inplace=True), ffn_drop=0.0, fc_bias=True, add_identity=True):
        super().__init__()
        assert num_fcs >= 2, f"num_fcs should be no less than 2. got {num_fcs}."
        self.embed_dim = embed_dim
        self.feedforward_dim = feedforward_dim
        self.num_fcs = num_fcs
        self.activation = activation
        output_dim = embed_dim if output_dim is None else output_dim
        layers, cin = [], embed_dim
        for _ in range(num_fcs - 1):
            layers.append(nn.Sequential(nn.Linear(cin, feedforward_dim, bias=fc_bias), self.activation,
                                        nn.Dropout(ffn_drop)))
            cin = feedforward_dim
        layers += [nn.Linear(feedforward_dim, output_dim, bias=fc_bias), nn.Dropout(ffn_drop)]
        self.layers = nn.Sequential(*layers)
        self.add_identity = add_identity

    def forward(self, x, identity=None) -> torch.Tensor:
        out = self.layers(x)
        if not self.add_identity:
            return out
        return (x if identity is None else identity) + out
