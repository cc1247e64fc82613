"""Small building blocks (reference semseg/models/layers/common.py)."""
import torch
from torch import nn, Tensor


class ConvModule(nn.Sequential):
    def __init__(self, c1, c2, k, s=1, p=0, d=1, g=1):
        super().__init__(nn.Conv2d(c1, c2, k, s, p, d, g, bias=False), nn.BatchNorm2d(c2), nn.ReLU(True))


class DropPath(nn.Module):
    """Stochastic depth per sample: x / keep * floor(keep + U[0, 1))."""

    def __init__(self, p: float = None):
        super().__init__()
        self.p = p

    def forward(self, x: Tensor) -> Tensor:
        if not self.p or not self.training:
            return x
        keep = 1 - self.p
        mask = (keep + torch.rand((x.shape[0],) + (1,) * (x.ndim - 1), dtype=x.dtype, device=x.device)).floor_()
        return x.div(keep) * mask


class Linear(nn.Linear):
    """nn.Linear that casts a frozen weight to the autocast dtype once instead of per call.

    Under torch.autocast, F.linear casts input, weight and bias to the autocast dtype on
    every call, and autocast's cast cache only keeps casts of leaf tensors that require
    grad, so a frozen weight (TRAIN_TYPE Adapter freezes the whole Swin trunk,
    optimizers.py:7-30) is re-cast at every use.  Here the cast copy is kept and reused;
    it is the same rounding autocast applies, and it is rebuilt whenever a parameter's
    version counter moves (optimizer step, load_state_dict, in-place edits).  Outside
    autocast, or for trainable weights, this is nn.Linear.  State-dict keys unchanged."""

    def amp_weights(self, dt):
        """(weight, bias) rounded to `dt`, cached until a parameter's version moves."""
        w, b = self.weight, self.bias
        key = (dt, w.data_ptr(), w._version, None if b is None else b._version)
        cache = self.__dict__.get("_amp_cache")
        if cache is None or cache[0] != key:
            with torch.no_grad():
                cache = (key, w.detach().to(dt), None if b is None else b.detach().to(dt))
            self.__dict__["_amp_cache"] = cache
        return cache[1], cache[2]

    def forward(self, x: Tensor) -> Tensor:
        w, b = self.weight, self.bias
        if (w.requires_grad or (b is not None and b.requires_grad) or not x.is_cuda
                or not torch.is_autocast_enabled("cuda")):
            return super().forward(x)
        dt = torch.get_autocast_dtype("cuda")
        wc, bc = self.amp_weights(dt)
        with torch.autocast("cuda", enabled=False):
            return torch.nn.functional.linear(x.to(dt), wc, bc)


class TrainLinear(nn.Linear):
    """nn.Linear for trainable weights (Adapters, MPG / DeformMPG projections, SegFormer
    MLPs): under bf16 autocast on the GPU the backward's weight/bias gradients come from the
    split-K irads_wgrad kernel (irads.ops.LinearFn); otherwise plain nn.Linear.
    State-dict keys unchanged."""

    def forward(self, x: Tensor) -> Tensor:
        from irads import ops
        return ops.linear(x, self.weight, self.bias)
