from torch.nn.init import trunc_normal_  # noqa: F401

from .common import ConvModule, DropPath  # noqa: F401
