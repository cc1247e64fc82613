from .resnet import BasicStem, BottleneckBlock, FrozenBatchNorm2d, ResNet

__all__ = ["ResNet", "BasicStem", "BottleneckBlock", "FrozenBatchNorm2d"]
