"""The vCLR DINO detector's modules around the transformer: ResNet-50 backbone, ChannelMapper neck
and the Hungarian matcher (reference detrex/modeling, detectron2's ResNet as dino_r50.py:23-32
configures it)."""
from .backbone import BasicStem, BottleneckBlock, FrozenBatchNorm2d, ResNet
from .matcher import HungarianMatcher
from .neck import ChannelMapper, ConvNormAct

__all__ = ["ResNet", "BasicStem", "BottleneckBlock", "FrozenBatchNorm2d", "ChannelMapper", "ConvNormAct",
           "HungarianMatcher"]
