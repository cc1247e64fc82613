from .channel_mapper import ChannelMapper, ConvNormAct

__all__ = ["ChannelMapper", "ConvNormAct"]
