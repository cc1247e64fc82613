from .cmnext import CMNeXt

__all__ = ['CMNeXt']
