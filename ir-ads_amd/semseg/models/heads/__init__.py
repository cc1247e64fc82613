from .segformer import SegFormerHead

__all__ = ['SegFormerHead']
