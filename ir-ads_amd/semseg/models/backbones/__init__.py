from .swin import SwinTransformer

__all__ = ['SwinTransformer']
