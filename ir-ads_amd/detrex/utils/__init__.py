from .misc import inverse_sigmoid

__all__ = ['inverse_sigmoid']
