"""Deterministic, name-hashed parameter fill (TEST INFRASTRUCTURE).

Used by the fixture generator (on the *reference* modules, in this container), by the
tests (on the oracle restatement and on the product modules, here and on the GPU box)
and by bench.py (random-init weights of the real architecture — there is no pretrained
checkpoint offline).  Because every value is a pure function of (state-dict key, shape,
seed), the reference, the oracle and the product receive identical weights without
shipping a state dict.

numpy's PCG64 stream is platform independent, so the GPU box regenerates the same bits.
"""
import zlib

import numpy as np
import torch

_SKIP = ("relative_position_index", "num_batches_tracked")


def _values(name, shape, seed):
    rng = np.random.Generator(np.random.PCG64(zlib.crc32(name.encode()) ^ (seed * 0x9E3779B1 & 0xFFFFFFFF)))
    u = rng.uniform(-1.0, 1.0, size=shape)
    leaf = name.rsplit(".", 1)[-1]
    if name.endswith("running_var"):
        return 1.0 + 0.5 * u
    if name.endswith("running_mean"):
        return 0.1 * u
    if "rpe_table" in name or "relative_position_bias_table" in name:
        return 0.5 * u
    if leaf in ("deform_weight",):
        return 0.6 + 0.3 * u
    if leaf in ("identity_weight",) or leaf.startswith("tfts_gamma"):
        return 1.0 + 0.1 * u
    if leaf.startswith("tfts_beta"):
        return 0.05 * u
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        return u * (1.0 / np.sqrt(max(fan_in, 1)))
    if leaf == "weight":  # LayerNorm / BatchNorm affine
        return 1.0 + 0.1 * u
    return 0.05 * u  # biases and other vectors


@torch.no_grad()
def fill_module(module: torch.nn.Module, seed: int = 0, dedup: bool = False) -> torch.nn.Module:
    """Overwrite every floating-point parameter/buffer of ``module`` in place.  dedup: a tensor
    registered under several names (DINO's heads, shared with its decoder) is filled once, from
    its alphabetically first name, so the result does not depend on module registration order."""
    items = module.state_dict(keep_vars=True).items()
    seen = set()
    if dedup:
        items = sorted(items)
    for name, t in items:
        if any(s in name for s in _SKIP) or not t.is_floating_point() or t.dim() == 0:
            continue
        if dedup:
            if id(t) in seen:
                continue
            seen.add(id(t))
        v = torch.from_numpy(_values(name, tuple(t.shape), seed)).to(t.dtype)
        t.data.copy_(v.to(t.device))
    return module


def seeded(shape, seed, kind="normal", dtype=np.float32, lo=0.0, hi=1.0):
    """Platform-independent test input generator."""
    rng = np.random.Generator(np.random.PCG64(seed))
    if kind == "normal":
        a = rng.standard_normal(size=shape)
    elif kind == "uniform":
        a = rng.uniform(lo, hi, size=shape)
    else:
        raise ValueError(kind)
    return a.astype(dtype)
