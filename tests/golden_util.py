"""Load golden fixtures; regenerate seeded inputs and verify their checksums."""
import os

import numpy as np
import torch

from fill import seeded

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def checksum(a):
    a = np.asarray(a, dtype=np.float64)
    return np.array([a.sum(), np.abs(a).sum(), (a * a).sum(), a.size])


class Fixture:
    def __init__(self, name):
        self.z = np.load(os.path.join(GOLDEN, name), allow_pickle=False)

    def __contains__(self, k):
        return k in self.z.files

    def keys(self):
        return self.z.files

    def __getitem__(self, k):
        return self.z[k]

    def t(self, k, dtype=None, device="cpu"):
        x = torch.from_numpy(np.ascontiguousarray(self.z[k]))
        if dtype is not None:
            x = x.to(dtype)
        return x.to(device)

    def regen(self, k, shape, seed, kind="normal", scale=1.0, lo=0.0, hi=1.0):
        """Regenerate a seeded input and check it against the stored checksum."""
        a = seeded(shape, seed, kind, lo=lo, hi=hi) * np.float32(scale) if scale != 1.0 else seeded(shape, seed, kind, lo=lo, hi=hi)
        cs = self.z[k + "__cs"]
        got = checksum(a)
        assert np.allclose(got, cs, rtol=1e-6, atol=1e-3), f"seeded input {k} drifted: {got} vs {cs}"
        return torch.from_numpy(np.ascontiguousarray(a))


def close(a, b, atol, rtol=0.0, what=""):
    a = a.detach().double().cpu()
    b = torch.as_tensor(b).double().cpu() if not torch.is_tensor(b) else b.detach().double().cpu()
    assert a.shape == b.shape, f"{what}: shape {tuple(a.shape)} vs {tuple(b.shape)}"
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol)
    if bad.any():
        i = int(bad.flatten().nonzero()[0])
        raise AssertionError(f"{what}: max err {err.max().item():.3e} (atol {atol}, rtol {rtol}); "
                             f"first bad flat idx {i}: {a.flatten()[i].item()} vs {b.flatten()[i].item()}; "
                             f"{int(bad.sum())}/{bad.numel()} bad")
