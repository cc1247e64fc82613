"""LightSB with full covariance (modules/sb.py is_diagonal=False; reference modules/sb.py:36-49,
83-98, 136-155, 163-175, 197-202, 217-219) against the dense restatement of the reference's
formulas (oracle/irads_ref.py lightsb_full_*: S and A as D x D matrices, the drift by autograd) on
the module's own orthogonal U.  geotorch (the reference's parametrisation) is absent: the map
from the stored parameter to U is PyTorch's, so a geotorch checkpoint's U is not reproduced
(parity unpinned there); everything downstream of U is pinned here in fp64."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ir-ads_amd")]

from oracle import irads_ref as R  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _fp64(fn):
    """Build in fp64 so that the parametrisation's orthogonal base is orthogonal to fp64 precision
    (an fp32-built U cast to fp64 is orthogonal only to ~4e-7, which both formulas assume exactly)."""
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        return fn()
    finally:
        torch.set_default_dtype(old)


def _model(dim=12, k=4, eps=0.1, seed=0):
    from modules.sb import LightSB
    torch.manual_seed(seed)
    m = _fp64(lambda: LightSB(dim=dim, n_potentials=k, epsilon=eps, is_diagonal=False)).to(DEV)
    with torch.no_grad():
        m.S_log_diagonal_matrix.copy_(torch.randn(k, dim) * 0.3 - 1.0)
        m.log_alpha_raw.copy_(torch.randn(k) * 0.05)
        m.r.copy_(torch.randn(k, dim))
    return m


def _args(m):
    U = m.S_rotation_matrix
    return m.r, m.S_log_diagonal_matrix, U, m.log_alpha_raw, m.epsilon


def test_state_dict_and_orthogonality():
    m = _model()
    keys = set(m.state_dict())
    assert "parametrizations.S_rotation_matrix.original" in keys
    U = m.S_rotation_matrix
    eye = torch.eye(U.shape[-1], device=DEV, dtype=U.dtype)
    torch.testing.assert_close(U @ U.transpose(1, 2), eye.expand_as(U), rtol=0, atol=1e-12)
    torch.testing.assert_close(m.get_S(), R.lightsb_full_S(U, m.S_log_diagonal_matrix))


def test_log_C_log_potential_and_gradients():
    m = _model()
    x = torch.randn(33, 12, device=DEV, dtype=torch.float64)
    lc, lc_ref = m.get_log_C(x), R.lightsb_full_log_C(x, *_args(m))
    torch.testing.assert_close(lc, lc_ref, rtol=1e-10, atol=1e-10)
    lp, lp_ref = m.get_log_potential(x), R.lightsb_full_log_potential(x, *_args(m))
    torch.testing.assert_close(lp, lp_ref, rtol=1e-10, atol=1e-9)
    params = [m.r, m.S_log_diagonal_matrix, m.log_alpha_raw, m.parametrizations.S_rotation_matrix.original]
    g = torch.autograd.grad((lc.sum() - lp.sum()), params)
    g_ref = torch.autograd.grad((R.lightsb_full_log_C(x, *_args(m)).sum()
                                 - R.lightsb_full_log_potential(x, *_args(m)).sum()), params)
    for a, b in zip(g, g_ref):
        torch.testing.assert_close(a, b, rtol=1e-8, atol=1e-9)


def test_drift_and_euler_maruyama():
    m = _model()
    x = torch.randn(17, 12, device=DEV, dtype=torch.float64)
    t = torch.rand(17, device=DEV, dtype=torch.float64) * 0.9
    torch.testing.assert_close(m.get_drift(x, t), R.lightsb_full_drift(x, t, *_args(m)), rtol=1e-9, atol=1e-9)
    noise = torch.randn(5, 17, 12, device=DEV, dtype=torch.float64)
    traj = m.sample_euler_maruyama(x, 5, noise=noise)
    xs, tt = x, torch.zeros(17, device=DEV, dtype=torch.float64)
    for i in range(5):  # sb.py:163-175 with the recorded noise
        xs = xs + R.lightsb_full_drift(xs, tt, *_args(m)) * 0.2 + (0.2 ** 0.5) * torch.sqrt(m.epsilon) * noise[i]
        tt = tt + 0.2
    torch.testing.assert_close(traj[:, -1], xs, rtol=1e-8, atol=1e-8)
    assert traj.shape == (17, 6, 12)


def test_forward_samples_the_conditional_gmm():
    """One potential: the conditional is N(r + S x, ε S) for every x; sample moments at 200k draws."""
    from modules.sb import LightSB
    torch.manual_seed(1)
    m = _fp64(lambda: LightSB(dim=3, n_potentials=1, epsilon=0.2, is_diagonal=False)).to(DEV)
    x0 = torch.tensor([0.3, -0.2, 0.5], device=DEV, dtype=torch.float64)
    y = m(x0.expand(200000, 3).contiguous())
    S = m.get_S()[0]
    mean = m.r[0] + S @ x0
    torch.testing.assert_close(y.mean(0), mean, rtol=0, atol=5e-3)
    cov = torch.cov(y.t())
    torch.testing.assert_close(cov, m.epsilon * S, rtol=0, atol=5e-3)


def test_cpu_tensors_refused():
    from modules.sb import LightSB
    m = LightSB(dim=4, n_potentials=2, is_diagonal=False)
    with pytest.raises(RuntimeError):
        m.get_log_C(torch.randn(3, 4))
