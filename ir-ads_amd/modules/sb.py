"""LightSB Schrödinger-bridge GMM (reference modules/sb.py:19-227), MI355X-native.

Same constructor, buffers, parameters and methods as the reference.  The diagonal
path's hot loops run in libirads.so:
  * ``get_drift``: closed-form gradient of the log-partition (no autograd.grad per step),
    one wave per row (``irads_sb_drift``);
  * ``sample_euler_maruyama``: every step inside one kernel launch with the row kept in
    registers (``irads_sb_em``);
  * ``forward`` / ``get_log_C``: GMM logits per row (``irads_sb_logits``), vectorised over
    rows instead of the reference's ``sampling_batch_size`` Python loop.
The reference has no caller for this module; the full-covariance path
needs geotorch's orthogonal parametrisation, which is not available, so
``is_diagonal=False`` raises NotImplementedError.
"""
import math

import torch
from torch import nn
from torch.distributions.categorical import Categorical

from irads import ops


class LightSB(nn.Module):
    def __init__(self, dim=512, n_potentials=10, epsilon=0.1, is_diagonal=True, sampling_batch_size=1,
                 S_diagonal_init=0.1):
        super().__init__()
        if not is_diagonal:
            raise NotImplementedError("LightSB(is_diagonal=False) needs geotorch.orthogonal (not available)")
        self.is_diagonal = is_diagonal
        self.dim = dim
        self.n_potentials = n_potentials
        self.register_buffer("epsilon", torch.tensor(epsilon))
        self.sampling_batch_size = sampling_batch_size
        self.log_alpha_raw = nn.Parameter(self.epsilon * torch.log(torch.ones(n_potentials) / n_potentials))
        self.r = nn.Parameter(torch.randn(n_potentials, dim))
        self.S_log_diagonal_matrix = nn.Parameter(torch.log(S_diagonal_init * torch.ones(n_potentials, self.dim)))
        self.S_rotation_matrix = nn.Parameter(torch.randn(n_potentials, self.dim, self.dim))

    def init_r_by_samples(self, samples):
        assert samples.shape[0] == self.r.shape[0]
        self.r.data = torch.clone(samples.to(self.r.device))

    def get_S(self):
        return torch.exp(self.S_log_diagonal_matrix)

    def get_r(self):
        return self.r

    def get_log_alpha(self):
        return (1 / self.epsilon) * self.log_alpha_raw

    def _eps(self):
        return float(self.epsilon)

    @torch.no_grad()
    def forward(self, x):
        """Sample the conditional GMM per row (sb.py:57-104), all rows at once."""
        logits, _ = ops.sb_logits(x, self.r, self.S_log_diagonal_matrix, self.log_alpha_raw, self._eps(),
                                  want_log_c=False)
        k = Categorical(logits=logits).sample()                       # (rows,)
        S = self.get_S().to(x.dtype)
        r_x = self.r.to(x.dtype)[k] + S[k] * x                          # r + S x (diagonal)
        scale = torch.sqrt(self.epsilon.to(x.dtype) * S[k])
        return r_x + scale * torch.randn_like(x)

    def get_drift(self, x, t):
        return ops.sb_drift(x, t, self.r, self.S_log_diagonal_matrix, self.log_alpha_raw, self._eps())

    def sample_euler_maruyama(self, x, n_steps, noise=None):
        if noise is None:
            noise = torch.randn((n_steps,) + tuple(x.shape), device=x.device, dtype=x.dtype)
        return ops.sb_em(x, noise, self.r, self.S_log_diagonal_matrix, self.log_alpha_raw, self._eps())

    def sample_at_time_moment(self, x, t):
        t = t.to(x.device)
        y = self(x)
        return t * y + (1 - t) * x + torch.sqrt(t * (1 - t) * self.epsilon) * torch.randn_like(x)

    def get_log_potential(self, x):
        """log Σ_k alpha_k N(x; r_k, eps S_k) + logsumexp(log alpha) (sb.py:183-204)."""
        S = self.get_S().to(x.dtype)
        r = self.r.to(x.dtype)
        var = self.epsilon.to(x.dtype) * S
        log_alpha = self.get_log_alpha().to(x.dtype)
        comp = -0.5 * (((x[:, None, :] - r[None]) ** 2) / var[None] + torch.log(2 * math.pi * var)[None]).sum(-1)
        mix = torch.log_softmax(log_alpha, -1)
        return torch.logsumexp(comp + mix[None], -1) + torch.logsumexp(log_alpha, -1)

    def get_log_C(self, x):
        _, log_c = ops.sb_logits(x, self.r, self.S_log_diagonal_matrix, self.log_alpha_raw, self._eps(),
                                 want_logits=False)
        return log_c

    def set_epsilon(self, new_epsilon):
        self.epsilon = torch.tensor(new_epsilon, device=self.epsilon.device)
