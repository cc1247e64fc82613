"""LightSB Schrödinger-bridge GMM (reference modules/sb.py:19-227), MI355X-native.

Same constructor, buffers, parameters and methods as the reference.  The diagonal
path's hot loops run in libirads.so:
  * ``get_drift``: closed-form gradient of the log-partition (no autograd.grad per step),
    one wave per row (``irads_sb_drift``);
  * ``sample_euler_maruyama``: every step inside one kernel launch with the row kept in
    registers (``irads_sb_em``);
  * ``forward`` / ``get_log_C``: GMM logits per row (``irads_sb_logits``), vectorised over
    rows instead of the reference's ``sampling_batch_size`` Python loop;
  * ``get_log_potential``: the mixture log-density per row (``irads_sb_log_potential``);
  * ``get_log_C`` and ``get_log_potential`` are differentiable in x and every parameter, as the
    reference's autograd graphs are (closed-form backwards, irads/ops.py), so LightSB's
    training objective E[log C(x0)] - E[log v(x1)] trains on this path.
The reference has no caller for this module; the full-covariance path
needs geotorch's orthogonal parametrisation, which is not available, so
``is_diagonal=False`` raises NotImplementedError.
"""
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
        # kept for state-dict parity; the diagonal path never reads it (no gradient, frozen)
        self.S_rotation_matrix = nn.Parameter(torch.randn(n_potentials, self.dim, self.dim), requires_grad=False)

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
        """epsilon as a host float for the kernel launches, read from the buffer once per value
        (a device read inside a captured HIP graph is not allowed; set_epsilon / load_state_dict
        move the buffer's version and refresh it)."""
        key = (self.epsilon.data_ptr(), self.epsilon._version)
        c = self.__dict__.get("_eps_cache")
        if c is None or c[0] != key:
            c = (key, float(self.epsilon))
            self.__dict__["_eps_cache"] = c
        return c[1]

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
        """log Σ_k alpha_k N(x; r_k, eps S_k) + logsumexp(log alpha) (sb.py:183-204), one wave per
        row on irads_sb_log_potential, differentiable (closed-form backward)."""
        return ops.sb_log_potential(x, self.r, self.S_log_diagonal_matrix, self.log_alpha_raw, self._eps())

    def get_log_C(self, x):
        """logsumexp_k of the GMM logits (sb.py:206-224); differentiable in x, r, S and alpha as
        the reference's (irads.ops.SBLogCFn: closed-form backward)."""
        return ops.sb_log_c(x, self.r, self.S_log_diagonal_matrix, self.log_alpha_raw, self._eps())

    def set_epsilon(self, new_epsilon):
        self.epsilon = torch.tensor(new_epsilon, device=self.epsilon.device)
