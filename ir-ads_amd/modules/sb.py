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
The reference has no caller for this module.

Full covariance (``is_diagonal=False``, sb.py:36-49, 83-98, 136-155, 197-202, 217-219): S_k =
U_k diag(s_k) U_kᵀ with U_k = ``S_rotation_matrix`` kept orthogonal by a parametrisation.  The
reference uses geotorch.orthogonal (a third-party package, absent here); this build registers
PyTorch's ``torch.nn.utils.parametrizations.orthogonal`` instead — the same state-dict layout
(``parametrizations.S_rotation_matrix.original`` / ``.0.base``), a different map from the
unconstrained parameter to the orthogonal matrix, so parity with a geotorch checkpoint is unpinned.
Every quantity is evaluated in each potential's eigenbasis (one batched GEMM y_k = U_kᵀ x): S_k,
A_k = t / (ε(1 - t)) I + (ε S_k)⁻¹ and their inverses share U_k, so xᵀS x, cᵀA⁻¹c, rᵀS⁻¹r and the
log-determinants are per-dimension sums, and the drift's gradient of the log-partition is closed
form (Σ_k w_k U_k diag(1/a_k) v_k / (ε(1 - t))) — the reference's dense (rows x K x D x D) A
matrices are never formed.  Sampling draws r_x + U_k (√(ε s_k) ⊙ z) (the reference's
MultivariateNormal uses the Cholesky factor: same distribution, other samples per z).  These paths
are PyTorch GEMMs and element-wise ops on the GPU (no kernel of their own; the diagonal path above
is the one the C4 hook runs) and refuse CPU tensors as the kernels do.
"""
import math

import torch
from torch import nn
from torch.distributions.categorical import Categorical

from irads import native as N
from irads import ops


class LightSB(nn.Module):
    def __init__(self, dim=512, n_potentials=10, epsilon=0.1, is_diagonal=True, sampling_batch_size=1,
                 S_diagonal_init=0.1):
        super().__init__()
        self.is_diagonal = is_diagonal
        self.dim = dim
        self.n_potentials = n_potentials
        self.register_buffer("epsilon", torch.tensor(epsilon))
        self.sampling_batch_size = sampling_batch_size
        self.log_alpha_raw = nn.Parameter(self.epsilon * torch.log(torch.ones(n_potentials) / n_potentials))
        self.r = nn.Parameter(torch.randn(n_potentials, dim))
        self.S_log_diagonal_matrix = nn.Parameter(torch.log(S_diagonal_init * torch.ones(n_potentials, self.dim)))
        self.S_rotation_matrix = nn.Parameter(torch.randn(n_potentials, self.dim, self.dim),
                                              requires_grad=not is_diagonal)
        if not is_diagonal:  # sb.py:36 (geotorch.orthogonal): PyTorch's orthogonal parametrisation
            torch.nn.utils.parametrizations.orthogonal(self, "S_rotation_matrix")
        # diagonal: kept for state-dict parity, never read (no gradient, frozen)

    def init_r_by_samples(self, samples):
        assert samples.shape[0] == self.r.shape[0]
        self.r.data = torch.clone(samples.to(self.r.device))

    def get_S(self):
        if self.is_diagonal:
            return torch.exp(self.S_log_diagonal_matrix)
        U = self.S_rotation_matrix
        return (U * torch.exp(self.S_log_diagonal_matrix)[:, None, :]) @ U.transpose(1, 2)

    # ---------------------------------------------------------------- full covariance (eigenbasis)
    def _full(self, x):
        """(U, s, log_alpha, eps, y = Uᵀx per potential (rows, K, D), rho = Uᵀr (K, D))."""
        N.check_device(x, "LightSB(is_diagonal=False) input")
        U = self.S_rotation_matrix.to(x.dtype)
        s = torch.exp(self.S_log_diagonal_matrix).to(x.dtype)
        y = torch.einsum("bd,kde->bke", x, U)
        rho = torch.einsum("kd,kde->ke", self.r.to(x.dtype), U)
        return U, s, self.get_log_alpha().to(x.dtype), self.epsilon.to(x.dtype), y, rho

    def _full_logits(self, x):
        """(xᵀS_k x + 2 xᵀr_k) / (2ε) + log α_k (sb.py:84-88, 217-221)."""
        U, s, log_alpha, eps, y, _ = self._full(x)
        x_S_x = (y * y * s[None]).sum(-1)
        x_r = x @ self.r.to(x.dtype).t()
        return (x_S_x + 2 * x_r) / (2 * eps) + log_alpha[None, :], (U, s, eps, y)

    def _full_drift(self, x, t):
        """sb.py:106-161 with is_diagonal=False, closed form in the eigenbases."""
        U, s, log_alpha, eps, y, rho = self._full(x)
        t = t.to(x.dtype)
        inv = 1.0 / (eps * (1 - t))                                      # (rows,)
        a = (t / (eps * (1 - t)))[:, None, None] + 1.0 / (eps * s)[None]  # (rows, K, D)
        v = y * inv[:, None, None] + (rho / (eps * s))[None]             # Uᵀc
        c_A_c = (v * v / a).sum(-1)
        r_S_r = (rho * rho / s).sum(-1)
        exp_arg = (log_alpha[None] - 0.5 * self.S_log_diagonal_matrix.to(x.dtype).sum(-1)[None]
                   - 0.5 * torch.log(a).sum(-1) - 0.5 * r_S_r[None] / eps + 0.5 * c_A_c)
        w = torch.softmax(exp_arg, dim=-1)                               # d lse / d exp_arg
        grad = torch.einsum("kde,bke->bd", U, (w[:, :, None] * v / a)) * inv[:, None]
        return (-x / (1 - t[:, None]) + eps * grad).detach()

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
        if not self.is_diagonal:
            logits, (U, s, eps, y) = self._full_logits(x)
            k = Categorical(logits=logits).sample()
            Uk, sk = U[k], s[k]
            rows = torch.arange(x.shape[0], device=x.device)
            r_x = self.r.to(x.dtype)[k] + torch.einsum("bde,be->bd", Uk, sk * y[rows, k])
            return r_x + torch.einsum("bde,be->bd", Uk, torch.sqrt(eps * sk) * torch.randn_like(x))
        logits, _ = ops.sb_logits(x, self.r, self.S_log_diagonal_matrix, self.log_alpha_raw, self._eps(),
                                  want_log_c=False)
        k = Categorical(logits=logits).sample()                       # (rows,)
        S = self.get_S().to(x.dtype)
        r_x = self.r.to(x.dtype)[k] + S[k] * x                          # r + S x (diagonal)
        scale = torch.sqrt(self.epsilon.to(x.dtype) * S[k])
        return r_x + scale * torch.randn_like(x)

    def get_drift(self, x, t):
        if not self.is_diagonal:
            return self._full_drift(x, t)
        return ops.sb_drift(x, t, self.r, self.S_log_diagonal_matrix, self.log_alpha_raw, self._eps())

    def sample_euler_maruyama(self, x, n_steps, noise=None):
        if noise is None:
            noise = torch.randn((n_steps,) + tuple(x.shape), device=x.device, dtype=x.dtype)
        if not self.is_diagonal:  # sb.py:163-175, step by step
            t = torch.zeros(x.shape[0], device=x.device, dtype=x.dtype)
            dt = 1.0 / n_steps
            traj = [x]
            sq = math.sqrt(dt) * torch.sqrt(self.epsilon.to(x.dtype))
            for i in range(n_steps):
                x = x + self._full_drift(x, t) * dt + sq * noise[i]
                t = t + dt
                traj.append(x)
            return torch.stack(traj, dim=1)
        return ops.sb_em(x, noise, self.r, self.S_log_diagonal_matrix, self.log_alpha_raw, self._eps())

    def sample_at_time_moment(self, x, t):
        t = t.to(x.device)
        y = self(x)
        return t * y + (1 - t) * x + torch.sqrt(t * (1 - t) * self.epsilon) * torch.randn_like(x)

    def get_log_potential(self, x):
        """log Σ_k alpha_k N(x; r_k, eps S_k) + logsumexp(log alpha) (sb.py:183-204), one wave per
        row on irads_sb_log_potential, differentiable (closed-form backward)."""
        if not self.is_diagonal:  # MultivariateNormal(r_k, ε S_k) mixture in the eigenbases
            U, s, log_alpha, eps, y, rho = self._full(x)
            u = y - rho[None]
            D = x.shape[-1]
            logn = -0.5 * (D * math.log(2 * math.pi) + torch.log(eps * s).sum(-1)[None] + (u * u / (eps * s)[None]).sum(-1))
            return torch.logsumexp(torch.log_softmax(log_alpha, -1)[None] + logn, -1) + torch.logsumexp(log_alpha, -1)
        return ops.sb_log_potential(x, self.r, self.S_log_diagonal_matrix, self.log_alpha_raw, self._eps())

    def get_log_C(self, x):
        """logsumexp_k of the GMM logits (sb.py:206-224); differentiable in x, r, S and alpha as
        the reference's (irads.ops.SBLogCFn: closed-form backward)."""
        if not self.is_diagonal:
            return torch.logsumexp(self._full_logits(x)[0], dim=-1)
        return ops.sb_log_c(x, self.r, self.S_log_diagonal_matrix, self.log_alpha_raw, self._eps())

    def set_epsilon(self, new_epsilon):
        self.epsilon = torch.tensor(new_epsilon, device=self.epsilon.device)
