"""The training iteration captured into a HIP graph (irads/graph_step.py) against the eager
iteration.  Eval mode removes the step's randomness (DropPath, Adapter dropout, apply_mask)
and a zero learning rate keeps the weights fixed, so a replay must reproduce the eager
loss (1e-5 relative) and every trainable parameter's gradient (1.5e-2 relative: MIOpen's
benchmark-mode solvers for the DSCF fuse_q convolution are not reproducible, and one bf16
rounding moved by an ulp is 2^-8; every irads kernel on the path reduces in a fixed order or in
integer fixed point since round 2, tests/test_gpu_determinism.py).  Then a nonzero
learning rate, filled into the device tensor between replays, must move the weights."""
import pytest
import torch

from fill import fill_module

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(seed):
    from semseg.models import CMNeXt
    from semseg.optimizers import get_optimizer
    from semseg.losses import get_loss
    m = CMNeXt("SwinTransformer-B", 40, ["img", "depth"]).to(DEV)
    fill_module(m, seed=seed)
    opt = get_optimizer(m, "adamw", 4e-4, "Adapter", 0.01, lr_on_device=True)
    m.eval()
    return m, opt, get_loss("CrossEntropy", 255)


def _fwd_bwd(m, loss_fn, batch):
    from semseg.losses import mmst_loss
    rgb, dep, lbl = batch
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y, yr, yd = m([rgb, dep])
        loss = mmst_loss(loss_fn, y, yr, yd, lbl)
    loss.backward()
    return loss


def test_graphed_step_matches_eager():
    from irads.graph_step import GraphedTrainStep
    g = torch.Generator().manual_seed(0)
    B, S = 4, 128
    batch = (torch.randn(B, 3, S, S, generator=g).to(DEV), torch.rand(B, 3, S, S, generator=g).to(DEV),
             torch.randint(0, 40, (B, S, S), generator=g).to(DEV))
    m0, opt0, lf = _setup(11)
    opt0.zero_grad(set_to_none=True)
    loss0 = _fwd_bwd(m0, lf, batch).item()
    m1, opt1, lf = _setup(11)
    lr = opt1.param_groups[0]["lr"]
    assert torch.is_tensor(lr) and lr.is_cuda
    lr.fill_(0.0)
    runner = GraphedTrainStep(m1.parameters(), lambda: _fwd_bwd(m1, lf, batch), opt1, warmup=1)
    loss1 = runner.step().item()
    assert abs(loss1 - loss0) <= 1e-5 * abs(loss0), (loss0, loss1)
    p0 = dict(m0.named_parameters())
    n_checked = 0
    # gradients that vanish mathematically (e.g. DAttn proj_k's bias: softmax is invariant to
    # a per-query shift) are pure rounding noise; they are measured against the model-wide
    # RMS gradient instead of their own norm
    refs = [p.grad for p in m0.parameters() if p.requires_grad]
    rms = (torch.stack([r.float().pow(2).sum() for r in refs]).sum() / sum(r.numel() for r in refs)).sqrt()
    for n, p in m1.named_parameters():
        if p.requires_grad:
            ref = p0[n].grad
            den = torch.maximum(ref.norm(), 0.1 * rms * ref.numel() ** 0.5)
            err = ((p.grad - ref).norm() / den).item()
            # MIOpen's solver for fuse_q may reorder its sums between the two runs: round 1
            # observed 0.0075-0.0085 run to run on the DAttn and MPG stage-0 weights (then with
            # float atomics in the DAttn backward as well); a real graph-capture bug shows up at O(1)
            assert err < 1.5e-2, (n, err)
            n_checked += 1
    assert n_checked > 100
    before = [p.detach().clone() for p in runner.params]
    lr.fill_(4e-4)  # what the scheduler does between replays
    loss2 = runner.step().item()
    moved = sum(int(not torch.equal(b, p.detach())) for b, p in zip(before, runner.params))
    assert moved == len(before)
    loss3 = runner.step().item()
    assert loss3 != loss2
