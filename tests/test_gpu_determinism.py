"""Run-to-run reproducibility of the C2 training step.

Every irads reduction on the path sums in a fixed order (the DAttn attention backward's partials,
the cross-entropy partials, the split-K weight gradients, the MSDA gather backward) or in int64
fixed point (the DAttn grid-sample backward's scatter, irads_dattn_sample_bwd_ws).  MIOpen's
default (benchmark) solvers for the DSCF fuse_q 3x3 convolution are not reproducible; with `torch.backends.cudnn.deterministic` they are
(bench.py --deterministic, +0.8 ms per step).  scripts/determinism_probe.py is the
diagnostic this test condenses."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_training_step_reproducible():
    """C2 model (Swin-B CMNeXt, eval mode so that no dropout / DropPath / apply_mask draws, batch 2,
    512x512, bf16 autocast), deterministic MIOpen solvers: two identical forward + backward passes
    give bit-identical logits and bit-identical gradients for every trainable tensor."""
    import bench
    prev = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        dev = torch.device("cuda", 0)
        torch.manual_seed(3407)
        model, _, _, loss_fn = bench.build(dev, 1, 0, 1000)
        model.eval()
        batch = bench.synthetic_batch(2, 512, dev, 3407)
        runs = []
        for _ in range(2):
            model.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                outs = model([batch[0], batch[1]])
            from semseg.losses import mmst_loss
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = mmst_loss(loss_fn, *outs, batch[2])
            loss.backward()
            torch.cuda.synchronize()
            runs.append(([o.detach().clone() for o in outs],
                         {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}))
        (o0, g0), (o1, g1) = runs
        assert all(torch.equal(a, b) for a, b in zip(o0, o1)), "forward not bit-reproducible"
        assert set(g0) == set(g1) and len(g0) > 100
        diff = [n for n in g0 if not torch.equal(g0[n], g1[n])]
        assert not diff, (len(diff), diff[:5])
    finally:
        torch.backends.cudnn.deterministic = prev
