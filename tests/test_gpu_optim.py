"""irads AdamW (irads_adamw launches, irads/optim.py) against torch.optim.AdamW: the reference's
optimizer (semseg/optimizers.py:33-49, betas (0.9, 0.999), eps 1e-8, weight decay 0.01)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _tensors(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(), (1,), (3,), (4096,), (4097,), (5, 7), (128, 384), (257, 33), (2, 3, 64, 65), (9000,)]
    ps = [torch.randn(s, generator=g) for s in shapes]
    # a contiguous view at an odd element offset (not 16-B aligned: the scalar path)
    base = torch.randn(1001, generator=g)
    ps.append(base[1:1000])
    return [p.to(DEV) for p in ps]


def _grads(ps, step):
    g = torch.Generator().manual_seed(100 + step)
    return [torch.randn(p.shape, generator=g).to(DEV) * (1 + 10 * (step % 2)) for p in ps]


@pytest.mark.parametrize("lr_tensor", [False, True])
def test_adamw_matches_torch(lr_tensor):
    from irads.optim import AdamW
    a = [torch.nn.Parameter(p.clone()) for p in _tensors(0)]
    b = [torch.nn.Parameter(p.clone()) for p in _tensors(0)]
    lr = torch.tensor(3e-3, device=DEV) if lr_tensor else 3e-3
    groups_a = [{"params": a[:6]}, {"params": a[6:], "weight_decay": 0.0}]
    groups_b = [{"params": b[:6]}, {"params": b[6:], "weight_decay": 0.0}]
    oa = AdamW(groups_a, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01)
    # torch's fused AdamW (what the product ran before): the same element expressions
    # (beta1 * m + (1 - beta1) * g, not the single-tensor path's lerp)
    ob = torch.optim.AdamW(groups_b, 3e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, fused=True)
    for step in range(4):
        for pa, pb, g in zip(a, b, _grads(a, step)):
            pa.grad = g.clone()
            pb.grad = g.clone()
        if step == 2:  # a parameter without a gradient is skipped (its step count stays behind)
            a[3].grad = None
            b[3].grad = None
        oa.step()
        ob.step()
    for pa, pb in zip(a, b):
        torch.testing.assert_close(pa.detach(), pb.detach(), rtol=2e-6, atol=1e-8)
    for pa, pb in zip(a, b):
        sa, sb = oa.state[pa], ob.state[pb]
        # moments to fp32 rounding at the tensor's scale (ATen forms some factors in double)
        for k in ("exp_avg", "exp_avg_sq"):
            scale = float(sb[k].abs().max())
            torch.testing.assert_close(sa[k], sb[k], rtol=2e-6, atol=2e-6 * scale)
        assert float(sa["step"]) == float(sb["step"])
    # the state dict has torch's layout and loads into torch's optimizer
    sd = oa.state_dict()
    oc = torch.optim.AdamW([{"params": b[:6]}, {"params": b[6:], "weight_decay": 0.0}], 3e-3)
    oc.load_state_dict(sd)
    assert set(oc.state_dict()["state"][0].keys()) == {"step", "exp_avg", "exp_avg_sq"}


def test_adamw_graph_replay_matches_eager():
    """Captured once, replayed: the device step counts and the tensor learning rate advance the
    same way as eager steps."""
    from irads.optim import AdamW
    a = [torch.nn.Parameter(p.clone()) for p in _tensors(1)]
    b = [torch.nn.Parameter(p.clone()) for p in _tensors(1)]
    grads = _grads(a, 0)
    for pa, pb, g in zip(a, b, grads):
        pa.grad = g.clone()
        pb.grad = g.clone()
    lr_a = torch.tensor(1e-3, device=DEV)
    oa = AdamW(a, lr_a, weight_decay=0.01)
    ob = AdamW(b, torch.tensor(1e-3, device=DEV), weight_decay=0.01)
    oa.step()  # state allocated outside the capture
    ob.step()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            oa.step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    # the capture did not run the update: both are at step 1 here
    for k in range(3):
        lr_a.fill_(1e-3 * (k + 1))
        ob.param_groups[0]["lr"].fill_(1e-3 * (k + 1))
        graph.replay()
        ob.step()
    torch.cuda.synchronize()
    for pa, pb in zip(a, b):
        torch.testing.assert_close(pa.detach(), pb.detach(), rtol=0, atol=0)
    assert float(oa.state[a[0]]["step"]) == float(ob.state[b[0]]["step"]) == 1 + 3


def test_adamw_capture_refuses_float_lr():
    """A captured step with a float learning rate would bake the value into the graph (replays
    never call step(), so a scheduler's later group['lr'] changes would be ignored): refused."""
    from irads.optim import AdamW
    a = [torch.nn.Parameter(p.clone()) for p in _tensors(1)]
    for pa, g in zip(a, _grads(a, 0)):
        pa.grad = g.clone()
    oa = AdamW(a, 1e-3, weight_decay=0.01)
    oa.step()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with pytest.raises(RuntimeError, match="device tensor"):
            with torch.cuda.graph(graph, stream=side):
                oa.step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()


def test_get_optimizer_uses_native_adamw():
    from irads.optim import AdamW
    from semseg.optimizers import get_optimizer
    m = torch.nn.Module()
    m.Adapter = torch.nn.Linear(8, 8).to(DEV)
    m.other = torch.nn.Linear(8, 8).to(DEV)
    opt = get_optimizer(m, "adamw", 1e-3, "Adapter", 0.01, lr_on_device=True)
    assert isinstance(opt, AdamW)
    assert not m.other.weight.requires_grad
