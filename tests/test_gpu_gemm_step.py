"""The shipped GEMM selection at the shape it was tuned on: one C2 training step (Swin-B 512², B = 8,
bf16 autocast, Adapter mode, MMST loss; BASELINE.json configs[1]) with IRADS_GEMM=table — the trunk
projections on irads_gemm_nt exactly as bench.py runs them, including the 256 x 256 tiling's fused
GELU / GELU' epilogues — against the same step with IRADS_GEMM=off (hipBLASLt everywhere).

The two arms differ only in the GEMMs' summation order, so their difference must be of the size of
bf16 rounding noise: loss relative 1e-3; the aggregate relative L2 over every trainable gradient at
most 2x the bf16 arm's own aggregate error against the product's fp32 step on the same inputs (the
bf16 noise of this step, measured here).  The aux heads' MMST target is taken from the fp32 step's
argmax in all three runs (teacher forcing, as tests/test_gpu_train_parity.py does), so a flipped
pixel decision cannot masquerade as a GEMM error.  Random draws off (oracle/train_fixture.py)."""
import collections

import pytest
import torch

from fill import fill_module
from train_fixture import adapter_trainable, deterministic_train_mode, train_inputs

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _step(model, batch, amp, aux):
    from irads import ops
    from semseg.losses import get_loss
    loss_fn = get_loss("CrossEntropy", 255)
    rgb, dep, lbl = batch
    for p in model.parameters():
        p.grad = None
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        y, yr, yd = model([rgb, dep])
        if aux is None:
            aux = torch.where(y.detach().argmax(1) == lbl, lbl, torch.full_like(lbl, 255))
        l1 = ops.cross_entropy(y, lbl, 255, None)
        loss = l1 + 0.01 * loss_fn(yr, aux) + 0.01 * loss_fn(yd, aux)
    loss.backward()
    grads = {n: p.grad.detach().float().clone() for n, p in model.named_parameters() if p.grad is not None}
    return float(loss.detach()), grads, aux


def _agg(a, b):
    num = sum(float((a[n] - b[n]).double().pow(2).sum()) for n in b)
    den = sum(float(b[n].double().pow(2).sum()) for n in b)
    return (num / den) ** 0.5


def test_c2_step_gemm_table_vs_hipblaslt(monkeypatch):
    from irads import native as N
    from semseg.models import CMNeXt
    torch.manual_seed(3407)
    model = CMNeXt("SwinTransformer-B", 40, ["img", "depth"])
    fill_module(model, seed=41)
    model = model.to(DEV)
    for n, p in model.named_parameters():
        p.requires_grad_(adapter_trainable(n))
    deterministic_train_mode(model)
    batch = [torch.from_numpy(a).to(DEV) for a in train_inputs(8, 512, 512, 40, 300)]

    _, g32, aux = _step(model, batch, amp=False, aux=None)
    counts = collections.Counter()
    orig = N.call

    def call(name, *args):
        if name == "irads_gemm_nt_variant":
            counts[(int(args[1]), int(args[0]))] += 1
        return orig(name, *args)
    monkeypatch.setattr(N, "call", call)
    monkeypatch.setenv("IRADS_GEMM", "off")
    l_off, g_off, _ = _step(model, batch, amp=True, aux=aux)
    assert not counts
    monkeypatch.setenv("IRADS_GEMM", "table")
    l_tab, g_tab, _ = _step(model, batch, amp=True, aux=aux)
    # the table really served this step: plain, GELU and GELU' epilogues, each on a tiling the
    # shipped table lists, and every tiling the table lists for C2 (M = 16384 · 4^-s) in use
    from irads import gemm as G
    table_variants = {v for (_, M, _, _), v in G._selected().items() if M in (262144, 65536, 16384, 4096)}
    assert {e for e, _ in counts} == {0, 1, 2}, dict(counts)
    assert {v for _, v in counts} == table_variants, (dict(counts), table_variants)
    assert sum(counts.values()) >= 60, dict(counts)
    assert sorted(g_tab) == sorted(g_off) == sorted(g32)
    for n in g_tab:
        assert torch.isfinite(g_tab[n]).all(), n
    loss_rel = abs(l_tab - l_off) / abs(l_off)
    noise = _agg(g_off, g32)
    diff = _agg(g_tab, g_off)
    print(f"loss {l_tab:.6f} vs {l_off:.6f} (rel {loss_rel:.2e}); aggregate gradient table-vs-off {diff:.3e}, "
          f"bf16 noise (off vs fp32) {noise:.3e}; irads_gemm_nt launches {dict(counts)}")
    assert loss_rel <= 1e-3, (l_tab, l_off)
    assert diff <= 2 * noise, (diff, noise)
