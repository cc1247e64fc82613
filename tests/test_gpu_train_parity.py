"""The benchmarked training path against the reference, end to end (C2 / C1 / C4 geometries).

The product runs exactly as bench.py runs it: CMNeXt in training mode under bf16 autocast,
TRAIN_TYPE Adapter, the fused Swin stages, the bf16 DAttn path, the HIP segmentation-head
kernels (BN batch statistics), the fused MMST loss, and the step captured into a HIP graph
and replayed.  Only the random draws are switched off (oracle/train_fixture.py:
apply_mask, DropPath, Adapter dropout, Dropout2d), identically in the reference fixture
(oracle/gen_golden.py gen_cmnext_train: the reference modules on CPU in fp32).

Tolerances.  The product computes in bf16 (autocast) and the fixture is the reference in
fp32, so every bound is set against the bf16 noise of the REFERENCE ITSELF: the fixture also
holds the deviation of the reference run under bf16 autocast (CPU) from its own fp32 run,
quantity by quantity ("ref16" below).  Checks:
  * MMST loss: relative 1e-2;
  * logits (stride-8 subsample of y, y_rgb, y_dte): relative L2 <= max(1e-2, 2 ref16);
  * argmax agreement of y >= 99 % where the reference's top-2 margin exceeds 0.05, and
    >= 97 % everywhere;
  * trainable gradients: relative L2 <= max(3e-2, 2 ref16) for the 14 tensors stored in
    full (measured on MI355X: the product's error is 0.8-1.1x the reference's own bf16 error,
    which reaches 0.3-0.5 for the stage-0 DAttn parameters: those gradients are that
    sensitive to bf16 rounding in the reference itself); for every trainable tensor, the norm
    and two seeded random projections (|<g - g_ref, r>| ~ ||g - g_ref||) aggregated over the
    model <= max(3e-2, 2 ref16), and per tensor <= max(0.15, 10 ref16) as a gross-error
    detector (a single-sample noise estimate per tensor is heavy-tailed: measured ratios of
    product to ref16 error have a median near 1 and reach 8 on tensors whose ref16 sample
    is small; a wrong gradient is off by O(1)).  Conv biases ahead of a training-mode
    BatchNorm have a mathematically zero gradient; their values are rounding noise on both
    sides, covered by the ref16 term.
"""
import numpy as np
import pytest
import torch

from fill import fill_module
from golden_util import Fixture
from train_fixture import (FULL_GRAD_KEYS, N_PROJ, TRAIN_FIXTURES, adapter_trainable, deterministic_train_mode,
                           projection, train_inputs)

DEV = torch.device("cuda", 0)

pytestmark = pytest.mark.gpu


def _rel_l2(a, b):
    a = torch.as_tensor(a).double().cpu().flatten()
    b = torch.as_tensor(b).double().cpu().flatten()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _build(fx):
    from semseg.models import CMNeXt
    B, H, W, n_cls, fseed, iseed = (int(v) for v in fx["cfg"])
    model = CMNeXt(str(fx["backbone"]), n_cls, ["img", "depth"])
    assert sorted(model.state_dict().keys()) == fx["state_keys"].tolist()
    fill_module(model, seed=fseed)
    model = model.to(DEV)
    for n, p in model.named_parameters():
        p.requires_grad_(adapter_trainable(n))
    deterministic_train_mode(model)
    rgb, dep, lbl = train_inputs(B, H, W, n_cls, iseed)
    return model, [torch.from_numpy(a).to(DEV) for a in (rgb, dep, lbl)]


def _fwd_bwd(model, loss_fn, batch):
    from semseg.losses import mmst_loss
    rgb, dep, lbl = batch
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y, yr, yd = model([rgb, dep])
        loss = mmst_loss(loss_fn, y, yr, yd, lbl)
    loss.backward()
    return loss, y, yr, yd


def _check(fx, model, loss, y, yr, yd, what, report, fails):
    ref_loss = float(fx["loss"][0])
    rl = abs(float(loss) - ref_loss) / abs(ref_loss)
    report[f"{what}.loss_rel"] = rl
    if not (rl <= 1e-2):
        fails.append(f"{what}: MMST loss {float(loss)} vs reference {ref_loss}")
    for name, t in (("y", y), ("y_rgb", yr), ("y_dte", yd)):
        sub = t.detach().float()[:, :, ::8, ::8].cpu()
        e = _rel_l2(sub, fx[name + "_sub"])
        report[f"{what}.{name}_rel_l2"] = e
        tol = max(1e-2, 2 * float(fx[f"bf16_{name}_rel_l2"]))
        if not (e <= tol):
            fails.append(f"{what}: {name} relative L2 {e:.3e} > {tol:.3e}")
    am = y.detach().argmax(1).cpu().numpy()
    ref_am = fx["y_argmax"].astype(np.int64)
    margin = fx["y_margin"].astype(np.float32)
    agree_all = float((am == ref_am).mean())
    decided = margin > 0.05
    agree = float((am == ref_am)[decided].mean())
    report[f"{what}.argmax_agree"] = agree_all
    report[f"{what}.argmax_agree_decided"] = agree
    report[f"{what}.decided_frac"] = float(decided.mean())
    if not (agree >= 0.99):
        fails.append(f"{what}: argmax agreement {agree:.4f} on decided pixels")
    if not (agree_all >= 0.97):
        fails.append(f"{what}: argmax agreement {agree_all:.4f} overall")
    names = fx["grad_names"].tolist()
    norms, projs = fx["grad_norms"], fx["grad_projs"]
    params = dict(model.named_parameters())
    assert sorted(names) == sorted(n for n, p in params.items() if p.requires_grad)
    num = den = 0.0
    worst = (0.0, "")
    table = []
    # conv biases ahead of a training-mode BatchNorm (DAttn fuse_q) have a mathematically zero
    # gradient (rounding noise on both sides): judged against an absolute floor
    floor = 1e-5 * float(norms.max())
    ref16 = fx["bf16_grad_err"]
    for k, n in enumerate(names):
        g = params[n].grad
        if g is None:
            fails.append(f"{what}: no gradient for {n}")
            continue
        g64 = g.detach().double().cpu().numpy()
        if "g." + n in fx:
            e = _rel_l2(g64, fx["g." + n])
            report[f"{what}.full.{n}"] = e
            tol = max(3e-2, 2 * float(fx["bf16_full_rel." + n]))
            if not (e <= tol):
                fails.append(f"{what}: gradient {n} relative L2 {e:.3e} > {tol:.3e}")
        nr = float(norms[k])
        d = [projection(n, g64, j) - float(projs[k][j]) for j in range(N_PROJ)]
        dn = float(np.sqrt((g64 * g64).sum())) - nr
        per = max(abs(x) for x in d + [dn]) / (nr + floor)
        tol = max(0.15, 10 * float(ref16[k]))
        table.append((per / max(float(ref16[k]), 1e-3), round(per, 4), round(float(ref16[k]), 4), n))
        if per / tol > worst[0]:
            worst = (per / tol, n)
        num += sum(x * x for x in d) / N_PROJ
        den += nr * nr
        if not (per <= tol):
            fails.append(f"{what}: gradient {n}: projection / norm error {per:.3e} > {tol:.3e}")
    agg = float(np.sqrt(num / den))
    report[f"{what}.grad_agg_rel"] = agg
    report[f"{what}.grad_worst_frac_of_tol"] = worst
    report[f"{what}.grad_ratio_to_ref16_median"] = float(np.median([r[0] for r in table]))
    if what == "eager":
        for row in sorted(table, reverse=True)[:5]:
            print("  ratio %.2f err %.4f ref16 %.4f %s" % row)
    tol = max(3e-2, 2 * float(fx["bf16_grad_agg_rel"]))
    if not (agg <= tol):
        fails.append(f"{what}: aggregate gradient error {agg:.3e} > {tol:.3e}")


@pytest.mark.parametrize("tag", list(TRAIN_FIXTURES))
def test_train_step_vs_reference(tag):
    from semseg.losses import get_loss
    from irads import swin_fused  # noqa: F401  (the fused stage must be the path that runs)
    fx = Fixture(f"train_{tag}.npz")
    model, batch = _build(fx)
    loss_fn = get_loss("CrossEntropy", 255)
    report, fails = {}, []
    # eager step: also the BatchNorm running statistics of one training step
    bn = model.decode_head.linear_fuse.bn
    loss, y, yr, yd = _fwd_bwd(model, loss_fn, batch)
    torch.cuda.synchronize()
    _check(fx, model, loss, y, yr, yd, "eager", report, fails)
    e = _rel_l2(bn.running_mean.detach().cpu(), fx["bn_rm.decode_head"])
    report["eager.bn_running_mean_rel_l2"] = e
    if e > 1e-2:
        fails.append(f"head BN running mean relative L2 {e:.3e}")
    # graph replay, as bench.py / GraphedTrainStep run it.  The eager step's autograd graph is
    # released first: capturing while it is alive ended in a segfault inside capture_end
    # (hipGraphInstantiate) on ROCm 7.2 / torch 2.10; GraphedTrainStep never holds one.
    del loss, y, yr, yd
    torch.cuda.synchronize()
    params = [p for p in model.parameters() if p.requires_grad]
    side = torch.cuda.Stream(DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(side):
        for _ in range(2):
            for p in params:
                p.grad = None
            _fwd_bwd(model, loss_fn, batch)
    torch.cuda.current_stream(DEV).wait_stream(side)
    torch.cuda.synchronize()
    for p in params:
        p.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = _fwd_bwd(model, loss_fn, batch)
    g.replay()
    torch.cuda.synchronize()
    _check(fx, model, *out, "graph", report, fails)
    print(tag, {k: (round(v, 6) if isinstance(v, float) else v) for k, v in report.items()})
    assert not fails, fails
