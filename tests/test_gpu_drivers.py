"""Drivers and metrics on the GPU: Metrics (semseg/metrics.py, irads_confusion_update)
against the reference's own tp/fp/fn/IoU fixture (exact integers), and a short
train_mm.py / val_mm.py run on the synthetic dataset (graph-captured training step,
evaluation, checkpoint round trip, multi-scale + flip evaluation)."""
import os

import numpy as np
import pytest
import torch
import yaml

from golden_util import Fixture

pytestmark = pytest.mark.gpu
DEV = "cuda"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("dtype,cl", [(torch.float32, False), (torch.bfloat16, True)])
def test_metrics_golden(dtype, cl):
    """Two updates (logits, flipped logits) as the fixture generator did with the reference
    Metrics (oracle/gen_golden.py): tp/fp/fn exact, IoU list and mIoU as the reference's."""
    from semseg.metrics import Metrics
    fx = Fixture("metrics_loss.npz")
    logits, gt = fx.t("logits", device=DEV), fx.t("gt", device=DEV)
    pre = ""
    if dtype == torch.bfloat16:
        # the fixture's bf16-exact twin: the reference scored the bf16-rounded logits, so the bf16
        # kernel sees the very same values (ties included) and must reproduce its integers
        pre = "bf16_"
    x = logits.to(dtype)
    xf = logits.flip(-1).to(dtype)
    if cl:
        x, xf = x.contiguous(memory_format=torch.channels_last), xf.contiguous(memory_format=torch.channels_last)
    m = Metrics(7, 255, DEV)
    m.update(x.softmax(dim=1) if dtype == torch.float32 else x, gt)
    m.update(xf.softmax(dim=1) if dtype == torch.float32 else xf, gt)
    assert m.tp == fx[pre + "tp"].tolist() and m.fp == fx[pre + "fp"].tolist() and m.fn == fx[pre + "fn"].tolist()
    ious, miou = m.compute_iou()
    np.testing.assert_allclose(ious, fx[pre + "ious"], rtol=0, atol=1e-12)
    assert miou == float(fx[pre + "miou"])
    m.reset()
    assert sum(m.tp) == 0


def test_metrics_edge_cases():
    """ignore pixels skipped; targets outside [0, C) that are not ignored still count as a
    false positive of the predicted class (reference: valid & pred == i & gt != i); ties
    go to the first class, NaN wins the arg-max as in torch.argmax."""
    from semseg.metrics import Metrics
    C = 3
    s = torch.tensor([[1., 0., 0.], [0., 2., 2.], [0., 0., 5.], [float('nan'), 9., 0.], [0., 1., 0.]], device=DEV)
    scores = s.t().reshape(1, C, 1, 5).contiguous()
    gt = torch.tensor([[[0, 1, 255, 2, 7]]], device=DEV)
    m = Metrics(C, 255, DEV)
    m.update(scores, gt)
    # pixel0: gt0 pred0 -> tp0; pixel1: gt1 pred1 (tie -> first) -> tp1; pixel2 ignored;
    # pixel3: gt2 pred0 (NaN) -> fp0, fn2; pixel4: gt7 (valid, out of range) pred1 -> fp1
    assert m.tp == [1, 1, 0] and m.fp == [1, 1, 0] and m.fn == [0, 0, 1]
    assert scores.argmax(1).flatten().tolist()[:4] == [0, 1, 2, 0]


def _cfg(tmp, **over):
    with open(os.path.join(ROOT, "configs", "nyu_rgbd.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["SAVE_DIR"] = str(tmp)
    cfg["DATASET"].update(NAME="Synthetic", LENGTH=8)
    cfg["TRAIN"].update(IMAGE_SIZE=[128, 128], BATCH_SIZE=4, EPOCHS=2, EVAL_START=0, EVAL_INTERVAL=1, WORKERS=0)
    cfg["EVAL"].update(IMAGE_SIZE=[128, 128], BATCH_SIZE=2)
    cfg["EVAL"]["MSF"].update(ENABLE=True, FLIP=True, SCALES=[0.5, 1.0])
    cfg["SCHEDULER"]["WARMUP"] = 1
    for k, v in over.items():
        cfg["TRAIN"][k] = v
    return cfg


@pytest.mark.parametrize("graph,amp,amp_dtype", [(True, True, "bf16"), (False, True, "bf16"), (True, False, "fp16"),
                                                 (False, True, "fp16")])
def test_train_and_val_drivers(tmp_path, graph, amp, amp_dtype):
    """2 epochs of train_mm.main + val_mm.main on the synthetic set in each numerics mode the YAML
    selects: bf16 autocast (graph / eager), fp32 (AMP false, graph) and the reference's fp16
    autocast + GradScaler (eager; train_mm.py:109-152)."""
    import train_mm
    import val_mm
    from pathlib import Path
    from semseg.utils.utils import get_logger
    torch.manual_seed(0)
    cfg = _cfg(tmp_path, GRAPH=graph, AMP=amp, AMP_DTYPE=amp_dtype)
    save = Path(tmp_path)
    best = train_mm.main(cfg, 0, save, get_logger(save / "train.log"))
    assert 0.0 <= best <= 100.0
    ckpts = sorted(p for p in os.listdir(save) if p.endswith("_checkpoint.pth"))
    assert len(ckpts) == 1
    ck = torch.load(save / ckpts[0], map_location="cpu", weights_only=True)
    assert set(ck) == {"epoch", "model_state_dict", "optimizer_state_dict", "loss", "scheduler_state_dict",
                       "best_miou"}
    assert np.isfinite(ck["loss"])
    weights = [p for p in os.listdir(save) if p.endswith(".pth") and "checkpoint" not in p][0]
    cfg["EVAL"]["MODEL_PATH"] = str(save / weights)
    (miou,) = val_mm.main(cfg)
    assert 0.0 <= miou <= 100.0
    assert any(p.startswith("eval_") for p in os.listdir(save))


def _tiny_model(n_cls=5):
    """Tiny-Swin CMNeXt (embed 32, head_dim 32; the fixture model of test_gpu_swin.py)."""
    from semseg.models.backbones.swin import SwinTransformer
    from semseg.models.heads import SegFormerHead
    from semseg.models.cmnext import CMNeXt

    class Tiny(torch.nn.Module):
        def forward(self, x):
            return CMNeXt.forward(self, x)
    h = Tiny()
    h.sb_cfg = None
    h.backbone = SwinTransformer(embed_dims=32, depths=(2, 2, 2, 2), num_heads=(1, 2, 4, 8), init_cfg=None)
    dims = [32, 64, 128, 256]
    h.decode_head = SegFormerHead(dims, 64, n_cls)
    h.decode_head_rgb = SegFormerHead(dims, 32, n_cls)
    h.decode_head_dte = SegFormerHead(dims, 32, n_cls)
    return h


def test_graph_step_keeps_optimizer_state(tmp_path):
    """GraphedTrainStep(restore=...) (train_mm.py's resume path) puts the optimizer state back as it
    was before its warm-up: a resumed run keeps its Adam moments and step counts, and a
    learning rate loaded as a CPU tensor is moved to the device for the captured AdamW."""
    from fill import fill_module
    from irads.graph_step import GraphedTrainStep, lr_to_device
    from semseg.losses import get_loss, mmst_loss
    from semseg.optimizers import get_optimizer
    torch.manual_seed(0)
    m = _tiny_model().to(DEV)
    fill_module(m, seed=3)
    opt = get_optimizer(m, "adamw", 1e-4, "Adapter", 0.01, lr_on_device=True)
    loss_fn = get_loss("CrossEntropy", 255)
    m.train()
    rgb, dep = torch.randn(4, 3, 64, 96, device=DEV), torch.rand(4, 3, 64, 96, device=DEV)
    lbl = torch.randint(0, 5, (4, 64, 96), device=DEV)

    def fwd_bwd():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y, yr, yd = m([rgb, dep])
            loss = mmst_loss(loss_fn, y, yr, yd, lbl)
        loss.backward()
        return loss
    for _ in range(2):  # the "checkpointed" run: some optimizer state
        opt.zero_grad(set_to_none=True)
        fwd_bwd()
        opt.step()
    sd = opt.state_dict()
    torch.save(sd, tmp_path / "opt.pth")
    sd = torch.load(tmp_path / "opt.pth", map_location="cpu", weights_only=True)  # lr comes back on the CPU
    opt.load_state_dict(sd)
    lr_to_device(opt, torch.device(DEV))
    assert all(g["lr"].device.type == "cuda" for g in opt.param_groups)
    want = {i: {k: v.clone() for k, v in st.items()} for i, st in sd["state"].items()}
    params = [p for p in m.parameters() if p.requires_grad]
    keep = params + list(m.buffers())
    GraphedTrainStep(m.parameters(), fwd_bwd, opt, warmup=2, restore=keep)
    for i, p in enumerate(params):
        st = opt.state[p]
        for k in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(st[k].cpu(), want[i][k].cpu()), (i, k)


@pytest.mark.gpu
def test_sb_hook_step():
    """The build-defined SB hook (CMNeXt(..., sb=...)): in one bf16 training step the
    hook's loss equals LightSB's objective E[log C(x)] - E[log v(x)] recomputed by the oracle in
    fp64 on the same fused head feature rows, and its parameter gradients equal the oracle's
    autograd gradients (relative 1e-3; the kernels run in fp32)."""
    import irads_ref as R
    from semseg.models import CMNeXt
    from semseg.losses import get_loss, mmst_loss
    from semseg.optimizers import get_optimizer
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    m = CMNeXt("SwinTransformer-B", 5, ["img", "depth"], sb={"weight": 0.5, "n_potentials": 10, "epsilon": 0.1})
    m = m.to(dev)
    opt = get_optimizer(m, "adamw", 1e-4, "Adapter", 0.01)
    names = {id(p): n for n, p in m.named_parameters()}
    assert {names[id(p)] for g in opt.param_groups for p in g["params"] if names[id(p)].startswith("sb.")} == \
        {"sb.r", "sb.S_log_diagonal_matrix", "sb.log_alpha_raw"}
    m.train()
    rgb = torch.randn(4, 3, 128, 128, device=dev)
    dep = torch.rand(4, 3, 128, 128, device=dev)
    lbl = torch.randint(0, 5, (4, 128, 128), device=dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y, yr, yd = m([rgb, dep])
        seg = mmst_loss(get_loss("CrossEntropy", 255), y, yr, yd, lbl)
        sbl = m.sb_loss()
    (seg + sbl).backward()
    x = m._sb_rows().double().cpu()
    assert x.shape == (4 * 32 * 32, 512)
    r = m.sb.r.detach().double().cpu().requires_grad_()
    Sl = m.sb.S_log_diagonal_matrix.detach().double().cpu().requires_grad_()
    la = m.sb.log_alpha_raw.detach().double().cpu().requires_grad_()
    eps = float(m.sb.epsilon)
    log_c = R.lightsb_log_C(x, r, Sl, la, eps)
    var = eps * torch.exp(Sl)
    comp = -0.5 * (((x[:, None, :] - r[None]) ** 2) / var[None] + torch.log(2 * np.pi * var)[None]).sum(-1)
    log_v = torch.logsumexp(comp + la[None] / eps, -1)  # log_softmax(log alpha) + logsumexp(log alpha)
    ref = 0.5 * (log_c.mean() - log_v.mean())
    assert abs(float(sbl) - float(ref)) <= 1e-3 * abs(float(ref)) + 1e-4, (float(sbl), float(ref))
    gr = torch.autograd.grad(ref, [r, Sl, la])
    for got, want, nm in zip((m.sb.r.grad, m.sb.S_log_diagonal_matrix.grad, m.sb.log_alpha_raw.grad), gr,
                             ("r", "S_log", "log_alpha_raw")):
        e = float((got.double().cpu() - want).norm() / want.norm())
        assert e < 1e-3, (nm, e)
    amap = m.sb_anomaly_map()
    assert amap.shape == (4, 32, 32) and torch.isfinite(amap).all()


@pytest.mark.parametrize("mode,kind", [("split", "tiny"), ("overlap", "tiny"), ("overlap", "c3")])
def test_dp_two_ranks_gradients(tmp_path, mode, kind):
    """Data parallel at model level (north_star: per-image batch sharded over GPUs, gradients
    all-reduced): 2 fresh processes, one per rank (gloo, on the one GPU of the box), each run
    GraphedTrainStep on half of a 4-image batch, with the captured split exchange or the
    overlapped bucketed one (tests/_dp_worker.py); rank 0's averaged gradients equal a
    single-process 4-image step's.  fp32 with deterministic MIOpen solvers, so the only
    difference left is GEMM tiling of batch 2 against batch 4: relative L2 1e-4 over all
    trainable tensors.  kind "c3" is BASELINE config C3's model and per-GPU share (Swin-B, 512x512,
    2 classes, 4 images per rank, 8 in the single-process reference)."""
    import subprocess
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _dp_worker as W
    out = str(tmp_path / "grads.pt")
    port = str(29600 + (os.getpid() + 101 * (mode == "overlap") + 211 * (kind == "c3")) % 300)
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_dp_worker.py"), str(r), "2", port, out, mode,
                               kind],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(2)]
    try:
        logs = [p.communicate(timeout=200)[0].decode()[-2000:] for p in procs]
    finally:
        for p in procs:  # our own children only
            if p.poll() is None:
                p.kill()
                p.wait()
    assert all(p.returncode == 0 for p in procs), logs
    got = torch.load(out, weights_only=True)
    dev = torch.device("cuda", 0)
    det = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        m = W.model(dev, kind)
        rgb, dep, lbl = W.batch(dev, kind)
        W.fwd_bwd_fn(m, rgb, dep, lbl)()
    finally:
        torch.backends.cudnn.deterministic = det
    # the aux heads' parameters get no gradient from the fused-logit loss (None here, zeros in the graph)
    want = {n: (p.grad if p.grad is not None else torch.zeros_like(p)).detach().cpu()
            for n, p in m.named_parameters() if p.requires_grad}
    assert set(got) == set(want)
    num = sum(float((got[n] - want[n]).double().norm() ** 2) for n in want)
    den = sum(float(want[n].double().norm() ** 2) for n in want)
    rel = (num / den) ** 0.5
    print(f"dp {mode} {kind}: relative L2 vs single process {rel:.3e}")
    assert rel < 1e-4, rel


def test_evaluate_msf_matches_reference():
    """val_mm.evaluate_msf (multi-scale + flip evaluation, the path the +-0.2 mIoU target is
    measured on) against the reference's evaluate_msf (val_mm.py:87-120) on the tiny fp32 CMNeXt:
    configs/nyu_rgbd.yaml's six scales with flip, two images one per batch (msf_eval.npz,
    oracle/gen_golden.py gen_msf).  The summed probabilities that reach Metrics.update within
    2e-5 of the reference (12 softmaxes of an fp32 model, CPU vs GPU summation order), the
    argmax identical wherever the reference's top-2 margin exceeds 1e-3, and the IoUs equal."""
    import val_mm
    from fill import fill_module
    from msf_case import MSF_CASE, msf_inputs
    from semseg.metrics import Metrics
    fx = Fixture("msf_eval.npz")
    c = MSF_CASE
    m = _tiny_model(c["n_cls"]).cuda()
    assert sorted(m.state_dict().keys()) == fx["state_keys"].tolist()
    fill_module(m, seed=c["fill_seed"])
    rgb, dep, lbl = (torch.from_numpy(a) for a in msf_inputs())
    seen = []

    class RecMetrics(Metrics):
        def update(self, pred, target):
            seen.append(pred.detach().float().cpu())
            return super().update(pred, target)

    class Loader(list):
        dataset = type("D", (), {"n_classes": c["n_cls"], "ignore_label": 255})
    loader = Loader([([rgb[i:i + 1], dep[i:i + 1]], lbl[i:i + 1]) for i in range(c["B"])])
    orig, amp = val_mm.Metrics, dict(val_mm._AMP)
    val_mm.Metrics = RecMetrics
    val_mm._AMP["dtype"] = None  # fp32, as the reference evaluates
    try:
        acc, macc, f1, mf1, ious, miou = val_mm.evaluate_msf(m, loader, torch.device("cuda"), list(c["scales"]),
                                                             c["flip"])
    finally:
        val_mm.Metrics = orig
        val_mm._AMP.update(amp)
    probs = torch.cat(seen)
    ref = torch.from_numpy(fx["probs"])
    err = float((probs - ref).abs().max())
    decided = torch.from_numpy(fx["margin"]) > 1e-3
    agree = float((probs.argmax(1) == torch.from_numpy(fx["argmax"]).long())[decided].float().mean())
    print(f"msf: max |dprob| {err:.2e}, argmax agreement on decided pixels {agree}, miou {miou} vs {float(fx['miou'])}")
    assert err <= 2e-5, err
    assert agree == 1.0
    assert np.allclose(np.asarray(ious, dtype=np.float64), fx["ious"], rtol=0, atol=1e-9), (ious, fx["ious"])
    assert float(miou) == float(fx["miou"])


def test_val_driver_c1_msf_settings(tmp_path):
    """C1 as configured: val_mm.main with configs/nyu_rgbd.yaml's evaluation settings unchanged
    (480x640, batch 1, MSF on with scales 0.5-1.75 and flip, Swin-B, fp32), on two synthetic
    RGB-D images (no dataset offline) and a freshly initialised, saved model."""
    import val_mm
    from fill import fill_module
    from semseg.models import CMNeXt
    with open(os.path.join(ROOT, "configs", "nyu_rgbd.yaml")) as f:
        cfg = yaml.safe_load(f)
    assert cfg["EVAL"]["IMAGE_SIZE"] == [480, 640] and cfg["EVAL"]["MSF"]["ENABLE"]
    assert cfg["EVAL"]["MSF"]["SCALES"] == [0.5, 0.75, 1.0, 1.25, 1.5, 1.75] and cfg["EVAL"]["MSF"]["FLIP"]
    cfg["SAVE_DIR"] = str(tmp_path)
    cfg["DATASET"].update(NAME="Synthetic", LENGTH=2)
    m = CMNeXt(cfg["MODEL"]["BACKBONE"], 40, cfg["DATASET"]["MODALS"])
    fill_module(m, seed=5)
    path = tmp_path / "model.pth"
    torch.save(m.state_dict(), path)
    cfg["EVAL"]["MODEL_PATH"] = str(path)
    (miou,) = val_mm.main(cfg)
    assert 0.0 <= miou <= 100.0
