"""vCLR DINO deformable transformer (encoder + two-stage selection + decoder) on the HIP MSDA,
against the reference's own modules (projects/vCLR_deformable_mask/modeling/dino_transformer.py
on reference detrex layers, CPU fp64), fixture tests/golden/dino_transformer.npz made by
oracle/gen_golden.py `dino` from the seeded inputs of oracle/dino_case.py.

The case keeps C5's architecture (6 + 6 layers, d = 256, 8 heads, 4 levels x 4 points, FFN 1024,
4-d reference boxes in the decoder, a padded second image, CDN attention mask) at reduced
spatial size (levels 10x14 ... 2x2, 30 proposals + 10 denoising queries).  Dropout is off (eval).
"""
import numpy as np
import pytest
import torch

from dino_case import DINO_LAYERS, DINO_LEVELS, DINO_PROPOSALS, dino_inputs
from fill import seeded
from golden_util import Fixture, checksum

pytestmark = pytest.mark.gpu
DEV = "cuda"
NAMES = ("inter_states", "init_reference", "inter_references", "target_unact", "topk_coords", "memory")


def _rel(a, b):
    a = a.detach().double().cpu()
    b = torch.as_tensor(b).double()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def _model(dtype):
    from fill import fill_module
    from projects.vCLR_deformable_mask.modeling import (DINOTransformer, DINOTransformerDecoder,
                                                        DINOTransformerEncoder, attach_detection_heads)
    torch.manual_seed(0)
    tr = DINOTransformer(DINOTransformerEncoder(num_layers=DINO_LAYERS), DINOTransformerDecoder(num_layers=DINO_LAYERS),
                         num_feature_levels=4, two_stage_num_proposals=DINO_PROPOSALS)
    attach_detection_heads(tr, num_classes=1)
    fill_module(tr, seed=9)
    return tr.to(DEV, dtype).eval()


def _run(dtype):
    fx = Fixture("dino_transformer.npz")
    tr = _model(dtype)
    feats, masks, dn_label, dn_box, attn = dino_inputs(torch.float64)
    feats = [f.to(DEV, dtype).requires_grad_() for f in feats]
    masks = [m.to(DEV) for m in masks]
    pos = [fx.t(f"pos_{i}", dtype, DEV) for i in range(4)]
    dn_label = dn_label.to(DEV, dtype).requires_grad_()
    outs = tr(feats, masks, pos, (dn_label, dn_box.to(DEV, dtype)), attn.to(DEV))
    gouts = [torch.from_numpy(seeded(tuple(o.shape), 60 + i)).to(DEV, dtype) for i, o in enumerate(outs)]
    loss = sum((o * g).sum() for o, g in zip(outs, gouts) if o.requires_grad)
    params = list(tr.named_parameters())
    grads = torch.autograd.grad(loss, feats + [dn_label] + [p for _, p in params], allow_unused=True)
    return fx, tr, outs, loss, grads, params


def test_position_embedding_sine_matches_reference():
    """detrex PositionEmbeddingSine (normalize, offset -0.5: the DINO config) on the padded masks."""
    from detrex.layers import PositionEmbeddingSine
    fx = Fixture("dino_transformer.npz")
    pe = PositionEmbeddingSine(num_pos_feats=128, temperature=10000, normalize=True, offset=-0.5)
    _, masks, _, _, _ = dino_inputs()
    for i, m in enumerate(masks):
        got = pe(m.to(DEV))
        assert got.shape == fx[f"pos_{i}"].shape
        err = np.abs(got.cpu().double().numpy() - fx[f"pos_{i}"])
        # Valid positions: fp32 sin/cos of arguments within [-π, 2π] agree to a few ulp.  At padded
        # positions the reference normalises 0 - 0.5 by eps = 1e-6 (arguments ~ -3e6), where fp32
        # sin/cos is ill-conditioned and host / device range reduction legitimately differ; those
        # rows are masked out of every attention value and proposal.
        valid = ~m.numpy()[:, None]
        assert err[np.broadcast_to(valid, err.shape)].max() < 1e-5, (i, err.max())


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32], ids=["fp64", "fp32"])
def test_dino_transformer_forward_backward(dtype):
    """Outputs, input gradients and every parameter gradient vs the reference.

    Tolerances (relative L2): fp64 1e-6 (the reference builds some constants in fp32 whatever
    the model dtype: linspace grids, the sine-embedding frequencies 10000^(2i/128) via fp32 pow,
    so host and device libm differ by an fp32 ulp there); fp32 outputs 1e-4 and
    gradients 2e-3 (six post-norm layers of fp32 GEMMs + the fp32 MSDA kernels; the
    fp32 rounding of 12 stacked LayerNorms is the error floor).  The two-stage top-k
    selection must pick the same proposals in the same order.
    """
    fx, tr, outs, loss, grads, params = _run(dtype)
    to, tg = (1e-6, 1e-6) if dtype == torch.float64 else (1e-4, 2e-3)
    with torch.no_grad():
        nl = tr.decoder.num_layers
        mask = torch.cat([m.flatten(1) for m in dino_inputs()[1]], 1).to(DEV)
        om, _ = tr.gen_encoder_output_proposals(outs[5], mask, torch.as_tensor(DINO_LEVELS, device=DEV))
        topk = torch.topk(tr.decoder.class_embed[nl](om).max(-1)[0], DINO_PROPOSALS, dim=1)[1]
    assert np.array_equal(topk.cpu().numpy(), fx["topk_index"]), "two-stage proposal selection differs"
    for n, o in zip(NAMES, outs):
        assert _rel(o, fx[n]) < to, (n, _rel(o, fx[n]))
    assert abs(loss.item() - float(fx["loss"])) <= to * 10 * abs(float(fx["loss"]))
    for i in range(4):
        assert _rel(grads[i], fx[f"gfeat_{i}"]) < tg, (i, _rel(grads[i], fx[f"gfeat_{i}"]))
    assert _rel(grads[4], fx["gdn_label"]) < tg
    nfull = 0
    for (n, p), g in zip(params, grads[5:]):
        g = torch.zeros_like(p) if g is None else g
        cs, ref = checksum(g.detach().double().cpu().numpy()), fx["gcs." + n]
        # L2 norm from the sum of squares, and the signed sum against the abs-sum scale
        assert abs(np.sqrt(cs[2]) - np.sqrt(ref[2])) <= tg * np.sqrt(ref[2]) + 1e-30, (n, cs, ref)
        assert abs(cs[0] - ref[0]) <= tg * ref[1] + 1e-30, (n, cs, ref)
        if "g." + n in fx:
            nfull += 1
            assert _rel(g, fx["g." + n]) < tg, (n, _rel(g, fx["g." + n]))
    assert nfull == 6


def test_dino_msda_runs_on_hip_kernels(monkeypatch):
    """Every MSDA call of the stack (6 encoder self-attn + 6 decoder cross-attn) goes through
    libirads.so's MSDA entry points (no PyTorch sampling path)."""
    from irads import native as N
    calls = []
    real = N.call

    def spy(name, *a):
        calls.append(name)
        return real(name, *a)

    monkeypatch.setattr(N, "call", spy)
    _run(torch.float32)
    assert calls.count("irads_msda_fwd") == 2 * DINO_LAYERS
    assert calls.count("irads_msda_bwd_gather") + calls.count("irads_msda_bwd") == 2 * DINO_LAYERS
