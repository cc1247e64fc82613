"""Which gradients of the C2 training step differ between two identical eager backward passes:
the bench model (eval mode: no dropout / DropPath / apply_mask draws), one batch, fwd + bwd
twice from the same state, per-parameter bitwise comparison, listed in backward order (the
order the gradients become final), so that the first differing tensor points at the first
non-reproducible kernel.

    python scripts/determinism_probe.py [--batch 2]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ir-ads_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--det-conv", action="store_true", help="torch.backends.cudnn.deterministic (MIOpen)")
    a = ap.parse_args()
    torch.backends.cudnn.deterministic = a.det_conv
    dev = torch.device("cuda", 0)
    torch.manual_seed(3407)
    model, opt, sched, loss_fn = bench.build(dev, 1, 0, 1000)
    model.eval()
    batch = bench.synthetic_batch(a.batch, 512, dev, 3407)
    order = []
    hooks = [p.register_post_accumulate_grad_hook(lambda p, n=n: order.append(n))
             for n, p in model.named_parameters() if p.requires_grad]
    grads = []
    for _ in range(2):
        order.clear()
        model.zero_grad(set_to_none=True)
        bench.fwd_bwd(model, loss_fn, batch)
        torch.cuda.synchronize()
        grads.append({n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None})
    for h in hooks:
        h.remove()
    g0, g1 = grads
    # the forward alone: logits of two identical forward passes
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        outs = [model([batch[0], batch[1]]) for _ in range(2)]
    for i, (u, v) in enumerate(zip(*outs)):
        print(f"forward output {i}: bit-identical {torch.equal(u, v)}, max |diff| {float((u - v).abs().max()):.3e}")
    # the first module (execution order) whose output differs while its tensor inputs agree
    rec = [[], []]
    cur = [0]

    def hook(mod, inp, out, name=None):
        ti = [t.detach().clone() for t in inp if torch.is_tensor(t)]
        to = out if torch.is_tensor(out) else (out[0] if isinstance(out, (tuple, list)) and out
                                                and torch.is_tensor(out[0]) else None)
        rec[cur[0]].append((name, ti, None if to is None else to.detach().clone()))
    hs = [m.register_forward_hook(lambda mod, i, o, n=n: hook(mod, i, o, n)) for n, m in model.named_modules() if n]
    for k in range(2):
        cur[0] = k
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            model([batch[0], batch[1]])
        torch.cuda.synchronize()
    for h in hs:
        h.remove()
    for (n, i0, o0), (_, i1, o1) in zip(*rec):
        same_in = len(i0) == len(i1) and all(torch.equal(u, v) for u, v in zip(i0, i1))
        same_out = o0 is None or torch.equal(o0, o1)
        if same_in and not same_out:
            print("first module with equal inputs and differing output:", n, type(dict(model.named_modules())[n]).__name__)
            break
    # every bf16 GEMM shape of the step, run twice (hipBLASLt's stream-K kernels reduce tiles with atomics)
    torch.backends.cuda.matmul.allow_bf16_reduced_precision_reduction = True
    xs = torch.randn(8 * 128 * 128, 512, device=dev, dtype=torch.bfloat16)
    w = torch.randn(128, 512, device=dev, dtype=torch.bfloat16)
    r0, r1 = xs @ w.t(), xs @ w.t()
    print("bf16 GEMM 131072x128x512 twice: bit-identical", torch.equal(r0, r1))
    diff = [n for n in order if not torch.equal(g0[n], g1[n])]
    print(f"{len(order)} gradients, {len(diff)} differ between two identical backward passes")
    first = order.index(diff[0]) if diff else None
    print("first differing (backward order index):", first, diff[0] if diff else None)
    for n in diff[:12]:
        r = float((g0[n] - g1[n]).float().norm() / g0[n].float().norm().clamp_min(1e-30))
        print(f"  {n:70s} rel {r:.2e}")
    same_before = order[:first] if diff else order
    print(f"{len(same_before)} gradients before the first difference are bit-identical; last of them:",
          same_before[-3:])


if __name__ == "__main__":
    main()
