"""Worker of test_gpu_drivers.py::test_dp_two_ranks_gradients (one process per rank, both on the
one GPU of the box): the training step of irads/graph_step.py with world = 2 over gloo, on this
rank's half of the batch (SHAPES), in fp32 with deterministic MIOpen solvers.  mode "split": the
graph-captured step (pack, one all-reduce between the backward and the optimizer graphs); mode
"overlap": the bucketed exchange from post-accumulate-grad hooks (OverlappedGradExchange, the
RCCL path's code with gloo collectives; eager, as gloo cannot be captured), >= 4 buckets.
Writes rank 0's averaged gradients."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "ir-ads_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


# kind "tiny": the tiny-Swin CMNeXt on 4 images of 64x96 (2 per rank); kind "c3": BASELINE config C3's
# model and per-GPU share, CMNeXt('SwinTransformer-B', 2 classes, ['img', 'hha']) on 8 images of 512x512
# (4 per rank, as C3's 32 over 8 GPUs)
SHAPES = {"tiny": (4, 64, 96, 5), "c3": (8, 512, 512, 2)}


def batch(dev, kind="tiny"):
    import torch
    n, H, W, ncls = SHAPES[kind]
    g = torch.Generator().manual_seed(11)
    rgb = torch.randn(n, 3, H, W, generator=g)
    dep = torch.rand(n, 3, H, W, generator=g)
    lbl = torch.randint(0, ncls, (n, H, W), generator=g)  # no ignore pixels: per-rank means average exactly
    return rgb.to(dev), dep.to(dev), lbl.to(dev)


def model(dev, kind="tiny"):
    from fill import fill_module
    if kind == "c3":
        from semseg.models import CMNeXt
        m = CMNeXt("SwinTransformer-B", 2, ["img", "hha"]).to(dev)
    else:
        from test_gpu_drivers import _tiny_model
        m = _tiny_model().to(dev)
    fill_module(m, seed=4)
    for n, p in m.named_parameters():
        p.requires_grad_(("Adapter" in n) or ("extra_patch_embed" in n) or ("head" in n) or ("MPG" in n))
    m.eval()  # deterministic (BN running stats, no dropout / DropPath / apply_mask): per-image independent
    return m


def fwd_bwd_fn(m, rgb, dep, lbl):
    import torch

    def fwd_bwd():
        y = m([rgb, dep])[0]
        loss = torch.nn.functional.cross_entropy(y.float(), lbl)
        loss.backward()
        return loss
    return fwd_bwd


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    mode = sys.argv[5] if len(sys.argv) > 5 else "split"
    kind = sys.argv[6] if len(sys.argv) > 6 else "tiny"
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = port
    import datetime
    import torch
    import torch.distributed as dist
    # a peer that dies surfaces as a collective timeout well inside the test's own bound
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
    from irads.graph_step import GraphedTrainStep
    torch.backends.cudnn.deterministic = True
    dev = torch.device("cuda", 0)
    m = model(dev, kind)
    rgb, dep, lbl = batch(dev, kind)
    per = rgb.shape[0] // world
    half = slice(rank * per, rank * per + per)
    opt = torch.optim.SGD([p for p in m.parameters() if p.requires_grad], lr=0.0)
    if mode == "split":
        step = GraphedTrainStep(m.parameters(), fwd_bwd_fn(m, rgb[half], dep[half], lbl[half]), opt, world=world,
                                warmup=1)
        assert step.comm == "split"
    else:
        step = GraphedTrainStep(m.parameters(), fwd_bwd_fn(m, rgb[half], dep[half], lbl[half]), opt, world=world,
                                comm="overlap", bucket_mb=0.02 if kind == "tiny" else 4.0, graph=False)
        assert len(step._buckets) >= 4, len(step._buckets)
    step.step()
    if mode == "overlap":
        assert step._exchange.issue_log == list(range(len(step._buckets)))
    torch.cuda.synchronize()
    if rank == 0:
        torch.save({n: (p.grad if p.grad is not None else torch.zeros_like(p)).detach().cpu()
                    for n, p in m.named_parameters() if p.requires_grad}, out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
