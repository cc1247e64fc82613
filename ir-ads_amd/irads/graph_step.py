"""One training iteration captured into a HIP graph.

The eager step issues ~3000 kernel launches (the Swin trunk, the fusion blocks, the heads,
AdamW) from Python; on MI355X their GPU time is ~45 ms per step while the host needs about
as long to issue them, so the eager step is launch-bound.  Capturing the iteration once and
replaying it removes the host from the loop: one hipGraphLaunch per step.

What makes the step capturable (all in this package):
  * every irads kernel takes torch's current stream and allocates nothing (C-ABI contract,
    include/irads.h), so capture records it like any aten kernel;
  * randomness is drawn on the device from torch's generator (DropPath, the Adapter's
    dropout seed, apply_mask's image choice): each replay advances the Philox offset and
    draws fresh values, as the eager step does;
  * the learning rate is a device tensor that the host-side scheduler fills between replays
    (fused AdamW reads it on the device);
  * gradients live in one flat fp32 buffer (each trainable parameter's .grad is a view of
    it), zeroed inside the graph; with several ranks the buffer is all-reduced (RCCL, AVG)
    between the backward graph and the optimizer graph, i.e. one bucket of 30 MB instead of
    DDP's per-bucket hooks (data-parallel semantics of train_mm.py:94 unchanged).
"""
import torch
import torch.distributed as dist


class GraphedTrainStep:
    def __init__(self, params, fwd_bwd, optimizer, world=1, warmup=3, before_capture=None):
        self.params = [p for p in params if p.requires_grad]
        self.world = world
        self.opt = optimizer
        dev = self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.flat = torch.zeros((total,), device=dev, dtype=torch.float32)
        off = 0
        for p in self.params:
            n = p.numel()
            p.grad = self.flat[off:off + n].view_as(p)
            off += n
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # warm-up (kernel selection, allocator pools) off the capture
            for _ in range(warmup):
                self.flat.zero_()
                fwd_bwd()
                self._allreduce()
                optimizer.step()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        if before_capture is not None:
            before_capture()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.flat.zero_()
            self.loss = fwd_bwd()
            if world == 1:
                optimizer.step()
        self.opt_graph = None
        if world > 1:
            self.opt_graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.opt_graph, pool=self.graph.pool()):
                optimizer.step()

    def _allreduce(self):
        if self.world > 1:
            dist.all_reduce(self.flat, op=dist.ReduceOp.AVG)

    def step(self):
        self.graph.replay()
        if self.opt_graph is not None:
            self._allreduce()
            self.opt_graph.replay()
        return self.loss


def events_capturable(device):
    """Whether HIP event records inside a captured graph time correctly on this stack."""
    try:
        x = torch.zeros(1 << 20, device=device)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        side = torch.cuda.Stream(device=device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            x.add_(1)
        torch.cuda.current_stream(device).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            a.record()
            x.add_(1)
            b.record()
        g.replay()
        torch.cuda.synchronize(device)
        return a.elapsed_time(b) >= 0.0
    except Exception:
        return False
