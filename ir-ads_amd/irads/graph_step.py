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
  * gradients are allocated by the captured backward itself (no .grad before capture, so
    autograd hands each parameter its freshly computed gradient instead of adding it into a
    zeroed one: no per-parameter add kernels); with several ranks they are packed into one
    flat fp32 buffer inside the backward graph, all-reduced (RCCL sum, then 1/world) between the backward
    graph and the optimizer graph, and unpacked by the optimizer graph: one 30 MB bucket
    instead of DDP's per-bucket hooks (data-parallel semantics of train_mm.py:94 unchanged).
"""
import torch
import torch.distributed as dist


class GraphedTrainStep:
    """restore: tensors (parameters, BN buffers) to snapshot before the warm-up iterations and
    put back after capture, together with a zeroed optimizer state, so that the warm-up
    leaves no trace on the training run (train_mm.py); the bench keeps its warm-up updates."""

    def __init__(self, params, fwd_bwd, optimizer, world=1, warmup=3, before_capture=None, restore=None):
        self.params = [p for p in params if p.requires_grad]
        snap = None if restore is None else [(t, t.detach().clone()) for t in restore]
        self.world = world
        self.opt = optimizer
        dev = self.params[0].device
        self.flat = None
        if world > 1:
            self.flat = torch.zeros((sum(p.numel() for p in self.params),), device=dev, dtype=torch.float32)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # warm-up (kernel selection, allocator pools) off the capture
            for _ in range(warmup):
                optimizer.zero_grad(set_to_none=True)
                fwd_bwd()
                if world > 1:
                    self._pack()
                    dist.all_reduce(self.flat)
                    self._unpack()
                optimizer.step()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        optimizer.zero_grad(set_to_none=True)
        if before_capture is not None:
            before_capture()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.loss = fwd_bwd()
            if world == 1:
                optimizer.step()
            else:
                self._pack()
        self.opt_graph = None
        if world > 1:
            self.opt_graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.opt_graph, pool=self.graph.pool()):
                self._unpack()
                optimizer.step()
        if snap is not None:
            with torch.no_grad():
                for t, v in snap:
                    t.copy_(v)
                for st in optimizer.state.values():  # in place: the graph holds these addresses
                    for v in st.values():
                        if torch.is_tensor(v):
                            v.zero_()
            torch.cuda.synchronize(dev)

    def _pack(self):
        pack_grads(self.params, self.flat)

    def _unpack(self):
        unpack_grads(self.params, self.flat, 1.0 / self.world)

    def step(self):
        self.graph.replay()
        if self.opt_graph is not None:
            dist.all_reduce(self.flat)  # RCCL sum over xGMI; the optimizer graph scales by 1/world
            self.opt_graph.replay()
        return self.loss


def pack_grads(params, flat):
    """Concatenate the parameters' gradients (zeros for a missing one) into `flat`."""
    torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in params], out=flat)


def unpack_grads(params, flat, scale=1.0):
    """Write `scale * flat` back into the parameters' gradients (created where missing)."""
    if scale != 1.0:
        flat.mul_(scale)
    for p in params:
        if p.grad is None:
            p.grad = torch.zeros_like(p)
    views = torch.split(flat, [p.numel() for p in params])
    torch._foreach_copy_([p.grad for p in params], [v.view_as(p) for v, p in zip(views, params)])


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
