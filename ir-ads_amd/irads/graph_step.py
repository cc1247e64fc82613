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
    zeroed one: no per-parameter add kernels).

Data parallel (world > 1; train_mm.py:94 / DDP semantics: gradients averaged over ranks):
  * comm="overlap" (default with the RCCL backend): the trainable parameters are split into
    buckets of ~bucket_mb in reverse registration order (the order their gradients become
    final in backward, as DDP's buckets).  A post-accumulate-grad hook copies each gradient
    into its slot of a flat fp32 buffer; when a bucket's last gradient lands, the bucket's
    all-reduce (RCCL sum) is issued on a side stream that waits on an event recorded at that
    point of the backward, so the exchange of bucket k overlaps the backward of the layers
    below it.  The optimizer waits for the side stream, unpacks with the 1/world scale and
    steps.  Hooks, events, collectives and the optimizer are captured into the one graph.
  * comm="split": the backward graph packs the gradients, one all-reduce of the flat buffer
    runs between the backward graph and the optimizer graph (no overlap; the collective is
    not captured).  Used with the gloo backend (CPU-side tests), which cannot be captured.
"""
import os

import torch
import torch.distributed as dist


def rccl_capture_env():
    """Process-group settings for capturing RCCL collectives into a HIP graph; call before
    init_process_group (they are read when the group is built; an explicit value is kept).
    Observed here: ProcessGroupNCCL's watchdog thread aborted the process with a HIP error from
    hipEventQuery on a collective's end event (WorkNCCL::finishedGPUExecutionInternal, stack
    captured by tests/test_gpu_zz_rccl.py) between the capture of the overlapped exchange and the
    first replay — the events of captured collectives are graph nodes, not recorded events, and
    the watchdog's event cache can hand a captured event to an eager work.  So: no event cache,
    and a watchdog that logs HIP errors instead of rethrowing them (a real device fault still
    surfaces on the main thread's next synchronising call)."""
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    os.environ.setdefault("TORCH_NCCL_RETHROW_CUDA_ERRORS", "0")

# "thread_local": only the capturing thread's capture-unsafe HIP calls are refused.  In the
# default "global" mode a call from any thread of the process fails while a capture is open,
# and a process with an RCCL communicator has threads of its own (RCCL's proxy thread, the
# process group's watchdog) that poll events and streams at any time: a poll that lands inside
# the capture window gets an error it treats as fatal.  Kernel launches from the autograd
# thread onto the capturing stream are still recorded (capture is per stream).
CAPTURE_MODE = "thread_local"


class GraphedTrainStep:
    """restore: tensors (parameters, BN buffers) to snapshot before the warm-up iterations and
    put back after capture, together with the optimizer state as it was before the warm-up
    (a resumed run keeps its Adam moments and step counts; a fresh one starts from zero), so
    that the warm-up leaves no trace on the training run (train_mm.py); the bench keeps its
    warm-up updates."""

    def __init__(self, params, fwd_bwd, optimizer, world=1, warmup=3, before_capture=None, restore=None,
                 comm=None, bucket_mb=8.0):
        self.params = [p for p in params if p.requires_grad]
        self.world = world
        self.opt = optimizer
        dev = self.params[0].device
        snap = None if restore is None else [(t, t.detach().clone()) for t in restore]
        opt_snap = _snapshot_optimizer(optimizer) if restore is not None else None
        if comm is None:
            comm = "none" if world == 1 else ("overlap" if dist.get_backend() == "nccl" else "split")
        self.comm = comm  # an explicit "overlap" / "split" also runs at world == 1 (tests)
        self.flat = None
        if self.comm != "none":
            self.flat = torch.zeros((sum(p.numel() for p in self.params),), device=dev, dtype=torch.float32)
            self._offsets = []
            o = 0
            for p in self.params:
                self._offsets.append(o)
                o += p.numel()
            if self.comm == "overlap":
                self._make_buckets(bucket_mb)
        if self.comm != "none":
            # first collective from this (the main) thread, before the backward's hooks issue
            # them from the autograd thread: the communicator's lazy set-up happens here
            w = torch.zeros((1,), device=dev, dtype=torch.float32)
            _all_reduce(w)
            torch.cuda.synchronize(dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # warm-up (kernel selection, allocator pools) off the capture
            for _ in range(warmup):
                optimizer.zero_grad(set_to_none=True)
                self._run(fwd_bwd, capture=False)
                optimizer.step()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        optimizer.zero_grad(set_to_none=True)
        if before_capture is not None:
            before_capture()
        self.graph = torch.cuda.CUDAGraph()
        self.opt_graph = None
        if self.comm == "split":
            with torch.cuda.graph(self.graph, capture_error_mode=CAPTURE_MODE):
                self.loss = fwd_bwd()
                pack_grads(self.params, self.flat)
            self.opt_graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.opt_graph, pool=self.graph.pool(), capture_error_mode=CAPTURE_MODE):
                unpack_grads(self.params, self.flat, 1.0 / self.world)
                optimizer.step()
        else:
            with torch.cuda.graph(self.graph, capture_error_mode=CAPTURE_MODE):
                self.loss = self._run(fwd_bwd, capture=True)
                optimizer.step()
        if snap is not None:
            with torch.no_grad():
                for t, v in snap:
                    t.copy_(v)
                _restore_optimizer(optimizer, opt_snap)
            torch.cuda.synchronize(dev)

    # ------------------------------------------------------------------ overlapped exchange
    def _make_buckets(self, bucket_mb):
        """Buckets of consecutive params in reverse registration order, ~bucket_mb each."""
        limit = int(bucket_mb * (1 << 20) / 4)
        order = list(range(len(self.params)))[::-1]
        self._bucket_of = {}
        self._buckets = []  # (lo, hi) element range of the flat buffer, param indices
        cur, size = [], 0
        for i in order:
            cur.append(i)
            size += self.params[i].numel()
            if size >= limit:
                self._buckets.append(cur)
                cur, size = [], 0
        if cur:
            self._buckets.append(cur)
        for b, idx in enumerate(self._buckets):
            for i in idx:
                self._bucket_of[i] = b
        self._comm_stream = torch.cuda.Stream(device=self.params[0].device)

    def _run(self, fwd_bwd, capture):
        """fwd + bwd, with the bucketed all-reduces issued as buckets complete (overlap) or one
        flat all-reduce after the backward (split, eager warm-up only)."""
        if self.comm == "none":
            return fwd_bwd()
        if self.comm == "split":
            loss = fwd_bwd()
            pack_grads(self.params, self.flat)
            _all_reduce(self.flat)
            unpack_grads(self.params, self.flat, 1.0 / self.world)
            return loss
        main = torch.cuda.current_stream()
        remaining = [len(b) for b in self._buckets]
        handles = []

        def make_hook(i):
            def hook(p):
                lo = self._offsets[i]
                self.flat[lo:lo + p.numel()].copy_(p.grad.reshape(-1))
                b = self._bucket_of[i]
                remaining[b] -= 1
                if remaining[b] == 0:
                    idx = self._buckets[b]
                    a = min(self._offsets[j] for j in idx)
                    z = max(self._offsets[j] + self.params[j].numel() for j in idx)
                    ev = torch.cuda.Event()
                    ev.record()  # on the stream the backward (and this hook's copy) runs on
                    self._comm_stream.wait_event(ev)
                    with torch.cuda.stream(self._comm_stream):
                        dist.all_reduce(self.flat[a:z])  # RCCL sum over xGMI, overlapping the backward
            return hook
        for i, p in enumerate(self.params):
            handles.append(p.register_post_accumulate_grad_hook(make_hook(i)))
        try:
            loss = fwd_bwd()
        finally:
            for h in handles:
                h.remove()
        # a parameter without a gradient this step (none in Adapter training) still joins its bucket
        for i, p in enumerate(self.params):
            if p.grad is None:
                p.grad = torch.zeros_like(p)
                make_hook(i)(p)
        main.wait_stream(self._comm_stream)
        unpack_grads(self.params, self.flat, 1.0 / self.world)
        return loss

    def step(self):
        self.graph.replay()
        if self.opt_graph is not None:
            _all_reduce(self.flat)  # RCCL / gloo sum; the optimizer graph scales by 1/world
            self.opt_graph.replay()
        return self.loss


def _all_reduce(flat):
    """Sum over ranks; gloo (tests) reduces a host copy."""
    if dist.get_backend() == "gloo" and flat.is_cuda:
        h = flat.cpu()
        dist.all_reduce(h)
        flat.copy_(h)
    else:
        dist.all_reduce(flat)


def _snapshot_optimizer(opt):
    """Clones of the optimizer's state tensors (empty for a fresh optimizer)."""
    return {id(p): {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in st.items()}
            for p, st in opt.state.items()}


def _restore_optimizer(opt, snap):
    """Put the state back IN PLACE (the captured graph holds these addresses); state created by
    the warm-up for a parameter that had none is zeroed (a fresh optimizer's start)."""
    for p, st in opt.state.items():
        old = snap.get(id(p))
        for k, v in st.items():
            if not torch.is_tensor(v):
                if old is not None and k in old:
                    st[k] = old[k]
                continue
            if old is not None and k in old and torch.is_tensor(old[k]):
                v.copy_(old[k].to(v.device, v.dtype))
            else:
                v.zero_()


def lr_to_device(optimizer, device):
    """After load_state_dict, a graph-mode optimizer's learning rate must be a device tensor at a
    stable address (the captured fused AdamW reads it; the scheduler fills it in place)."""
    for g in optimizer.param_groups:
        lr = g["lr"]
        val = float(lr.detach().cpu()) if torch.is_tensor(lr) else float(lr)
        if torch.is_tensor(lr) and lr.device == device:
            lr.fill_(val)
        else:
            g["lr"] = torch.tensor(val, device=device)


def broadcast_module(module, src=0):
    """Parameters and buffers from rank `src` to every rank (DDP does this at construction;
    the graph path has no DDP wrapper)."""
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src)


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
