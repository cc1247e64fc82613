"""AdamW whose update runs as the native irads_adamw launches.

The reference trains with torch.optim.AdamW (semseg/optimizers.py:33-49).  PyTorch's fused
multi-tensor AdamW splits the ~420 trainable tensors of the Adapter step into a dozen launches
whose blocks follow its fixed tensor-list chunks, so one large tensor leaves a launch nearly
idle (0.41 ms per step for 7.5 M parameters, ~0.5 TB/s).  `AdamW` keeps torch's optimizer
object (param groups, state layout exp_avg / exp_avg_sq / step, state_dict, capturable
semantics with the step count and a tensor learning rate on the device) and replaces only
the update: the steps are incremented with one foreach add, then irads_adamw updates up to 72
tensors per launch with blocks in proportion to their sizes.
"""
import ctypes

import torch

from . import native as N


class AdamW(torch.optim.AdamW):
    """torch.optim.AdamW(params, lr, betas, eps, weight_decay) for fp32 CUDA parameters, always
    capturable (device step counts).  amsgrad / maximize / differentiable are not served."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, capturable=True)
        self._lr_dev = {}    # group index -> device lr tensor (for float learning rates)
        self._arrays = {}    # group index -> (pointer key, ctypes arrays)

    def _lr_tensor(self, gi, group, device):
        lr = group["lr"]
        if torch.is_tensor(lr):
            if lr.device != device or lr.dtype != torch.float32 or lr.numel() != 1:
                raise RuntimeError("irads AdamW: a tensor learning rate must be one fp32 value on the parameters' "
                                   "device")
            return lr
        if torch.cuda.is_current_stream_capturing():
            # a replay never calls step(): a float lr would be baked into the graph and later
            # scheduler changes to group['lr'] silently ignored
            raise RuntimeError("irads AdamW: a captured step needs the learning rate as a device tensor "
                               "(lr_on_device); group['lr'] is a float")
        ent = self._lr_dev.get(gi)
        if ent is None or ent[0].device != device:
            t = torch.tensor(float(lr), dtype=torch.float32, device=device)
            self._lr_dev[gi] = (t, float(lr))
            return t
        t, val = ent
        if val != float(lr):
            t.fill_(float(lr))
            self._lr_dev[gi] = (t, float(lr))
        return t

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            if group.get("amsgrad") or group.get("maximize") or group.get("differentiable"):
                raise NotImplementedError("irads AdamW: amsgrad / maximize / differentiable are not served")
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            dev = params[0].device
            for p in params:
                if not (p.is_cuda and p.device == dev and p.dtype == torch.float32 and p.is_contiguous()):
                    raise RuntimeError("irads AdamW: parameters must be contiguous fp32 tensors on one GPU")
                if p.grad.is_sparse or p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
                    raise RuntimeError("irads AdamW: gradients must be dense contiguous fp32")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.zeros((), dtype=torch.float32, device=dev)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            lr = self._lr_tensor(gi, group, dev)
            steps = [self.state[p]["step"] for p in params]
            torch._foreach_add_(steps, 1.0)
            ms = [self.state[p]["exp_avg"] for p in params]
            vs = [self.state[p]["exp_avg_sq"] for p in params]
            key = tuple((p.data_ptr(), p.grad.data_ptr(), m.data_ptr(), v.data_ptr(), s.data_ptr(), p.numel())
                        for p, m, v, s in zip(params, ms, vs, steps)) + (lr.data_ptr(), float(group["weight_decay"]))
            cached = self._arrays.get(gi)
            if cached is None or cached[0] != key:
                n = len(params)
                vp = ctypes.c_void_p * n
                arrays = (vp(*[p.data_ptr() for p in params]), vp(*[p.grad.data_ptr() for p in params]),
                          vp(*[m.data_ptr() for m in ms]), vp(*[v.data_ptr() for v in vs]),
                          vp(*[s.data_ptr() for s in steps]), vp(*([lr.data_ptr()] * n)),
                          (ctypes.c_float * n)(*([float(group["weight_decay"])] * n)),
                          (ctypes.c_long * n)(*[p.numel() for p in params]))
                cached = (key, arrays)
                self._arrays[gi] = cached
            b1, b2 = group["betas"]
            N.call("irads_adamw", len(params), *cached[1], float(b1), float(b2), float(group["eps"]), N.stream())
            # the kernel wrote p, m, v through raw pointers: bump their version counters as torch's
            # in-place update would (autograd's saved-tensor checks, amp_cache's staleness check)
            torch.autograd.graph.increment_version(params + ms + vs)
        return loss
