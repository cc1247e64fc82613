"""In-step kernel spans from in-kernel wall-clock stamps (bench.py's roofline lines).

The C side is irads_stamp_next / irads_wall_clock_khz (include/irads.h); the kernels write their
workgroups' entry / exit clocks into the armed region.
"""
import ctypes
import os
import threading

import torch

from . import native as N


class StepStamps:
    """In-step kernel spans from in-kernel wall-clock stamps (irads_stamp_next, include/irads.h).

    While armed for a kernel name, each of its launch entries gets its own region of STAMP_CAP
    (start, end) pairs, which its workgroups fill with their entry / exit clocks on the device's
    constant-rate wall clock; the launch's span is the first start to the last end.  The region
    pointer is a kernel argument, so a captured graph keeps it: after `reset()` one replay of the
    graph refills every region with that replay's clocks — the kernels' durations inside the real
    step, beside the other streams' work (what rocprofv3's kernel trace reports), with no events and
    no eager re-run.  bench.py reads its roofline lines here."""

    CAPACITY = 192      # stamped launches (C2 step: 24 + 24 window-attention, 4 + 4 DAttn, <= 48 GEMM followers)
    STAMP_CAP = 16384   # workgroups per region (IRADS_STAMP_CAP)

    FOLLOWED = ("winattn_fwd", "winattn_bwd")

    def __init__(self):
        self.armed = set()
        self.buf = None
        self.slots = []  # (name, algorithmic bytes, flops, real-token bytes)
        self.follows = {}  # stamped launch slot -> the slot of the irads GEMM launched right after it
        self._tls = threading.local()

    def arm(self, names, device):
        if os.environ.get("IRADS_NO_STAMPS"):  # A/B: the same step with no stamp regions captured
            self.armed, self.slots = set(), []
            return
        if self.buf is None or self.buf.device != torch.device(device):
            self.buf = torch.zeros((self.CAPACITY, self.STAMP_CAP, 2), device=device, dtype=torch.int64)
        self.slots = []
        self.follows = {}
        self.armed = set(names)
        self.reset()

    def disarm(self):
        self.armed = set()

    def reset(self):
        if self.buf is not None and self.slots:
            self.buf.zero_()

    def take(self, name, nbytes, flops, real_bytes=None):
        """Arm the next stamped launch entry of this thread for `name` (call right before it)."""
        self._tls.pending = None
        if name not in self.armed or len(self.slots) >= self.CAPACITY:
            return
        i = len(self.slots)
        self.slots.append((name, nbytes, flops, nbytes if real_bytes is None else real_bytes))
        N.load().irads_stamp_next(ctypes.c_void_p(self.buf[i].data_ptr()))
        if name in self.FOLLOWED:
            self._tls.pending = i

    def follow(self, irads_kernel):
        """Called by irads.gemm right before the launch that follows a stamped window-attention launch
        on this thread (the proj GEMM after the forward, the qkv dX GEMM after the backward): if
        that launch is irads_gemm_nt, its workgroups' start clocks close the window-attention
        launch's PERIOD (its first workgroup's start to the next kernel's), which on one stream is
        the kernel's dispatch-to-completion time as rocprofv3 traces it (the end-of-kernel cache
        write-back included); on hipBLASLt the launch keeps its own span."""
        i = getattr(self._tls, "pending", None)
        self._tls.pending = None
        if i is None or not irads_kernel or len(self.slots) >= self.CAPACITY:
            return
        j = len(self.slots)
        self.slots.append(("_follow", 0, 0, 0))
        self.follows[i] = j
        N.load().irads_stamp_next(ctypes.c_void_p(self.buf[j].data_ptr()))

    def dump(self, path):
        """The raw per-workgroup (start, end) clocks of every filled slot, with the slot names and the
        clock rate, to an .npz (workgroup timelines: scripts/stamp_timeline.py)."""
        import numpy as np
        torch.cuda.synchronize()
        n = len(self.slots)
        np.savez_compressed(path, regions=self.buf[:n].cpu().numpy(), names=np.array([s[0] for s in self.slots]),
                            bytes=np.array([s[1] for s in self.slots]), khz=N.load().irads_wall_clock_khz(),
                            follows=np.array(sorted(self.follows.items()), dtype=np.int64).reshape(-1, 2))

    def read(self):
        """{name: {"launches", "total_ms", "bytes", "flops", "real_bytes", "spans_ms", "own_spans_ms",
        "periods"}} of the filled slots: total_ms / spans_ms are the launch's period where an irads GEMM
        followed it (first workgroup start to that GEMM's first start), else its own span."""
        torch.cuda.synchronize()
        if not self.slots:
            return {}
        khz = N.load().irads_wall_clock_khz()
        if khz <= 0:
            raise RuntimeError("irads_wall_clock_khz: device wall-clock rate unavailable")
        reg = self.buf[:len(self.slots)]
        st = reg[..., 0]
        first = torch.where(st > 0, st, torch.full_like(st, torch.iinfo(torch.int64).max)).amin(1)
        last = reg[..., 1].amax(1)
        out = {}
        first, last = first.cpu().tolist(), last.cpu().tolist()
        for i, ((name, nb, fl, rb), s, e) in enumerate(zip(self.slots, first, last)):
            if name == "_follow" or e <= 0 or e <= s:  # a follower, or not launched in the replay
                continue
            d = out.setdefault(name, {"launches": 0, "total_ms": 0.0, "bytes": 0, "flops": 0, "real_bytes": 0,
                                      "spans_ms": [], "own_spans_ms": [], "periods": 0})
            own = (e - s) / khz
            ms = own
            j = self.follows.get(i)
            if j is not None and first[j] > e and first[j] < (1 << 62):
                ms = (first[j] - s) / khz
                d["periods"] += 1
            d["own_spans_ms"].append(own)
            d["launches"] += 1
            d["total_ms"] += ms
            d["bytes"] += nb
            d["flops"] += fl
            d["real_bytes"] += rb
            d["spans_ms"].append(ms)
        return out


STAMPS = StepStamps()
