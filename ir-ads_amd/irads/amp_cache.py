"""bf16 copies of the trainable parameters, made in ONE cast per training step.

Under torch.autocast every F.linear casts its fp32 weight and bias to bf16 on every call
(one small copy kernel each: ~160 launches per CMNeXt step for the MPG / DSCF / DAttn /
head Linears).  `refresh` concatenates all trainable parameters and casts them in two
launches at the start of the forward; `lookup` hands LinearFn the bf16 view of a parameter
(or of a view of one, e.g. a 1x1 conv weight seen as a matrix).  The copies are exactly the
roundings autocast would apply.  Entries are keyed by storage address and checked against
the parameter's version counter, so an optimizer step or load_state_dict since the refresh
makes lookups miss (and fall back to the per-call cast) instead of returning stale values.
Inside a captured HIP graph the refresh kernels are part of the graph, so every replay
re-casts the weights the previous replay's optimizer step updated.
"""
import torch

_entries = {}  # data_ptr -> (param, version, bf16 view)


def refresh(params):
    params = [p for p in params if p.is_cuda and p.dtype == torch.float32]
    _entries.clear()
    if not params:
        return
    with torch.no_grad():
        flat = torch.cat([p.detach().reshape(-1) for p in params]).to(torch.bfloat16)
    off = 0
    for p in params:
        n = p.numel()
        _entries[p.data_ptr()] = (p, p._version, flat[off:off + n].view(p.shape))
        off += n


def lookup(t):
    """bf16 copy of parameter `t` (or of a view with the same storage start and size), or None."""
    e = _entries.get(t.data_ptr())
    if e is None:
        return None
    p, ver, v = e
    if p._version != ver or v.numel() != t.numel():
        return None
    return v.view(t.shape)


def clear():
    _entries.clear()
