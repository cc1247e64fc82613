"""Model EMA for the vCLR DINO teacher (reference detrex/modeling/ema.py: EMAState, EMAUpdater,
apply_model_ema_and_restore, and EMAHook's before_train / after_step as the trainer drives them;
configured at deformable_train_voc_eval_nonvoc.py:151-153: enabled, decay 0.999).

The EMA covers every parameter AND every buffer of the model, by name.  ``apply_and_restore``
swaps the averaged values into the live model for the duration of a ``with`` block (the teacher
pass of ``DINO.infer_results``) and copies the student's values back afterwards, in place, so
optimizer state and graph-captured addresses stay valid."""
from contextlib import contextmanager

import torch


def _named_state(model):
    yield from model.named_parameters()
    yield from model.named_buffers()


class EMAState:
    """name -> detached tensor for every parameter and buffer of a model."""

    def __init__(self, state=None):
        self.state = dict(state or {})

    @classmethod
    def from_model(cls, model, device=None):
        return cls({n: (v.detach().clone() if device is None else v.detach().to(device, copy=True))
                    for n, v in _named_state(model)})

    def has_inited(self):
        return bool(self.state)

    def apply_to(self, model):
        with torch.no_grad():
            for n, v in _named_state(model):
                if n not in self.state:
                    raise KeyError(f"EMA state has no entry {n!r}")
                v.copy_(self.state[n])

    @contextmanager
    def apply_and_restore(self, model):
        saved = EMAState.from_model(model)
        self.apply_to(model)
        try:
            yield saved
        finally:
            saved.apply_to(model)

    def state_dict(self):
        return self.state

    def load_state_dict(self, state_dict):
        self.state = dict(state_dict)


class EMAUpdater:
    """ema = decay * ema + (1 - decay) * value for fp32 / fp16 entries (one fused multi-tensor
    update), the same formula elementwise for the rest (integer buffers such as BatchNorm's
    num_batches_tracked, rounded by the copy as the reference's copy_ rounds them)."""

    def __init__(self, state, decay=0.999):
        self.state, self.decay = state, decay

    def init_state(self, model):
        self.state.state = EMAState.from_model(model).state

    @torch.no_grad()
    def update(self, model):
        avg, cur = [], []
        for n, v in _named_state(model):
            e = self.state.state[n]
            if v.dtype in (torch.float32, torch.float16):
                avg.append(e)
                cur.append(v.to(e.device))
            else:
                e.copy_(e * self.decay + v.to(e.device) * (1.0 - self.decay))
        if avg:
            torch._foreach_mul_(avg, self.decay)
            torch._foreach_add_(avg, cur, alpha=1.0 - self.decay)


def may_build_model_ema(model):
    """Attach an (empty) EMA state as ``model.ema_state`` (the name the reference reserves)."""
    model = getattr(model, "module", model)
    if not hasattr(model, "ema_state") or model.ema_state is None:
        model.ema_state = EMAState()
    return model.ema_state


def apply_model_ema_and_restore(model, state=None):
    model = getattr(model, "module", model)
    state = state if state is not None else model.ema_state
    return state.apply_and_restore(model)
