"""One detector training iteration as the reference Trainer.run_step does it
(projects/vCLR_deformable_mask/train_net.py:83-129, amp off as configured): loss dict from the
model, their sum, zero_grad, backward, gradient clipping (max_norm 0.1, L2: the config's
train.clip_grad, deformable_train_voc_eval_nonvoc.py:119-121), optimizer step, and the model EMA
the teacher reads (detrex EMAHook: initialised before the first step, updated after each;
deformable_train_voc_eval_nonvoc.py:151-153, decay 0.999) when ``ema_updater`` is given."""
import torch

from detrex.modeling.ema import EMAUpdater, may_build_model_ema


def build_ema(model, decay=0.999):
    """EMAHook.before_train: attach the EMA state to the model and initialise it from the weights."""
    updater = EMAUpdater(may_build_model_ema(model), decay=decay)
    if not updater.state.has_inited():
        updater.init_state(getattr(model, "module", model))
    return updater


def run_step(model, optimizer, data, clip_grad_params=None, ema_updater=None):
    assert model.training, "[Trainer] model was changed to eval mode!"
    loss_dict = model(data)
    losses = loss_dict if isinstance(loss_dict, torch.Tensor) else sum(loss_dict.values())
    optimizer.zero_grad()
    losses.backward()
    if clip_grad_params is not None:
        params = [p for p in model.parameters() if p.requires_grad and p.grad is not None]
        if params:
            torch.nn.utils.clip_grad_norm_(parameters=params, **clip_grad_params)
    optimizer.step()
    if ema_updater is not None:  # EMAHook.after_step
        ema_updater.update(getattr(model, "module", model))
    return losses.detach(), {k: v.detach() for k, v in loss_dict.items()}
