"""One detector training iteration as the reference Trainer.run_step does it
(projects/vCLR_deformable_mask/train_net.py:83-129, amp off as configured): loss dict from the
model, their sum, zero_grad, backward, gradient clipping (max_norm 0.1, L2: the config's
train.clip_grad, deformable_train_voc_eval_nonvoc.py:119-121), optimizer step."""
import torch


def run_step(model, optimizer, data, clip_grad_params=None):
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
    return losses.detach(), {k: v.detach() for k, v in loss_dict.items()}
