"""Optimizer factory (reference semseg/optimizers.py:5-49).

TRAIN_TYPE 'Adapter' trains only parameters whose name contains Adapter /
extra_patch_embed / head / MPG (optimizers.py:7-30) and freezes the rest.  On GPU the
AdamW update runs as irads_adamw (irads/optim.py: torch's AdamW object and state, capturable,
the update in launches of up to 72 tensors sized to the tensors, irads_adamw)."""
import torch
from torch import nn
from torch.optim import AdamW, SGD


def adapter_trainable(name: str) -> bool:
    return ("Adapter" in name) or ("extra_patch_embed" in name) or ("head" in name) or ("MPG" in name)


def sb_trainable(name: str) -> bool:
    """The build-defined SB hook's LightSB (CMNeXt(..., sb=...)): trained alongside the Adapters."""
    return name.startswith("sb.") and "S_rotation_matrix" not in name


def get_optimizer(model: nn.Module, optimizer: str, lr: float, train_type: str, weight_decay: float = 0.01,
                  verbose: bool = False, lr_on_device: bool = False):
    """lr_on_device: keep the learning rate as a device tensor (fused AdamW reads it on the GPU,
    the scheduler fills it in place), which makes the optimizer step graph-capturable."""
    fused = {}
    if 'Adapter' in train_type:
        params = [p for n, p in model.named_parameters()
                  if (adapter_trainable(n) or sb_trainable(n)) and p.requires_grad]
        for n, p in model.named_parameters():
            if "Adap" not in n and "extra_patch_embed" not in n and "head" not in n and "MPG" not in n \
                    and not sb_trainable(n):
                p.requires_grad = False
            elif verbose:
                print(n)
        groups = [{"params": params}]
    else:
        wd = [p for p in model.parameters() if p.requires_grad and p.dim() != 1]
        nwd = [p for p in model.parameters() if p.requires_grad and p.dim() == 1]
        groups = [{"params": wd}, {"params": nwd, "weight_decay": 0}]
    on_gpu = all(p.is_cuda for g in groups for p in g["params"])
    if optimizer == 'adamw':
        if on_gpu:
            fused = {"fused": True}
            if lr_on_device:
                dev = groups[0]["params"][0].device
                lr = torch.tensor(float(lr), device=dev)
                fused["capturable"] = True
        if on_gpu:  # the update as irads_adamw launches (irads/optim.py): torch's AdamW object and state
            from irads.optim import AdamW as NativeAdamW
            return NativeAdamW(groups, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=weight_decay)
        return AdamW(groups, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=weight_decay, **fused)
    return SGD(groups, lr, momentum=0.9, weight_decay=weight_decay)
