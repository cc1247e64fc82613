"""Training driver (reference train_mm.py): same --cfg YAML schema, model initialisation,
TRAIN_TYPE optimiser, warm-up poly LR, MMST objective, evaluation schedule, checkpoint
dicts and logs.  Numerics follow the YAML as the reference's do:
  * TRAIN.AMP false: fp32 training (the reference's configs, e.g. nyu_rgbd.yaml:24);
    TRAIN.AMP true: autocast + GradScaler in fp16 as the reference (train_mm.py:109,133,150-152),
    or in bf16 without a scaler when TRAIN.AMP_DTYPE is 'bf16' (a build extension: the fast
    fused-stage path and the one bench.py times);
  * iters_per_epoch uses the reference's hard-coded gpus = 1 (train_mm.py:37,85): under DDP the
    warm-up and poly horizon are stretched by the world size exactly as in the reference.
MI355X-first differences:
  * with TRAIN.GRAPH (default on; not with the fp16 GradScaler, whose step syncs the host) the
    iteration is captured once into a HIP graph and replayed (irads/graph_step.py); with DDP
    the gradients are all-reduced over RCCL in buckets overlapped with the backward, inside the
    graph; parameters and buffers are broadcast from rank 0 first (DDP's construction does it);
  * the loss is accumulated on the device and read once per epoch (the reference syncs
    every iteration, train_mm.py:154,160).

    python train_mm.py --cfg configs/nyu_rgbd.yaml
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train_mm.py --cfg configs/deepcrack.yaml
"""
import argparse
import math
import os
import sys
import time
from pathlib import Path

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ir-ads_amd"))

import torch  # noqa: E402
import yaml  # noqa: E402
from tabulate import tabulate  # noqa: E402
from torch import distributed as dist  # noqa: E402
from torch import nn  # noqa: E402
from torch.utils.data import DataLoader, DistributedSampler, RandomSampler  # noqa: E402

from semseg.augmentations_mm import get_train_augmentation, get_val_augmentation  # noqa: E402
from semseg.losses import get_loss, mmst_loss  # noqa: E402
from semseg.models import CMNeXt  # noqa: E402,F401
from semseg.optimizers import get_optimizer  # noqa: E402
from semseg.schedulers import get_scheduler  # noqa: E402
from semseg.utils.utils import cleanup_ddp, fix_seeds, get_logger, print_iou, setup_cudnn, setup_ddp  # noqa: E402
from semseg.utils.utils import cal_flops  # noqa: E402
from val_mm import evaluate, make_dataset  # noqa: E402


def init_extra(model):
    """train_mm.py:51-77: re-initialise the prompt/adapter projections and copy the rgb
    patch-embed / output-norm weights into their extra_ (depth) twins."""
    extra = {}
    for k, v in model.state_dict().items():
        if 'D_fc1.weight' in k:
            nn.init.kaiming_uniform_(v, a=math.sqrt(5))
            extra[k] = v
        if 'D_fc2.weight' in k and 'MPG' in k:
            nn.init.kaiming_uniform_(v, a=math.sqrt(5))
            extra[k] = v
        if 'D_fc2.weight' in k and 'Adapter' in k:
            nn.init.zeros_(v)
            extra[k] = v
        if 'patch_embed' in k and 'extra_' not in k:
            p = k.split('.')
            p[1] = 'extra_' + p[1]
            extra['.'.join(p)] = v
        if 'norm' in k and 'block' not in k and 'extra_' not in k and 'stages' not in k:
            p = k.split('.')
            p[1] = 'extra_' + p[1]
            extra['.'.join(p)] = v
    model.load_state_dict(extra, strict=False)


def main(cfg, gpu, save_dir, logger):
    start = time.time()
    best_mIoU, best_epoch = 0.0, 0
    ddp = bool(cfg['TRAIN']['DDP']) and dist.is_initialized()
    rank0 = (not ddp) or dist.get_rank() == 0
    world = dist.get_world_size() if ddp else 1
    device = torch.device(cfg['DEVICE'], gpu) if cfg['DEVICE'] == 'cuda' else torch.device(cfg['DEVICE'])
    train_cfg, eval_cfg = cfg['TRAIN'], cfg['EVAL']
    dataset_cfg, model_cfg = cfg['DATASET'], cfg['MODEL']
    loss_cfg, optim_cfg, sched_cfg = cfg['LOSS'], cfg['OPTIMIZER'], cfg['SCHEDULER']
    epochs, lr = train_cfg['EPOCHS'], optim_cfg['LR']
    amp = bool(train_cfg['AMP'])
    amp_dtype = torch.float16 if str(train_cfg.get('AMP_DTYPE', 'fp16')).lower() in ('fp16', 'float16') \
        else torch.bfloat16
    scaled = amp and amp_dtype == torch.float16  # the reference's GradScaler path
    use_graph = bool(train_cfg.get('GRAPH', True)) and not scaled
    trainset = make_dataset(cfg, 'train', get_train_augmentation(train_cfg['IMAGE_SIZE'],
                                                                 seg_fill=dataset_cfg['IGNORE_LABEL']))
    valset = make_dataset(cfg, 'val', get_val_augmentation(eval_cfg['IMAGE_SIZE']))
    class_names = trainset.CLASSES
    extra = {'sb': model_cfg['SB']} if model_cfg.get('SB') else {}  # build-defined SB hook
    model = globals()[model_cfg['NAME']](model_cfg['BACKBONE'], trainset.n_classes, dataset_cfg['MODALS'], **extra)
    resume = None
    if os.path.isfile(model_cfg['RESUME']):
        resume = torch.load(model_cfg['RESUME'], map_location='cpu', weights_only=True)
        logger.info(model.load_state_dict(resume['model_state_dict']))
    elif model_cfg.get('PRETRAINED'):
        model.init_pretrained(model_cfg['PRETRAINED'])
    init_extra(model)
    model = model.to(device)
    gpus = 1  # reference train_mm.py:37 (`gpus = 1#int(os.environ['WORLD_SIZE'])`), kept for schedule parity
    iters_per_epoch = len(trainset) // train_cfg['BATCH_SIZE'] // gpus
    loss_fn = get_loss(loss_cfg['NAME'], trainset.ignore_label, None)
    optimizer = get_optimizer(model, optim_cfg['NAME'], lr, optim_cfg['TRAIN_TYPE'], optim_cfg['WEIGHT_DECAY'],
                              lr_on_device=use_graph)
    scheduler = get_scheduler(sched_cfg['NAME'], optimizer, int((epochs + 1) * iters_per_epoch), sched_cfg['POWER'],
                              iters_per_epoch * sched_cfg['WARMUP'], sched_cfg['WARMUP_RATIO'])
    sampler = DistributedSampler(trainset, world, dist.get_rank(), shuffle=True) if ddp else RandomSampler(trainset)
    train_model = model
    if ddp and not use_graph:
        from torch.nn.parallel import DistributedDataParallel as DDP
        train_model = DDP(model, device_ids=[gpu], static_graph=True)
    start_epoch = 0
    if resume:
        start_epoch = resume['epoch'] - 1
        optimizer.load_state_dict(resume['optimizer_state_dict'])
        scheduler.load_state_dict(resume['scheduler_state_dict'])
        best_mIoU = resume['best_miou']
        if use_graph:  # the captured AdamW reads lr from the device (a checkpoint may carry a CPU tensor)
            from irads.graph_step import lr_to_device
            lr_to_device(optimizer, device)
    if ddp and use_graph:
        from irads.graph_step import broadcast_module
        broadcast_module(model)
    trainloader = DataLoader(trainset, batch_size=train_cfg['BATCH_SIZE'], num_workers=train_cfg.get('WORKERS', 4),
                             drop_last=True, pin_memory=True, sampler=sampler)
    valloader = DataLoader(valset, batch_size=eval_cfg['BATCH_SIZE'], num_workers=2, pin_memory=True)
    scaler = torch.amp.GradScaler("cuda", enabled=scaled)
    if rank0:
        logger.info('================== model complexity =====================')
        cal_flops(model, dataset_cfg['MODALS'], logger)
        logger.info('================== training config =====================')
        logger.info(cfg)

    # static device-side batch buffers: the captured graph reads its inputs from fixed addresses
    static = None
    runner = None

    def fwd_bwd():
        xs, lbl = static
        with torch.autocast("cuda", dtype=amp_dtype, enabled=amp):
            logits, logits_rgb, logits_dte = train_model(xs)
            loss = mmst_loss(loss_fn, logits, logits_rgb, logits_dte, lbl)
            if getattr(model, 'sb_cfg', None):
                loss = loss + model.sb_loss()
        scaler.scale(loss).backward()
        return loss

    train_loss = torch.zeros((), device=device)
    for epoch in range(start_epoch, epochs):
        model.train()
        if ddp:
            sampler.set_epoch(epoch)
        train_loss.zero_()
        n_iter = 0
        for it, (sample, lbl) in enumerate(trainloader):
            if it >= iters_per_epoch:
                break
            sample = [x.to(device, non_blocking=True) for x in sample]
            lbl = lbl.to(device, non_blocking=True)
            if static is None:
                static = ([x.clone() for x in sample], lbl.clone())
            else:
                for d, s in zip(static[0], sample):
                    d.copy_(s, non_blocking=True)
                static[1].copy_(lbl, non_blocking=True)
            if use_graph:
                if runner is None:
                    from irads.graph_step import GraphedTrainStep
                    keep = [p for p in model.parameters() if p.requires_grad] + list(model.buffers())
                    runner = GraphedTrainStep(model.parameters(), fwd_bwd, optimizer, world=world, warmup=3,
                                              restore=keep)
                loss = runner.step()
            else:
                optimizer.zero_grad(set_to_none=True)
                loss = fwd_bwd()
                scaler.step(optimizer)
                scaler.update()
            scheduler.step()
            train_loss += loss.detach()
            n_iter += 1
        train_loss_v = float(train_loss.item()) / max(n_iter, 1)
        cur_lr = scheduler.get_last_lr()
        cur_lr = float(sum(float(x) for x in cur_lr) / len(cur_lr))
        if rank0:
            logger.info(f"Epoch: [{epoch + 1}/{epochs}] Iter: [{n_iter}/{iters_per_epoch}] LR: {cur_lr:.8f} "
                        f"Loss: {train_loss_v:.8f}")
        if ((epoch + 1) % train_cfg['EVAL_INTERVAL'] == 0 and (epoch + 1) > train_cfg['EVAL_START']) or \
                (epoch + 1) == epochs:
            if rank0:
                acc, macc, _, _, ious, miou = evaluate(model, valloader, device)
                if miou > best_mIoU:
                    stem = f"{model_cfg['NAME']}_{model_cfg['BACKBONE']}_{dataset_cfg['NAME']}"
                    for p in (save_dir / f"{stem}_epoch{best_epoch}_{best_mIoU}_checkpoint.pth",
                              save_dir / f"{stem}_epoch{best_epoch}_{best_mIoU}.pth"):
                        if os.path.isfile(p):
                            os.remove(p)
                    best_mIoU, best_epoch = miou, epoch + 1
                    torch.save(model.state_dict(), save_dir / f"{stem}_epoch{best_epoch}_{best_mIoU}.pth")
                    torch.save({'epoch': best_epoch, 'model_state_dict': model.state_dict(),
                                'optimizer_state_dict': optimizer.state_dict(), 'loss': train_loss_v,
                                'scheduler_state_dict': scheduler.state_dict(), 'best_miou': best_mIoU},
                               save_dir / f"{stem}_epoch{best_epoch}_{best_mIoU}_checkpoint.pth")
                    logger.info(print_iou(epoch, ious, miou, acc, macc, class_names))
                logger.info(f"Current epoch:{epoch} mIoU: {miou} Best mIoU: {best_mIoU}")
    end = time.gmtime(time.time() - start)
    table = [['Best mIoU', f"{best_mIoU:.2f}"], ['Total Training Time', time.strftime("%H:%M:%S", end)]]
    if rank0:
        logger.info(tabulate(table, numalign='right'))
    return best_mIoU


if __name__ == '__main__':
    parser = argparse.ArgumentParser()
    parser.add_argument('--cfg', type=str, default='configs/nyu_rgbd.yaml', help='Configuration file to use')
    args = parser.parse_args()
    with open(args.cfg) as f:
        cfg = yaml.load(f, Loader=yaml.SafeLoader)
    fix_seeds(3407)
    setup_cudnn()
    gpu = setup_ddp()
    modals = ''.join([m[0] for m in cfg['DATASET']['MODALS']])
    exp_name = '_'.join([cfg['DATASET']['NAME'], cfg['MODEL']['BACKBONE'], modals])
    save_dir = Path(cfg['SAVE_DIR'], exp_name)
    if os.path.isfile(cfg['MODEL']['RESUME']):
        save_dir = Path(os.path.dirname(cfg['MODEL']['RESUME']))
    os.makedirs(save_dir, exist_ok=True)
    logger = get_logger(save_dir / 'train.log')
    main(cfg, gpu, save_dir, logger)
    cleanup_ddp()
