"""Host-side helpers of the training / evaluation drivers (reference semseg/utils/utils.py)."""
import datetime
import logging
import os
import random

import numpy as np
import torch
import torch.distributed as dist
from torch.backends import cudnn


def fix_seeds(seed: int = 3407) -> None:
    torch.manual_seed(seed)
    torch.cuda.manual_seed(seed)
    np.random.seed(seed)
    random.seed(seed)


def setup_cudnn() -> None:
    cudnn.benchmark = True  # MIOpen find for the convolutions
    cudnn.deterministic = False


def setup_ddp():
    """One process per GPU (torchrun env); RCCL ("nccl") process group.  Returns the local
    GPU index (0 without a launcher)."""
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
        gpu = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(gpu)
        dist.init_process_group("nccl", timeout=datetime.timedelta(seconds=7200),
                                device_id=torch.device("cuda", gpu))
        dist.barrier()
        return gpu
    return 0


def cleanup_ddp():
    if dist.is_initialized():
        dist.destroy_process_group()


def reduce_tensor(tensor):
    rt = tensor.clone()
    dist.all_reduce(rt, op=dist.ReduceOp.SUM)
    rt /= dist.get_world_size()
    return rt


def get_logger(log_file=None):
    formatter = logging.Formatter('%(asctime)s - %(name)s - %(levelname)s: - %(message)s', datefmt='%Y%m%d %H:%M:%S')
    logger = logging.getLogger()
    logger.setLevel(logging.INFO)
    del logger.handlers[:]
    if log_file:
        fh = logging.FileHandler(log_file, mode='w')
        fh.setLevel(logging.INFO)
        fh.setFormatter(formatter)
        logger.addHandler(fh)
    sh = logging.StreamHandler()
    sh.setFormatter(formatter)
    sh.setLevel(logging.INFO)
    logger.addHandler(sh)
    return logger


def print_iou(epoch, iou, miou, acc, macc, class_names):
    assert len(iou) == len(class_names)
    assert len(acc) == len(class_names)
    lines = ['\n%-8s\t%-8s\t%-8s' % ('Class', 'IoU', 'Acc')]
    for i in range(len(iou)):
        cls = 'Class %d:' % (i + 1) if class_names is None else '%d %s' % (i + 1, class_names[i])
        lines.append('%-8s\t%.2f\t%.2f' % (cls, iou[i], acc[i]))
    lines.append('== %-8s\t%d\t%-8s\t%.2f\t%-8s\t%.2f' % ('Epoch:', epoch, 'mean_IoU', miou, 'mean_Acc', macc))
    return "\n".join(lines)
