"""Host-side helpers of the training / evaluation drivers (reference semseg/utils/utils.py)."""
import datetime
import functools
import logging
import os
import random
import time

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
        from irads.graph_step import rccl_capture_env
        rccl_capture_env()  # the training step captures its RCCL all-reduces (TRAIN.GRAPH)
        dist.init_process_group("nccl", timeout=datetime.timedelta(seconds=7200),
                                device_id=torch.device("cuda", gpu))
        dist.barrier()
        return gpu
    return 0


def cleanup_ddp():
    if dist.is_initialized():
        from irads.graph_step import quiesce_process_groups, release_capture_groups
        quiesce_process_groups()  # teardown with captured graphs alive: no work left to poll
        dist.destroy_process_group()
        release_capture_groups()


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


def time_sync() -> float:
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return time.time()


def get_model_size(model) -> float:
    """Size of the parameters and buffers in MB (reference utils.py:36-45 saves a temporary
    state_dict to measure it; the byte count is the same)."""
    n = sum(t.numel() * t.element_size() for t in list(model.parameters()) + list(model.buffers()))
    return n / 1e6


def test_model_latency(model, inputs, use_cuda: bool = False) -> float:
    """Milliseconds for one forward (reference utils.py:47-50; timed with device events here)."""
    with torch.no_grad():
        if use_cuda and torch.cuda.is_available():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            model(inputs)
            b.record()
            torch.cuda.synchronize()
            return a.elapsed_time(b)
        t0 = time.perf_counter()
        model(inputs)
        return (time.perf_counter() - t0) * 1e3


def count_parameters(model) -> float:
    """Trainable parameters in millions (reference utils.py:52-53)."""
    return sum(p.numel() for p in model.parameters() if p.requires_grad) / 1e6


@torch.no_grad()
def throughput(dataloader, model, times: int = 30):
    """Images / s of the forward over `times` batches after a warm-up (reference utils.py:89-100)."""
    model.eval()
    images, _ = next(iter(dataloader))
    images = [x.cuda(non_blocking=True) for x in images] if isinstance(images, list) else images.cuda()
    B = (images[0] if isinstance(images, list) else images).shape[0]
    for _ in range(3):
        model(images)
    t0 = time_sync()
    for _ in range(times):
        model(images)
    return B * times / (time_sync() - t0)


def show_models():
    from semseg import models
    print(models.__all__)


def timer(func):
    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        t0 = time.perf_counter()
        out = func(*args, **kwargs)
        print(f"Elapsed time: {(time.perf_counter() - t0) * 1e3:.2f}ms")
        return out
    return wrapper


def cal_flops(model, modals, logger):
    """Model-complexity report of train_mm.py:113 (reference utils.py:147-161).  The reference
    builds 512x512 dummy inputs, moves the model to the GPU and leaves its fvcore FLOP count
    commented out, so it logs nothing; here the parameter counts are logged instead (fvcore is
    not a dependency, and the HIP kernels are invisible to op-level FLOP counters)."""
    m = model.module if hasattr(model, "module") else model
    total = sum(p.numel() for p in m.parameters())
    train = sum(p.numel() for p in m.parameters() if p.requires_grad)
    if logger is not None:
        logger.info(f"parameters: {total / 1e6:.2f} M total, {train / 1e6:.2f} M trainable; "
                    f"modals {list(modals)}")
    return total, train


def nchw_to_nlc(x):
    """(N, C, H, W) -> (N, H*W, C) (reference utils.py:178-188)."""
    assert len(x.shape) == 4
    return x.flatten(2).transpose(1, 2).contiguous()


def nlc_to_nchw(x, hw_shape):
    """(N, H*W, C) -> (N, C, H, W) (reference utils.py:190-204)."""
    H, W = hw_shape
    assert len(x.shape) == 3
    B, L, C = x.shape
    assert L == H * W, 'The seq_len does not match H, W'
    return x.transpose(1, 2).reshape(B, C, H, W).contiguous()


def nlc2nchw2nlc(module, x, hw_shape, contiguous=False, **kwargs):
    """Apply a (N, C, H, W) module to a (N, L, C) tensor (reference utils.py:206-...)."""
    H, W = hw_shape
    assert len(x.shape) == 3
    B, L, C = x.shape
    assert L == H * W, 'The seq_len doesn\'t match H, W'
    if not contiguous:
        x = x.transpose(1, 2).reshape(B, C, H, W)
        x = module(x, **kwargs)
        return x.flatten(2).transpose(1, 2)
    x = x.transpose(1, 2).reshape(B, C, H, W).contiguous()
    x = module(x, **kwargs)
    return x.flatten(2).transpose(1, 2).contiguous()
