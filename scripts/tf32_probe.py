import torch
print("cudnn.allow_tf32", torch.backends.cudnn.allow_tf32, "matmul.allow_tf32", torch.backends.cuda.matmul.allow_tf32)
