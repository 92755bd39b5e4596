"""Small helpers shared by bench.py / smoke(): the deterministic parameter
fill of SURVEY §8c (weights keyed by crc32 of the state-dict name), so every
host rebuilds identical non-zero weights without shipping a checkpoint."""
import math
import zlib

import torch
import torch.nn as nn


def deterministic_fill_(module: nn.Module):
    """ndim>=2 -> randn/sqrt(fan_in); 1-D gains -> 1+0.1*randn; biases -> 0.01*randn."""
    with torch.no_grad():
        for name, p in module.named_parameters():
            g = torch.Generator().manual_seed(zlib.crc32(name.encode()))
            r = torch.randn(p.shape, generator=g, dtype=torch.float64)
            if name.endswith("bias"):
                v = 0.01 * r
            elif p.ndim >= 2:
                v = r / math.sqrt(max(p[0].numel(), 1))
            else:
                v = 1.0 + 0.1 * r
            p.copy_(v.to(p.dtype))
    return module
