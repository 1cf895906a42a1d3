"""Scores 3000 random 40-dim rows through a TDNN config with the bf16x6
GEMM (the library and schedule from CATEARS_HIP_LIB / CATEARS_X6_VARIANT)
and saves the output rows: the bit comparisons of tools/experiments/gpu_r5z*.sh.
    python tools/experiments/x6_child.py <config> <out.npy>"""
import sys

import numpy as np
import torch

from catears_amd import gpu

ctx = gpu.Context(0)
model = gpu.Model(ctx, sys.argv[1])
x = np.random.default_rng(750).normal(9.0, 3.0, size=(3000, 40)).astype(np.float32)
np.save(sys.argv[2], gpu.nnet_propagate(ctx, model, torch.from_numpy(x).to("cuda:0")).cpu().numpy())
