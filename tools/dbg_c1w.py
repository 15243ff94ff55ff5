import sys, os
sys.path[:0] = ["split-learning-k8s_amd", ".", "tests"]
import numpy as np, torch
from splitcnn import ops
from splitcnn.data import SyntheticMNIST, init_models
from test_x3_gpu import _relu_bits
gpu = torch.device("cuda:0")
for B in (1, 4, 64):
    a, b = init_models(seed=B + 40)
    x, y = SyntheticMNIST(B + 41).batch(B)
    x, y = x.to(gpu), y.to(gpu)
    W1, b1 = a.conv1.weight.detach().to(gpu), a.conv1.bias.detach().to(gpu)
    W2, b2 = b.conv2.weight.detach().to(gpu), b.conv2.bias.detach().to(gpu)
    W3, b3 = b.fc1.weight.detach().to(gpu), b.fc1.bias.detach().to(gpu)
    act = ops.conv1_fwd(x, W1, b1)
    pooled, code = ops.conv2_fwd_pool(act, W2, b2, impl="x3")
    dpa = torch.empty(B, device=gpu)
    _, _, _, dp = ops.fc_xent(pooled, W3, b3, y, 1.0 / B, dp_amax=dpa)
    slabs = ops.conv2_dgrad_client_slabs(dp, code, W2, x, _relu_bits(x, W1, b1), dp_amax=dpa)
    fused = ops.reduce_slabs(slabs).cpu().numpy()
    g = ops.conv2_dgrad(dp, code, W2, impl="x3", dp_amax=dpa)
    sep = ops.reduce_slabs(ops.conv1_wgrad_remask_slabs(x, W1, b1, g)).cpu().numpy()
    dW_f, dW_s = fused[:288].reshape(32, 9), sep[:288].reshape(32, 9)
    print("B", B, "max|sep|", np.abs(sep).max())
    print(" per-tap max err", np.abs(dW_f - dW_s).max(0) / np.abs(sep).max())
    print(" per-ci max err (first 32)", np.round(np.abs(dW_f - dW_s).max(1) / np.abs(sep).max(), 4))
    print(" db err", np.round(np.abs(fused[288:] - sep[288:]) / np.abs(sep[288:]).max(), 4))
    print(" ratio fused/sep tap0", np.round(dW_f[:8, 0] / dW_s[:8, 0], 3))
