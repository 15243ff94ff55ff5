"""A/B timing of the conv2 Winograd kernels at B=4096 (HIP events on the launch stream, interleaved
reps): production slk_conv2_fwd_pool vs the previous forward (slk_conv2_fwd_pool_v1, if exported),
plus dgrad and wgrad; prints one JSON line. Profiling tool, not a test."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]

import torch  # noqa: E402

from splitcnn import _lib, ops  # noqa: E402
from splitcnn.data import SyntheticMNIST, init_models  # noqa: E402

B = int(os.environ.get("AB_B", "4096"))
REPS = int(os.environ.get("AB_REPS", "20"))
dev = torch.device("cuda:0")
a, b = init_models(seed=0)
x, y = SyntheticMNIST(42).batch(B)
x = x.to(dev)
W1, b1 = a.conv1.weight.detach().to(dev), a.conv1.bias.detach().to(dev)
W2, b2 = b.conv2.weight.detach().to(dev).contiguous(), b.conv2.bias.detach().to(dev)
act = ops.conv1_fwd(x, W1, b1) if hasattr(ops, "conv1_fwd") else None
lib = _lib.load(os.environ["AB_LIB"]) if os.environ.get("AB_LIB") else _lib.load()
st = torch.cuda.current_stream(dev)
sp = ctypes.c_void_p(st.cuda_stream)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
pooled = torch.empty((B, 64, 12, 12), device=dev)
code = torch.empty((B, 64, 12, 12), device=dev, dtype=torch.uint8)
pooled1, code1 = torch.empty_like(pooled), torch.empty_like(code)
dpooled = torch.randn((B, 64, 12, 12), device=dev) * 1e-3
gcut = torch.empty((B, 32, 26, 26), device=dev)
nslab = lib.slk_conv2_wgrad_nslab(B)
slabs = torch.empty((nslab, 64 * 288 + 64), device=dev)

calls = {
    "fwd": lambda: lib.slk_conv2_fwd_pool(P(act), P(W2), P(b2), P(pooled), P(code), B, sp),
    "dgrad": lambda: lib.slk_conv2_dgrad(P(dpooled), P(code), P(W2), P(gcut), B, sp),
    "wgrad": lambda: lib.slk_conv2_wgrad(P(act), P(dpooled), P(code), P(slabs), B, sp),
}
if hasattr(lib, "slk_conv2_fwd_pool_v1"):
    calls["fwd_v1"] = lambda: lib.slk_conv2_fwd_pool_v1(P(act), P(W2), P(b2), P(pooled1), P(code1), B, sp)
for f in calls.values():
    assert f() == 0
torch.cuda.synchronize()
out = {}
if "fwd_v1" in calls:
    out["fwd_vs_v1_pooled_maxrel"] = float(((pooled - pooled1).abs().max() / pooled1.abs().max()).item())
    out["fwd_vs_v1_code_mismatch"] = int((code != code1).sum().item())
times = {k: [] for k in calls}
for _ in range(REPS):
    for k, f in calls.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        f()
        e1.record(st)
        times[k].append((e0, e1))
torch.cuda.synchronize()
for k, v in times.items():
    ms = sorted(e0.elapsed_time(e1) for e0, e1 in v)
    out[k + "_ms_median"] = round(ms[len(ms) // 2], 4)
    out[k + "_ms_min"] = round(ms[0], 4)
out["lib"] = os.environ.get("AB_LIB", "production")
print(json.dumps(out))
