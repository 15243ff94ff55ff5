"""Profiling-only: time the conv2 kernels of several libslk builds (tuning-knob variants from
tools/build_variant.sh, or older trees) side by side in ONE process, interleaved rounds, HIP events on one stream.
usage: python tools/ablate.py lib0.so lib1.so ... [--batch 4096 --rounds 5]"""
import argparse
import ctypes
import os
import json

import torch

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--cases", default="", help="comma-separated subset of the cases (default: all)")
args = ap.parse_args()
B = args.batch
dev = torch.device("cuda:0")
P = ctypes.c_void_p
libs = []
for path in args.libs:
    L = ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL | os.RTLD_DEEPBIND)  # own symbols first
    for n in ("slk_conv2_fwd_pool", "slk_conv2_dgrad", "slk_conv2_wgrad", "slk_conv1_fwd", "slk_conv1_wgrad",
              "slk_fc_xent", "slk_fc_wgrad", "slk_conv1_wgrad_remask"):
        getattr(L, n).restype = ctypes.c_int
    L.slk_sgd_from_slabs.restype = ctypes.c_int
    L.slk_conv2_wgrad_nslab.restype = ctypes.c_int
    L.slk_conv1_wgrad_nslab.restype = ctypes.c_int
    L.slk_fc_wgrad_nslab.restype = ctypes.c_int
    libs.append(L)
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(B, 1, 28, 28, device=dev, generator=g)
act = torch.rand(B, 32, 26, 26, device=dev, generator=g)
W1 = torch.randn(32, 1, 3, 3, device=dev, generator=g) * 0.3
b1 = torch.randn(32, device=dev, generator=g) * 0.1
W2 = torch.randn(64, 32, 3, 3, device=dev, generator=g) * 0.05
b2 = torch.randn(64, device=dev, generator=g) * 0.05
W3 = torch.randn(10, 9216, device=dev, generator=g) * 0.01
b3 = torch.zeros(10, device=dev)
y = torch.randint(0, 10, (B,), device=dev, generator=g)
pooled = torch.empty(B, 9216, device=dev)
code = torch.empty(B, 9216, dtype=torch.uint8, device=dev)
dp = torch.randn(B, 9216, device=dev, generator=g) * 1e-4
gcut = torch.empty(B, 32, 26, 26, device=dev)
logits = torch.empty(B, 10, device=dev)
loss_i = torch.empty(B, device=dev)
dl = torch.empty(B, 10, device=dev)
dp2 = torch.empty(B, 9216, device=dev)
slabs = torch.empty(256 * 18496 + 4096 * 320 + 64 * 92170, device=dev)
s = torch.cuda.current_stream().cuda_stream
p = lambda t: P(t.data_ptr())  # noqa: E731

def calls(L):
    extra = {}
    if hasattr(L, "slk_conv2_dgrad_fc"):
        L.slk_conv2_dgrad_fc.restype = ctypes.c_int
        L.slk_conv2_wgrad_fc.restype = ctypes.c_int
        extra = {
            "fc_xent_nodp": lambda: L.slk_fc_xent(p(pooled), p(W3), p(b3), p(y), p(logits), p(loss_i), p(dl), None,
                                                  ctypes.c_float(1.0 / B), None, B, P(s)),
            "conv2_dgrad_fc": lambda: L.slk_conv2_dgrad_fc(p(dl), p(W3), p(code), p(W2), p(gcut), B, P(s)),
            "conv2_wgrad_fc": lambda: L.slk_conv2_wgrad_fc(p(act), p(dl), p(W3), p(code), p(slabs), B, P(s)),
        }
    for n in ("slk_conv2_fwd_pool_direct", "slk_conv2_dgrad_direct", "slk_conv2_wgrad_direct"):
        if hasattr(L, n):
            getattr(L, n).restype = ctypes.c_int
    if hasattr(L, "slk_conv2_fwd_pool_direct"):
        extra["conv2_fwd_pool_direct"] = lambda: L.slk_conv2_fwd_pool_direct(p(act), p(W2), p(b2), p(pooled), p(code), B, P(s))
    if hasattr(L, "slk_conv2_dgrad_direct"):
        extra["conv2_dgrad_direct"] = lambda: L.slk_conv2_dgrad_direct(p(dp), p(code), p(W2), p(gcut), B, P(s))
    if hasattr(L, "slk_conv2_wgrad_direct"):
        extra["conv2_wgrad_direct"] = lambda: L.slk_conv2_wgrad_direct(p(act), p(dp), p(code), p(slabs), B, P(s))
    return {**extra,
        "conv2_fwd_pool": lambda: L.slk_conv2_fwd_pool(p(act), p(W2), p(b2), p(pooled), p(code), B, P(s)),
        "fc_xent": lambda: L.slk_fc_xent(p(pooled), p(W3), p(b3), p(y), p(logits), p(loss_i), p(dl), p(dp2),
                                         ctypes.c_float(1.0 / B), None, B, P(s)),
        "conv2_dgrad": lambda: L.slk_conv2_dgrad(p(dp), p(code), p(W2), p(gcut), B, P(s)),
        "conv2_wgrad": lambda: L.slk_conv2_wgrad(p(act), p(dp), p(code), p(slabs), B, P(s)),
        "conv1_fwd": lambda: L.slk_conv1_fwd(p(x), p(W1), p(b1), p(act), B, P(s)),
        "conv1_wgrad": lambda: L.slk_conv1_wgrad(p(x), p(act), p(gcut), p(slabs), B, P(s)),
        "conv1_wgrad_remask": lambda: L.slk_conv1_wgrad_remask(p(x), p(W1), p(b1), p(gcut), p(slabs), B, P(s)),
        "fc_wgrad": lambda: L.slk_fc_wgrad(p(dl), p(pooled), p(slabs), B, P(s)),
        "row_amax": lambda: L.slk_row_amax(p(act), B, 32 * 26 * 26, p(amx), P(s)),
        # the step's two server slab sets through the fused reduce + SGD (64 fc slabs, 256 conv2 slabs)
        "sgd_fc": lambda: L.slk_sgd_from_slabs(p(prm), p(grd), p(slabs), 64, 92170, ctypes.c_float(0.01), P(s)),
        "sgd_conv2": lambda: L.slk_sgd_from_slabs(p(prm), p(grd), p(slabs), 256, 18496, ctypes.c_float(0.01), P(s)),
    }

amx = torch.empty(B, device=dev)
prm = torch.zeros(92170, device=dev)
grd = torch.empty(92170, device=dev)
_all_calls = calls
if args.cases:
    calls = lambda L: {k: v for k, v in _all_calls(L).items() if k in args.cases.split(",")}  # noqa: E731
res = {i: {} for i in range(len(libs))}
for r in range(args.rounds):
    for i, L in enumerate(libs):
        for name, fn in calls(L).items():
            assert fn() == 0, name
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[i].setdefault(name, []).append(e0.elapsed_time(e1) / args.reps)
for i, path in enumerate(args.libs):
    extra = {}
    if "abl16" in path:  # clock diagnostic build: pooled[0:256] holds per-workgroup GHz
        calls(libs[i])["conv2_fwd_pool"]()
        torch.cuda.synchronize()
        g = pooled.view(-1)[:256].float()
        extra = {"fwd_clock_ghz_mean": round(float(g.mean()), 3), "fwd_clock_ghz_min": round(float(g.min()), 3)}
    print(json.dumps({"lib": path, **{k: round(min(v), 4) for k, v in res[i].items()}, **extra}))
