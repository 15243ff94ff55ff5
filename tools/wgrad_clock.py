"""Profiling-only: conv2 wgrad time and mean in-kernel shader clock (variants built with
-DSLK_WW_ABL=512|...: slab[0] of each workgroup holds its GHz). usage: python tools/wgrad_clock.py a.so b.so"""
import ctypes
import json
import sys

import torch

B = 4096
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
act = torch.rand(B, 32, 26, 26, device=dev, generator=g)
dp = torch.randn(B, 9216, device=dev, generator=g) * 1e-4
code = torch.randint(0, 5, (B, 9216), device=dev, generator=g).to(torch.uint8)
slabs = torch.empty(256, 18496, device=dev)
s = torch.cuda.current_stream().cuda_stream
P = ctypes.c_void_p
libs = [ctypes.CDLL(p) for p in sys.argv[1:]]
res = {p: [] for p in sys.argv[1:]}
for r in range(7):
    for p, L in zip(sys.argv[1:], libs):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            assert L.slk_conv2_wgrad(P(act.data_ptr()), P(dp.data_ptr()), P(code.data_ptr()), P(slabs.data_ptr()), B, P(s)) == 0
        e1.record()
        torch.cuda.synchronize()
        res[p].append((e0.elapsed_time(e1) / 5, float(slabs[:, 0].mean())))
for p, v in res.items():
    t = min(x[0] for x in v)
    print(json.dumps({"lib": p, "ms": round(t, 4), "ghz": round(sorted(x[1] for x in v)[len(v) // 2], 3)}))
