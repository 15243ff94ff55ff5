"""Profiling-only: time the widened-model (K5) kernels of several libslk builds side by side in ONE
process, interleaved rounds, HIP events on one stream (random operands: DVFS-realistic).
usage: python tools/ablate_wide.py lib0.so lib1.so ... [--batch 4096 --rounds 5 --reps 5]"""
import argparse
import ctypes
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
g = torch.Generator(device=dev).manual_seed(0)


def bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=dev, generator=g) * scale).to(torch.bfloat16)


def codes(*shape):
    return torch.randint(0, 5, shape, device=dev, generator=g).to(torch.uint8)


x = torch.randn(B, 3, 32, 32, device=dev, generator=g)
a1 = bf(B, 8, 32, 32, 8).abs()
p2 = bf(B, 16, 16, 16, 8).abs()
code2 = codes(B, 16, 16, 16, 8)
cut = bf(B, 32, 8, 8, 8)
code3 = codes(B, 32, 8, 8, 8)
dcut = bf(B, 32, 8, 8, 8, scale=1e-3)
da1m = bf(B, 8, 32, 32, 8, scale=1e-3)
w1b, w2f, w2d, w3f, w3d = bf(64 * 32, scale=0.1), bf(73728, scale=0.05), bf(73728, scale=0.05), bf(294912, scale=0.03), bf(294912, scale=0.03)
b1, b2, b3 = (torch.randn(n, device=dev, generator=g) * 0.01 for n in (64, 128, 256))
out_a1 = torch.empty_like(a1)
out_p2, out_c2 = torch.empty_like(p2), torch.empty_like(code2)
out_cut, out_c3 = torch.empty_like(cut), torch.empty_like(code3)
out_da1m = torch.empty_like(da1m)
dp2 = bf(B, 16, 16, 16, 8, scale=1e-3)
out_dp2 = torch.empty_like(dp2)
slabs = torch.empty(256 * (73728 + 128) + 64 * (294912 + 256), device=dev)
s = torch.cuda.current_stream().cuda_stream
p = lambda t: P(t.data_ptr())  # noqa: E731
FLOP = 150_994_944 * B

# the head (dropout p = 0.25 as WideServerStage: keep iff hash >= 2^30, kept values x 4/3)
wf8 = torch.randn(10 * 16384, device=dev, generator=g) * 0.01
bfc = torch.randn(10, device=dev, generator=g) * 0.01
stepc = torch.zeros(1, dtype=torch.int32, device=dev)
hlog = torch.empty(B, 10, device=dev)
hdl = torch.randn(B, 10, device=dev, generator=g) / B
hdcut = torch.empty_like(cut)

libs = []
a1bits = torch.empty(B, 1024, dtype=torch.int64, device=dev)
out_bits = torch.empty_like(a1bits)
for path in args.libs:
    L = ctypes.CDLL(path)
    L._bits = hasattr(L, "slk_wide_relu_bits")
    if L._bits:
        assert L.slk_wide_relu_bits(p(a1), p(a1bits), B, P(s)) == 0
    L.slk_wide_head_work.restype = ctypes.c_int
    L.slk_wide_head_nslab.restype = ctypes.c_int
    L.slk_wide_head_fwd.argtypes = [P] * 4 + [ctypes.c_uint, ctypes.c_uint, ctypes.c_float] + [P] + [ctypes.c_int] * 2 + [P]
    L.slk_wide_head_bwd.argtypes = [P] * 4 + [ctypes.c_uint, ctypes.c_uint, ctypes.c_float] + [P] * 2 + [ctypes.c_int] * 2 + [P]
    L._hwork = torch.empty(L.slk_wide_head_work(B), device=dev)
    L._hslabs = torch.empty(L.slk_wide_head_nslab(B), 163850, device=dev)
    L.slk_wide_head.argtypes = [P] * 5 + [ctypes.c_uint, ctypes.c_uint, ctypes.c_float, ctypes.c_float] + [P] * 7 + [ctypes.c_int] * 2 + [P]
    L._hout = {"logits": torch.empty(B, 10, device=dev), "loss_i": torch.empty(B, device=dev),
               "dlogits": torch.empty(B, 10, device=dev), "dcut": torch.empty_like(cut),
               "slabs": torch.empty(L.slk_wide_head_nslab(B), 163850, device=dev)}
    libs.append(L)
hlab = torch.randint(0, 10, (B,), device=dev, generator=g)
ad_p, ad_m, ad_v = torch.zeros(295168, device=dev), torch.zeros(295168, device=dev), torch.zeros(295168, device=dev)
herr = torch.zeros(1, dtype=torch.int32, device=dev)


def calls(L):
    return {
        # round 5 ABI: conv1 also writes the ReLU words, conv2's dgrad reads them instead of a1
        "conv1_fwd": (lambda: L.slk_wide_conv1_fwd(p(x), p(w1b), p(b1), p(out_a1), p(out_bits), B, P(s))) if L._bits
        else (lambda: L.slk_wide_conv1_fwd(p(x), p(w1b), p(b1), p(out_a1), B, P(s))),
        "conv2_fwd": lambda: L.slk_wide_conv2_fwd(p(a1), p(w2f), p(b2), p(out_p2), p(out_c2), B, P(s)),
        "conv3_fwd": lambda: L.slk_wide_conv3_fwd(p(p2), p(w3f), p(b3), p(out_cut), p(out_c3), B, P(s)),
        # pooled gradients + codes: conv3's kernels route dcut by code3, conv2's route dp2 by code2
        "conv3_wgrad": lambda: L.slk_wide_conv3_wgrad(p(dcut), p(code3), p(p2), p(slabs), B, P(s)),
        "conv3_dgrad": lambda: L.slk_wide_conv3_dgrad(p(dcut), p(code3), p(w3d), p(out_dp2), B, P(s)),
        "conv2_wgrad": lambda: L.slk_wide_conv2_wgrad(p(dp2), p(code2), p(a1), p(slabs), B, P(s)),
        "conv2_dgrad": lambda: L.slk_wide_conv2_dgrad(p(dp2), p(code2), p(w2d), p(a1bits if L._bits else a1),
                                                      p(out_da1m), B, P(s)),
        "conv1_wgrad": lambda: L.slk_wide_conv1_wgrad(p(x), p(da1m), p(slabs), B, P(s)),
        # Adam from slabs at the step's two <= 64-slab sets: conv3's (64 x 295,168) and the head's (64 x 163,850)
        "adam_conv3": lambda: L.slk_adam_from_slabs(p(ad_p), None, p(ad_m), p(ad_v), p(slabs), 64, 295168,
                                                    ctypes.c_float(1e-3), ctypes.c_float(0.9), ctypes.c_float(0.999),
                                                    ctypes.c_float(1e-8), p(stepc), P(s)),
        "adam_fc": lambda: L.slk_adam_from_slabs(p(ad_p), None, p(ad_m), p(ad_v), p(slabs), 64, 163850,
                                                 ctypes.c_float(1e-3), ctypes.c_float(0.9), ctypes.c_float(0.999),
                                                 ctypes.c_float(1e-8), p(stepc), P(s)),
        "head_fwd": lambda: L.slk_wide_head_fwd(p(cut), p(wf8), p(bfc), p(stepc), 7, 1 << 30, 4.0 / 3.0, p(hlog),
                                                0, B, P(s)),
        "head_bwd": lambda: L.slk_wide_head_bwd(p(cut), p(wf8), p(hdl), p(stepc), 7, 1 << 30, 4.0 / 3.0, p(hdcut),
                                                p(L._hslabs), 0, B, P(s)),
        # the training step's head (forward + CE + cut gradient + fc weight-gradient slabs)
        "head": lambda: L.slk_wide_head(p(cut), p(wf8), p(bfc), p(hlab), p(stepc), 7, 1 << 30, 4.0 / 3.0, 1.0 / B,
                                        *(p(L._hout[k]) for k in ("logits", "loss_i", "dlogits", "dcut", "slabs")),
                                        p(L._hwork), p(herr), 0, B, P(s)),
    }


res = {i: {} for i in range(len(libs))}
for r in range(args.rounds):
    for i, L in enumerate(libs):
        for name, fn in calls(L).items():
            if args.cases and name not in args.cases.split(","):
                continue
            assert fn() == 0, name
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[i].setdefault(name, []).append(e0.elapsed_time(e1) / args.reps)
torch.cuda.synchronize()
chk = {}
for i, L in enumerate(libs[1:], 1):  # the fused head's outputs vs the first library's
    for k, t in L._hout.items():
        ref = libs[0]._hout[k].float()
        if k == "slabs":
            t, ref = t.sum(0), ref.sum(0)
        chk[f"{args.libs[i]}:{k}"] = float((t.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
# conv kernels: every library's output bitwise against the first library's (same operands)
outs = {"conv2_fwd": [out_p2, out_c2], "conv3_fwd": [out_cut, out_c3], "conv3_dgrad": [out_dp2],
        "conv2_dgrad": [out_da1m], "conv3_wgrad": [slabs], "conv2_wgrad": [slabs], "conv1_fwd": [out_a1],
        "conv1_wgrad": [slabs]}
for name, ts in outs.items():
    if args.cases and name not in args.cases.split(","):
        continue
    for t in ts:
        t.zero_()
    assert calls(libs[0])[name]() == 0
    torch.cuda.synchronize()
    ref = [t.clone() for t in ts]
    for i, L in enumerate(libs[1:], 1):
        for t in ts:
            t.zero_()
        assert calls(L)[name]() == 0
        torch.cuda.synchronize()
        chk[f"{args.libs[i]}:{name}:bitwise"] = all(torch.equal(a, b) for a, b in zip(ts, ref))
        if name.endswith("wgrad"):  # summed slabs (the gradient) relative to the first library's
            g0, g1 = ref[0].double().sum(0), ts[0].double().sum(0)
            chk[f"{args.libs[i]}:{name}:rel"] = float((g1 - g0).abs().max() / g0.abs().max().clamp_min(1e-30))
out = {"check_vs_lib0": chk}
for i, path in enumerate(args.libs):
    d = {}
    for name, v in res[i].items():
        ms = sorted(v)[len(v) // 2]
        d[name] = {"ms": round(ms, 4)}
        if name.startswith(("conv2_", "conv3_")):
            d[name]["TFs"] = round(FLOP / (ms * 1e-3) / 1e12, 1)
    out[path] = d
print(json.dumps(out, indent=1))
