"""Interleaved timing of the conv2 kernel implementations (wino / direct / x3) at B = 4096, HIP events
on the launch stream, median of N rounds. Usage: python tools/x3_time.py [--rounds 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--ops", default="fwd")
    args = ap.parse_args()
    from splitcnn import ops
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import ClientStage
    dev = torch.device("cuda:0")
    a, b = init_models(seed=1)
    x, y = SyntheticMNIST(2).batch(args.B)
    act = ClientStage(a, device=dev).forward(x.to(dev)).clone()
    W2, b2 = b.conv2.weight.detach().to(dev).contiguous(), b.conv2.bias.detach().to(dev).contiguous()
    W3, b3 = b.fc1.weight.detach().to(dev).contiguous(), b.fc1.bias.detach().to(dev).contiguous()
    amax = ops.row_amax(act)
    dpa = None
    pooled, code = ops.conv2_fwd_pool(act, W2, b2)
    _, _, _, dp = ops.fc_xent(pooled, W3, b3, y.to(dev), 1.0 / args.B)
    dpa = ops.row_amax(dp)
    cases = {}
    for impl in ("wino", "direct", "x3"):
        if "fwd" in args.ops:
            po, co = torch.empty_like(pooled), torch.empty_like(code)
            cases[f"fwd_{impl}"] = (lambda impl=impl, po=po, co=co: ops.conv2_fwd_pool(
                act, W2, b2, po, co, impl=impl, act_amax=amax))
        if "fwd" in args.ops and impl == "x3":
            a16 = torch.empty(ops.conv2_act16_bytes(args.B), dtype=torch.uint8, device=dev)
            po, co = torch.empty_like(pooled), torch.empty_like(code)
            cases["fwd_x3s"] = (lambda po=po, co=co, a16=a16: ops.conv2_fwd_pool(
                act, W2, b2, po, co, impl="x3", act_amax=amax, act16=a16))
    if "dgrad" in args.ops:
        for impl in ("wino", "direct", "x3"):
            g = torch.empty_like(act)
            cases[f"dgrad_{impl}"] = (lambda impl=impl, g=g: ops.conv2_dgrad(dp, code, W2, g, impl=impl, dp_amax=dpa))
    if "wgrad" in args.ops:
        for impl in ("wino", "x3"):
            sl = torch.empty(ops.conv2_wgrad_nslab(args.B, impl=impl), ops.CONV2_SLAB, device=dev)
            cases[f"wgrad_{impl}"] = (lambda impl=impl, sl=sl: ops.conv2_wgrad_slabs(act, dp, code, sl, impl=impl, act_amax=amax, dp_amax=dpa))
    if "wgrad" in args.ops:
        a16 = torch.empty(ops.conv2_act16_bytes(args.B), dtype=torch.uint8, device=dev)
        ops.conv2_fwd_pool(act, W2, b2, impl="x3", act_amax=amax, act16=a16)
        sl = torch.empty(ops.conv2_wgrad_nslab(args.B, impl="x3"), ops.CONV2_SLAB, device=dev)
        cases["wgrad_x3s"] = (lambda sl=sl, a16=a16: ops.conv2_wgrad_slabs(act, dp, code, sl, impl="x3", act_amax=amax, dp_amax=dpa, act16=a16))
    cases["row_amax"] = lambda: ops.row_amax(act, amax)
    times = {k: [] for k in cases}
    for _ in range(3):
        for f in cases.values():
            f()
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for k, f in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1))
    for k, v in times.items():
        v.sort()
        print(f"{k:14s} median {v[len(v) // 2]:.4f} ms  min {v[0]:.4f}", flush=True)


if __name__ == "__main__":
    main()
