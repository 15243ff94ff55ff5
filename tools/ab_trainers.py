"""Profiling only: K2 SplitTrainer variants (engine attributes) captured as HIP graphs and timed
interleaved in ONE process, B = 4096. usage: python tools/ab_trainers.py [--rounds 8]
Variants: the conv presets (engine.CONV_PRESETS) and the default without its fusions. (Round 2 also timed
launch-order knobs here — fc wgrad early, conv2 wgrad first — both slower; round 4 re-times them with
--order after the head moved to the MFMA.)"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]

import torch  # noqa: E402

from bench import make_pool  # noqa: E402
from splitcnn.data import init_models  # noqa: E402
from splitcnn.engine import SplitTrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--order", action="store_true", help="the launch-order knobs instead of the presets")
    args = ap.parse_args()
    B = 4096
    dev = torch.device("cuda:0")
    X, Y = make_pool(B, 4, dev)
    variants = {}
    configs = {"x3": {}, "x3_unfused": {"fuse_client_backward": False}, "x3w": {"conv": "x3w"}, "f32": {"conv": "f32"}}
    # the default splits the head (fc_split); the fused-head orders set it off
    server_attrs = {"x3_fused_head": {"fc_split": False}, "x3_two_launch_head": {"fc_one_launch": False},
                    "x3_fcw_early": {"fc_split": False, "fc_wgrad_early": True},
                    "x3_wgrad_first": {"wgrad_first": True}}
    ap_head = os.environ.get("AB_HEAD") == "1"  # the round-6 one-launch head vs the two launches only
    if args.order:
        configs = {"x3": {}, **{k: {} for k in server_attrs}}
    if ap_head:
        configs = {"x3": {}, "x3_two_launch_head": {}}
    for name, kw in configs.items():
        tr = SplitTrainer(*init_models(seed=0), device=dev, graph=True, **kw)
        for a, v in server_attrs.get(name, {}).items():
            setattr(tr.server, a, v)
        for i in range(5):
            tr.step(X[i % 4], Y[i % 4])
        variants[name] = tr
    times = {k: [] for k in variants}
    for _ in range(args.rounds):
        for k, tr in variants.items():
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(args.steps):
                tr.step(X[i % 4], Y[i % 4])
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / args.steps)
    for k, v in times.items():
        v.sort()
        print(f"{k:10s} median {v[len(v) // 2]:.4f} ms/step  min {v[0]:.4f}", flush=True)
    if args.order:  # every order ran the same steps on the same batches: parameters must be bit-identical
        ref = variants["x3"]
        for k, tr in variants.items():
            same = (torch.equal(tr.server.params, ref.server.params)
                    and torch.equal(tr.client.params, ref.client.params))
            print(f"{k:10s} parameters bit-identical to x3: {same}", flush=True)


if __name__ == "__main__":
    main()
