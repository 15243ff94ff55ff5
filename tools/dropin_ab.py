"""Profiling only: A/B of the drop-in module step (bench.run_dropin: the reference's step code on the
drop-in modules) with the conv2 forward computing the per-sample max |act| itself (slk_conv2_fwd_pool_x3sa,
the product path) vs the previous row_amax pass + forward. Interleaved rounds in one process; medians."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]

import torch  # noqa: E402

import bench  # noqa: E402
from splitcnn import library, ops  # noqa: E402


class _RowAmaxOps:
    """ops with conv2_fwd_pool(act_amax_out=...) turned back into row_amax + the forward."""

    def __getattr__(self, k):
        return getattr(ops, k)

    @staticmethod
    def conv2_fwd_pool(act, W2, b2, act_amax_out=None, **kw):
        if act_amax_out is not None:
            act_amax_out.copy_(ops.row_amax(act))
            return ops.conv2_fwd_pool(act, W2, b2, act_amax=act_amax_out, **kw)
        return ops.conv2_fwd_pool(act, W2, b2, **kw)


def _op_times(rounds):
    """Kernel-level: row_amax + the act16 forward vs the forward with the in-kernel max (HIP events, B = 4096)."""
    from splitcnn.data import SyntheticMNIST, init_models
    from splitcnn.engine import ClientStage
    dev = torch.device("cuda:0")
    a, s = init_models(seed=0)
    x, _ = SyntheticMNIST(0).batch(4096)
    act = ClientStage(a, device=dev).forward(x.to(dev)).clone()
    W2, b2 = s.conv2.weight.detach().to(dev).contiguous(), s.conv2.bias.detach().to(dev).contiguous()
    a16 = torch.empty(ops.conv2_act16_bytes(4096), dtype=torch.uint8, device=dev)
    am = torch.empty(4096, device=dev)
    pooled = torch.empty(4096, 64, 12, 12, device=dev)
    code = torch.empty(4096, 64, 12, 12, dtype=torch.uint8, device=dev)
    cases = {
        "row_amax": lambda: ops.row_amax(act),
        "fwd_x3s": lambda: ops.conv2_fwd_pool(act, W2, b2, pooled, code, impl="x3", act_amax=am, act16=a16),
        "fwd_x3sa": lambda: ops.conv2_fwd_pool(act, W2, b2, pooled, code, impl="x3", act16=a16, act_amax_out=am),
    }
    res = {k: [] for k in cases}
    for _ in range(rounds):
        for k, f in cases.items():
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                f()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / 20)
    for k, v in res.items():
        print(f"op {k:10s} median {statistics.median(v):.4f} ms  min {min(v):.4f}", flush=True)


if __name__ == "__main__":
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    _op_times(rounds)
    X, Y = bench.make_pool(4096, 4, torch.device("cuda:0"))
    cases = {"fused_amax": ops, "row_amax": _RowAmaxOps()}
    res = {k: [] for k in cases}
    for k, o in cases.items():  # warm-up
        library.ops = o
        bench.run_dropin(X, Y, 10, 3)
    for _ in range(rounds):
        for k, o in cases.items():
            library.ops = o
            r = bench.run_dropin(X, Y, 30, 2)
            res[k].append(r["ms_per_step"])
    library.ops = ops
    for k, v in res.items():
        print(f"{k:12s} median {statistics.median(v):.4f} ms/step  min {min(v):.4f}  "
              f"({4096 / statistics.median(v) / 1e3:.3f} M samples/s)", flush=True)
    print(json.dumps(res))
