"""Profiling only: bench.run_dropin (the reference's step code on the drop-in modules, B = 4096) with the eager
autograd.Function fast path (library.eager) on and off, interleaved rounds in one process; medians of ms/step."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]

import torch  # noqa: E402

import bench  # noqa: E402
from splitcnn import library  # noqa: E402

if __name__ == "__main__":
    X, Y = bench.make_pool(4096, 4, torch.device("cuda:0"))
    res = {"fast": [], "custom_ops": []}
    for r in range(6):
        for k in res:
            library._EAGER = k == "fast"
            res[k].append(bench.run_dropin(X, Y, 20, 3)["ms_per_step"])
    for k, v in res.items():
        print(f"{k:11s} median {statistics.median(v):.3f} ms/step  min {min(v):.3f}  ({4096 / statistics.median(v) / 1e3:.3f} M samples/s)")
    print(json.dumps(res))
