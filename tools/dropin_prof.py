"""Profiling only: bench.py's drop-in module step (the reference's step code on the drop-in modules) alone,
for `rocprofv3 --kernel-trace --stats -- python tools/dropin_prof.py`. Prints the bench's dict."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    X, Y = bench.make_pool(4096, 4, torch.device("cuda:0"))
    print(json.dumps(bench.run_dropin(X, Y, steps, 3)), flush=True)
