"""Profiling only: host-side (Python) cost of bench.py's drop-in module step — cProfile over 30 steps after
warm-up. The reference's step code syncs once per step (loss.item()), so the host work after that sync
(cut-gradient clone, client backward, both optimizers, the next forward's dispatch) is on the critical path."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    X, Y = bench.make_pool(4096, 4, torch.device("cuda:0"))
    bench.run_dropin(X, Y, 10, 3)            # warm-up (graphs, caches, allocator)
    pr = cProfile.Profile()
    pr.enable()
    r = bench.run_dropin(X, Y, 30, 1)
    pr.disable()
    print(r["ms_per_step"], "ms/step", flush=True)
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(40)
