"""Profiling aid: the K4 hub server's chunked step on one GPU (bench.py's k4_server_loopback) alone.
usage: python tools/hub_loopback.py [--micro 4] [--batch 4096] [--dense-exchange] [--no-graph]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]

import bench  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--micro", type=int, default=4)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--dense-exchange", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    a = ap.parse_args()
    print(bench.hub_loopback_rate(a, None, None))
