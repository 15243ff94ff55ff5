"""Profiling-only: run bench.py against an alternative libslk build. usage: python tools/bench_with_lib.py LIB [bench args]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "split-learning-k8s_amd"), ROOT]
from splitcnn import _lib  # noqa: E402

_lib.load(sys.argv[1])
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
