"""Build libslk.so (the gfx950 HIP kernels + C-ABI) in-tree with hipcc.

The library is built into this package directory so it travels with the repository snapshot to the
GPU box (a JIT cache under ~/.cache would not). `python -m splitcnn.build` or
`__graft_entry__.build()` drive it; it cross-compiles without a GPU.
"""
from __future__ import annotations

import hashlib
import os
import re
import shutil
import subprocess
import sys
import tempfile

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC_DIR = os.path.join(os.path.dirname(PKG_DIR), "csrc")
INCLUDE_DIR = os.path.join(os.path.dirname(os.path.dirname(PKG_DIR)), "include")
LIB_PATH = os.path.join(PKG_DIR, "libslk.so")
SOURCES = ["slk_client.hip", "slk_server.hip", "slk_optim.hip", "slk_data.hip", "slk_wide.hip",
           "slk_wide_head.hip", "slk_wino.hip", "slk_codec.hip", "slk_x3.hip"]
ARCH = "gfx950"
# Per-source extra hipcc flags (none needed at present; tools/build_variant.sh passes -D defines).
EXTRA_FLAGS: dict = {}


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the splitcnn kernels need ROCm's hipcc to build")


def _inputs():
    srcs = [os.path.join(CSRC_DIR, s) for s in SOURCES]
    hdrs = [os.path.join(CSRC_DIR, f) for f in os.listdir(CSRC_DIR) if f.endswith(".h")]
    hdrs.append(os.path.join(INCLUDE_DIR, "slk.h"))
    return srcs, hdrs


def source_hash(defines=()) -> str:
    """sha256 over every input of the library (the HIP sources, csrc/*.h, include/slk.h, by name and
    content) and the extra -D defines it is compiled with (none for the product library). It is
    compiled into libslk.so (slk_build_id), so a binary is tied to its sources AND its defines: a
    variant build with tuning defines never passes as the product library."""
    srcs, hdrs = _inputs()
    h = hashlib.sha256()
    h.update(b"defines:" + " ".join(sorted(defines)).encode() + b"\0")
    for f in sorted(srcs + hdrs, key=os.path.basename):
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


_TAG = re.compile(rb"SLK_BUILD_ID:([0-9a-f]{64})")


def library_build_id(path: str = LIB_PATH):
    """The source hash baked into a built library (read from the file, without loading it)."""
    try:
        with open(path, "rb") as fh:
            m = _TAG.search(fh.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def needs_build() -> bool:
    """True unless the library exists AND was built from exactly the current sources (hash, not mtime)."""
    return library_build_id(LIB_PATH) != source_hash()


def _compile_cmd(src: str, obj: str, defines) -> list:
    return [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-I", INCLUDE_DIR, *defines,
            f'-DSLK_BUILD_ID="{source_hash(defines)}"', *EXTRA_FLAGS.get(os.path.basename(src), []), "-c", src,
            "-o", obj]


def defines_path(lib_path: str) -> str:
    """Where a variant build records its -D defines (next to the library)."""
    return os.path.splitext(lib_path)[0] + ".defines"


def build_library(force: bool = False, verbose: bool = False, out: str | None = None, defines=()) -> str:
    """Compile every HIP source for gfx950 (one object per source, in parallel, with its per-source
    flags) and link libslk.so next to this file — or `out` with extra `defines` (profiling variants)."""
    target = out or LIB_PATH
    if out is None and not force and not needs_build():
        return LIB_PATH
    srcs, _ = _inputs()
    tmpdir = tempfile.mkdtemp(prefix="slk_build_")
    try:
        jobs = []
        for src in srcs:
            obj = os.path.join(tmpdir, os.path.basename(src) + ".o")
            cmd = _compile_cmd(src, obj, list(defines))
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            jobs.append((src, obj, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
        failed = []
        for src, _, proc in jobs:
            _, err = proc.communicate()
            if proc.returncode != 0:
                failed.append(f"{os.path.basename(src)} ({proc.returncode}):\n{err[-4000:]}")
        if failed:
            raise RuntimeError("hipcc failed: " + "\n".join(failed))
        tmp = target + ".tmp"
        link = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *[obj for _, obj, _ in jobs], "-o", tmp]
        if verbose:
            print(" ".join(link), file=sys.stderr)
        res = subprocess.run(link, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"hipcc link failed ({res.returncode}):\n{res.stderr[-4000:]}")
        os.replace(tmp, target)
        if out is not None:
            with open(defines_path(target), "w") as fh:
                fh.write(" ".join(sorted(defines)) + "\n")
    finally:
        shutil.rmtree(tmpdir, ignore_errors=True)
    return target


if __name__ == "__main__":
    print(build_library(force="--force" in sys.argv, verbose=True))
