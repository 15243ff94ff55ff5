"""ctypes binding of libslk.so (include/slk.h).

The library must already be built (splitcnn.build / __graft_entry__.build()). There is no CPU or
PyTorch fallback: if the library is missing, or the device is not a ROCm GPU, every op raises.
torch is imported first so that the process's HIP runtime is torch's libamdhip64.so.7; libslk.so
names the same soname and therefore binds to that one runtime instance.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime before libslk.so)

from .build import CSRC_DIR, LIB_PATH, source_hash

_c_float_p = ctypes.c_void_p  # device pointers travel as integers
_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_U = ctypes.c_uint
_L = ctypes.c_int64

# name -> argtypes (restype is int unless listed in _RESTYPES)
_SIGS = {
    "slk_abi_version": [],
    "slk_cut_blocks": [_L],
    "slk_cut_encode": [_P, _L, _P, _P, _P, _P, _P, _P],
    "slk_cut_offsets": [_P, _L, _P, _P, _P, _P],
    "slk_cut_pack": [_P, _L, _P, _P, _P, _P],
    "slk_cut_unpack": [_P, _L, _P, _P, _P, _P],
    "slk_cut_ranks": [_P, _L, _P, _P, _P],
    "slk_cut_unpack_x3": [_P, _P, _P, _P, _I, _P, _P],
    "slk_conv2_dgrad_x3_pack": [_P, _P, _P, _P, _P, _P, _P, _I, _P],
    "slk_cut_offsets_ranks_parts": [_P, _I, _L, _P],
    "slk_cut_unpack_x3_parts": [_P, _I, _P, _I, _P, _P],
    "slk_conv2_dgrad_x3_pack_parts": [_P, _P, _P, _P, _P, _I, _I, _P],
    "slk_error_string": [_I],
    "slk_build_id": [],
    "slk_conv1_fwd": [_P, _P, _P, _P, _I, _P],
    "slk_conv1_fwd_amax": [_P, _P, _P, _P, _P, _I, _P],
    "slk_conv1_wgrad": [_P, _P, _P, _P, _I, _P],
    "slk_conv1_wgrad_nslab": [_I],
    "slk_conv1_wgrad_remask": [_P, _P, _P, _P, _P, _I, _P],
    "slk_conv2_fwd_pool": [_P, _P, _P, _P, _P, _I, _P],
    "slk_conv2_fwd_pool_direct": [_P, _P, _P, _P, _P, _I, _P],
    "slk_fc_fwd": [_P, _P, _P, _P, _I, _P],
    "slk_xent_fwd_bwd": [_P, _P, _P, _P, _F, _P, _I, _P],
    "slk_fc_logits_xent": [_P, _P, _P, _P, _P, _P, _P, _F, _P, _I, _P],
    "slk_fc_dgrad": [_P, _P, _P, _I, _P],
    "slk_fc_dgrad_amax": [_P, _P, _P, _P, _I, _P],
    "slk_fc_xent": [_P, _P, _P, _P, _P, _P, _P, _P, _F, _P, _I, _P],
    "slk_fc_xent_amax": [_P, _P, _P, _P, _P, _P, _P, _P, _P, _F, _P, _I, _P],
    "slk_fc_wgrad": [_P, _P, _P, _I, _P],
    "slk_fc_wgrad_nslab": [_I],
    "slk_conv2_dgrad": [_P, _P, _P, _P, _I, _P],
    "slk_conv2_dgrad_direct": [_P, _P, _P, _P, _I, _P],
    "slk_conv2_wgrad": [_P, _P, _P, _P, _I, _P],
    "slk_conv2_wgrad_nslab": [_I],
    "slk_conv2_wgrad_direct": [_P, _P, _P, _P, _I, _P],
    "slk_conv2_wgrad_direct_nslab": [_I],
    "slk_row_amax": [_P, _I, _I, _P, _P],
    "slk_conv2_fwd_pool_x3": [_P, _P, _P, _P, _P, _P, _I, _P],
    "slk_conv2_dgrad_x3": [_P, _P, _P, _P, _P, _I, _P],
    "slk_conv2_wgrad_x3": [_P, _P, _P, _P, _P, _P, _I, _P],
    "slk_conv2_wgrad_x3_nslab": [_I],
    "slk_conv2_fwd_pool_x3s": [_P, _P, _P, _P, _P, _P, _P, _I, _P],
    "slk_conv2_fwd_pool_x3sa": [_P, _P, _P, _P, _P, _P, _P, _I, _P],
    "slk_mfma_probe": [_P, _I, _P],
    "slk_mfma_probe_blocks": [],
    "slk_conv2_wgrad_x3s": [_P, _P, _P, _P, _P, _P, _I, _P],
    "slk_conv2_wgrad_x3_form": [],
    "slk_conv2_act16_bytes": [_I],
    "slk_conv1_fwd_x3": [_P, _P, _P, _P, _P, _P, _P, _I, _P],
    "slk_relu_bits_bytes": [_I],
    "slk_conv2_fwd_pool_x3i": [_P, _P, _P, _P, _P, _P, _I, _P],
    "slk_conv2_dgrad_x3_c1w": [_P, _P, _P, _P, _P, _P, _P, _I, _P],
    "slk_conv2_dgrad_x3_c1w_nslab": [_I],
    "slk_reduce_slabs": [_P, _I, _I, _P, _I, _P],
    "slk_sgd_from_slabs": [_P, _P, _P, _I, _I, _F, _P],
    "slk_sgd": [_P, _P, _I, _F, _P],
    "slk_loss_sum": [_P, _I, _F, _P, _P],
    "slk_loss_log": [_P, _I, _F, _P, _I, _P, _P],
    "slk_sgd_multi_from_slabs": [_P, _P, _P, _P, _P, _I, _F, _P, _I, _F, _P, _I, _P, _P],
    "slk_mnist_batch": [_P, _P, _I, _P, _I, _F, _F, _P, _P, _P, _P],
    # widened split CNN (BASELINE config 5)
    "slk_wide_conv1_fwd": [_P, _P, _P, _P, _P, _I, _P],
    "slk_wide_relu_bits": [_P, _P, _I, _P],
    "slk_wide_conv2_fwd": [_P, _P, _P, _P, _P, _I, _P],
    "slk_wide_conv3_fwd": [_P, _P, _P, _P, _P, _I, _P],
    "slk_wide_head": [_P, _P, _P, _P, _P, _U, _U, _F, _F, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P],
    "slk_wide_head_nslab": [_I],
    "slk_wide_head_fwd": [_P, _P, _P, _P, _U, _U, _F, _P, _I, _I, _P],
    "slk_wide_head_bwd": [_P, _P, _P, _P, _U, _U, _F, _P, _P, _I, _I, _P],
    "slk_wide_head_work": [_I],
    "slk_wide_conv3_wgrad": [_P, _P, _P, _P, _I, _P],
    "slk_wide_conv3_wgrad_nslab": [_I],
    "slk_wide_conv3_dgrad": [_P, _P, _P, _P, _I, _P],
    "slk_wide_conv2_wgrad": [_P, _P, _P, _P, _I, _P],
    "slk_wide_conv2_wgrad_nslab": [_I],
    "slk_wide_wgrad_form": [],
    "slk_wide_conv2_dgrad": [_P, _P, _P, _P, _P, _I, _P],
    "slk_wide_conv1_wgrad": [_P, _P, _P, _I, _P],
    "slk_wide_conv1_wgrad_nslab": [_I],
    "slk_adam_from_slabs": [_P, _P, _P, _P, _P, _I, _I, _F, _F, _F, _F, _P, _P],
    "slk_adam_multi_from_slabs": [_P, _P, _P, _P, _P, _P, _P, _I, _F, _F, _F, _F, _P, _P],
    "slk_wide_shadows": [_P, _P, _P, _P, _P, _P, _P, _P, _P],
    "slk_wide_fc_shadow": [_P, _P, _P],
    "slk_tick": [_P, _P],
}
_RESTYPES = {"slk_error_string": ctypes.c_char_p, "slk_build_id": ctypes.c_char_p, "slk_conv2_act16_bytes": ctypes.c_int64,
             "slk_relu_bits_bytes": ctypes.c_int64}

SYMBOLS = tuple(_SIGS)

_lib = None


class SLKError(RuntimeError):
    """A libslk.so entry point returned a nonzero hipError_t."""


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libslk.so once and attach the signatures; raises if it is missing or incomplete."""
    global _lib
    if _lib is not None:
        return _lib
    # profiling only: run the same Python path over a variant build (tools/build_variant.sh output). Its
    # build id hashes the sources AND its -D defines (recorded next to it), so it is checked against
    # those, and VARIANT_DEFINES says so to every caller (bench.py prints it in its JSON line).
    global VARIANT_DEFINES
    defines = ()
    if os.environ.get("SLK_LIB_VARIANT"):
        path = os.environ["SLK_LIB_VARIANT"]
        from .build import defines_path
        try:
            defines = tuple(open(defines_path(path)).read().split())
        except OSError:
            raise ImportError(f"splitcnn: variant {path} has no {defines_path(path)} (build it with "
                              "tools/build_variant.sh)")
    if not os.path.exists(path):
        raise ImportError(
            f"splitcnn: {path} is missing. Build the HIP kernels first "
            "(python -c 'import __graft_entry__ as g; g.build()'). There is no CPU fallback.")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, args in _SIGS.items():
        fn = getattr(lib, name)  # AttributeError here means the .so does not match slk.h
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    # provenance: the library must have been built from exactly the sources in this tree
    if os.path.isdir(CSRC_DIR):
        built, want = lib.slk_build_id().decode(), source_hash(defines)
        if built != want:
            raise ImportError(
                f"splitcnn: {path} was built from other sources (build id {built[:12]}, tree {want[:12]}). "
                "Rebuild it (python -c 'import __graft_entry__ as g; g.build()').")
    VARIANT_DEFINES = defines if os.environ.get("SLK_LIB_VARIANT") else None
    _lib = lib
    return lib


VARIANT_DEFINES = None   # the -D defines of a loaded variant build (None: the product library)


def build_id() -> str:
    """slk_build_id of the loaded library (sha256 of its sources and defines)."""
    return load().slk_build_id().decode()


def call(name: str, *args) -> None:
    """Invoke an slk_* entry point and raise SLKError on a nonzero hipError_t."""
    err = getattr(load(), name)(*args)
    if err != 0:
        msg = load().slk_error_string(err)
        raise SLKError(f"{name} failed: hipError {err} ({msg.decode() if msg else '?'})")


def query(name: str, *args) -> int:
    """Invoke a size-query entry point (returns a value, not a status)."""
    return int(getattr(load(), name)(*args))
