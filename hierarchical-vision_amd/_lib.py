"""ctypes binding of libhvk.so (C ABI declared in include/hvk.h).

The product path has exactly one implementation of every hot op: the HIP
kernels in this library.  There is no CPU or eager fallback -- if the library
is missing or a tensor is not on the GPU the call raises.
"""
import contextlib
import ctypes
import os

import torch  # noqa: F401  -- must be imported first: libhvk binds to torch's HIP runtime

_HERE = os.path.dirname(os.path.abspath(__file__))
# HVK_LIB_PATH: another build of the same library (A/B runs of kernel variants, tools/gpu_ab_lib.sh)
LIB_PATH = os.environ.get("HVK_LIB_PATH") or os.path.join(_HERE, "libhvk.so")

_p = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
_sz = ctypes.c_size_t

# name -> (restype, argtypes); kept in the order of include/hvk.h
SIGNATURES = {
    "hvk_abi_version": (_i, []),
    "hvk_kernel_timer_enable": (_i, [_i]),
    "hvk_kernel_timer_read": (_i, [_i, _p, _p]),
    "hvk_kernel_timer_read_work": (_i, [_i, _p, _p, _p]),
    "hvk_kernel_timer_kinds": (_i, [_i]),
    "hvk_kernel_timer_launch": (_i, [_i, _p, _p, _p]),
    "hvk_kernel_timer_launch_shape": (_i, [_i, ctypes.c_char_p, _i, _p, _p]),
    "hvk_last_error_string": (ctypes.c_char_p, []),
    "hvk_set_option": (_i, [ctypes.c_char_p, ctypes.c_longlong, _p]),
    "hvk_get_option": (_i, [ctypes.c_char_p, _p]),
    "hvk_wmsa_fwd": (_i, [_p, _p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p]),
    "hvk_wmsa_bwd_workspace_bytes": (_sz, [_i, _i]),
    "hvk_wmsa_fwd_normed": (_i, [_p, _p, _p, _p, _i, _i, _i, _i, _i, _i, _i, _p]),
    "hvk_wmsa_bwd_normed": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _sz, _i, _i, _i, _i, _i, _i, _i,
                                 _p]),
    "hvk_qk_normalize": (_i, [_p, _p, _p, _i, _i, _p]),
    "hvk_linear_supported": (_i, [_i, _i, _i]),
    "hvk_linear_fwd": (_i, [_p, _p, _p, _p, _i, _i, _i, _p]),
    "hvk_cpb_fwd": (_i, [_p, _p, _p, _p, _p, _f, _i, _i, _i, _p, _p, _p]),
    "hvk_cpb_bwd_workspace_bytes": (_sz, [_i, _i]),
    "hvk_cpb_bwd": (_i, [_p, _p, _p, _p, _p, _f, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _sz,
                         _p]),
    "hvk_linear_qkv_supported": (_i, [_i, _i, _i]),
    "hvk_linear_qkv_fwd": (_i, [_p, _p, _p, _p, _p, _p, _i, _i, _i, _p]),
    "hvk_gemm_qkv_fwd": (_i, [_p, _p, _p, _p, _p, _p, _i, _i, _i, _p]),
    "hvk_linear_gelu_supported": (_i, [_i, _i, _i]),
    "hvk_linear_gelu_fwd": (_i, [_p, _p, _p, _p, _p, _i, _i, _i, _p]),
    "hvk_gemm_supported": (_i, [_i, _i, _i]),
    "hvk_gemm_fwd": (_i, [_p, _p, _p, _p, _i, _i, _i, _p]),
    "hvk_gemm_gelu_fwd": (_i, [_p, _p, _p, _p, _p, _i, _i, _i, _p]),
    "hvk_gemm_gelu_bwd": (_i, [_p, _p, _p, _p, _i, _i, _i, _p]),
    "hvk_weight_grad_supported": (_i, [_i, _i, _i]),
    "hvk_head_supported": (_i, [_i, _i, _i]),
    "hvk_head_fwd": (_i, [_p, _p, _p, _p, _i, _i, _i, _p]),
    "hvk_head_bwd_workspace_bytes": (_sz, [_i, _i, _i]),
    "hvk_head_bwd": (_i, [_p, _p, _p, _p, _p, _p, _i, _i, _i, _p, _sz, _p]),
    "hvk_cast_weights": (_i, [_i, _p, _p, _p, _p, _p, _p]),
    "hvk_block_bias_fwd": (_i, [_p, _p, _p, _p, _i, _p, _p, _p, _p, _p, _f, _i, _i, _i, _p, _p, _p, _p, _p,
                                _p]),
    "hvk_block_bias_bwd": (_i, [_p, _p, _p, _i, _p, _p, _p, _p, _p, _p, _p, _p, _f, _i, _i, _i, _p, _p, _p,
                                _p, _p, _p, _p, _p, _sz, _p]),
    "hvk_attn_bias_fwd": (_i, [_p, _p, _p, _p, _i, _p, _p, _p, _p]),
    "hvk_attn_bias_bwd": (_i, [_p, _p, _p, _i, _p, _p, _p, _p]),
    "hvk_sgdw_workspace_bytes": (_sz, [_i, _p]),
    "hvk_sgdw_step": (_i, [_i, _p, _p, _p, _p, _p, _p, _p, _p, _i, _p, _f, _f, _f, _f, _i, _i, _f, _p, _sz,
                           _p]),
    "hvk_weight_grad_workspace": (_sz, [_i, _i, _i]),
    "hvk_weight_grad": (_i, [_p, _p, _p, _p, _i, _i, _i, _p, _sz, _p]),
    "hvk_weight_grad_shift": (_i, [_p, _p, _p, _p, _p, _i, _i, _i, _p, _sz, _p]),
    "hvk_linear_gelu_bwd_supported": (_i, [_i, _i, _i]),
    "hvk_mlp_fwd_supported": (_i, [_i, _i, _i, _i]),
    "hvk_mlp_fwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p]),
    "hvk_linear_ln_supported": (_i, [_i, _i, _i]),
    "hvk_merge_gemm_supported": (_i, [_i, _i, _i, _i, _i]),
    "hvk_merge_gemm_fwd": (_i, [_p, _p, _p, _i, _i, _i, _i, _i, _p]),
    "hvk_merge_linear_ln_supported": (_i, [_i, _i, _i, _i, _i]),
    "hvk_merge_linear_ln_fwd": (_i, [_p, _p, _i, _i, _i, _i, _i, _p, _p, _f, _p, _p, _p, _p, _p, _p]),
    "hvk_merge_gemm_dgrad": (_i, [_p, _p, _p, _i, _i, _i, _i, _i, _p]),
    "hvk_merge_weight_grad_supported": (_i, [_i, _i, _i, _i, _i]),
    "hvk_merge_weight_grad": (_i, [_p, _p, _p, _i, _i, _i, _i, _i, _p, _sz, _p]),
    "hvk_linear_ln_fwd": (_i, [_p, _p, _i, _i, _i, _p, _p, _p, _p, _p, _i, _f, _p, _p, _p, _p, _p, _p]),
    "hvk_mlp_ln_supported": (_i, [_i, _i, _i, _i]),
    "hvk_mlp_ln_fwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _i, _f, _p, _p, _p, _p,
                            _p]),
    "hvk_mlp_bwd_supported": (_i, [_i, _i, _i, _i]),
    "hvk_mlp_bwd": (_i, [_p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p]),
    "hvk_linear_gelu_in_supported": (_i, [_i, _i, _i]),
    "hvk_linear_gelu_in_fwd": (_i, [_p, _p, _p, _p, _i, _i, _i, _p]),
    "hvk_weight_grad_gelu_x_supported": (_i, [_i, _i, _i]),
    "hvk_weight_grad_gelu_x": (_i, [_p, _p, _p, _p, _i, _i, _i, _p, _sz, _p]),
    "hvk_linear_gelu_bwd": (_i, [_p, _p, _p, _p, _p, _i, _i, _i, _p]),
    "hvk_wmsa_bwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _sz, _i, _i, _i, _i, _i, _i, _i,
                          _p]),
    "hvk_ln_residual_fwd": (_i, [_p, _p, _p, _p, _p, _p, _i, _i, _i, _f, _p, _p, _p, _p, _p]),
    "hvk_ln_bwd_workspace_bytes": (_sz, [_i]),
    "hvk_ln_residual_bwd": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p, _p,
                                 _p, _sz, _p]),
    "hvk_ln_residual_bwd_split": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p, _p,
                                       _p, _sz, _p, _p]),
    "hvk_bias_gelu_fwd": (_i, [_p, _p, _p, _i, _i, _p]),
    "hvk_bias_gelu_bwd_workspace_bytes": (_sz, [_i]),
    "hvk_bias_gelu_bwd": (_i, [_p, _p, _p, _p, _p, _p, _sz, _i, _i, _p]),
    "hvk_patch_merge_gather": (_i, [_p, _p, _i, _i, _i, _i, _p]),
    "hvk_patch_merge_scatter": (_i, [_p, _p, _i, _i, _i, _i, _p]),
    "hvk_ln_pool_supported": (_i, [_i]),
    "hvk_ln_pool_fwd": (_i, [_p, _p, _p, _i, _i, _i, _f, _p, _p, _p, _p, _p, _p, _p]),
    "hvk_ln_pool_bwd": (_i, [_p, _p, _p, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p]),
    "hvk_patchify_bf16": (_i, [_p, _p, _i, _i, _i, _i, _p]),
    "hvk_patchify_u8_bf16": (_i, [_p, _p, _p, _p, _i, _i, _i, _i, _p]),
    "hvk_normalize_u8": (_i, [_p, _p, _p, _p, _i, _i, _i, _p]),
    "hvk_multitask_ce_fwd": (_i, [_p, _i, _i, _i, _p, _p, _p, _p, _p, _p]),
    "hvk_multitask_ce_bwd": (_i, [_p, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p]),
    "hvk_hxe_fwd": (_i, [_p, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "hvk_hxe_bwd": (_i, [_p, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
}

_lib = None
ABI_VERSION = 14  # include/hvk.h's HVK_ABI_VERSION, the ABI this binding's SIGNATURES describe


def load():
    """Load libhvk.so once and attach the signatures of include/hvk.h."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                "g.build()'` (or `make -C hierarchical-vision_amd/csrc`).  There is no fallback.")
        lib = ctypes.CDLL(LIB_PATH)
        # an older build (an A/B variant through HVK_LIB_PATH) may export the same names with
        # other argument lists: calling those would shift pointers, so refuse it outright
        lib.hvk_abi_version.restype = _i
        abi = lib.hvk_abi_version()
        if abi != ABI_VERSION:
            raise RuntimeError(f"{LIB_PATH} has C ABI {abi}, this binding expects {ABI_VERSION}: "
                               "rebuild it (make -C hierarchical-vision_amd/csrc)")
        for name, (res, args) in SIGNATURES.items():
            # an older A/B build (HVK_LIB_PATH) may predate an entry point; the shipped one may not
            fn = getattr(lib, name, None)
            if fn is None:
                if os.environ.get("HVK_LIB_PATH"):
                    continue
                raise RuntimeError(f"{LIB_PATH} does not export {name} (stale build?)")
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


# the library's named options (include/hvk.h, hvk_set_option); bench.py prints options()
LIB_OPTIONS = ("wmsa_fwd_form", "wmsa_bwd_nt", "wmsa_bwd_slice_bytes", "tile_wide", "dw_tile", "wmsa_fwd_hg",
               "dw_chunks")


def options():
    """{name: value} of every libhvk option (what a result line names beside options.as_dict())."""
    return {n: get_option(n) for n in LIB_OPTIONS}


def set_option(name, value):
    """Set a libhvk option (include/hvk.h); returns the previous value."""
    lib = load()
    prev = ctypes.c_longlong()
    rc = lib.hvk_set_option(name.encode(), int(value), ctypes.byref(prev))
    if rc != 0:
        raise RuntimeError(f"hvk_set_option failed: {lib.hvk_last_error_string().decode(errors='replace')}")
    return prev.value


def get_option(name):
    lib = load()
    v = ctypes.c_longlong()
    if lib.hvk_get_option(name.encode(), ctypes.byref(v)) != 0:
        raise RuntimeError(f"hvk_get_option failed: {lib.hvk_last_error_string().decode(errors='replace')}")
    return v.value


@contextlib.contextmanager
def option(name, value):
    """with option("wmsa_fwd_form", 1): ... -- restores the previous value on exit."""
    prev = set_option(name, value)
    try:
        yield
    finally:
        set_option(name, prev)


def call(name, *args):
    """Invoke an hvk_* entry point and raise RuntimeError on a non-zero status."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.hvk_last_error_string().decode(errors="replace")
        raise RuntimeError(f"{name} failed (status {rc}): {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL).  Refuses CPU tensors."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("libhvk ops run on the GPU only; got a CPU tensor")
    if not t.is_contiguous():
        raise RuntimeError("libhvk ops need contiguous tensors")
    return ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
