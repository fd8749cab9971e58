"""ctypes binding of the C-ABI in include/msda_hip.h (libmsda_hip.so, built for gfx950).

This is the only place that touches the shared library.  There is no fallback: if the
library is missing or fails to load, every MSDA call raises ``RuntimeError`` (the
reference's native op likewise raises ``AT_ERROR("Not implemented on the CPU")`` for
CPU tensors, models/ops/src/cpu/ms_deform_attn_cpu.cpp:17-41).
"""
import ctypes
import os
import threading

import torch

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = os.path.join(LIB_DIR, "libmsda_hip.so")
# tools only (e.g. a phase-timing debug build); never set by the product path or the tests
LIB_PATH = os.environ.get("MSDA_HIP_LIB", LIB_PATH)

# keep in sync with include/msda_hip.h
DTYPE_TAGS = {torch.float32: 0, torch.float64: 1, torch.bfloat16: 2, torch.float16: 3}
PAD_TAGS = {"border": 0, "zeros": 1}
COORD_API, COORD_LEVEL_MAJOR = 0, 1
MAX_LEVELS = 16
ABI_VERSION = 8

# every symbol include/msda_hip.h declares (checked by tests/test_capi.py)
EXPORTED_SYMBOLS = (
    "msda_hip_forward",
    "msda_hip_backward",
    "msda_hip_backward_ex",
    "msda_hip_backward_workspace_bytes",
    "msda_hip_forward_tiles_bytes",
    "msda_hip_forward_tiles",
    "msda_hip_backward_tiles",
    "msda_hip_prologue_forward",
    "msda_hip_prologue_backward",
    "msda_hip_prologue_forward_ex",
    "msda_hip_prologue_backward_ex",
    "msda_hip_dam_flat_grid",
    "msda_hip_level_major_ok",
    "msda_hip_forward_tiles_layout",
    "msda_hip_backward_tiles_layout",
    "msda_hip_prologue_forward_layout",
    "msda_hip_prologue_backward_layout",
    # include/flat_adamw.h (training-step runtime, same library)
    "flat_adamw_workspace_bytes",
    "flat_adamw_step",
    "flat_adamw_last_error",
    "mfl_colsum_workspace_bytes",
    "mfl_colsum",
    "mfl_colsum_ex",
    "mfl_sum_slabs",
    "mfl_sum_slabs_ex",
    "mfl_stream_create",
    # include/add_layernorm.h
    "mfl_add_layernorm_workspace_bytes",
    "mfl_add_layernorm_forward",
    "mfl_add_layernorm_backward",
    "mfl_add_layernorm_forward_ex",
    "mfl_add_layernorm_backward_ex",
    "mfl_add_layernorm_backward_ex2",
    "mfl_groupnorm_cl_workspace_bytes",
    "mfl_groupnorm_cl_forward",
    "mfl_groupnorm_cl_backward",
    "mfl_carry_entry_forward",
    "mfl_carry_entry_backward",
    "mfl_add_layernorm_last_error",
    # include/ffn_glue.h
    "mfl_relu_dropout_forward",
    "mfl_relu_dropout_backward",
    "mfl_gelu_dropout_forward",
    "mfl_gelu_dropout_backward",
    "mfl_word_prob_backward",
    "mfl_relu_dropout_colsum_workspace_bytes",
    "mfl_relu_dropout_backward_colsum",
    "mfl_level_pos_flatten",
    "mfl_level_pos_flatten_ex",
    "mfl_level_colsum_workspace_bytes",
    "mfl_level_colsum",
    "mfl_pyramid_pos_flatten",
    "mfl_relu_dropout_last_error",
    "mfl_zero_masked_rows",
    "mfl_zero_masked_rows_batched",
    "mfl_augment_rows",
    "mfl_augment_weights",
    "mfl_gather_keep_backward",
    # include/gemm_small.h
    "mfl_gemm_nt_bf16",
    "mfl_gemm_nn_bf16",
    "mfl_gemm_last_error",
    # include/seg_attention.h
    "mfl_seg_attention_forward",
    "mfl_seg_attention_backward",
    "mfl_seg_attention_backward_ex",
    "mfl_seg_attention_forward_ex",
    "mfl_seg_attention_backward_ex2",
    "mfl_seg_attention_drop_bits_bytes",
    "mfl_seg_attention_bias_parts",
    "mfl_seg_attention_workspace_bytes",
    "mfl_seg_attention_last_error",
    # include/host_lsa.h (host code)
    "mfl_lsa",
    "mfl_lsa_levels",
    "msda_hip_last_error",
    "msda_hip_abi_version",
)

_lock = threading.Lock()
_lib = None


def _declare(lib):
    i64, vp, i32 = ctypes.c_int64, ctypes.c_void_p, ctypes.c_int
    p64 = ctypes.POINTER(ctypes.c_int64)
    lib.msda_hip_forward.restype = i32
    lib.msda_hip_forward.argtypes = [vp, i32, p64, p64, i64, vp, vp, vp,
                                     i64, i64, i64, i64, i64, i64, i32, vp]
    lib.msda_hip_backward.restype = i32
    lib.msda_hip_backward.argtypes = [vp, i32, p64, p64, i64, vp, vp, vp, vp, vp, vp, vp,
                                      i64, i64, i64, i64, i64, i64, i32, vp]
    lib.msda_hip_backward_ex.restype = i32
    lib.msda_hip_backward_ex.argtypes = [vp, i32, p64, p64, i64, vp, vp, vp, vp, vp, vp, vp,
                                         i64, i64, i64, i64, i64, i64, i32, i64, vp]
    lib.msda_hip_forward_tiles_bytes.restype = ctypes.c_size_t
    lib.msda_hip_forward_tiles_bytes.argtypes = [i32, p64, i64, i64, i64, i64, i64, i64, i64]
    lib.msda_hip_forward_tiles.restype = i32
    lib.msda_hip_forward_tiles.argtypes = [vp, i32, p64, p64, i64, vp, vp, vp, vp,
                                           i64, i64, i64, i64, i64, i64, i32, vp]
    lib.msda_hip_backward_tiles.restype = i32
    lib.msda_hip_backward_tiles.argtypes = [vp, i32, p64, p64, i64, vp, vp, vp, vp, vp, vp, vp, vp,
                                            i64, i64, i64, i64, i64, i64, i32, vp]
    lib.msda_hip_backward_workspace_bytes.restype = ctypes.c_size_t
    lib.msda_hip_backward_workspace_bytes.argtypes = [i32, i64, i64, i64, i64, i64, i64, i64]
    lib.msda_hip_prologue_forward.restype = i32
    lib.msda_hip_prologue_forward.argtypes = [vp, vp, i32, vp, i32, p64, i64, i64, i64, i64, i64, vp, vp, vp]
    lib.msda_hip_prologue_forward_ex.restype = i32
    lib.msda_hip_prologue_forward_ex.argtypes = [vp, vp, i32, vp, i32, p64, i64, i64, i64, i64, i64, i64, vp, vp, vp]
    lib.msda_hip_prologue_backward_ex.restype = i32
    lib.msda_hip_prologue_backward_ex.argtypes = [vp, vp, vp, vp, i32, vp, i32, p64, i64, i64, i64, i64, i64, i64,
                                                  vp, vp, vp, vp]
    lib.msda_hip_prologue_backward.restype = i32
    lib.msda_hip_prologue_backward.argtypes = [vp, vp, vp, vp, i32, vp, i32, p64, i64, i64, i64, i64, i64,
                                               vp, vp, vp, vp]
    lib.msda_hip_level_major_ok.restype = i32
    lib.msda_hip_level_major_ok.argtypes = [i32, p64, i64, i64, i64, i64, i64, i64, i64]
    lib.msda_hip_forward_tiles_layout.restype = i32
    lib.msda_hip_forward_tiles_layout.argtypes = [vp, i32, p64, p64, i64, vp, vp, vp, vp,
                                                  i64, i64, i64, i64, i64, i64, i32, i32, vp]
    lib.msda_hip_backward_tiles_layout.restype = i32
    lib.msda_hip_backward_tiles_layout.argtypes = [vp, i32, p64, p64, i64, vp, vp, vp, vp, vp, vp, vp, vp,
                                                   i64, i64, i64, i64, i64, i64, i32, i32, vp]
    lib.msda_hip_prologue_forward_layout.restype = i32
    lib.msda_hip_prologue_forward_layout.argtypes = [vp, vp, i32, vp, i32, p64, i64, i64, i64, i64, i64, i64, i32,
                                                     vp, vp, vp]
    lib.msda_hip_prologue_backward_layout.restype = i32
    lib.msda_hip_prologue_backward_layout.argtypes = [vp, vp, vp, vp, i32, vp, i32, p64, i64, i64, i64, i64, i64,
                                                      i64, i32, vp, vp, vp, vp]
    lib.msda_hip_dam_flat_grid.restype = i32
    lib.msda_hip_dam_flat_grid.argtypes = [vp, vp, p64, p64, i64, i64, i64, i64, i64, vp, vp]
    f32 = ctypes.c_float
    lib.mfl_stream_create.restype = ctypes.c_int
    lib.mfl_stream_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    lib.flat_adamw_workspace_bytes.restype = ctypes.c_size_t
    lib.flat_adamw_workspace_bytes.argtypes = []
    lib.flat_adamw_step.restype = i32
    lib.flat_adamw_step.argtypes = [vp, vp, vp, vp, vp, i64, vp, vp, f32, f32, f32, f32, f32, f32, vp, vp]
    lib.mfl_colsum_workspace_bytes.restype = ctypes.c_size_t
    lib.mfl_colsum_workspace_bytes.argtypes = [i64, i64]
    lib.mfl_sum_slabs.restype = i32
    lib.mfl_sum_slabs.argtypes = [vp, i64, i64, vp, vp]
    lib.mfl_colsum.restype = i32
    lib.mfl_colsum.argtypes = [vp, i32, i64, i64, vp, vp, vp]
    lib.mfl_colsum_ex.restype = i32
    lib.mfl_colsum_ex.argtypes = [vp, i32, i64, i64, vp, i32, vp, vp]
    lib.mfl_sum_slabs_ex.restype = i32
    lib.mfl_sum_slabs_ex.argtypes = [vp, i64, i64, i64, vp, i32, vp]
    lib.mfl_add_layernorm_workspace_bytes.restype = ctypes.c_size_t
    lib.mfl_add_layernorm_workspace_bytes.argtypes = [i64, i64]
    lib.mfl_add_layernorm_forward.restype = i32
    lib.mfl_add_layernorm_forward.argtypes = [vp, i32, vp, i32, vp, vp, i64, i64, f32, vp, vp, vp, vp]
    lib.mfl_add_layernorm_backward.restype = i32
    lib.mfl_add_layernorm_backward.argtypes = [vp, vp, i32, vp, i32, vp, vp, vp, i64, i64, vp, vp, vp, vp, vp, vp]
    lib.mfl_add_layernorm_forward_ex.restype = i32
    lib.mfl_add_layernorm_forward_ex.argtypes = [vp, i32, vp, i32, vp, vp, i64, i64, f32, vp, vp, vp, vp, vp, vp, f32,
                                                 vp, vp]
    lib.mfl_add_layernorm_backward_ex.restype = i32
    lib.mfl_add_layernorm_backward_ex.argtypes = [vp, vp, vp, vp, i32, vp, i32, vp, vp, vp, i64, i64, vp, vp, vp, vp,
                                                  vp, f32, vp, vp, vp]
    lib.mfl_add_layernorm_backward_ex2.restype = i32
    lib.mfl_add_layernorm_backward_ex2.argtypes = [vp, vp, vp, vp, i32, vp, i32, vp, vp, vp, i64, i64, vp, vp, vp, vp,
                                                   vp, i32, vp, f32, vp, vp, vp]
    lib.mfl_gemm_nt_bf16.restype = i32
    lib.mfl_gemm_nt_bf16.argtypes = [vp, vp, vp, vp, i64, i64, i64, i64, i64, i64, vp]
    lib.mfl_gather_keep_backward.restype = i32
    lib.mfl_gather_keep_backward.argtypes = [vp, vp, vp, i64, i64, i64, i64, vp, vp, vp]
    lib.mfl_groupnorm_cl_workspace_bytes.restype = ctypes.c_size_t
    lib.mfl_groupnorm_cl_workspace_bytes.argtypes = [i64, i64, i64, i64]
    lib.mfl_groupnorm_cl_forward.restype = i32
    lib.mfl_groupnorm_cl_forward.argtypes = [vp, vp, vp, i64, i64, i64, i64, f32, vp, i64, vp, vp, vp, vp, vp]
    lib.mfl_groupnorm_cl_backward.restype = i32
    lib.mfl_groupnorm_cl_backward.argtypes = [vp, i64, vp, vp, vp, vp, vp, i64, i64, i64, i64, vp, vp, vp, i32, vp,
                                              vp]
    lib.mfl_carry_entry_forward.restype = i32
    lib.mfl_carry_entry_forward.argtypes = [vp, vp, i64, vp, vp, vp]
    lib.mfl_carry_entry_backward.restype = i32
    lib.mfl_carry_entry_backward.argtypes = [vp, vp, vp, i64, vp, vp, i32, vp]
    lib.mfl_level_pos_flatten.restype = i32
    lib.mfl_level_pos_flatten.argtypes = [vp, p64, i64, i64, i64, vp, vp, vp]
    lib.mfl_level_pos_flatten_ex.restype = i32
    lib.mfl_level_pos_flatten_ex.argtypes = [vp, vp, p64, i64, i64, i64, vp, vp, vp]
    lib.mfl_level_colsum_workspace_bytes.restype = ctypes.c_size_t
    lib.mfl_level_colsum_workspace_bytes.argtypes = [p64, i64, i64, i64]
    lib.mfl_pyramid_pos_flatten.restype = i32
    lib.mfl_pyramid_pos_flatten.argtypes = [vp, p64, i64, i64, i64, vp, vp, vp, i32, f32, f32, vp, vp]
    lib.mfl_level_colsum.restype = i32
    lib.mfl_level_colsum.argtypes = [vp, p64, i64, i64, i64, vp, i32, vp, vp]
    lib.mfl_gemm_nn_bf16.restype = i32
    lib.mfl_gemm_nn_bf16.argtypes = [vp, vp, vp, vp, i64, i64, i64, i64, i64, i64, vp]
    lib.mfl_gemm_last_error.restype = ctypes.c_char_p
    lib.mfl_seg_attention_forward.restype = i32
    lib.mfl_seg_attention_forward.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, f32, f32,
                                              vp, vp, vp, vp]
    lib.mfl_seg_attention_backward.restype = i32
    lib.mfl_seg_attention_backward.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, f32, f32,
                                               vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.mfl_seg_attention_backward_ex.restype = i32
    lib.mfl_seg_attention_backward_ex.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, f32,
                                                  f32, vp, vp, vp, vp, vp, vp, vp, i64, i64, vp, vp, vp]
    lib.mfl_seg_attention_forward_ex.restype = i32
    lib.mfl_seg_attention_forward_ex.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, f32,
                                                 f32, vp, vp, vp, vp, vp]
    lib.mfl_seg_attention_backward_ex2.restype = i32
    lib.mfl_seg_attention_backward_ex2.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, f32,
                                                   f32, vp, vp, vp, vp, vp, vp, vp, i64, i64, vp, vp, vp, vp]
    lib.mfl_seg_attention_drop_bits_bytes.restype = i64
    lib.mfl_seg_attention_drop_bits_bytes.argtypes = [i64, i64, i64]
    lib.mfl_seg_attention_bias_parts.restype = i64
    lib.mfl_seg_attention_bias_parts.argtypes = [i64]
    lib.mfl_seg_attention_workspace_bytes.restype = i64
    lib.mfl_seg_attention_workspace_bytes.argtypes = [i64, i64]
    lib.mfl_seg_attention_last_error.restype = ctypes.c_char_p
    lib.mfl_seg_attention_last_error.argtypes = []
    lib.mfl_relu_dropout_forward.restype = i32
    lib.mfl_relu_dropout_forward.argtypes = [vp, i64, f32, vp, vp, vp]
    lib.mfl_relu_dropout_backward.restype = i32
    lib.mfl_relu_dropout_backward.argtypes = [vp, vp, i64, f32, i32, vp, vp]
    lib.mfl_gelu_dropout_forward.restype = i32
    lib.mfl_gelu_dropout_forward.argtypes = [vp, i64, f32, vp, vp, vp]
    lib.mfl_gelu_dropout_backward.restype = i32
    lib.mfl_gelu_dropout_backward.argtypes = [vp, vp, i64, f32, vp, vp, vp]
    lib.mfl_word_prob_backward.restype = i32
    lib.mfl_word_prob_backward.argtypes = [vp, vp, vp, i64, i64, vp, vp]
    lib.mfl_relu_dropout_colsum_workspace_bytes.restype = ctypes.c_size_t
    lib.mfl_relu_dropout_colsum_workspace_bytes.argtypes = [i64, i64]
    lib.mfl_relu_dropout_backward_colsum.restype = i32
    lib.mfl_relu_dropout_backward_colsum.argtypes = [vp, vp, i64, i64, f32, i32, vp, vp, vp, vp]
    lib.mfl_zero_masked_rows.restype = i32
    lib.mfl_zero_masked_rows.argtypes = [vp, i64, i64, vp, vp]
    lib.mfl_zero_masked_rows_batched.restype = i32
    lib.mfl_zero_masked_rows_batched.argtypes = [vp, i64, i64, i64, vp, vp]
    lib.mfl_augment_rows.restype = i32
    lib.mfl_augment_rows.argtypes = [vp, i64, i64, i64, vp, vp]
    lib.mfl_augment_weights.restype = i32
    lib.mfl_augment_weights.argtypes = [vp, vp, i64, i64, i64, i64, vp, vp]
    lib.mfl_relu_dropout_last_error.restype = ctypes.c_char_p
    lib.mfl_relu_dropout_last_error.argtypes = []
    lib.mfl_add_layernorm_last_error.restype = ctypes.c_char_p
    lib.mfl_add_layernorm_last_error.argtypes = []
    lib.flat_adamw_last_error.restype = ctypes.c_char_p
    lib.flat_adamw_last_error.argtypes = []
    lib.msda_hip_last_error.restype = ctypes.c_char_p
    lib.msda_hip_last_error.argtypes = []
    lib.msda_hip_abi_version.restype = i32
    lib.msda_hip_abi_version.argtypes = []
    lib.mfl_lsa.restype = i32
    lib.mfl_lsa.argtypes = [vp, i64, i64, vp, vp]
    lib.mfl_lsa_levels.restype = i32
    lib.mfl_lsa_levels.argtypes = [vp, i64, i64, i64, i64, vp, vp, vp, vp]
    return lib


def load_library():
    """Load (once) and return the ctypes handle of libmsda_hip.so; raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"MSDA HIP library not built: {LIB_PATH} is missing. "
                    "Run `python -c 'import __graft_entry__ as g; g.build()'` first.")
            lib = _declare(ctypes.CDLL(LIB_PATH))
            ver = lib.msda_hip_abi_version()
            if ver != ABI_VERSION:
                raise RuntimeError(f"libmsda_hip.so ABI {ver} != expected {ABI_VERSION}; rebuild")
            _lib = lib
    return _lib


def last_error():
    return load_library().msda_hip_last_error().decode(errors="replace")


MSDA_ERR_UNSUPPORTED = 3  # include/msda_hip.h


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed (status {rc}): {last_error()}")


def host_i64_array(values):
    arr = (ctypes.c_int64 * len(values))(*[int(v) for v in values])
    return arr


def stream_handle(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


_own_streams = {}


def own_stream(device, tag):
    """A HIP stream of the package's own on ``device`` (include/flat_adamw.h mfl_stream_create), wrapped as
    a torch stream, one per (device, tag) for the process: the trainer's capture and bucket-collective
    streams, which must never be a pool stream that the RCCL process group also uses."""
    device = torch.device(device)
    key = (device.index if device.index is not None else torch.cuda.current_device(), tag)
    s = _own_streams.get(key)
    if s is None:
        ptr = ctypes.c_void_p()
        rc = load_library().mfl_stream_create(key[0], ctypes.byref(ptr))
        if rc != 0:
            raise RuntimeError(load_library().flat_adamw_last_error().decode())
        s = torch.cuda.ExternalStream(ptr.value, device=torch.device("cuda", key[0]))
        _own_streams[key] = s
    return s
