"""ctypes binding of the C ABI in ``include/stylemc_hip.h`` (``stylemc_amd/_lib/libstylemc_hip.so``).

The library is loaded after ``import torch`` so its ``libamdhip64.so.7`` dependency resolves to the
HIP runtime torch already loaded (one runtime, so torch's streams are valid handles here).
There is no fallback: if the library is missing or a call fails, a RuntimeError is raised.
"""
import contextlib
import ctypes
import os
import threading

import torch

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SMC_HIP_LIB", os.path.join(PKG, "_lib", "libstylemc_hip.so"))

c_int, c_int64, c_float, c_void_p, c_char_p = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p, ctypes.c_char_p

ACT_CODES = {"linear": 1, "relu": 2, "lrelu": 3, "tanh": 4, "sigmoid": 5, "elu": 6, "selu": 7, "softplus": 8,
             "swish": 9}
EPI_STORE, EPI_MODACT, EPI_PRELU, EPI_PRELU_GRAD, EPI_AFFINE = 0, 1, 2, 3, 4


class ConvPhase(ctypes.Structure):
    _fields_ = [("ntaps", c_int), ("tap_dy", c_int * 9), ("tap_dx", c_int * 9), ("in_stride", c_int),
                ("out_h", c_int), ("out_w", c_int), ("out_oy", c_int), ("out_ox", c_int), ("out_sy", c_int),
                ("out_sx", c_int), ("wk", c_void_p), ("wino_u", c_void_p), ("wk_x3", c_void_p)]


class ConvEpilogue(ctypes.Structure):
    _fields_ = [("mode", c_int), ("d", c_void_p), ("noise", c_void_p), ("noise_nstride", c_int64),
                ("noise_strength", c_void_p), ("bias", c_void_p), ("act", c_int), ("alpha", c_float),
                ("gain", c_float), ("clamp", c_float), ("u_save", c_void_p), ("scale_c", c_void_p),
                ("alpha_c", c_void_p), ("act_ref", c_void_p), ("residual", c_void_p), ("residual_stride", c_int),
                ("grad_from_y", c_int)]


class LinearEpilogue(ctypes.Structure):
    _fields_ = [("bias", c_void_p), ("dact_pre", c_void_p), ("ld_dact", c_int), ("act", c_int),
                ("pre_save", c_void_p), ("ld_pre", c_int), ("residual", c_void_p), ("ld_res", c_int)]


class VitConfig(ctypes.Structure):
    _fields_ = [("width", c_int), ("layers", c_int), ("heads", c_int), ("patch", c_int), ("grid", c_int),
                ("out_dim", c_int), ("in_ch", c_int), ("ln_eps", c_float), ("products", c_int)]


LIN_ACT_NONE, LIN_ACT_QUICKGELU = 0, 1

P = c_void_p
_SIGS = {
    "smc_abi_version": (c_int, []),
    "smc_set_plan_batch": (c_int, [c_int, c_int]),
    "smc_conv_gemm_last_x3": (c_int, []),
    "smc_last_error": (c_char_p, []),
    "smc_bias_act_f32": (c_int, [P, P, P, P, P, P, c_int64, c_int64, c_int64, c_int, c_int, c_float, c_float, c_float,
                                 P]),
    "smc_upfirdn2d_f32": (c_int, [P, P, P, c_int64] + [c_int] * 15 + [c_float, P]),
    "smc_conv_gemm_workspace_size": (c_int64, [c_int, c_int, c_int, c_int, c_int, P, c_int]),
    "smc_conv_gemm_f32": (c_int, [P, c_int, c_int, c_int, c_int, P, c_int, c_int, c_int, P, c_int, P, P, P, c_int64,
                                  P]),
    "smc_conv_weights_x3_bytes": (c_int64, [c_int, c_int, c_int]),
    "smc_conv_weights_x3": (c_int, [P, c_int, c_int, c_int, P, P]),
    "smc_conv3x3_wino_supported": (c_int, [c_int, c_int, c_int, c_int, c_int]),
    "smc_conv3x3_wino_f32": (c_int, [P, c_int, c_int, c_int, c_int, P, c_int, P, P, P, P]),
    "smc_conv3x3_wino_workspace_size": (c_int64, [c_int, c_int, c_int, c_int, c_int]),
    "smc_set_wino_x3": (c_int, [c_int]),
    "smc_conv3x3_wino_ws_f32": (c_int, [P, c_int, c_int, c_int, c_int, P, c_int, P, P, P, P, c_int64, P]),
    "smc_wino_weights_f32": (c_int, [P, c_int, c_int, c_int, P, P]),
    "smc_conv3x3_wino4_supported": (c_int, [c_int, c_int, c_int, c_int, c_int]),
    "smc_conv3x3_wino4_f32": (c_int, [P, c_int, c_int, c_int, c_int, P, c_int, P, P, P, P]),
    "smc_wino4_weights_f32": (c_int, [P, c_int, c_int, c_int, P, P]),
    "smc_wino_sp_supported": (c_int, [c_int, c_int, c_int, c_int, c_int]),
    "smc_wino_sp_workspace_size": (c_int64, [c_int, c_int, c_int, c_int, c_int]),
    "smc_wino_taps_f32": (c_int, [P, c_int, c_int, P, P]),
    "smc_conv3x3_wino_sp_f32": (c_int, [P, c_int, c_int, c_int, c_int, P, c_int, P, P, P, c_int64, P]),
    "smc_modconv_epilogue_f32": (c_int, [P, c_int, c_int64, P, c_int, c_int, c_int, c_int, P, P]),
    "smc_modconv_blur_act_f32": (c_int, [P, c_int, c_int64, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P,
                                         c_int, c_int, c_int, c_int, c_float, c_int, P, P]),
    "smc_modconv_blur_act_bwd_f32": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, c_int,
                                             c_int, c_int, c_int, c_float, c_int, P, P, c_int64, P]),
    "smc_modconv_blur_act_bwd_workspace_size": (c_int64, [c_int] * 6),
    "smc_modconv_demod_f32": (c_int, [P, P, P, c_int, c_int, c_int, c_float, P]),
    "smc_row_dot_f32": (c_int, [P, c_int64, P, c_int64, P, c_int, c_int, P]),
    "smc_direction_head_f32": (c_int, [P, c_int64, P, c_int64, P, P, P, c_int, c_int, c_float, P]),
    "smc_modconv_act_bwd_f32": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, P, P, c_int64, P]),
    "smc_modconv_act_bwd_workspace_size": (c_int64, [c_int] * 4),
    "smc_channel_dot_f32": (c_int, [P, P, P, P, P, c_int64, c_int64, c_int, P]),
    "smc_modconv_demod_bwd_f32": (c_int, [P, P, P, P, P, c_int, c_int, c_int, P]),
    "smc_torgb_fwd_f32": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_float, P]),
    "smc_torgb_bwd_f32": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_float, c_int, c_int, P]),
    "smc_torgb_act_bwd_f32": (c_int, [P, P, P, P, c_float, P, P, P, c_int, c_int, c_int, c_int, c_int, P, P]),
    "smc_face_crop_f32": (c_int, [P, c_int64] + [c_int] * 10 + [P, P]),
    "smc_face_crop_bwd_f32": (c_int, [P, c_int64] + [c_int] * 10 + [P, P]),
    "smc_clip_unprocess_f32": (c_int, [P] + [c_int] * 6 + [P, P, P, P]),
    "smc_clip_unprocess_bwd_f32": (c_int, [P, P] + [c_int] * 6 + [P, P, P, P]),
    "smc_clip_preprocess_nada_f32": (c_int, [P] + [c_int] * 6 + [P, P, P, P]),
    "smc_clip_preprocess_nada_bwd_f32": (c_int, [P, P] + [c_int] * 6 + [P, P, P, P]),
    "smc_linear_workspace_size": (c_int64, [c_int, c_int, c_int]),
    "smc_linear_f32": (c_int, [P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, P, P, c_int64, P]),
    "smc_layernorm_fwd_f32": (c_int, [P, c_int64, P, P, P, c_int64, P, P, c_int, c_int, c_float, P]),
    "smc_layernorm_bwd_f32": (c_int, [P, c_int64, P, c_int64, P, P, P, P, c_int64, P, c_int64, c_int, c_int, P]),
    "smc_attention_fwd_f32": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_float, P]),
    "smc_attention_bwd_f32": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_float, P]),
    "smc_attention_causal_fwd_f32": (c_int, [P, P, c_int, c_int, c_int, c_int, c_float, P]),
    "smc_patch_im2col_f32": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, P]),
    "smc_vit_packed_floats": (c_int64, [P]),
    "smc_vit_saved_floats": (c_int64, [P, c_int]),
    "smc_vit_pack_x3": (c_int, [P, P, P]),
    "smc_vit_workspace_bytes": (c_int64, [P, c_int]),
    "smc_vit_forward_f32": (c_int, [P, P, P, c_int, P, P, P, c_int64, P]),
    "smc_vit_backward_f32": (c_int, [P, P, P, c_int, c_int, P, P, P, c_int64, P]),
    "smc_irse_saved_floats": (c_int64, [P, c_int]),
    "smc_irse_workspace_bytes": (c_int64, [P, c_int]),
    "smc_irse_forward_f32": (c_int, [P, P, c_int, P, P, P, c_int64, P]),
    "smc_irse_backward_f32": (c_int, [P, P, c_int, c_int, P, P, P, c_int64, P]),
}

_lib = None
_lock = threading.Lock()


def exported_symbols():
    return sorted(_SIGS)


def load(path=None):
    """Load (once) and return the ctypes library; raises if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise RuntimeError(f"stylemc_amd: HIP kernel library not found at {p}; build it with "
                               f"`python -m stylemc_amd.build` (there is no CPU fallback)")
        lib = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.smc_abi_version() != 4:
            raise RuntimeError("stylemc_amd: ABI version mismatch, rebuild the library")
        if path is None:
            _lib = lib
        return lib


def check(rc, name):
    if rc != 0:
        msg = load().smc_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (code {rc}): {msg}")


def call(name, *args):
    check(getattr(load(), name)(*args), name)


def ptr(t):
    """Device pointer of an fp32 CUDA tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("stylemc_amd kernels run on the GPU only (got a CPU tensor)")
    if t.dtype != torch.float32:
        raise NotImplementedError(f"stylemc_amd kernels are fp32-only (got {t.dtype})")
    return t.data_ptr()


_plan_state = (0, 0)


@contextlib.contextmanager
def plan_batch(plan, local):
    """Plan every batch-dependent launch decision (split-K, tile configuration, channel split) of the work enqueued
    inside as for ``plan`` images per ``local`` images of the call (smc_set_plan_batch): a data-parallel shard of
    ``local`` images of a ``plan``-image batch then computes each image bit for bit as the whole batch does.
    Restores the previous setting on exit (nestable)."""
    global _plan_state
    prev = _plan_state
    new = (0, 0) if not plan or not local or plan == local else (int(plan), int(local))
    if new != prev:
        call("smc_set_plan_batch", *new)
        _plan_state = new
    try:
        yield
    finally:
        if _plan_state != prev:
            call("smc_set_plan_batch", *prev)
            _plan_state = prev


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream():
    """hipStream_t of torch's current stream on the current device (as an int for ctypes)."""
    if _raw_stream is not None:
        return _raw_stream(torch.cuda.current_device())
    return torch.cuda.current_stream().cuda_stream


# --------------------------------------------------------------------------------- launch timing

class KernelTimer:
    """Records HIP events around selected launches (bench.py's live roofline measurement)."""

    def __init__(self, family):
        self.family = family
        self.records = []  # (start_event, end_event, flops, algorithmic bytes, kind, direct-equivalent flops)

    def wrap(self, flops, nbytes=0, kind="direct", equiv_flops=None):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        return s, e, flops, nbytes, kind, flops if equiv_flops is None else equiv_flops

    def finish(self, token, kind=None):
        s, e, flops, nbytes, kind0, eq = token
        kind = kind0 if kind is None else kind
        e.record()
        self.records.append((s, e, flops, nbytes, kind, eq))

    def summary(self):
        torch.cuda.synchronize()
        out = {"launches": 0, "seconds": 0.0, "flops": 0.0, "bytes": 0, "equiv_flops": 0.0, "kinds": {}}
        for s, e, flops, nbytes, kind, eq in self.records:
            t = s.elapsed_time(e) * 1e-3
            for d in (out, out["kinds"].setdefault(kind, {"launches": 0, "seconds": 0.0, "flops": 0.0, "bytes": 0,
                                                          "equiv_flops": 0.0})):
                d["launches"] += 1
                d["seconds"] += t
                d["flops"] += flops
                d["bytes"] += nbytes
                d["equiv_flops"] += eq
        return out


_timer = None


def set_timer(timer):
    global _timer
    _timer = timer


def timer():
    return _timer
