"""ctypes binding of libic2ops.so (the C ABI declared in include/ic2ops.h).

The product path has NO CPU fallback: every public op requires ROCm tensors and the in-tree
HIP library; anything else raises.  (The CPU restatement in ``oracle/`` is test infrastructure.)
"""
from __future__ import annotations

import ctypes
import os
import sys
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libic2ops.so")
# diagnostic builds (tools/build_abl.sh) are loaded instead only under IC2_DEV=1 with IC2_DEV_LIB set
if os.environ.get("IC2_DEV") == "1" and os.environ.get("IC2_DEV_LIB"):
    LIB_PATH = os.environ["IC2_DEV_LIB"]

F32, BF16, F16, BF16X3, F16X2 = 0, 1, 2, 3, 4
F16_IEEE = 5   # out_dtype only: f16 output converted IEEE (overflow -> inf), the training path's gradient convs
ACT_LINEAR, ACT_LRELU = 0, 1
NHWC, NCHW, NHWC16 = 0, 1, 2

_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_F = ctypes.c_float

# name -> argtypes (restype int unless listed in _RESTYPE)
_SIGS = {
    "ic2_abi_version": [],
    "ic2_dev_mode": [],
    "ic2_conv_plan": [_I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I],
    "ic2_quantize_uniform": [_P, _I64, _I, _P, _P, _P],
    "ic2_quantize_codebook_argmin": [_P, _I64, _P, _I, _P, _P, _P, _P],
    "ic2_codebook_lookup": [_P, _I64, _P, _I, _P, _P, _P],
    "ic2_code_record": [_P, _I, _I, _I, _P, _I64, _P, _P],
    "ic2_gumbel_softmax_quantize": [_P, _I64, _P, _I, _P, _F, _I, ctypes.c_uint64, ctypes.c_uint64, _P, _P, _P, _P,
                                    _P],
    "ic2_gumbel_softmax_quantize_dseed": [_P, _I64, _P, _I, _P, _F, _I, _P, ctypes.c_uint64, _P, _P, _P, _P, _P],
    "ic2_bias_act": [_P, _P, _P, _I, _I64, _I64, _I64, _I, _F, _F, _F, _P],
    "ic2_upfirdn2d": [_P, _P, _I, _I64, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _F, _P],
    "ic2_filtered_lrelu": [_P, _P, _I, _I64, _I64, _I, _I, _I, _I, _P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, _F, _F,
                           _F, _I, _P],
    "ic2_flrelu_nhwc": [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, _F, _F, _F,
                        _I, _P, _P],
    "ic2_flrelu_nhwc16": [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, _F, _F,
                          _F, _I, _P, _P],
    "ic2_fc": [_P, _I64, _P, _P, _P, _I, _I, _I, _F, _F, _I, _F, _F, _P],
    "ic2_pack_weight": [_P, _I, _I, _I, _I, _I, _I, _I, _F, _P, _I, _P, _P],
    "ic2_modconv_prep": [_P, _P, _I, _I, _I, _I, _I, _I, _F, _F, _P, _P, _P, _P],
    "ic2_modconv_prep_batched": [_P, _I64, _I, _I, _I, _P, _P],
    "ic2_conv_igemm": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _I, _F, _F, _F, _F, _I,
                       _P],
    "ic2_conv_igemm_ws_bytes": [_I, _I, _I, _I, _I, _I, _I, _I, _I],
    "ic2_conv_igemm_ws": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _I, _F, _F, _F, _F,
                          _I, _P, _I64, _P],
    "ic2_pack_weight_wino": [_P, _I, _I, _I, _I, _I, _F, _P, _I, _P],
    "ic2_pack_weight_adjoint": [_P, _I, _I, _I, _I, _I, _I, _P, _I, _P],
    "ic2_conv_wino": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _I, _F, _F, _F, _F, _I, _P],
    "ic2_conv_wino_plan": [_I, _I, _I, _I, _I, _I],
    "ic2_conv_wino_preferred": [_I, _I, _I, _I, _I, _I, _I, _I, _I],
    "ic2_conv_wino_stamps": [_P, _I64],
    "ic2_synth_input_features": [_P, _P, _P, _P, _I, _I, _I, _I, _F, _F, _P, _I, _P],
    "ic2_nchw_to_nhwc": [_P, _P, _I, _I, _I, _I, _I, _I, _P, _P],
    "ic2_from_rgb_conv": [_P, _I, _P, _I, _P, _P, _I, _I, _I, _I, _P],
    "ic2_from_rgb_conv_x3": [_P, _I, _P, _I, _P, _P, _I, _I, _I, _I, _P],
    "ic2_from_rgb_conv_f16": [_P, _I, _P, _I, _P, _P, _I, _I, _I, _I, _P],
    "ic2_nhwc_to_nchw": [_P, _I, _P, _I, _I, _I, _I, _I, _P],
    "ic2_group_norm_stats_floats": [_I, _I, _I],
    "ic2_group_norm_stats": [_P, _I, _I, _I, _I, _I, _I, _F, _P, _P],
    "ic2_gn_lrelu_pool": [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _F, _I, _P],
    "ic2_global_avg_pool_floats": [_I, _I, _I, _I],
    "ic2_global_avg_pool": [_P, _I, _I, _I, _I, _I, _P, _P],
    "ic2_reparameterize": [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P],
    "ic2_uint8_sse_scratch_doubles": [_I64],
    "ic2_uint8_sse": [_P, _P, _I64, _I64, _P, _P, _P],
    "ic2_resize_bilinear": [_P, _P, _I64, _I, _I, _I, _I, _P],
    "ic2_rc_bound": [_I64, _I64],
    "ic2_rc_encode": [_P, _I64, _I, _I, _I, _P, _I64, _P, _I],
    "ic2_rc_decode": [_P, _P, _I64, _I, _I, _I, _P, _I],
    "ic2_conv_wgrad_ws_floats": [_I, _I, _I, _I, _I, _I, _I, _I],
    "ic2_conv_wgrad": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _I64, _P],
    "ic2_conv_wgrad_oihw": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _I64, _P],
    "ic2_gn_lrelu_pool_bwd_floats": [_I, _I, _I, _I, _I],
    "ic2_gn_lrelu_pool_bwd": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _F, _I, _P, _P, _P, _I64,
                              _P],
    "ic2_gn_lrelu_pool_bwd_db": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _F, _I, _P, _P, _P, _P,
                                 _I64, _P],
    "ic2_gap_bwd": [_P, _P, _I, _I, _I, _I, _I, _P],
    "ic2_flrelu_bwd_ydot_floats": [_I, _I, _I, _I, _I],
    "ic2_flrelu_bwd_nhwc_ex": [_P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, _I,
                               _F, _F, _F, _I, _P, _P, _P, _I64, _P],
    "ic2_scale_bwd_part_floats": [_I, _I, _I],
    "ic2_colsum_div": [_P, _I, _I, _I, _P, _P, _P],
    "ic2_scale_bwd_nhwc": [_P, _P, _P, _P, _I, _I, _I, _I, _P, _I64, _P],
    "ic2_scale_nhwc": [_P, _P, _P, _I, _I, _I, _I, _P],
    "ic2_conv3x3_gn_stats_floats": [_I, _I, _I, _I, _I, _I, _I, _I, _I, _I],
    "ic2_conv3x3_gn_fwd": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _I, _F, _P, _I64, _P, _I64, _I,
                           _P],
    "ic2_conv3x3_gn_fwd_scaled": [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _F, _I, _F, _P, _I64, _P,
                                  _I64, _I, _P],
    "ic2_conv3x3_gnin_supported": [_I, _I, _I, _I, _I, _I, _I, _I, _I],
    "ic2_conv3x3_gn_fuses": [_I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I],
    "ic2_gn_affine_table": [_P, _P, _P, _I, _I, _I, _I, _P, _P],
    "ic2_conv3x3_gnin_gn_fwd": [_P, _P, _F, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _I, _F, _P, _I64, _P,
                                _I64, _I, _P],
    "ic2_flrelu_bwd_nhwc": [_P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _F, _F,
                            _F, _I, _P],
}
_RESTYPE = {"ic2_conv_plan": ctypes.c_char_p, "ic2_conv_wino_plan": ctypes.c_char_p, "ic2_conv_igemm_ws_bytes": _I64, "ic2_group_norm_stats_floats": _I64, "ic2_global_avg_pool_floats": _I64,
            "ic2_uint8_sse_scratch_doubles": _I64, "ic2_rc_bound": _I64, "ic2_conv_wgrad_ws_floats": _I64,
            "ic2_gn_lrelu_pool_bwd_floats": _I64, "ic2_conv3x3_gn_stats_floats": _I64,
            "ic2_flrelu_bwd_ydot_floats": _I64, "ic2_scale_bwd_part_floats": _I64}

_lib = None
_lock = threading.Lock()


class NativeUnavailable(RuntimeError):
    pass


def load():
    """Load libic2ops.so (built in-tree by ``build_native``).  Raises if missing -- no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeUnavailable(
                f"{LIB_PATH} is missing: build it with `python -m image_compression_2_amd.build_native` "
                "(there is no CPU fallback for the product path)")
        lib = ctypes.CDLL(LIB_PATH)
        lib.ic2_last_error.restype = ctypes.c_char_p
        lib.ic2_last_error.argtypes = []
        for name, args in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = _RESTYPE.get(name, _I)
        _lib = lib
    return _lib


def exported_symbols():
    return ["ic2_last_error"] + list(_SIGS)


def call(name, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.ic2_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (code {rc}): {msg}")
    return rc


def query(name, *args):
    return getattr(load(), name)(*args)


def conv_plan(dtype, out_dtype, out_layout, n, h, w, cin_p, cout_p, cout_valid, kh, kw, pad):
    """Name of the kernel instance(s) ic2_conv_igemm_ws launches for this geometry (the library's launch plan)."""
    return query("ic2_conv_plan", dtype, out_dtype, out_layout, n, h, w, cin_p, cout_p, cout_valid, kh, kw,
                 pad).decode()


def conv_igemm(x, w, y, dtype, out_dtype, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, ho, wo, oscale, bias,
               act, slope, act_gain, clamp, out_mul, out_layout, stream, device):
    """ic2_conv_igemm with the split-K workspace the launch plan asks for (a stream-ordered torch allocation: the
    call allocates nothing else and never synchronises the host).  Whole-step capture of the f16 training step is not
    part of the product (training.py: its round-4 trial replayed a negative rec_loss, see DESIGN.md Training)."""
    nbytes = int(query("ic2_conv_igemm_ws_bytes", dtype, n, h, w_, cin_p, cout_p, kh, kw, pad))
    ws = torch.empty([max(nbytes, 16) // 4], dtype=torch.float32, device=device) if nbytes > 0 else None
    return call("ic2_conv_igemm_ws", x, w, y, dtype, out_dtype, n, h, w_, cin_p, cout_p, cout_valid, kh, kw, pad, ho,
                wo, oscale, bias, act, slope, act_gain, clamp, out_mul, out_layout, ptr(ws), nbytes, stream)


def wino_preferred(dtype, n, h, w, cin_p, cout_p, kh, kw, pad):
    """True when the library's launch plan runs this conv as the Winograd kernel (ic2_conv_wino)."""
    return bool(query("ic2_conv_wino_preferred", dtype, n, h, w, cin_p, cout_p, kh, kw, pad))


def wino_plan(n, h, w, cin_p, cout_p, pad):
    """Name of the ic2_conv_wino instance (tile) for this geometry."""
    return query("ic2_conv_wino_plan", n, h, w, cin_p, cout_p, pad).decode()


def conv_wino(x, u, y, dtype, out_dtype, n, h, w_, cin_p, cout_p, cout_valid, pad, ho, wo, oscale, bias, act, slope,
              act_gain, clamp, out_mul, out_layout, stream):
    """ic2_conv_wino: the 3x3 conv as a fused Winograd F(2,3) along x (f16 operands; u from ic2_pack_weight_wino)."""
    return call("ic2_conv_wino", x, u, y, dtype, out_dtype, n, h, w_, cin_p, cout_p, cout_valid, pad, ho, wo, oscale,
                bias, act, slope, act_gain, clamp, out_mul, out_layout, stream)


_flops_hook = None   # installed by bench.py's instrumented pass: receives each conv's algorithmic FLOPs


def note_flops(alg_flops):
    """Announce the algorithmic (unpadded, reference) FLOPs of the conv launch that follows (accounting for the
    benchmark's per-call roofline; a no-op unless an instrumented pass installed a hook)."""
    if _flops_hook is not None:
        _flops_hook(alg_flops)


def knob(name, default):
    """Development knob (the native library's rule, errors.hip): the environment variable `name` is read only when
    IC2_DEV=1, so the default launch plan never depends on the process environment."""
    v = os.environ.get(name)
    if os.environ.get("IC2_DEV") != "1":
        if v is not None:
            print(f"[ic2] {name}={v} ignored: development knobs need IC2_DEV=1", file=sys.stderr)
        return default
    return default if v is None else type(default)(v)


# ------------------------------------------------------------------------------------------------
# tensor helpers
# ------------------------------------------------------------------------------------------------
def require_gpu(*tensors):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("image_compression_2_amd runs on ROCm devices only (got a CPU tensor); "
                               "the CPU restatement lives in oracle/ and is test infrastructure")
        if not t.is_contiguous():
            raise RuntimeError("expected a contiguous tensor")


class AutogradUnsupported(RuntimeError):
    pass


def grad_inputs(tensors=(), modules=()):
    """The tensors / parameters a graph would have to reach: [] unless grad mode is on."""
    if not torch.is_grad_enabled():
        return []
    req = [t for t in tensors if isinstance(t, torch.Tensor) and t.requires_grad]
    return req + [p for m in modules for p in m.parameters() if p.requires_grad]


class _RefuseBackward(torch.autograd.Function):
    """Graph node for HIP forwards without a backward: the forward result is returned as is (no copy); a
    backward through it raises instead of silently producing no gradient."""

    @staticmethod
    def forward(ctx, what, n_out, *args):
        ctx.what = what
        return tuple(a.detach() for a in args[:n_out])

    @staticmethod
    def backward(ctx, *grads):
        raise AutogradUnsupported(
            f"{ctx.what}: backward through the HIP path is not implemented for this module (training, SURVEY.md "
            "8(f) #3; the reference trains only the encoder, through a frozen generator).  Freeze the module with "
            ".requires_grad_(False) or detach its inputs")


def refuse_backward(what, outputs, tensors=(), modules=()):
    """Return `outputs` (a tensor or a tuple) unchanged when no graph is wanted; otherwise attached to a node whose
    backward raises AutogradUnsupported (inference in grad mode keeps working; only .backward() fails)."""
    req = grad_inputs(tensors, modules)
    if not req:
        return outputs
    single = isinstance(outputs, torch.Tensor)
    outs = [outputs] if single else list(outputs)
    fl = [i for i, o in enumerate(outs) if isinstance(o, torch.Tensor) and o.is_floating_point()]
    wrapped = _RefuseBackward.apply(what, len(fl), *[outs[i] for i in fl], *req)
    for k, i in enumerate(fl):
        outs[i] = wrapped[k]
    return outs[0] if single else tuple(outs)


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_of(t=None):
    dev = t.device if t is not None else None
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def dtype_code(dt):
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    if dt == torch.float16:
        return F16
    raise TypeError(f"unsupported dtype {dt}")


def torch_dtype(precision):
    if precision in ("fp32", "f32", torch.float32):
        return torch.float32
    if precision in ("bf16", torch.bfloat16):
        return torch.bfloat16
    if precision in ("f16", "fp16", torch.float16):
        return torch.float16
    raise ValueError(f"precision must be 'fp32', 'bf16' or 'f16', got {precision!r}")


ENCODER_PRECISIONS = ("fp32", "bf16", "bf16x3", "f16")


def encoder_dtype(precision):
    """HVAE_VGG_Encoder precision -> (activation storage dtype, split).  'bf16x3' = split bf16 (ic2ops.h
    IC2_BF16X3): bf16 MFMA operands [hi | hi | lo] x [hi | lo | hi], f32 conv outputs, GroupNorm in f32.  'f16': f16
    activations and MFMA operands (the f16 training precision, BASELINE config 5's fp16; loss-scaled)."""
    if precision == "bf16x3":
        return torch.bfloat16, True
    if precision in ("fp32", "bf16", "f16"):
        return torch_dtype(precision), False
    raise ValueError(f"encoder precision must be one of {ENCODER_PRECISIONS}, got {precision!r}")


def pad32(c):
    return (int(c) + 31) // 32 * 32


def pad_synth(c):
    """Synthesis activation channel stride: multiple of 32 up to 128 channels, of 64 above.  The SG3-T-1024
    widths 323 / 203 then land on 384 / 256, whose K-chunks are 64 deep and whose o-tiles are 128 / 256 wide,
    so those layers run on the 8-phase MFMA kernels instead of the 32-row tile (measured: L8_276_203 2.33 ms
    at batch 8 on the 352 / 224 strides); 81 / 51 keep 96 / 64 (the filtered-lrelu pays for every padded
    channel).  The SG3-T-256 strides (181 -> 192, 362 -> 384) are unchanged."""
    c = int(c)
    return pad32(c) if c <= 128 else (c + 63) // 64 * 64


def colsum_div(part, n, c, den=None):
    """out [n, c] f32 = part.view(n, -1, c).sum(1) / den (0 where den == 0; den None: the plain sum), one launch
    (ic2_colsum_div)."""
    part = part.contiguous()
    rows = part.numel() // (n * c)
    assert rows * n * c == part.numel(), (part.shape, n, c)
    out = torch.empty([n, c], dtype=torch.float32, device=part.device)
    call("ic2_colsum_div", ptr(part), n, rows, c, None if den is None else ptr(den.contiguous()), ptr(out),
         stream_of(part))
    return out
