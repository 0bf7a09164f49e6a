"""ctypes binding of libtt2.so (include/tt2.h).

There is no CPU fallback: if the HIP library is missing or fails to load, every model call raises
``TT2NotBuilt``.  Build it with ``make -C tacotron-2_amd`` (or ``__graft_entry__.build()``).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# TT2_LIB: an alternative build of the same ABI (A/B kernel experiments); default = in-tree
LIB_PATH = os.environ.get("TT2_LIB") or os.path.join(os.path.dirname(_HERE), "libtt2.so")

TT2_OK = 0
_STATUS = {-1: "INVALID_ARG", -2: "SHAPE_MISMATCH", -3: "OOM", -4: "HIP_ERROR", -5: "NOT_LOADED",
           -6: "STATE"}


class TT2Error(RuntimeError):
    """A libtt2 call failed; ``status`` is the tt2_status code."""

    def __init__(self, status, msg):
        super().__init__("{} ({}): {}".format(_STATUS.get(status, "ERROR"), status, msg))
        self.status = status


class TT2NotBuilt(RuntimeError):
    pass


class Config(ctypes.Structure):
    """tt2_config (include/tt2.h)."""
    _fields_ = [(n, ctypes.c_int) for n in (
        "num_mels", "n_symbols", "embedding_dim", "enc_conv_num_layers", "enc_conv_kernel_size",
        "enc_conv_channels", "encoder_lstm_units", "attention_dim", "attention_filters",
        "attention_kernel", "prenet_units", "decoder_lstm_units", "postnet_num_layers",
        "postnet_kernel_size", "postnet_channels", "use_gst", "emt_only", "num_gst", "num_heads",
        "style_embed_depth", "style_att_dim", "reference_depth")] + [
        ("reference_filters", ctypes.c_int * 6),
        ("zoneout", ctypes.c_float), ("max_abs_value", ctypes.c_float),
        ("lower_bound_decay", ctypes.c_float)] + [(n, ctypes.c_int) for n in (
            "symmetric_mels", "clip_outputs", "stop_at_any", "mask_encoder", "cumulative_weights",
            "synthesis_constraint", "constraint_monotonic", "attention_win_size", "max_batch",
            "max_T_in", "max_T_ref", "max_iters", "emt_attn", "emt_ref_gru", "n_emt", "style_mode",
            "predict_linear", "num_freq", "cbhg_kernels", "cbhg_conv_channels", "cbhg_pool_size",
            "cbhg_projection", "cbhg_projection_kernel_size", "cbhg_highwaynet_layers",
            "cbhg_highway_units", "cbhg_rnn_units", "smoothing", "outputs_per_step")]


class WnConfig(ctypes.Structure):
    """tt2_wn_config (include/tt2.h)."""
    _fields_ = [(n, ctypes.c_int) for n in (
        "layers", "stacks", "residual_channels", "gate_channels", "skip_out_channels",
        "kernel_size", "cin_channels", "out_channels", "legacy", "residual_legacy")] + [
        ("log_scale_min", ctypes.c_float), ("n_upsample", ctypes.c_int),
        ("upsample_scales", ctypes.c_int * 8), ("freq_axis_kernel_size", ctypes.c_int),
        ("max_batch", ctypes.c_int), ("max_samples", ctypes.c_int64),
        ("upsample_type", ctypes.c_int), ("upsample_activation", ctypes.c_int),
        ("leaky_alpha", ctypes.c_float), ("NN_init", ctypes.c_int),
        ("log_scale_min_gauss", ctypes.c_float), ("gin_channels", ctypes.c_int),
        ("n_speakers", ctypes.c_int), ("input_type", ctypes.c_int), ("quantize_channels", ctypes.c_int)]


class GlConfig(ctypes.Structure):
    """tt2_gl_config (include/tt2.h)."""
    _fields_ = [(n, ctypes.c_int) for n in ("n_fft", "hop_size", "win_size", "num_mels")] + [
        (n, ctypes.c_float) for n in ("magnitude_power", "power", "ref_level_db", "min_level_db",
                                      "max_abs_value")] + [
        (n, ctypes.c_int) for n in ("symmetric_mels", "allow_clipping_in_normalization",
                                    "griffin_lim_iters")]


class TrainConfig(ctypes.Structure):
    """tt2_train_config (include/tt2.h)."""
    _fields_ = [(n, ctypes.c_int) for n in (
        "batch", "max_T_in", "max_T_out", "memory_dim", "num_mels", "prenet_units",
        "decoder_lstm_units", "attention_dim", "attention_filters", "attention_kernel")] + [
        (n, ctypes.c_float) for n in ("zoneout", "reg_weight", "adam_beta1", "adam_beta2",
                                      "adam_epsilon", "clip_norm")] + [
        ("precision", ctypes.c_int), ("clip_outputs", ctypes.c_int), ("clip_lo", ctypes.c_float),
        ("clip_hi", ctypes.c_float)] + [(n, ctypes.c_int) for n in (
            "postnet", "postnet_layers", "postnet_channels", "postnet_kernel")] + [
        ("bn_momentum", ctypes.c_float), ("bn_eps", ctypes.c_float)] + [
        (n, ctypes.c_int) for n in (
            "frontend", "n_symbols", "embedding_dim", "enc_conv_layers", "enc_conv_kernel",
            "enc_conv_channels", "encoder_lstm_units", "emt_only", "num_gst", "num_heads",
            "style_embed_depth", "style_att_dim", "reference_depth")] + [
        ("reference_filters", ctypes.c_int * 6), ("max_T_ref", ctypes.c_int),
        ("mask_decoder", ctypes.c_int), ("pos_weight", ctypes.c_float),
        ("n_emt", ctypes.c_int), ("n_spk", ctypes.c_int), ("orthog_weight", ctypes.c_float),
        ("use_gst", ctypes.c_int), ("adain", ctypes.c_int), ("smoothing", ctypes.c_int),
        ("outputs_per_step", ctypes.c_int)]


class DecoderState(ctypes.Structure):
    """tt2_decoder_state (include/tt2.h): pointers to caller-owned host arrays."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("h1", "c1", "h2", "c2", "attention", "alignments",
                                              "max_attentions")] + [("time", ctypes.c_int32)]


_P = ctypes.c_void_p
_I = ctypes.c_int
_U64 = ctypes.c_uint64
_F = ctypes.c_float

#: every symbol include/tt2.h declares, with (restype, argtypes)
SIGNATURES = {
    "tt2_last_error": (ctypes.c_char_p, []),
    "tt2_version": (ctypes.c_char_p, []),
    "tt2_default_config": (None, [ctypes.POINTER(Config), _I, _I, _I, _I]),
    "tt2_create": (_I, [ctypes.POINTER(Config), _I, ctypes.POINTER(_P)]),
    "tt2_destroy": (None, [_P]),
    "tt2_load_tensor": (_I, [_P, ctypes.c_char_p, _P, _P, _I]),
    "tt2_finalize_weights": (_I, [_P]),
    "tt2_encode": (_I, [_P, _P, _P, _I, _I, _P, _I, _P, _I, _P, _P]),
    "tt2_decode": (_I, [_P, _I, _P, _U64, _P, _I, _P, _P, _P, _P]),
    "tt2_postnet": (_I, [_P, _P, _I, _I, _P, _P]),
    "tt2_synthesize_dev": (_I, [_P, _P, _P, _P, _I, _I, _P, _I, _P, _I, _I, _P, _U64, _P, _P, _P,
                                _P]),
    "tt2_output_lengths_dev": (_I, [_P, _I, _I, _I, _P, _P]),
    "tt2_last_timings": (_I, [_P, _P]),
    "tt2_profile_decoder_kernels": (_I, [_P, _I, _P]),
    "tt2_debug_stamps": (_I, [_P, _P]),
    "tt2_decoder_path": (_I, [_P, _P, _P]),
    "tt2_debug_pd_stamps": (_I, [_P, _P]),
    "tt2_hbm_copy_gbps": (_I, [_I, ctypes.c_longlong, _I, _P]),
    "tt2_set_emt_labels": (_I, [_P, _P, _I]),
    "tt2_linear_outputs": (_I, [_P, _P, _I, _I, _P]),
    "tt2_linear_outputs_dev": (_I, [_P, _P, _I, _I, _P, _P]),
    "tt2_emt_alignments": (_I, [_P, _P, _P, _P]),
    "tt2_wn_last_timings": (_I, [_P, _P]),
    "tt2_wn_debug_stamps": (_I, [_P, _P]),
    "tt2_wn_default_config": (None, [ctypes.POINTER(WnConfig), _I, ctypes.c_int64]),
    "tt2_wn_create": (_I, [ctypes.POINTER(WnConfig), _I, ctypes.POINTER(_P)]),
    "tt2_wn_destroy": (None, [_P]),
    "tt2_wn_load_tensor": (_I, [_P, ctypes.c_char_p, _P, _P, _I]),
    "tt2_wn_finalize": (_I, [_P]),
    "tt2_wn_generate": (_I, [_P, _P, _I, _I, _P, _P, _U64, _P, _P, _P, _P, _P]),
    "tt2_wn_generate_dev": (_I, [_P, _P, _I, _I, _P, _P, _U64, _P, _P, _P, _P, _P]),
    "tt2_wn_generate_unconditional": (_I, [_P, _I, ctypes.c_int64, _P, _P, _U64, _P, _P, _P, _P]),
    "tt2_wn_cond_from_mels_dev": (_I, [_P, _I, _P, _I, _I, _I, _F, _F, _I, _I, _P, _P]),
    "tt2_gl_default_config": (None, [ctypes.POINTER(GlConfig)]),
    "tt2_gl_create": (_I, [ctypes.POINTER(GlConfig), _I, ctypes.POINTER(_P)]),
    "tt2_gl_destroy": (None, [_P]),
    "tt2_gl_set_inv_mel_basis": (_I, [_P, _P]),
    "tt2_gl_synthesize": (_I, [_P, _P, _I, _I, _I, _P]),
    "tt2_gl_synthesize_dev": (_I, [_P, _P, _I, _I, _I, _P, _P]),
    "tt2_mol_sample": (_I, [_P, _P, _P, _I, _I, _F, _P, _P]),
    "tt2_prenet_keep_bits": (_I, [_U64, _I, _I, _I, _P]),
    "tt2_decoder_step": (_I, [_P, _P, _P, ctypes.POINTER(DecoderState),
                              ctypes.POINTER(DecoderState), _P, _P, _P]),
    "tt2_wn_noise": (_I, [_U64, _I, _I, _I, _I, _P, _P]),
    "tt2_train_default_config": (None, [ctypes.POINTER(TrainConfig), _I, _I, _I]),
    "tt2_train_create": (_I, [ctypes.POINTER(TrainConfig), _I, ctypes.POINTER(_P)]),
    "tt2_train_destroy": (None, [_P]),
    "tt2_train_load_tensor": (_I, [_P, ctypes.c_char_p, _P, _P, _I]),
    "tt2_train_finalize": (_I, [_P]),
    "tt2_train_bind_grads_dev": (_I, [_P, _P, ctypes.POINTER(ctypes.c_int64)]),
    "tt2_train_moving_stats_dev": (_I, [_P, _P, ctypes.POINTER(ctypes.c_int64), _I, _P]),
    "tt2_train_forward_backward_dev": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P]),
    "tt2_train_forward_backward_text_dev": (_I, [_P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P,
                                                 _P, _I, _I, _P]),
    "tt2_train_apply_dev": (_I, [_P, _F, _I, _P]),
    "tt2_train_set_target_lengths": (_I, [_P, _P]),
    "tt2_exit_guard": (None, [_I, _I]),
    "tt2_wn_set_global_condition": (_I, [_P, _P, _P, _I]),
    "tt2_train_set_teacher_forcing": (_I, [_P, _P, _I]),
    "tt2_train_set_style_labels": (_I, [_P, _P, _P]),
    "tt2_train_style_losses": (_I, [_P, _P]),
    "tt2_train_losses": (_I, [_P, _P, _P]),
    "tt2_train_get_tensor": (_I, [_P, ctypes.c_char_p, _I, _P]),
    "tt2_train_outputs": (_I, [_P, _P, _P, _P]),
}

_lib = None


def load_library(path=LIB_PATH):
    """Load libtt2.so (once).  Raises TT2NotBuilt if it is absent or unloadable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise TT2NotBuilt("HIP library not built: {} is missing (run `make -C tacotron-2_amd`)"
                          .format(path))
    try:
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:
        raise TT2NotBuilt("failed to load {}: {}".format(path, e))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


#: the synthesis subset libtt2_cpu.so (cpu/tt2_cpu.cpp) exports, same signatures
CPU_SYMBOLS = (
    "tt2_last_error", "tt2_version", "tt2_default_config", "tt2_create", "tt2_destroy",
    "tt2_load_tensor", "tt2_finalize_weights", "tt2_encode", "tt2_decode", "tt2_decoder_step",
    "tt2_postnet", "tt2_prenet_keep_bits", "tt2_wn_default_config", "tt2_wn_create",
    "tt2_wn_destroy", "tt2_wn_load_tensor", "tt2_wn_finalize", "tt2_wn_generate", "tt2_wn_noise",
    "tt2_mol_sample")
CPU_LIB_PATH = os.path.join(os.path.dirname(LIB_PATH), "libtt2_cpu.so")
_cpu_lib = None


def load_cpu_library(path=CPU_LIB_PATH):
    """libtt2_cpu.so: the same ABI on host cores (the CPU baseline / second implementation).
    Loaded RTLD_LOCAL beside libtt2.so; never a fallback of the HIP path."""
    global _cpu_lib
    if _cpu_lib is not None:
        return _cpu_lib
    if not os.path.exists(path):
        raise TT2NotBuilt("CPU library not built: {} is missing (run `make -C tacotron-2_amd`)"
                          .format(path))
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    for name in CPU_SYMBOLS:
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = SIGNATURES[name]
    _cpu_lib = lib
    return lib


def check(status, lib=None):
    if status != TT2_OK:
        msg = (lib or load_library()).tt2_last_error()
        raise TT2Error(status, msg.decode() if msg else "")


def ptr(a):
    """Pointer of a C-contiguous numpy array (or None)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return a.ctypes.data_as(ctypes.c_void_p)


def f32(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float32)


def i32(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.int32)


def load_tensor(fn, handle, name, arr, lib=None):
    arr = np.ascontiguousarray(arr, dtype=np.float32)
    shape = (ctypes.c_int64 * max(arr.ndim, 1))(*arr.shape)
    check(fn(handle, name.encode(), ptr(arr), ctypes.cast(shape, ctypes.c_void_p), arr.ndim), lib)
