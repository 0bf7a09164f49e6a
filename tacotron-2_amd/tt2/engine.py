"""Host engines over libtt2.so: one context per (process, device), weights uploaded once.

``TacotronEngine`` / ``WaveNetEngine`` hold the C-ABI handles; the reference-named classes in
``tacotron.models`` / ``wavenet_vocoder.models`` are thin eager front-ends over them.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, f32, i32, ptr
from .hparams import get_hop_size
from .weights import EMT_ATTN, EMT_REF_GRU, STYLE_MODES, memory_width, style_mode


def tacotron_config(hp, max_batch, max_T_in, max_T_ref, max_iters, emt_only=False,
                    synthesis_constraint=False, emt_attn=None, emt_ref_gru="none", n_emt=4,
                    lib=None, style="gst"):
    """tt2_config from hparams (names mirror code/hparams.py).  ``emt_attn`` selects the
    Tacotron_emt_attn model (args.attn: 'simple' / 'multihead' / 'style_tokens'; None = the
    Tacotron model), ``emt_ref_gru`` its args.emt_ref_gru; ``style`` the Tacotron model's style path
    ('gst' | 'embed' = args.pretrained_emb_disc_all | 'adain' = args.adain, tacotron.py:236-308)."""
    lib = lib or _lib.load_library()
    cfg = _lib.Config()
    lib.tt2_default_config(ctypes.byref(cfg), max_batch, max_T_in, max_T_ref, max_iters)
    cfg.num_mels = hp.num_mels
    cfg.embedding_dim = hp.embedding_dim
    cfg.enc_conv_num_layers = hp.enc_conv_num_layers
    cfg.enc_conv_kernel_size = hp.enc_conv_kernel_size[0]
    cfg.enc_conv_channels = hp.enc_conv_channels
    cfg.encoder_lstm_units = hp.encoder_lstm_units
    cfg.attention_dim = hp.attention_dim
    cfg.attention_filters = hp.attention_filters
    cfg.attention_kernel = hp.attention_kernel[0]
    if len(hp.prenet_layers) != 2 or hp.prenet_layers[0] != hp.prenet_layers[1]:
        raise NotImplementedError("prenet_layers must be two equal widths on this build")
    cfg.prenet_units = hp.prenet_layers[0]
    if hp.decoder_layers != 2:
        raise NotImplementedError("decoder_layers must be 2 on this build")
    cfg.decoder_lstm_units = hp.decoder_lstm_units
    cfg.postnet_num_layers = hp.postnet_num_layers
    cfg.postnet_kernel_size = hp.postnet_kernel_size[0]
    cfg.postnet_channels = hp.postnet_channels
    cfg.use_gst = 1 if hp.use_gst else 0
    cfg.emt_only = 1 if emt_only else 0
    cfg.num_gst = hp.num_gst
    cfg.num_heads = hp.num_heads
    cfg.style_embed_depth = hp.style_embed_depth
    cfg.style_att_dim = hp.style_att_dim
    cfg.reference_depth = hp.reference_depth
    for i, f in enumerate(hp.reference_filters):
        cfg.reference_filters[i] = f
    cfg.zoneout = hp.tacotron_zoneout_rate
    cfg.max_abs_value = hp.max_abs_value
    cfg.lower_bound_decay = hp.lower_bound_decay
    cfg.symmetric_mels = 1 if hp.symmetric_mels else 0
    cfg.clip_outputs = 1 if hp.clip_outputs else 0
    cfg.stop_at_any = 1 if hp.stop_at_any else 0
    cfg.mask_encoder = 1 if hp.mask_encoder else 0
    cfg.cumulative_weights = 1 if hp.cumulative_weights else 0
    cfg.synthesis_constraint = 1 if synthesis_constraint else 0
    cfg.constraint_monotonic = 1 if hp.synthesis_constraint_type == "monotonic" else 0
    cfg.attention_win_size = hp.attention_win_size
    cfg.outputs_per_step = hp.outputs_per_step     # r frames per decoder step (tacotron.py:322-324)
    cfg.smoothing = 1 if hp.smoothing else 0        # attention.py:71-80,150
    cfg.style_mode = STYLE_MODES.index(style_mode(hp, style))
    cfg.predict_linear = 1 if hp.predict_linear else 0    # CBHG post-net (tacotron.py:466-481)
    cfg.num_freq = hp.num_freq
    for k in ("cbhg_kernels", "cbhg_conv_channels", "cbhg_pool_size", "cbhg_projection",
              "cbhg_projection_kernel_size", "cbhg_highwaynet_layers", "cbhg_highway_units",
              "cbhg_rnn_units"):
        setattr(cfg, k, getattr(hp, k))
    if emt_attn is not None:
        if emt_attn not in EMT_ATTN or emt_ref_gru not in EMT_REF_GRU:
            raise ValueError("emt_attn must be one of {}, emt_ref_gru one of {}".format(
                EMT_ATTN, EMT_REF_GRU))
        cfg.emt_attn = 1 + EMT_ATTN.index(emt_attn)
        cfg.emt_ref_gru = EMT_REF_GRU.index(emt_ref_gru)
        cfg.n_emt = n_emt
    return cfg


#: rows of one tt2_ctx (tt2_create's capacity: the persistent decoder's 32-row blocks)
MAX_CONTEXT_BATCH = 32


def chunk_ranges(B, cap=MAX_CONTEXT_BATCH):
    """Row ranges [(s, e)] of a batch split into ceil(B / cap) near-equal contexts."""
    n = max(1, -(-B // cap))
    q, r = divmod(B, n)
    out, s = [], 0
    for i in range(n):
        e = s + q + (1 if i < r else 0)
        out.append((s, e))
        s = e
    return out


def global_stop_steps(stop, stop_at_any, r=1):
    """dynamic_decode's batch-level stop over the whole tower (TacoTestHelper, helpers.py:40-54):
    finished = round(stop) [B, r] per step (round half to even as tf.round); reduce_all over the
    batch axis first, then any (stop_at_any) / all over the step's r frames -- at r = 1 both are
    "every row rounds to 1".  The stopping step is emitted, so the decode keeps step + 1 steps.
    stop [B, n * r] -> n_steps (n when the rule never fires)."""
    fin = np.rint(np.asarray(stop, np.float32)) == 1.0
    B, nr = fin.shape
    per_frame = fin.reshape(B, nr // r, r).all(axis=0)
    cond = per_frame.any(axis=1) if stop_at_any else per_frame.all(axis=1)
    return int(np.argmax(cond)) + 1 if cond.any() else nr // r


class TacotronEngine(object):
    """Owns one tt2_ctx, or for a batch above MAX_CONTEXT_BATCH rows one context per row chunk
    decoding without its own stop rule, with the tower's one batch-level stop step taken over all
    chunks' stop tokens afterwards (the reference decodes a tower in one dynamic_decode,
    tacotron.py:349-354; hparams.py:44 tacotron_batch_size 96)."""

    def __init__(self, hp, weights, max_batch, max_T_in, max_T_ref, max_iters, device=0,
                 emt_only=False, synthesis_constraint=False, emt_attn=None, emt_ref_gru="none",
                 n_emt=4, lib=None, style="gst", never_stop=False):
        # lib: libtt2.so by default; _lib.load_cpu_library() binds the same ABI on host cores
        self.lib = lib or _lib.load_library()
        self.hp = hp
        self.emt_only = emt_only
        self.emt_attn = emt_attn
        self.h = None
        self._chunks = None
        if max_batch > MAX_CONTEXT_BATCH:
            rng = chunk_ranges(max_batch)
            self._chunks = [TacotronEngine(hp, weights, e - s, max_T_in, max_T_ref, max_iters, device, emt_only,
                                           synthesis_constraint, emt_attn, emt_ref_gru, n_emt, lib, style,
                                           never_stop=True) for s, e in rng]
            self.cfg = self._chunks[0].cfg
            self.caps = (max_batch, max_T_in, max_T_ref, max_iters)
            self.style = style
            self.D = self._chunks[0].D
            return
        self.cfg = tacotron_config(hp, max_batch, max_T_in, max_T_ref, max_iters, emt_only,
                                   synthesis_constraint, emt_attn, emt_ref_gru, n_emt, self.lib, style)
        if never_stop:
            self.cfg.stop_at_any = 2
        self.caps = (max_batch, max_T_in, max_T_ref, max_iters)
        # Tacotron_emt_attn attends over the encoder outputs alone (tacotron_emt_attn.py:244-246)
        self.style = style
        self.D = 2 * hp.encoder_lstm_units if emt_attn else memory_width(hp, emt_only, style)
        h = ctypes.c_void_p()
        self._ok(self.lib.tt2_create(ctypes.byref(self.cfg), device, ctypes.byref(h)))
        self.h = h
        for name, arr in weights.items():
            if name.startswith("Tacotron_model/"):
                _lib.load_tensor(self.lib.tt2_load_tensor, self.h, name, arr, self.lib)
        self._ok(self.lib.tt2_finalize_weights(self.h))

    def _ok(self, status):
        _lib.check(status, self.lib)

    def close(self):
        for ch in getattr(self, "_chunks", None) or ():
            ch.close()
        if getattr(self, "h", None):
            self.lib.tt2_destroy(self.h)
            self.h = None

    __del__ = close

    def fits(self, B, T_in, T_ref, max_iters):
        c = self.caps
        return B <= c[0] and T_in <= c[1] and T_ref <= c[2] and max_iters <= c[3]

    def _ranges(self, B):
        """Row ranges of the chunk contexts for a batch of B rows (the first chunks fill first)."""
        out, s = [], 0
        for ch in self._chunks:
            e = min(B, s + ch.caps[0])
            out.append((s, e))
            s = e
        return out

    def encode(self, ids, lengths, ref_emt, ref_spk):
        ids = i32(ids)
        lengths = i32(lengths)
        B, T = ids.shape
        self._B, self._T_in = B, T
        if self._chunks:
            parts = [ch.encode(ids[s:e], lengths[s:e], None if ref_emt is None else f32(ref_emt)[s:e],
                               None if ref_spk is None else f32(ref_spk)[s:e])
                     for ch, (s, e) in zip(self._chunks, self._ranges(B)) if e > s]
            return np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])
        ref_emt = f32(ref_emt) if ref_emt is not None else None
        ref_spk = f32(ref_spk) if ref_spk is not None else None
        mem = np.zeros((B, T, self.D), np.float32)
        sw = self.D - 2 * self.hp.encoder_lstm_units
        style = np.zeros((B, max(sw, 1)), np.float32)
        self._ok(self.lib.tt2_encode(self.h, ptr(ids), ptr(lengths), B, T, ptr(ref_emt),
                                  ref_emt.shape[1] if ref_emt is not None else 0, ptr(ref_spk),
                                  ref_spk.shape[1] if ref_spk is not None else 0, ptr(mem),
                                  ptr(style)))
        return mem, style[:, :sw]

    def decode(self, max_iters, prenet_masks=None, seed=0, targets=None):
        B = self._B
        if self._chunks:
            return self._decode_chunked(max_iters, prenet_masks, seed, targets)
        masks = None if prenet_masks is None else np.ascontiguousarray(prenet_masks, np.uint8)
        if masks is not None and masks.shape[0] < max_iters:
            raise ValueError("prenet_masks must cover max_iters steps")
        if masks is not None and masks.shape[1:] != (2, B, self.hp.prenet_layers[0]):
            raise ValueError("prenet_masks must be [max_iters, 2, B, prenet_units] = [{}, 2, {}, {}]"
                             ", got {}".format(max_iters, B, self.hp.prenet_layers[0],
                                               masks.shape))
        if masks is not None:
            masks = np.ascontiguousarray(masks[:max_iters])
        tg = f32(targets)
        r = self.hp.outputs_per_step
        frames = np.zeros((B, max_iters * r, self.hp.num_mels), np.float32)
        stop = np.zeros((B, max_iters * r), np.float32)
        align = np.zeros((B, self._T_in, max_iters), np.float32)
        n = ctypes.c_int32()
        self._ok(self.lib.tt2_decode(self.h, max_iters, ptr(masks), seed, ptr(tg),
                                  tg.shape[1] if tg is not None else 0, ptr(frames), ptr(stop),
                                  ptr(align), ctypes.byref(n)))
        n = n.value
        self._n_steps = n
        return frames[:, :n * r], stop[:, :n * r], align[:, :, :n]

    def _decode_chunked(self, max_iters, prenet_masks, seed, targets):
        """Every chunk decodes max_iters steps (T_targets under GTA) without its own stop rule; the
        tower's stop step over all rows truncates the outputs.  Injected prenet masks cover the
        whole batch and are sliced per chunk; the device RNG of chunk c is keyed by seed + c."""
        B = self._B
        fr, st, al = [], [], []
        for c, (ch, (s, e)) in enumerate(zip(self._chunks, self._ranges(B))):
            if e <= s:
                continue
            pm = None if prenet_masks is None else np.asarray(prenet_masks)[:, :, s:e]
            tg = None if targets is None else f32(targets)[s:e]
            f, so, a = ch.decode(max_iters, pm, seed + c, tg)
            fr.append(f)
            st.append(so)
            al.append(a)
        frames, stop, align = np.concatenate(fr), np.concatenate(st), np.concatenate(al)
        r = self.hp.outputs_per_step
        n = (frames.shape[1] // r if targets is not None else
             global_stop_steps(stop, self.hp.stop_at_any, r))
        self._n_steps = n
        # each chunk decoded past the tower's stop step: postnet(None) takes these n·r frames
        self._frames = np.ascontiguousarray(frames[:, :n * r])
        return self._frames, stop[:, :n * r], align[:, :, :n]

    def zero_state(self):
        """TacotronDecoderCell.zero_state (Architecture_wrappers.py:158-195) for the batch of the last
        encode: dict of numpy arrays h1, c1, h2, c2 [B,H], attention [B,D_mem], alignments
        [B,T_in], max_attentions [B] int32, time."""
        B, T, H = self._B, self._T_in, self.hp.decoder_lstm_units
        z = lambda *s: np.zeros(s, np.float32)  # noqa: E731
        return dict(h1=z(B, H), c1=z(B, H), h2=z(B, H), c2=z(B, H), attention=z(B, self.D),
                    alignments=z(B, T), max_attentions=np.zeros(B, np.int32), time=0)

    def decoder_step(self, frame_in, prenet_masks, state):
        """tt2_decoder_step: one TacotronDecoderCell.__call__ (Architecture_wrappers.py:197-267)
        on the memory of the last encode.  frame_in [B,80], prenet_masks [2,B,P] uint8, state as
        zero_state() returns.  Returns (frame [B,80], stop [B], alignments [B,T_in], next_state).
        outputs_per_step = 1 only (r > 1 decodes through decode())."""
        B, T = self._B, self._T_in
        P = self.hp.prenet_layers[0]
        fi = f32(frame_in)
        m = np.ascontiguousarray(prenet_masks, np.uint8)
        if self._chunks:
            outs = []
            for ch, (s, e) in zip(self._chunks, self._ranges(B)):
                if e > s:
                    sub = {k: (v if k == "time" else np.asarray(v)[s:e]) for k, v in state.items()}
                    outs.append(ch.decoder_step(fi[s:e], m[:, s:e], sub))
            nxt = {k: np.concatenate([o[3][k] for o in outs]) for k in outs[0][3] if k != "time"}
            nxt["time"] = outs[0][3]["time"]
            return (np.concatenate([o[0] for o in outs]), np.concatenate([o[1] for o in outs]),
                    np.concatenate([o[2] for o in outs]), nxt)
        if fi.shape != (B, self.hp.num_mels) or m.shape != (2, B, P):
            raise ValueError("frame_in must be [B, num_mels] and prenet_masks [2, B, prenet_units]")
        names = ("h1", "c1", "h2", "c2", "attention", "alignments")
        cin = {k: f32(state[k]) for k in names}
        cin["max_attentions"] = i32(state["max_attentions"])
        nxt = {k: np.zeros_like(v) for k, v in cin.items()}

        def struct(d, time):
            return _lib.DecoderState(*[d[k].ctypes.data for k in names + ("max_attentions",)],
                                     int(time))
        sin, sout = struct(cin, state.get("time", 0)), struct(nxt, 0)
        frame = np.zeros((B, self.hp.num_mels), np.float32)
        stop = np.zeros((B,), np.float32)
        align = np.zeros((B, T), np.float32)
        self._ok(self.lib.tt2_decoder_step(self.h, ptr(fi), ptr(m), ctypes.byref(sin),
                                        ctypes.byref(sout), ptr(frame), ptr(stop), ptr(align)))
        nxt["time"] = sout.time
        return frame, stop, align, nxt

    def linear_outputs(self, mels):
        """tt2_linear_outputs: clip(FrameProjection(num_freq)(CBHG(mels))) for mels [B,T,num_mels]
        (hp.predict_linear; tacotron.py:466-481)."""
        m = f32(mels)
        B, T, _ = m.shape
        if self._chunks:
            return np.concatenate([ch.linear_outputs(m[s:e]) for ch, (s, e) in
                                   zip(self._chunks, self._ranges(B)) if e > s])
        out = np.zeros((B, T, self.hp.num_freq), np.float32)
        self._ok(self.lib.tt2_linear_outputs(self.h, ptr(m), B, T, ptr(out)))
        return out

    def set_emt_labels(self, labels):
        """Tacotron_emt_attn: emotion labels [B] (the emt_labels placeholder, synthesizer.py:35) used
        by the next encode ('style_tokens' one-hot query)."""
        lab = i32(labels)
        if self._chunks:
            for ch, (s, e) in zip(self._chunks, self._ranges(lab.shape[0])):
                if e > s:
                    ch.set_emt_labels(lab[s:e])
            return
        self._ok(self.lib.tt2_set_emt_labels(self.h, ptr(lab), lab.shape[0]))

    def emt_alignments(self):
        """Tacotron_emt_attn: emotion attention weights of the last decode, [B, heads, T_v, n_steps]
        (tower_alignments_emt)."""
        if self._chunks:
            n = self._n_steps
            return np.concatenate([ch.emt_alignments()[..., :n] for ch, (s, e) in
                                   zip(self._chunks, self._ranges(self._B)) if e > s])
        heads, tv = ctypes.c_int32(), ctypes.c_int32()
        self._ok(self.lib.tt2_emt_alignments(self.h, None, ctypes.byref(heads), ctypes.byref(tv)))
        n = self._n_steps
        out = np.zeros((n, self._B, heads.value, tv.value), np.float32)
        self._ok(self.lib.tt2_emt_alignments(self.h, ptr(out), ctypes.byref(heads), ctypes.byref(tv)))
        return out.transpose(1, 2, 3, 0)

    def decoder_path(self):
        """(persistent, kernel_ms): 1 when the single-launch persistent decoder serves the current
        shapes (k_decode_persist), 0 for the per-step launch path; HIP-event time of the last
        persistent decode launch."""
        if self._chunks:
            return self._chunks[0].decoder_path()
        p = ctypes.c_int()
        ms = ctypes.c_float()
        self._ok(self.lib.tt2_decoder_path(self.h, ctypes.byref(p), ctypes.byref(ms)))
        return p.value, ms.value

    def postnet(self, frames=None, B=None, T=None):
        if frames is not None:
            frames = f32(frames)
            B, T = frames.shape[:2]
        if self._chunks:
            if frames is None:
                frames = self._frames
                T = frames.shape[1]
            parts = [ch.postnet(frames[s:e], e - s, T)
                     for ch, (s, e) in zip(self._chunks, self._ranges(B)) if e > s]
            return np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])
        dec = np.zeros((B, T, self.hp.num_mels), np.float32)
        mel = np.zeros((B, T, self.hp.num_mels), np.float32)
        self._ok(self.lib.tt2_postnet(self.h, ptr(frames), B, T, ptr(dec), ptr(mel)))
        return dec, mel

    def synthesize(self, ids, lengths, ref_emt, ref_spk, max_iters, prenet_masks=None, seed=0,
                   targets=None):
        """encode → decode → postnet; returns the tower_* outputs of one tower."""
        ids = i32(ids)
        self._B, self._T_in = ids.shape
        mem, style = self.encode(ids, lengths, ref_emt, ref_spk)
        frames, stop, align = self.decode(max_iters, prenet_masks, seed, targets)
        dec, mel = self.postnet(None, self._B, frames.shape[1])
        return dict(encoder_outputs=mem, style=style, decoder_output=dec, mel_outputs=mel,
                    stop_token_prediction=stop, alignments=align, frames=frames)


#: tt2_wn_config.upsample_type codes (wavenet.py:163-203)
UPSAMPLE_TYPES = ("2D", "1D", "Resize", "SubPixel", "NearestNeighbor")


def wavenet_config(hp, max_batch, max_samples, lib=None):
    lib = lib or _lib.load_library()
    cfg = _lib.WnConfig()
    lib.tt2_wn_default_config(ctypes.byref(cfg), max_batch, max_samples)
    cfg.layers = hp.layers
    cfg.stacks = hp.stacks
    cfg.residual_channels = hp.residual_channels
    cfg.gate_channels = hp.gate_channels
    cfg.skip_out_channels = hp.skip_out_channels
    cfg.kernel_size = hp.kernel_size
    cfg.cin_channels = hp.cin_channels
    cfg.out_channels = hp.out_channels
    cfg.legacy = 1 if hp.legacy else 0
    cfg.residual_legacy = 1 if hp.residual_legacy else 0
    cfg.log_scale_min = hp.log_scale_min
    if hp.upsample_type not in UPSAMPLE_TYPES:
        raise ValueError("upsample_type {!r} not in {}".format(hp.upsample_type, UPSAMPLE_TYPES))
    cfg.upsample_type = UPSAMPLE_TYPES.index(hp.upsample_type)
    acts = (None, "Relu", "LeakyRelu")
    if hp.upsample_activation not in acts:
        raise ValueError("upsample_activation {!r} not in {}".format(hp.upsample_activation, acts))
    cfg.upsample_activation = acts.index(hp.upsample_activation)
    cfg.leaky_alpha = hp.leaky_alpha
    cfg.NN_init = 1 if hp.NN_init else 0
    cfg.log_scale_min_gauss = hp.log_scale_min_gauss
    cfg.gin_channels = hp.gin_channels if hp.gin_channels > 0 else -1       # wavenet.py:152-158
    cfg.n_speakers = hp.n_speakers if (hp.gin_channels > 0 and hp.use_speaker_embedding) else 0
    itype = getattr(hp, "input_type", "raw")
    cfg.input_type = ("raw", "mulaw", "mulaw-quantize").index(itype)
    cfg.quantize_channels = hp.quantize_channels
    if itype == "mulaw-quantize" and hp.out_channels != hp.quantize_channels:
        raise ValueError("mulaw-quantize: out_channels must equal quantize_channels (hparams.py:222)")
    if hp.cin_channels <= 0:   # unconditional: no upsampling network
        return cfg
    cfg.n_upsample = len(hp.upsample_scales)
    for i, s in enumerate(hp.upsample_scales):
        cfg.upsample_scales[i] = s
    cfg.freq_axis_kernel_size = hp.freq_axis_kernel_size
    prod = int(np.prod(hp.upsample_scales))
    if prod != get_hop_size(hp):
        raise ValueError("prod(upsample_scales)={} != hop_size={} (hparams.py:241 asserts this)"
                         .format(prod, get_hop_size(hp)))
    return cfg


class WaveNetEngine(object):
    """Owns one tt2_wn_ctx."""

    def __init__(self, hp, weights, max_batch, max_samples, device=0, lib=None):
        self.lib = lib or _lib.load_library()
        self.hp = hp
        self.cfg = wavenet_config(hp, max_batch, max_samples, self.lib)
        self.caps = (max_batch, max_samples)
        self.hop = int(np.prod(hp.upsample_scales)) if hp.cin_channels > 0 else 1
        self.quantize = getattr(hp, "input_type", "raw") == "mulaw-quantize"
        h = ctypes.c_void_p()
        self._ok(self.lib.tt2_wn_create(ctypes.byref(self.cfg), device, ctypes.byref(h)))
        self.h = h
        for name, arr in weights.items():
            if name.startswith("WaveNet_model/"):
                _lib.load_tensor(self.lib.tt2_wn_load_tensor, self.h, name, arr, self.lib)
        self._ok(self.lib.tt2_wn_finalize(self.h))

    def _ok(self, status):
        _lib.check(status, self.lib)

    def close(self):
        if getattr(self, "h", None):
            self.lib.tt2_wn_destroy(self.h)
            self.h = None

    __del__ = close

    def fits(self, B, T):
        return B <= self.caps[0] and T <= self.caps[1]

    def set_global_condition(self, g, B):
        """g: speaker ids [B] (int, with the gc_embedding table) or features [B, gin_channels]
        (float); None clears it.  WaveNet.incremental's g (wavenet.py:770-775)."""
        if g is None:
            self._ok(self.lib.tt2_wn_set_global_condition(self.h, None, None, 0))
            return
        g = np.asarray(g)
        if np.issubdtype(g.dtype, np.integer):
            ids = np.ascontiguousarray(g.reshape(B), np.int32)
            self._ok(self.lib.tt2_wn_set_global_condition(self.h, ptr(ids), None, B))
        else:
            feat = np.ascontiguousarray(g.reshape(B, -1), np.float32)
            if feat.shape[1] != self.hp.gin_channels:
                raise ValueError("global condition features must be [B, gin_channels]")
            self._ok(self.lib.tt2_wn_set_global_condition(self.h, None, ptr(feat), B))

    def generate(self, cond, u_mix=None, u_log=None, seed=0, teacher=None, want_logits=False,
                 want_upsampled=False, g=None):
        """cond [B, T_f, cin] (clipped + interp'd); g: global condition (set_global_condition;
        required when gin_channels > 0).  Returns dict(y [B,T], k [B,T], logits?,
        upsampled? [B, cin, T])."""
        cond = f32(cond)
        B, T_f, F = cond.shape
        if self.hp.gin_channels > 0:
            if g is None:
                raise ValueError("gin_channels > 0: a global condition g is required")
            self.set_global_condition(g, B)
        T = T_f * self.hop
        nr = self.hp.out_channels // 3
        um, ul, tg = f32(u_mix), f32(u_log), f32(teacher)
        if self.hp.out_channels == 2 or self.quantize:
            um = None  # Gaussian head: the N(0,1) draws in u_log; mulaw-quantize: tf.multinomial's uniforms
        if um is not None and um.shape != (T, B, nr):
            raise ValueError("u_mix must be [T, B, nr_mix] = {}".format((T, B, nr)))
        if ul is not None and ul.shape != (T, B):
            raise ValueError("u_log must be [T, B]")
        if tg is not None and tg.shape != (B, T):
            raise ValueError("teacher (test_inputs) must be [B, T]")
        y = np.zeros((B, T), np.float32)
        k = np.zeros((B, T), np.int32)
        lg = np.zeros((B, T, self.hp.out_channels), np.float32) if want_logits else None
        up = np.zeros((B, F, T), np.float32) if want_upsampled else None
        self._ok(self.lib.tt2_wn_generate(self.h, ptr(cond), B, T_f, ptr(um), ptr(ul), seed, ptr(tg),
                                       ptr(y), ptr(k), ptr(lg), ptr(up)))
        return dict(y=y, k=k, logits=lg, upsampled=up)

    def generate_unconditional(self, B, T, u_mix=None, u_log=None, seed=0, teacher=None,
                               want_logits=False, g=None):
        """cin_channels <= 0: T samples per row without a local condition (wavenet.py:410-411,
        synthesis_length); the sampler / teacher contract of generate()."""
        if self.hp.gin_channels > 0:
            if g is None:
                raise ValueError("gin_channels > 0: a global condition g is required")
            self.set_global_condition(g, B)
        nr = self.hp.out_channels // 3
        um, ul, tg = f32(u_mix), f32(u_log), f32(teacher)
        if self.hp.out_channels == 2 or self.quantize:
            um = None
        if um is not None and um.shape != (T, B, nr):
            raise ValueError("u_mix must be [T, B, nr_mix] = {}".format((T, B, nr)))
        if ul is not None and ul.shape != (T, B):
            raise ValueError("u_log must be [T, B]")
        if tg is not None and tg.shape != (B, T):
            raise ValueError("teacher (test_inputs) must be [B, T]")
        y = np.zeros((B, T), np.float32)
        k = np.zeros((B, T), np.int32)
        lg = np.zeros((B, T, self.hp.out_channels), np.float32) if want_logits else None
        self._ok(self.lib.tt2_wn_generate_unconditional(self.h, B, T, ptr(um), ptr(ul), seed, ptr(tg),
                                                     ptr(y), ptr(k), ptr(lg)))
        return dict(y=y, k=k, logits=lg)


def mol_sample(logits, u_mix, u_log, log_scale_min):
    """tt2_mol_sample: logits [n, 3*nr], u_mix [n, nr], u_log [n] -> (x [n], k [n])."""
    lib = _lib.load_library()
    logits = f32(logits)
    u_mix = f32(u_mix)
    u_log = f32(u_log)
    n, C = logits.shape
    x = np.zeros((n,), np.float32)
    k = np.zeros((n,), np.int32)
    check(lib.tt2_mol_sample(ptr(logits), ptr(u_mix), ptr(u_log), n, C // 3, log_scale_min,
                             ptr(x), ptr(k)))
    return x, k


def prenet_keep_bits(seed, max_iters, B, P):
    """tt2_prenet_keep_bits: the keep bits [max_iters, 2, B, P] tt2_decode draws from the device RNG
    for ``seed`` when no prenet_masks are injected."""
    lib = _lib.load_library()
    out = np.zeros((max_iters, 2, B, P), np.uint8)
    check(lib.tt2_prenet_keep_bits(seed, max_iters, B, P, ptr(out)))
    return out


def wavenet_noise(seed, T, B, nr_mix=10, gaussian=False):
    """tt2_wn_noise: (u_mix [T,B,nr_mix] or None, u_log [T,B]) that tt2_wn_generate draws from the
    device RNG for ``seed`` when none are injected (Gaussian head: u_log = the N(0,1) draws)."""
    lib = _lib.load_library()
    um = None if gaussian else np.zeros((T, B, nr_mix), np.float32)
    ul = np.zeros((T, B), np.float32)
    check(lib.tt2_wn_noise(seed, T, B, nr_mix, 1 if gaussian else 0, ptr(um), ptr(ul)))
    return um, ul
