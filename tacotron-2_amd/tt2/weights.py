"""Canonical weight key space (the reference's TF variable names) and seeded random init.

The reference ships no trained Tacotron/WaveNet checkpoints, so benchmarks and
parity tests run on random-init weights of the reference architecture.  Names follow the TF
variable scopes the reference builds (``Tacotron_model/inference/...`` from
``code/tacotron/synthesizer.py:38`` + ``tacotron.py:201``; ``WaveNet_model/inference/...`` from
``code/wavenet_vocoder/synthesizer.py:27`` + ``wavenet.py:269``).  Scope names inside TF
library cells (``lstm_cell``, ``gru_cell``, ``bidirectional_rnn``) follow TF 1.x conventions and
are unverified without TensorFlow (no real checkpoint for these layers exists in the reference).
"""
import numpy as np

TP = "Tacotron_model/inference/"
WP = "WaveNet_model/inference/"


def _bn(scope, c):
    s = scope + "batch_normalization/"
    return [(s + "gamma", (c,), "bn_gamma"), (s + "beta", (c,), "bn_beta"),
            (s + "moving_mean", (c,), "bn_mean"), (s + "moving_variance", (c,), "bn_var")]


def _text_encoder_specs(hp):
    """embedding, EncoderConvolutions, EncoderRNN (tacotron.py:215-231)."""
    S = []
    n_sym = 66  # tacotron/utils/symbols.py:9-17
    E = hp.embedding_dim
    S.append((TP + "inputs_embedding", (n_sym, E), "glorot"))
    cin = E
    kw = hp.enc_conv_kernel_size[0]
    for i in range(1, hp.enc_conv_num_layers + 1):
        sc = TP + "encoder_convolutions/conv_layer_{}_encoder_convolutions/".format(i)
        S.append((sc + "conv1d/kernel", (kw, cin, hp.enc_conv_channels), "glorot"))
        S.append((sc + "conv1d/bias", (hp.enc_conv_channels,), "bias"))
        S += _bn(sc, hp.enc_conv_channels)
        cin = hp.enc_conv_channels
    U = hp.encoder_lstm_units
    for d in ("fw", "bw"):
        sc = TP + "encoder_LSTM/bidirectional_rnn/{}/lstm_cell/".format(d)
        S.append((sc + "kernel", (cin + U, 4 * U), "glorot"))
        S.append((sc + "bias", (4 * U,), "bias"))
    return S


def _refnet_convs(hp, sc):
    """ReferenceEncoder CNN stack (modules.py:22-33); returns (specs, flattened output width)."""
    S = []
    c_in, F = 1, hp.num_mels
    for i, f in enumerate(hp.reference_filters):
        s2 = sc + "conv2d_{}/".format(i)
        S.append((s2 + "conv2d/kernel", (3, 3, c_in, f), "glorot"))
        S.append((s2 + "conv2d/bias", (f,), "bias"))
        S += _bn(s2, f)
        c_in = f
        F = -(-F // 2)
    return S, F * c_in


def _gru_specs(sc, gin, D):
    """TF1 GRUCell variables under ``sc`` (gates [r, u] and candidate)."""
    return [(sc + "gates/kernel", (gin + D, 2 * D), "glorot"),
            (sc + "gates/bias", (2 * D,), "gru_gate_bias"),
            (sc + "candidate/kernel", (gin + D, D), "glorot"),
            (sc + "candidate/bias", (D,), "bias")]


def _mha_specs(mh, q_in, v_in, A, heads):
    """MultiheadAttention mlp_attention, normalize=True (multihead_attention.py:43-110)."""
    return [(mh + "conv1d/kernel", (1, q_in, A), "glorot"), (mh + "conv1d/bias", (A,), "bias"),
            (mh + "conv1d_1/kernel", (1, v_in, A), "glorot"), (mh + "conv1d_1/bias", (A,), "bias"),
            (mh + "attention_v", (A // heads,), "glorot"), (mh + "attention_g", (), "mha_g"),
            (mh + "attention_b", (A // heads,), "bias")]


def _decoder_specs(hp, Dm, extra=0):
    """memory layer, LocationSensitiveAttention, Prenet, DecoderRNN, projections
    (tacotron.py:310-338); ``extra`` = LSTM-1 input columns after [prenet | context]."""
    S = []
    Ad = hp.attention_dim
    S.append((TP + "memory_layer/kernel", (Dm, Ad), "glorot"))
    S.append((TP + "decoder/query_layer/kernel", (hp.decoder_lstm_units, Ad), "glorot"))
    la = TP + "decoder/Location_Sensitive_Attention/"
    S.append((la + "location_features_convolution/kernel",
              (hp.attention_kernel[0], 1, hp.attention_filters), "glorot"))
    S.append((la + "location_features_convolution/bias", (hp.attention_filters,), "bias"))
    S.append((la + "location_features_layer/kernel", (hp.attention_filters, Ad), "glorot"))
    S.append((la + "attention_variable_projection", (Ad,), "glorot"))
    S.append((la + "attention_bias", (Ad,), "bias"))
    p_in = hp.num_mels
    for i, n in enumerate(hp.prenet_layers):
        sc = TP + "decoder/decoder_prenet/dense_{}/".format(i + 1)
        S.append((sc + "kernel", (p_in, n), "glorot"))
        S.append((sc + "bias", (n,), "bias"))
        p_in = n
    H = hp.decoder_lstm_units
    x_in = p_in + Dm + extra
    for l in range(hp.decoder_layers):
        sc = TP + "decoder/decoder_LSTM/multi_rnn_cell/cell_{}/lstm_cell/".format(l)
        S.append((sc + "kernel", (x_in + H, 4 * H), "glorot"))
        S.append((sc + "bias", (4 * H,), "bias"))
        x_in = H
    fp = TP + "decoder/linear_transform_projection/projection_linear_transform_projection/"
    S.append((fp + "kernel", (H + Dm, hp.num_mels * hp.outputs_per_step), "glorot"))
    S.append((fp + "bias", (hp.num_mels * hp.outputs_per_step,), "bias"))
    sp = TP + "decoder/stop_token_projection/projection_stop_token_projection/"
    S.append((sp + "kernel", (H + Dm, hp.outputs_per_step), "glorot"))
    S.append((sp + "bias", (hp.outputs_per_step,), "stop_bias"))
    return S


def _postnet_specs(hp):
    """Postnet + postnet_projection (tacotron.py:366-375)."""
    S = []
    cin = hp.num_mels
    kw = hp.postnet_kernel_size[0]
    for i in range(1, hp.postnet_num_layers + 1):
        sc = TP + "postnet_convolutions/conv_layer_{}_postnet_convolutions/".format(i)
        S.append((sc + "conv1d/kernel", (kw, cin, hp.postnet_channels), "glorot"))
        S.append((sc + "conv1d/bias", (hp.postnet_channels,), "bias"))
        S += _bn(sc, hp.postnet_channels)
        cin = hp.postnet_channels
    pp = TP + "postnet_projection/projection_postnet_projection/"
    S.append((pp + "kernel", (cin, hp.num_mels), "glorot"))
    S.append((pp + "bias", (hp.num_mels,), "bias"))
    return S


#: style paths of Tacotron.initialize (tacotron.py:236-308): GST attention over style tokens, the
#: reference embeddings themselves (args.pretrained_emb_disc_all, or hp.use_gst=False), or the AdaIN
#: reference encoder (args.adain)
STYLE_MODES = ("gst", "embed", "adain")


def style_mode(hp, style="gst"):
    """Effective style path: 'gst' needs hp.use_gst (tacotron.py:269), else the embeddings."""
    if style not in STYLE_MODES:
        raise ValueError("style must be one of {}".format(STYLE_MODES))
    return "embed" if style == "gst" and not hp.use_gst else style


def _adain_refnet_specs(hp, sc):
    """ReferenceEncoderAdaIn (modules.py:66-107): conv2d without batch norm, strides
    (2,2),(2,2),(1,1)x4 (tacotron.py:237), one GRU + dense(128, tanh) over the mixed speaker map.
    The speaker and emotion stacks each call conv2d(..., 'conv2d_%d') in scope 'refnet' (speaker
    first): tf.layers.conv2d uniquifies its default layer name in the re-entered scope, so the
    speaker convs are conv2d_i/conv2d/* and the emotion convs conv2d_i/conv2d_1/*."""
    S = []
    c_in, F = 1, hp.num_mels
    for i, f in enumerate(hp.reference_filters):
        s2 = sc + "conv2d_{}/".format(i)
        for ly in ("conv2d", "conv2d_1"):
            S.append((s2 + ly + "/kernel", (3, 3, c_in, f), "glorot"))
            S.append((s2 + ly + "/bias", (f,), "bias"))
        c_in = f
        if i < 2:
            F = -(-F // 2)
    D = hp.reference_depth
    S += _gru_specs(sc + "rnn/gru_cell/", F * c_in, D)
    S.append((sc + "dense/kernel", (D, 128), "glorot"))
    S.append((sc + "dense/bias", (128,), "bias"))
    return S


def cbhg_weight_specs(hp, name="CBHG_postnet"):
    """The post-processing CBHG + linear projection (modules.py:125-184, tacotron.py:466-478:
    commented out in the reference, built by predict_linear here).  Conv bank / projections via
    conv1d() (conv1d + batch_normalization scopes), the residual dense when num_mels !=
    highway_units, HighwayNet H / T layers (T bias init -1), named GRU cells under
    bidirectional_rnn/{fw,bw} (TF-internal naming unverified, like the other cells)."""
    S = []
    sc = TP + name + "/"
    nm, C = hp.num_mels, hp.cbhg_conv_channels
    for k in range(1, hp.cbhg_kernels + 1):
        s2 = sc + "conv_bank/conv1d_{}/".format(k)
        S += [(s2 + "conv1d/kernel", (k, nm, C), "glorot"), (s2 + "conv1d/bias", (C,), "bias")]
        S += _bn(s2, C)
    kp = hp.cbhg_projection_kernel_size
    for nm_, cin, cout in (("proj1", hp.cbhg_kernels * C, hp.cbhg_projection),
                           ("proj2", hp.cbhg_projection, nm)):
        s2 = sc + nm_ + "/"
        S += [(s2 + "conv1d/kernel", (kp, cin, cout), "glorot"), (s2 + "conv1d/bias", (cout,), "bias")]
        S += _bn(s2, cout)
    Hu = hp.cbhg_highway_units
    if nm != Hu:
        S += [(sc + "dense/kernel", (nm, Hu), "glorot"), (sc + "dense/bias", (Hu,), "bias")]
    for i in range(1, hp.cbhg_highwaynet_layers + 1):
        s2 = sc + "{}_highwaynet_{}/".format(name, i)
        S += [(s2 + "H/kernel", (Hu, Hu), "glorot"), (s2 + "H/bias", (Hu,), "bias"),
              (s2 + "T/kernel", (Hu, Hu), "glorot"), (s2 + "T/bias", (Hu,), "highway_t_bias")]
    R = hp.cbhg_rnn_units
    for d, cell in (("fw", "forward"), ("bw", "backward")):
        S += _gru_specs(sc + "bidirectional_rnn/{}/{}_{}_RNN/".format(d, name, cell), Hu, R)
    ps = TP + "cbhg_linear_specs_projection/projection_cbhg_linear_specs_projection/"
    S += [(ps + "kernel", (2 * R, hp.num_freq), "glorot"), (ps + "bias", (hp.num_freq,), "bias")]
    return S


def tacotron_weight_specs(hp, emt_only=False, style="gst"):
    """(name, shape, init) for every variable on the synthesis path (tacotron.py:215-381)."""
    mode = style_mode(hp, style)
    S = _text_encoder_specs(hp)
    if mode == "adain":   # one shared encoder 'refnet' over both references (tacotron.py:236-242)
        S += _adain_refnet_specs(hp, TP + "refnet/")
    else:
        # reference encoders (modules.py:9-64) and GST (tacotron.py:219-282)
        tags = ["emt"] if emt_only else ["emt", "spk"]
        for tag in tags:
            sc = TP + "refnet_{}/".format(tag)
            conv, gin = _refnet_convs(hp, sc)
            S += conv
            D = hp.reference_depth
            S += _gru_specs(sc + "rnn/gru_cell/", gin, D)
            S.append((sc + "dense/kernel", (D, 128), "glorot"))
            S.append((sc + "dense/bias", (128,), "bias"))
            if mode == "gst":
                tok_d = hp.style_embed_depth // hp.num_heads
                S.append((TP + "style_tokens_{}".format(tag), (hp.num_gst, tok_d), "gst_tokens"))
                S += _mha_specs(TP + "Multihead-attention-{}/".format(tag), 128, tok_d,
                                hp.style_att_dim, hp.num_heads)
    S += _decoder_specs(hp, memory_width(hp, emt_only, style))
    S += _postnet_specs(hp)
    return S + (cbhg_weight_specs(hp) if hp.predict_linear else [])


#: args.attn / args.emt_ref_gru values of Tacotron_emt_attn (train.py:147-150); codes 1.. / 0..
EMT_ATTN = ("simple", "multihead", "style_tokens")
EMT_REF_GRU = ("none", "gru", "gru_multi")


def emt_value_width(hp, attn, emt_ref_gru):
    """Width of one attended row: tanh(style_tokens) 16; refnet_emt all_outputs (modules.py:35-55):
    the reshaped CNN output ('none'), [fw | bw] GRU outputs ('gru'), dense(128) ('gru_multi')."""
    if attn == "style_tokens":
        return 16
    _, gin = _refnet_convs(hp, "")
    return {"none": gin, "gru": 2 * hp.reference_depth, "gru_multi": 128}[emt_ref_gru]


def emt_lstm_extra(hp, attn, emt_only=False):
    """LSTM-1 input columns after [prenet | context] (Architecture_wrappers.py:203-211): the emotion
    context (attention_dim / 128 / 64 wide, :116-123) and, concatenated ('simple') or added
    ('multihead'), refnet_spk's 128."""
    spk = attn != "style_tokens" and not emt_only
    if attn == "simple":
        return hp.attention_dim + (128 if spk else 0)
    if attn == "multihead":
        return 128
    return 4 * 16


def tacotron_emt_weight_specs(hp, attn, emt_ref_gru="none", emt_only=False, n_emt=4):
    """(name, shape, init) of Tacotron_emt_attn's synthesis graph (tacotron_emt_attn.py:198-381).

    Variables built inside the decoder cell live under ``decoder/`` (dynamic_decode's scope):
    SimpleBahdanauAttention's Dense layers ``W1``/``W2``/``V`` (built at first call,
    attention.py:237-250), ``Multihead-attention-attn_emt`` and the multi-head output dense
    ``attn_emt/dense`` (Architecture_wrappers.py:233-234).  Like the other TF-internal scope names
    these are unverified without TensorFlow (no checkpoint of this model ships)."""
    if attn not in EMT_ATTN or emt_ref_gru not in EMT_REF_GRU:
        raise ValueError("attn must be one of {} and emt_ref_gru one of {}".format(EMT_ATTN,
                                                                                  EMT_REF_GRU))
    S = _text_encoder_specs(hp)
    D = hp.reference_depth
    H = hp.decoder_lstm_units
    if attn == "style_tokens":
        S.append((TP + "style_tokens", (24, 16), "gst_tokens"))
    else:
        sc = TP + "refnet_emt/"
        conv, gin = _refnet_convs(hp, sc)
        S += conv
        if emt_ref_gru == "gru":
            for d in ("fw", "bw"):
                S += _gru_specs(sc + "bidirectional_rnn/{}/gru_cell/".format(d), gin, D)
        elif emt_ref_gru == "gru_multi":
            for i in range(8):
                S += _gru_specs(sc + "gru_{}/rnn/gru_cell/".format(i), gin, D)
                S.append((sc + "gru_{}/dense/kernel".format(i), (D, 128), "glorot"))
                S.append((sc + "gru_{}/dense/bias".format(i), (128,), "bias"))
        if not emt_only:
            sc = TP + "refnet_spk/"
            conv, gin = _refnet_convs(hp, sc)
            S += conv
            S += _gru_specs(sc + "rnn/gru_cell/", gin, D)
            S.append((sc + "dense/kernel", (D, 128), "glorot"))
            S.append((sc + "dense/bias", (128,), "bias"))
    Dm = 2 * hp.encoder_lstm_units
    S += _decoder_specs(hp, Dm, emt_lstm_extra(hp, attn, emt_only))
    Dv = emt_value_width(hp, attn, emt_ref_gru)
    if attn == "simple":
        A = hp.attention_dim
        S += [(TP + "decoder/W1/kernel", (Dv, A), "glorot"), (TP + "decoder/W1/bias", (A,), "bias"),
              (TP + "decoder/W2/kernel", (H, A), "glorot"), (TP + "decoder/W2/bias", (A,), "bias"),
              (TP + "decoder/V/kernel", (A, 1), "glorot"), (TP + "decoder/V/bias", (1,), "bias")]
    else:
        q_in = H + (n_emt if attn == "style_tokens" else 0)
        S += _mha_specs(TP + "decoder/Multihead-attention-attn_emt/", q_in, Dv, hp.style_att_dim,
                        hp.num_heads)
        if attn == "multihead":
            S += [(TP + "decoder/attn_emt/dense/kernel", (hp.num_heads * Dv, 128), "glorot"),
                  (TP + "decoder/attn_emt/dense/bias", (128,), "bias")]
    return S + _postnet_specs(hp)


def memory_width(hp, emt_only=False, style="gst"):
    """D_mem = 2·encoder_lstm_units + style width (tacotron.py:297-308): per
    reference a GST embedding (style_embed_depth) or the 128-wide reference embedding; AdaIN
    passes one 128-wide embedding (:266-268)."""
    mode = style_mode(hp, style)
    if mode == "adain":
        return 2 * hp.encoder_lstm_units + 128
    w = hp.style_embed_depth if mode == "gst" else 128
    return 2 * hp.encoder_lstm_units + (w if emt_only else 2 * w)


def wavenet_weight_specs(hp):
    """(name, shape, init) of the WaveNet synthesis graph (wavenet.py:89-208)."""
    S = []
    R, G, Sk = hp.residual_channels, hp.gate_channels, hp.skip_out_channels
    # one-hot input of quantize_channels classes for 'mulaw-quantize' (Conv1D1x1 builds its kernel on
    # the input's channels, wavenet.py:102-115), a scalar otherwise
    qin = hp.quantize_channels if getattr(hp, "input_type", "raw") == "mulaw-quantize" else 1
    S.append((WP + "input_convolution/kernel", (1, qin, R), "glorot"))
    S.append((WP + "input_convolution/bias", (R,), "bias"))
    for l in range(hp.layers):
        s = WP + "ResidualConv1DGLU_{}/".format(l)
        kinds = [("causal", (hp.kernel_size, R, G)), ("cin", (1, hp.cin_channels, G)),
                 ("skip", (1, G // 2, Sk)), ("out", (1, G // 2, R))]
        if hp.cin_channels <= 0:  # local conditioning disabled: no conv1x1c (modules.py:421-426)
            kinds.pop(1)
        if hp.gin_channels > 0:   # conv1x1g (modules.py:427-433)
            kinds.insert(2, ("gin", (1, hp.gin_channels, G)))
        for kind, shape in kinds:
            sc = s + "residual_block_{}_conv_ResidualConv1DGLU_{}/".format(kind, l)
            S.append((sc + "kernel", shape, "glorot"))
            S.append((sc + "bias", (shape[-1],), "bias"))
    S.append((WP + "skip_convolutions/final_convolution_1/kernel", (1, Sk, Sk), "glorot"))
    S.append((WP + "skip_convolutions/final_convolution_1/bias", (Sk,), "bias"))
    S.append((WP + "skip_convolutions/final_convolution_2/kernel", (1, Sk, hp.out_channels), "glorot"))
    S.append((WP + "skip_convolutions/final_convolution_2/bias", (hp.out_channels,), "bias"))
    if hp.gin_channels > 0 and hp.use_speaker_embedding:   # Embedding, truncated normal std 0.1
        S.append(("WaveNet_model/gc_embedding", (hp.n_speakers, hp.gin_channels), "embed:0.1"))
    ut = hp.upsample_type
    if ut == "NearestNeighbor" or hp.cin_channels <= 0:  # NearestNeighborUpsample: no variables
        return S                                          # (modules.py:524-536); no upsampler without c
    name = {"2D": "ConvTranspose2D", "1D": "ConvTranspose1D", "Resize": "ResizeConvolution",
            "SubPixel": "SubPixelConvolution"}[ut]
    kf, nl = hp.freq_axis_kernel_size, len(hp.upsample_scales)
    for i, s in enumerate(hp.upsample_scales):
        sc = WP + "local_conditioning_upsampling_{}/{}_layer_{}/".format(i + 1, name, i)
        if ut == "1D":     # Conv2DTranspose kernel [1, s, out=cin, in=cin], bias [cin]
            S.append((sc + "kernel", (1, s, hp.cin_channels, hp.cin_channels),
                      "nn_up1d:{}".format(nl)))
            S.append((sc + "bias", (hp.cin_channels,), "bias"))
        elif ut == "SubPixel":  # Conv2D (kf, 3), 1 -> s filters
            S.append((sc + "kernel", (kf, 3, 1, s), "nn_subpixel:{}".format(nl)))
            S.append((sc + "bias", (s,), "bias"))
        else:              # 2D / Resize: (kf, s) 1 -> 1
            S.append((sc + "kernel", (kf, s, 1, 1), "nn_{}:{}".format(ut.lower(), nl)))
            S.append((sc + "bias", (1,), "bias"))
    return S


def _init(rng, shape, kind, hp):
    shape = tuple(shape)
    if kind == "glorot":
        if len(shape) == 0:
            return np.float32(rng.uniform(-1, 1))
        if len(shape) == 1:
            fi = fo = shape[0]
        else:
            rf = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
            fi, fo = shape[-2] * rf, shape[-1] * rf
        lim = np.sqrt(6.0 / (fi + fo))
        return rng.uniform(-lim, lim, shape).astype(np.float32)
    if kind == "bias":
        return rng.uniform(-0.1, 0.1, shape).astype(np.float32)
    if kind == "stop_bias":
        # negative so that an untrained (random) model decodes to max_iters instead of stopping on
        # a coin flip; tests that exercise the stop rule override this bias explicitly
        return rng.uniform(-3.5, -2.5, shape).astype(np.float32)
    if kind == "highway_t_bias":  # HighwayNet T layer: bias_initializer=constant(-1) (modules.py:116)
        return (-1.0 + rng.uniform(-0.1, 0.1, shape)).astype(np.float32)
    if kind == "gru_gate_bias":
        return (1.0 + rng.uniform(-0.1, 0.1, shape)).astype(np.float32)  # TF GRUCell bias init 1.0
    if kind == "bn_gamma":
        return rng.uniform(0.8, 1.2, shape).astype(np.float32)
    if kind in ("bn_beta", "bn_mean"):
        return rng.uniform(-0.1, 0.1, shape).astype(np.float32)
    if kind == "bn_var":
        return rng.uniform(0.8, 1.2, shape).astype(np.float32)
    if kind.startswith("embed:"):  # truncated_normal_initializer(0, std) (modules.py:13-20)
        # TF redraws samples beyond 2 std (it does not clip them onto the bound)
        std = float(kind.split(":")[1])
        v = rng.normal(0, std, shape)
        bad = np.abs(v) > 2 * std
        while bad.any():
            v[bad] = rng.normal(0, std, int(bad.sum()))
            bad = np.abs(v) > 2 * std
        return v.astype(np.float32)
    if kind == "gst_tokens":  # truncated_normal(stddev=0.5), tacotron.py:221-224
        v = rng.normal(0, 0.5, shape)
        return np.clip(v, -1.0, 1.0).astype(np.float32)
    if kind == "mha_g":  # sqrt(1/num_units), multihead_attention.py:103-105
        return np.float32(np.sqrt(1.0 / (hp.style_att_dim // hp.num_heads)))
    if kind.startswith("nn_"):
        # the reference's NN_init kernels (modules.py:645-654, 686-694, 723-733, 761-770) scaled by
        # NN_scaler^(1/up_layers), plus a small perturbation so every tap is exercised by the
        # parity tests
        kind, up_layers = kind.split(":")
        scale = hp.NN_scaler ** (1.0 / int(up_layers))
        if kind == "nn_up1d":
            _, kw, co, ci = shape
            k = np.tile(np.eye(co, ci)[None, None], (1, kw, 1, 1))
            return (k * scale + rng.uniform(-0.05, 0.05, shape)).astype(np.float32)
        kh, kw = shape[0], shape[1]
        k = np.zeros((kh, kw), np.float64)
        if kind == "nn_2d":
            k[kh // 2, :] = 1.0
        else:  # resize / subpixel: centre tap(s)
            js = [kw // 2 - 1, kw // 2] if kw % 2 == 0 else [kw // 2]
            for j in js:
                k[kh // 2, j] = 0.5 if kw % 2 == 0 else 1.0
        k = k.reshape(kh, kw, 1, 1) * scale
        k = np.broadcast_to(k, shape) + rng.uniform(-0.05, 0.05, shape)
        return k.astype(np.float32)
    raise ValueError(kind)


def init_weights(specs, hp, seed=5339):
    """Seeded random init (seed defaults to tacotron_random_seed/wavenet_random_seed = 5339)."""
    rng = np.random.default_rng(seed)
    return {name: np.asarray(_init(rng, shape, kind, hp), np.float32).reshape(shape)
            for name, shape, kind in specs}


def init_tacotron_weights(hp, seed=5339, emt_only=False, style="gst"):
    return init_weights(tacotron_weight_specs(hp, emt_only, style), hp, seed)


def init_tacotron_emt_weights(hp, attn, emt_ref_gru="none", emt_only=False, n_emt=4, seed=5339):
    return init_weights(tacotron_emt_weight_specs(hp, attn, emt_ref_gru, emt_only, n_emt), hp, seed)


def init_wavenet_weights(hp, seed=5339):
    return init_weights(wavenet_weight_specs(hp), hp, seed)
