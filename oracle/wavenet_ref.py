"""TEST INFRASTRUCTURE ONLY — numpy restatement of the WaveNet MoL vocoder's synthesis path
(fast-WaveNet incremental generation) of mwhitehill/Tacotron-2 (see ``oracle/__init__.py``:
parity unpinned, never imported by the product).

Weights are keyed by the canonical TF names from ``tt2.weights.wavenet_weight_specs``
(prefix ``WaveNet_model/inference/``).
"""
import numpy as np

P = "WaveNet_model/inference/"
SQRT_HALF = np.float32(np.sqrt(0.5))


def _w(W, name, dt=np.float32):
    return np.asarray(W[P + name], dtype=dt)


def receptive_field_size(total_layers, num_cycles, kernel_size):
    """wavenet.py:54-71."""
    per = total_layers // num_cycles
    return (kernel_size - 1) * sum(2 ** (i % per) for i in range(total_layers)) + 1


def interp_condition(mel, max_abs_value=4.0):
    """Host-side conditioning prep of wavenet_vocoder/synthesizer.py:63-70: clip to
    [-max, max] then wavenet_vocoder/feeder.py:426-428 _interp to [0, 1]."""
    m = np.clip(np.asarray(mel, np.float32), -max_abs_value, max_abs_value)
    return ((m + np.float32(max_abs_value)) / np.float32(2 * max_abs_value)).astype(np.float32)


def condition_batch(mels, max_abs_value=4.0, symmetric=True, clip=True, normalize=True):
    """wavenet_vocoder/synthesizer.py:52-70 for a list of ragged mels [T_i, 80]: clip to
    T2_output_range (clip_for_wavenet), _pad_inputs with T2_output_range[0] to maxlen (:117-118),
    _interp to [0, 1] (normalize_for_wavenet, feeder.py:426-428).  Returns [B, maxlen, 80] f32."""
    lo, hi = (-max_abs_value, max_abs_value) if symmetric else (0.0, max_abs_value)
    maxlen = max(len(m) for m in mels)
    if clip:
        mels = [np.clip(m, lo, hi) for m in mels]
    c = np.stack([np.pad(m, [(0, maxlen - len(m)), (0, 0)], mode='constant', constant_values=lo)
                  for m in mels]).astype(np.float32)
    if normalize:
        c = ((c - np.float32(lo)) / np.float32(hi - lo)).astype(np.float32)
    return c


def upsample_2d(c, W, scales, freq_kernel=3, act="Relu", alpha=0.4):
    """ConvTranspose2D stack + ReLU (wavenet.py:171-203, 782-803; modules.py:736-770).

    c [B, F, T_f] (channels_first, expanded to [B,1,F,T]); per scale s a 1→1 channel
    conv2d_transpose with kernel (freq_kernel, s), strides (1, s), 'same':
        out[f, i·s + j] = Σ_d in[f + pad − d, i] · K[d, j] + b,  pad = (freq_kernel−1)//2
    (the adjoint of TF's 'same' correlation), then ReLU.  Returns [B, F, T_f·Πs]."""
    x = np.asarray(c, np.float32)
    B, F, _ = x.shape
    pad = (freq_kernel - 1) // 2
    for i, s in enumerate(scales):
        scope = "local_conditioning_upsampling_{}/ConvTranspose2D_layer_{}/".format(i + 1, i)
        K = _w(W, scope + "kernel")[:, :, 0, 0]   # [freq_kernel, s]
        b = _w(W, scope + "bias")[0]
        T = x.shape[-1]
        out = np.zeros((B, F, T, s), np.float32)
        for d in range(freq_kernel):
            sh = pad - d                          # out[f] += in[f + sh] * K[d]
            src = np.zeros_like(x)
            if sh >= 0:
                src[:, :F - sh] = x[:, sh:]
            else:
                src[:, -sh:] = x[:, :F + sh]
            out += src[..., None] * K[d][None, None, None, :]
        x = _act(out.reshape(B, F, T * s) + b, act, alpha)
    return x


def _act(x, act, alpha):
    """upsample activation (modules.py:23-41): None / 'Relu' / 'LeakyRelu' = max(x, alpha·x)."""
    if act == "Relu":
        return np.maximum(x, np.float32(0))
    if act == "LeakyRelu":
        return np.maximum(x, np.float32(alpha) * x)
    return x


def _shift_freq(x, sh):
    """src[:, f] = x[:, f + sh] (zero outside), x [B, F, T]."""
    F = x.shape[1]
    src = np.zeros_like(x)
    if sh >= 0:
        src[:, :F - sh] = x[:, sh:]
    else:
        src[:, -sh:] = x[:, :F + sh]
    return src


def _shift_time(x, sh):
    """src[..., t] = x[..., t + sh] (zero outside)."""
    T = x.shape[-1]
    src = np.zeros_like(x)
    if sh >= 0:
        src[..., :T - sh] = x[..., sh:]
    else:
        src[..., -sh:] = x[..., :T + sh]
    return src


def upsample_network(c, W, hp):
    """The conditioning upsampling network of wavenet.py:163-203 applied as at :782-803, for every
    upsample_type.  c [B, F, T_f] channels-first; returns [B, F, T_f·hop].

    '2D'       ConvTranspose2D 1→1, kernel (KF, s), stride (1, s), 'same' (modules.py:736-770)
    '1D'       ConvTranspose1D F→F, kernel (1, s), stride (1, s), 'same' (modules.py:697-733):
               out[o, i·s+j] = Σ_c in[c, i] · K[0, j, o, c] + b[o]  (kernel == stride: no overlap)
    'Resize'   NN resize ×s on time, then Conv2D 1→1 kernel (KF, s) 'same' (modules.py:657-694)
    'SubPixel' Conv2D 1→s kernel (KF, 3) 'same', then periodic shuffle out[f, w·s+k] = conv[f, w, k]
               (modules.py:539-654); NN_init=False tiles output channel 0 (:585-593)
    'NearestNeighbor'  tf.image.resize NEAREST ×hop (modules.py:524-536), no activation
    TF 'same' for stride 1: pad_before = (k−1)//2.  Activation upsample_activation after every
    learnable layer."""
    ut = hp.get("upsample_type", "2D")
    act, alpha = hp.get("upsample_activation", "Relu"), hp.get("leaky_alpha", 0.4)
    KF = hp.get("freq_axis_kernel_size", 3)
    scales = hp["upsample_scales"]
    x = np.asarray(c, np.float32)
    if ut == "2D":
        up = upsample_2d(x, W, scales, KF, act=act, alpha=alpha)
        return up
    if ut == "NearestNeighbor":
        return np.repeat(x, int(np.prod(scales)), axis=-1)
    name = {"1D": "ConvTranspose1D", "Resize": "ResizeConvolution",
            "SubPixel": "SubPixelConvolution"}[ut]
    B, F, _ = x.shape
    pf = (KF - 1) // 2
    for i, s in enumerate(scales):
        scope = "local_conditioning_upsampling_{}/{}_layer_{}/".format(i + 1, name, i)
        K = _w(W, scope + "kernel")
        b = _w(W, scope + "bias")
        T = x.shape[-1]
        if ut == "1D":
            # [B, c, T] x K[0, j, o, c] -> [B, o, T, j]
            out = np.einsum("bct,joc->botj", x, K[0]).astype(np.float32) + b[None, :, None, None]
            x = out.reshape(B, F, T * s)
        elif ut == "Resize":
            nn = np.repeat(x, s, axis=-1)
            pt = (s - 1) // 2
            out = np.zeros_like(nn)
            for d in range(KF):
                src_f = _shift_freq(nn, d - pf)
                for q in range(s):
                    out += _shift_time(src_f, q - pt) * K[d, q, 0, 0]
            x = out + b[0]
        else:  # SubPixel
            K = K[:, :, 0, :]                                   # [KF, 3, s]
            if not hp.get("NN_init", True):
                K = np.broadcast_to(K[:, :, :1], K.shape)
            conv = np.zeros((B, F, T, s), np.float32)
            for d in range(KF):
                src_f = _shift_freq(x, d - pf)
                for q in range(3):
                    conv += _shift_time(src_f, q - 1)[..., None] * K[d, q][None, None, None, :]
            x = (conv + b[None, None, None, :]).reshape(B, F, T * s)
        x = _act(x.astype(np.float32), act, alpha)
    return x


def mol_sample(logits, u_mix, u_log, log_scale_min):
    """sample_from_discretized_mix_logistic (mixture.py:76-107) with injected uniforms.

    logits [N, 3·nr_mix]; u_mix [N, nr_mix]; u_log [N].  The Gumbel term log(−log u) and the
    logistic noise log u − log(1−u) are evaluated in float64 and rounded to float32 (documented
    build convention, identical on the HIP path) so that the mixture index k is reproducible
    bit-for-bit across devices.  Returns (x float32 [N], k int32 [N])."""
    logits = np.asarray(logits, np.float32)
    nr = logits.shape[1] // 3
    u_mix = np.asarray(u_mix, np.float32).astype(np.float64)   # the ABI carries fp32 uniforms
    u_log = np.asarray(u_log, np.float32).astype(np.float64)
    gl = np.log(-np.log(u_mix)).astype(np.float32)
    temp = logits[:, :nr] - gl                                  # :92
    k = np.argmax(temp, axis=1).astype(np.int32)                # :93 (first max)
    rows = np.arange(logits.shape[0])
    means = logits[rows, nr + k]                                # :98
    log_scales = np.maximum(logits[rows, 2 * nr + k], np.float32(log_scale_min))   # :99-100
    noise = (np.log(u_log) - np.log(1.0 - u_log)).astype(np.float32)
    x = means + np.exp(log_scales) * noise                      # :105
    return np.minimum(np.maximum(x, np.float32(-1)), np.float32(1)).astype(np.float32), k


def categorical_sample(logits, u):
    """tf.multinomial(logits, 1) (wavenet.py:861-867 with softmax=False: the logits are the
    unnormalised log-probabilities) with injected uniforms, restating TF's multinomial kernel: the
    running total of exp(logit - max) in float64 over the finite logits (the cdf), then the first
    class whose cdf exceeds u * total (std::upper_bound).  logits [N, Q]; u [N] (fp32 uniforms in
    [0, 1)).  Returns k int32 [N]."""
    lg = np.asarray(logits, np.float32).astype(np.float64)
    u = np.asarray(u, np.float32).astype(np.float64)
    fin = np.isfinite(lg)
    mx = np.max(np.where(fin, lg, -np.inf), axis=1, keepdims=True)
    e = np.where(fin, np.exp(lg - mx), 0.0)
    cdf = np.cumsum(e, axis=1)
    target = u * cdf[:, -1]
    k = np.array([np.searchsorted(cdf[i], target[i], side="right") for i in range(lg.shape[0])])
    return np.minimum(k, lg.shape[1] - 1).astype(np.int32)


def inv_mulaw_quantize_f32(k):
    """util.inv_mulaw_quantize on the synthesis graph's tensors (wavenet.py:450-452): float32
    arithmetic, mu hard-coded to 255 (util.py:105-129)."""
    mu = np.float32(255.0)
    y = np.float32(2.0) * np.asarray(k, np.float32) / mu - np.float32(1.0)
    return (np.sign(y) * (np.float32(1.0) / mu) * (np.power(np.float32(1.0) + mu, np.abs(y)) - np.float32(1.0))
            ).astype(np.float32)


def incremental(c_up, W, hp, u_mix, u_log, test_inputs=None, return_logits=False, g=None, T=None):
    """WaveNet.incremental (wavenet.py:724-911) for scalar ('raw' / 'mulaw') input with the MoL or
    Gaussian head (out_channels == 2: u_log carries the N(0,1) draws, u_mix is unused), or for
    'mulaw-quantize' input (one-hot of quantize_channels classes, wavenet.py:433-446) with the
    softmax head sampled by tf.multinomial (u_log [T, B] carries its uniforms; y is the sampled
    class through inv_mulaw_quantize, k the class).  c_up None: unconditional synthesis of T samples
    (no conv1x1c term, wavenet.py:410-411).

    c_up: upsampled conditioning [B, T, cin]; u_mix [T, B, nr_mix]; u_log [T, B];
    test_inputs [B, T] overrides next_input (wavenet.py:876-878); g: global condition -- speaker
    ids [B] (int: rows of WaveNet_model/gc_embedding, wavenet.py:770-773) or features [B, gin]
    (float) -- whose conv1x1g term joins both gate halves (modules.py:505-509).  Returns y [B, T] (float32),
    k [B, T] (int32) and, optionally, logits [B, T, out_channels]."""
    quant = hp.get("input_type", "raw") == "mulaw-quantize"
    if c_up is None:
        B = np.asarray(u_log).shape[1] if test_inputs is None else np.asarray(test_inputs).shape[0]
    else:
        c_up = np.asarray(c_up, np.float32)
        B, T, _ = c_up.shape
    L, stacks = hp["layers"], hp["stacks"]
    per = L // stacks
    R = hp["residual_channels"]
    legacy, res_legacy = hp.get("legacy", False), hp.get("residual_legacy", False)
    kw = hp.get("kernel_size", 3)
    Q = hp.get("quantize_channels", 256) if quant else 1
    first_k = _w(W, "input_convolution/kernel").reshape(Q, R)
    first_b = _w(W, "input_convolution/bias")
    if g is not None:
        g = np.asarray(g)
        if np.issubdtype(g.dtype, np.integer):
            g = np.asarray(W["WaveNet_model/gc_embedding"], np.float32)[g.reshape(B)]
        g = np.asarray(g, np.float32).reshape(B, -1)
    layers = []
    for l in range(L):
        s = "ResidualConv1DGLU_{}/".format(l)
        cs = s + "residual_block_causal_conv_ResidualConv1DGLU_{}/".format(l)
        layers.append(dict(
            d=2 ** (l % per),
            k=_w(W, cs + "kernel").reshape(kw * R, -1), b=_w(W, cs + "bias"),
            kc=None if c_up is None else _w(W, s + "residual_block_cin_conv_ResidualConv1DGLU_{}/kernel".format(l))[0],
            bc=None if c_up is None else _w(W, s + "residual_block_cin_conv_ResidualConv1DGLU_{}/bias".format(l)),
            ks=_w(W, s + "residual_block_skip_conv_ResidualConv1DGLU_{}/kernel".format(l))[0],
            bs=_w(W, s + "residual_block_skip_conv_ResidualConv1DGLU_{}/bias".format(l)),
            ko=_w(W, s + "residual_block_out_conv_ResidualConv1DGLU_{}/kernel".format(l))[0],
            bo=_w(W, s + "residual_block_out_conv_ResidualConv1DGLU_{}/bias".format(l))))
        if g is not None:                                  # conv1x1g of g, constant over time
            gs = s + "residual_block_gin_conv_ResidualConv1DGLU_{}/".format(l)
            layers[-1]["gc"] = g @ _w(W, gs + "kernel")[0] + _w(W, gs + "bias")
    f1k = _w(W, "skip_convolutions/final_convolution_1/kernel")[0]
    f1b = _w(W, "skip_convolutions/final_convolution_1/bias")
    f2k = _w(W, "skip_convolutions/final_convolution_2/kernel")[0]
    f2b = _w(W, "skip_convolutions/final_convolution_2/bias")
    queues = [np.zeros((B, kw + (kw - 1) * (ly["d"] - 1), R), np.float32) for ly in layers]  # :815
    cur = np.zeros((B, 1), np.float32)   # initial_input = 0 ('raw'), wavenet.py:437-445
    kcur = np.full((B,), 127, np.int64)  # 'mulaw-quantize': one_hot(mulaw_quantize(0)) (util.py:99-102: mu = 255)
    ys = np.zeros((B, T), np.float32)
    ks = np.zeros((B, T), np.int32)
    lg = np.zeros((B, T, f2b.shape[0]), np.float32) if return_logits else None
    zero = np.float32(0)
    for t in range(T):
        ct = None if c_up is None else c_up[:, t]
        if quant:   # first_conv of a one-hot row = that row of the kernel
            x = first_k[kcur] + first_b
        else:
            x = cur @ first_k + first_b                   # first_conv.incremental_step :826
        skips = None
        for ly, q in zip(layers, queues):                 # :830-837
            residual = x
            q[:, :-1] = q[:, 1:].copy()                   # modules.py:285-288 shift + append
            q[:, -1] = x
            taps = q[:, ::ly["d"]]                        # modules.py:291-292
            h = taps.reshape(B, -1) @ ly["k"] + ly["b"]   # modules.py:295-297
            G2 = h.shape[1] // 2
            cc = np.zeros_like(h) if ct is None else ct @ ly["kc"] + ly["bc"]   # modules.py:497-501
            if g is not None:
                cc = cc + ly["gc"]                        # modules.py:505-509
            a = h[:, :G2] + cc[:, :G2]
            bgate = h[:, G2:] + cc[:, G2:]
            z = np.tanh(a) * (1.0 / (1.0 + np.exp(-bgate))).astype(np.float32)   # :510
            sk = z @ ly["ks"] + ly["bs"]                  # :512
            x = z @ ly["ko"] + ly["bo"]                   # :515
            x = (x + residual) * SQRT_HALF if res_legacy else x + residual    # :517-520
            if skips is None:
                skips = sk
            else:
                skips = (skips + sk) * SQRT_HALF if legacy else skips + sk   # wavenet.py:833-836
        x = np.maximum(skips, zero) @ f1k + f1b          # :840-844
        x = np.maximum(x, zero) @ f2k + f2b
        if lg is not None:
            lg[:, t] = x
        if quant:             # tf.multinomial over the logits, one_hot of the draw (wavenet.py:861-867)
            k = categorical_sample(x, u_log[t])
            y = inv_mulaw_quantize_f32(k)
        elif x.shape[1] == 2:   # Gaussian head: sample_from_gaussian (gaussian.py:39-52), u_log = N(0,1)
            ls = np.maximum(x[:, 1], np.float32(hp["log_scale_min_gauss"]))
            y = np.clip(x[:, 0] + np.exp(ls) * np.asarray(u_log[t], np.float32), -1, 1).astype(np.float32)
            k = np.zeros((B,), np.int32)
        else:
            y, k = mol_sample(x, u_mix[t], u_log[t], hp["log_scale_min"])
        ys[:, t] = y
        ks[:, t] = k
        if quant:
            kcur = k.astype(np.int64) if test_inputs is None else np.asarray(test_inputs)[:, t].astype(np.int64)
        cur = y[:, None] if test_inputs is None else np.asarray(test_inputs, np.float32)[:, t:t + 1]
    return (ys, ks, lg) if return_logits else (ys, ks)


def synthesize(mel, W, hp, u_mix, u_log, test_inputs=None, return_logits=False):
    """wavenet_vocoder/synthesizer.py:46-103 for one batch of equal-length mels [B, T_f, 80]:
    clip + interp, upsample, incremental generation of T_f·hop samples."""
    c = interp_condition(mel, hp.get("max_abs_value", 4.0))       # [B, T_f, 80]
    c_up = upsample_network(c.transpose(0, 2, 1), W, hp)         # [B, 80, T]
    return incremental(c_up.transpose(0, 2, 1), W, hp, u_mix, u_log, test_inputs, return_logits)
