"""TEST INFRASTRUCTURE ONLY — torch (CPU, float64 autograd) restatement of the teacher-forced
Tacotron-2 decoder training step of mwhitehill/Tacotron-2 (SURVEY.md §8f rank 1, configs[4]).

Only ``tests/`` and ``bench.py``'s ``cpu_baseline`` leg may import this module, as the checker;
the product path (``tacotron-2_amd``) never does.  Parity status: **parity unpinned** (TensorFlow
is absent, the reference has no training fixtures); the forward half is pinned to the numpy
inference oracle (``oracle/tacotron_ref.py``) by running it with inference zoneout, and the
gradients are torch autograd of this restatement.

Scope of the slice ("decoder training step"): memory (encoder outputs ⊕ style, as the decoder
receives it) → memory_layer keys → teacher-forced ``dynamic_decode`` with TacoTrainingHelper
(ratio 1, constant mode: hparams.py:300-301, helpers.py:118-129) → frame/stop projections →
losses ``before`` (MSE, mask_decoder=False: tacotron.py:774) + stop sigmoid cross-entropy
(tacotron.py:778-779) + L2 regularisation of the decoder-slice kernels (tacotron.py:865-867) →
gradients → tower mean + clip_by_global_norm(1.0) (tacotron.py:1194-1221) → TF AdamOptimizer
(tacotron.py:1029) with the exponential learning-rate decay (tacotron.py:1227-1251;
hparams.py:272-282).  The Postnet
``after`` loss is ``postnet=True``; the front end (encoder, reference encoders, GST) in training
mode is ``frontend_forward`` / ``train_grads_frontend``.

Training-mode zoneout (modules.py:236-240): ``c = (1-z)·dropout(c_new - c_prev, 1-z) + c_prev``,
i.e. ``c = c_prev + m·(c_new - c_prev)`` with keep bits m ~ Bernoulli(1-z) (injected).
"""
import numpy as np
import torch

P = "Tacotron_model/inference/"
LA = P + "decoder/Location_Sensitive_Attention/"
L1 = P + "decoder/decoder_LSTM/multi_rnn_cell/cell_0/lstm_cell/"
L2 = P + "decoder/decoder_LSTM/multi_rnn_cell/cell_1/lstm_cell/"
FP = P + "decoder/linear_transform_projection/projection_linear_transform_projection/"
SP = P + "decoder/stop_token_projection/projection_stop_token_projection/"


PN = P + "postnet_convolutions/conv_layer_{}_postnet_convolutions/"
PP = P + "postnet_projection/projection_postnet_projection/"


def postnet_var_names(layers=5):
    """Trainable Postnet variables (modules.py:451-497; tacotron.py:362-375), library order."""
    names = []
    for i in range(1, layers + 1):
        s = PN.format(i)
        names += [s + "conv1d/kernel", s + "conv1d/bias", s + "batch_normalization/gamma",
                  s + "batch_normalization/beta"]
    return names + [PP + "kernel", PP + "bias"]


def postnet_stat_names(layers=5):
    return [PN.format(i) + "batch_normalization/" + n for i in range(1, layers + 1)
            for n in ("moving_mean", "moving_variance")]


def train_var_names(n_prenet=2):
    """The decoder-slice trainable variables, in the order of the library's flat buffers."""
    names = [P + "memory_layer/kernel", P + "decoder/query_layer/kernel",
             LA + "location_features_convolution/kernel", LA + "location_features_convolution/bias",
             LA + "location_features_layer/kernel", LA + "attention_variable_projection",
             LA + "attention_bias"]
    for i in range(n_prenet):
        s = P + "decoder/decoder_prenet/dense_{}/".format(i + 1)
        names += [s + "kernel", s + "bias"]
    names += [L1 + "kernel", L1 + "bias", L2 + "kernel", L2 + "bias",
              FP + "kernel", FP + "bias", SP + "kernel", SP + "bias"]
    return names


def regularized(name):
    """tacotron.py:865-867: every variable except biases, '_projection', embeddings, RNN/LSTM."""
    return not ("bias" in name or "Bias" in name or "_projection" in name
                or "inputs_embedding" in name or "RNN" in name or "LSTM" in name)


def _conv_same(cum, k, b):
    """tf.layers.conv1d 'same', 1 input channel (attention.py:193-195): cum [B,T], k [kw,1,F]."""
    kw = k.shape[0]
    pad = (kw - 1) // 2
    x = torch.nn.functional.pad(cum, (pad, kw - 1 - pad))
    cols = x.unfold(1, kw, 1)                          # [B,T,kw]
    return cols @ k[:, 0, :] + b                       # [B,T,F]


def forward(W, memory, lengths, targets, prenet_masks, zoneout_masks=None, zoneout=0.1, feed_target=None,
            smoothing=False):
    """Teacher-forced decoder forward.  W: dict name -> torch tensor (requires_grad as wanted);
    memory [B,T_in,D]; lengths [B]; targets [B,T·r,80] with r = outputs_per_step (the width of the
    stop projection, tacotron.py:322-324); prenet_masks [T,2,B,P] keep bits per decoder step;
    zoneout_masks [T,4,B,H] keep bits (c1,h1,c2,h2; training zoneout) or None (inference mix);
    feed_target [T] (None = all 1): the outcome of TacoTrainingHelper.next_inputs' per-step draw
    u < ratio (helpers.py:122-133) -- step t (t >= 1) gets the target frame t·r-1 when 1
    (targets[:, r-1::r], helpers.py:78), else the last of the decoder's own unclipped r frames of
    step t-1 (outputs[:, -output_dim:], helpers.py:129), through which gradients flow.
    smoothing: hp.smoothing (attention.py:71-91,150), a = sigmoid(e) / sum sigmoid(e) over the
    unmasked positions (sigmoid(-inf) = 0) instead of the softmax.
    Returns frames [B,T·r,80], stop logits [B,T·r] (the reshapes of tacotron.py:355-358),
    alignments [B,T_in,T]."""
    B, T_in, D = memory.shape
    nm = targets.shape[2]
    r = W[SP + "bias"].shape[0]
    assert targets.shape[1] % r == 0, "targets must hold a multiple of outputs_per_step frames"
    T = targets.shape[1] // r
    dt = memory.dtype
    mask = (torch.arange(T_in)[None, :] < torch.as_tensor(lengths)[:, None]).to(dt)
    values = memory * mask[:, :, None]                                  # BahdanauAttention memory
    keys = values @ W[P + "memory_layer/kernel"]                        # memory_layer, no bias
    H = W[L1 + "bias"].shape[0] // 4
    c1 = h1 = c2 = h2 = torch.zeros(B, H, dtype=dt)
    ctx = torch.zeros(B, D, dtype=dt)
    cum = torch.zeros(B, T_in, dtype=dt)
    frame_in = torch.zeros(B, targets.shape[2], dtype=dt)               # _go_frames helpers.py:136
    big_neg = torch.tensor(float("-inf"), dtype=dt)
    frames, stops, aligns = [], [], []

    def cell(x, c, h, k, b, mc, mh):
        z = torch.cat([x, h], 1) @ k + b
        i, j, f, o = z.chunk(4, 1)
        cn = torch.sigmoid(f + 1.0) * c + torch.sigmoid(i) * torch.tanh(j)
        hn = torch.sigmoid(o) * torch.tanh(cn)
        if mc is None:
            return hn, (1 - zoneout) * cn + zoneout * c, (1 - zoneout) * hn + zoneout * h
        return hn, c + mc * (cn - c), h + mh * (hn - h)

    for t in range(T):
        x = frame_in
        for i in range(2):
            s = P + "decoder/decoder_prenet/dense_{}/".format(i + 1)
            x = torch.relu(x @ W[s + "kernel"] + W[s + "bias"]) / 0.5 * prenet_masks[t, i]
        zm = [None] * 4 if zoneout_masks is None else [zoneout_masks[t, q] for q in range(4)]
        o1, c1, h1 = cell(torch.cat([x, ctx], 1), c1, h1, W[L1 + "kernel"], W[L1 + "bias"],
                          zm[0], zm[1])
        o2, c2, h2 = cell(o1, c2, h2, W[L2 + "kernel"], W[L2 + "bias"], zm[2], zm[3])
        q = o2 @ W[P + "decoder/query_layer/kernel"]
        f = _conv_same(cum, W[LA + "location_features_convolution/kernel"],
                       W[LA + "location_features_convolution/bias"])
        loc = f @ W[LA + "location_features_layer/kernel"]
        e = (W[LA + "attention_variable_projection"]
             * torch.tanh(keys + q[:, None, :] + loc + W[LA + "attention_bias"])).sum(2)
        e = torch.where(mask > 0, e, big_neg)
        if smoothing:
            sg = torch.sigmoid(e)
            a = sg / sg.sum(1, keepdim=True)
        else:
            a = torch.softmax(e, 1)
        cum = cum + a
        ctx = (a[:, :, None] * values).sum(1)
        pin = torch.cat([o2, ctx], 1)
        frames.append(pin @ W[FP + "kernel"] + W[FP + "bias"])      # [B, nm·r]
        stops.append(pin @ W[SP + "kernel"] + W[SP + "bias"])       # [B, r]
        aligns.append(a)
        if feed_target is None or t + 1 >= T or feed_target[t + 1]:
            frame_in = targets[:, t * r + r - 1]
        else:
            frame_in = frames[-1][:, -nm:]
    return (torch.stack(frames, 1).reshape(B, T * r, nm), torch.stack(stops, 1).reshape(B, T * r),
            torch.stack(aligns, 2))


def clip_decoder_output(frames, clip=(-4.1, 4.0)):
    """tacotron.py:360-361: decoder_output = min(max(frames, lo - lower_bound_decay), hi) when
    clip_outputs (T2_output_range = (-max_abs_value, max_abs_value) for symmetric mels)."""
    return frames if clip is None else torch.clamp(frames, clip[0], clip[1])


def masked_mse(targets, outputs, target_lengths):
    """MaskedMSE (modules.py:532-551): tf.losses.mean_squared_error with weights = the [B,T,1]
    sequence mask broadcast over the mels, reduced SUM_BY_NONZERO_WEIGHTS."""
    T = targets.shape[1]
    w = (torch.arange(T)[None, :] < torch.as_tensor(target_lengths)[:, None]).to(targets.dtype)
    w = w[:, :, None].expand_as(targets)
    return (w * (outputs - targets) ** 2).sum() / (w != 0).sum()


def masked_stop_loss(stop_targets, logits, target_lengths, pos_weight):
    """MaskedSigmoidCrossEntropy (modules.py:553-575): TF weighted_cross_entropy_with_logits
    (1-z)x + (1+(q-1)z)(log1p(exp(-|x|)) + max(-x,0)), masked, summed, divided by the count of
    nonzero masked losses."""
    T = logits.shape[1]
    w = (torch.arange(T)[None, :] < torch.as_tensor(target_lengths)[:, None]).to(logits.dtype)
    x, z = logits, stop_targets
    l = 1 + (pos_weight - 1) * z
    v = w * ((1 - z) * x + l * (torch.log1p(torch.exp(-x.abs())) + torch.clamp(-x, min=0)))
    return v.sum() / (v != 0).sum()


def losses(frames, stop_logits, targets, stop_targets, W, reg_weight, clip=(-4.1, 4.0),
           target_lengths=None, pos_weight=1.0):
    """before (tf.losses.mean_squared_error on the clipped decoder output), stop (mean sigmoid
    CE: the unmasked path ignores pos_weight, tacotron.py:778-779), reg; target_lengths given =
    mask_decoder (tacotron.py:758-767)."""
    if target_lengths is not None:
        before = masked_mse(targets, clip_decoder_output(frames, clip), target_lengths)
        stop = masked_stop_loss(stop_targets, stop_logits, target_lengths, pos_weight)
    else:
        before = ((clip_decoder_output(frames, clip) - targets) ** 2).mean()
        x, z = stop_logits, stop_targets
        stop = (torch.clamp(x, min=0) - x * z + torch.log1p(torch.exp(-x.abs()))).mean()
    reg = sum((v ** 2).sum() / 2 for n, v in W.items() if regularized(n)) * reg_weight
    return before, stop, reg


def postnet_train(W, dec, masks, eps=1e-3, layers=5):
    """Postnet in training mode (modules.py:474-497, conv1d with bnorm='after'): per layer
    conv1d 'same' + tanh (identity for the last), batch normalisation with the BATCH statistics
    over all B·T positions (tf.layers.batch_normalization(training=True); biased variance),
    dropout(rate 0.5) with keep bits ``masks [layers, B, T, C]`` (None = no dropout); then
    postnet_projection (tacotron.py:368-372).  Returns (projected residual, [(mean, var)])."""
    x = dec
    stats = []
    for i in range(1, layers + 1):
        s = PN.format(i)
        k = W[s + "conv1d/kernel"]                                       # [kw, Cin, C]
        kw = k.shape[0]
        pad = (kw - 1) // 2
        xp = torch.nn.functional.pad(x, (0, 0, pad, kw - 1 - pad))      # [B, T+kw-1, Cin]
        cols = xp.unfold(1, kw, 1)                                       # [B, T, Cin, kw]
        z = torch.einsum("btck,kcn->btn", cols, k) + W[s + "conv1d/bias"]
        a = torch.tanh(z) if i < layers else z
        mean = a.mean(dim=(0, 1))
        var = ((a - mean) ** 2).mean(dim=(0, 1))
        stats.append((mean, var))
        y = (W[s + "batch_normalization/gamma"] * (a - mean) / torch.sqrt(var + eps)
             + W[s + "batch_normalization/beta"])
        x = y if masks is None else y / 0.5 * masks[i - 1]
    return x @ W[PP + "kernel"] + W[PP + "bias"], stats


# ---- front end: encoder + reference encoders + GST in training mode ----------

EC = P + "encoder_convolutions/conv_layer_{}_encoder_convolutions/"
EL = P + "encoder_LSTM/bidirectional_rnn/{}/lstm_cell/"
RN = P + "refnet_{}/"
MH = P + "Multihead-attention-{}/"


def frontend_var_names(emt_only=False, conv_layers=3, ref_layers=6, use_gst=True, adain=False):
    """Trainable front-end variables (tacotron.py:215-308, modules.py:9-64,251-323,
    multihead_attention.py:35-132), in the library's flat-buffer order.  use_gst=False: no style
    tokens / style attention (tacotron.py:284-291).  adain: ReferenceEncoderAdaIn's 'refnet'
    (modules.py:66-107): per layer the speaker conv (conv2d_i/conv2d) and the emotion conv
    (conv2d_i/conv2d_1, tf.layers' uniquified default name), no batch norm, one GRU + dense."""
    names = [P + "inputs_embedding"]
    for i in range(1, conv_layers + 1):
        s = EC.format(i)
        names += [s + "conv1d/kernel", s + "conv1d/bias", s + "batch_normalization/gamma",
                  s + "batch_normalization/beta"]
    for d in ("fw", "bw"):
        names += [EL.format(d) + "kernel", EL.format(d) + "bias"]
    if adain:
        r = P + "refnet/"
        for i in range(ref_layers):
            for ly in ("conv2d", "conv2d_1"):
                names += [r + "conv2d_{}/{}/kernel".format(i, ly), r + "conv2d_{}/{}/bias".format(i, ly)]
        return names + [r + "rnn/gru_cell/gates/kernel", r + "rnn/gru_cell/gates/bias",
                        r + "rnn/gru_cell/candidate/kernel", r + "rnn/gru_cell/candidate/bias",
                        r + "dense/kernel", r + "dense/bias"]
    for tag in (("emt",) if emt_only else ("emt", "spk")):
        r = RN.format(tag)
        for i in range(ref_layers):
            s = r + "conv2d_{}/".format(i)
            names += [s + "conv2d/kernel", s + "conv2d/bias", s + "batch_normalization/gamma",
                      s + "batch_normalization/beta"]
        names += [r + "rnn/gru_cell/gates/kernel", r + "rnn/gru_cell/gates/bias",
                  r + "rnn/gru_cell/candidate/kernel", r + "rnn/gru_cell/candidate/bias",
                  r + "dense/kernel", r + "dense/bias"]
        if not use_gst:
            continue
        names += [P + "style_tokens_" + tag]
        m = MH.format(tag)
        names += [m + "conv1d/kernel", m + "conv1d/bias", m + "conv1d_1/kernel", m + "conv1d_1/bias",
                  m + "attention_v", m + "attention_g", m + "attention_b"]
    return names


def _bn_train(a, gamma, beta, dims, eps=1e-3, moving=None):
    """tf.layers.batch_normalization(training=True): batch statistics over ``dims`` (biased);
    ``moving`` = (moving_mean, moving_variance) evaluates it in inference mode instead."""
    if moving is not None:
        mean, var = moving
    else:
        mean = a.mean(dim=dims)
        var = ((a - mean) ** 2).mean(dim=dims)
    return gamma * (a - mean) / torch.sqrt(var + eps) + beta, (mean, var)


def _conv2d_same_s2(x, k, b, st=2):
    """tf.layers.conv2d 3x3 stride st (2 by default) padding='same' NHWC (odd pad bottom/right)."""
    N, H, Wd, C = x.shape
    outs = []
    pads = []
    for n, kk in ((H, k.shape[0]), (Wd, k.shape[1])):
        o = -(-n // st)
        tot = max((o - 1) * st + kk - n, 0)
        pads.append((tot // 2, tot - tot // 2))
    xp = torch.nn.functional.pad(x, (0, 0, pads[1][0], pads[1][1], pads[0][0], pads[0][1]))
    Ho, Wo = -(-H // st), -(-Wd // st)
    cols = []
    for i in range(k.shape[0]):
        for j in range(k.shape[1]):
            cols.append(xp[:, i:i + (Ho - 1) * st + 1:st, j:j + (Wo - 1) * st + 1:st, :])
    cols = torch.cat(cols, -1)
    return cols @ k.reshape(-1, k.shape[3]) + b


def _lstm_dir(x, lengths, k, b, masks, reverse):
    """One direction of bidirectional_dynamic_rnn (modules.py:315-321) with training zoneout:
    c = c_prev + m_c·(c_new - c_prev), h likewise (modules.py:236-240), emitted output h_new; past a
    row's length output 0 and state copied; the backward direction runs on the length-reversed
    sequence.  masks [T, 2 (c, h), B, U] keep bits by recurrence step, or None (inference mix)."""
    B, T, _ = x.shape
    U = b.shape[0] // 4
    dt = x.dtype
    c = h = torch.zeros(B, U, dtype=dt)
    lens = torch.as_tensor(np.asarray(lengths))
    out = [None] * T
    for t in range(T):
        act = (t < lens)[:, None].to(dt)
        if reverse:
            pos = torch.clamp(lens - 1 - t, min=0)
            xt = x[torch.arange(B), pos]
        else:
            xt = x[:, t]
        z = torch.cat([xt, h], 1) @ k + b
        i, j, f, o = z.chunk(4, 1)
        cn = torch.sigmoid(f + 1.0) * c + torch.sigmoid(i) * torch.tanh(j)
        hn = torch.sigmoid(o) * torch.tanh(cn)
        if masks is None:
            c2, h2 = 0.9 * cn + 0.1 * c, 0.9 * hn + 0.1 * h
        else:
            c2, h2 = c + masks[t, 0] * (cn - c), h + masks[t, 1] * (hn - h)
        out[t] = hn * act
        c = act * c2 + (1 - act) * c
        h = act * h2 + (1 - act) * h
    o = torch.stack(out, 1)                                   # step-major
    if not reverse:
        return o
    rows = []
    for bi in range(B):                                       # back to position order
        L = int(lens[bi])
        rows.append(torch.cat([o[bi, :L].flip(0), o[bi, L:]], 0))
    return torch.stack(rows, 0)


def _gru_last(x, W, r):
    kg, bg = W[r + "rnn/gru_cell/gates/kernel"], W[r + "rnn/gru_cell/gates/bias"]
    kc, bc = W[r + "rnn/gru_cell/candidate/kernel"], W[r + "rnn/gru_cell/candidate/bias"]
    N, T2, _ = x.shape
    D = bc.shape[0]
    h = torch.zeros(N, D, dtype=x.dtype)
    for t in range(T2):
        v = torch.sigmoid(torch.cat([x[:, t], h], 1) @ kg + bg)
        rr, u = v[:, :D], v[:, D:]
        cc = torch.tanh(torch.cat([x[:, t], rr * h], 1) @ kc + bc)
        h = u * h + (1 - u) * cc
    return h


def _gst(ref, W, tag, heads=4):
    m = MH.format(tag)
    tok = torch.tanh(W[P + "style_tokens_" + tag])              # [10, 64]
    q = ref @ W[m + "conv1d/kernel"][0] + W[m + "conv1d/bias"]
    kk = tok @ W[m + "conv1d_1/kernel"][0] + W[m + "conv1d_1/bias"]
    N, A = q.shape
    d = A // heads
    v, g, bb = W[m + "attention_v"], W[m + "attention_g"], W[m + "attention_b"]
    nv = g * v / torch.sqrt((v ** 2).sum())
    qs = q.reshape(N, heads, 1, d)
    ks = kk.reshape(1, -1, heads, d).permute(0, 2, 1, 3)
    s = (nv * torch.tanh(ks + qs + bb)).sum(-1)                   # [N, H, 10]
    w = torch.softmax(s, -1)
    return (w @ tok).reshape(N, -1)


def _adain_refnet(W, ref_spk, ref_emt, dt):
    """ReferenceEncoderAdaIn (modules.py:75-107) with strides (2,2),(2,2),(1,1)x4 (tacotron.py:237):
    speaker and emotion stacks of conv2d + ReLU without batch norm (conv2d_i/conv2d, conv2d_i/conv2d_1),
    per (row, channel) moments over (time, freq) (tf.nn.moments: biased variance), speaker map
    0.9 x + 0.1 tf.nn.batch_normalization(x, m_s, v_s, offset=m_e, scale=v_e, 1e-9), GRU over every
    frame, last output -> Dense(128, tanh)."""
    r = P + "refnet/"
    strides = (2, 2, 1, 1, 1, 1)
    hs = [torch.as_tensor(np.asarray(m), dtype=dt)[..., None] for m in (ref_spk, ref_emt)]
    for i in range(6):
        s = r + "conv2d_{}/".format(i)
        hs = [torch.relu(_conv2d_same_s2(h, W[s + ly + "/kernel"], W[s + ly + "/bias"], strides[i]))
              for h, ly in zip(hs, ("conv2d", "conv2d_1"))]
    spk, emt = hs
    m_s = spk.mean(dim=(1, 2), keepdim=True)
    v_s = ((spk - m_s) ** 2).mean(dim=(1, 2), keepdim=True)
    m_e = emt.mean(dim=(1, 2), keepdim=True)
    v_e = ((emt - m_e) ** 2).mean(dim=(1, 2), keepdim=True)
    inv = v_e / torch.sqrt(v_s + 1e-9)
    x = spk * 0.9 + (spk * inv + (m_e - m_s * inv)) * 0.1
    N, T2, F2, C = x.shape
    hl = _gru_last(x.reshape(N, T2, F2 * C), W, r)
    return torch.tanh(hl @ W[r + "dense/kernel"] + W[r + "dense/bias"])


def frontend_forward(W, ids, lengths, ref_emt, ref_spk, enc_masks=None, enc_zm=None, emt_only=False,
                     eps=1e-3, moving=None, refs_out=None, use_gst=True, adain=False):
    """Training-mode front end -> memory [B,T_in,D] (unmasked: the decoder masks it) and the batch
    statistics [(mean, var)] of every batch norm (encoder convs, then refnet convs).
    enc_masks [3, B, T_in, C] conv dropout keep bits (rate 0.5) or None; enc_zm [T_in, 2 (fw, bw),
    2 (c, h), B, U] LSTM zoneout keep bits or None.  ``moving`` (dict name -> array) evaluates the
    batch norms with the moving statistics: with no masks that is the inference graph, pinned to
    oracle/tacotron_ref.py (tests/test_train.py).  ``refs_out`` (a list) receives the reference
    encoders' outputs refnet_outputs_emt / _spk [B, 128] (tacotron.py:260-261).  use_gst=False:
    those outputs are the style embeddings themselves (tacotron.py:284-291)."""
    def mv(scope):
        if moving is None:
            return None
        return tuple(torch.as_tensor(np.asarray(moving[scope + "batch_normalization/" + n]), dtype=dt)
                     for n in ("moving_mean", "moving_variance"))
    dt = W[P + "inputs_embedding"].dtype
    x = W[P + "inputs_embedding"][torch.as_tensor(np.asarray(ids)).long()]
    stats = []
    for i in range(1, 4):                        # modules.py:485-497, bnorm 'after': conv->relu->BN->dropout
        s = EC.format(i)
        k = W[s + "conv1d/kernel"]
        kw = k.shape[0]
        pad = (kw - 1) // 2
        xp = torch.nn.functional.pad(x, (0, 0, pad, kw - 1 - pad))
        a = torch.relu(torch.einsum("btck,kcn->btn", xp.unfold(1, kw, 1), k) + W[s + "conv1d/bias"])
        y, st = _bn_train(a, W[s + "batch_normalization/gamma"], W[s + "batch_normalization/beta"],
                          (0, 1), eps, mv(s))
        stats.append(st)
        x = y if enc_masks is None else y / 0.5 * torch.as_tensor(np.asarray(enc_masks[i - 1]), dtype=dt)
    zm = None if enc_zm is None else torch.as_tensor(np.asarray(enc_zm), dtype=dt)
    fw = _lstm_dir(x, lengths, W[EL.format("fw") + "kernel"], W[EL.format("fw") + "bias"],
                   None if zm is None else zm[:, 0], False)
    bw = _lstm_dir(x, lengths, W[EL.format("bw") + "kernel"], W[EL.format("bw") + "bias"],
                   None if zm is None else zm[:, 1], True)
    parts = [fw, bw]
    B, T = x.shape[:2]
    if adain:  # the speaker embedding of the AdaIN encoder is the style embedding (tacotron.py:266-268)
        refo = _adain_refnet(W, ref_spk, ref_emt, dt)
        if refs_out is not None:
            refs_out.append(refo)
        parts.append(refo[:, None, :].expand(B, T, refo.shape[1]))
        return torch.cat(parts, -1), stats
    for tag, ref in (("emt", ref_emt),) + ((() if emt_only else (("spk", ref_spk),))):
        r = RN.format(tag)
        h = torch.as_tensor(np.asarray(ref), dtype=dt)[..., None]
        for i in range(6):                       # conv2d(): conv -> BN (training) -> ReLU
            s = r + "conv2d_{}/".format(i)
            a = _conv2d_same_s2(h, W[s + "conv2d/kernel"], W[s + "conv2d/bias"])
            y, st = _bn_train(a, W[s + "batch_normalization/gamma"],
                              W[s + "batch_normalization/beta"], (0, 1, 2), eps, mv(s))
            stats.append(st)
            h = torch.relu(y)
        N, T2, F2, C = h.shape
        hl = _gru_last(h.reshape(N, T2, F2 * C), W, r)
        refo = torch.tanh(hl @ W[r + "dense/kernel"] + W[r + "dense/bias"])
        if refs_out is not None:
            refs_out.append(refo)
        style = _gst(refo, W, tag) if use_gst else refo
        parts.append(style[:, None, :].expand(B, T, style.shape[1]))
    return torch.cat(parts, -1), stats


def style_disc_var_names(emt_only=False, n_emt=0, n_spk=0):
    """Style_Emb_Disc dense layers (modules.py:626-644 under scopes style_disc_emt / _spk,
    tacotron.py:489-493): built when n_emt (n_spk, unless emt_only) classes are given."""
    names = []
    for tag, n in (("emt", n_emt),) + ((() if emt_only else (("spk", n_spk),))):
        if n:
            names += [P + "style_disc_{}/dense/kernel".format(tag), P + "style_disc_{}/dense/bias".format(tag)]
    return names


def style_emb_losses(W, refs, emt_labels, spk_labels, n_emt=0, n_spk=0, orthog_weight=0.0):
    """The style-embedding losses of the default (GST, not adain / pretrained_emb_disc_all)
    training graph (tacotron.py:812-820, 840-846): per reference encoder a dense classifier of
    its output and tf.nn.softmax_cross_entropy_with_logits against tf.one_hot(labels) (an
    out-of-range label is a zero row: loss 0, gradient 0), averaged over the batch; the
    orthogonality loss orthog_weight * ||refnet_emt · refnet_spkᵀ||_F (Frobenius; 0.02 in the
    reference, off for emt_only).  Returns (loss_emt, loss_spk, loss_orthog) tensors."""
    out = []
    for i, (tag, lab, n) in enumerate((("emt", emt_labels, n_emt), ("spk", spk_labels, n_spk))):
        if not n or i >= len(refs):
            out.append(torch.zeros((), dtype=refs[0].dtype))
            continue
        logit = refs[i] @ W[P + "style_disc_{}/dense/kernel".format(tag)] + W[P + "style_disc_{}/dense/bias".format(tag)]
        lab = np.asarray(lab).astype(np.int64)
        y = torch.zeros_like(logit)
        ok = (lab >= 0) & (lab < n)
        y[np.nonzero(ok)[0], lab[ok]] = 1.0
        out.append((-(y * torch.log_softmax(logit, -1)).sum(-1)).mean())
    if orthog_weight and len(refs) > 1:
        out.append(orthog_weight * torch.linalg.norm(refs[0] @ refs[1].T))
    else:
        out.append(torch.zeros((), dtype=refs[0].dtype))
    return tuple(out)


def train_grads_frontend(Wnp, ids, lengths, ref_emt, ref_spk, targets, stop_targets, prenet_masks,
                         zoneout_masks, enc_masks, enc_zm, reg_weight=1e-6, dtype=torch.float64,
                         clip=(-4.1, 4.0), postnet_masks=None, emt_only=False, style=None, use_gst=True,
                         adain=False):
    """The whole configs[4] step: front end (training mode) -> memory -> decoder + Postnet; returns
    (losses, grads of every front-end, decoder and Postnet variable, [(mean, var)] batch stats of
    the front end's batch norms).  ``style`` = dict(emt_labels, spk_labels, n_emt, n_spk,
    orthog_weight) adds the style-embedding losses (style_emb_losses); the losses tuple then
    gains (loss_emt, loss_spk, loss_orthog)."""
    st_kw = dict(style or {})
    names = (frontend_var_names(emt_only, use_gst=use_gst, adain=adain) + style_disc_var_names(emt_only, st_kw.get("n_emt", 0), st_kw.get("n_spk", 0))
             + train_var_names() + postnet_var_names())
    W = {n: torch.tensor(np.asarray(Wnp[n]), dtype=dtype, requires_grad=True) for n in names}
    refs = []
    mem, stats = frontend_forward(W, ids, lengths, ref_emt, ref_spk, enc_masks, enc_zm, emt_only, refs_out=refs,
                                  use_gst=use_gst, adain=adain)
    tg = torch.tensor(np.asarray(targets), dtype=dtype)
    st = torch.tensor(np.asarray(stop_targets), dtype=dtype)
    pm = torch.tensor(np.asarray(prenet_masks), dtype=dtype)
    zm = None if zoneout_masks is None else torch.tensor(np.asarray(zoneout_masks), dtype=dtype)
    fr, sl, al = forward(W, mem, lengths, tg, pm, zm)
    b, s, r = losses(fr, sl, tg, st, W, reg_weight, clip)
    dec = clip_decoder_output(fr, clip)
    pmk = None if postnet_masks is None else torch.tensor(np.asarray(postnet_masks), dtype=dtype)
    proj, _ = postnet_train(W, dec, pmk)
    mel = clip_decoder_output(dec + proj, clip)
    after = ((mel - tg) ** 2).mean()
    total = b + s + r + after
    extra = ()
    if style is not None:
        extra = style_emb_losses(W, refs, st_kw.get("emt_labels"), st_kw.get("spk_labels"), st_kw.get("n_emt", 0),
                                 0 if emt_only else st_kw.get("n_spk", 0),
                                 0.0 if emt_only else st_kw.get("orthog_weight", 0.0))
        total = total + sum(extra)
    total.backward()
    g = {n: W[n].grad.numpy() for n in names}
    return (b.item(), s.item(), r.item(), after.item()) + tuple(x.item() for x in extra), g, \
        [(m.detach().numpy(), v.detach().numpy()) for m, v in stats]


def train_grads(Wnp, memory, lengths, targets, stop_targets, prenet_masks, zoneout_masks,
                reg_weight=1e-6, dtype=torch.float64, clip=(-4.1, 4.0), postnet=False,
                postnet_masks=None, feed_target=None, target_lengths=None, pos_weight=1.0, smoothing=False):
    """One forward + backward; returns (outputs dict, losses tuple, grads dict incl. 'memory').
    postnet=True adds the Postnet and the ``after`` loss (tacotron.py:362-381, 775-776): losses
    become (before, stop, reg, after) and outputs gain 'mel_outputs' and 'bn_stats'.
    feed_target: teacher-forcing draw (forward); target_lengths: mask_decoder losses."""
    names = train_var_names() + (postnet_var_names() if postnet else [])
    W = {n: torch.tensor(np.asarray(Wnp[n]), dtype=dtype, requires_grad=True) for n in names}
    mem = torch.tensor(np.asarray(memory), dtype=dtype, requires_grad=True)
    tg = torch.tensor(np.asarray(targets), dtype=dtype)
    st = torch.tensor(np.asarray(stop_targets), dtype=dtype)
    pm = torch.tensor(np.asarray(prenet_masks), dtype=dtype)
    zm = None if zoneout_masks is None else torch.tensor(np.asarray(zoneout_masks), dtype=dtype)
    fr, sl, al = forward(W, mem, lengths, tg, pm, zm, feed_target=feed_target, smoothing=smoothing)
    b, s, r = losses(fr, sl, tg, st, W, reg_weight, clip, target_lengths, pos_weight)
    total = b + s + r
    out = dict(frames=clip_decoder_output(fr, clip).detach().numpy(), stop_logits=sl.detach().numpy(),
               alignments=al.detach().numpy())
    if postnet:
        dec = clip_decoder_output(fr, clip)
        pmk = None if postnet_masks is None else torch.tensor(np.asarray(postnet_masks), dtype=dtype)
        proj, stats = postnet_train(W, dec, pmk)
        mel = clip_decoder_output(dec + proj, clip)                      # tacotron.py:375-378
        after = ((mel - tg) ** 2).mean() if target_lengths is None else masked_mse(tg, mel, target_lengths)
        total = total + after
        out["mel_outputs"] = mel.detach().numpy()
        out["bn_stats"] = [(m.detach().numpy(), v.detach().numpy()) for m, v in stats]
    total.backward()
    g = {n: W[n].grad.numpy() for n in names}
    g["memory"] = mem.grad.numpy()
    L = (b.item(), s.item(), r.item()) + ((after.item(),) if postnet else ())
    return out, L, g


def bn_moving_update(moving, batch, momentum=0.99):
    """tf.layers.batch_normalization UPDATE_OPS (run with the optimizer, tacotron.py:1088-1090):
    moving -= (moving - batch)·(1 - momentum)."""
    return moving - (moving - batch) * (1 - momentum)


def teacher_forcing_ratio(global_step, hp):
    """TacoTrainingHelper's ratio (helpers.py:65,113-118,140-180): constant mode ->
    tacotron_teacher_forcing_ratio; scheduled -> init before start_decay, else
    exponential_decay(init, gs - start_decay, decay_steps, decay_exp_rate) (not staircase)."""
    if hp.tacotron_teacher_forcing_mode != "scheduled":
        return float(hp.tacotron_teacher_forcing_ratio)
    init = hp.tacotron_teacher_forcing_init_ratio
    if global_step < hp.tacotron_teacher_forcing_start_decay:
        return float(init)
    return float(init * hp.tacotron_teacher_forcing_decay_exp_rate ** (
        (global_step - hp.tacotron_teacher_forcing_start_decay) / hp.tacotron_teacher_forcing_decay_steps))


def learning_rate(step, hp):
    """Tacotron._learning_rate_decay (tacotron.py:1227-1251): exponential_decay from
    tacotron_start_decay, clipped to [final, initial]."""
    init = hp.tacotron_initial_learning_rate
    lr = init * hp.tacotron_decay_rate ** ((step - hp.tacotron_start_decay) / hp.tacotron_decay_steps)
    return min(max(lr, hp.tacotron_final_learning_rate), init)


def clip_and_adam(params, grads, m, v, step, lr, beta1=0.9, beta2=0.999, eps=1e-6, clip=1.0):
    """tf.clip_by_global_norm(grads, 1.) then tf.train.AdamOptimizer.apply_gradients (step =
    the post-increment count t >= 1): lr_t = lr·sqrt(1-b2^t)/(1-b1^t); m,v moments; w -= lr_t·m/
    (sqrt(v)+eps).  Mutates params/m/v (dicts of float64 numpy arrays); returns the global norm."""
    gn = float(np.sqrt(sum(float((np.asarray(g, np.float64) ** 2).sum()) for g in grads.values())))
    scale = clip / max(gn, clip)
    lr_t = lr * np.sqrt(1 - beta2 ** step) / (1 - beta1 ** step)
    for n in params:
        g = np.asarray(grads[n], np.float64) * scale
        m[n] = beta1 * m[n] + (1 - beta1) * g
        v[n] = beta2 * v[n] + (1 - beta2) * g * g
        params[n] = params[n] - lr_t * m[n] / (np.sqrt(v[n]) + eps)
    return gn
