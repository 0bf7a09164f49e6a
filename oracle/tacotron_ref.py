"""TEST INFRASTRUCTURE ONLY — numpy restatement of the Tacotron-2 inference path of
mwhitehill/Tacotron-2 (see ``oracle/__init__.py``: parity unpinned, never imported by the product).

Every function cites the reference line it restates (paths relative to the reference's ``code/``).
Arithmetic defaults to float32 (the reference's dtype); pass ``dt=np.float64`` for a
high-precision cross-check.  Weights are a ``dict`` keyed by the canonical TF variable names
produced by ``tt2.weights.tacotron_weight_specs`` (prefix ``Tacotron_model/inference/``).
"""
import numpy as np

P = "Tacotron_model/inference/"


def _w(W, name, dt):
    return np.asarray(W[P + name], dtype=dt)


def sigmoid(x):
    with np.errstate(over="ignore"):
        return (1.0 / (1.0 + np.exp(-x))).astype(x.dtype)


def dense(x, k, b=None):
    """tf.layers.dense: matmul + bias_add (activation applied by caller)."""
    y = x @ k
    return y if b is None else y + b


def conv1d_same(x, k, b=None):
    """tf.layers.conv1d(padding='same', stride 1): x [B,T,Cin], k [kw,Cin,Cout].

    'same' pads floor((kw-1)/2) on the left (TF Conv1D geometry), used by modules.py:488-493 and
    the location convolution attention.py:160-162."""
    B, T, C = x.shape
    kw = k.shape[0]
    pl = (kw - 1) // 2
    pr = kw - 1 - pl
    xp = np.pad(x, ((0, 0), (pl, pr), (0, 0)))
    cols = np.concatenate([xp[:, i:i + T, :] for i in range(kw)], axis=-1)  # [B,T,kw*C]
    y = cols @ k.reshape(kw * C, -1)
    return y if b is None else y + b


def batch_norm(x, W, scope, dt, eps=1e-3):
    """tf.layers.batch_normalization(training=False) (modules.py:494, 508): moving statistics,
    computed as TF's nn.batch_normalization: x*inv + (beta - mean*inv), inv = gamma*rsqrt(var+eps)."""
    g = _w(W, scope + "batch_normalization/gamma", dt)
    be = _w(W, scope + "batch_normalization/beta", dt)
    m = _w(W, scope + "batch_normalization/moving_mean", dt)
    v = _w(W, scope + "batch_normalization/moving_variance", dt)
    inv = (g / np.sqrt(v + dt(eps))).astype(dt)
    return x * inv + (be - m * inv)


def conv1d_block(x, W, scope, act, dt):
    """modules.py:485-497 conv1d() with bnorm='after': activation inside the conv, then BN;
    dropout is identity at inference (training=False)."""
    y = conv1d_same(x, _w(W, scope + "conv1d/kernel", dt), _w(W, scope + "conv1d/bias", dt))
    y = act(y)
    return batch_norm(y, W, scope, dt)


def lstm_cell(x, c_prev, h_prev, k, b, forget_bias=1.0):
    """TF1 tf.nn.rnn_cell.LSTMCell (used at modules.py:206): gates [i,j,f,o] =
    split([x,h]·W + b); c = σ(f+forget_bias)·c + σ(i)·tanh(j); h = σ(o)·tanh(c)."""
    dt = x.dtype.type
    z = np.concatenate([x, h_prev], axis=-1) @ k + b
    n = c_prev.shape[-1]
    i, j, f, o = z[:, :n], z[:, n:2 * n], z[:, 2 * n:3 * n], z[:, 3 * n:]
    c = sigmoid(f + dt(forget_bias)) * c_prev + sigmoid(i) * np.tanh(j)
    h = sigmoid(o) * np.tanh(c)
    return c, h


def zoneout_lstm(x, c_prev, h_prev, k, b, zoneout):
    """ZoneoutLSTMCell.__call__ at inference (modules.py:220-248): the emitted output is the raw
    LSTMCell output (h_new), the carried state is the zoneout mix (modules.py:243-244)."""
    dt = x.dtype.type
    c_new, h_new = lstm_cell(x, c_prev, h_prev, k, b)
    z = dt(zoneout)
    one_m_z = dt(1.0 - zoneout)
    c = one_m_z * c_new + z * c_prev
    h = one_m_z * h_new + z * h_prev
    return h_new, c, h


def embedding(ids, W, dt):
    """tacotron.py:215-217 embedding_lookup on the [66, 512] table."""
    return _w(W, "inputs_embedding", dt)[ids]


def encoder(ids, lengths, W, hp, dt=np.float32):
    """TacotronEncoderCell (Architecture_wrappers.py:36-45): EncoderConvolutions
    (modules.py:274-280) then EncoderRNN bidirectional Zoneout-LSTM (modules.py:313-323)."""
    x = embedding(ids, W, dt)
    relu = lambda v: np.maximum(v, dt(0))
    for i in range(1, 4):
        x = conv1d_block(x, W, "encoder_convolutions/conv_layer_{}_encoder_convolutions/".format(i),
                         relu, dt)
    return bidirectional_lstm(x, lengths, W, "encoder_LSTM/bidirectional_rnn/", hp["zoneout"], dt)


def _dynamic_zoneout_lstm(x, lengths, k, b, zoneout):
    """tf.nn.dynamic_rnn with sequence_length: past a row's length the output is 0 and the state
    is copied through (TF rnn._rnn_step)."""
    B, T, _ = x.shape
    n = b.shape[0] // 4
    dt = x.dtype.type
    c = np.zeros((B, n), dt)
    h = np.zeros((B, n), dt)
    out = np.zeros((B, T, n), dt)
    for t in range(T):
        act = (t < lengths)[:, None]
        o, c2, h2 = zoneout_lstm(x[:, t], c, h, k, b, zoneout)
        out[:, t] = np.where(act, o, dt(0))
        c = np.where(act, c2, c)
        h = np.where(act, h2, h)
    return out


def _reverse_sequence(x, lengths):
    """tf.reverse_sequence(seq_axis=1): reverse each row's first `len` steps, keep the tail."""
    y = x.copy()
    for bi, L in enumerate(lengths):
        y[bi, :L] = x[bi, :L][::-1]
    return y


def bidirectional_lstm(x, lengths, W, scope, zoneout, dt):
    """tf.nn.bidirectional_dynamic_rnn (modules.py:315-321): bw runs on the length-reversed input
    and its outputs are reversed back; outputs concatenated [fw, bw] (modules.py:323)."""
    lengths = np.asarray(lengths)
    kf = _w(W, scope + "fw/lstm_cell/kernel", dt)
    bf = _w(W, scope + "fw/lstm_cell/bias", dt)
    kb = _w(W, scope + "bw/lstm_cell/kernel", dt)
    bb = _w(W, scope + "bw/lstm_cell/bias", dt)
    fw = _dynamic_zoneout_lstm(x, lengths, kf, bf, zoneout)
    bw = _reverse_sequence(_dynamic_zoneout_lstm(_reverse_sequence(x, lengths), lengths, kb, bb,
                                                 zoneout), lengths)
    return np.concatenate([fw, bw], axis=-1)


# ---------------------------------------------------------------------------------------------
# Reference encoder + GST (per utterance preamble)
# ---------------------------------------------------------------------------------------------

def _same_pad(n, k, s):
    out = -(-n // s)
    tot = max((out - 1) * s + k - n, 0)
    return out, tot // 2, tot - tot // 2


def conv2d_same(x, k, b, stride):
    """tf.layers.conv2d(padding='same') NHWC: x [N,H,W,Cin], k [kh,kw,Cin,Cout]
    (modules.py:499-506); TF 'same' puts the odd pad at the bottom/right."""
    N, H, Wd, C = x.shape
    kh, kw, _, O = k.shape
    sh, sw = stride
    Ho, pt, pb = _same_pad(H, kh, sh)
    Wo, pl, pr = _same_pad(Wd, kw, sw)
    xp = np.pad(x, ((0, 0), (pt, pb), (pl, pr), (0, 0)))
    cols = []
    for i in range(kh):
        for j in range(kw):
            cols.append(xp[:, i:i + (Ho - 1) * sh + 1:sh, j:j + (Wo - 1) * sw + 1:sw, :])
    cols = np.concatenate(cols, axis=-1)  # [N,Ho,Wo,kh*kw*C], order (i, j, c)
    return cols @ k.reshape(kh * kw * C, O) + b


def gru_cell(x, h, kg, bg, kc, bc):
    """TF1 tf.nn.rnn_cell.GRUCell (modules.py:59): [r,u] = σ([x,h]·Wg+bg);
    c = tanh([x, r·h]·Wc+bc); h' = u·h + (1-u)·c."""
    dt = x.dtype.type
    v = sigmoid(np.concatenate([x, h], -1) @ kg + bg)
    n = h.shape[-1]
    r, u = v[:, :n], v[:, n:]
    c = np.tanh(np.concatenate([x, r * h], -1) @ kc + bc)
    return u * h + (dt(1) - u) * c


def reference_encoder(mel, W, scope, dt=np.float32):
    """ReferenceEncoder.__call__ (modules.py:20-64), all_outputs=False: 6×[conv2d 3×3 s2 same → BN
    → ReLU] (conv2d() modules.py:499-511), reshape [N,T',F'·C], GRU over every padded step,
    last output → Dense(128, tanh)."""
    x = np.asarray(mel, dt)[..., None]
    for i in range(6):
        s = scope + "conv2d_{}/".format(i)
        x = conv2d_same(x, _w(W, s + "conv2d/kernel", dt), _w(W, s + "conv2d/bias", dt), (2, 2))
        x = batch_norm(x, W, s, dt)
        x = np.maximum(x, dt(0))
    N, T2, F2, C = x.shape
    x = x.reshape(N, T2, F2 * C)
    kg = _w(W, scope + "rnn/gru_cell/gates/kernel", dt)
    bg = _w(W, scope + "rnn/gru_cell/gates/bias", dt)
    kc = _w(W, scope + "rnn/gru_cell/candidate/kernel", dt)
    bc = _w(W, scope + "rnn/gru_cell/candidate/bias", dt)
    h = np.zeros((N, bc.shape[0]), dt)
    for t in range(T2):
        h = gru_cell(x[:, t], h, kg, bg, kc, bc)
    return np.tanh(dense(h, _w(W, scope + "dense/kernel", dt), _w(W, scope + "dense/bias", dt)))


def gst_attention(ref, W, tag, num_heads=4, dt=np.float32):
    """Style tokens + MultiheadAttention mlp_attention, normalize=True
    (tacotron.py:276-282; multihead_attention.py:35-54, 91-132). ref [N,128] → [N, 256]."""
    s = "Multihead-attention-{}/".format(tag)
    tokens = _w(W, "style_tokens_" + tag, dt)                     # [10, 64]
    value = np.tanh(tokens)[None]                                 # [1,10,64] (tile is a broadcast)
    q = dense(ref, _w(W, s + "conv1d/kernel", dt)[0], _w(W, s + "conv1d/bias", dt))        # [N,128]
    k = dense(value[0], _w(W, s + "conv1d_1/kernel", dt)[0], _w(W, s + "conv1d_1/bias", dt))  # [10,128]
    N = ref.shape[0]
    U = q.shape[-1]
    d = U // num_heads
    qs = q.reshape(N, num_heads, 1, d)
    ks = k.reshape(1, 10, num_heads, d).transpose(0, 2, 1, 3)    # [1,H,10,d]
    v = _w(W, s + "attention_v", dt)
    g = _w(W, s + "attention_g", dt)
    bb = _w(W, s + "attention_b", dt)
    normed_v = g * v * (dt(1) / np.sqrt(np.sum(np.square(v))))
    add = np.sum(normed_v * np.tanh(ks + qs + bb), axis=-1)      # [N,H,10]
    add = add - add.max(-1, keepdims=True)
    e = np.exp(add)
    wts = e / e.sum(-1, keepdims=True)                            # [N,H,10]
    ctx = wts @ value[0]                                          # [N,H,64]
    return ctx.reshape(N, num_heads * value.shape[-1])


def reference_encoder_adain(mel_spk, mel_emt, W, dt=np.float32, scope="refnet/"):
    """ReferenceEncoderAdaIn.__call__ (modules.py:75-107) with strides (2,2),(2,2),(1,1)x4
    (tacotron.py:237): conv2d + ReLU stacks without batch norm on both mels; per sample and
    channel moments over (time, freq); spk_norm = tf.nn.batch_normalization(spk, mean_spk, var_spk,
    offset=mean_emt, scale=var_emt, 1e-9); spk = 0.9·spk + 0.1·spk_norm; GRU over every frame;
    last output -> Dense(128, tanh).  Both stacks call conv2d(..., 'conv2d_%d' % i) in the same
    variable scope, speaker first (modules.py:84-87): tf.layers.conv2d's default layer name is
    uniquified inside the re-entered scope, so the speaker stack owns conv2d_i/conv2d/* and the
    emotion stack conv2d_i/conv2d_1/* (two weight sets, not one shared)."""
    strides = [(2, 2), (2, 2), (1, 1), (1, 1), (1, 1), (1, 1)]
    xs = [np.asarray(m, dt)[..., None] for m in (mel_spk, mel_emt)]
    for i in range(6):
        s = scope + "conv2d_{}/".format(i)
        xs = [np.maximum(conv2d_same(x, _w(W, s + ly + "/kernel", dt), _w(W, s + ly + "/bias", dt), strides[i]),
                         dt(0)) for x, ly in zip(xs, ("conv2d", "conv2d_1"))]
    spk, emt = xs
    m_s = spk.mean(axis=(1, 2), keepdims=True)
    v_s = np.square(spk - m_s).mean(axis=(1, 2), keepdims=True)
    m_e = emt.mean(axis=(1, 2), keepdims=True)
    v_e = np.square(emt - m_e).mean(axis=(1, 2), keepdims=True)
    inv = (dt(1) / np.sqrt(v_s + dt(1e-9))) * v_e                 # nn.batch_normalization
    norm = spk * inv + (m_e - m_s * inv)
    spk = spk * dt(0.9) + norm * dt(0.1)
    N, T2, F2, C = spk.shape
    x = spk.reshape(N, T2, F2 * C)
    kg = _w(W, scope + "rnn/gru_cell/gates/kernel", dt)
    bg = _w(W, scope + "rnn/gru_cell/gates/bias", dt)
    kc = _w(W, scope + "rnn/gru_cell/candidate/kernel", dt)
    bc = _w(W, scope + "rnn/gru_cell/candidate/bias", dt)
    h = np.zeros((N, bc.shape[0]), dt)
    for t in range(T2):
        h = gru_cell(x[:, t], h, kg, bg, kc, bc)
    return np.tanh(dense(h, _w(W, scope + "dense/kernel", dt), _w(W, scope + "dense/bias", dt)))


def style_embedding(ref_emt, ref_spk, W, hp, dt=np.float32):
    """tacotron.py:236-308: hp['style'] 'gst' (the fork default: refnet_emt/refnet_spk → GST
    emt/spk → concat [N, 512]), 'embed' (args.pretrained_emb_disc_all or use_gst=False: the
    reference embeddings themselves, :284-291) or 'adain' (args.adain, :266-268); emt_only drops
    the speaker half."""
    mode = hp.get("style", "gst")
    if mode == "adain":
        return reference_encoder_adain(ref_spk, ref_emt, W, dt)
    r_e = reference_encoder(ref_emt, W, "refnet_emt/", dt)
    parts = [gst_attention(r_e, W, "emt", hp.get("num_heads", 4), dt) if mode == "gst" else r_e]
    if not hp.get("emt_only", False):
        r_s = reference_encoder(ref_spk, W, "refnet_spk/", dt)
        parts.append(gst_attention(r_s, W, "spk", hp.get("num_heads", 4), dt) if mode == "gst"
                     else r_s)
    return np.concatenate(parts, axis=-1)


def memory_and_keys(enc_out, style, lengths, W, dt=np.float32):
    """tacotron.py:307-308 concat(encoder_outputs, tile(style)) then TF BahdanauAttention
    _prepare_memory (attention.py:153-158): values = memory·seq_mask; keys = memory_layer(values)."""
    B, T, _ = enc_out.shape
    mem = np.concatenate([enc_out, np.broadcast_to(style[:, None, :], (B, T, style.shape[-1]))], -1)
    mask = (np.arange(T)[None, :] < np.asarray(lengths)[:, None]).astype(dt)[..., None]
    values = (mem * mask).astype(dt)
    keys = values @ _w(W, "memory_layer/kernel", dt)
    return values, keys


# ---------------------------------------------------------------------------------------------
# Decoder
# ---------------------------------------------------------------------------------------------

def prenet(x, masks, W, dt):
    """Prenet.__call__ (modules.py:346-357): Dense+ReLU then dropout(rate .5, training=True) — the
    dropout stays on at inference; masks [2,B,256] are the injected keep bits (TF dropout:
    x / keep · floor(keep + U))."""
    for i in range(2):
        s = "decoder/decoder_prenet/dense_{}/".format(i + 1)
        x = np.maximum(dense(x, _w(W, s + "kernel", dt), _w(W, s + "bias", dt)), dt(0))
        x = (x / dt(0.5)) * masks[i].astype(dt)
    return x


class DecoderState:
    """TacotronDecoderCell.zero_state (Architecture_wrappers.py:158-195)."""

    def __init__(self, B, T_in, D, units, dt):
        self.c1 = np.zeros((B, units), dt)
        self.h1 = np.zeros((B, units), dt)
        self.c2 = np.zeros((B, units), dt)
        self.h2 = np.zeros((B, units), dt)
        self.ctx = np.zeros((B, D), dt)
        self.cum = np.zeros((B, T_in), dt)     # initial_alignments = zeros
        self.max_att = np.zeros((B,), np.int32)


def attention_step(query, st, keys, values, lengths, W, hp, dt):
    """LocationSensitiveAttention.__call__ (attention.py:170-227) + _compute_attention context
    (attention.py:10-35).  Returns alignments, next cumulative state, max_attentions, context."""
    s = "decoder/Location_Sensitive_Attention/"
    q = query @ _w(W, "decoder/query_layer/kernel", dt)                        # :187
    f = conv1d_same(st.cum[..., None], _w(W, s + "location_features_convolution/kernel", dt),
                    _w(W, s + "location_features_convolution/bias", dt))      # :193-195
    loc = f @ _w(W, s + "location_features_layer/kernel", dt)                 # :197
    va = _w(W, s + "attention_variable_projection", dt)
    ba = _w(W, s + "attention_bias", dt)
    energy = np.sum(va * np.tanh(keys + q[:, None, :] + loc + ba), axis=2)    # :69
    T = energy.shape[1]
    tt = np.arange(T)[None, :]
    if hp.get("synthesis_constraint", False):                                  # :202-215
        w = int(hp.get("attention_win_size", 7))
        pm = st.max_att[:, None]
        if hp.get("synthesis_constraint_type", "window") == "monotonic":
            key_m = tt < pm
            rev_m = tt >= (pm + w)
        else:
            key_m = tt < (pm - (w // 2 + (1 if w % 2 != 0 else 0)))
            rev_m = tt >= (pm + w // 2)
        energy = np.where(key_m | rev_m, dt(-2 ** 32 + 1), energy)
    if hp.get("mask_encoder", True):                                           # TF _maybe_mask_score
        energy = np.where(tt < np.asarray(lengths)[:, None], energy, dt(-np.inf))
    if hp.get("smoothing", False):                                             # :71-80, :150
        with np.errstate(over="ignore"):
            e = (1 / (1 + np.exp(-energy))).astype(dt)                        # sigmoid(-inf) = 0
    else:
        m = energy.max(axis=1, keepdims=True)
        e = np.exp(energy - m)
    align = (e / e.sum(axis=1, keepdims=True)).astype(dt)                     # probability_fn :218
    max_att = np.argmax(align, axis=1).astype(np.int32)                       # :219
    cum = align + st.cum if hp.get("cumulative", True) else align             # :222-225
    ctx = np.einsum("bt,btd->bd", align, values)                              # :27
    return align, cum, max_att, ctx


def decoder_step(frame_in, masks, st, keys, values, lengths, W, hp, dt=np.float32):
    """TacotronDecoderCell.__call__ (Architecture_wrappers.py:197-267) for the default (no emt
    attention) decoder.  Mutates ``st``; returns (frames [B, num_mels * r], stop probs, alignments):
    FrameProjection(num_mels * outputs_per_step) and StopProjection(shape=outputs_per_step)
    (tacotron.py:322-324); the stop probs are [B] at r = 1, [B, r] above."""
    z = hp["zoneout"]
    pre = prenet(frame_in, masks, W, dt)                                               # :199
    x1 = np.concatenate([pre, st.ctx], axis=-1)                                        # :202
    k1 = _w(W, "decoder/decoder_LSTM/multi_rnn_cell/cell_0/lstm_cell/kernel", dt)
    b1 = _w(W, "decoder/decoder_LSTM/multi_rnn_cell/cell_0/lstm_cell/bias", dt)
    k2 = _w(W, "decoder/decoder_LSTM/multi_rnn_cell/cell_1/lstm_cell/kernel", dt)
    b2 = _w(W, "decoder/decoder_LSTM/multi_rnn_cell/cell_1/lstm_cell/bias", dt)
    o1, st.c1, st.h1 = zoneout_lstm(x1, st.c1, st.h1, k1, b1, z)                      # :214
    o2, st.c2, st.h2 = zoneout_lstm(o1, st.c2, st.h2, k2, b2, z)
    align, st.cum, st.max_att, st.ctx = attention_step(o2, st, keys, values, lengths, W, hp, dt)
    pin = np.concatenate([o2, st.ctx], axis=-1)                                        # :243
    fs = "decoder/linear_transform_projection/projection_linear_transform_projection/"
    ss = "decoder/stop_token_projection/projection_stop_token_projection/"
    frame = dense(pin, _w(W, fs + "kernel", dt), _w(W, fs + "bias", dt))               # :246
    stop = sigmoid(dense(pin, _w(W, ss + "kernel", dt), _w(W, ss + "bias", dt)))       # :247
    return frame, (stop[:, 0] if stop.shape[1] == 1 else stop), align


def dynamic_decode(keys, values, lengths, W, hp, prenet_masks, max_iters, targets=None,
                   dt=np.float32):
    """tf.contrib.seq2seq.dynamic_decode(CustomDecoder, impute_finished=False,
    maximum_iterations=max_iters) (tacotron.py:349-354) with TacoTestHelper (helpers.py:6-59) or,
    when ``targets`` is given, the GTA TacoTrainingHelper with ratio 1 (helpers.py:62-133).

    The loop emits every step including the stopping one; it ends when time+1 ≥ max_iters (or,
    GTA, time+1 ≥ T_targets / r) or on the helper's stop rule.  r = outputs_per_step is the stop
    projection's width (tacotron.py:322-324): each step emits r frames, the last of which is the next
    step's input (helpers.py:57), and GTA feeds every r-th target frame, targets[:, r-1::r]
    (helpers.py:78).  Stop rule (helpers.py:40-54): finished = round(stop) [B, r]; reduce_all over the
    batch axis first, then any (stop_at_any) / all over the r frames -- at r = 1 both are "every row
    rounds to 1".  Returns frames [B, T*r, num_mels], stop [B, T*r], alignments [B, T_in, T] (the
    reshapes of tacotron.py:357-360)."""
    B, T_in, D = values.shape
    units = W[P + "decoder/decoder_LSTM/multi_rnn_cell/cell_0/lstm_cell/bias"].shape[0] // 4
    st = DecoderState(B, T_in, D, units, dt)
    nm = hp.get("num_mels", 80)
    r = W[P + "decoder/stop_token_projection/projection_stop_token_projection/bias"].shape[0]
    frame_in = np.zeros((B, nm), dt)                                    # _go_frames helpers.py:136
    frames, stops, aligns = [], [], []
    tin = None if targets is None else np.asarray(targets)[:, r - 1::r]  # helpers.py:78
    n_limit = max_iters if targets is None else min(max_iters, tin.shape[1])
    for t in range(n_limit):
        frame, stop, align = decoder_step(frame_in, prenet_masks[t], st, keys, values, lengths, W,
                                          hp, dt)
        stop = stop.reshape(B, r)
        frames.append(frame.reshape(B, r, nm))
        stops.append(stop)
        aligns.append(align)
        if targets is not None:
            frame_in = np.asarray(tin[:, t], dt)                        # helpers.py:126-129
            continue
        fin = np.round(stop) == 1.0                                      # helpers.py:40
        per_frame = np.all(fin, axis=0)                                  # reduce_all(axis=0) -> [r]
        done = bool(np.any(per_frame) if hp.get("stop_at_any", False) else np.all(per_frame))
        if done:
            break
        frame_in = frame[:, -nm:]                                        # helpers.py:57
    return (np.concatenate(frames, 1), np.concatenate(stops, 1), np.stack(aligns, 2))


def postnet_and_clip(dec, W, hp, dt=np.float32):
    """tacotron.py:362-381: clip decoder output to [-max-lower_bound_decay, max], Postnet
    (modules.py:474-482: 4×conv tanh + 1×conv linear, each followed by BN), postnet_projection
    Dense(80), mel = clip(dec + proj)."""
    lo = dt(-hp["max_abs_value"] - hp["lower_bound_decay"])
    hi = dt(hp["max_abs_value"])
    if hp.get("clip_outputs", True):
        dec = np.minimum(np.maximum(dec, lo), hi)
    x = dec
    for i in range(1, 6):
        act = np.tanh if i < 5 else (lambda v: v)
        x = conv1d_block(x, W, "postnet_convolutions/conv_layer_{}_postnet_convolutions/".format(i),
                         act, dt)
    ps = "postnet_projection/projection_postnet_projection/"
    proj = dense(x, _w(W, ps + "kernel", dt), _w(W, ps + "bias", dt))
    mel = dec + proj
    if hp.get("clip_outputs", True):
        mel = np.minimum(np.maximum(mel, lo), hi)
    return dec, mel


def synthesize(ids, lengths, ref_emt, ref_spk, W, hp, prenet_masks, max_iters, targets=None,
               dt=np.float32):
    """Tacotron.initialize synthesis graph (tacotron.py:215-381) for one tower; returns the
    tower_* outputs as a dict of numpy arrays."""
    enc = encoder(ids, lengths, W, hp, dt)
    style = style_embedding(ref_emt, ref_spk, W, hp, dt)
    values, keys = memory_and_keys(enc, style, lengths, W, dt)
    frames, stop, align = dynamic_decode(keys, values, lengths, W, hp, prenet_masks, max_iters,
                                         targets, dt)
    dec, mel = postnet_and_clip(frames, W, hp, dt)
    return dict(encoder_outputs=values, keys=keys, style=style, decoder_output=dec,
                mel_outputs=mel, stop_token_prediction=stop, alignments=align)


def get_output_lengths(stop_tokens):
    """tacotron/synthesizer.py:384-387: per row, the index of the first 1 in np.round(stop)
    (round half to even), else the row length."""
    return [row.index(1) if 1 in row else len(row) for row in np.round(stop_tokens).tolist()]


# ---------------------------------------------------------------------------------------------
# CBHG post-processing network (modules.py:110-184; its one caller is commented out at
# tacotron.py:466-478: linear_outputs = clip(FrameProjection(num_freq)(CBHG(mel_outputs)))
# ---------------------------------------------------------------------------------------------

def max_pool1d_same(x, pool):
    """tf.layers.max_pooling1d(strides=1, padding='same'): window [t − (pool−1)//2, +pool),
    padded positions ignored."""
    B, T, C = x.shape
    pl = (pool - 1) // 2
    out = np.full_like(x, -np.inf)
    for d in range(pool):
        src = np.arange(T) + d - pl
        ok = (src >= 0) & (src < T)
        out[:, ok] = np.maximum(out[:, ok], x[:, src[ok]])
    return out


def highway(x, W, scope, dt):
    """HighwayNet (modules.py:110-122): H = relu(x·W_H + b_H), T = σ(x·W_T + b_T),
    y = H·T + x·(1 − T)."""
    Hh = np.maximum(dense(x, _w(W, scope + "H/kernel", dt), _w(W, scope + "H/bias", dt)), dt(0))
    Tg = sigmoid(dense(x, _w(W, scope + "T/kernel", dt), _w(W, scope + "T/bias", dt)))
    return Hh * Tg + x * (dt(1) - Tg)


def _gru_seq(x, W, scope, dt, reverse=False):
    kg, bg = _w(W, scope + "gates/kernel", dt), _w(W, scope + "gates/bias", dt)
    kc, bc = _w(W, scope + "candidate/kernel", dt), _w(W, scope + "candidate/bias", dt)
    N, T, _ = x.shape
    h = np.zeros((N, bc.shape[0]), dt)
    out = np.zeros((N, T, bc.shape[0]), dt)
    for t in (range(T - 1, -1, -1) if reverse else range(T)):
        h = gru_cell(x[:, t], h, kg, bg, kc, bc)
        out[:, t] = h
    return out


def cbhg(x, W, hp, dt=np.float32, name="CBHG_postnet"):
    """CBHG.__call__(inputs, None) (modules.py:143-184): conv bank of kernel sizes 1..K (conv1d()
    with ReLU, bnorm 'after'), max-pool 'same' stride 1, two projection convs (ReLU, linear), the
    residual with the input, dense to the highway width when they differ, the highway stack, a
    bidirectional GRU over every frame (input_lengths None); [B, T, 2·rnn_units]."""
    sc = name + "/"
    x = np.asarray(x, dt)
    relu = lambda v: np.maximum(v, dt(0))   # noqa: E731
    bank = np.concatenate([conv1d_block(x, W, sc + "conv_bank/conv1d_{}/".format(k), relu, dt)
                           for k in range(1, hp["cbhg_kernels"] + 1)], axis=-1)
    mp = max_pool1d_same(bank, hp["cbhg_pool_size"])
    p1 = conv1d_block(mp, W, sc + "proj1/", relu, dt)
    p2 = conv1d_block(p1, W, sc + "proj2/", lambda v: v, dt)
    h = p2 + x
    if h.shape[-1] != hp["cbhg_highway_units"]:
        h = dense(h, _w(W, sc + "dense/kernel", dt), _w(W, sc + "dense/bias", dt))
    for i in range(hp["cbhg_highwaynet_layers"]):
        h = highway(h, W, sc + "{}_highwaynet_{}/".format(name, i + 1), dt)
    fw = _gru_seq(h, W, sc + "bidirectional_rnn/fw/{}_forward_RNN/".format(name), dt)
    bw = _gru_seq(h, W, sc + "bidirectional_rnn/bw/{}_backward_RNN/".format(name), dt, reverse=True)
    return np.concatenate([fw, bw], axis=-1)


def linear_outputs(mel, W, hp, dt=np.float32):
    """The post-processing net of tacotron.py:466-478: CBHG → FrameProjection(num_freq) → clip."""
    ps = "cbhg_linear_specs_projection/projection_cbhg_linear_specs_projection/"
    y = dense(cbhg(mel, W, hp, dt), _w(W, ps + "kernel", dt), _w(W, ps + "bias", dt))
    if hp.get("clip_outputs", True):
        y = np.minimum(np.maximum(y, dt(-hp["max_abs_value"] - hp["lower_bound_decay"])),
                       dt(hp["max_abs_value"]))
    return y
