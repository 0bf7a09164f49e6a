"""TEST INFRASTRUCTURE ONLY — numpy restatement of Tacotron_emt_attn's synthesis graph
(mwhitehill/Tacotron-2 ``code/tacotron/models/tacotron_emt_attn.py``), built on the Tacotron
restatement in ``tacotron_ref.py`` (parity unpinned: the reference ships no checkpoint or fixture of
this model; see ``oracle/__init__.py``).  Never imported by the product.

What the variant changes (file:line in the reference's ``code/``):
* memory = encoder outputs only, no GST (tacotron_emt_attn.py:244-246);
* refnet_emt keeps every output (ReferenceEncoder all_outputs, modules.py:35-55) and the decoder
  attends over them each step with its LSTM output as the query (Architecture_wrappers.py:228-240):
  'simple' SimpleBahdanauAttention (attention.py:230-260), 'multihead' MultiheadAttention +
  dense(128), 'style_tokens' MultiheadAttention over tanh(24 x 16 tokens) with the one-hot emotion
  label appended to the query;
* that context (plus refnet_spk) joins the next step's LSTM-1 input (Architecture_wrappers.py:
  203-211).
"""
import numpy as np

from . import tacotron_ref as T
from .tacotron_ref import _w, dense, sigmoid

EMT_ATTN = ("simple", "multihead", "style_tokens")
EMT_REF_GRU = ("none", "gru", "gru_multi")


def reference_cnn(mel, W, scope, dt=np.float32):
    """ReferenceEncoder CNN stack (modules.py:22-33) -> [N, T', F'·C]."""
    x = np.asarray(mel, dt)[..., None]
    for i in range(6):
        s = scope + "conv2d_{}/".format(i)
        x = T.conv2d_same(x, _w(W, s + "conv2d/kernel", dt), _w(W, s + "conv2d/bias", dt), (2, 2))
        x = np.maximum(T.batch_norm(x, W, s, dt), dt(0))
    N, T2, F2, C = x.shape
    return x.reshape(N, T2, F2 * C)


def _gru_run(x, W, scope, dt, reverse=False):
    """TF1 GRUCell over every frame (no sequence_length); returns all outputs [N, T', D]."""
    kg = _w(W, scope + "gates/kernel", dt)
    bg = _w(W, scope + "gates/bias", dt)
    kc = _w(W, scope + "candidate/kernel", dt)
    bc = _w(W, scope + "candidate/bias", dt)
    N, T2, _ = x.shape
    h = np.zeros((N, bc.shape[0]), dt)
    out = np.zeros((N, T2, bc.shape[0]), dt)
    order = range(T2 - 1, -1, -1) if reverse else range(T2)
    for t in order:
        h = T.gru_cell(x[:, t], h, kg, bg, kc, bc)
        out[:, t] = h
    return out


def emotion_values(ref_emt, W, attn, emt_ref_gru, dt=np.float32):
    """What the emotion attention attends over: tanh(style_tokens) [24,16] broadcast per row
    (tacotron_emt_attn.py:212-214), or refnet_emt's all_outputs (modules.py:35-55):
    'none' the CNN output, 'gru' [fw | bw] bidirectional_dynamic_rnn outputs (full-length reverse),
    'gru_multi' 8 × (GRU last output → dense(128, tanh))."""
    if attn == "style_tokens":
        return np.tanh(_w(W, "style_tokens", dt))[None]
    x = reference_cnn(ref_emt, W, "refnet_emt/", dt)
    if emt_ref_gru == "none":
        return x
    if emt_ref_gru == "gru":
        fw = _gru_run(x, W, "refnet_emt/bidirectional_rnn/fw/gru_cell/", dt)
        bw = _gru_run(x, W, "refnet_emt/bidirectional_rnn/bw/gru_cell/", dt, reverse=True)
        return np.concatenate([fw, bw], -1)
    outs = []
    for i in range(8):
        s = "refnet_emt/gru_{}/".format(i)
        h = _gru_run(x, W, s + "rnn/gru_cell/", dt)[:, -1]
        outs.append(np.tanh(dense(h, _w(W, s + "dense/kernel", dt), _w(W, s + "dense/bias", dt))))
    return np.stack(outs, 1)


def emotion_attention(query, values, W, attn, labels=None, n_emt=4, num_heads=4, dt=np.float32):
    """Per-step emotion context and its attention weights [N, heads, T_v].

    'simple' (attention.py:241-260): score = V(tanh(W1(values) + W2(query))), softmax over T_v,
    context = Σ a·values.  Multi-head (multihead_attention.py:35-132, mlp_attention, normalize):
    q = conv1d(query), k = conv1d(values), per head v·tanh(k + q + b) with v = g·v/‖v‖, softmax,
    context = a·values per head, heads concatenated; 'multihead' then dense(128)
    (Architecture_wrappers.py:233-234); 'style_tokens' queries with [LSTM_output, one_hot(label)]
    (:236)."""
    N = query.shape[0]
    vals = np.broadcast_to(values, (N,) + values.shape[1:])
    if attn == "simple":
        k = dense(vals, _w(W, "decoder/W1/kernel", dt), _w(W, "decoder/W1/bias", dt))
        q = dense(query, _w(W, "decoder/W2/kernel", dt), _w(W, "decoder/W2/bias", dt))
        score = dense(np.tanh(k + q[:, None, :]), _w(W, "decoder/V/kernel", dt),
                      _w(W, "decoder/V/bias", dt))[..., 0]                 # [N, T_v]
        score = score - score.max(-1, keepdims=True)
        e = np.exp(score)
        a = (e / e.sum(-1, keepdims=True)).astype(dt)
        return np.einsum("nt,ntd->nd", a, vals), a[:, None, :]
    mh = "decoder/Multihead-attention-attn_emt/"
    if attn == "style_tokens":
        oh = np.zeros((N, n_emt), dt)
        for b, l in enumerate(np.asarray(labels)):
            if 0 <= l < n_emt:                                             # tf.one_hot: else zeros
                oh[b, l] = 1
        query = np.concatenate([query, oh], -1)
    q = dense(query, _w(W, mh + "conv1d/kernel", dt)[0], _w(W, mh + "conv1d/bias", dt))
    k = dense(vals, _w(W, mh + "conv1d_1/kernel", dt)[0], _w(W, mh + "conv1d_1/bias", dt))
    A = q.shape[-1]
    d = A // num_heads
    Tv = vals.shape[1]
    qs = q.reshape(N, num_heads, 1, d)
    ks = k.reshape(N, Tv, num_heads, d).transpose(0, 2, 1, 3)
    v = _w(W, mh + "attention_v", dt)
    g = _w(W, mh + "attention_g", dt)
    bb = _w(W, mh + "attention_b", dt)
    nv = g * v * (dt(1) / np.sqrt(np.sum(np.square(v))))
    add = np.sum(nv * np.tanh(ks + qs + bb), axis=-1)                     # [N, heads, T_v]
    add = add - add.max(-1, keepdims=True)
    e = np.exp(add)
    a = (e / e.sum(-1, keepdims=True)).astype(dt)
    ctx = np.einsum("nht,ntd->nhd", a, vals).reshape(N, num_heads * vals.shape[-1])  # _combine_heads
    if attn == "multihead":
        ctx = dense(ctx, _w(W, "decoder/attn_emt/dense/kernel", dt),
                    _w(W, "decoder/attn_emt/dense/bias", dt))
    return ctx, a


def decoder_step(frame_in, masks, st, keys, values, lengths, emt_values, spk, W, hp, attn,
                 labels=None, n_emt=4, dt=np.float32):
    """TacotronDecoderCell.__call__ with an emotion attention (Architecture_wrappers.py:197-267).
    ``st.ctx_emt`` carries attention_emt (zero_state: zeros, :182)."""
    z = hp["zoneout"]
    pre = T.prenet(frame_in, masks, W, dt)
    parts = [pre, st.ctx]
    if spk is not None:
        parts += [spk + st.ctx_emt] if attn == "multihead" else [st.ctx_emt, spk]   # :204-209
    else:
        parts += [st.ctx_emt]                                                         # :211
    x1 = np.concatenate(parts, axis=-1)
    k1 = _w(W, "decoder/decoder_LSTM/multi_rnn_cell/cell_0/lstm_cell/kernel", dt)
    b1 = _w(W, "decoder/decoder_LSTM/multi_rnn_cell/cell_0/lstm_cell/bias", dt)
    k2 = _w(W, "decoder/decoder_LSTM/multi_rnn_cell/cell_1/lstm_cell/kernel", dt)
    b2 = _w(W, "decoder/decoder_LSTM/multi_rnn_cell/cell_1/lstm_cell/bias", dt)
    o1, st.c1, st.h1 = T.zoneout_lstm(x1, st.c1, st.h1, k1, b1, z)
    o2, st.c2, st.h2 = T.zoneout_lstm(o1, st.c2, st.h2, k2, b2, z)
    align, st.cum, st.max_att, st.ctx = T.attention_step(o2, st, keys, values, lengths, W, hp, dt)
    st.ctx_emt, a_emt = emotion_attention(o2, emt_values, W, attn, labels, n_emt,
                                          hp.get("num_heads", 4), dt)           # :228-240
    pin = np.concatenate([o2, st.ctx], axis=-1)
    fs = "decoder/linear_transform_projection/projection_linear_transform_projection/"
    ss = "decoder/stop_token_projection/projection_stop_token_projection/"
    frame = dense(pin, _w(W, fs + "kernel", dt), _w(W, fs + "bias", dt))
    stop = sigmoid(dense(pin, _w(W, ss + "kernel", dt), _w(W, ss + "bias", dt)))[:, 0]
    return frame, stop, align, a_emt


def emt_state_width(W, attn):
    """attention_emt zero-state width (Architecture_wrappers.py:116-123): the 'simple' units."""
    if attn == "simple":
        return W[T.P + "decoder/W1/bias"].shape[0]
    return {"multihead": 128, "style_tokens": 64}[attn]


def synthesize(ids, lengths, ref_emt, ref_spk, W, hp, attn, emt_ref_gru, prenet_masks, max_iters,
               labels=None, n_emt=4, emt_only=False, targets=None, dt=np.float32):
    """Tacotron_emt_attn.initialize synthesis (tacotron_emt_attn.py:198-381) for one tower, with
    the TacoTestHelper / GTA loop of ``tacotron_ref.dynamic_decode``."""
    enc = T.encoder(ids, lengths, W, hp, dt)
    B, T_in, D = enc.shape
    mask = (np.arange(T_in)[None, :] < np.asarray(lengths)[:, None]).astype(dt)[..., None]
    values = (enc * mask).astype(dt)
    keys = values @ _w(W, "memory_layer/kernel", dt)
    ev = emotion_values(ref_emt, W, attn, emt_ref_gru, dt)
    spk = None
    if attn != "style_tokens" and not emt_only:
        spk = T.reference_encoder(ref_spk, W, "refnet_spk/", dt)
    units = W[T.P + "decoder/decoder_LSTM/multi_rnn_cell/cell_0/lstm_cell/bias"].shape[0] // 4
    st = T.DecoderState(B, T_in, D, units, dt)
    st.ctx_emt = np.zeros((B, emt_state_width(W, attn)), dt)
    nm = hp.get("num_mels", 80)
    frame_in = np.zeros((B, nm), dt)
    frames, stops, aligns, aligns_emt = [], [], [], []
    n_limit = max_iters if targets is None else min(max_iters, targets.shape[1])
    for t in range(n_limit):
        frame, stop, align, a_emt = decoder_step(frame_in, prenet_masks[t], st, keys, values,
                                                 lengths, ev, spk, W, hp, attn, labels, n_emt, dt)
        frames.append(frame)
        stops.append(stop)
        aligns.append(align)
        aligns_emt.append(a_emt)
        if targets is not None:
            frame_in = np.asarray(targets[:, t], dt)
            continue
        fin = np.round(stop) == 1.0
        if bool(np.all(fin)):  # helpers.py:40-54: batch axis reduced first (stop_at_any: r frames, r = 1)
            break
        frame_in = frame
    frames = np.stack(frames, 1)
    dec, mel = T.postnet_and_clip(frames, W, hp, dt)
    return dict(encoder_outputs=values, keys=keys, emt_values=ev, spk=spk, frames=frames,
                decoder_output=dec, mel_outputs=mel, stop_token_prediction=np.stack(stops, 1),
                alignments=np.stack(aligns, 2), alignments_emt=np.stack(aligns_emt, 0))
