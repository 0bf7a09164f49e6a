"""Generate the golden fixtures under tests/golden/ from the numpy oracle.

The reference has no golden vectors, no tests and no trained checkpoints, and TensorFlow 1.x is
not installable here, so these fixtures pin the oracle restatement itself
(parity unpinned against the reference).  Inputs + outputs are stored; the small-config weights are
regenerated from their seed by tt2.weights, and a weight checksum is stored so that a change of the
initializer is detected instead of silently changing the fixtures.

Run: python tests/golden/make_golden.py   (writes tests/golden/*.npz, each < 1 MB)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "tacotron-2_amd"), ROOT, os.path.join(ROOT, "tests")]

from _common import full_hparams, small_hparams, small_wavenet_hparams  # noqa: E402
from oracle import tacotron_ref as TR  # noqa: E402
from oracle import wavenet_ref as WR  # noqa: E402
from oracle.hp import oracle_hp, wavenet_oracle_hp  # noqa: E402
from tt2.synthetic import mol_uniforms, prenet_masks, tacotron_inputs  # noqa: E402
from tt2.weights import init_tacotron_weights, init_wavenet_weights  # noqa: E402


def weight_checksum(W):
    h = 0.0
    for k in sorted(W):
        v = np.asarray(W[k], np.float64).ravel()
        h += float(np.sum(v * np.arange(1, v.size + 1) % 7.0)) + len(k)
    return np.float64(h)


def tacotron_fixtures():
    hp = small_hparams()
    W = init_tacotron_weights(hp, seed=5339)
    oh = oracle_hp(hp)
    B, T, TR_ = 3, 11, 70
    ids, lens, re, rs = tacotron_inputs(B, T, TR_, seed=7)
    n = 20
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=7)
    out = TR.synthesize(ids, lens, re, rs, W, oh, masks, n)
    np.savez_compressed(os.path.join(HERE, "tacotron_small_freerun.npz"), ids=ids, lengths=lens,
                        ref_emt=re, ref_spk=rs, prenet_masks=masks, max_iters=n,
                        weight_checksum=weight_checksum(W), **{k: v for k, v in out.items()})
    # GTA (teacher-forced) 30 steps
    tg = np.random.default_rng(3).uniform(-4, 4, (B, 30, 80)).astype(np.float32)
    masks2 = prenet_masks(40, B, hp.prenet_layers[0], seed=8)
    out = TR.synthesize(ids, lens, re, rs, W, oh, masks2, 40, targets=tg)
    np.savez_compressed(os.path.join(HERE, "tacotron_small_gta.npz"), ids=ids, lengths=lens,
                        ref_emt=re, ref_spk=rs, prenet_masks=masks2, max_iters=40, targets=tg,
                        weight_checksum=weight_checksum(W),
                        mel_outputs=out["mel_outputs"], stop_token_prediction=out["stop_token_prediction"],
                        alignments=out["alignments"])
    # window-constrained synthesis (args.synth_constraint)
    out = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp, True), masks, n)
    np.savez_compressed(os.path.join(HERE, "tacotron_small_window.npz"), ids=ids, lengths=lens,
                        ref_emt=re, ref_spk=rs, prenet_masks=masks, max_iters=n,
                        weight_checksum=weight_checksum(W), mel_outputs=out["mel_outputs"],
                        alignments=out["alignments"])


def decoder_step_inputs(seed=61):
    """Single decoder-step fixture inputs at the fork widths (B=2, T_in=7,
    D_mem=1024): memory from the oracle encoder + style path, and a non-trivial carried state."""
    hp = full_hparams()
    W = init_tacotron_weights(hp, seed=5339)
    oh = oracle_hp(hp)
    B, T = 2, 7
    ids, lens, re, rs = tacotron_inputs(B, T, 64, seed=seed)
    enc = TR.encoder(ids, lens, W, oh)
    style = TR.style_embedding(re, rs, W, oh)
    values, keys = TR.memory_and_keys(enc, style, lens, W)
    rng = np.random.default_rng(seed)
    H, D = hp.decoder_lstm_units, values.shape[2]
    st = TR.DecoderState(B, T, D, H, np.float32)
    st.h1, st.c1, st.h2, st.c2 = [rng.uniform(-0.5, 0.5, (B, H)).astype(np.float32) for _ in range(4)]
    a = rng.random((B, T)) * (np.arange(T)[None] < lens[:, None])
    a = (a / a.sum(1, keepdims=True)).astype(np.float32)
    st.ctx = np.einsum("bt,btd->bd", a, values).astype(np.float32)
    st.cum = (a * 3.0).astype(np.float32)
    st.max_att = np.array([min(3, lens[b] - 1) for b in range(B)], np.int32)
    frame_in = rng.uniform(-4, 4, (B, hp.num_mels)).astype(np.float32)
    masks = prenet_masks(1, B, hp.prenet_layers[0], seed=seed)[0]
    return hp, W, ids, lens, re, rs, values, keys, st, frame_in, masks


def decoder_step_fixtures():
    hp, W, ids, lens, re, rs, values, keys, st, frame_in, masks = decoder_step_inputs()
    state_in = dict(h1=st.h1, c1=st.c1, h2=st.h2, c2=st.c2, attention=st.ctx, alignments=st.cum,
                    max_attentions=st.max_att)
    frame, stop, align = TR.decoder_step(frame_in, masks, st, keys, values, lens, W, oracle_hp(hp))
    np.savez_compressed(
        os.path.join(HERE, "tacotron_decoder_step.npz"), ids=ids, lengths=lens, ref_emt=re,
        ref_spk=rs, frame_in=frame_in, prenet_masks=masks, weight_checksum=weight_checksum(W),
        **{"in_" + k: v for k, v in state_in.items()},
        out_h1=st.h1, out_c1=st.c1, out_h2=st.h2, out_c2=st.c2, out_attention=st.ctx,
        out_alignments=st.cum, out_max_attentions=st.max_att, frame=frame, stop=stop, align=align)


def wavenet_fixtures():
    hp = small_wavenet_hparams(6, 2)
    W = init_wavenet_weights(hp, seed=5339)
    rng = np.random.default_rng(21)
    B, T_f = 2, 1
    T = T_f * 275
    mel = rng.uniform(-4, 4, (B, T_f, 80)).astype(np.float32)
    cond = WR.interp_condition(mel)
    um, ul = mol_uniforms(T, B, seed=3)
    teacher = rng.uniform(-0.9, 0.9, (B, T)).astype(np.float32)
    c_up = WR.upsample_2d(cond.transpose(0, 2, 1), W, hp.upsample_scales)
    y, k, lg = WR.incremental(c_up.transpose(0, 2, 1), W, wavenet_oracle_hp(hp), um, ul, teacher,
                              return_logits=True)
    np.savez_compressed(os.path.join(HERE, "wavenet_small_teacher.npz"), mel=mel, cond=cond, u_mix=um,
                        u_log=ul, teacher=teacher, upsampled=c_up, y=y, k=k, logits=lg,
                        weight_checksum=weight_checksum(W))
    yf, kf = WR.incremental(c_up.transpose(0, 2, 1), W, wavenet_oracle_hp(hp), um, ul)
    np.savez_compressed(os.path.join(HERE, "wavenet_small_freerun.npz"), cond=cond, u_mix=um,
                        u_log=ul, y=yf, k=kf, weight_checksum=weight_checksum(W))


def mol_fixtures():
    rng = np.random.default_rng(0)
    n, nr = 512, 10
    logits = rng.normal(0, 2, (n, 3 * nr)).astype(np.float32)
    logits[:64, 1] = logits[:64, 0]
    um = rng.uniform(1e-5, 1 - 1e-5, (n, nr)).astype(np.float32)
    um[:32, 1] = um[:32, 0]   # exact ties -> lowest index (tf.argmax)
    logits[64:80, 2 * nr:] = -100.0  # log-scale clamp at log_scale_min
    ul = rng.uniform(1e-5, 1 - 1e-5, (n,)).astype(np.float32)
    lsm = float(np.log(1e-14))
    x, k = WR.mol_sample(logits, um, ul, lsm)
    np.savez_compressed(os.path.join(HERE, "mol_sampler.npz"), logits=logits, u_mix=um, u_log=ul,
                        log_scale_min=lsm, x=x, k=k)


if __name__ == "__main__":
    decoder_step_fixtures()
    tacotron_fixtures()
    wavenet_fixtures()
    mol_fixtures()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)), "bytes")
