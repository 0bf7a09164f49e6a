"""Per-component loss trajectory of the configs[4] whole training step on one fixed batch
(the bench's total loss rose 18.62 -> 23.83 over two clipped-Adam updates).

Runs the bench's exact batch (tt2.synthetic, seeds of bench.py's train leg) for --steps updates at
each (precision, lr, style-loss) setting from the same initial weights and prints one JSON line per
setting with every loss component per step (the forward loss BEFORE that step's update), the global
gradient norm, and the relative size of each update of a few variables.

    python scripts/diag_train_loss.py --steps 8 > gpurun_out/diag_loss.jsonl
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tacotron-2_amd"))

KEYS = ("before", "after", "stop_token", "regularization", "style_emb_loss_emt", "style_emb_loss_spk",
        "style_emb_orthog_loss", "loss", "grad_norm")
WATCH = ("Tacotron_model/inference/decoder/decoder_LSTM/multi_rnn_cell/cell_0/lstm_cell/kernel",
         "Tacotron_model/inference/decoder/linear_transform_projection/projection_linear_transform_projection/kernel",
         "Tacotron_model/inference/style_disc_emt/dense/kernel")


def run(prec, lr, steps, n_cls, orthog, B=64, Ti=150, T=800, Tr=800):
    import torch
    from tt2.hparams import hparams
    from tt2.synthetic import (enc_conv_masks, enc_zoneout_masks, postnet_masks, prenet_masks,
                               tacotron_inputs, train_batch, zoneout_masks)
    from tt2.train import TacotronTrainer
    from tt2.weights import init_tacotron_weights, memory_width
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1, tacotron_use_orthog_loss=bool(orthog)))
    D = memory_width(hp)
    W = init_tacotron_weights(hp, seed=hp.tacotron_random_seed)
    tr = TacotronTrainer(hp, W, B, Ti, T, 0, precision=prec, frontend=True, max_T_ref=Tr,
                         n_emt=n_cls, n_spk=n_cls)
    if n_cls:
        lab = np.random.default_rng(99).integers(0, n_cls, (2, B))
        tr.set_style_labels(lab[0], lab[1])
    dev = torch.device("cuda", 0)
    _, _, tg, st = train_batch(B, Ti, T, D, seed=1234)
    ids, tlens, re, rs = tacotron_inputs(B, Ti, Tr, seed=1234)
    fb = [torch.from_numpy(x).to(dev) for x in (ids, tlens, re, rs, tg, st)]
    fb.append(torch.from_numpy(prenet_masks(T, B, hp.prenet_layers[0], seed=7)).to(dev))
    fb.append(torch.from_numpy(zoneout_masks(T, B, hp.decoder_lstm_units, seed=7)).to(dev))
    fb.append(torch.from_numpy(postnet_masks(hp.postnet_num_layers, B, T, hp.postnet_channels, seed=7)).to(dev))
    fb.append(torch.from_numpy(enc_conv_masks(hp.enc_conv_num_layers, B, Ti, hp.enc_conv_channels, seed=7)).to(dev))
    fb.append(torch.from_numpy(enc_zoneout_masks(Ti, B, hp.encoder_lstm_units, seed=7)).to(dev))
    hist = {k: [] for k in KEYS}
    watch = [n for n in WATCH if n in W or n in tr.style_disc_weights]
    upd = {n: [] for n in watch}
    t0 = time.perf_counter()
    try:
        for s in range(1, steps + 1):
            before = {n: tr.get(n, 0, tr_shape(W, tr, n)) for n in watch}
            tr.forward_backward_text(*fb)
            tr.apply(s, lr=lr)
            L = tr.losses()
            for k in KEYS:
                hist[k].append(round(L[k], 6))
            for n in watch:
                a = tr.get(n, 0, before[n].shape)
                upd[n].append(float(np.linalg.norm(a - before[n]) / max(np.linalg.norm(before[n]), 1e-30)))
        # the loss AFTER the last update, with no further update
        tr.forward_backward_text(*fb)
        L = tr.losses()
        for k in KEYS:
            hist[k].append(round(L[k], 6))
    finally:
        tr.close()
    return dict(precision=prec, lr=lr, steps=steps, n_cls=n_cls, orthog=bool(orthog), losses=hist,
                rel_update={"/".join(n.split("/")[-3:]): [round(x, 6) for x in v] for n, v in upd.items()},
                seconds=round(time.perf_counter() - t0, 1))


def tr_shape(W, tr, n):
    if n in W:
        return np.asarray(W[n]).shape
    return np.asarray(tr.style_disc_weights[n]).shape


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--settings", default="bf16:1e-3:4:1,bf16:1e-4:4:1,bf16:1e-5:4:1,fp32:1e-3:4:1,bf16:1e-3:0:0")
    a = ap.parse_args()
    for item in a.settings.split(","):
        prec, lr, n_cls, orthog = item.split(":")
        r = run(prec, float(lr), a.steps, int(n_cls), int(orthog))
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
