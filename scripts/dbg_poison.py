"""Debug: the front-end training step (run under TT2_POISON_ALLOC=1, or after the tests that
precede it in the failing order with argument "order") -- per-variable gradient error vs
the oracle, then the encoder conv-1 weight-gradient operands checked one by one on the host."""
import os
import sys
import numpy as np
sys.path[:0] = ['tacotron-2_amd', '.', 'tests']
from _common import small_hparams
from oracle import train_ref as TRN
from test_train import _front_case, _rel
from tt2.train import TacotronTrainer
import test_train
if "order" in sys.argv:
    test_train.test_gpu_train_bf16_gemms_close_to_oracle()
    test_train.test_gpu_train_full_size_properties()
    print("preceding tests done", flush=True)

hp = small_hparams()
masks = "nomasks" not in sys.argv
W, ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm = _front_case(hp, masks=masks)
B, T_in, T_out = ids.shape[0], ids.shape[1], tg.shape[1]
tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, frontend=True, max_T_ref=re.shape[1])
tr.forward_backward_text(ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm)
L, g, stats = TRN.train_grads_frontend(W, ids, lens, re, rs, tg, st, pm, zm, em, ezm, hp.tacotron_reg_weight,
                                        postnet_masks=pnm, style=dict(orthog_weight=0.02))
bad = []
for n in TRN.frontend_var_names() + TRN.train_var_names() + TRN.postnet_var_names():
    got = tr.get(n, 1, np.asarray(W[n]).shape)
    e = _rel(got, g[n]) if np.abs(g[n]).max() > 1e-12 else np.abs(got).max()
    flag = "BAD" if not (e < 2e-4) else ""
    if flag:
        bad.append(n)
    print("{:90s} {:.3e} {}".format(n[25:], e, flag), flush=True)
print("bad:", bad)

P = "Tacotron_model/inference/"
E, C, K = hp.embedding_dim, hp.enc_conv_channels, hp.enc_conv_kernel_size[0]
M = B * T_in
ex = tr.get("debug:enc_embedded", 0, (M, E))
fb = tr.get("debug:enc_conv1_im2col", 0, (K * E, M))
dz = tr.get("debug:enc_conv1_dz", 0, (M, C))
tab = np.asarray(W[P + "inputs_embedding"], np.float32)
want_ex = tab[np.asarray(ids).reshape(-1)]
print("embedded  max err", np.abs(ex - want_ex).max(), "nan", np.isnan(ex).sum())
pad = (K - 1) // 2
x3 = ex.reshape(B, T_in, E)
want_fb = np.zeros((K * E, M), np.float32)
for tap in range(K):
    for t in range(T_in):
        ts = t + tap - pad
        if 0 <= ts < T_in:
            want_fb[tap * E:(tap + 1) * E, np.arange(B) * T_in + t] = x3[:, ts, :].T
print("im2col    max err", np.abs(fb - want_fb).max(), "nan", np.isnan(fb).sum())
print("dz nan", np.isnan(dz).sum(), "max", np.abs(dz).max())
sc = P + "encoder_convolutions/conv_layer_1_encoder_convolutions/conv1d/kernel"
got = tr.get(sc, 1, (K, E, C)).reshape(K * E, C)
host = (fb.astype(np.float64) @ dz.astype(np.float64))
want = np.asarray(g[sc]).reshape(K * E, C)
print("device grad vs host fb@dz: rel", _rel(got, host), " host fb@dz vs oracle: rel", _rel(host, want))
err = np.abs(got - want) > 2e-4 * np.abs(want).max()
rows, cols = np.nonzero(err)
print("wrong entries", err.sum(), "of", err.size, "rows", sorted(set((rows // E).tolist())), "(taps)",
      "cols", sorted(set(cols.tolist()))[:20])
tr.close()
