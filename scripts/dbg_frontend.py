"""Debug: per-variable relative gradient error of the front-end training step vs the oracle."""
import sys
import numpy as np
sys.path[:0] = ['tacotron-2_amd', '.', 'tests']
from _common import small_hparams
from oracle import train_ref as TRN
from test_train import _front_case, _rel
from tt2.train import TacotronTrainer
hp = small_hparams()
masks = len(sys.argv) < 2
W, ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm = _front_case(hp, masks=masks)
B, T_in, T_out = ids.shape[0], ids.shape[1], tg.shape[1]
tr = TacotronTrainer(hp, W, B, T_in, T_out, 0, frontend=True, max_T_ref=re.shape[1])
tr.forward_backward_text(ids, lens, re, rs, tg, st, pm, zm, pnm, em, ezm)
L, g, stats = TRN.train_grads_frontend(W, ids, lens, re, rs, tg, st, pm, zm, em, ezm, hp.tacotron_reg_weight,
                                        postnet_masks=pnm, style=dict(orthog_weight=0.02))
for n in TRN.frontend_var_names():
    got = tr.get(n, 1, np.asarray(W[n]).shape)
    print("{:80s} {:.3e} {:.3e}".format(n[25:], _rel(got, g[n]), np.abs(g[n]).max()))
import torch
names = TRN.frontend_var_names()
Wt = {n: torch.tensor(np.asarray(W[n]), dtype=torch.float64) for n in names}
mem, _ = TRN.frontend_forward(Wt, ids, lens, re, rs, em, ezm)
gm = tr.get("frontend:memory", 0, tuple(mem.shape))
D2 = 2 * hp.encoder_lstm_units
print("memory enc part", np.abs(gm[..., :D2] - mem.numpy()[..., :D2]).max(), "style part",
      np.abs(gm[..., D2:] - mem.numpy()[..., D2:]).max(axis=(0, 1)).reshape(2, -1).max(1))
