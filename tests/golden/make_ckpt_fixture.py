"""Extract the reference's trained emotion reference-encoder weights (refnet_emt) from its TF
checkpoint into tests/golden/refnet_emt_ckpt5200.npz with tt2.ckpt (no TensorFlow).

Source: code/spk_disc/pretrained_model_emt_disc/emt_disc_model.ckpt-5200 — the checkpoint the
reference restores into Tacotron's refnet_emt scope (tacotron/train.py:284, 330-333).  Only data
(the 42 refnet_emt variables) is stored; run from the repository root with /root/reference present:
    python tests/golden/make_ckpt_fixture.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tacotron-2_amd"))
from tt2 import ckpt  # noqa: E402

SRC = "/root/reference/code/spk_disc/pretrained_model_emt_disc/emt_disc_model.ckpt-5200"
DST = os.path.join(ROOT, "tests", "golden", "refnet_emt_ckpt5200.npz")


def main():
    d = {k: v for k, v in ckpt.read_checkpoint(SRC).items() if "/refnet_emt/" in k}
    np.savez_compressed(DST, **d)
    print("wrote", DST, len(d), "tensors", sum(v.size for v in d.values()), "values")


if __name__ == "__main__":
    main()
