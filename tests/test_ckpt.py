"""TF tensor-bundle checkpoint reader (tt2.ckpt), CPU only.

* a synthetic bundle written by a minimal SSTable/protobuf writer below round-trips exactly;
* when /root/reference is present (build container only): both trained reference-encoder
  checkpoints the reference restores into its refnet scopes (tacotron/train.py:284-285,
  330-338) parse, map 1:1 onto this build's variable names/shapes, and the committed fixture
  tests/golden/refnet_emt_ckpt5200.npz equals the checkpoint bit for bit;
* the oracle reference encoder runs on the trained weights (finite, tanh-bounded output).
"""
import os
import struct

import numpy as np
import pytest

from _common import full_hparams, oracle_hp

HERE = os.path.dirname(os.path.abspath(__file__))
REF_CKPTS = {
    "refnet_emt": "/root/reference/code/spk_disc/pretrained_model_emt_disc",
    "refnet_spk": "/root/reference/code/spk_disc/pretrained_model_spk_disc",
}
FIXTURE = os.path.join(HERE, "golden", "refnet_emt_ckpt5200.npz")


# ---- a minimal tensor-bundle writer (test-only) ----
def _vint(n):
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def _field(num, wt, payload):
    if wt == 0:
        return _vint(num << 3) + _vint(payload)
    return _vint((num << 3) | 2) + _vint(len(payload)) + payload


def _block(entries):
    body = bytearray()
    prev = b""
    for k, v in entries:  # prefix-compress against the previous key like LevelDB
        shared = 0
        while shared < min(len(prev), len(k)) and prev[shared] == k[shared]:
            shared += 1
        body += _vint(shared) + _vint(len(k) - shared) + _vint(len(v)) + k[shared:] + v
        prev = k
    body += struct.pack("<I", 0) + struct.pack("<I", 1)  # one restart point at 0
    return bytes(body) + b"\x00" + b"\x00\x00\x00\x00"    # trailer: no compression, crc unchecked


def write_bundle(prefix, tensors):
    data = bytearray()
    entries = [(b"", _field(1, 0, 1))]  # BundleHeaderProto num_shards = 1
    for name in sorted(tensors):
        a = np.asarray(tensors[name], np.float32, order="C")
        shape = b"".join(_field(2, 2, _field(1, 0, d)) for d in a.shape)
        proto = _field(1, 0, 1) + _field(2, 2, shape) + _field(4, 0, len(data)) + _field(5, 0, a.nbytes)
        entries.append((name.encode(), proto))
        data += a.tobytes()
    with open(prefix + ".data-00000-of-00001", "wb") as f:
        f.write(bytes(data))
    blob = bytearray()
    dblock = _block(entries)
    d_handle = (0, len(dblock) - 5)
    blob += dblock
    mblock = _block([])
    m_handle = (len(blob), len(mblock) - 5)
    blob += mblock
    iblock = _block([(entries[-1][0], _vint(d_handle[0]) + _vint(d_handle[1]))])
    i_handle = (len(blob), len(iblock) - 5)
    blob += iblock
    footer = _vint(m_handle[0]) + _vint(m_handle[1]) + _vint(i_handle[0]) + _vint(i_handle[1])
    footer = footer + b"\x00" * (40 - len(footer)) + struct.pack("<Q", 0xdb4775248b80fb57)
    with open(prefix + ".index", "wb") as f:
        f.write(bytes(blob) + footer)


def test_bundle_round_trip(tmp_path):
    from tt2 import ckpt
    rng = np.random.default_rng(0)
    t = {"Tacotron_model/inference/a/kernel": rng.standard_normal((3, 5)).astype(np.float32),
         "Tacotron_model/inference/a/bias": rng.standard_normal(5).astype(np.float32),
         "Tacotron_model/inference/b/w": rng.standard_normal((2, 2, 4)).astype(np.float32),
         "global_step": np.array(7.0, np.float32)}
    prefix = str(tmp_path / "model.ckpt-7")
    write_bundle(prefix, t)
    (tmp_path / "checkpoint").write_text('model_checkpoint_path: "model.ckpt-7"\n')
    assert ckpt.latest_checkpoint(str(tmp_path)) == prefix
    assert dict(ckpt.list_variables(prefix)) == {k: v.shape for k, v in t.items()}
    got = ckpt.read_checkpoint(prefix)
    for k, v in t.items():
        np.testing.assert_array_equal(got[k], v)


def test_shim_load_checkpoint_scopes(tmp_path):
    """Tacotron.load_checkpoint restores only the scoped variables, like the reference's
    Saver(var_list=[v ... if 'refnet_emt' in v.name]).restore (tacotron/train.py:284)."""
    from tacotron.models import create_model
    hp = full_hparams()
    model = create_model("Tacotron", hp)
    model.init_random_weights(seed=1)
    before = dict(model._weights)
    rng = np.random.default_rng(2)
    k1 = "Tacotron_model/inference/refnet_emt/dense/kernel"
    k2 = "Tacotron_model/inference/refnet_spk/dense/kernel"
    new = {k1: rng.standard_normal(before[k1].shape).astype(np.float32),
           k2: rng.standard_normal(before[k2].shape).astype(np.float32)}
    write_bundle(str(tmp_path / "m.ckpt-1"), new)
    (tmp_path / "checkpoint").write_text('model_checkpoint_path: "m.ckpt-1"\n')
    restored = model.load_checkpoint(str(tmp_path), scopes=["refnet_emt"])
    assert restored == [k1]
    np.testing.assert_array_equal(model._weights[k1], new[k1])
    np.testing.assert_array_equal(model._weights[k2], before[k2])
    bad = {k1: np.zeros((3, 3), np.float32)}
    write_bundle(str(tmp_path / "bad.ckpt-1"), bad)
    with pytest.raises(ValueError):
        model.load_checkpoint(str(tmp_path / "bad.ckpt-1"))


@pytest.mark.skipif(not os.path.isdir(REF_CKPTS["refnet_emt"]), reason="reference checkout not present")
def test_reference_refnet_checkpoints_map_onto_model():
    from tt2 import ckpt
    from tt2.weights import init_tacotron_weights
    W = init_tacotron_weights(full_hparams())
    for scope, d in REF_CKPTS.items():
        prefix = ckpt.latest_checkpoint(d)
        vals = ckpt.read_checkpoint(prefix)
        ours = {k: v for k, v in vals.items() if "/%s/" % scope in k}
        assert len(ours) == 42
        for k, v in ours.items():
            assert k in W and W[k].shape == v.shape, k
            assert np.isfinite(v).all()
    emt = ckpt.read_checkpoint(ckpt.latest_checkpoint(REF_CKPTS["refnet_emt"]))
    with np.load(FIXTURE) as z:
        assert set(z.files) == {k for k in emt if "/refnet_emt/" in k}
        for k in z.files:
            np.testing.assert_array_equal(z[k], emt[k])


def test_oracle_refnet_on_trained_weights():
    """The trained refnet_emt (fixture) through the oracle's ReferenceEncoder: finite output in
    (-1, 1) (dense tanh, modules.py:63) that differs between two different reference mels."""
    from oracle import tacotron_ref as TR
    with np.load(FIXTURE) as z:
        W = {k: z[k] for k in z.files}
    rng = np.random.default_rng(3)
    mel = rng.uniform(-4, 4, (2, 96, 80)).astype(np.float32)
    out = TR.reference_encoder(mel, W, "refnet_emt/")
    assert out.shape == (2, 128) and np.isfinite(out).all() and np.abs(out).max() < 1
    assert np.abs(out[0] - out[1]).max() > 1e-3
