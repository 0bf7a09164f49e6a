"""WaveNet (code/wavenet_vocoder/models/wavenet.py:86-923), synthesis path on MI355X.

``initialize`` / ``incremental`` keep the reference signatures and run eagerly through libtt2.so
(upsampling network + fast-WaveNet incremental generation + MoL sampler); the results land in
``tower_y_hat`` / ``tower_synth_upsampled_local_features`` like the reference's graph outputs.
"""
import os

import numpy as np

from tt2.engine import WaveNetEngine
from tt2.hparams import get_hop_size
from tt2.weights import init_wavenet_weights
from wavenet_vocoder.util import inv_mulaw, is_mulaw, is_mulaw_quantize, is_scalar_input


def receptive_field_size(total_layers, num_cycles, kernel_size, dilation=lambda x: 2 ** x):
    """wavenet.py:54-71."""
    assert total_layers % num_cycles == 0
    layers_per_cycle = total_layers // num_cycles
    dilations = [dilation(i % layers_per_cycle) for i in range(total_layers)]
    return (kernel_size - 1) * sum(dilations) + 1


class WaveNet():
    """Tacotron-2 Wavenet Vocoder model."""

    def __init__(self, hparams, init):
        self._hparams = hparams
        if self.local_conditioning_enabled():
            assert hparams.num_mels == hparams.cin_channels
        assert hparams.layers % hparams.stacks == 0
        self.scalar_input = is_scalar_input(hparams.input_type)
        self.receptive_field = receptive_field_size(hparams.layers, hparams.stacks,
                                                    hparams.kernel_size)
        self._weights = None
        self._engine = None
        self.device = int(os.environ.get("TT2_DEVICE", os.environ.get("LOCAL_RANK", "0")))

    def local_conditioning_enabled(self):
        return self._hparams.cin_channels > 0

    def global_conditioning_enabled(self):
        return self._hparams.gin_channels > 0

    def has_speaker_embedding(self):
        return False

    # -- weights (replaces create_shadow_saver/load_averaged_model, wavenet_vocoder/train.py:67-86)
    def load_weights(self, weights):
        if isinstance(weights, str):
            with np.load(weights, allow_pickle=False) as z:
                weights = {k: z[k] for k in z.files}
        self._weights = dict(weights)
        self._engine = None

    def load_checkpoint(self, checkpoint):
        """create_shadow_saver + load_averaged_model (wavenet_vocoder/train.py:67-86) without
        TensorFlow: every model variable <v> is restored from the bundle's EMA shadow
        ``<v>/ExponentialMovingAverage`` (falling back to <v> itself when the bundle holds no
        shadow, e.g. a plain Saver checkpoint).  Returns the restored model names."""
        from tt2 import ckpt
        prefix = ckpt.latest_checkpoint(checkpoint) if os.path.isdir(checkpoint) else checkpoint
        avail = dict(ckpt.list_variables(prefix))
        if self._weights is None:
            self.init_random_weights()
        want = {}
        for n in self._weights:
            sh = n + "/ExponentialMovingAverage"
            if sh in avail:
                want[sh] = n
            elif n in avail:
                want[n] = n
        values = ckpt.read_checkpoint(prefix, set(want))
        for src, v in values.items():
            n = want[src]
            if self._weights[n].shape != v.shape:
                raise ValueError("checkpoint variable {} has shape {}, model expects {}".format(
                    src, v.shape, self._weights[n].shape))
            self._weights[n] = v.astype(np.float32)
        self._engine = None
        return sorted(want.values())

    def init_random_weights(self, seed=None):
        hp = self._hparams
        self.load_weights(init_wavenet_weights(hp, hp.wavenet_random_seed if seed is None else seed))

    def _check_path(self):
        hp = self._hparams
        if not is_scalar_input(hp.input_type) and hp.out_channels != hp.quantize_channels:
            raise ValueError("mulaw-quantize: out_channels must equal quantize_channels (hparams.py:222)")

    def _get_engine(self, B, T):
        if self._weights is None:
            raise RuntimeError("WaveNet weights not loaded: call load_weights() or "
                               "init_random_weights()")
        e = self._engine
        if e is None or not e.fits(B, T):
            if e is not None:
                e.close()
            self._engine = None
            e = WaveNetEngine(self._hparams, self._weights, max(B, 1), T, self.device)
            self._engine = e
        return e

    def initialize(self, y, c, g, input_lengths, x=None, synthesis_length=None, test_inputs=None,
                   split_infos=None, u_mix=None, u_log=None, seed=0):
        """wavenet.py:218-473 (synthesis branch :408-465).  c: [B, T_frames, cin] conditioning,
        already clipped + _interp'd by the caller (wavenet_vocoder/synthesizer.py:63-70).
        u_mix [T,B,10] / u_log [T,B] inject the MoL sampler's uniforms (None = device RNG);
        'mulaw-quantize': u_log [T,B] the uniforms of tf.multinomial, y the drawn class through
        inv_mulaw_quantize (wavenet.py:450-452), test_inputs class indices."""
        hp = self._hparams
        self.is_training = x is not None
        self.is_evaluating = not self.is_training and y is not None
        if self.is_training or self.is_evaluating:
            raise NotImplementedError("WaveNet training / eval-loss graphs are not on the synthesis "
                                      "path")
        self._check_path()
        if c is None:   # wavenet.py:410-411: synthesis_length samples without a local condition
            if self.local_conditioning_enabled():
                raise ValueError("cin_channels > 0: the local condition c is required")
            if synthesis_length is None:
                raise ValueError("unconditional synthesis needs synthesis_length")
            B = 1 if test_inputs is None else np.asarray(test_inputs).reshape(
                -1, int(synthesis_length)).shape[0]
            if g is not None:
                B = np.asarray(g).reshape(-1, max(hp.gin_channels, 1) if not np.issubdtype(
                    np.asarray(g).dtype, np.integer) else 1).shape[0]
            T = int(synthesis_length)
            ti = None if test_inputs is None else np.asarray(test_inputs, np.float32).reshape(B, T)
            out = self._get_engine(B, T).generate_unconditional(
                B, T, u_mix, u_log, seed, ti, g=g if self.global_conditioning_enabled() else None)
            y = out["y"]
            if is_mulaw(hp.input_type):
                y = inv_mulaw(y, hp.quantize_channels).astype(np.float32)
            self.tower_y_hat = [y]
            self.tower_synth_upsampled_local_features = [None]
            self.tower_mix_indices = [out["k"]]
            return
        c = np.asarray(c, np.float32)
        if c.ndim != 3 or c.shape[2] != hp.cin_channels:
            raise ValueError('Expected 3 dimension shape [batch_size(1), time_length, {}] for local '
                             'condition features but found {}'.format(hp.cin_channels, c.shape))
        if self.global_conditioning_enabled() and g is None:
            raise ValueError("gin_channels > 0 needs the global condition g (speaker ids)")
        ntow = hp.wavenet_num_gpus
        cs = np.split(c, ntow, axis=0) if ntow > 1 else [c]
        gs = [None] * ntow if not self.global_conditioning_enabled() else \
            np.split(np.asarray(g).reshape(c.shape[0], -1), ntow, axis=0)
        tis = ([None] * ntow if test_inputs is None else
               np.split(np.asarray(test_inputs, np.float32).reshape(c.shape[0], -1), ntow, axis=0))
        self.tower_y_hat = []
        self.tower_synth_upsampled_local_features = []
        self.tower_mix_indices = []
        hop = get_hop_size(hp)
        for i, ci in enumerate(cs):
            B, T_f, _ = ci.shape
            T = T_f * hop
            um = ul = None
            if u_mix is not None:
                um = np.asarray(u_mix, np.float32)[:, i * B:(i + 1) * B]
                ul = np.asarray(u_log, np.float32)[:, i * B:(i + 1) * B]
            out = self._get_engine(B, T).generate(ci, um, ul, seed, tis[i], want_upsampled=True,
                                                  g=gs[i])
            y = out["y"]
            if is_mulaw(hp.input_type):  # wavenet.py:459-460: samples are companded, expand them
                y = inv_mulaw(y, hp.quantize_channels).astype(np.float32)
            self.tower_y_hat.append(y)
            self.tower_synth_upsampled_local_features.append(out["upsampled"])
            self.tower_mix_indices.append(out["k"])

    def incremental(self, initial_input, c=None, g=None, time_length=100, test_inputs=None,
                    softmax=True, quantize=True, log_scale_min=-7.0, log_scale_min_gauss=-7.0,
                    u_mix=None, u_log=None, seed=0, return_logits=False):
        """wavenet.py:724-911: returns generated samples [B, 1, T] (the reference returns
        [batch_size, channels, time_length]).  c: [B, cin, T_frames] (channels first, as the
        reference passes it at wavenet.py:427) — upsampled inside, like the reference."""
        self._check_path()
        hp = self._hparams
        if not is_scalar_input(hp.input_type):
            # one_hot(mulaw_quantize(0)) = class 127 (wavenet.py:433-446)
            if initial_input is not None:
                ii = np.asarray(initial_input).reshape(-1, hp.quantize_channels)
                if not np.all(np.argmax(ii, 1) == 127) or not np.all(ii.sum(1) == 1):
                    raise NotImplementedError("initial_input must be one_hot(mulaw_quantize(0))")
        elif initial_input is not None and np.any(np.asarray(initial_input) != 0):
            # the start silence of both scalar input types: 0.0 ('raw'), mulaw(0.0) = 0 ('mulaw')
            raise NotImplementedError("initial_input must be the silence value 0")
        if c is None:
            B = np.asarray(initial_input).shape[0] if initial_input is not None else 1
            out = self._get_engine(B, int(time_length)).generate_unconditional(
                B, int(time_length), u_mix, u_log, seed,
                None if test_inputs is None else np.asarray(test_inputs, np.float32).reshape(B, -1),
                want_logits=return_logits, g=g if self.global_conditioning_enabled() else None)
            self.upsampled_local_features = None
            y = self._incremental_outputs(out)
            return (y, out["logits"]) if return_logits else y
        if abs(log_scale_min - self._hparams.log_scale_min) > 1e-6:
            raise ValueError("log_scale_min must equal hparams.log_scale_min on this build")
        c = np.asarray(c, np.float32).transpose(0, 2, 1)
        out = self._get_engine(c.shape[0], c.shape[1] * get_hop_size(self._hparams)).generate(
            c, u_mix, u_log, seed,
            None if test_inputs is None else np.asarray(test_inputs, np.float32).reshape(c.shape[0], -1),
            want_logits=return_logits, want_upsampled=True,
            g=g if self.global_conditioning_enabled() else None)
        self.upsampled_local_features = out["upsampled"]
        y = self._incremental_outputs(out)
        return (y, out["logits"]) if return_logits else y

    def _incremental_outputs(self, out):
        """[B, channels, T]: the samples ([B, 1, T]) or, for 'mulaw-quantize', the one-hot draws
        [B, quantize_channels, T] (wavenet.py:866-874, 911)"""
        hp = self._hparams
        if is_scalar_input(hp.input_type):
            return out["y"][:, None, :]
        k = out["k"]
        oh = np.zeros((k.shape[0], hp.quantize_channels, k.shape[1]), np.float32)
        np.put_along_axis(oh, k[:, None, :].astype(np.int64), 1.0, axis=1)
        return oh
