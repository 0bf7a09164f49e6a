"""End-to-end text -> mel -> wav on one device, and utterance-sharded over ranks (BASELINE.json
configs[3]).

The reference runs the two models one after the other through files: ``synthesize.py:33-43``
calls ``tacotron_synthesize`` (mels written as ``mel-*.npy`` + ``map.txt``), resets the TF graph,
then ``wavenet_synthesize`` reads them back (``wavenet_vocoder/synthesize.py:20-62``).  Here the
hand-off stays in HBM: the Tacotron engine's mels and stop tokens feed two small device kernels
(``tt2_output_lengths_dev`` = ``get_output_lengths``, tacotron/synthesizer.py:384-387;
``tt2_wn_cond_from_mels_dev`` = clip + pad + ``_interp``, wavenet_vocoder/synthesizer.py:56-70)
and the WaveNet engine generates from that buffer.  The only host round trip is the per-row
length vector (its maximum sizes the WaveNet run, as ``maxlen`` does at synthesizer.py:56).

Sharding (``synthesize_sharded``): rank r takes utterances ``shard_range(n, r, world)``, runs the
whole chain locally, and one all_gather (RCCL over xGMI under backend ``nccl``) collects the
trimmed waveforms — the reference's per-tower split (tacotron.py:83-138, wavenet.py:227-239) with
no exchange during compute.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check
from .engine import MAX_CONTEXT_BATCH, TacotronEngine, WaveNetEngine
from .hparams import bench_wavenet_hparams, get_hop_size


def e2e_hparams(max_iters=1000):
    """configs[3]: the fork's Tacotron-2 architecture (identical in paper_hparams) with the
    paper_hparams audio/WaveNet settings of configs[2] (hop 275, 22.05 kHz, 24-layer MoL WaveNet
    at R=64); ``max_iters`` = the decoder step cap."""
    hp = bench_wavenet_hparams()
    hp.override_from_dict(dict(max_iters=max_iters, tacotron_num_gpus=1, wavenet_num_gpus=1))
    return hp


def output_range(hp):
    """T2_output_range (tacotron/synthesizer.py:108-109, wavenet_vocoder/synthesizer.py:59)."""
    return (-hp.max_abs_value, hp.max_abs_value) if hp.symmetric_mels else (0.0, hp.max_abs_value)


class TextToSpeech(object):
    """Tacotron-2 + WaveNet on one device with the mel hand-off in HBM.

    ``synthesize_dev`` works on torch CUDA tensors (device pointers) and returns device outputs;
    ``synthesize`` is the host-array convenience wrapper.
    """

    def __init__(self, hp, taco_weights, wn_weights, max_batch, max_T_in, max_T_ref, max_iters,
                 device=0, synthesis_constraint=False):
        if max_batch > MAX_CONTEXT_BATCH:
            # the device-resident chain drives one tt2_ctx; TacotronEngine splits larger towers
            raise ValueError("TextToSpeech holds at most {} rows per call (got {}); split the batch"
                             .format(MAX_CONTEXT_BATCH, max_batch))
        self.hp = hp
        self.device = device
        self.max_iters = max_iters
        self.taco = TacotronEngine(hp, taco_weights, max_batch, max_T_in, max_T_ref, max_iters,
                                   device, synthesis_constraint=synthesis_constraint)
        self.hop = get_hop_size(hp)
        if int(np.prod(hp.upsample_scales)) != self.hop:
            raise ValueError("prod(upsample_scales) != hop_size")
        self.wn = WaveNetEngine(hp, wn_weights, max_batch, max_iters * hp.outputs_per_step * self.hop,
                                device)
        self.lib = _lib.load_library()

    @property
    def torch_device(self):
        import torch
        return torch.device("cuda", self.device)

    def close(self):
        for e in (getattr(self, "taco", None), getattr(self, "wn", None)):
            if e is not None:
                e.close()
        self.taco = self.wn = None

    def synthesize_dev(self, ids_d, lens_d, lens_h, ref_emt_d, ref_spk_d, seed=0, stream=None,
                       max_iters=None, u_mix_d=None, u_log_d=None, prenet_masks_d=None):
        """ids_d [B,T_in] int32, lens_d [B] int32 (device) + lens_h (host copy), reference mels
        [B,T_ref,80] (device).  Returns dict(wav [B, T_f*hop] device tensor, lengths (host int
        array of mel frames per row), audio_lengths = lengths*hop, mel [B,n,80], stop [B,max_iters],
        n_steps = decoded frames, steps x outputs_per_step).  Everything between the two models stays
        on the device.  Injected randomness
        (parity runs): prenet_masks_d [max_iters,2,B,P] uint8 keep bits; u_mix_d [>=T,B,10] and
        u_log_d [>=T,B] MoL uniforms for T = max(lengths)*hop samples (t-major, so a buffer sized
        for max_iters*hop serves any decoded length).  None = the device RNGs keyed by ``seed``."""
        import torch
        dev = ids_d.device
        if stream is None:
            # one explicit stream for the whole chain: torch's default stream is the NULL handle,
            # which the library maps to each context's OWN non-blocking stream -- two contexts
            # (Tacotron, WaveNet) plus the hand-off kernels would then run unordered
            if getattr(self, "_stream", None) is None:
                self._stream = torch.cuda.Stream(dev)
            self._stream.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(self._stream):
                out = self.synthesize_dev(ids_d, lens_d, lens_h, ref_emt_d, ref_spk_d, seed,
                                          self._stream.cuda_stream, max_iters, u_mix_d, u_log_d,
                                          prenet_masks_d)
            torch.cuda.current_stream(dev).wait_stream(self._stream)
            return out
        hp = self.hp
        B, T_in = ids_d.shape
        mi = self.max_iters if max_iters is None else max_iters
        r = hp.outputs_per_step                   # r frames per decoder step (tacotron.py:322-324)
        st = ctypes.c_void_p(stream)
        lens_h = np.ascontiguousarray(lens_h, np.int32)
        mel = torch.empty((B, mi * r, hp.num_mels), dtype=torch.float32, device=dev)
        stop = torch.empty((B, mi * r), dtype=torch.float32, device=dev)
        n = ctypes.c_int32()
        check(self.lib.tt2_synthesize_dev(
            self.taco.h, ids_d.data_ptr(), lens_d.data_ptr(), _lib.ptr(lens_h), B, T_in,
            ref_emt_d.data_ptr(), ref_emt_d.shape[1],
            None if ref_spk_d is None else ref_spk_d.data_ptr(),
            0 if ref_spk_d is None else ref_spk_d.shape[1], mi,
            None if prenet_masks_d is None else prenet_masks_d.data_ptr(), seed, mel.data_ptr(),
            stop.data_ptr(), ctypes.byref(n), st))
        n = n.value * r                           # decoded frames
        lengths_d = torch.empty((B,), dtype=torch.int32, device=dev)
        check(self.lib.tt2_output_lengths_dev(stop.data_ptr(), B, n, mi * r, lengths_d.data_ptr(), st))
        lengths = lengths_d.cpu().numpy()  # the one host round trip (on this stream): sizes WaveNet
        T_f = int(lengths.max()) if B else 0
        wav = torch.zeros((B, max(T_f, 0) * self.hop), dtype=torch.float32, device=dev)
        cond = None
        if T_f > 0:
            lo, hi = output_range(hp)
            cond = torch.empty((B, hp.num_mels, T_f), dtype=torch.float32, device=dev)
            # mel_d of tt2_synthesize_dev is [B, n, 80] contiguous (row stride n frames)
            check(self.lib.tt2_wn_cond_from_mels_dev(
                mel.data_ptr(), n, lengths_d.data_ptr(), B, T_f, hp.num_mels, lo, hi,
                int(bool(hp.clip_for_wavenet)), int(bool(hp.normalize_for_wavenet)),
                cond.data_ptr(), st))
            check(self.lib.tt2_wn_generate_dev(
                self.wn.h, cond.data_ptr(), B, T_f,
                None if u_mix_d is None else u_mix_d.data_ptr(),
                None if u_log_d is None else u_log_d.data_ptr(), seed, None, wav.data_ptr(),
                None, None, st))
        return dict(wav=wav, lengths=lengths, audio_lengths=lengths.astype(np.int64) * self.hop,
                    mel=mel.view(-1)[:B * n * hp.num_mels].view(B, n, hp.num_mels), stop=stop,
                    n_steps=n, cond=cond)

    def synthesize(self, ids, lengths, ref_emt, ref_spk, seed=0, u_mix=None, u_log=None,
                   prenet_masks=None):
        """Host arrays in, list of trimmed waveforms (np.float32) + mel frame lengths out."""
        import torch
        dev = torch.device("cuda", self.device)
        ids_d = torch.from_numpy(np.ascontiguousarray(ids, np.int32)).to(dev)
        lens_h = np.ascontiguousarray(lengths, np.int32)
        lens_d = torch.from_numpy(lens_h).to(dev)
        re_d = torch.from_numpy(np.ascontiguousarray(ref_emt, np.float32)).to(dev)
        rs_d = None if ref_spk is None else \
            torch.from_numpy(np.ascontiguousarray(ref_spk, np.float32)).to(dev)
        um = None if u_mix is None else torch.from_numpy(np.ascontiguousarray(u_mix, np.float32)).to(dev)
        ul = None if u_log is None else torch.from_numpy(np.ascontiguousarray(u_log, np.float32)).to(dev)
        pm = None if prenet_masks is None else \
            torch.from_numpy(np.ascontiguousarray(prenet_masks, np.uint8)).to(dev)
        out = self.synthesize_dev(ids_d, lens_d, lens_h, re_d, rs_d, seed, u_mix_d=um, u_log_d=ul,
                                  prenet_masks_d=pm)
        torch.cuda.synchronize(dev)
        wav = out["wav"].cpu().numpy()
        wavs = [wav[b, :int(out["audio_lengths"][b])] for b in range(wav.shape[0])]
        return dict(wavs=wavs, lengths=out["lengths"], mel=out["mel"].cpu().numpy(),
                    stop=out["stop"][:, :out["n_steps"]].cpu().numpy(), n_steps=out["n_steps"],
                    cond=None if out["cond"] is None else out["cond"].cpu().numpy())


def synthesize_sharded(tts, ids, lengths, ref_emt, ref_spk, seed=0, group=None, u_mix=None,
                       u_log=None, prenet_masks=None):
    """Utterance-sharded text -> wav over torch.distributed ranks (each rank holds ``tts`` on its
    own GPU).  Every rank passes the SAME global batch; rank r synthesises its contiguous slice
    and one all_gather returns every rank the trimmed waveforms in global utterance order.  The
    waveforms stay on the device up to the collective (RCCL under "nccl").  Optional injected
    noise covers the GLOBAL batch and is sliced per rank: prenet_masks [max_iters,2,B,P],
    u_mix [T,B,10], u_log [T,B] (parity runs); None = the device RNGs keyed by ``seed + rank``."""
    import torch
    import torch.distributed as dist
    from .parallel import gather_padded, shard, shard_range
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    ids_r, len_r, re_r, rs_r = shard([np.asarray(ids), np.asarray(lengths), np.asarray(ref_emt),
                                      None if ref_spk is None else np.asarray(ref_spk)], rank, world)
    s, e = shard_range(np.asarray(ids).shape[0], rank, world)
    if ids_r.shape[0]:
        dev = tts.torch_device

        def up(a, dt):
            return None if a is None else torch.from_numpy(np.ascontiguousarray(a, dt)).to(dev)
        lens_h = np.ascontiguousarray(len_r, np.int32)
        out = tts.synthesize_dev(up(ids_r, np.int32), up(lens_h, np.int32), lens_h,
                                 up(re_r, np.float32), up(rs_r, np.float32), seed + rank,
                                 u_mix_d=None if u_mix is None else up(np.asarray(u_mix)[:, s:e], np.float32),
                                 u_log_d=None if u_log is None else up(np.asarray(u_log)[:, s:e], np.float32),
                                 prenet_masks_d=None if prenet_masks is None else
                                 up(np.asarray(prenet_masks)[:, :, s:e], np.uint8))
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        local, alen = out["wav"], out["audio_lengths"]
    else:
        local, alen = np.zeros((0, 1), np.float32), np.zeros((0,), np.int64)
    return gather_padded(local, alen, group=group)
