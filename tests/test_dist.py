"""Multi-process (gloo, world_size 2) tests of utterance-batch sharding (tt2/parallel.py).

The MI355X path shards utterances across ranks with no data-path collective and all-gathers the
padded outputs once at the end.  Here each rank runs the oracle on its shard
(stand-in for the device path, which needs a GPU) and the gathered result must equal the
single-process run over the whole batch, utterance by utterance."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tt2.parallel import shard, shard_range


def test_shard_range_covers_exactly():
    for n in range(0, 23):
        for w in range(1, 9):
            got = [shard_range(n, r, w) for r in range(w)]
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(got[i][1] == got[i + 1][0] for i in range(w - 1))
            sizes = [e - s for s, e in got]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "tacotron-2_amd"), root, os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from _common import small_hparams
    from oracle import tacotron_ref as TR
    from oracle.hp import oracle_hp
    from tt2.parallel import gather_padded, shard, shard_range
    from tt2.synthetic import prenet_masks, tacotron_inputs
    from tt2.weights import init_tacotron_weights

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hp = small_hparams()
        W = init_tacotron_weights(hp, seed=5339)
        B, n = 5, 9
        ids, lens, re, rs = tacotron_inputs(B, 12, 40, seed=13)
        masks = prenet_masks(n, B, hp.prenet_layers[0], seed=13)    # [n, 2, B, P]
        ids_r, lens_r, re_r, rs_r = shard([ids, lens, re, rs], rank, world)
        s, e = shard_range(B, rank, world)
        out = TR.synthesize(ids_r, lens_r, re_r, rs_r, W, oracle_hp(hp), masks[:, :, s:e], n)
        mel = out["mel_outputs"]
        lengths = np.full((mel.shape[0],), mel.shape[1], np.int64)
        got = gather_padded(mel, lengths)
        if rank == 0:
            np.savez(os.path.join(out_dir, "gathered.npz"), *got)
    finally:
        dist.destroy_process_group()


def test_gloo_world2_sharded_synthesis_matches_single_process(tmp_path):
    from _common import small_hparams
    from oracle import tacotron_ref as TR
    from oracle.hp import oracle_hp
    from tt2.synthetic import prenet_masks, tacotron_inputs
    from tt2.weights import init_tacotron_weights

    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    with np.load(str(tmp_path / "gathered.npz"), allow_pickle=False) as z:
        got = [z["arr_{}".format(i)] for i in range(len(z.files))]
    hp = small_hparams()
    W = init_tacotron_weights(hp, seed=5339)
    B, n = 5, 9
    ids, lens, re, rs = tacotron_inputs(B, 12, 40, seed=13)
    masks = prenet_masks(n, B, hp.prenet_layers[0], seed=13)
    ref = TR.synthesize(ids, lens, re, rs, W, oracle_hp(hp), masks, n)["mel_outputs"]
    assert len(got) == B
    for b in range(B):
        np.testing.assert_allclose(got[b], ref[b], rtol=0, atol=1e-5)


def test_shard_arrays_none_passthrough():
    a = np.arange(10).reshape(5, 2)
    x, y = shard([a, None], 1, 2)
    np.testing.assert_array_equal(x, a[3:])
    assert y is None


class _StubTTS(object):
    """CPU stand-in for tt2.e2e.TextToSpeech (the device path needs a GPU): utterance i gets a
    waveform of length 3 * (sum of its ids) % 17 + 1 whose samples encode its ids."""
    import torch
    torch_device = torch.device("cpu")

    def synthesize(self, ids, lengths, ref_emt, ref_spk, seed=0):
        wavs = []
        for b in range(ids.shape[0]):
            n = 3 * int(ids[b, :lengths[b]].sum()) % 17 + 1
            wavs.append(np.arange(n, dtype=np.float32) + float(ids[b, 0]))
        return dict(wavs=wavs)

    def synthesize_dev(self, ids_d, lens_d, lens_h, re_d, rs_d, seed=0, **noise):
        """Same waveforms as synthesize(), returned like TextToSpeech.synthesize_dev (padded
        tensor + per-row audio lengths)."""
        import torch
        wavs = self.synthesize(ids_d.numpy(), lens_h, None, None, seed)["wavs"]
        wav = torch.zeros((len(wavs), max(w.shape[0] for w in wavs)))
        for i, w in enumerate(wavs):
            wav[i, :w.shape[0]] = torch.from_numpy(w)
        return dict(wav=wav, audio_lengths=np.array([w.shape[0] for w in wavs], np.int64))


def _e2e_worker(rank, world, port, out_dir, B=5):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "tacotron-2_amd"), root, os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from test_dist import _StubTTS
    from tt2.e2e import synthesize_sharded
    from tt2.synthetic import tacotron_inputs
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids, lens, re, rs = tacotron_inputs(B, 9, 4, seed=21)
        got = synthesize_sharded(_StubTTS(), ids, lens, re, rs)
        np.savez(os.path.join(out_dir, "r{}.npz".format(rank)), *got)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,B", [(2, 5), (3, 5), (8, 8)])
def test_gloo_sharded_e2e_gathers_in_global_order(tmp_path, world, B):
    """tt2.e2e.synthesize_sharded: every rank ends with the trimmed waveforms of ALL utterances in
    global order (ragged lengths, uneven shards: 5 utterances over 2 or 3 ranks; configs[3]'s shape,
    8 utterances over 8 ranks, one per rank)."""
    from tt2.synthetic import tacotron_inputs
    mp.start_processes(_e2e_worker, args=(world, _free_port(), str(tmp_path), B), nprocs=world,
                       join=True, start_method="spawn")
    ids, lens, re, rs = tacotron_inputs(B, 9, 4, seed=21)
    ref = _StubTTS().synthesize(ids, lens, re, rs)["wavs"]
    for r in range(world):
        with np.load(str(tmp_path / "r{}.npz".format(r)), allow_pickle=False) as z:
            got = [z["arr_{}".format(i)] for i in range(len(z.files))]
        assert len(got) == B
        for g, w in zip(got, ref):
            np.testing.assert_array_equal(g, w)


def _train_worker(rank, world, port, out_dir):
    """Each rank = one tower: oracle gradients on its shard of the batch, flattened in the
    library's variable order, tower-averaged with tt2.parallel.tower_mean_ over gloo."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "tacotron-2_amd"), root, os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from _common import small_hparams
    from oracle import train_ref as TRN
    from tt2.parallel import shard, shard_range, tower_mean_
    from tt2.synthetic import prenet_masks, train_batch, zoneout_masks
    from tt2.weights import init_tacotron_weights, memory_width
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hp = small_hparams()
    W = init_tacotron_weights(hp, seed=5339)
    B, T_in, T = 4, 7, 5
    mem, lens, tg, st = train_batch(B, T_in, T, memory_width(hp), seed=3)
    pm = prenet_masks(T, B, hp.prenet_layers[0], seed=3)
    zm = zoneout_masks(T, B, hp.decoder_lstm_units, seed=3)
    m, l, t, s = shard([mem, lens, tg, st], rank, world)
    sl = slice(*shard_range(B, rank, world))
    _, _, g = TRN.train_grads(W, m, l, t, s, pm[:, :, sl], zm[:, :, sl], hp.tacotron_reg_weight)
    flat = torch.from_numpy(np.concatenate([g[n].ravel() for n in TRN.train_var_names()]))
    tower_mean_(flat)
    np.save(os.path.join(out_dir, "grads_{}.npy".format(rank)), flat.numpy())
    dist.destroy_process_group()


def test_train_tower_mean_over_two_ranks(tmp_path):
    """world_size 2 (gloo): the all-reduced flat gradients equal the reference's tower mean —
    the average of the two towers' gradients computed separately — on every rank."""
    import sys
    from _common import small_hparams
    from oracle import train_ref as TRN
    from tt2.synthetic import prenet_masks, train_batch, zoneout_masks
    from tt2.weights import init_tacotron_weights, memory_width
    world = 2
    mp.spawn(_train_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    hp = small_hparams()
    W = init_tacotron_weights(hp, seed=5339)
    B, T_in, T = 4, 7, 5
    mem, lens, tg, st = train_batch(B, T_in, T, memory_width(hp), seed=3)
    pm = prenet_masks(T, B, hp.prenet_layers[0], seed=3)
    zm = zoneout_masks(T, B, hp.decoder_lstm_units, seed=3)
    towers = []
    for r in range(world):
        s, e = shard_range(B, r, world)
        _, _, g = TRN.train_grads(W, mem[s:e], lens[s:e], tg[s:e], st[s:e], pm[:, :, s:e],
                                  zm[:, :, s:e], hp.tacotron_reg_weight)
        towers.append(np.concatenate([g[n].ravel() for n in TRN.train_var_names()]))
    want = (towers[0] + towers[1]) / 2
    for r in range(world):
        got = np.load(str(tmp_path / "grads_{}.npy".format(r)))
        np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-15)
