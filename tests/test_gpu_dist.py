"""The multi-GPU PRODUCT path (tt2.e2e.synthesize_sharded, TacotronTrainer.allreduce_grads) run as
two gloo ranks that share the one GPU of the test box, against single-process runs of the same
library (the world>1 branches had only run with the oracle standing in).

* configs[3]-shaped end-to-end text -> mel -> wav, utterances sharded 2 + 2 over the ranks with the
  global injected noise sliced per rank, one all_gather: every gathered waveform equals the
  single-process full-batch run.
* One data-parallel training step: each rank forward/backward on its tower, the tower mean as an
  all-reduce of the flat gradient buffer, clipped Adam: the updated parameters equal a single
  process that averages the two towers' device gradients itself, and they moved at step 1; the
  batch-norm moving statistics are the per-shard updates composed in rank order (as the
  reference's towers update one shared variable) and equal on both ranks.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, T_IN, T_REF, MAX_IT = 4, 15, 32, 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _paths():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "tacotron-2_amd"), root, os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _e2e_case():
    from tt2.e2e import e2e_hparams
    from tt2.synthetic import mol_uniforms, prenet_masks, tacotron_inputs
    from tt2.weights import init_tacotron_weights, init_wavenet_weights
    hp = e2e_hparams(MAX_IT)
    W = init_tacotron_weights(hp, seed=5339)
    WW = init_wavenet_weights(hp, seed=5339)
    ids, lens, re, rs = tacotron_inputs(B, T_IN, T_REF, seed=51)
    pm = prenet_masks(MAX_IT, B, hp.prenet_layers[0], seed=51)
    um, ul = mol_uniforms(MAX_IT * 275, B, seed=51)
    return hp, W, WW, ids, lens, re, rs, pm, um, ul


def _train_case():
    from _common import small_hparams
    from tt2.synthetic import postnet_masks, prenet_masks, train_batch, zoneout_masks
    from tt2.weights import init_tacotron_weights, memory_width
    hp = small_hparams()
    W = init_tacotron_weights(hp, seed=5339)
    T_in, T = 9, 7
    mem, lens, tg, st = train_batch(B, T_in, T, memory_width(hp), seed=52)
    pm = prenet_masks(T, B, hp.prenet_layers[0], seed=52)
    zm = zoneout_masks(T, B, hp.decoder_lstm_units, seed=52)
    pnm = postnet_masks(hp.postnet_num_layers, B, T, hp.postnet_channels, seed=52)
    return hp, W, T_in, T, (mem, lens, tg, st, pm, zm, pnm)


def _tower(batch, s, e):
    mem, lens, tg, st, pm, zm, pnm = batch
    return (mem[s:e], lens[s:e], tg[s:e], st[s:e], pm[:, :, s:e], zm[:, :, s:e], pnm[:, s:e])


VAR = "Tacotron_model/inference/decoder/decoder_LSTM/multi_rnn_cell/cell_0/lstm_cell/kernel"
BNM = ("Tacotron_model/inference/postnet_convolutions/conv_layer_1_postnet_convolutions/"
       "batch_normalization/moving_mean")


def _worker(rank, world, port, out_dir):
    _paths()
    import torch.distributed as dist
    from tt2.e2e import TextToSpeech, synthesize_sharded
    from tt2.parallel import shard_range
    from tt2.train import TacotronTrainer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hp, W, WW, ids, lens, re, rs, pm, um, ul = _e2e_case()
        tts = TextToSpeech(hp, W, WW, B, T_IN, T_REF, MAX_IT, 0)
        wavs = synthesize_sharded(tts, ids, lens, re, rs, seed=3, u_mix=um, u_log=ul,
                                  prenet_masks=pm)
        tts.close()
        np.savez(os.path.join(out_dir, "wavs_{}.npz".format(rank)), *wavs)
        thp, TW, T_in, T, batch = _train_case()
        s, e = shard_range(B, rank, world)
        tr = TacotronTrainer(thp, TW, e - s, T_in, T, 0)
        L = tr.step(*_tower(batch, s, e))
        np.save(os.path.join(out_dir, "param_{}.npy".format(rank)),
                tr.get(VAR, 0, np.asarray(TW[VAR]).shape))
        np.save(os.path.join(out_dir, "loss_{}.npy".format(rank)), np.array([L["loss"]]))
        np.save(os.path.join(out_dir, "bnm_{}.npy".format(rank)), tr.get(BNM, 0, (thp.postnet_channels,)))
        tr.close()
    finally:
        dist.destroy_process_group()


def test_gloo_world2_product_path_on_one_gpu(tmp_path):
    import torch
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    from tt2.e2e import TextToSpeech
    from tt2.train import TacotronTrainer
    # end to end: the single-process full batch with the same (global) injected noise
    hp, W, WW, ids, lens, re, rs, pm, um, ul = _e2e_case()
    tts = TextToSpeech(hp, W, WW, B, T_IN, T_REF, MAX_IT, 0)
    ref = tts.synthesize(ids, lens, re, rs, seed=3, u_mix=um, u_log=ul, prenet_masks=pm)["wavs"]
    tts.close()
    for r in range(world):
        with np.load(str(tmp_path / "wavs_{}.npz".format(r)), allow_pickle=False) as z:
            got = [z["arr_{}".format(i)] for i in range(len(z.files))]
        assert len(got) == B
        for g, w in zip(got, ref):
            assert g.shape == w.shape and g.shape[0] > 0
            np.testing.assert_allclose(g, w, atol=1e-5)
    # training: average the two towers' device gradients by hand, one clipped Adam update
    thp, TW, T_in, T, batch = _train_case()
    tr = TacotronTrainer(thp, TW, B // 2, T_in, T, 0)
    grads = []
    for s, e in ((0, B // 2), (B // 2, B)):
        tr.forward_backward(*_tower(batch, s, e))
        torch.cuda.synchronize()
        grads.append(tr.grad_buf.clone())
    tr.grad_buf.copy_((grads[0] + grads[1]) / 2)
    torch.cuda.synchronize()
    tr.apply(1)
    want = tr.get(VAR, 0, np.asarray(TW[VAR]).shape)
    tr.close()
    assert np.abs(want - TW[VAR]).max() > 1e-5          # step 1 moved the parameters
    for r in range(world):
        got = np.load(str(tmp_path / "param_{}.npy".format(r)))
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-6)
    # BN moving statistics: the reference's towers compose their updates of ONE variable; with the
    # rank order m2 = mu·(mu·m0 + (1-mu)·x0) + (1-mu)·x1 = mu·u0 + u1 - mu·m0 for the single-tower
    # updates u_k (sync_moving_stats); identical on both ranks
    per_tower = []
    for s, e in ((0, B // 2), (B // 2, B)):
        t1 = TacotronTrainer(thp, TW, B // 2, T_in, T, 0)
        t1.forward_backward(*_tower(batch, s, e))
        t1.apply(1)
        per_tower.append(t1.get(BNM, 0, (thp.postnet_channels,)))
        t1.close()
    assert np.abs(per_tower[0] - per_tower[1]).max() > 1e-6   # the shards' statistics differ
    bn = [np.load(str(tmp_path / "bnm_{}.npy".format(r))) for r in range(world)]
    np.testing.assert_array_equal(bn[0], bn[1])
    mu, m0 = 0.99, np.asarray(TW[BNM], np.float64)
    np.testing.assert_allclose(bn[0], mu * per_tower[0] + per_tower[1] - mu * m0, rtol=0, atol=1e-6)


def _nccl_worker(rank, port, q):
    """One rank, backend "nccl" (RCCL): the device branches of gather_padded and tower_mean_ and
    TacotronTrainer.sync_moving_stats' collective, which only the RCCL backend takes."""
    _paths()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from tt2.parallel import gather_padded, tower_mean_
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        rng = np.random.default_rng(3)
        x = rng.normal(size=(3, 7, 5)).astype(np.float32)
        lens = np.array([7, 2, 5])
        xd = torch.from_numpy(x).cuda()
        got = gather_padded(xd, lens)                       # RCCL all_gather of device tensors
        ok_gather = len(got) == 3 and all(np.array_equal(g, x[i, :lens[i]]) for i, g in enumerate(got))
        g = torch.arange(1000, dtype=torch.float32, device="cuda")
        tower_mean_(g)                                      # RCCL all_reduce SUM / world, in place
        torch.cuda.synchronize()
        ok_reduce = bool(torch.equal(g.cpu(), torch.arange(1000, dtype=torch.float32)))
        q.put((ok_gather, ok_reduce, dist.get_backend()))
    finally:
        dist.destroy_process_group()


def test_rccl_backend_paths_one_rank():
    """The "nccl" (RCCL) branches of the multi-GPU helpers execute on the device: a one-rank process
    group on the box's GPU (two ranks cannot share one GPU under RCCL; the two-rank product path
    above runs on gloo)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(0, _free_port(), q))
    p.start()
    p.join(120)
    assert p.exitcode == 0, p.exitcode
    ok_gather, ok_reduce, backend = q.get(timeout=5)
    assert backend == "nccl" and ok_gather and ok_reduce


N_FORK = 60


def _fork_worker(rank, world, port, out_dir):
    _paths()
    import torch.distributed as dist
    from _common import fork_e2e_case
    from tt2.e2e import TextToSpeech, synthesize_sharded
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hp, W, WW, ids, lens, re, rs, pm, um, ul = fork_e2e_case(N_FORK, B=4)
        tts = TextToSpeech(hp, W, WW, 2, ids.shape[1], re.shape[1], N_FORK, 0)
        wavs = synthesize_sharded(tts, ids, lens, re, rs, seed=3, u_mix=um, u_log=ul,
                                  prenet_masks=pm)
        path = tts.taco.decoder_path()[0]
        tts.close()
        np.savez(os.path.join(out_dir, "fork_{}.npz".format(rank)), np.array([path]), *wavs)
    finally:
        dist.destroy_process_group()


def test_gloo_world2_configs3_fork_widths(tmp_path):
    """configs[3] at the fork widths (4 utterances of 136-201 characters, 60 decoder steps on the
    persistent decoder, 16,500 samples each) sharded 2 + 2 over two gloo ranks sharing the GPU:
    every gathered waveform equals the single-process full-batch run."""
    world = 2
    mp.start_processes(_fork_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    from _common import fork_e2e_case
    from tt2.e2e import TextToSpeech
    hp, W, WW, ids, lens, re, rs, pm, um, ul = fork_e2e_case(N_FORK, B=4)
    tts = TextToSpeech(hp, W, WW, 4, ids.shape[1], re.shape[1], N_FORK, 0)
    ref = tts.synthesize(ids, lens, re, rs, seed=3, u_mix=um, u_log=ul, prenet_masks=pm)["wavs"]
    tts.close()
    for r in range(world):
        with np.load(str(tmp_path / "fork_{}.npz".format(r)), allow_pickle=False) as z:
            assert int(z["arr_0"][0]) == 1              # the persistent decoder served each shard
            got = [z["arr_{}".format(i)] for i in range(1, len(z.files))]
        assert len(got) == 4
        for g, w in zip(got, ref):
            assert g.shape == w.shape == (N_FORK * 275,)
            np.testing.assert_allclose(g, w, atol=1e-5)
