#!/usr/bin/env python
"""bench.py — MI355X throughput of the Tacotron-2 synthesis path (BASELINE.json).

Headline (``value``): mel-frames/s of Tacotron-2 encoder + decoder loop + Postnet inference on
configs[1] ("decoder+Postnet inference, batch=32x200-char synthetic, 1xMI355X"): one step = one full
synthesis of a 32-utterance batch (200 chars + EOS, T_out = 1000 decoder frames, random-init fp32
weights of the fork-default architecture, D_mem = 1024).  The ``wavenet`` object carries
configs[2] (24-layer R=64 MoL WaveNet, batch 1, 22.05 kHz): audio-samples/s.

Multi-GPU (``--gpus N``; bench.py starts the N ranks itself under torch.distributed.run when it is
not already one of them, and refuses a WORLD_SIZE that disagrees with --gpus): one rank per GPU,
each rank synthesises its own batch (utterance-batch sharding) — weak scaling, no collective in the timed
region; the timed region is bracketed by barrier + synchronize and the max over ranks is reported.
"""
import argparse
import json
import os
import sys
import time

import ctypes

if os.environ.get("TT2_DUMP_MAPS"):  # debug: the process's mappings at interpreter exit (maps native
    import atexit                    # backtrace addresses of an exit-time crash to libraries)
    atexit.register(lambda: open(os.environ["TT2_DUMP_MAPS"], "w").write(open("/proc/self/maps").read()))

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "tacotron-2_amd"), ROOT]

from tt2 import _lib  # noqa: E402

METRIC = "mel-frames/sec (decoder) + audio-samples/sec (WaveNet) @1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.29 TB/s measured copy


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--chars", type=int, default=200)
    p.add_argument("--ref-frames", type=int, default=400)
    p.add_argument("--t-out", type=int, default=1000)
    p.add_argument("--wavenet-frames", type=int, default=80, help="mel frames per WaveNet utterance")
    p.add_argument("--wavenet-steps", type=int, default=1)
    p.add_argument("--no-wavenet", action="store_true")
    p.add_argument("--no-wavenet-widths", action="store_true",
                   help="skip the R=128 / R=256 WaveNet legs (k_generate_wide)")
    p.add_argument("--no-e2e", action="store_true")
    p.add_argument("--e2e-frames", type=int, default=1000,
                   help="decoder frames per utterance of the end-to-end leg (configs[3])")
    p.add_argument("--no-griffin-lim", action="store_true")
    p.add_argument("--no-train", action="store_true")
    p.add_argument("--train-batch", type=int, default=64)
    p.add_argument("--train-t-in", type=int, default=150)
    p.add_argument("--train-t-out", type=int, default=800)
    p.add_argument("--train-steps", type=int, default=2)
    p.add_argument("--train-decoder-only", action="store_true",
                   help="time the decoder + Postnet slice from a given memory (round-1 leg) instead "
                        "of the whole step from ids + reference mels")
    p.add_argument("--train-t-ref", type=int, default=800, help="reference mel frames (configs[4])")
    p.add_argument("--train-precision", default="bf16", choices=["bf16", "fp32"],
                   help="configs[4] names bf16 (GEMM operands; fp32 accumulation and state)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-variants", action="store_true",
                   help="skip the model-variant legs (Tacotron_emt_attn, style paths, CBHG)")
    p.add_argument("--profile-iters", type=int, default=50)
    p.add_argument("--dry-run", action="store_true",
                   help="launcher rehearsal without a GPU: the ranks rendezvous over gloo, run the "
                        "barrier / max-over-ranks timing around a CPU stand-in step and print the JSON "
                        "line (tests/test_bench_launcher.py)")
    return p.parse_args()


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s_:
        s_.bind(("127.0.0.1", 0))
        return s_.getsockname()[1]


def launch_ranks(a):
    """``--gpus N`` (N > 1) outside torch.distributed.run: start the N ranks as ONE child
    ``python -m torch.distributed.run --nproc-per-node N`` (rendezvous on 127.0.0.1) and return its
    exit status.  Runs before anything touches the GPU (counting devices does not initialise HIP on
    this image), and never exec()s: the ranks are children of this process."""
    import subprocess
    if not a.dry_run:
        import torch
        n = torch.cuda.device_count()
        if n < a.gpus:
            sys.exit("bench.py: --gpus {} but only {} GPU(s) visible".format(a.gpus, n))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node={}".format(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    env = dict(os.environ, TT2_BENCH_LAUNCHED="1")
    return subprocess.call(cmd, env=env)


def world_from_env(a):
    """(world, rank, local) of this rank; the world must agree with --gpus."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        sys.exit("bench.py: --gpus {} disagrees with WORLD_SIZE={} (run `python bench.py --gpus N` "
                 "or torch.distributed.run --nproc-per-node N ... bench.py --gpus N)".format(a.gpus, world))
    return world, rank, local


def dry_run(a, world, rank):
    """The multi-rank skeleton of main() on CPU: gloo rendezvous, warmup, barrier-bracketed timed
    steps of a fixed CPU stand-in workload, max over ranks, one JSON line from rank 0."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", init_method="env://", world_size=world, rank=rank)
    x = np.random.default_rng(rank).standard_normal((256, 256)).astype(np.float32)

    def step():
        y = x
        for _ in range(4):
            y = np.tanh(y @ x)
        return int(a.batch)

    for _ in range(a.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    frames = sum(step() for _ in range(a.steps))
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        fr = torch.tensor([frames], dtype=torch.int64)
        dist.all_reduce(fr)
        frames = int(fr.item())
    if rank == 0:
        print(json.dumps(dict(metric=METRIC, value=round(frames / el, 1), unit="stand-in rows/s", n_gpus=world,
                              steps=a.steps, warmup=a.warmup, ms_per_step=round(1e3 * el / a.steps, 3),
                              higher_is_better=True, scaling="weak", dry_run=True,
                              ranks_launched_by_bench=os.environ.get("TT2_BENCH_LAUNCHED") == "1")))
    if world > 1:
        dist.destroy_process_group()


def lstm_bytes(K, H, M=32):
    """Algorithmic HBM bytes of one k_lstm launch: critical-path weights (K rows) + bias + input
    activations + recurrent/style gate terms + c r/w + h_prev + h outputs (raw + zoneout)."""
    return 4 * (K * 4 * H + 4 * H + M * K + M * 4 * H + 2 * M * H + 3 * M * H)


DECODER_STEP_SCOPES = ("decoder/decoder_prenet/", "decoder/decoder_LSTM/", "decoder/query_layer/",
                       "decoder/Location_Sensitive_Attention/", "decoder/linear_transform_projection/",
                       "decoder/stop_token_projection/")


def decoder_step_bytes(W, hp, B, T):
    """Algorithmic HBM bytes of one decoder step: every weight the step touches
    (prenet, 2 LSTM layers, query/location/attention weights, frame + stop projections), the
    attention keys [B,T,A] and values [B,T,D_mem], and the cumulative alignments read + written."""
    P = "Tacotron_model/inference/"
    params = sum(v.size for k, v in W.items()
                 if k.startswith(P) and any(k[len(P):].startswith(sc) for sc in DECODER_STEP_SCOPES))
    D = 2 * hp.encoder_lstm_units + 2 * hp.style_embed_depth
    return 4 * (params + B * T * hp.attention_dim + B * T * D + 2 * B * T)


def cpu_baseline_tacotron(hp, W, B, T, T_ref, t_out, seed):
    """libtt2_cpu.so (cpu/tt2_cpu.cpp: the same C ABI on host cores, fp32, OpenMP) on the WHOLE
    configs[1] workload of the GPU leg: same weights, ids, reference mels and prenet keep bits
    (rng.h stream of `seed`), encoder + every decoder step + Postnet, no extrapolation."""
    from tt2.engine import TacotronEngine
    from tt2.synthetic import tacotron_inputs
    lib = _lib.load_cpu_library()
    ids, lens, re, rs = tacotron_inputs(B, T, T_ref, seed=seed, ragged=False)
    eng = TacotronEngine(hp, W, B, T, T_ref, t_out, 0, lib=lib)
    t0 = time.perf_counter()
    eng.encode(ids, lens, re, rs)
    t1 = time.perf_counter()
    frames, _, _ = eng.decode(t_out, None, 5339)
    t2 = time.perf_counter()
    eng.postnet(None, B, frames.shape[1])
    t3 = time.perf_counter()
    eng.close()
    return dict(value=B * frames.shape[1] / (t3 - t0), t_encoder_s=t1 - t0, t_decoder_s=t2 - t1,
                t_postnet_s=t3 - t2, decoded=int(frames.shape[1]))


def cpu_baseline_wavenet(hp, W, samples, B=1):
    """libtt2_cpu.so tt2_wn_generate: B utterances of `samples` audio samples of configs[2]
    (conditioning upsampling included), injected uniforms; the library runs one OpenMP thread per
    utterance (the sample chain inside an utterance is sequential).  Returns (samples/s, T)."""
    from tt2.engine import WaveNetEngine
    lib = _lib.load_cpu_library()
    hop = int(np.prod(hp.upsample_scales))
    T_f = max(1, samples // hop)
    rng = np.random.default_rng(5339)
    cond = rng.uniform(0, 1, (B, T_f, hp.num_mels)).astype(np.float32)
    T = T_f * hop
    um = rng.uniform(1e-5, 1 - 1e-5, (T, B, 10)).astype(np.float32)
    ul = rng.uniform(1e-5, 1 - 1e-5, (T, B)).astype(np.float32)
    eng = WaveNetEngine(hp, W, B, T, 0, lib=lib)
    t0 = time.perf_counter()
    eng.generate(cond, um, ul, 0, None)
    dt = time.perf_counter() - t0
    eng.close()
    return B * T / dt, T


def threads_used():
    """OpenMP threads of libtt2_cpu.so (libgomp honours OMP_NUM_THREADS; 16 on the GPU box)."""
    try:
        from threadpoolctl import threadpool_info
        n = [i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "openmp"]
        if n:
            return max(n)
    except Exception:
        pass
    return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


def load_traffic(kernel):
    """HBM bytes/launch from the committed rocprofv3 PMC summary (profiles/), FETCH_SIZE x2 +
    WRITE_SIZE per MI355X_MICROARCH.md §HBM, or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d["kernels"][kernel]["hbm_bytes_per_launch"]
    except Exception:
        return None


def traffic_source():
    """Where load_traffic's bytes come from: the committed PMC passes named in
    profiles/pmc_traffic.json (counted in a separate rocprofv3 --pmc run of the same build, not
    in this bench run)."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            d = json.load(f)
        return ("profiles/pmc_traffic.json ({} PMC passes: {}); counted in a separate rocprofv3 --pmc "
                "run, not in this bench run".format(d.get("source"), d.get("method")))
    except Exception:
        return None

def bench_griffin_lim(local, frames=1000):
    """tt2_gl_synthesize_dev on a synthetic normalised mel [1000, 80] (paper_hparams audio: n_fft
    2048, win 1100, hop 275; 60 iterations), HIP-event timed; audio-samples/s of the output."""
    import torch
    from tt2.audio import GriffinLim
    from tt2.hparams import paper_hparams
    hp = paper_hparams.copy()
    gl = GriffinLim(hp, local)
    rng = np.random.default_rng(7)
    mel = np.clip(rng.uniform(-4, 2, (1, 80)) + np.cumsum(rng.normal(0, 0.3, (frames, 80)), 0),
                  -4, 4).astype(np.float32)
    dev = torch.device("cuda", local)
    mel_d = torch.from_numpy(mel).to(dev)
    L = (frames - 1) * hp.hop_size + hp.win_size
    wav_d = torch.empty((L,), dtype=torch.float32, device=dev)
    st = torch.cuda.current_stream(dev)

    def run():
        _lib.check(gl.lib.tt2_gl_synthesize_dev(gl.h, mel_d.data_ptr(), frames, 1, -1, wav_d.data_ptr(),
                                                ctypes.c_void_p(st.cuda_stream)))

    run()
    # wall clock between device-wide synchronizes: torch's default stream is the NULL handle, so
    # the library runs on its own stream and torch events would not bracket it
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(3):
        run()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) * 1e3 / 3
    gl.close()
    n = hp.n_fft
    # algorithmic bytes per iteration: spec read + angle write/read + frame buffer write/read
    it_bytes = frames * (4 * (n // 2 + 1) * 3 + 4 * 2 * hp.win_size * 2)
    return dict(metric="audio-samples/sec (Griffin-Lim, 60 iterations)", value=round(L / (ms * 1e-3), 1),
                unit="audio-samples/s", ms_per_utterance=round(ms, 3), frames=frames, samples=L,
                iters=hp.griffin_lim_iters, n_fft=n, win=hp.win_size, hop=hp.hop_size,
                algorithmic_gb_per_s=round(it_bytes * hp.griffin_lim_iters / (ms * 1e-3) / 1e9, 1))


def train_step_flops(B, T_in, T, hp, D):
    """Algorithmic FLOPs of one teacher-forced decoder training step (forward + backward): the
    matrix products (per step-row: LSTM-1 [P+D+H]x4H, LSTM-2 2Hx4H, query HxA, projections
    (H+D)x81; prenet once over all rows; keys once per batch; Postnet convs + projection) counted
    3x (forward, input gradient, weight gradient) plus the attention's location/energy/context
    terms (2x)."""
    H, A, F, KW, P, NM = (hp.decoder_lstm_units, hp.attention_dim, hp.attention_filters,
                          hp.attention_kernel[0], hp.prenet_layers[0], hp.num_mels)
    row = 2 * ((P + D + H) * 4 * H + 2 * H * 4 * H + H * A + (H + D) * (NM + 1) + NM * P + P * P)
    att = 2 * T_in * (F * KW + F * A + 2 * A + D)
    C, kw, L = hp.postnet_channels, hp.postnet_kernel_size[0], hp.postnet_num_layers
    post = 2 * (kw * NM * C + (L - 1) * kw * C * C + C * NM)
    return B * T * (3 * row + 2 * att + 3 * post) + 3 * 2 * B * T_in * D * A


def front_end_flops(B, Ti, T_ref, hp, emt_only=False):
    """Forward FLOPs of the training front end (matrix products): encoder convs, BiLSTM input and
    recurrent products, reference-encoder conv2d stacks, GRU, dense, GST."""
    E, C, K, U = hp.embedding_dim, hp.enc_conv_channels, hp.enc_conv_kernel_size[0], hp.encoder_lstm_units
    M = B * Ti
    fl = sum(2.0 * M * K * (E if i == 0 else C) * C for i in range(hp.enc_conv_num_layers))
    fl += 2.0 * M * C * 8 * U + 2.0 * M * U * 8 * U
    H, W, ci = T_ref, hp.num_mels, 1
    ref = 0.0
    for f in hp.reference_filters:
        H, W = (H + 1) // 2, (W + 1) // 2
        ref += 2.0 * B * H * W * 9 * ci * f
        ci = f
    D = hp.reference_depth
    ref += 2.0 * B * H * (W * ci + D) * 3 * D + 2.0 * B * D * 128
    return fl + ref * (1 if emt_only else 2)


LOSS_PARTS = ("before", "after", "stop_token", "regularization", "style_emb_loss_emt", "style_emb_loss_spk",
              "style_emb_orthog_loss")


def bench_train(a, rank, world, local, barrier, max_over_ranks):
    """configs[4]: teacher-forced decoder training step (fork-default widths, D_mem 1024) at
    B = 64 rows per GPU, T_in = 150, T_out = 800 (LJSpeech-shaped); data-parallel over ranks with
    one RCCL all-reduce of the flat gradient buffer; K timed steps of forward + backward +
    all-reduce + clipped Adam, max over ranks."""
    import torch
    from tt2.hparams import hparams
    from tt2.synthetic import postnet_masks, prenet_masks, train_batch, zoneout_masks
    from tt2.train import TacotronTrainer
    from tt2.weights import init_tacotron_weights, memory_width
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1))
    B, Ti, T = a.train_batch, a.train_t_in, a.train_t_out
    D = memory_width(hp)
    W = init_tacotron_weights(hp, seed=hp.tacotron_random_seed)
    front = not a.train_decoder_only
    Tr = a.train_t_ref
    # the default training graph's style-embedding classifiers (tacotron.py:486-495, 812-820) over
    # 4 emotion / 4 speaker classes with synthetic labels, and the orthogonality loss
    n_cls = 4 if front else 0
    tr = TacotronTrainer(hp, W, B, Ti, T, local, precision=a.train_precision, frontend=front,
                         max_T_ref=Tr, n_emt=n_cls, n_spk=n_cls)
    if n_cls:
        lab = np.random.default_rng(99 + rank).integers(0, n_cls, (2, B))
        tr.set_style_labels(lab[0], lab[1])
    if world > 1:
        tr.bind_grad_buffer()
    dev = torch.device("cuda", local)
    mem, lens, tg, st = train_batch(B, Ti, T, D, seed=1234 + rank)
    batch = [torch.from_numpy(x).to(dev) for x in (mem, lens, tg, st)]
    batch.append(torch.from_numpy(prenet_masks(T, B, hp.prenet_layers[0], seed=7 + rank)).to(dev))
    batch.append(torch.from_numpy(zoneout_masks(T, B, hp.decoder_lstm_units, seed=7 + rank)).to(dev))
    batch.append(torch.from_numpy(postnet_masks(hp.postnet_num_layers, B, T, hp.postnet_channels,
                                                seed=7 + rank)).to(dev))
    if front:  # the whole configs[4] step: ids + reference mels, encoder dropout / zoneout bits
        from tt2.synthetic import enc_conv_masks, enc_zoneout_masks, tacotron_inputs
        ids, tlens, re, rs = tacotron_inputs(B, Ti, Tr, seed=1234 + rank)
        fb = [torch.from_numpy(x).to(dev) for x in (ids, tlens, re, rs)] + batch[2:]
        fb.append(torch.from_numpy(enc_conv_masks(hp.enc_conv_num_layers, B, Ti, hp.enc_conv_channels,
                                                  seed=7 + rank)).to(dev))
        fb.append(torch.from_numpy(enc_zoneout_masks(Ti, B, hp.encoder_lstm_units, seed=7 + rank)).to(dev))
    losses = []

    def step():
        if front:
            tr.forward_backward_text(*fb)
        else:
            tr.forward_backward(*batch)
        tr.allreduce_grads()
        tr.apply()
        tr.sync_moving_stats()

    step()
    losses.append(tr.losses())
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.train_steps):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    el = max_over_ranks(time.perf_counter() - t0)
    L = tr.losses()
    tr.close()
    ms = 1e3 * el / a.train_steps
    fl = train_step_flops(B, Ti, T, hp, D) + (3.0 * front_end_flops(B, Ti, Tr, hp) if front else 0.0)
    tf = fl / (ms * 1e-3) / 1e12
    peak = 2500.0 if a.train_precision == "bf16" else 157.3
    return dict(metric="mel-frames/sec (teacher-forced training step)",
                value=round(world * B * T / (ms * 1e-3), 1), unit="mel-frames/s",
                ms_per_step=round(ms, 2), steps=a.train_steps, warmup=1,
                forward_backward_ms=round(L["forward_backward_ms"], 2),
                loss_first=round(losses[0]["loss"], 5), loss_last=round(L["loss"], 5),
                # every component of the first step's and the last timed step's forward loss (the
                # total's rise over the first clipped-Adam updates is the orthogonality loss at
                # lr 1e-3: DESIGN.md §5.6h, scripts/diag_train_loss.py)
                losses_first={k: round(v, 5) for k, v in losses[0].items() if k in LOSS_PARTS},
                losses_last={k: round(v, 5) for k, v in L.items() if k in LOSS_PARTS},
                updates_before_last=a.train_steps,
                grad_norm=round(L["grad_norm"], 5), dtype=a.train_precision,
                config=dict(workload=("configs[4]: whole Tacotron-2 training step from ids + reference mels "
                                      "(encoder, 2 reference encoders + GST, teacher-forced decoder, Postnet; "
                                      "training BN / dropout / zoneout; style-embedding classifiers (4+4 "
                                      "classes) + orthogonality loss), B={} rows/GPU, T_in={}, T_out={}, "
                                      "T_ref={}, D_mem={}".format(B, Ti, T, Tr, D)) if front else
                                     ("configs[4] slice: decoder + Postnet training step from a given memory, "
                                      "B={} rows/GPU, T_in={}, T_out={}, D_mem={}".format(B, Ti, T, D)),
                            global_batch=B * world, parallelism="dp{} (RCCL grad all-reduce)".format(world)),
                roofline=dict(bound="mfma", achieved=round(tf, 2), peak=peak, unit="TFLOP/s",
                              frac=round(tf / peak, 4), algorithmic_flops_per_step=int(fl),
                              note="dense MFMA peak of the GEMM dtype ({}); whole-step average".format(
                                  "v_mfma_f32_32x32x16_bf16" if a.train_precision == "bf16"
                                  else "v_mfma_f32_32x32x2_f32")))


E2E_TEXT = ("Scientists at the CERN laboratory say they have discovered a new particle. "
            "The buses aren't the problem, they actually provide a solution. Does the quick "
            "brown fox jump over the lazy dog? He thought it was time to present the present.")


def bench_e2e(a, rank, world, local, barrier, max_over_ranks):
    """configs[3]: end-to-end text -> mel -> wav, batch = world utterances sharded one per rank
    (8 over 8 GPUs in the config), each a 200-character text through the text frontend,
    Tacotron-2 (T_out = a.e2e_frames decoder frames, stop ignored by the random-init stop bias) and
    the 24-layer R=64 MoL WaveNet (T_out x 275 samples); one all_gather of the trimmed waveforms
    (RCCL) closes the timed region.  Weak scaling: utterances/s = world / max-over-ranks time."""
    import torch
    from tacotron.utils.text import text_to_sequence
    from tt2.e2e import TextToSpeech, e2e_hparams, synthesize_sharded
    from tt2.weights import init_tacotron_weights, init_wavenet_weights
    hp = e2e_hparams(a.e2e_frames)
    text = E2E_TEXT[:200]
    seq = text_to_sequence(text, [c.strip() for c in hp.cleaners.split(",")])
    ids = np.asarray([seq] * world, np.int32)
    lens = np.full((world,), len(seq), np.int32)
    rng = np.random.default_rng(1234)
    re = rng.uniform(-4, 4, (world, a.ref_frames, hp.num_mels)).astype(np.float32)
    rs = rng.uniform(-4, 4, (world, a.ref_frames, hp.num_mels)).astype(np.float32)
    W = init_tacotron_weights(hp, seed=hp.tacotron_random_seed)
    WW = init_wavenet_weights(hp, seed=hp.wavenet_random_seed)
    tts = TextToSpeech(hp, W, WW, 1, ids.shape[1], a.ref_frames, a.e2e_frames, local)

    def run():
        if world > 1:
            return synthesize_sharded(tts, ids, lens, re, rs, seed=5339)
        return tts.synthesize(ids, lens, re, rs, seed=5339)["wavs"]

    # warm-up: every kernel once on a short decode (same shapes except the step count)
    dev = torch.device("cuda", local)
    tts.synthesize_dev(torch.from_numpy(ids[:1]).to(dev), torch.from_numpy(lens[:1]).to(dev),
                       lens[:1], torch.from_numpy(re[:1]).to(dev), torch.from_numpy(rs[:1]).to(dev),
                       seed=1, max_iters=8)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    wavs = run()
    torch.cuda.synchronize()
    barrier()
    el = max_over_ranks(time.perf_counter() - t0)
    ms3 = (ctypes.c_float * 3)()
    _lib.check(tts.lib.tt2_last_timings(tts.taco.h, ms3))
    wms = (ctypes.c_float * 3)()
    _lib.check(tts.lib.tt2_wn_last_timings(tts.wn.h, wms))
    samples = int(sum(w.shape[0] for w in wavs))
    tts.close()
    return dict(metric="utterances/sec (text->mel->wav)", value=round(world / el, 4),
                unit="utterances/s", audio_samples_per_s=round(samples / el, 1),
                realtime_factor=round(samples / el / hp.sample_rate / world, 3),
                seconds=round(el, 3), utterances=world, per_rank_utterances=1,
                chars=len(seq) - 1, decoder_frames=a.e2e_frames, samples_per_utterance=samples // world,
                rank0_phases_ms=dict(encode=round(ms3[0], 2), decode=round(ms3[1], 2),
                                     postnet=round(ms3[2], 2), upsample=round(wms[0], 2),
                                     cond_gemm=round(wms[1], 2), generate=round(wms[2], 2)),
                config="configs[3]: end-to-end text->mel->wav, {} utterance(s) sharded one per "
                       "GPU, waveforms all-gathered{}".format(world, " over RCCL" if world > 1 else ""))


def bench_variants(a, local):
    """Model variants on the configs[1] shape (B=32 x 201 chars, T_ref 400, T_out 1000; rank 0):
    Tacotron_emt_attn (args.attn 'multihead', 'style_tokens' and 'simple': persistent decoder, k_decode_persist<true>),
    the AdaIN and reference-embedding style paths (persistent decoder), and the CBHG linear post-net
    over the 32 x 1000 mel frames.  Device-resident inputs, tt2_synthesize_dev, HIP-event phases."""
    import torch
    from tt2.engine import TacotronEngine
    from tt2.hparams import hparams
    from tt2.synthetic import tacotron_inputs
    from tt2.weights import init_tacotron_emt_weights, init_tacotron_weights
    dev = torch.device("cuda", local)
    B, T, TR, n = a.batch, a.chars + 1, a.ref_frames, a.t_out
    ids, lens, re, rs = tacotron_inputs(B, T, TR, seed=1234, ragged=False)
    ids_d, lens_d = torch.from_numpy(ids).to(dev), torch.from_numpy(lens).to(dev)
    re_d, rs_d = torch.from_numpy(re).to(dev), torch.from_numpy(rs).to(dev)
    mel_d = torch.empty((B, n, 80), dtype=torch.float32, device=dev)
    stop_d = torch.empty((B, n), dtype=torch.float32, device=dev)
    lens_h = np.ascontiguousarray(lens, np.int32)
    out = {}

    def run(eng, label, extra=None):
        lib, ns = eng.lib, ctypes.c_int32()
        stream = torch.cuda.current_stream(dev).cuda_stream

        def once():
            _lib.check(lib.tt2_synthesize_dev(
                eng.h, ids_d.data_ptr(), lens_d.data_ptr(), _lib.ptr(lens_h), B, T, re_d.data_ptr(), TR,
                rs_d.data_ptr(), TR, n, None, 5339, mel_d.data_ptr(), stop_d.data_ptr(),
                ctypes.byref(ns), ctypes.c_void_p(stream)), lib)
        once()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        once()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        ms3 = (ctypes.c_float * 3)()
        _lib.check(lib.tt2_last_timings(eng.h, ms3), lib)
        persist, _ = eng.decoder_path()
        d = dict(value=round(B * ns.value / el, 1), unit="mel-frames/s", ms_per_batch=round(1e3 * el, 2),
                 decode_us_per_step=round(1e3 * ms3[1] / max(ns.value, 1), 2), steps=ns.value,
                 decoder="persistent" if persist else "launch path")
        if extra:
            d.update(extra)
        out[label] = d

    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1, max_iters=n))
    for attn, rg in (("multihead", "gru"), ("style_tokens", "none"), ("simple", "gru_multi")):
        W = init_tacotron_emt_weights(hp, attn, rg, seed=hp.tacotron_random_seed)
        eng = TacotronEngine(hp, W, B, T, TR, n, local, emt_attn=attn, emt_ref_gru=rg)
        if attn == "style_tokens":
            eng.set_emt_labels(np.arange(B, dtype=np.int32) % 4)
        run(eng, "emt_attn_" + attn, dict(emt_ref_gru=rg))
        eng.close()
    for style in ("adain", "embed"):
        W = init_tacotron_weights(hp, seed=hp.tacotron_random_seed, style=style)
        eng = TacotronEngine(hp, W, B, T, TR, n, local, style=style)
        run(eng, "style_" + style)
        eng.close()
    hpl = hp.copy()
    hpl.predict_linear = True
    W = init_tacotron_weights(hpl, seed=hp.tacotron_random_seed)
    eng = TacotronEngine(hpl, W, B, T, TR, n, local)
    lin_d = torch.empty((B, n, hpl.num_freq), dtype=torch.float32, device=dev)
    x_d = torch.rand((B, n, 80), dtype=torch.float32, device=dev) * 8 - 4
    stream = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _lib.check(eng.lib.tt2_linear_outputs_dev(eng.h, x_d.data_ptr(), B, n, lin_d.data_ptr(),
                                                  ctypes.c_void_p(stream)), eng.lib)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    eng.close()
    out["cbhg_linear"] = dict(value=round(B * n / el, 1), unit="mel-frames/s", ms_per_batch=round(1e3 * el, 2),
                              frames=B * n, num_freq=hpl.num_freq)
    return out


def _profiled():
    """Running under rocprofv3 (its tool library is preloaded), or TT2_EXIT_GUARD=1."""
    return ("rocprofiler" in os.environ.get("LD_PRELOAD", "")
            or os.environ.get("TT2_EXIT_GUARD", "0") != "0")


def main():
    a = parse()
    if a.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))  # the N ranks run as children; their rank 0 prints the line
    world, rank, local = world_from_env(a)
    if a.dry_run:
        return dry_run(a, world, rank)
    import torch
    import torch.distributed as dist
    if torch.cuda.device_count() < world:
        sys.exit("bench.py: WORLD_SIZE={} but only {} GPU(s) visible".format(world, torch.cuda.device_count()))
    guard = _profiled()
    if guard:  # before the first device call: see tt2_exit_guard (include/tt2.h), DESIGN.md §7
        _lib.load_library().tt2_exit_guard(1, 1)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", init_method="env://", world_size=world, rank=rank,
                                device_id=torch.device("cuda", local))

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    from tt2.engine import TacotronEngine, WaveNetEngine
    from tt2.hparams import bench_wavenet_hparams, hparams
    from tt2.weights import init_tacotron_weights, init_wavenet_weights
    from tt2.synthetic import tacotron_inputs

    lib = _lib.load_library()
    # measured HBM copy bandwidth of this GPU (the spec peak confirmed on the box),
    # reported beside the spec-priced roofline fractions
    hbm_meas = ctypes.c_double(0.0)
    _lib.check(lib.tt2_hbm_copy_gbps(local, ctypes.c_longlong(1 << 30), 5, ctypes.byref(hbm_meas)))
    hbm_meas = round(hbm_meas.value, 1)

    def meas(achieved):  # the measured-peak companion fields of an HBM roofline
        return dict(peak_measured=hbm_meas, frac_of_measured=round(achieved / hbm_meas, 4),
                    peak_measured_how="tt2_hbm_copy_gbps: 1 GiB -> 1 GiB float4 copy, best of 6 shapes x 5, read + write")
    hp = hparams.copy()
    hp.override_from_dict(dict(tacotron_num_gpus=1, max_iters=a.t_out))
    B, T = a.batch, a.chars + 1
    W = init_tacotron_weights(hp, seed=hp.tacotron_random_seed)
    eng = TacotronEngine(hp, W, B, T, a.ref_frames, a.t_out, local)
    ids, lens, re, rs = tacotron_inputs(B, T, a.ref_frames, seed=1234 + rank, ragged=False)
    dev = torch.device("cuda", local)
    ids_d = torch.from_numpy(ids).to(dev)
    lens_d = torch.from_numpy(lens).to(dev)
    re_d = torch.from_numpy(re).to(dev)
    rs_d = torch.from_numpy(rs).to(dev)
    mel_d = torch.empty((B, a.t_out, hp.num_mels), dtype=torch.float32, device=dev)
    stop_d = torch.empty((B, a.t_out), dtype=torch.float32, device=dev)
    lens_h = np.ascontiguousarray(lens, np.int32)
    n_steps = ctypes.c_int32()
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step():
        _lib.check(lib.tt2_synthesize_dev(
            eng.h, ids_d.data_ptr(), lens_d.data_ptr(), _lib.ptr(lens_h), B, T, re_d.data_ptr(),
            a.ref_frames, rs_d.data_ptr(), a.ref_frames, a.t_out, None, 5339 + rank,
            mel_d.data_ptr(), stop_d.data_ptr(), ctypes.byref(n_steps), ctypes.c_void_p(stream)))
        return n_steps.value

    for _ in range(a.warmup):
        step()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    frames = 0
    for _ in range(a.steps):
        frames += B * step()
    torch.cuda.synchronize()
    barrier()
    el = max_over_ranks(time.perf_counter() - t0)
    total_frames = frames * world
    value = total_frames / el
    ms3 = (ctypes.c_float * 3)()
    _lib.check(lib.tt2_last_timings(eng.h, ms3))
    phases = dict(encode_ms=round(ms3[0], 3), decode_ms=round(ms3[1], 3), postnet_ms=round(ms3[2], 3),
                  decode_us_per_step=round(1000.0 * ms3[1] / max(n_steps.value, 1), 3))

    # --- dominant kernel roofline ---
    persist, pd_ms = eng.decoder_path()
    stamps = None
    if persist:
        # k_decode_persist runs the whole decode loop in one launch; algorithmic bytes per step =
        # every decoder-step weight + keys + values + cum-align r/w (fp32)
        n = n_steps.value
        step_bytes = decoder_step_bytes(W, hp, B, T)
        achieved = step_bytes * n / (pd_ms * 1e-3) / 1e9
        traffic = load_traffic("k_decode_persist<false>") or load_traffic("k_decode_persist")
        # priced against the HBM roofline, but the PMC counters show the weights
        # resident on chip (traffic ~0.1x the algorithmic bytes): the limiter is the latency of
        # the chip-wide hand-offs per step, hence the bound label
        roofline = dict(kernel="k_decode_persist (whole dynamic_decode loop, one launch)",
                        bound="latency (chip-wide hand-offs; weights on-chip)", roofline="hbm",
                        achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(achieved / HBM_PEAK_GBS, 4), traffic=traffic,
                        traffic_source=traffic_source() if traffic else None,
                        algorithmic_bytes_per_launch=int(step_bytes * n),
                        algorithmic_bytes_per_step=int(step_bytes), steps_per_launch=n,
                        avg_launch_us=round(pd_ms * 1000.0, 1),
                        us_per_step=round(pd_ms * 1000.0 / max(n, 1), 3),
                        traffic_per_step=(round(traffic / n) if traffic else None), **meas(achieved))
        if os.environ.get("TT2_STAMP_STEP"):
            st = (ctypes.c_longlong * 8192)()
            _lib.check(lib.tt2_debug_pd_stamps(eng.h, st))
            arr = np.array(st[:], dtype=np.int64).reshape(256, 32)
            t0 = arr[:, 0][arr[:, 0] > 0].min()
            rel = np.where(arr > 0, (arr - t0) * 0.01, np.nan)
            stamps = {"persist_stage_us_wg0": [round(float(v), 2) for v in rel[0]],
                      "persist_stage_us_min": [round(float(v), 2) for v in np.nanmin(rel, 0)],
                      "persist_stage_us_max": [round(float(v), 2) for v in np.nanmax(rel, 0)],
                      "persist_stage_argmax_wg": [int(v) for v in np.nanargmax(np.nan_to_num(rel, nan=-1), 0)]}
            np.save(os.path.join(ROOT, "gpurun_out", "pd_stamps.npy"), arr)
    else:
        us7 = (ctypes.c_float * 10)()
        _lib.check(lib.tt2_profile_decoder_kernels(eng.h, a.profile_iters, us7))
        st64 = (ctypes.c_longlong * 64)()
        _lib.check(lib.tt2_debug_stamps(eng.h, st64))
        stamps = {"prenet": [st64[i] - st64[0] for i in range(6)],
                  "energy": [st64[i] - st64[8] for i in range(8, 13)],
                  "lstm": [st64[i] - st64[16] for i in range(16, 20)]}
        H, P = hp.decoder_lstm_units, hp.prenet_layers[0]
        E2 = 2 * hp.encoder_lstm_units
        by = 0.5 * (lstm_bytes(P + E2, H) + lstm_bytes(H, H))
        lstm_us = us7[1]
        achieved = by / (lstm_us * 1e-6) / 1e9
        traffic = load_traffic("k_lstm")
        roofline = dict(kernel="k_lstm (decoder Zoneout-LSTM, layers 1/2 alternating)", bound="hbm",
                        achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(achieved / HBM_PEAK_GBS, 4), traffic=traffic,
                        traffic_source=traffic_source() if traffic else None,
                        algorithmic_bytes_per_launch=int(by), avg_launch_us=round(lstm_us, 3),
                        per_kernel_us=dict(zip(["prenet", "lstm_avg", "query", "energy",
                                                "softmax_context", "projection", "lstm2", "side_job_only",
                                                "energy_only", "softmax_only"],
                                               [round(v, 3) for v in us7])))

    # --- WaveNet (configs[2]) ---
    wn = None
    if not a.no_wavenet:
        whp = bench_wavenet_hparams()
        WW = init_wavenet_weights(whp, seed=whp.wavenet_random_seed)
        hop = 275
        Tn = a.wavenet_frames * hop
        weng = WaveNetEngine(whp, WW, 1, Tn, local)
        rng = np.random.default_rng(5339 + rank)
        cond = ((np.clip(rng.uniform(-4, 4, (1, 80, a.wavenet_frames)), -4, 4) + 4) / 8).astype(np.float32)
        cond_d = torch.from_numpy(cond).to(dev)
        wav_d = torch.empty((1, Tn), dtype=torch.float32, device=dev)

        def wstep():
            _lib.check(lib.tt2_wn_generate_dev(weng.h, cond_d.data_ptr(), 1, a.wavenet_frames, None,
                                               None, 5339 + rank, None, wav_d.data_ptr(), None,
                                               None, ctypes.c_void_p(stream)))

        wstep()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.wavenet_steps):
            wstep()
        torch.cuda.synchronize()
        barrier()
        wel = max_over_ranks(time.perf_counter() - t0)
        wms = (ctypes.c_float * 3)()
        _lib.check(lib.tt2_wn_last_timings(weng.h, wms))
        gen_s = wms[2] / 1000.0
        st = (ctypes.c_longlong * 512)()
        _lib.check(lib.tt2_wn_debug_stamps(weng.h, st))
        nst = (whp.layers + 2) // 3
        base = st[0]
        wn_stamps = [[round((st[s_ * 8 + k] - base) * 0.01, 2) if st[s_ * 8 + k] else None
                      for k in range(8)] for s_ in range(nst)]
        wn_clock_mhz = [round((st[448 + 2 * s_ + 1] - st[448 + 2 * s_]) /
                              max(1e-9, (st[s_ * 8 + 3] - st[s_ * 8 + 0]) * 0.01), 1) for s_ in range(nst)]
        # algorithmic bytes per sample: dilated conv + skip/out weights + head + conditioning row
        R, G, S_, L = whp.residual_channels, whp.gate_channels, whp.skip_out_channels, whp.layers
        wbytes = 4 * (L * (3 * R * G + G + (G // 2) * (S_ + R) + S_ + R) + S_ * S_ + S_ * 30 + L * G)
        wach = wbytes * Tn / gen_s / 1e9
        wn = dict(metric="audio-samples/sec", value=round(world * Tn * a.wavenet_steps / wel, 1),
                  unit="audio-samples/s", per_gpu_batch=1, samples_per_utterance=Tn,
                  realtime_factor=round((Tn * a.wavenet_steps / wel) / 22050.0, 3),
                  phases_ms=dict(upsample=round(wms[0], 3), cond_gemm=round(wms[1], 3),
                                 generate=round(wms[2], 3)),
                  us_per_sample=round(1e6 * gen_s / Tn, 3),
                  roofline=dict(kernel="k_generate_pipe",
                                bound="latency (serial sample chain; weights register-resident)",
                                achieved=round(wach, 2), peak=HBM_PEAK_GBS, unit="GB/s",
                                frac=round(wach / HBM_PEAK_GBS, 5),
                                algorithmic_bytes_per_sample=int(wbytes), **meas(wach)),
                  diag_stage_stamps_us=wn_stamps, diag_shader_clock_mhz=wn_clock_mhz)
        weng.close()
        # batched synthesis at wavenet_synthesis_batch_size (hparams.py:332): 20 utterances of the
        # configs[2] model in one generation launch (k_generate_pipe, 8 CUs per utterance)
        nb = whp.wavenet_synthesis_batch_size
        weng = WaveNetEngine(whp, WW, nb, Tn, local)
        condb = ((rng.uniform(-4, 4, (nb, 80, a.wavenet_frames)) + 4) / 8).astype(np.float32)
        condb_d = torch.from_numpy(condb).to(dev)
        wavb_d = torch.empty((nb, Tn), dtype=torch.float32, device=dev)

        def wstep_b():
            _lib.check(lib.tt2_wn_generate_dev(weng.h, condb_d.data_ptr(), nb, a.wavenet_frames, None,
                                               None, 5339 + rank, None, wavb_d.data_ptr(), None,
                                               None, ctypes.c_void_p(stream)))
        wstep_b()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        wstep_b()
        torch.cuda.synchronize()
        barrier()
        welb = max_over_ranks(time.perf_counter() - t0)
        _lib.check(lib.tt2_wn_last_timings(weng.h, wms))
        wn["batch"] = dict(per_gpu_batch=nb, value=round(world * nb * Tn / welb, 1), unit="audio-samples/s",
                           realtime_factor_per_utterance=round(Tn / welb / 22050.0, 3),
                           us_per_sample=round(1e3 * wms[2] / Tn, 3), samples_per_utterance=Tn)
        weng.close()

    # --- WaveNet at the reference's own widths (k_generate_wide): fork default R=128 (20 layers /
    #     2 stacks, Gaussian head, SubPixel) and paper default R=256 (24 / 4, MoL), B=1 ---
    if wn is not None and not a.no_wavenet_widths:
        from tt2.hparams import hparams as fork_hp, paper_hparams
        widths = {}
        for tag, base in (("fork_r128", fork_hp), ("paper_r256", paper_hparams)):
            whp = base.copy()
            whp.override_from_dict(dict(hop_size=275, wavenet_num_gpus=1))
            WW = init_wavenet_weights(whp, seed=whp.wavenet_random_seed)
            nf = a.wavenet_frames
            Tn = nf * 275
            weng = WaveNetEngine(whp, WW, 1, Tn, local)
            cond = ((np.random.default_rng(7 + rank).uniform(-4, 4, (1, 80, nf)) + 4) / 8).astype(np.float32)
            cond_d = torch.from_numpy(cond).to(dev)
            wav_d = torch.empty((1, Tn), dtype=torch.float32, device=dev)

            def wstep():
                _lib.check(lib.tt2_wn_generate_dev(weng.h, cond_d.data_ptr(), 1, nf, None, None, 5339 + rank,
                                                   None, wav_d.data_ptr(), None, None, ctypes.c_void_p(stream)))
            wstep()
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            wstep()
            torch.cuda.synchronize()
            barrier()
            wel = max_over_ranks(time.perf_counter() - t0)
            wms = (ctypes.c_float * 3)()
            _lib.check(lib.tt2_wn_last_timings(weng.h, wms))
            R, G, S_, L = whp.residual_channels, whp.gate_channels, whp.skip_out_channels, whp.layers
            wbytes = 4 * (L * (3 * R * G + G + (G // 2) * (S_ + R) + S_ + R) + S_ * S_ + S_ * whp.out_channels)
            gen_s = wms[2] / 1000.0
            widths[tag] = dict(value=round(world * Tn / wel, 1), unit="audio-samples/s",
                               realtime_factor=round(Tn / wel / 22050.0, 3), samples=Tn,
                               residual_channels=R, layers=L, stacks=whp.stacks,
                               head="gaussian" if whp.out_channels == 2 else "mol",
                               us_per_sample=round(1e6 * gen_s / Tn, 3), kernel="k_generate_wide",
                               algorithmic_bytes_per_sample=int(wbytes),
                               achieved_gbs=round(wbytes * Tn / gen_s / 1e9, 1))
            weng.close()
        wn["widths"] = widths

    # --- end-to-end text -> mel -> wav (configs[3]): one utterance per rank, RCCL gather ---
    e2e = None
    if not a.no_e2e:
        e2e = bench_e2e(a, rank, world, local, barrier, max_over_ranks)

    # --- Griffin-Lim vocoder (GL_on_GPU path, 60 iterations) on a 1000-frame mel ---
    glr = None
    if not a.no_griffin_lim:
        glr = bench_griffin_lim(local)

    # --- teacher-forced decoder training step (configs[4]) ---
    trn = None
    if not a.no_train:
        trn = bench_train(a, rank, world, local, barrier, max_over_ranks)

    # --- model variants (rank 0, N = 1 only) ---
    variants = None
    if rank == 0 and world == 1 and not a.no_variants:
        variants = bench_variants(a, local)

    # --- CPU baseline (rank 0, N = 1 only) ---
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        c = cpu_baseline_tacotron(hp, W, B, T, a.ref_frames, a.t_out, 1234 + rank)
        cores = threads_used()
        cpu = dict(value=round(c["value"], 2), unit="mel-frames/s", cores=cores, kind="port",
                   sample="libtt2_cpu.so (cpu/tt2_cpu.cpp, same C ABI, fp32, OpenMP x{}) on the whole "
                          "configs[1] workload: B=32x201 chars, encoder + {} decoder steps + Postnet, "
                          "no extrapolation (enc {:.2f}s, dec {:.2f}s, postnet {:.2f}s)".format(
                              cores, c["decoded"], c["t_encoder_s"], c["t_decoder_s"],
                              c["t_postnet_s"]),
                   label="CPU restatement of the reference path (not TF)")
        if wn is not None:
            whp = bench_wavenet_hparams()
            WW = init_wavenet_weights(whp, seed=whp.wavenet_random_seed)
            v, n = cpu_baseline_wavenet(whp, WW, 2000)
            wn["cpu_baseline"] = dict(value=round(v, 1), unit="audio-samples/s", cores=1, kind="port",
                                      sample="libtt2_cpu.so tt2_wn_generate, {} samples, B=1: one "
                                             "utterance is a sequential per-sample chain, one core "
                                             "(the GPU leg is B=1 too)".format(n))
            if "batch" in wn:  # batched synthesis on as many threads as the decoder baseline
                vb, nb_ = cpu_baseline_wavenet(whp, WW, 1100, B=cores)
                wn["batch"]["cpu_baseline"] = dict(
                    value=round(vb, 1), unit="audio-samples/s", cores=cores, kind="port",
                    sample="libtt2_cpu.so tt2_wn_generate, B={} utterances x {} samples, one OpenMP "
                           "thread per utterance".format(cores, nb_))

    if rank == 0:
        out = dict(metric=METRIC, value=round(value, 1), unit="mel-frames/s", n_gpus=world,
                   steps=a.steps, warmup=a.warmup, ms_per_step=round(1000.0 * el / a.steps, 3),
                   higher_is_better=True, scaling="weak", vs_baseline=None, dtype="f32",
                   dtype_note=("fp32 storage and accumulation; the decoder / encoder / WaveNet products run as "
                               "split fp16x3 MFMA (hi/lo fp16 halves, ~2^-22 relative; DESIGN 5.1)"),
                   data="synthetic (seeded ids/ref mels, random-init weights)",
                   config=dict(workload="configs[1]: Tacotron-2 encoder+decoder+Postnet inference, "
                                        "batch=32x200-char synthetic, T_out=1000, 1 batch per GPU",
                               global_batch=B * world, chars=a.chars, t_out=a.t_out,
                               decoded_steps=n_steps.value, ref_frames=a.ref_frames,
                               parallelism="utterance-batch sharding x{}".format(world)),
                   phases=phases, roofline=roofline, cpu_baseline=cpu, wavenet=wn, e2e=e2e,
                   griffin_lim=glr, train=trn, variants=variants,
                   diag_stamps=stamps)
        print(json.dumps(out))
    eng.close()
    if world > 1:
        dist.destroy_process_group()
    if guard:
        _lib.load_library().tt2_exit_guard(0, 0)  # success: the guard's _exit status


if __name__ == "__main__":
    main()
