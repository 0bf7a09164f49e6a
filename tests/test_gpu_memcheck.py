"""Device-memory checks of the training step (round 3).

Round 2 left an order-dependent wrong gradient: test_gpu_train_frontend_matches_oracle[True] got the
encoder conv-1 kernel gradient at relative error 1.65 when it ran after the bf16 and full-size
training tests.  The cause was two Postnet buffers sized for postnet_channels where layer 1 has
num_mels input channels (the transposed im2col TBUF and the flipped kernels WFLIP, both too small
whenever num_mels > postnet_channels, as in the small test widths): their overflow landed on
whatever allocation followed, which in that order was the front end's embedding output.  The
DevBuf debug modes that found it (csrc/common.h) are exercised here:

* TT2_REDZONE=1: every allocation gets a 64 KiB guard band; every ABI call (and every phase of a
  training step) fails with the name of any buffer a kernel wrote past.
* TT2_POISON_ALLOC=<byte>: every allocation starts filled with that byte, so a read of a buffer
  before the call writes it changes the result deterministically.

Each case runs in a fresh subprocess (the modes are read once per process; the order case needs
a process whose allocation history is exactly the listed tests)."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

# num_mels (80) > postnet_channels (64) at the small widths: the shape class that overflowed
FRONT = ["test_gpu_train_frontend_matches_oracle:True", "test_gpu_train_frontend_matches_oracle:False"]
POSTNET = ["test_gpu_train_edge_shapes:1,5,1", "test_gpu_train_edge_shapes:5,16,3",
           "test_gpu_train_with_postnet:True"]


def _run(specs, env_extra, timeout=280):
    env = dict(os.environ)
    env.update(env_extra)
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "_memcheck_run.py")] + specs, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=timeout)
    out = p.stdout.decode(errors="replace")
    assert p.returncode == 0 and "__MEMCHECK_OK__" in out, out[-4000:]


@pytest.mark.gpu
def test_training_step_redzones_intact():
    """No kernel of the decoder / Postnet / front-end training step writes past its buffer.  The bf16
    case at decoder width 1024 with a small T·B: the round-3 d W_loc pass once sized its 512 blocks
    of partials without checking TBUF, which is T·B-sized (full run order: an illegal access)."""
    _run(POSTNET + FRONT + ["test_gpu_train_bf16_gemms_close_to_oracle"], {"TT2_REDZONE": "1"})


@pytest.mark.gpu
@pytest.mark.parametrize("fill", ["255", "66"])
def test_frontend_gradients_under_poisoned_allocations(fill):
    """The whole configs[4] step's gradients match the oracle when every allocation starts as NaN
    (0xFF) or as a finite 48.6f (0x42): nothing is read before the call writes it."""
    _run(FRONT + POSTNET[:1], {"TT2_POISON_ALLOC": fill, "TT2_REDZONE": "1"})


@pytest.mark.gpu
def test_frontend_gradients_after_the_round2_failing_order():
    """The exact order that failed in round 2 (bf16 + full-size training tests, then the front-end
    case) in a fresh process, without debug modes."""
    _run(["test_gpu_train_bf16_gemms_close_to_oracle", "test_gpu_train_full_size_properties"] + FRONT, {},
         timeout=400)
