"""sample_from_discretized_mix_logistic (code/wavenet_vocoder/models/mixture.py:76-107) on MI355X."""
import numpy as np

from tt2.engine import mol_sample


def sample_from_discretized_mix_logistic(y, log_scale_min=-7., u_mix=None, u_log=None, seed=None):
    """y: [batch_size, channels, time_length] -> samples in [-1, 1] of shape [batch_size, time_length].

    u_mix [B, T, nr_mix] and u_log [B, T] are the uniforms the reference draws with
    tf.random_uniform(minval=1e-5, maxval=1-1e-5) (:91, :104); when omitted they are drawn here
    from numpy's default_rng(seed).  Returns (x, k) when ``return_index`` semantics are needed via
    ``sample_with_index``."""
    return sample_with_index(y, log_scale_min, u_mix, u_log, seed)[0]


def sample_with_index(y, log_scale_min=-7., u_mix=None, u_log=None, seed=None):
    y = np.asarray(y, np.float32)
    if y.shape[1] % 3 != 0:
        raise ValueError("channels must be 3 * nr_mix")
    B, C, T = y.shape
    nr = C // 3
    if u_mix is None or u_log is None:
        rng = np.random.default_rng(seed)
        u_mix = rng.uniform(1e-5, 1. - 1e-5, (B, T, nr))
        u_log = rng.uniform(1e-5, 1. - 1e-5, (B, T))
    logits = y.transpose(0, 2, 1).reshape(B * T, C)
    x, k = mol_sample(logits, np.asarray(u_mix, np.float32).reshape(B * T, nr),
                      np.asarray(u_log, np.float32).reshape(B * T), log_scale_min)
    return x.reshape(B, T), k.reshape(B, T)
