"""Utterance-batch sharding across ranks.

The reference splits a batch into per-GPU towers on the CPU (tacotron.py:83-138,
wavenet.py:227-239) and concatenates the outputs on the host (tacotron/synthesizer.py:177-179).
Here each rank (one process per GPU) synthesises a contiguous slice of the utterances with no
exchange during compute; the only collective is one all_gather of the padded outputs and their
lengths at the end (RCCL over xGMI with backend "nccl", or gloo on CPU).  The batch-level stop
rule is per shard, exactly like the reference's per-tower dynamic_decode.
"""
import numpy as np


def shard_range(n, rank, world):
    """Contiguous slice [start, end) of n utterances owned by `rank` (remainder spread over the
    first ranks, as np.array_split does)."""
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def shard(arrays, rank, world):
    """Slice every array along axis 0 to this rank's utterances."""
    n = arrays[0].shape[0]
    s, e = shard_range(n, rank, world)
    return [None if a is None else a[s:e] for a in arrays]


def gather_padded(local, lengths, group=None, pad_value=0.0):
    """All-gather per-rank outputs [B_r, T_r, ...] with per-utterance lengths [B_r] (time axis 1).

    Returns (list of per-utterance arrays trimmed to their lengths, in global utterance order).
    ``local`` may be a numpy array or a torch tensor.  Under backend "nccl" (RCCL over xGMI) a CUDA
    tensor is padded and gathered on the device -- no host round trip before the collective, only
    the trimmed results come back to the host; gloo gathers CPU tensors."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device()) \
        if dist.get_backend(group) == "nccl" else torch.device("cpu")
    if isinstance(local, torch.Tensor):
        t_local = local.to(dev, torch.float32)
    else:
        t_local = torch.from_numpy(np.ascontiguousarray(local, np.float32)).to(dev)
    lengths = torch.as_tensor(np.asarray(lengths, np.int64)).to(dev)
    shape = tuple(t_local.shape)
    meta = torch.tensor([shape[0], shape[1] if len(shape) > 1 else 0], dtype=torch.int64,
                        device=dev)
    metas = [torch.zeros_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    metas = [m.cpu() for m in metas]
    bmax = int(max(m[0] for m in metas))
    tmax = int(max(m[1] for m in metas))
    t = torch.full((bmax, tmax) + shape[2:], pad_value, dtype=torch.float32, device=dev)
    t[:shape[0], :shape[1]] = t_local
    lt = torch.zeros((bmax,), dtype=torch.int64, device=dev)
    lt[:shape[0]] = lengths
    outs = [torch.empty_like(t) for _ in range(world)]
    louts = [torch.empty_like(lt) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    dist.all_gather(louts, lt, group=group)
    res = []
    for r in range(world):
        nb = int(metas[r][0])
        ls = louts[r].cpu().numpy()
        for i in range(nb):
            res.append(outs[r][i, :int(ls[i])].cpu().numpy())
    return res


def all_reduce_sum_(t, group=None):
    """In-place SUM all-reduce: RCCL over xGMI for CUDA tensors under "nccl"; under gloo a CUDA
    tensor is reduced through a host copy (the CPU rehearsal of the path)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return t
    if t.is_cuda and dist.get_backend(group) != "nccl":
        host = t.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        t.copy_(host)
        return t
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def tower_mean_(flat_grads, group=None):
    """Data-parallel training: the reference averages the per-tower gradients on the CPU
    (Tacotron.get_clipped_grads, tacotron.py:1194-1208: reduce_mean over the tower axis) before
    clip_by_global_norm; here each rank is one tower and the mean is one all-reduce (SUM, then
    divide) over the flat gradient buffer, in place.  RCCL over xGMI for CUDA tensors ("nccl"),
    gloo for CPU tensors."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return flat_grads
    all_reduce_sum_(flat_grads, group)
    flat_grads.div_(dist.get_world_size(group))
    return flat_grads
