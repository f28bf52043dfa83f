"""Data-parallel view sharding for the rasterizer hot path.

Each rasterizer call is a pure function of (Gaussians at the view's time, camera, bg), so a batch of V
views shards across ranks with no data-path collective: rank r renders views {v : v mod world == r}
(train.py:197-209 loops the views of a batch independently).  Every rank holds a full replica of the
Gaussian parameters.  The only exchanges are the ones a data-parallel training step needs:

* the batch loss, summed over ranks (one scalar; the benchmark's only collective), and
* the parameter gradients, summed over ranks so that every replica takes the same optimizer step as
  the single-process batch (train.py:229-268 sums the viewspace/param grads over the views of the
  batch).  Gradients are flattened into ~bucket_mb buckets so that each all-reduce is one large RCCL
  ring transfer over xGMI rather than one per tensor.

Everything here is backend-agnostic torch.distributed (nccl = RCCL on the GPU box, gloo in the CPU
tests) and renderer-agnostic: the render function is a parameter.
"""
from typing import Callable, Dict, List, Sequence

import torch
import torch.distributed as dist


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def shard_views(num_views: int, r: int = None, w: int = None) -> List[int]:
    """Views of a batch rendered by rank r: {v : v mod w == r} (round-robin keeps per-rank work equal)."""
    r = rank() if r is None else r
    w = world() if w is None else w
    return [v for v in range(num_views) if v % w == r]


def allreduce_sum_(tensors: Sequence[torch.Tensor], bucket_mb: float = 64.0) -> None:
    """In-place SUM all-reduce of a list of same-device, same-dtype tensors, bucketed by size."""
    if world() == 1 or not tensors:
        return
    limit = int(bucket_mb * (1 << 20))
    bucket: List[torch.Tensor] = []
    size = 0

    def flush():
        nonlocal bucket, size
        if not bucket:
            return
        flat = torch.cat([t.reshape(-1) for t in bucket])
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        off = 0
        for t in bucket:
            n = t.numel()
            t.copy_(flat[off:off + n].view_as(t))
            off += n
        bucket, size = [], 0

    for t in tensors:
        nbytes = t.numel() * t.element_size()
        if size and size + nbytes > limit:
            flush()
        bucket.append(t)
        size += nbytes
    flush()


def batch_step(params: Dict[str, torch.Tensor], views: Sequence, render_loss: Callable, num_views: int,
               bucket_mb: float = 64.0):
    """One data-parallel batch: this rank's views -> summed loss / gradients identical on every rank.

    render_loss(params, view) -> scalar loss of one view.  The batch loss is the mean over all
    num_views views (train.py's L1 over the batch); each rank back-propagates its share
    (sum of its views' losses / num_views), then the parameter gradients and the loss are summed
    over ranks.  Returns the batch loss (a 0-dim tensor, equal on all ranks).
    """
    for p in params.values():
        p.grad = None
    mine = shard_views(num_views)
    local = None
    for v in mine:
        lv = render_loss(params, views[v]) / num_views
        local = lv if local is None else local + lv
    if local is not None:
        local.backward()
    grads = []
    for p in params.values():
        if p.grad is None:
            p.grad = torch.zeros_like(p)
        grads.append(p.grad)
    loss = (local.detach() if local is not None else torch.zeros((), device=next(iter(params.values())).device)).clone()
    allreduce_sum_(grads + [loss.reshape(1)], bucket_mb)
    return loss
