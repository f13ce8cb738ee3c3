"""Multi-GPU helpers: independent frames shard across ranks.

One process per GPU.  Each rank decodes a contiguous slice of the batch with
no communication in the data path; afterwards the packed outputs are
all-gathered and the counters all-reduced (RCCL on GPUs, gloo on CPU).
"""


def shard_range(B, rank, world):
    """Contiguous slice [lo, hi) of B frames for `rank` (sizes differ by <= 1)."""
    base, extra = divmod(int(B), int(world))
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def gather_outputs(dist, packed, counters, device=None):
    """All-gather every rank's packed bytes (ragged allowed) and all-reduce
    the counters.  packed: torch uint8 tensor [b, KB]; counters: list of
    numbers.  Returns (packed of all ranks in rank order, summed counters)."""
    import torch
    world = dist.get_world_size()
    dev = packed.device if device is None else device
    n = torch.tensor([packed.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes)
    pad = torch.zeros((mx, packed.shape[1]), dtype=packed.dtype, device=dev)
    pad[:packed.shape[0]] = packed
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    full = torch.cat([p[:s] for p, s in zip(parts, sizes)], 0)
    c = torch.tensor([float(x) for x in counters], dtype=torch.float64, device=dev)
    dist.all_reduce(c)
    return full, c.tolist()
