"""Host-side multi-GPU plumbing: the path shards by index and has
no exchange step, so ranks only need (1) their contiguous shard and (2) a
barrier + max-over-ranks wall time for reporting.  torch.distributed with the
gloo backend is used for that control plane only -- no RCCL on the data path.
"""
import os


def world_info():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(total: int, world: int, rank: int, align: int = 1):
    """Contiguous [lo, hi) of `total` items for `rank`; boundaries are multiples
    of `align` (64 keeps verdict bitmap words whole) except the final end."""
    per = -(-total // world) if world else total
    per = -(-per // align) * align
    lo = min(total, rank * per)
    hi = min(total, lo + per)
    return lo, hi


def reduce_max(x: float) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(x: float) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def gather_bytes(local: bytes, world: int):
    """All ranks' byte strings (verdict bitmaps / digests) on every rank."""
    import torch.distributed as dist
    if world == 1:
        return [local]
    out = [None] * world
    dist.all_gather_object(out, local)
    return out


def gather_object(x, world: int = None):
    """Every rank's picklable object on every rank (gloo all_gather_object;
    called outside timed regions only)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [x]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, x)
    return out


def rank_summary(rows, rate_key="rate", time_key="kernel_ms"):
    """Per-rank rows of one config plus the min / max / mean of its rate and
    kernel time, so an N-rank line shows a slow rank or a straggling shard
    instead of only the max-over-ranks wall time."""
    rates = [r[rate_key] for r in rows]
    times = [r[time_key] for r in rows]
    return {"per_rank": rows,
            rate_key + "_min": round(min(rates), 1), rate_key + "_max": round(max(rates), 1),
            rate_key + "_mean": round(sum(rates) / len(rates), 1),
            time_key + "_min": round(min(times), 3), time_key + "_max": round(max(times), 3),
            "slowest_rank": rows[rates.index(min(rates))]["rank"]}
