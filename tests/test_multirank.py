"""world_size-2 gloo tests of the N>1 path on CPU: contiguous sharding with no
data-path collective, max-over-ranks timing and host gather of the verdicts.
The device kernel is stood in by the oracle here (the CPU checker); the GPU
sharding itself is covered by tests/test_gpu_sharding.py."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "narwhal-tusk_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from ntcrypto import dist as nd
    import _oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
        n = len(d["cat"])
        lo, hi = nd.shard(n, world, rank, align=64)
        orc = _oracle.load()
        bits = orc.verify_strict_many(d["pk"][lo:hi], d["sig"][lo:hi], d["msg"], d["off"][lo:hi], d["len"][lo:hi])
        allb = nd.gather_bytes(np.packbits(bits, bitorder="little").tobytes() + bytes([hi - lo & 0xff, hi - lo >> 8]),
                               world)
        t = nd.reduce_max(float(rank + 1))
        s = nd.reduce_sum(float(hi - lo))
        if rank == 0:
            got = []
            for b in allb:
                cnt = b[-2] | (b[-1] << 8)
                got.append(np.unpackbits(np.frombuffer(b[:-2], np.uint8), bitorder="little")[:cnt])
            q.put((np.concatenate(got).astype(bool), t, s))
    finally:
        dist.destroy_process_group()


def test_shard_cover_disjoint():
    from ntcrypto.dist import shard
    for total in (0, 1, 63, 64, 65, 1000, 16384, 100000):
        for world in (1, 2, 3, 4, 8):
            parts = [shard(total, world, r, align=64) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == total
            for (a, b), (c, e) in zip(parts, parts[1:]):
                assert b == c and a <= b
            for a, b in parts:
                assert a == b or a % 64 == 0  # every non-empty shard starts on a bitmap word


def test_two_rank_gloo_verify_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, t, s = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    assert np.array_equal(got, d["strict"].astype(bool))
    assert t == 2.0 and s == len(d["cat"])
