"""worker::DigestBatcher (narwhal-tusk_amd/host/narwhal.hpp):
the two Processor tasks of a worker (worker/src/worker.rs:182-188 own batches,
:227-233 others' batches) submit from their own threads into one batcher whose
flusher hashes everything queued in one nt_sha512_trunc32 call.

GPU: two submitter threads of real-size 508,052-B batches, digests against
hashlib and the Processor output message (processor.rs:38-48); the flush rules
(batch count, age); small-call path off (GPU) and AUTO (host lane)."""
import hashlib
import struct
import threading
import time

import numpy as np
import pytest

from ntcrypto import narwhal as N


def _batches(seed, k, size=508052):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, size, dtype=np.uint8).tobytes() for _ in range(k)]


def _message(own, digest, wid):
    return struct.pack("<I", 0 if own else 1) + digest + struct.pack("<I", wid)


@pytest.mark.gpu
@pytest.mark.parametrize("small", [0, 1])
def test_two_processors_real_batches(small):
    N.set_small_call_path(small, 8)
    b = N.DigestBatcher(max_bytes=64 << 20, max_batches=4096, max_delay_us=3000)
    try:
        jobs = {True: _batches(1, 10), False: _batches(2, 10)}
        got = {}

        def processor(own):
            # a Processor that keeps its batches in flight and awaits them in order
            tickets = [b.submit(7, own, x) for x in jobs[own]]
            got[own] = [b.wait(t) for t in tickets]

        th = [threading.Thread(target=processor, args=(own,)) for own in (True, False)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        for own in (True, False):
            for x, (d, m) in zip(jobs[own], got[own]):
                want = hashlib.sha512(x).digest()[:32]
                assert d == want
                assert m == _message(own, want, 7)
        st = b.stats()
        assert st["batches"] == 20 and st["bytes"] == 20 * 508052
        assert st["flushes"] < 20  # the two streams were coalesced
        # one Processor hashing one batch at a time (the reference's loop)
        x = _batches(3, 1)[0]
        d, m = b.process(1, False, x)
        assert d == hashlib.sha512(x).digest()[:32] and m == _message(False, d, 1)
    finally:
        b.close()
        N.set_small_call_path(0)


@pytest.mark.gpu
def test_flush_rules():
    N.set_small_call_path(0)
    xs = [bytes([i]) * (1000 + i) for i in range(12)]
    # batch-count rule: the 4th queued batch triggers a flush (the age rule
    # would take 10 s)
    b = N.DigestBatcher(max_bytes=1 << 30, max_batches=4, max_delay_us=10_000_000)
    try:
        t0 = time.perf_counter()
        tickets = [b.submit(0, True, x) for x in xs[:4]]
        for x, t in zip(xs, tickets):
            assert b.wait(t)[0] == hashlib.sha512(x).digest()[:32]
        assert time.perf_counter() - t0 < 5.0
        # explicit flush of a partial queue
        tickets = [b.submit(0, True, x) for x in xs[4:6]]
        b.flush()
        assert [b.wait(t)[0] for t in tickets] == [hashlib.sha512(x).digest()[:32] for x in xs[4:6]]
        assert time.perf_counter() - t0 < 5.0
        assert b.stats()["batches"] == 6
    finally:
        b.close()
    # age rule: a lone batch is hashed after max_delay_us without any flush()
    b = N.DigestBatcher(max_bytes=1 << 30, max_batches=1 << 20, max_delay_us=20_000)
    try:
        t0 = time.perf_counter()
        d, _ = b.process(0, True, b"lone batch")
        dt = time.perf_counter() - t0
        assert d == hashlib.sha512(b"lone batch").digest()[:32]
        assert 0.015 < dt < 5.0
    finally:
        b.close()
    # byte rule: two 600 kB batches with max_bytes 1 MB flush on the second
    b = N.DigestBatcher(max_bytes=1 << 20, max_batches=1 << 20, max_delay_us=10_000_000)
    try:
        ys = _batches(4, 2, 600_000)
        t = [b.submit(0, True, y) for y in ys]
        assert [b.wait(x)[0] for x in t] == [hashlib.sha512(y).digest()[:32] for y in ys]
    finally:
        b.close()


_FAIL_PROBE = r"""
import sys
sys.path.insert(0, sys.argv[1])
from ntcrypto import narwhal as N
b = N.DigestBatcher(max_batches=2, max_delay_us=100)
ok = 0
for round_ in range(2):  # the flusher survives a failed flush and serves the next one
    ts = [b.submit(0, True, bytes(1000)) for _ in range(3)]
    for t in ts:
        try:
            b.wait(t)
        except N.NtError:
            ok += 1
b.close()
print("failed-waiters", ok)
"""


def test_backend_failure_reaches_every_waiter():
    """a flush whose backend cannot start (Backend::global() throws
    BackendError: here NT_DEVICE names a device that does not exist, so the
    first nt_init_device fails) must fail each waiter's future -- not end the
    flusher thread, and with it the process, in std::terminate.  Runs in a
    subprocess (a regression would abort it) on CPU and GPU boxes alike."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NT_DEVICE="97")
    r = subprocess.run([sys.executable, "-c", _FAIL_PROBE, os.path.join(root, "narwhal-tusk_amd")], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    assert "failed-waiters 6" in r.stdout, r.stdout
