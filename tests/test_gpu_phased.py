"""GPU parity of the phased verify kernel (k_verify.inc: a persistent grid
pulling third-of-a-signature tasks, state handed between waves on any CU or XCD
through HBM).  Launches of at least one signature per resident lane take it
(131,072 on MI355X at occupancy 2), so these batches are sized just above and
well above that bound, with ragged tails (n not a multiple of 64):

* strict and cofactorless verdicts equal the expected labels -- GPU-signed
  honest entries (valid), every golden-corpus category tiled in (strict /
  batch_rule columns, their own message lengths) and single message-bit flips;
* the device entry point (one phased launch) and the host entry point (chunks
  of whole rounds on two streams) agree; a repeated launch is identical;
* two different batches enqueued back to back on two streams, no host sync in
  between (the two phased workspaces run at once: consumers on CUs whose L1
  holds the other launch's lines, uneven load), keep their own verdicts.
"""
import os
import types

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = 512


@pytest.fixture(scope="module")
def env():
    import torch
    import ntcrypto
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    be = ntcrypto.Backend(0)
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    yield types.SimpleNamespace(torch=torch, ntcrypto=ntcrypto, dev=dev, be=be, streams=streams)
    torch.cuda.synchronize(dev)
    be.close()


def _batch(be, n, seed):
    """n entries: GPU-signed 512-B messages, every 29th replaced by a corpus
    entry (its own message appended to the buffer), 2,048 bit flips."""
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msg = rng.integers(0, 256, n * L, dtype=np.uint8)
    off = np.arange(n, dtype=np.uint64) * L
    ln = np.full(n, L, np.uint64)
    pk, sig = be.sign_batch(seeds, msg, off, ln)
    pk, sig = pk.copy(), sig.copy()
    corpus = np.load(os.path.join(ROOT, "tests", "golden", "ed25519_corpus.npz"))
    nc = len(corpus["cat"])
    pos = np.arange(int(rng.integers(0, 29)), n, 29)
    src = (np.arange(len(pos)) * 7) % nc
    strict = np.ones(n, bool)
    batch = np.ones(n, bool)
    extra = []
    tail = n * L
    for p, s in zip(pos, src):
        o, m = int(corpus["off"][s]), int(corpus["len"][s])
        pk[p], sig[p] = corpus["pk"][s], corpus["sig"][s]
        off[p], ln[p] = tail, m
        extra.append(corpus["msg"][o:o + m])
        tail += m
        strict[p] = bool(corpus["strict"][s])
        batch[p] = bool(corpus["batch_rule"][s])
    msg = np.concatenate([msg] + extra + [np.zeros(64, np.uint8)])
    honest = np.setdiff1d(np.arange(n), pos)
    flip = np.sort(rng.choice(honest, size=2048, replace=False))
    msg[(off[flip] + rng.integers(0, L, len(flip)).astype(np.uint64)).astype(np.int64)] ^= np.uint8(0x10)
    strict[flip] = False
    batch[flip] = False
    return types.SimpleNamespace(n=n, pk=pk, sig=sig, msg=msg, off=off, ln=ln, strict=strict, batch=batch)


def _dev(torch, dev, b):
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return types.SimpleNamespace(pk=t(b.pk), sig=t(b.sig), msg=t(b.msg), off=t(b.off.view(np.int64)),
                                 ln=t(b.ln.view(np.int64)),
                                 out=torch.zeros((b.n + 63) // 64, dtype=torch.int64, device=dev))


def _launch(be, ntc, stream, mode, d, n):
    be.dev_verify(0, stream.cuda_stream, mode, d.pk.data_ptr(), d.sig.data_ptr(), d.msg.data_ptr(),
                  d.off.data_ptr(), d.ln.data_ptr(), n, d.out.data_ptr())


def _bits(out, n):
    return np.unpackbits(out.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)


@pytest.mark.parametrize("n", [131_109, 300_007])
def test_phased_strict_and_cofactorless(env, n):
    torch, be, ntc = env.torch, env.be, env.ntcrypto
    b = _batch(be, n, seed=n)
    d = _dev(torch, env.dev, b)
    torch.cuda.synchronize(env.dev)
    for mode, want in ((ntc.NT_MODE_STRICT, b.strict), (ntc.NT_MODE_COFACTORLESS, b.batch)):
        runs = []
        for _ in range(2):
            d.out.zero_()
            _launch(be, ntc, env.streams[0], mode, d, n)
            torch.cuda.synchronize(env.dev)
            runs.append(_bits(d.out, n))
        bad = np.nonzero(runs[0] != want)[0]
        assert len(bad) == 0, (mode, len(bad), bad[:10].tolist())
        assert np.array_equal(runs[0], runs[1])
    hv = be.verify_strict(b.pk, b.sig, b.msg, b.off, b.ln)
    assert np.array_equal(hv, b.strict)


def test_phased_two_streams_concurrent(env):
    torch, be, ntc = env.torch, env.be, env.ntcrypto
    b1, b2 = _batch(be, 262_147, seed=11), _batch(be, 196_613, seed=12)
    d1, d2 = _dev(torch, env.dev, b1), _dev(torch, env.dev, b2)
    torch.cuda.synchronize(env.dev)
    for _ in range(3):
        d1.out.zero_()
        d2.out.zero_()
        torch.cuda.synchronize(env.dev)
        _launch(be, ntc, env.streams[0], ntc.NT_MODE_STRICT, d1, b1.n)
        _launch(be, ntc, env.streams[1], ntc.NT_MODE_COFACTORLESS, d2, b2.n)
        _launch(be, ntc, env.streams[1], ntc.NT_MODE_STRICT, d2, b2.n)
        torch.cuda.synchronize(env.dev)
        assert np.array_equal(_bits(d1.out, b1.n), b1.strict)
        assert np.array_equal(_bits(d2.out, b2.n), b2.strict)
