"""GPU parity at BASELINE.json's full sizes, through size-independent properties
(the oracle checks the same kernels at small sizes in test_gpu_parity.py):

* config 2 -- 1M verify_strict of 512-B messages, GPU-signed, 1 % Appendix-B
  edge cases from the golden corpus: every verdict equals the corpus label /
  "valid", the device and host entry points agree, a second launch is
  identical, and flipping one message bit of 4,096 valid entries rejects
  exactly those (crypto_tests.rs:74-83 at scale).
* config 3 -- 100k certificates of an n=100 committee (67 votes + header):
  keyset and uncached paths both equal the expected verdicts (bench.py's own
  construction, incl. forged votes, wrong ids and bad header signatures).
* config 4 -- 16,384 x 500,000 B SHA-512: sampled digests equal hashlib, the
  launch is deterministic, and a one-byte edit changes exactly that digest.
"""
import hashlib
import os
import sys
import types

import numpy as np
import pytest


def nbytes(t):
    """byte size of a device tensor: the msg_bytes argument of the nt_dev_* entry points"""
    return int(t.numel()) * int(t.element_size())


pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def env():
    import torch
    import ntcrypto
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    be = ntcrypto.Backend(0)
    stream = torch.cuda.Stream(dev)
    yield types.SimpleNamespace(torch=torch, ntcrypto=ntcrypto, dev=dev, be=be, stream=stream,
                                sp=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    be.close()


def _bits(torch, out, n):
    return np.unpackbits(out.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)


def test_cfg2_million_verifies(env):
    torch, be, dev, sp = env.torch, env.be, env.dev, env.sp
    n, L = 1_000_000, 512
    g = torch.Generator(device=dev)
    g.manual_seed(99)
    with torch.cuda.stream(env.stream):
        seeds = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device=dev, generator=g)
        msgs = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
        off = torch.arange(n, dtype=torch.int64, device=dev) * L
        ln = torch.full((n,), L, dtype=torch.int64, device=dev)
        pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    be.dev_sign(0, sp, seeds.data_ptr(), msgs.data_ptr(), nbytes(msgs), off.data_ptr(), ln.data_ptr(), n, pk.data_ptr(),
                sig.data_ptr())
    torch.cuda.synchronize(dev)

    corpus = np.load(os.path.join(ROOT, "tests", "golden", "ed25519_corpus.npz"))
    pool = np.nonzero(corpus["len"] == L)[0]
    rng = np.random.default_rng(5)
    pos = np.sort(rng.choice(n, size=n // 100, replace=False))
    src = pool[np.arange(len(pos)) % len(pool)]
    expect = np.ones(n, dtype=bool)
    expect[pos] = corpus["strict"][src].astype(bool)
    pk_h, sig_h, msg_h = pk.cpu().numpy(), sig.cpu().numpy(), msgs.cpu().numpy()
    for p, s in zip(pos, src):
        o = int(corpus["off"][s])
        pk_h[p], sig_h[p] = corpus["pk"][s], corpus["sig"][s]
        msg_h[p * L:(p + 1) * L] = corpus["msg"][o:o + L]
    # one flipped message bit on 4,096 otherwise-valid entries
    valid = np.setdiff1d(np.arange(n), pos)
    flip = np.sort(rng.choice(valid, size=4096, replace=False))
    msg_h[flip * L + rng.integers(0, L, len(flip))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    expect[flip] = False
    pk.copy_(torch.from_numpy(pk_h))
    sig.copy_(torch.from_numpy(sig_h))
    msgs.copy_(torch.from_numpy(msg_h))
    torch.cuda.synchronize(dev)

    words = (n + 63) // 64
    runs = []
    for _ in range(2):
        out = torch.zeros(words, dtype=torch.int64, device=dev)
        be.dev_verify(0, sp, env.ntcrypto.NT_MODE_STRICT, pk.data_ptr(), sig.data_ptr(), msgs.data_ptr(), nbytes(msgs),
                      off.data_ptr(), ln.data_ptr(), n, out.data_ptr())
        torch.cuda.synchronize(dev)
        runs.append(_bits(torch, out, n))
    got = runs[0]
    bad = np.nonzero(got != expect)[0]
    assert len(bad) == 0, ("mismatches", len(bad), bad[:10].tolist())
    assert np.array_equal(runs[0], runs[1])
    # the host entry point (pageable buffers, chunked copies) gives the same bitmap
    hv = be.verify_strict(pk_h, sig_h, msg_h, off.cpu().numpy().astype(np.uint64),
                          ln.cpu().numpy().astype(np.uint64))
    assert np.array_equal(hv, got)


def test_cfg3_hundred_thousand_certificates(env):
    sys.path.insert(0, ROOT)
    import bench
    args = types.SimpleNamespace(committee=100, certs=100_000, steps=1, warmup=1, no_cpu=True)
    with env.torch.cuda.stream(env.stream):
        res = bench.bench_certs(args, env.torch, env.dev, env.be, env.sp, env.stream, 1, 0,
                                lambda: env.torch.cuda.synchronize(env.dev), lambda x: x)
    assert res["keyset"]["mismatches_vs_expected"] == 0
    assert res["uncached"]["mismatches_vs_expected"] == 0


def test_cfg4_sha512_full_size(env):
    torch, be, dev, sp = env.torch, env.be, env.dev, env.sp
    m, ml = 16384, 500_000
    g = torch.Generator(device=dev)
    g.manual_seed(4)
    with torch.cuda.stream(env.stream):
        data = torch.randint(0, 256, (m * ml,), dtype=torch.uint8, device=dev, generator=g)
        off = torch.arange(m, dtype=torch.int64, device=dev) * ml
        ln = torch.full((m,), ml, dtype=torch.int64, device=dev)
        out0 = torch.empty((m, 32), dtype=torch.uint8, device=dev)
        out1 = torch.empty((m, 32), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    be.dev_sha512(0, sp, data.data_ptr(), nbytes(data), off.data_ptr(), ln.data_ptr(), m, out0.data_ptr())
    torch.cuda.synchronize(dev)
    rng = np.random.default_rng(3)
    idx = np.unique(np.concatenate([[0, 63, 64, m - 1], rng.integers(0, m, 12)]))
    d0 = out0.cpu().numpy()
    for i in idx:
        b = data[i * ml:(i + 1) * ml].cpu().numpy().tobytes()
        assert d0[i].tobytes() == hashlib.sha512(b).digest()[:32], int(i)
    # one byte edited in message j: only digest j changes
    j, k = int(rng.integers(0, m)), int(rng.integers(0, ml))
    data[j * ml + k] ^= 0x5A
    torch.cuda.synchronize(dev)
    be.dev_sha512(0, sp, data.data_ptr(), nbytes(data), off.data_ptr(), ln.data_ptr(), m, out1.data_ptr())
    torch.cuda.synchronize(dev)
    d1 = out1.cpu().numpy()
    changed = np.nonzero((d0 != d1).any(axis=1))[0]
    assert changed.tolist() == [j]
    b = data[j * ml:(j + 1) * ml].cpu().numpy().tobytes()
    assert d1[j].tobytes() == hashlib.sha512(b).digest()[:32]


def test_random_corruptions_vs_oracle_200k(env, oracle):
    """200k GPU-signed verifications with a seeded mix of corruptions (bit flips
    in R, s, A and the message; s + L; s with bit 255; R replaced by a random
    encoding; A replaced by another key) and 32-1,024-B messages, each verdict
    equal to the CPU oracle's: the half-size lattice reduction (Lehmer batches),
    the joint ladder and the 24-bit comb of B meet ~200k different scalars."""
    torch, be, dev, sp = env.torch, env.be, env.dev, env.sp
    rng = np.random.default_rng(2024)
    n = 200_000
    lens = rng.integers(32, 1025, n).astype(np.uint64)
    off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    msg = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pk, sig = be.sign_batch(seeds, msg, off, lens)
    pk, sig, msg = pk.copy(), sig.copy(), msg.copy()
    kind = rng.integers(0, 10, n)                         # 0-2: untouched
    L = 2 ** 252 + 27742317777372353535851937790883648493
    for i in np.nonzero(kind == 3)[0]:
        sig[i, rng.integers(0, 32)] ^= np.uint8(1 << rng.integers(0, 8))        # R
    for i in np.nonzero(kind == 4)[0]:
        sig[i, 32 + rng.integers(0, 32)] ^= np.uint8(1 << rng.integers(0, 8))   # s
    for i in np.nonzero(kind == 5)[0]:
        pk[i, rng.integers(0, 32)] ^= np.uint8(1 << rng.integers(0, 8))         # A
    for i in np.nonzero(kind == 6)[0]:
        msg[int(off[i]) + int(rng.integers(0, int(lens[i])))] ^= 1            # message
    for i in np.nonzero(kind == 7)[0]:                                          # s + L (< 2^256)
        s = int.from_bytes(sig[i, 32:].tobytes(), "little") + L
        sig[i, 32:] = np.frombuffer(s.to_bytes(32, "little"), np.uint8)
    sig[kind == 8, 63] |= 0x80                                                  # s bit 255
    r9 = np.nonzero(kind == 9)[0]
    sig[r9[: len(r9) // 2], :32] = rng.integers(0, 256, (len(r9) // 2, 32), dtype=np.uint8)  # random R
    pk[r9[len(r9) // 2:]] = pk[(r9[len(r9) // 2:] + 1) % n]                    # another key
    got = be.verify_strict(pk, sig, msg, off, lens)
    want = oracle.verify_strict_many(pk, sig, msg, off, lens, nthreads=16).astype(bool)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, [(int(i), int(kind[i])) for i in bad[:20]]
    assert want[kind <= 2].all() and not want[(kind >= 4) & (kind <= 8)].any()


def test_sha512_bounded_hint_selects_kernel_not_result(env):
    """nt_dev_sha512_trunc32_bounded: max_len only selects the kernel (one-lane
    below 16 KB, the two-wave pipe above, for launches of <= 32,768 messages):
    digests equal hashlib whatever the hint says -- a right bound, a bound
    below some lengths (a wrong hint) and no hint -- over lengths around every
    padding edge and across the 16 KB switch."""
    torch, be, dev, sp = env.torch, env.be, env.dev, env.sp
    rng = np.random.default_rng(16)
    lens = [0, 1, 72, 111, 112, 127, 128, 129, 239, 240, 3336, 16383, 16384, 16385, 40000]
    lens += rng.integers(0, 20000, 200).tolist()
    off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    blob = rng.integers(0, 256, int(sum(lens)) + 64, dtype=np.uint8)
    want = [hashlib.sha512(blob[o:o + n].tobytes()).digest()[:32] for o, n in zip(off, lens)]
    n = len(lens)
    with torch.cuda.stream(env.stream):
        d = torch.from_numpy(blob).to(dev)
        o = torch.from_numpy(off).to(dev)
        ln = torch.tensor(lens, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    for hint in (None, max(lens), 4096, 72):
        out = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)
        be.dev_sha512(0, sp, d.data_ptr(), nbytes(d), o.data_ptr(), ln.data_ptr(), n, out.data_ptr(), max_len=hint)
        torch.cuda.synchronize(dev)
        got = out.cpu().numpy()
        bad = [i for i in range(n) if got[i].tobytes() != want[i]]
        assert not bad, (hint, bad[:5])
