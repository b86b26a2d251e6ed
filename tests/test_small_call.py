"""The small-call path of the C ABI (include/ntcrypto.h
nt_set_small_call_path): calls below the host/GPU crossover run the SAME
device arithmetic compiled for the host (narwhal-tusk_amd/csrc/cpu_lane.cpp).

CPU: the host lane (built from the product source into tests/cpp/build/
libntlane.so) against the golden corpus -- strict verdicts, the cofactorless
batch rule, certificate groups -- and the SHA-512 vectors / reference fixtures.
GPU: through the C ABI with the path forced (NT_SMALL_ALWAYS) and in AUTO mode
(small calls served on the host, large ones on the GPU, same verdicts)."""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
LANE = os.path.join(ROOT, "tests", "cpp", "build", "libntlane.so")
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)


@pytest.fixture(scope="module")
def lane():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp"), "build/libntlane.so"], check=True)
    lib = ctypes.CDLL(LANE)
    lib.ntl_init(4)
    return lib


def _p(a, t=_u8p):
    return a.ctypes.data_as(t)


def _verify_many(lib, mode, pk, sig, msg, off, ln, threads=4):
    n = len(off)
    out = np.zeros(max(n, 1), np.uint8)
    pk, sig = np.ascontiguousarray(pk, np.uint8), np.ascontiguousarray(sig, np.uint8)
    msg = np.ascontiguousarray(msg, np.uint8) if len(msg) else np.zeros(1, np.uint8)
    off, ln = np.ascontiguousarray(off, np.uint64), np.ascontiguousarray(ln, np.uint64)
    lib.ntl_verify_many(mode, _p(pk), _p(sig), _p(msg), _p(off, _u64p), _p(ln, _u64p), ctypes.c_uint64(n), _p(out),
                        threads)
    return out[:n].astype(bool)


def _corpus():
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    return {k: d[k] for k in d.files}


def test_host_lane_corpus_strict_and_batch_rule(lane):
    c = _corpus()
    got = _verify_many(lane, 0, c["pk"], c["sig"], c["msg"], c["off"], c["len"])
    assert np.array_equal(got, c["strict"].astype(bool))
    got = _verify_many(lane, 1, c["pk"], c["sig"], c["msg"], c["off"], c["len"])
    assert np.array_equal(got, c["batch_rule"].astype(bool))


def test_host_lane_batch_groups(lane):
    g = np.load(os.path.join(GOLD, "batch_groups.npz"))
    nsig = len(g["pk"])
    off = np.zeros(nsig, np.uint64)
    for i in range(len(g["cnt"])):
        f, k = int(g["first"][i]), int(g["cnt"][i])
        off[f:f + k] = 32 * i
    bits = _verify_many(lane, 1, g["pk"], g["sig"], g["msg32"].reshape(-1), off, np.full(nsig, 32, np.uint64))
    for i in range(len(g["cnt"])):
        f, k = int(g["first"][i]), int(g["cnt"][i])
        assert bool(np.all(bits[f:f + k])) == bool(g["expect"][i]), i


def test_host_lane_sha512(lane):
    import hashlib
    vec = json.load(open(os.path.join(GOLD, "sha512_vectors.json")))
    rng = np.random.default_rng(5)
    lens = [0, 1, 3, 111, 112, 127, 128, 129, 239, 240, 255, 256, 1000, 4097, 65537]
    msgs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    # odd starting alignment: pack with a 1-byte phase
    data = np.frombuffer(b"\x00" + b"".join(msgs), np.uint8).copy()
    off = np.cumsum([1] + lens[:-1]).astype(np.uint64)
    ln = np.array(lens, np.uint64)
    out = np.zeros((len(msgs), 32), np.uint8)
    lane.ntl_sha512_trunc32_many(_p(data), _p(off, _u64p), _p(ln, _u64p), ctypes.c_uint64(len(msgs)), _p(out), 3)
    for m, d in zip(msgs, out):
        assert d.tobytes() == hashlib.sha512(m).digest()[:32]
    # the reference's fixtures: processor_tests.rs:9-46 (228-B batch), "Hello, world!",
    # the real 977 x 512-B worker batch (508,052 B) and a 500,000-B buffer
    import struct
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _oracle import expand
    ref = vec["reference_fixtures"]
    rb = ref["real_batch_977x512"]
    txs = [expand((rb["tx_label"] % i).encode(), rb["tx_len"]) for i in range(rb["ntx"])]
    blobs = [bytes.fromhex(ref["processor_batch_228B"]["hex"]), bytes.fromhex(ref["hello_world"]["hex"]),
             struct.pack("<IQ", 0, len(txs)) + b"".join(struct.pack("<Q", len(t)) + t for t in txs),
             expand(ref["buffer_500000"]["label"].encode(), 500000)]
    want = [ref[k]["digest32"] for k in ("processor_batch_228B", "hello_world", "real_batch_977x512", "buffer_500000")]
    data = np.frombuffer(b"".join(blobs), np.uint8).copy()
    ln = np.array([len(b) for b in blobs], np.uint64)
    off = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    out = np.zeros((len(blobs), 32), np.uint8)
    lane.ntl_sha512_trunc32_many(_p(data), _p(off, _u64p), _p(ln, _u64p), ctypes.c_uint64(len(blobs)), _p(out), 4)
    assert [d.tobytes().hex() for d in out] == want


# ------------------------------------------------------------------ GPU, through the C ABI
@pytest.fixture(scope="module")
def be():
    import ntcrypto
    b = ntcrypto.Backend(device=0)
    yield b
    b.close()


@pytest.mark.gpu
def test_c_abi_forced_host_lane_matches_corpus(be):
    import ntcrypto
    c = _corpus()
    be.set_small_call_path(ntcrypto.NT_SMALL_ALWAYS, 4)
    try:
        h0, g0 = be.call_counts()
        got = be.verify_strict(c["pk"], c["sig"], c["msg"], c["off"], c["len"])
        assert np.array_equal(got, c["strict"].astype(bool))
        g = np.load(os.path.join(GOLD, "batch_groups.npz"))
        ok = be.verify_batch_groups(g["pk"], g["sig"], g["first"], g["cnt"], g["msg32"].reshape(-1))
        assert np.array_equal(ok, g["expect"].astype(bool))
        import hashlib
        msgs = [b"", b"Hello, world!", bytes(range(256)) * 9]
        d = be.digest_many(msgs)
        assert [x.tobytes() for x in d] == [hashlib.sha512(m).digest()[:32] for m in msgs]
        h1, g1 = be.call_counts()
        assert h1 - h0 == 3 and g1 == g0  # all three on the host lane
    finally:
        be.set_small_call_path(ntcrypto.NT_SMALL_OFF)


@pytest.mark.gpu
def test_c_abi_auto_small_on_host_large_on_gpu(be, oracle):
    """AUTO: one verify / one 67-vote certificate / one batch digest run on the
    host lane, a 16k-signature call on the GPU; verdicts equal either way."""
    import ntcrypto
    be.set_small_call_path(ntcrypto.NT_SMALL_AUTO, 8)
    try:
        rng = np.random.default_rng(9)
        n = 16384
        seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        msg = rng.integers(0, 256, n * 32, dtype=np.uint8)
        off = np.arange(n, dtype=np.uint64) * 32
        ln = np.full(n, 32, np.uint64)
        pk, sig = be.sign_batch(seeds, msg, off, ln)
        sig = sig.copy()
        sig[::7, 33] ^= 2
        want = np.ones(n, bool)
        want[::7] = False
        h0, g0 = be.call_counts()
        assert np.array_equal(be.verify_strict(pk[:1], sig[:1], msg, off[:1], ln[:1]), want[:1])
        h1, g1 = be.call_counts()
        assert (h1 - h0, g1 - g0) == (1, 0)
        assert np.array_equal(be.verify_strict(pk, sig, msg, off, ln), want)
        h2, g2 = be.call_counts()
        assert (h2 - h1, g2 - g1) == (0, 1)
        # one certificate of 67 votes over one digest
        d = msg[:32]
        m67 = np.tile(d, 67)
        pk67, sig67 = be.sign_batch(seeds[:67], m67, np.arange(67, dtype=np.uint64) * 32, np.full(67, 32, np.uint64))
        ok = be.verify_batch_groups(pk67, sig67, np.array([0], np.uint64), np.array([67], np.uint32), d)
        assert ok[0] and oracle.verify_batch(list(map(bytes, pk67)), list(map(bytes, sig67)), d.tobytes())
        h3, g3 = be.call_counts()
        assert (h3 - h2, g3 - g2) == (1, 0)
        # one 508,052-B worker batch
        import hashlib
        big = rng.integers(0, 256, 508052, dtype=np.uint8).tobytes()
        assert be.digest_many([big])[0].tobytes() == hashlib.sha512(big).digest()[:32]
        h4, g4 = be.call_counts()
        assert (h4 - h3, g4 - g3) == (1, 0)
    finally:
        be.set_small_call_path(ntcrypto.NT_SMALL_OFF)


@pytest.mark.gpu
def test_c_abi_auto_follows_calibrated_model(be):
    """The first AUTO nt_set_small_call_path calibrates the cost model on this
    context (host-lane verify / SHA-512 on one thread, pool wake-up, GPU call
    floors from real calls); AUTO routing then follows it: a verify call of the
    model's crossover size n* runs on the host lane and n* + 1 on the GPU, and
    the same for a digest call of 4 KiB messages."""
    import math

    import ntcrypto
    T = 4
    be.set_small_call_path(ntcrypto.NT_SMALL_AUTO, T)
    try:
        m = be.small_call_model()
        assert m["calibrated"] and m["threads"] == T
        assert 5 < m["cpu_verify_us"] < 500 and 100 < m["gpu_verify_us"] < 20000, m
        assert 50 < m["cpu_sha_mbs"] < 5000 and m["gpu_lane_mbs"] > 1 and m["gpu_call_us"] > 1, m

        def host_verify(n):
            t = min(T, n)
            return math.ceil(n / t) * m["cpu_verify_us"] + (m["spawn_us"] if t > 1 else 0.0) < m["gpu_verify_us"]

        def host_sha(n, L):
            t = min(T, n)
            cpu = max(L, n * L / t) / m["cpu_sha_mbs"] + (m["spawn_us"] if t > 1 else 0.0)
            gpu = m["gpu_call_us"] + L / m["gpu_lane_mbs"] + n * L / (m["pcie_gbs"] * 1e3)
            return cpu < gpu

        def crossover(pred, limit):
            ns = [n for n in range(1, limit) if pred(n)]
            return max(ns) if ns and max(ns) < limit - 1 else None

        rng = np.random.default_rng(17)
        nv = crossover(host_verify, 4000)
        assert nv is not None, m
        n = nv + 1
        seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        msg = rng.integers(0, 256, n * 32, dtype=np.uint8)
        off = np.arange(n, dtype=np.uint64) * 32
        ln = np.full(n, 32, np.uint64)
        pk, sig = be.sign_batch(seeds, msg, off, ln)
        for k, where in ((nv, "host"), (nv + 1, "gpu")):
            h0, g0 = be.call_counts()
            assert be.verify_strict(pk[:k], sig[:k], msg, off[:k], ln[:k]).all()
            h1, g1 = be.call_counts()
            assert (h1 - h0, g1 - g0) == ((1, 0) if where == "host" else (0, 1)), (k, where, m)
        L = 4096
        ns = crossover(lambda k: host_sha(k, L), 20000)
        if ns is not None:
            blob = rng.integers(0, 256, (ns + 1) * L, dtype=np.uint8)
            for k, where in ((ns, "host"), (ns + 1, "gpu")):
                msgs = [blob[i * L:(i + 1) * L].tobytes() for i in range(k)]
                h0, g0 = be.call_counts()
                be.digest_many(msgs)
                h1, g1 = be.call_counts()
                assert (h1 - h0, g1 - g0) == ((1, 0) if where == "host" else (0, 1)), (k, where, m)
    finally:
        be.set_small_call_path(ntcrypto.NT_SMALL_OFF)
