"""CPU tests of the exact device arithmetic (narwhal-tusk_amd/csrc/*.hpp compiled
for the host by tests/cpp/).  These stress the radix-2^25.5 bound discipline at
the extreme limb values the point formulas can produce (a silent u64 overflow
would only show on adversarial limbs, never on random signatures), and replay
the golden corpus through the same verify_one<> / sign_one the kernels run.
"""
import hashlib
import json
import os
import random

import numpy as np
import pytest

import _hostarith as H

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
M26, M25 = (1 << 26) - 1, (1 << 25) - 1

# largest limbs the formulas in ge25519.hpp can feed into mul/sq (see fe25519.hpp header)
F_MAX = [0xFFFFFB4 + 0x8000000 if i == 0 else (0xFFFFFFC + 0x8000000 if i % 2 == 0 else 0x7FFFFFC + 0x4000000)
         for i in range(10)]                                   # fe_sub4 of (2x reduced) -> f side only
G_MAX = [0x7FFFFDA + 0x4000000 if i == 0 else (0x7FFFFFE + 0x4000000 if i % 2 == 0 else 0x3FFFFFE + 0x2000000 + (1 << 18))
         for i in range(10)]                                   # fe_sub of reduced -> either side
S_MAX = [2 * M26 if i % 2 == 0 else 2 * M25 + (1 << 18) for i in range(10)]  # sum of two reduced -> sq input


def _is_reduced(limbs):
    return all(l <= (M26 if i % 2 == 0 else M25 + (1 << 19)) for i, l in enumerate(limbs))


def _rand_limbs(rng, mx):
    return [rng.randint(0, m) for m in mx]


def test_fe_mul_extreme_bounds():
    rng = random.Random(1)
    cases = [(F_MAX, G_MAX), (F_MAX, F_MAX[:0] + [min(a, b) for a, b in zip(G_MAX, G_MAX)])]
    for _ in range(3000):
        cases.append((_rand_limbs(rng, F_MAX), _rand_limbs(rng, G_MAX)))
    for k in range(10):  # single-limb maxima
        f = [0] * 10
        f[k] = F_MAX[k]
        cases.append((f, G_MAX))
    for f, g in cases:
        out = H.fe_mul(f, g)
        assert H.value(out) % H.P == H.value(f) * H.value(g) % H.P
        assert _is_reduced(out), out


def test_fe_sq_extreme_bounds():
    rng = random.Random(2)
    cases = [S_MAX] + [_rand_limbs(rng, S_MAX) for _ in range(3000)]
    for f in cases:
        out = H.fe_sq(f)
        assert H.value(out) % H.P == H.value(f) ** 2 % H.P
        assert _is_reduced(out)


def test_fe_tobytes_canonical():
    vals = [0, 1, H.P - 1, H.P, H.P + 1, H.P + 18, 2 ** 255 - 1, 2 ** 255 - 20, 19, 2 ** 254]
    rng = random.Random(3)
    vals += [rng.randrange(0, 2 ** 255) for _ in range(500)]
    for v in vals:
        limbs = H.to_limbs(v)
        assert H.fe_tobytes(limbs) == (v % H.P).to_bytes(32, "little")
    # unreduced limb patterns (carry input) also canonicalize
    for _ in range(500):
        limbs = _rand_limbs(rng, G_MAX)
        assert H.fe_tobytes(limbs) == (H.value(limbs) % H.P).to_bytes(32, "little")


def test_sc_reduce512():
    rng = random.Random(4)
    for _ in range(2000):
        x = rng.randrange(0, 2 ** 512)
        assert H.sc_reduce512(x.to_bytes(64, "little")) == (x % H.L).to_bytes(32, "little")
    for x in (0, H.L - 1, H.L, H.L + 1, 2 ** 512 - 1, H.L * (2 ** 259)):
        x %= 2 ** 512
        assert H.sc_reduce512(x.to_bytes(64, "little")) == (x % H.L).to_bytes(32, "little")


def test_sha512_host_build():
    for n in (0, 1, 111, 112, 127, 128, 129, 255, 256, 1000, 5000):
        m = bytes(range(256)) * (n // 256 + 1)
        m = m[:n]
        assert H.sha512(m) == hashlib.sha512(m).digest()


def test_corpus_through_device_code():
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    for i in range(len(d["cat"])):
        o, n = int(d["off"][i]), int(d["len"][i])
        pk, sig, m = d["pk"][i].tobytes(), d["sig"][i].tobytes(), d["msg"][o:o + n].tobytes()
        assert H.verify(0, pk, sig, m) == bool(d["strict"][i]), i
        assert H.verify(1, pk, sig, m) == bool(d["batch_rule"][i]), i


def test_sign_fixture_through_device_code():
    with open(os.path.join(GOLD, "fixtures_reference.json")) as f:
        ref = json.load(f)
    d = bytes.fromhex(ref["hello_digest"])
    for k, s in zip(ref["keys"], ref["hello_signatures"]):
        pk, sig = H.sign(bytes.fromhex(k["seed"]), d)
        assert pk.hex() == k["pk"]
        assert sig.hex() == s


def test_opcount_matches_committed_profile():
    """profiles/opcount.json (roofline numerator) must match the current code."""
    path = os.path.join(os.path.dirname(GOLD), "..", "profiles", "opcount.json")
    if not os.path.exists(path):
        pytest.skip("profiles/opcount.json not generated yet (tools/opcount.py)")
    with open(path) as f:
        committed = json.load(f)
    import importlib.util
    spec = importlib.util.spec_from_file_location("opcount", os.path.join(os.path.dirname(GOLD), "..",
                                                                          "tools", "opcount.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    cur = mod.measure()
    for key in ("verify_strict_fe_mul", "verify_strict_fe_sq", "verify_strict_mads"):
        assert cur[key] == committed[key], key
