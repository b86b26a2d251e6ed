"""CPU tests of the host-side routing rules of the C ABI
and of the key registry's host index (narwhal-tusk_amd/csrc/small_model.hpp,
key_table.hpp, compiled into the host harness).

Routing: a verify call runs on the host lane iff ceil(n / T) x cpu_verify_us
(+ spawn_us when T > 1) is below the GPU floor of the kernel the call would
run -- gpu_keyset_us for key-cache calls, gpu_verify_us for the uncached
kernel.  So the key cache's lower floor moves the crossover down: a
67-vote certificate (Certificate::verify's verify_batch,
primary/src/core.rs:349-411) can go to the host lane against the uncached
kernel's ~1.3 ms and to the GPU against the key cache's few hundred us.

Key index: every registered key is found at its own index, repeated keys keep
their first index, keys that share their first 8 bytes with a registered one
(the slot's fast-reject word) and random keys miss, for several hash seeds."""
import ctypes
import math

import numpy as np

import _hostarith


def route(m, nsig, threads, kind):
    arr = (ctypes.c_double * 4)(m["cpu_verify_us"], m["spawn_us"], m["gpu_verify_us"], m["gpu_keyset_us"])
    return bool(_hostarith.load().nth_small_verify_on_host(arr, ctypes.c_ulonglong(nsig), threads, kind))


def model_rule(m, nsig, threads, kind):
    t = max(1, min(threads, nsig))
    cpu = math.ceil(nsig / t) * m["cpu_verify_us"] + (m["spawn_us"] if t > 1 else 0.0)
    return cpu < (m["gpu_keyset_us"] if kind == 1 else m["gpu_verify_us"])


# a calibrated model of the kind nt_small_call_model reports on MI355X + EPYC (bench.py latency)
MODEL = {"cpu_verify_us": 36.0, "spawn_us": 15.0, "gpu_verify_us": 1300.0, "gpu_keyset_us": 250.0}


def test_route_matches_the_documented_rule():
    for m in (MODEL, dict(MODEL, gpu_keyset_us=90.0), dict(MODEL, cpu_verify_us=80.0, spawn_us=40.0)):
        for threads in (1, 4, 16):
            for kind in (0, 1):
                for n in list(range(1, 200)) + [511, 512, 1024, 4096, 65536]:
                    assert route(m, n, threads, kind) == model_rule(m, n, threads, kind), (m, n, threads, kind)


def test_key_cache_floor_moves_the_crossover():
    T = 16
    # a lone strict vote / header: the host lane wins against either kernel
    assert route(MODEL, 1, T, 0) and route(MODEL, 1, T, 1)
    # one 67-vote certificate: host lane against the uncached kernel, GPU against the key cache
    # (5 rounds of 36 us + 15 us spawn = 195 us < 250 us: still host with this model) ...
    assert route(MODEL, 67, T, 0)
    assert route(MODEL, 67, T, 1)
    # ... and the GPU once the key-cache floor is below the host lane's time
    fast = dict(MODEL, gpu_keyset_us=150.0)
    assert route(fast, 67, T, 0) and not route(fast, 67, T, 1)

    def crossover(m, kind):
        return max(n for n in range(1, 100000) if route(m, n, T, kind))

    nu, nk = crossover(MODEL, 0), crossover(MODEL, 1)
    assert nk < nu
    assert model_rule(MODEL, nk, T, 1) and not model_rule(MODEL, nk + 1, T, 1)
    assert model_rule(MODEL, nu, T, 0) and not model_rule(MODEL, nu + 1, T, 0)


def _find(keys, queries, seed=0):
    keys = np.ascontiguousarray(keys, np.uint8).reshape(-1, 32)
    queries = np.ascontiguousarray(queries, np.uint8).reshape(-1, 32)
    out = np.zeros(max(1, len(queries)), np.uint32)
    kb = keys if len(keys) else np.zeros((1, 32), np.uint8)
    _hostarith.load().nth_key_table_find(kb.ctypes.data_as(ctypes.c_void_p), len(keys), ctypes.c_ulonglong(seed),
                                         queries.ctypes.data_as(ctypes.c_void_p), ctypes.c_ulonglong(len(queries)),
                                         out.ctypes.data_as(ctypes.c_void_p))
    return out[:len(queries)]


MISS = 0xFFFFFFFF


def test_key_table_finds_every_registered_key():
    rng = np.random.default_rng(3)
    for n in (1, 2, 4, 67, 100, 1000, 4095):
        keys = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        for seed in (0, 1, 12345):
            got = _find(keys, keys, seed)
            assert np.array_equal(got, np.arange(n, dtype=np.uint32)), (n, seed)
            other = rng.integers(0, 256, (500, 32), dtype=np.uint8)
            assert (_find(keys, other, seed) == MISS).all()


def test_key_table_near_misses_and_repeats():
    rng = np.random.default_rng(4)
    keys = rng.integers(0, 256, (100, 32), dtype=np.uint8)
    # same first 8 bytes (the slot's fast-reject word), any later byte different
    near = keys.copy()
    near[np.arange(100), 8 + np.arange(100) % 24] ^= 1
    assert (_find(keys, near) == MISS).all()
    # same tail, different head
    near2 = keys.copy()
    near2[:, 0] ^= 0x80
    assert (_find(keys, near2) == MISS).all()
    # a repeated key keeps its first index; an empty table finds nothing
    rep = np.concatenate([keys[:10], keys[3:4], keys[10:]])
    got = _find(rep, keys)
    assert np.array_equal(got, np.concatenate([np.arange(10), np.arange(11, 101)]).astype(np.uint32))
    assert (_find(np.zeros((0, 32), np.uint8), keys[:5]) == MISS).all()
    # colliding heads: keys that differ only after byte 8 all land in one probe run
    same = np.tile(keys[:1], (64, 1))
    same[:, 31] = np.arange(64)
    assert np.array_equal(_find(same, same), np.arange(64, dtype=np.uint32))
    q = same.copy()
    q[:, 31] += 64
    assert (_find(same, q) == MISS).all()
