"""CPU tests of the key-cache launch plan (narwhal-tusk_amd/csrc/ks_plan.hpp,
compiled into the host harness): a launch's rows of 64 signatures are cut into
rounds x waves chunks of base or base + 1 rows (<= the per-lane cap), every row
in exactly one chunk, and the config-3 shard sizes of 1/2/4/8 GPUs get plans
whose worst wave carries at most one row more than the average (VERDICT r02:
the fixed 8-rows-per-wave grid left 0.54 of a round for the 8-GPU shard)."""
import ctypes
import math

import pytest

import _hostarith


def plan(n, cus=256, cap=8, force=0):
    out = (ctypes.c_uint32 * 6)()
    _hostarith.load().nth_ks_plan(ctypes.c_ulonglong(n), cus, cap, force, out)
    return dict(zip(("waves", "chunks", "base", "extra", "per_simd", "rounds"), list(out)))


def check(n, cus, cap, force):
    p = plan(n, cus, cap, force)
    rows = (n + 63) // 64
    assert p["per_simd"] in (2, 3)
    if force:
        assert p["per_simd"] == force
    assert 1 <= p["waves"] <= p["per_simd"] * 4 * cus
    assert p["waves"] == min(rows, p["per_simd"] * 4 * cus)
    assert p["chunks"] == min(p["rounds"] * p["waves"], rows)
    # every row in exactly one chunk: chunk c = [c*base + min(c, extra), +base + (c < extra))
    assert p["base"] * p["chunks"] + p["extra"] == rows
    assert p["base"] >= 1 and p["extra"] < p["chunks"]
    assert p["base"] + (1 if p["extra"] else 0) <= cap
    # the fewest rounds at <= cap rows per chunk, or two instead of one (ks_plan.hpp: one claim per
    # wave leaves nothing to rebalance)
    kmin = math.ceil(rows / (cap * p["waves"]))
    assert p["rounds"] == kmin or (kmin == 1 and p["rounds"] == 2)
    return p


@pytest.mark.parametrize("cus", [1, 4, 80, 256, 304])
def test_plan_invariants(cus):
    for n in [1, 2, 63, 64, 65, 1000, 4095, 65536, 131071, 200_000, 850_000, 1_000_000, 1_703_375, 3_406_750,
              6_813_500, 8 << 20]:
        for cap in (1, 3, 5, 8, 26, 64):
            for force in (0, 2, 3):
                check(n, cus, cap, force)


def test_config3_shards_are_balanced():
    """Config 3's mixed launch: 100k certificates x (67 votes + 1 header) on one
    GPU, and the 50k / 25k / 12.5k-certificate shards of 2/4/8 GPUs."""
    for certs, cap in [(c, cap) for c in (100_000, 50_000, 25_000, 12_500) for cap in (8, 64)]:
        n = certs * 68
        p = check(n, 256, cap, 0)
        rows = (n + 63) // 64
        per_wave = rows / p["waves"]
        pmax = p["base"] + (1 if p["extra"] else 0)
        # the worst wave runs `rounds` chunks of pmax rows: at most `rounds` rows above the average
        assert p["rounds"] * pmax - per_wave <= p["rounds"]
        # and every SIMD slot of the plan has work (no lone tail waves)
        assert p["waves"] == p["per_simd"] * 4 * 256
    # 1 GPU: 3 waves per SIMD, 5 rounds of 7-8 rows (was: 13,282 waves of 8 rows = 4.32 rounds)
    p = plan(6_800_000)
    assert (p["per_simd"], p["rounds"], p["base"]) == (3, 5, 6)


def test_default_cap_plans():
    """The default cap (64 rows per chunk, NT_KS_PER_LANE): the plans the
    round-3 A/B measured best (profiles/r03/ab_ks_plan*): 1 GPU 2 waves per SIMD
    x 2 chunks of 25-26 rows; the 2-GPU shard 2 x 12-13; the 4- and 8-GPU
    shards one chunk of 12-13 / 6-7 rows."""
    want = {6_800_000: (2, 2, 25), 3_400_000: (2, 2, 12), 1_700_000: (2, 1, 12), 850_000: (2, 1, 6)}
    for n, (w, k, base) in want.items():
        p = check(n, 256, 64, 0)
        assert (p["per_simd"], p["rounds"], p["base"]) == (w, k, base), (n, p)


def stream_plan(n, cus=256, cap=64, force=0):
    out = (ctypes.c_uint32 * 4)()
    _hostarith.load().nth_ks_stream_plan(ctypes.c_ulonglong(n), cus, cap, force, out)
    return dict(zip(("waves", "rows", "prow", "per_simd"), list(out)))


@pytest.mark.parametrize("cus", [1, 4, 80, 256, 304])
def test_stream_plan_invariants(cus):
    """Streamed rows (ks_stream_plan, the default): every SIMD slot of the
    grid has a wave while rows last, a wave stages at most `cap` rows per
    inversion and room for two rows above the average, so the stash
    (waves x prow rows) covers every row of the launch whenever cap allows."""
    for n in [1, 63, 64, 65, 4095, 65536, 200_000, 850_000, 1_000_000, 1_703_375, 3_406_750, 6_813_500, 8 << 20]:
        for cap in (1, 3, 8, 26, 64):
            for force in (0, 2, 3):
                p = stream_plan(n, cus, cap, force)
                rows = (n + 63) // 64
                per = force or (3 if rows >= 16 * 12 * cus else 2)
                assert p["per_simd"] == per
                assert p["rows"] == rows
                assert p["waves"] == min(rows, per * 4 * cus)
                avg = math.ceil(rows / p["waves"])
                assert p["prow"] == min(cap, avg + 2) >= 1
                if cap >= avg + 2:
                    assert p["waves"] * p["prow"] >= rows + 2 * p["waves"]


def test_stream_plan_config3_shards():
    """Config 3 (100k certificates x 68 signatures) and its 2/4/8-GPU shards:
    3 waves per SIMD on 1 and 2 GPUs (35 / 17 rows per wave), 2 on 4 and 8, one
    inversion per wave (the stash holds every row a wave takes, two to spare)."""
    for certs, waves in ((100_000, 3072), (50_000, 3072), (25_000, 2048), (12_500, 2048)):
        p = stream_plan(certs * 68)
        assert p["waves"] == waves
        assert p["prow"] == math.ceil(p["rows"] / waves) + 2 <= 64


def test_stash_bound_covers_every_smaller_launch():
    """the host entry points size both stashes once for their
    largest chunk and launch smaller chunks into them, so the stash size
    (ks_stash_rows_bound, keyset_stash_bytes) must bound waves x stash rows of
    EVERY plan of a launch of at most that many rows -- the chunked plan's own
    figure is not monotone (36,864 rows on 256 CUs plan 18,432 stash rows with
    2 waves per SIMD x 2 rounds; 30,720 rows plan 30,720 with 3 x 1)."""
    lib = _hostarith.load()
    lib.nth_ks_stash_rows_bound.restype = ctypes.c_ulonglong
    bound = lambda rows, cus: lib.nth_ks_stash_rows_bound(ctypes.c_ulonglong(rows), cus)
    def stash_rows(p):
        return p["waves"] * (p["base"] + (1 if p["extra"] else 0))
    # the worked example: the smaller launch needs the larger stash
    assert stash_rows(plan(30_720 * 64, 256, 64, 0)) > stash_rows(plan(36_864 * 64, 256, 64, 0))
    for cus in (4, 80, 256):
        prev = 0
        for rows in list(range(1, 3000, 37)) + [12_287, 12_288, 13_282, 26_563, 30_720, 36_864, 53_125, 106_250,
                                                131_072]:
            b = bound(rows, cus)
            assert b >= prev  # monotone
            prev = b
            n = rows * 64
            for cap in (1, 8, 26, 64):
                for force in (0, 2, 3):
                    p = plan(n, cus, cap, force)
                    assert stash_rows(p) <= b, (rows, cus, cap, force)
                for force in (0, 1, 2, 3):  # 1: NT_KEYSET_WAVES=1, streamed plan only
                    s = stream_plan(n, cus, cap, force)
                    assert s["waves"] * s["prow"] <= b, (rows, cus, cap, force)
