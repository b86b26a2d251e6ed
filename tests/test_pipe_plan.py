"""CPU tests of the host entry points' chunk plans (narwhal-tusk_amd/csrc/pipe_plan.hpp,
compiled into the host harness).  Every chunk boundary but the
end is a multiple of 64 items (a chunk owns whole 64-bit verdict words: a
boundary off 64 made two chunks write one word, the round-5 regression the GPU
test test_chunked_host_calls_match caught), the sizes add up, the count stays
within the pipeline's 16 chunk events, and the verify plan has the shape its
tail needs: a quarter-round first chunk, whole rounds, and at most half a
round last."""
import ctypes

import pytest

import _hostarith

R1 = 256 * 2 * 4 * 64  # one round at one signature per lane: 256 CUs, 2 waves per SIMD


def verify_chunks(total, r1=R1, cap=16):
    out = (ctypes.c_ulonglong * 64)()
    n = _hostarith.load().nth_verify_chunk_targets(ctypes.c_ulonglong(total), ctypes.c_ulonglong(r1),
                                                   ctypes.c_ulonglong(cap), out, 64)
    return list(out[:n])


def chunks(total, r, cap=16, round4=False):
    out = (ctypes.c_ulonglong * 64)()
    n = _hostarith.load().nth_chunk_targets(ctypes.c_ulonglong(total), ctypes.c_ulonglong(r), ctypes.c_ulonglong(cap),
                                            int(round4), out, 64)
    return list(out[:n])


def check_boundaries(t, total, cap):
    assert sum(t) == total
    assert 1 <= len(t) <= max(1, cap)
    assert all(x > 0 for x in t) or total == 0
    pos = 0
    for x in t[:-1]:
        pos += x
        assert pos % 64 == 0, t


@pytest.mark.parametrize("total", [1, 63, 64, 65, 3001, R1 // 2, R1 // 2 + R1 // 4, R1 // 2 + R1 // 4 + 1,
                                   R1, 1_000_000, 1_000_001, 6_800_000, 20_000_000])
@pytest.mark.parametrize("cap", [1, 2, 3, 16])
def test_verify_chunk_plan(total, cap):
    t = verify_chunks(total, R1, cap)
    check_boundaries(t, total, cap)
    if len(t) == 1:
        assert cap < 3 or total <= R1 // 2 + R1 // 4
        return
    assert t[0] == R1 // 4                       # the first kernel starts after a short copy
    assert t[-1] <= R1 // 2                      # the tail after the last copy: one short launch
    mids = t[1:-1]
    assert all(m % R1 == 0 for m in mids[:-1])  # whole rounds (the last middle chunk may be short)


def test_verify_chunk_plan_config2():
    """config 2's 1M verifies: a quarter round, six rounds, a part round, the last half round"""
    t = verify_chunks(1_000_000)
    assert t == [32768] + [R1] * 6 + [115264, 65536]


@pytest.mark.parametrize("pipe_round", [64, 640, 1000 // 64 * 64])
def test_small_rounds_keep_word_boundaries(pipe_round):
    """NT_PIPE_ROUND shrinks the round in tests: 3001 items split into many chunks"""
    for total in (3001, 2937, 4096, 65):
        check_boundaries(verify_chunks(total, pipe_round, 16), total, 16)
        for r4 in (False, True):
            check_boundaries(chunks(total, pipe_round, 16, r4), total, 16)


@pytest.mark.parametrize("total", [1, 100, 65536, 1_000_000, 6_800_000])
@pytest.mark.parametrize("r", [64, 1 << 16, 393216])
@pytest.mark.parametrize("round4", [False, True])
def test_chunk_plan(total, r, round4):
    for cap in (1, 2, 3, 16):
        check_boundaries(chunks(total, r, cap, round4), total, cap)


def test_group_chunks_whole_words():
    """certificate groups: chunk ends at multiples of 64 groups (whole group-verdict
    words) except the last; ragged and empty groups; every group in one chunk"""
    import numpy as np
    rng = np.random.default_rng(5)
    for G in (1, 63, 64, 203, 1000):
        cnt = rng.integers(0, 70, G).astype(np.uint32)
        total = int(cnt.sum())
        for tgt in ([total], [64 * 30, 64 * 30, total], [500] * 15 + [total]):
            targets = (ctypes.c_ulonglong * len(tgt))(*tgt)
            out = (ctypes.c_ulonglong * 64)()
            n = _hostarith.load().nth_plan_group_chunks(ctypes.c_ulonglong(G), cnt.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                                        targets, len(tgt), out, 64)
            ends = list(out[:n])
            assert ends[-1] == G and n <= len(tgt)
            assert all(e % 64 == 0 for e in ends[:-1]) and ends == sorted(ends)


@pytest.mark.parametrize("total", [2 * 393216, 2 * 393216 + 1, 3_000_000, 6_700_000, 6_800_000, 20_000_000, 100_000_000])
def test_chunk_plan_ramp(total):
    """key-cache / group plans ramp at both ends: R/8, R/4, R/2, middle chunks of
    about R/2 (bigger only when the 16-chunk cap needs it), R/4, at most R/8 last"""
    r = 1572864
    if total < 2 * r:
        r = 393216
    t = chunks(total, r, 16)
    check_boundaries(t, total, 16)
    assert t[:3] == [r // 8, r // 4, r // 2]
    assert t[-1] <= r // 8 and (t[-2] == r // 4 or t[-1] == r // 4)
    mids = t[3:-2] if t[-2] == r // 4 else t[3:-1]
    if total <= 11 * r // 2 + 5 * r // 4:  # 11 middle chunks of R/2 fit the cap
        assert all(m <= r // 2 + 64 for m in mids)
    assert max(mids) - min(mids) <= 64 or len(mids) <= 1 or mids[-1] < mids[0]


def test_chunk_plan_config3():
    """config 3's 6.8M signatures at one key-cache round of 1,572,864"""
    t = chunks(6_800_000, 1572864)
    assert t[:3] == [196608, 393216, 786432] and t[-2:] == [393216, 196608] and len(t) == 12
