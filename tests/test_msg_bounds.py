"""The message bound of the device entry points, on the
host-compiled kernel code (tests/cpp/nt_host_harness.cpp; CPU only).

Every kernel that reads caller messages takes item i's slice through
msg_slice (narwhal-tusk_amd/csrc/nt_common.hpp): in bounds iff off <= bytes
and len <= bytes - off (no overflow); out of bounds it gets an empty slice at
the buffer's start and the item is rejected, never read.  nth_verify_item is
one item of k_ed25519_verify's body: slice, verify, AND with the bound.  An
offset the code dereferenced would crash this process (2^63 past a 1 KB
buffer), so passing these cases also shows the offset is never followed."""
import ctypes
import os

import numpy as np

import _hostarith as H

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
U64 = (1 << 64) - 1


def _slice(off, ln, nbytes):
    o = (ctypes.c_uint64 * 3)()
    H.load().nth_msg_slice(ctypes.c_uint64(off), ctypes.c_uint64(ln), ctypes.c_uint64(nbytes), o)
    return tuple(int(x) for x in o)


def test_msg_slice_edges():
    cases = [  # (off, len, bytes) -> in bounds?
        (0, 0, 0, True), (0, 0, 1024, True), (1024, 0, 1024, True), (1025, 0, 1024, False),
        (0, 1024, 1024, True), (1, 1024, 1024, False), (1000, 24, 1024, True), (1000, 25, 1024, False),
        (U64, 0, 1024, False), (U64, 2, 1024, False), (5, U64 - 3, 1024, False), (1 << 63, (1 << 63) - 1, U64, True), (1 << 63, 1 << 63, U64, False),
        ((1 << 63) + 1, 1 << 63, U64, False), (U64, 0, U64, True), (0, U64, U64, True),
    ]
    for off, ln, nb, ok in cases:
        so, sl, sok = _slice(off, ln, nb)
        assert sok == int(ok), (off, ln, nb)
        assert (so, sl) == ((off, ln) if ok else (0, 0)), (off, ln, nb)


def test_verify_item_rejects_out_of_bounds_without_reading():
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    lib = H.load()
    lib.nth_verify_item.restype = ctypes.c_int
    lib.nth_verify_item.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64,
                                    ctypes.c_uint64, ctypes.c_uint64]
    honest = [i for i in range(len(d["cat"])) if d["strict"][i] and int(d["len"][i]) > 0][:4]
    assert honest
    for i in honest:
        o, n = int(d["off"][i]), int(d["len"][i])
        pk, sig = d["pk"][i].tobytes(), d["sig"][i].tobytes()
        buf = bytes(64) + d["msg"][o:o + n].tobytes() + bytes(64)   # the message at offset 64 of the buffer
        nb = len(buf)
        for mode in (0, 1):
            assert lib.nth_verify_item(mode, pk, sig, buf, nb, 64, n) == 1, i
            assert lib.nth_verify_item(mode, pk, sig, buf, 64 + n, 64, n) == 1, i      # slice ends at the edge
            for off, ln, size in ((64, n, 64 + n - 1), (nb + 1, 0, nb), (1 << 63, n, nb), (U64, 2, nb),
                                  (64, U64 - 63, nb), (nb, 1, nb)):
                assert lib.nth_verify_item(mode, pk, sig, buf, size, off, ln) == 0, (i, off, ln, size)
