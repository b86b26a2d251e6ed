"""CPU-only checks of the drop-in boundary: libntcrypto.so loads, exports every
function include/ntcrypto.h declares, and fails loudly (no CPU fallback) when
no gfx950 device is present."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "ntcrypto.h")
LIB = os.path.join(ROOT, "narwhal-tusk_amd", "lib", "libntcrypto.so")


def _declared():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nt_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "narwhal-tusk_amd")], check=True)
    return ctypes.CDLL(LIB)


def test_header_declares_the_boundary():
    names = _declared()
    for must in ("nt_init", "nt_free", "nt_sha512_trunc32", "nt_ed25519_verify_strict",
                 "nt_ed25519_verify_batch_groups", "nt_dev_ed25519_verify"):
        assert must in names


def test_every_declared_symbol_is_exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (nt_[a-z0-9_]+)", out))
    missing = [n for n in _declared() if n not in exported]
    assert not missing, missing
    for n in _declared():
        getattr(lib, n)


def test_python_binding_covers_the_header():
    import ntcrypto
    assert sorted(ntcrypto.EXPORTED) == _declared()


def test_no_cpu_path(lib):
    ctx = ctypes.c_void_p()
    lib.nt_strerror.restype = ctypes.c_char_p
    assert lib.nt_init(ctypes.byref(ctx), -1) == -4  # NT_ENODEV: CPU-only is refused
    assert b"no usable gfx950 device" in lib.nt_strerror(-4)
    lib.nt_version.restype = ctypes.c_char_p
    assert b"gfx950" in lib.nt_version()


def test_python_backend_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import ntcrypto
    with pytest.raises(ntcrypto.NtError):
        ntcrypto.Backend(0)


def test_product_library_does_not_link_the_oracle():
    out = subprocess.run(["ldd", LIB], capture_output=True, text=True).stdout
    assert "ntoracle" not in out and "nthost" not in out
    syms = subprocess.run(["nm", "-D", LIB], capture_output=True, text=True).stdout
    assert "ntor_" not in syms
