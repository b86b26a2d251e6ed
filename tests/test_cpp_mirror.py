"""The reference's own hot-path tests (crypto_tests.rs, processor_tests.rs,
core_tests.rs fixtures) re-expressed in C++ against the crate mirror
(narwhal-tusk_amd/host/) -- run on the GPU through the C ABI."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")


def _build():
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "narwhal-tusk_amd")], check=True)
    subprocess.run(["make", "-s", "-C", CPP, "build/test_narwhal"], check=True)
    return os.path.join(CPP, "build", "test_narwhal")


def _golden_pks():
    with open(os.path.join(ROOT, "tests", "golden", "fixtures_reference.json")) as f:
        return [k["pk"] for k in json.load(f)["keys"]]


def test_mirror_builds_and_refuses_cpu():
    import torch
    exe = _build()
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu test")
    r = subprocess.run([exe] + _golden_pks(), capture_output=True, text=True, timeout=60)
    assert r.returncode == 3 and "no usable gfx950 device" in r.stdout


@pytest.mark.gpu
def test_reference_tests_on_gpu():
    exe = _build()
    r = subprocess.run([exe] + _golden_pks(), capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failed" in r.stdout
