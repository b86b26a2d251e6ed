"""Kernel time vs signatures per launch (device-resident inputs): how much a
launch that fills the resident waves once costs compared with the steady state
of a large launch.  Prints one JSON line per kernel.

    python tools/launch_scaling.py
"""
import json
import os
import sys


def nbytes(t):
    """byte size of a device tensor: the msg_bytes argument of the nt_dev_* entry points"""
    return int(t.numel()) * int(t.element_size())


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "narwhal-tusk_amd"))


def main():
    import torch
    import ntcrypto
    dev = torch.device("cuda", 0)
    be = ntcrypto.Backend(device=0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    sp = st.cuda_stream
    N, L = 2_097_152, 512
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    seeds = torch.randint(0, 256, (N, 32), dtype=torch.uint8, device=dev, generator=g)
    msgs = torch.randint(0, 256, (N * L + 64,), dtype=torch.uint8, device=dev, generator=g)
    off = torch.arange(N, dtype=torch.int64, device=dev) * L
    ln = torch.full((N,), L, dtype=torch.int64, device=dev)
    pk = torch.empty((N, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((N, 64), dtype=torch.uint8, device=dev)
    be.dev_sign(0, sp, seeds.data_ptr(), msgs.data_ptr(), nbytes(msgs), off.data_ptr(), ln.data_ptr(), N, pk.data_ptr(),
                sig.data_ptr())
    out = torch.zeros(N // 64 + 1, dtype=torch.int64, device=dev)
    res = {}
    for n in (131072, 250000, 262144, 524288, 1048576):
        def step():
            be.dev_verify(0, sp, ntcrypto.NT_MODE_STRICT, pk.data_ptr(), sig.data_ptr(), msgs.data_ptr(), nbytes(msgs),
                          off.data_ptr(), ln.data_ptr(), n, out.data_ptr())
        step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(3):
            step()
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 3
        res[n] = {"ms": round(ms, 3), "ns_per_sig": round(ms * 1e6 / n, 2)}
        print(json.dumps({"kernel": "verify_strict", "n": n, **res[n]}), flush=True)
    # four launches of a quarter each, at their offsets (what a chunked host call does)
    for n in (250000, 262144):
        def chunked():
            for c in range(4):
                a = c * n
                be.dev_verify(0, sp, ntcrypto.NT_MODE_STRICT, pk.data_ptr() + 32 * a, sig.data_ptr() + 64 * a,
                              msgs.data_ptr(), nbytes(msgs), off.data_ptr() + 8 * a, ln.data_ptr() + 8 * a, n,
                              out.data_ptr() + 8 * (a // 64))
        chunked()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        chunked()
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        print(json.dumps({"kernel": "verify_strict x4 chunks", "n_each": n, "ms": round(ms, 3),
                          "ns_per_sig": round(ms * 1e6 / (4 * n), 2)}), flush=True)
    be.close()


if __name__ == "__main__":
    main()
