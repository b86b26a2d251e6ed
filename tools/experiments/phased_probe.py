"""Probe of a verify launch on the GPU (written for the phased-kernel experiment,
DESIGN.md §10, which is not in the product): one launch at a time with
timestamps, so a slow or stuck step names itself (faulthandler dumps the
Python stack if a step takes longer than the watchdog)."""
import faulthandler
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "narwhal-tusk_amd"))
faulthandler.dump_traceback_later(int(os.environ.get("PROBE_WATCHDOG", "60")), repeat=True)
T0 = time.time()


def say(*a):
    print("[%7.2f]" % (time.time() - T0), *a, flush=True)


import torch  # noqa: E402
import ntcrypto  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
say("torch up")
be = ntcrypto.Backend(0)
say("backend up")
st = torch.cuda.Stream(dev)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 131_109
L = 512
g = torch.Generator(device=dev)
g.manual_seed(5)
seeds = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device=dev, generator=g)
msgs = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
off = torch.arange(n, dtype=torch.int64, device=dev) * L
ln = torch.full((n,), L, dtype=torch.int64, device=dev)
pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
torch.cuda.synchronize(dev)
be.dev_sign(0, st.cuda_stream, seeds.data_ptr(), msgs.data_ptr(), off.data_ptr(), ln.data_ptr(), n, pk.data_ptr(),
            sig.data_ptr())
torch.cuda.synchronize(dev)
say("signed", n)
out = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
for rep in range(3):
    t = time.time()
    be.dev_verify(0, st.cuda_stream, ntcrypto.NT_MODE_STRICT, pk.data_ptr(), sig.data_ptr(), msgs.data_ptr(),
                  off.data_ptr(), ln.data_ptr(), n, out.data_ptr())
    say("launched")
    torch.cuda.synchronize(dev)
    bits = np.unpackbits(out.cpu().numpy().view(np.uint8), bitorder="little")[:n]
    say("verify %d: %.2f ms, %d valid of %d" % (rep, (time.time() - t) * 1e3, int(bits.sum()), n))
    bad = np.nonzero(bits == 0)[0]
    if len(bad):
        units, cnt = np.unique(bad // 64, return_counts=True)
        say("  bad units %d: first %s counts %s lanes %s" % (len(units), units[:12].tolist(), cnt[:12].tolist(),
                                                          np.unique(bad % 64)[:16].tolist()))
say("done")
