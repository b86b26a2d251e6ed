"""Why do the same launches run slower on the library's compute streams?
  One process, one GPU: a config-3-shaped step (SHA-512
of 100k 72-byte preimages, one NT_MODE_MIXED key-cache launch over 6.8M
signatures, a group AND) timed kernel by kernel with HIP events on several
streams, before and after a large-scratch kernel (keygen/signing) has run on
some of them.  Prints one JSON line per (phase, stream).
Usage: python tools/stream_probe.py [reps]"""
import json
import os
import sys
import time

import numpy as np
import torch


def nbytes(t):
    """byte size of a device tensor: the msg_bytes argument of the nt_dev_* entry points"""
    return int(t.numel()) * int(t.element_size())


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "narwhal-tusk_amd"))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    torch.cuda.init()
    import ntcrypto
    be = ntcrypto.Backend(device=0)
    nk, G, Q = 100, 100_000, 67
    rng = np.random.default_rng(5)
    seeds_h = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
    pks = be.sign_batch(seeds_h)
    ks = be.keyset(pks)          # comb of B + key combs, built on library stream 0
    seeds = torch.from_numpy(seeds_h).to(dev)
    cur = torch.cuda.Stream(dev)   # like bench.py: a created stream is torch's current one
    torch.cuda.set_stream(cur)
    pre = torch.randint(0, 256, (G, 72), dtype=torch.uint8, device=dev)
    c_off = torch.arange(G, dtype=torch.int64, device=dev) * 72
    c_len = torch.full((G,), 72, dtype=torch.int64, device=dev)
    cd = torch.empty((2 * G, 32), dtype=torch.uint8, device=dev)
    be.dev_sha512(0, cur.cuda_stream, pre.data_ptr(), nbytes(pre), c_off.data_ptr(), c_len.data_ptr(), G, cd.data_ptr())
    voters = torch.rand((G, nk), device=dev).argsort(dim=1)[:, :Q].contiguous()
    V = G * Q
    vkey = torch.cat([voters.reshape(-1).to(torch.int32), torch.randint(0, nk, (G,), device=dev, dtype=torch.int32)
                      + torch.iinfo(torch.int32).min]).contiguous()
    m_off = torch.cat([(torch.arange(V, device=dev, dtype=torch.int64) // Q) * 32,
                       G * 32 + torch.arange(G, device=dev, dtype=torch.int64) * 32]).contiguous()
    m_len = torch.full((V + G,), 32, dtype=torch.int64, device=dev)
    sig = torch.empty((V + G, 64), dtype=torch.uint8, device=dev)
    tpk = torch.empty((V + G, 32), dtype=torch.uint8, device=dev)
    sd = seeds[(vkey & 0x7fffffff).long()].contiguous()
    be.dev_sign(0, cur.cuda_stream, sd.data_ptr(), cd.data_ptr(), nbytes(cd), m_off.data_ptr(), m_len.data_ptr(), V + G,
                tpk.data_ptr(), sig.data_ptr())
    first = torch.arange(G, dtype=torch.int64, device=dev) * Q
    cnt = torch.full((G,), Q, dtype=torch.int32, device=dev)
    mbits = torch.zeros(((V + G + 63) // 64 + 1,), dtype=torch.int64, device=dev)
    gbits = torch.zeros(((G + 63) // 64,), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    def streams():
        return {"lib0": torch.cuda.ExternalStream(be.dev_stream(0, 0), device=dev),
                "lib1": torch.cuda.ExternalStream(be.dev_stream(0, 1), device=dev),
                "torchA": sA, "torchB": sB}
    sA, sB = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def step(st, ev):
        q = st.cuda_stream
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        e[0].record(st)
        be.dev_sha512(0, q, pre.data_ptr(), nbytes(pre), c_off.data_ptr(), c_len.data_ptr(), G, cd.data_ptr(), max_len=72)
        e[1].record(st)
        ks.dev_verify(0, q, ntcrypto.NT_MODE_MIXED, vkey.data_ptr(), sig.data_ptr(), cd.data_ptr(), nbytes(cd), m_off.data_ptr(),
                      m_len.data_ptr(), V + G, mbits.data_ptr())
        e[2].record(st)
        be.dev_group_and(0, q, first.data_ptr(), cnt.data_ptr(), G, mbits.data_ptr(), gbits.data_ptr())
        e[3].record(st)
        ev.append(e)

    def run(phase, fork=None, names=None):
        for name, st in streams().items():
            if names and name not in names:
                continue
            torch.cuda.synchronize()
            if fork is not None:
                # the bench's fork: this stream waits for an event recorded on torch's current stream
                e0 = torch.cuda.Event(enable_timing=(fork == "timing"))
                e0.record(cur)
                if st.cuda_stream != cur.cuda_stream:
                    st.wait_event(e0)
            evs = []
            t0 = time.perf_counter()
            for _ in range(reps):
                step(st, evs)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / reps
            d = np.array([[a.elapsed_time(b) for a, b in zip(e[:-1], e[1:])] for e in evs[1:]])
            ok = int(np.unpackbits(gbits.cpu().numpy().view(np.uint8))[:G].sum())
            print(json.dumps({"phase": phase, "stream": name, "sha72_ms": round(d[:, 0].mean(), 4),
                              "keyset_ms": round(d[:, 1].mean(), 4), "group_and_ms": round(d[:, 2].mean(), 4),
                              "wall_ms_per_step": round(wall * 1e3, 3), "groups_ok": ok}), flush=True)

    run("after_setup")
    for rnd in range(2):
        for fk in ("timing", "plain", None):
            run("fork_%s_%d" % (fk, rnd), fork=fk, names=("lib0", "torchA"))
    ks.close()
    be.close()


if __name__ == "__main__":
    main()
