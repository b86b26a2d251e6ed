#!/usr/bin/env python3
"""Benchmark of the Narwhal/Tusk crypto hot path on MI355X (gfx950).

Metric (BASELINE.json): "Ed25519 verifies/sec + SHA-512 GB/s at 1/2/4/8 MI355X vs
dalek host-core base".

Headline line (`value`): BASELINE config 2 -- 1,000,000 independent
verify_strict calls (crypto/src/lib.rs:200-204) over 512-byte messages with
random keys and a 1 % edge-case mix (drawn from the
committed golden corpus), inputs resident in HBM, per GPU (weak scaling: every
rank verifies its own 1M).  A step = one verify launch over the 1M batch;
consecutive steps alternate between two streams on separate hardware queues
(pipelined: the next batch fills the last round the previous one leaves
idle), the strictly back-to-back rate is reported beside it (`one_stream`),
and the roofline uses the back-to-back launches' own durations.

Secondary (same JSON line, "sha512"): BASELINE config 4 -- SHA-512[..32] of
16,384 x 500,000-byte batches (worker/src/processor.rs:38), GB/s.

`roofline` is for the dominant kernel (k_ed25519_verify<strict>): it is an
integer-VALU kernel, so achieved/peak are 32x32->64 multiply-accumulates per
second (the algorithmic v_mad_u64_u32 count per verify)
against the gfx950 issue peak of that instruction.

`cpu_baseline`: the repo's CPU restatement (oracle/, radix-2^51 like the
curve25519-dalek u64 backend) on a bounded sample of the same workload,
rank 0 at N=1 only -- a reported baseline, also used as an in-bench parity
check of the sample.

Launch: python bench.py [--gpus N --steps K --warmup W].  One process per GPU;
gloo only for the barrier and the max-over-ranks timing (the data path has no
collective).  Under torch.distributed.run (WORLD_SIZE set) each process is one
rank; a plain `python bench.py --gpus N` with N > 1 starts the N ranks itself
(torch.distributed.run as a child process, before this process touches the
GPU) and exits with their status.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np


def nbytes(t):
    """byte size of a device tensor: the msg_bytes argument of the nt_dev_* entry points"""
    return int(t.numel()) * int(t.element_size())


ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "narwhal-tusk_amd"))

METRIC = "Ed25519 verifies/sec + SHA-512 GB/s at 1/2/4/8 MI355X vs dalek host-core base"
MAD_PEAK_TS = 256 * 4 * 64 * 2.4e9 / 4 / 1e12  # v_mad_u64_u32: 4 cycles per wave64 per SIMD
MAD_MEASURED_TS = 32.80  # profiles/r01_alu_rate.txt (tools/microbench): 4.80 cycles per wave64 per SIMD
HBM_PEAK_GBS = 8000.0
PMC_PROFILE = os.path.join("r06", "pmc_verify_sha.json")  # tools/runs/r06/r06p.sh + tools/pmc_summarize.py
PMC_KEYSET_PROFILE = os.path.join("r06", "pmc_keyset.json")  # cfg3 key-cache launch (streamed rows)
PMC_N = 1_000_000  # signatures per launch in that profile (the default config-2 run)
SODIUM = "/opt/conda/lib/libsodium.so.23"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sigs", type=int, default=1_000_000, help="signatures per GPU (config 2: 1M)")
    ap.add_argument("--msg-len", type=int, default=512)
    ap.add_argument("--sha-msgs", type=int, default=16384, help="config 4 messages (total, sharded)")
    ap.add_argument("--sha-len", type=int, default=500_000)
    ap.add_argument("--no-sha", action="store_true")
    ap.add_argument("--certs", type=int, default=100_000, help="config 3 certificates (total, sharded)")
    ap.add_argument("--committee", type=int, default=100)
    ap.add_argument("--no-certs", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-ingest", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--ingest-threads", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-seconds of baseline work")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0 = every CPU this process may use, see host_cpu)")
    return ap.parse_args()


def host_cpu():
    """The host the CPU baselines run on: the machine's CPU count and model, and
    how many of those CPUs this process may actually use (affinity mask and
    cgroup CPU quota).  On the GPU pool a one-GPU box is a share of a larger
    machine (16 CPUs per GPU) whose nproc counts every CPU of the machine:
    threads beyond the share only time-slice, so the baseline runs on the
    usable CPUs and `full_host_estimate` scales its per-thread rate to nproc."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = nproc
    quota = None
    for path, conv in (("/sys/fs/cgroup/cpu.max", lambda t: None if t[0] == "max" else int(t[0]) / int(t[1])),
                       ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as f:
                txt = f.read().split()
            if conv is not None:
                quota = conv(txt)
            else:
                q = int(txt[0])
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    per = int(f.read().split()[0])
                quota = None if q <= 0 else q / per
            break
        except Exception:
            continue
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    policy_cap = None
    if quota is None and usable > 16 and os.environ.get("GRAFT_REPO_ROOT"):
        policy_cap = 16  # the pool's per-GPU CPU share when the box does not enforce one
        usable = 16
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except Exception:
        pass
    return {"nproc": nproc, "affinity_cpus": aff, "cgroup_quota_cpus": quota, "usable_cpus": usable,
            "policy_cap": policy_cap, "model": model}


def cpu_threads(args):
    return args.cpu_threads if args.cpu_threads > 0 else host_cpu()["usable_cpus"]


def full_host(rate, threads, host):
    """Per-thread rate x the machine's CPU count: what the same code would reach
    on every core of the host (an extrapolation, labelled as such)."""
    return {"value": round(rate / threads * host["nproc"], 1), "cores": host["nproc"],
            "note": "measured rate / %d threads x nproc %d (linear in cores: independent items, no shared "
                    "state); an estimate, not a measurement" % (threads, host["nproc"])}


def pipeline_streams(torch, be, dev, stream, n):
    """The n streams consecutive steps alternate between: the library's own
    compute streams (nt_dev_stream: the streams its host entry points pipeline
    on, so the line measures the product's stream layout).
    NT_BENCH_LIB_STREAMS=0 (A/B): `stream` and n - 1 more torch streams, as
    rounds 1-4 did (profiles/r05/ab_streams.txt)."""
    if os.environ.get("NT_BENCH_LIB_STREAMS", "1") != "0":
        return [torch.cuda.ExternalStream(be.dev_stream(0, k), device=dev) for k in range(n)]
    if n == 1:
        return [stream]
    return [stream] + [torch.cuda.Stream(dev) for _ in range(n - 1)]


class Region:
    """A timed region whose steps run on several streams.  start(): an event on
    `stream` that every other stream of the region waits for (complete when the
    wait is issued: regions start after a barrier).  end(): an end event on
    every stream; the region's GPU time is the latest of them.  There is no
    GPU-side join: a wait for the other streams enqueued on an idle `stream`
    stays pending for the whole region, and a cross-queue wait left pending
    slowed the dispatches of the other hardware queues (short kernels ~5 us ->
    ~50 us; config 3 on one library stream -5 %: profiles/r05/ab_join.txt)."""

    def __init__(self, torch, streams, stream):
        self.torch, self.stream = torch, stream
        self.others = [s for s in streams if s.cuda_stream != stream.cuda_stream]

    def start(self):
        self.ev0 = self.torch.cuda.Event(enable_timing=True)
        self.ev0.record(self.stream)
        for st in self.others:
            st.wait_event(self.ev0)

    def end(self):
        self.ends = []
        for st in [self.stream] + self.others:
            e = self.torch.cuda.Event(enable_timing=True)
            e.record(st)
            self.ends.append(e)

    def ms(self):
        """GPU time from start() to the last stream's end (call after a synchronize)"""
        return max(self.ev0.elapsed_time(e) for e in self.ends)


class ClockProbe:
    """The run's own clock: nt_dev_clock_probe -- the verify
    kernels' mix of v_mad_u64_u32 and 64-bit carry adds on every SIMD at two
    waves per SIMD for ~2.5 ms, each wave stamping the shader-clock and the
    100 MHz wall-clock counters -- run right before and right after a timed
    region on the region's stream.  The chip holds a clock that depends on the
    load (MI355X_MICROARCH.md "DVFS give-back"), so this is the box's clock
    under a verify-like integer load, measured in the same process; the timed
    kernels' own clock relates to it by the ratio DESIGN.md §9 records from a
    same-box PMC profile."""
    ITERS = 8192

    def __init__(self, torch, be, dev):
        self.torch, self.be = torch, be
        self.buf = torch.zeros(2, dtype=torch.int64, device=dev)

    def ghz(self, stream):
        khz = self.be.dev_clock_probe(0, stream.cuda_stream, self.ITERS, self.buf.data_ptr())
        stream.synchronize()
        cyc, wall = (int(x) for x in self.buf.cpu())
        return cyc / max(wall, 1) * khz / 1e6


def side_streams(torch, dev, n):
    """Streams for the header-id digests of the pipelined config-3 steps (one per
    pipeline slot, the highest priority: HIP keeps a queue pool per priority,
    so they never share a queue with a pipeline stream).  The header ids are
    only needed by the verdict, so their 3.3 KB serial SHA-512 chains run beside
    the signature launches instead of between two of them on the pipeline
    stream; NT_BENCH_SIDE=0: on the pipeline stream, after the
    signature launch (A/B)."""
    if n < 2 or os.environ.get("NT_BENCH_SIDE", "1") == "0":
        return None
    lo, hi = torch.cuda.Stream.priority_range()
    pr = lo if os.environ.get("NT_BENCH_SIDE_PRIO", "high") == "normal" else hi
    return [torch.cuda.Stream(dev, priority=pr) for _ in range(n)]


_T0 = time.time()
# NT_BENCH_SIDE_JOIN=0 (A/B): the pipeline stream does not wait for its step's
# side-stream header-id digests (the region's end events and barrier still do)
SIDE_JOIN = os.environ.get("NT_BENCH_SIDE_JOIN", "1") != "0"


def progress(what):
    """one stderr line per finished phase (rank 0): a long default run keeps
    writing, and the log shows where the time went"""
    if os.environ.get("RANK", "0") == "0":
        print("[bench %6.1fs] %s" % (time.time() - _T0, what), file=sys.stderr, flush=True)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_launch(argv, n, port, env=None):
    """(argv, env) of the child that runs `n` ranks of this script: one process
    per GPU through torch.distributed.run on 127.0.0.1 (the path
    shards by index, each rank verifies its own shard).  Every rank gets
    LOCAL_RANK = its device ordinal from the launcher."""
    env = dict(os.environ if env is None else env)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return cmd, env


def main():
    args = parse()
    if os.environ.get("NT_BENCH_STACKS"):
        # diagnostics: every thread's Python stack to stderr every N seconds
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["NT_BENCH_STACKS"]), repeat=True)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # nothing here has initialised the GPU: start the ranks as a child and
        # report its status (no exec from this process)
        cmd, env = rank_launch(sys.argv[1:], args.gpus, free_port())
        sys.exit(subprocess.run(cmd, env=env).returncode)
    if os.environ.get("NT_BENCH_RANK_PROBE"):
        # launcher rehearsal (tests/test_bench_launch.py): report the rank layout, touch no GPU
        local = int(os.environ.get("LOCAL_RANK", "0"))
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "world": int(os.environ.get("WORLD_SIZE", "1")),
                          "local_rank": local, "device": int(os.environ.get("NT_BENCH_DEVICE", local))}), flush=True)
        return
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    # NT_BENCH_DEVICE pins every rank to one ordinal (rehearsing N>1 on a 1-GPU box)
    local = int(os.environ.get("NT_BENCH_DEVICE", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import ntcrypto
    # precondition (INTEGRATION.md "PyTorch in the same process"): torch's bundled
    # HIP runtime starts before libntcrypto maps its tables
    assert torch.cuda.is_initialized(), "torch's HIP runtime must be initialised before nt_init"
    be = ntcrypto.Backend(device=local)
    # a real (non-null) stream: the library launches on it and the HIP events
    # bracketing the timed region are recorded on it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    assert sp != 0

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()

    from ntcrypto import dist as nd

    def max_over_ranks(x):
        return nd.reduce_max(x)

    # ---------------------------------------------------------------- inputs (config 2)
    n, L = args.sigs, args.msg_len
    g = torch.Generator(device=dev)
    g.manual_seed(20241220 + rank)
    seeds = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device=dev, generator=g)
    msgs = torch.randint(0, 256, (n * L + 64,), dtype=torch.uint8, device=dev, generator=g)
    off = torch.arange(n, dtype=torch.int64, device=dev) * L
    ln = torch.full((n,), L, dtype=torch.int64, device=dev)
    pk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    t0 = time.time()
    be.dev_sign(0, sp, seeds.data_ptr(), msgs.data_ptr(), nbytes(msgs), off.data_ptr(), ln.data_ptr(), n, pk.data_ptr(),
                sig.data_ptr())
    torch.cuda.synchronize(dev)
    gen_s = time.time() - t0
    progress("cfg2 inputs signed on the GPU (%.1f s)" % gen_s)

    # 1 % edge cases from the golden corpus (512-B entries), evenly over categories
    corpus = np.load(os.path.join(ROOT, "tests", "golden", "ed25519_corpus.npz"))
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "ed25519_corpus.json")))
    pool = [i for i in range(len(corpus["cat"])) if int(corpus["len"][i]) == L
            and meta["categories"][int(corpus["cat"][i])] != "honest"]
    by_cat = {}
    for i in pool:
        by_cat.setdefault(int(corpus["cat"][i]), []).append(i)
    cats = sorted(by_cat)
    n_edge = n // 100
    rng = np.random.default_rng(7 + rank)
    pos = np.sort(rng.choice(n, size=n_edge, replace=False))
    src = np.array([by_cat[cats[j % len(cats)]][(j // len(cats)) % len(by_cat[cats[j % len(cats)]])]
                    for j in range(n_edge)], dtype=np.int64)
    expect = np.ones(n, dtype=bool)
    expect[pos] = corpus["strict"][src].astype(bool)
    pk_h = pk.cpu().numpy()
    sig_h = sig.cpu().numpy()
    msg_h = msgs.cpu().numpy()
    for p, s in zip(pos, src):
        o = int(corpus["off"][s])
        pk_h[p] = corpus["pk"][s]
        sig_h[p] = corpus["sig"][s]
        msg_h[p * L:(p + 1) * L] = corpus["msg"][o:o + L]
    pk.copy_(torch.from_numpy(pk_h))
    sig.copy_(torch.from_numpy(sig_h))
    msgs.copy_(torch.from_numpy(msg_h))
    words = (n + 63) // 64
    # The headline: launches strictly back to back on one stream.
    # NT_BENCH_STREAMS=2 (A/B only): consecutive steps alternate between two
    # streams (nt_dev_ed25519_verify alternates its two workspaces, so the
    # launches are independent) -- measured slower or equal for config 2
    # (DESIGN.md §10), unlike config 3.
    nstreams = 2 if os.environ.get("NT_BENCH_STREAMS", "1") == "2" else 1
    streams = pipeline_streams(torch, be, dev, stream, nstreams)
    reg = Region(torch, streams, stream)
    outs = [torch.zeros(words, dtype=torch.int64, device=dev) for _ in range(2)]
    out = outs[0]
    lev = []  # per-launch (start, end) events: each launch's own duration (what rocprof reports)

    def step(i, timed=False):
        st = streams[i % nstreams]
        if timed:
            lev.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
            lev[-1][0].record(st)
        be.dev_verify(0, st.cuda_stream, ntcrypto.NT_MODE_STRICT, pk.data_ptr(), sig.data_ptr(), msgs.data_ptr(), nbytes(msgs),
                      off.data_ptr(), ln.data_ptr(), n, outs[i % nstreams].data_ptr())
        if timed:
            lev[-1][1].record(st)

    barrier()  # the inputs were written on `stream`; the library's streams are ordered against no other
    probe = ClockProbe(torch, be, dev)
    for i in range(args.warmup):
        step(i)
    clk_before = probe.ghz(streams[0])  # after the warm-up launches: the clock under load
    barrier()
    t0 = time.perf_counter()
    reg.start()
    for i in range(args.steps):
        step(i, timed=True)
    reg.end()
    barrier()
    wall = time.perf_counter() - t0
    clk_after = probe.ghz(streams[0])
    step_ms = reg.ms() / args.steps          # per batch, steady state
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in lev]))  # per launch
    ranks_cfg2 = nd.gather_object({"rank": rank, "device": local, "signatures": n, "kernel_ms": round(kernel_ms, 3),
                                   "gpu_ms_per_step": round(step_ms, 3),
                                   "wall_ms_per_step": round(wall * 1e3 / args.steps, 3),
                                   "rate": round(n * args.steps / wall, 1)})
    wall = max_over_ranks(wall)
    mism = 0
    for o in outs[:min(nstreams, args.steps)]:
        got = np.unpackbits(o.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
        mism += int((got != expect).sum())
    mism = int(max_over_ranks(mism))
    progress("cfg2 timed: %.1f M verifies/s" % (n * world * args.steps / max_over_ranks(wall) / 1e6))

    total = n * world * args.steps
    value = total / wall
    ms_per_step = wall * 1e3 / args.steps

    # algorithmic multiply-accumulates per verify (counted by tests/cpp/opcount)
    mads = mads_per_verify(L)
    achieved = mads * n / (kernel_ms * 1e-3) / 1e12
    prof = load_profile(PMC_PROFILE)
    pv = (prof or {}).get("kernels", {}).get("verify", {})
    pvl = pv.get("per_launch", {})
    roofline = {"bound": "valu", "achieved": round(achieved, 3), "peak": round(MAD_PEAK_TS, 2),
                "unit": "Tmad/s (v_mad_u64_u32 32x32->64 multiply-accumulates)",
                "frac": round(achieved / MAD_PEAK_TS, 4),
                "measured_mad_rate": MAD_MEASURED_TS,
                "frac_vs_measured_mad_rate": round(achieved / MAD_MEASURED_TS, 4),
                "measured_mad_rate_note": "v_mad_u64_u32 throughput of a dependency-free microbenchmark on the "
                                          "same GPU (profiles/r01_alu_rate.txt: 4.80 cycles per wave-instruction "
                                          "per SIMD against the nominal 4)",
                "traffic": pv.get("hbm_bytes_per_launch"),
                "traffic_note": ("HBM bytes per launch from rocprofv3 FETCH_SIZE*2 + WRITE_SIZE (profiles/%s, "
                                 "same kernel build, separate --pmc passes; the config-2 launch, grouped by grid size). "
                                 "Algorithmic minimum ~2.0 KB/verify (608 B of input + 11 comb lines of B); the rest "
                                 "(%.1f KB/verify measured) is this kernel's own per-lane [j]A/[j]R table workspace "
                                 "(2,880 B written, ~10.5 KB read) plus line over-fetch -- ~2.1 TB/s, not the limiter "
                                 "of an issue-bound kernel"
                                 % (PMC_PROFILE, (pv.get("hbm_bytes_per_launch") or 0) / PMC_N / 1e3))
                if pv else None,
                "kernel": "k_ed25519_verify<strict>", "kernel_ms": round(kernel_ms, 3),
                "mads_per_verify": mads,
                "valu_instr_per_verify": round(pvl["SQ_INSTS_VALU"] * 64 / PMC_N) if "SQ_INSTS_VALU" in pvl else None,
                "valu_issue_share": round(pv["valu_issue_share_4cyc"], 3) if "valu_issue_share_4cyc" in pv else None,
                "effective_clock_ghz": round(pv["effective_clock_ghz"], 3) if "effective_clock_ghz" in pv else None,
                "frac_at_effective_clock": (round(achieved / (MAD_PEAK_TS * pv["effective_clock_ghz"] / 2.4), 4)
                                            if "effective_clock_ghz" in pv else None),
                "clock_note": "effective clock of the config-2 launch in the PMC profile: GRBM_GUI_ACTIVE / 8 / the "
                              "dispatch's duration (MI355X_MICROARCH.md, DVFS give-back); frac_at_effective_clock "
                              "prices the mad peak at that clock instead of 2.4 GHz",
                "issue_note": "the kernel is VALU-issue-bound (issue share from the PMC profile); non-mad VALU work "
                              "(carries, pre-scaling, SHA-512, lattice reduction) is why mad frac < issue share",
                "pmc_source": "traffic, valu_instr_per_verify, valu_issue_share and effective_clock_ghz come from "
                              "profiles/%s (a separate rocprofv3 --pmc run of the same build, on another box); "
                              "run_clock is this run's own" % PMC_PROFILE}
    run_ghz = (clk_before + clk_after) / 2
    roofline["run_clock"] = {"probe_ghz_before": round(clk_before, 3), "probe_ghz_after": round(clk_after, 3),
                             "probe_ghz": round(run_ghz, 3),
                             "note": "nt_dev_clock_probe right before and right after the one-stream timed region on "
                                     "its stream (ClockProbe): the shader clock this box holds under a verify-like "
                                     "v_mad_u64_u32 load in this run"}
    # The launch's cycle count does not depend on the box: GRBM_GUI_ACTIVE per 1M launch is 188.05 /
    # 187.11 / 187.42 M in the r04 / r05 / r06 profiles (the same 5.33 G VALU).  So this run's kernel
    # clock is that count over this run's launch time, and the r05 -> now comparison separates clock
    # from code: equal cycles, different time = a different clock.
    cyc_now = pv["per_launch"]["GRBM_GUI_ACTIVE"] / 8 if "GRBM_GUI_ACTIVE" in pvl else None
    r05p = (load_profile(os.path.join("r05", "pmc_verify_sha.json")) or {}).get("kernels", {}).get("verify", {})
    cyc_r05 = r05p["per_launch"]["GRBM_GUI_ACTIVE"] / 8 if "GRBM_GUI_ACTIVE" in r05p.get("per_launch", {}) else None
    kclk = cyc_now / (kernel_ms * 1e-3) / 1e9 if cyc_now else None
    roofline["kernel_clock"] = {"cycles_per_launch": round(cyc_now) if cyc_now else None,
                                "implied_ghz": round(kclk, 3) if kclk else None,
                                "implied_over_probe": round(kclk / run_ghz, 4) if kclk else None,
                                "note": "cycles = GRBM_GUI_ACTIVE / 8 per 1M launch (%s, the same build; equal within "
                                        "0.5 %% in the r04, r05 and r06 profiles); implied_ghz = those cycles / this "
                                        "run's kernel_ms" % PMC_PROFILE}
    roofline["frac_at_run_clock"] = round(achieved / (MAD_PEAK_TS * (kclk or run_ghz) / 2.4), 4)
    # round 5's driver run: 11.308 ms per 1M launch (BENCH_r05.json); no clock was measured in that
    # run -- its launch's cycle count (r05 profile, same instruction stream) gives its implied clock
    r05_ms = 11.308
    roofline["vs_r05"] = {"kernel_ms_r05": r05_ms, "kernel_ms": round(kernel_ms, 3),
                          "time_ratio_r05_over_now": round(r05_ms / kernel_ms, 4),
                          "cycles_r05": round(cyc_r05) if cyc_r05 else None,
                          "cycles_now": round(cyc_now) if cyc_now else None,
                          "cycle_ratio_r05_over_now": round(cyc_r05 / cyc_now, 4) if cyc_r05 and cyc_now else None,
                          "implied_clock_r05_ghz": round(cyc_r05 / (r05_ms * 1e-3) / 1e9, 3) if cyc_r05 else None,
                          "implied_clock_now_ghz": round(kclk, 3) if kclk else None,
                          "note": "cycle_ratio ~1: the same code; time_ratio = the clock ratio of the two runs "
                                  "(r05's driver box held ~2.07 GHz on this launch, this box implied_clock_now)"}

    # the other two halves of the metric, filled in when their configs have run, so
    # that they sit near the front of the line (a reader of its first few hundred
    # bytes sees all of it): config 4's SHA-512 GB/s and config 3's certificates/s
    line = {"metric": METRIC, "value": round(value, 1), "unit": "verifies/s", "sha512_gbs": None,
            "certs_per_s": None, "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32 limbs / u64 acc",
            "data": "synthetic (seeded random keys and 512-B messages, GPU-signed; 1% Appendix-B edge cases "
                    "from tests/golden/ed25519_corpus.npz)",
            "config": {"workload": "cfg2: %s verify_strict per GPU, %d-B messages, 1%% edge mix"
                                   % ("1M" if n == 1_000_000 else str(n), L),
                       "n_per_gpu": n, "msg_len": L, "edge_cases": n_edge,
                       "parallelism": "shard-by-index, one process per GPU, no collective"},
            "roofline": roofline,
            "parity": {"mismatches_vs_expected": mism, "checked": n * world},
            "input_gen_s": round(gen_s, 3)}
    line["streams"] = nstreams
    if nstreams == 1 and os.environ.get("NT_BENCH_CFG2_PIPE", "1") != "0":
        ts = cfg2_two_streams(torch, be, dev, stream, ntcrypto, pk, sig, msgs, off, ln, n, words,
                              expect, args, barrier, max_over_ranks, world)
        progress("cfg2 two streams")
        if os.environ.get("NT_BENCH_HEADLINE", "pipelined") == "pipelined":
            # the headline: the same K batches of 1M, consecutive batches on two
            # streams (each batch's verdicts in its own buffer, both checked); the
            # strictly back-to-back figure stays beside it, and the roofline is
            # that run's per-launch kernel time (a pipelined launch's own span
            # covers its neighbour's tail)
            line["one_stream"] = {"value": line["value"], "ms_per_step": line["ms_per_step"],
                                  "note": "the same steps strictly back to back on one stream"}
            line["roofline"]["kernel_ms_note"] = (
                "per-launch duration from the one_stream timed region (HIP events around each launch on its "
                "stream); in the pipelined region a launch's span covers its neighbour's tail, so the "
                "kernel's own time is taken where launches do not overlap")
            line["value"] = ts["verifies_per_s"]
            line["ms_per_step"] = ts["ms_per_step"]
            line["streams"] = 2
            line["parity"]["mismatches_vs_expected"] += ts["mismatches_vs_expected"]
            line["parity"]["checked"] += n * world
            line["pipelining"] = ("value: K consecutive 1M batches alternating between two streams on separate "
                                  "hardware queues (the next batch's waves take the SIMDs the previous batch's "
                                  "last round leaves idle: 1M signatures are 15.26 lanes' worth per SIMD, run as "
                                  "16); one_stream: the same batches strictly back to back")
        else:
            line["two_streams"] = ts

    # ------------------------------------------- same cfg2 batch through the host entry point
    # (caller buffers in ordinary host memory: PCIe-inclusive, never `value`)
    h_off = np.arange(n, dtype=np.uint64) * L
    h_len = np.full(n, L, np.uint64)
    hv = be.verify_strict(pk_h, sig_h, msg_h, h_off, h_len)
    barrier()
    t0 = time.perf_counter()
    for _ in range(3):
        hv = be.verify_strict(pk_h, sig_h, msg_h, h_off, h_len)
    barrier()
    hwall = max_over_ranks((time.perf_counter() - t0) / 3)
    line["host_api"] = {"verify_strict_per_s": round(n * world / hwall, 1), "ms_per_call": round(hwall * 1e3, 3),
                        "verdicts_equal_device_path": bool(np.array_equal(hv, got)),
                        "note": "nt_ed25519_verify_strict on the same cfg2 batch from pageable host buffers "
                                "(608 MB over PCIe per call, copies of chunk c+1 under the kernels of chunk c)"}
    # the same inputs in nt_host_alloc (pinned) memory: DMA'd without the staging copy
    pk_p, sig_p, msg_p = be.pinned(pk_h.shape), be.pinned(sig_h.shape), be.pinned(msg_h.shape)
    pk_p[...] = pk_h
    sig_p[...] = sig_h
    msg_p[...] = msg_h
    hp = be.verify_strict(pk_p, sig_p, msg_p, h_off, h_len)
    barrier()
    t0 = time.perf_counter()
    for _ in range(3):
        hp = be.verify_strict(pk_p, sig_p, msg_p, h_off, h_len)
    barrier()
    pwall = max_over_ranks((time.perf_counter() - t0) / 3)
    line["host_api"]["pinned"] = {"verify_strict_per_s": round(n * world / pwall, 1),
                                  "ms_per_call": round(pwall * 1e3, 3),
                                  "verdicts_equal_device_path": bool(np.array_equal(hp, got)),
                                  "note": "inputs in nt_host_alloc memory (what a caller that owns its receive "
                                          "buffers can do): DMA straight from them"}
    del pk_p, sig_p, msg_p
    progress("cfg2 host entry point")

    # ------------------------------------------------- small calls: per-call latency
    if not args.no_latency:
        line["latency"] = bench_latency(be, pk_h, sig_h, msg_h, L)
        progress("lone-call latency")

    # ----------------------- worker digest batching (§8(f).3) and device-slot contention
    if not args.no_latency and world == 1:
        line["digest_batcher"] = bench_batcher()
        line["contention"] = bench_contention(ntcrypto, local)
        progress("digest batcher, contention")

    # ---------------------------------------------------------------- config 4: SHA-512 GB/s
    if not args.no_sha:
        line["sha512"] = bench_sha(args, torch, dev, be, sp, stream, world, rank, barrier, max_over_ranks)
        line["sha512"]["real_batch"] = bench_sha_real(args, torch, dev, be, sp, stream, world, rank, barrier,
                                                      max_over_ranks)
        progress("cfg4 SHA-512: %.0f GB/s" % line["sha512"]["value"])

    # ---------------------------------------------------------------- config 3: certificates
    if not args.no_certs:
        line["certificates"] = bench_certs(args, torch, dev, be, sp, stream, world, rank, barrier, max_over_ranks)
        progress("cfg3 certificates: %.2f M/s" % (line["certificates"]["value"] / 1e6))

    # ---------------------------------------------------------------- §8(f).2: wire ingestion
    if not args.no_ingest:
        line["ingest"] = bench_ingest(args, be, world, rank, local, max_over_ranks, barrier)
        progress("cfg3 wire ingestion")

    # ---------------------------------------------------------------- CPU baseline (rank 0, N=1)
    if world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(args, pk_h, sig_h, msg_h, L, got)
        progress("CPU baselines")

    if "sha512" in line:
        line["sha512_gbs"] = line["sha512"]["value"]
    if "certificates" in line:
        line["certs_per_s"] = line["certificates"]["value"]
    if world > 1:
        # what each rank did and how long it took (gathered outside the timed regions)
        line["per_rank"] = {"cfg2": nd.rank_summary(ranks_cfg2)}
        for key, sub in (("cfg4", line.get("sha512")), ("cfg3", line.get("certificates"))):
            if sub and "_ranks" in sub:
                line["per_rank"][key] = sub.pop("_ranks")
    else:
        for sub in (line.get("sha512"), line.get("certificates")):
            if sub:
                sub.pop("_ranks", None)
    if rank == 0:
        print(json.dumps(line), flush=True)
    be.close()
    if world > 1:
        dist.destroy_process_group()


def cfg2_two_streams(torch, be, dev, stream, ntcrypto, pk, sig, msgs, off, ln, n, words, expect, args, barrier,
                     max_over_ranks, world):
    """Config 2 with consecutive 1M batches alternating between two streams
    (pipeline_streams): the next batch's waves take the SIMDs the previous batch's last round leaves
    idle (1M signatures are 15.26 signature slots per SIMD lane, run as 16:
    DESIGN.md §12).  The headline `value` unless NT_BENCH_HEADLINE=one; verdicts of both
    output buffers checked."""
    streams = pipeline_streams(torch, be, dev, stream, 2)
    reg = Region(torch, streams, stream)
    outs = [torch.zeros(words, dtype=torch.int64, device=dev) for _ in range(2)]

    def step(i):
        be.dev_verify(0, streams[i % 2].cuda_stream, ntcrypto.NT_MODE_STRICT, pk.data_ptr(), sig.data_ptr(),
                      msgs.data_ptr(), nbytes(msgs), off.data_ptr(), ln.data_ptr(), n, outs[i % 2].data_ptr())

    barrier()  # outs (zeroed on `stream`) are written on the pipeline streams
    for i in range(max(2, args.warmup)):
        step(i)
    barrier()
    t0 = time.perf_counter()
    reg.start()
    for i in range(args.steps):
        step(i)
    reg.end()
    barrier()
    wall = max_over_ranks(time.perf_counter() - t0)
    mism = 0
    for o in outs[:min(2, args.steps)]:
        got = np.unpackbits(o.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
        mism += int((got != expect).sum())
    return {"verifies_per_s": round(n * world * args.steps / wall, 1), "ms_per_step": round(wall * 1e3 / args.steps, 3),
            "gpu_ms_per_step": round(reg.ms() / args.steps, 3),
            "mismatches_vs_expected": int(max_over_ranks(mism)),
            "note": "consecutive 1M batches alternating between two streams on different hardware queues: the "
                    "headline `value` (NT_BENCH_HEADLINE=one makes it the one-stream rate, launches strictly back "
                    "to back, which `one_stream` reports beside it)"}


def bench_sha(args, torch, dev, be, sp, stream, world, rank, barrier, max_over_ranks):
    from ntcrypto import dist as nd
    m_total, ml = args.sha_msgs, args.sha_len
    lo, hi = nd.shard(m_total, world, rank)  # this rank's shard of the 16,384 messages
    m = hi - lo
    g = torch.Generator(device=dev)
    g.manual_seed(4242 + rank)
    data = torch.randint(0, 256, (m * ml + 64,), dtype=torch.uint8, device=dev, generator=g)
    off = torch.arange(m, dtype=torch.int64, device=dev) * ml
    ln = torch.full((m,), ml, dtype=torch.int64, device=dev)
    out = torch.empty((m, 32), dtype=torch.uint8, device=dev)

    def step():
        be.dev_sha512(0, sp, data.data_ptr(), nbytes(data), off.data_ptr(), ln.data_ptr(), m, out.data_ptr())

    steps = max(1, min(args.steps, 5))
    for _ in range(max(1, args.warmup)):
        step()
    barrier()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        step()
    ev1.record(stream)
    barrier()
    wall_r = time.perf_counter() - t0
    wall = max_over_ranks(wall_r)
    kms = ev0.elapsed_time(ev1) / steps
    ranks = nd.gather_object({"rank": rank, "messages": m, "kernel_ms": round(kms, 3),
                              "wall_ms_per_step": round(wall_r * 1e3 / steps, 3),
                              "rate": round(m * ml * steps / wall_r / 1e9, 2) if wall_r > 0 else 0.0})
    # spot-check 4 digests against hashlib
    import hashlib
    ok = True
    idx = [0, m // 3, (2 * m) // 3, m - 1] if m else []
    for i in idx:
        b = data[i * ml:(i + 1) * ml].cpu().numpy().tobytes()
        ok &= hashlib.sha512(b).digest()[:32] == out[i].cpu().numpy().tobytes()
    padded = (ml + 17 + 127) // 128 * 128
    gbs = m_total * ml / wall * steps / 1e9 if wall > 0 else 0.0
    pv = (load_profile(PMC_PROFILE) or {}).get("kernels", {}).get("sha512", {})
    res = {"value": round(gbs, 2), "unit": "GB/s (message bytes)", "workload": "cfg4: %d x %d B" % (m_total, ml),
           "ms_per_step": round(wall * 1e3 / steps, 3), "kernel_ms": round(kms, 3),
           "hbm_frac": round((m * padded / (kms * 1e-3)) / 1e9 / HBM_PEAK_GBS, 4),
           "valu_issue_share": round(pv["valu_issue_share_4cyc"], 3) if "valu_issue_share_4cyc" in pv else None,
           "note": "k_sha512_pipe: per 64 messages a producer wave expands K+W into LDS, a consumer wave runs the rounds; bound by the consumer wave's serial per-block stream (latency-bound, SURVEY H2), not HBM; valu_issue_share from the PMC profile (256 consumer + 256 producer waves on 1,024 SIMDs)",
           "spot_check_ok": bool(ok), "_ranks": nd.rank_summary(ranks)}
    # the shards one GPU holds when config 4 runs on N = 2 / 4 / 8 GPUs: each is
    # timed on this GPU, and the N-GPU aggregate follows as N x its per-GPU rate.
    # A lane per message is bound by one lane's serial ~3,907-block chain, so the
    # shard takes about as long as the whole batch: the aggregate stays flat.
    if world == 1 and m:
        res["shard_of"] = {}
        res["expected_aggregate_gbs"] = {"1": res["value"]}
        for N in (2, 4, 8):
            mN = (m_total + N - 1) // N
            if mN > m:
                continue

            def stepN():
                be.dev_sha512(0, sp, data.data_ptr(), nbytes(data), off.data_ptr(), ln.data_ptr(), mN, out.data_ptr())
            stepN()
            barrier()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(steps):
                stepN()
            e1.record(stream)
            barrier()
            kN = e0.elapsed_time(e1) / steps
            per = mN * ml / (kN * 1e-3) / 1e9
            res["shard_of"][str(N)] = {"messages": mN, "kernel_ms": round(kN, 3), "gb_per_s_per_gpu": round(per, 2)}
            res["expected_aggregate_gbs"][str(N)] = round(N * per, 2)
        res["scaling_note"] = ("config 4 does not scale with GPUs: a message's SHA-512 is one serial Merkle-Damgard "
                               "chain (~3,907 blocks of 500,000 B), so a GPU's shard of 16,384 / N messages takes "
                               "about as long as the whole batch; expected_aggregate_gbs = N x the measured per-GPU "
                               "rate of that shard on this GPU")
    # the same shard through the host entry point from pinned host memory
    # (PCIe-inclusive: BASELINE.md reports GPU numbers with and without H2D)
    if m:
        host = be.pinned((m * ml,))
        host[...] = data[:m * ml].cpu().numpy()
        hoff = np.arange(m, dtype=np.uint64) * ml
        hlen = np.full(m, ml, np.uint64)
        hd = be.sha512_trunc32(host, hoff, hlen)
        barrier()
        t0 = time.perf_counter()
        for _ in range(2):
            hd = be.sha512_trunc32(host, hoff, hlen)
        barrier()
        hwall = max_over_ranks((time.perf_counter() - t0) / 2)
        res["host_api"] = {"gb_per_s": round(m_total * ml / hwall / 1e9, 2), "ms_per_call": round(hwall * 1e3, 3),
                           "digests_equal_device_path": bool(np.array_equal(hd, out.cpu().numpy())),
                           "note": "nt_sha512_trunc32 on the shard from nt_host_alloc (pinned) memory: %.2f GB "
                                   "over PCIe per call, copies of chunk c+1 under the kernel of chunk c"
                                   % (m * ml / 1e9)}
        del host
    if world == 1 and not args.no_cpu:
        res["cpu_baseline"] = sha_cpu_baseline(args, data, out, m, ml)
    return res


def bench_sha_real(args, torch, dev, be, sp, stream, world, rank, barrier, max_over_ranks):
    """SURVEY §8(d) config 4 variants on the REAL worker batch: the bincode
    WorkerMessage::Batch of 977 x 512-B transactions (508,052 B, the digest
    worker/src/processor.rs:38 computes; golden digest in
    tests/golden/sha512_vectors.json).  One batch alone (the latency the
    Processor sees per call) and 16,384 copies sharded over ranks."""
    import hashlib
    import struct
    from ntcrypto import dist as nd
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "sha512_vectors.json")))
    rb = gold["reference_fixtures"]["real_batch_977x512"]
    txs = [expand((rb["tx_label"] % i).encode(), rb["tx_len"]) for i in range(rb["ntx"])]
    real = struct.pack("<IQ", 0, len(txs)) + b"".join(struct.pack("<Q", len(t)) + t for t in txs)
    bl = len(real)
    one = torch.frombuffer(bytearray(real), dtype=torch.uint8).to(dev)
    m_total = args.sha_msgs
    lo, hi = nd.shard(m_total, world, rank)
    m = hi - lo
    data = one.repeat(m)
    off = torch.arange(m, dtype=torch.int64, device=dev) * bl
    ln = torch.full((m,), bl, dtype=torch.int64, device=dev)
    out = torch.empty((m, 32), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)

    def timed(k, reps):
        be.dev_sha512(0, sp, data.data_ptr(), nbytes(data), off.data_ptr(), ln.data_ptr(), k, out.data_ptr())
        barrier()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(reps):
            be.dev_sha512(0, sp, data.data_ptr(), nbytes(data), off.data_ptr(), ln.data_ptr(), k, out.data_ptr())
        ev1.record(stream)
        barrier()
        return max_over_ranks(time.perf_counter() - t0) / reps, ev0.elapsed_time(ev1) / reps

    single_wall, single_k = timed(1, 3)
    ok1 = out[0].cpu().numpy().tobytes().hex() == rb["digest32"]
    wall, kms = timed(m, max(1, min(args.steps, 3)))
    d = out.cpu().numpy()
    okall = bool((d == d[0]).all()) and d[0].tobytes().hex() == rb["digest32"]
    return {"bytes": bl, "digest_matches_golden": bool(ok1 and okall),
            "single_batch_ms": round(single_k, 3),
            "single_batch_note": "one 508,052-B batch = one lane's serial chain of 3,970 blocks: the per-call "
                                 "latency a lone Processor call would see (SURVEY H3; batching via DigestBatcher)",
            "copies": m_total, "gbs": round(m_total * bl / wall / 1e9, 2), "kernel_ms": round(kms, 3)}


def sha_cpu_baseline(args, data, out, m, ml):
    """Config 4 on the host cores: the oracle's C SHA-512 (oracle/ntoracle.c, FIPS 180-4
    restatement of sha2's software compress) over a bounded sample of the same
    messages, args.cpu_threads threads, 1 warm-up + median of 5 runs; digests compared with the GPU's."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle
    orc = _oracle.load()
    th = cpu_threads(args)
    k = int(min(m, max(th * 8, 1024)))             # 1,024 x 500 KB = 512 MB of host copy
    host = data[:k * ml].cpu().numpy()
    offs = np.arange(k, dtype=np.uint64) * ml
    lens = np.full(k, ml, np.uint64)
    t0 = time.perf_counter()
    orc.sha512_trunc32_many(host, offs[:1], lens[:1], nthreads=1)
    one = time.perf_counter() - t0
    # repeat the sample until ~args.cpu_seconds of CPU work per run; 1 warm-up + median of 5 runs
    reps = max(1, int(round(args.cpu_seconds / 3 / (k * one))))

    def sha_run():
        for _ in range(reps):
            d = orc.sha512_trunc32_many(host, offs, lens, nthreads=th)
        return d
    dt, dig = timed_median(sha_run)
    dt /= reps
    gpu = out[:k].cpu().numpy()
    agree = int((dig == gpu).all(axis=1).sum())
    # external comparator: OpenSSL's SHA-512 through hashlib (releases the GIL), th Python threads
    import hashlib
    import threading
    ext_dig = [None] * k

    def work(t):
        for i in range(t, k, th):
            ext_dig[i] = hashlib.sha512(memoryview(host)[i * ml:(i + 1) * ml]).digest()[:32]
    def ext_run():
        for _ in range(reps):
            ts = [threading.Thread(target=work, args=(t,)) for t in range(th)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
    edt, _ = timed_median(ext_run)
    edt /= reps
    eagree = sum(int(ext_dig[i] == gpu[i].tobytes()) for i in range(k))
    host = host_cpu()
    gbs = k * ml / dt / 1e9
    return {"value": round(gbs, 3), "unit": "GB/s (message bytes)", "cores": th, "kind": "port",
            "label": "FIPS 180-4 C restatement of sha2 0.9's software compress (oracle/sha512_ref.c)",
            "sample": "first %d of the same %d-B cfg4 messages (%.0f MB) hashed %d times per run, 1 warm-up + median of 5 "
                      "runs (%.2f s wall each)" % (k, ml, k * ml / 1e6, reps, dt * reps),
            "host": host, "full_host_estimate": full_host(gbs, th, host),
            "single_thread_gbs": round(ml / one / 1e9, 3),
            "digests_agree_with_gpu": "%d/%d" % (agree, k),
            "external": {"name": "OpenSSL SHA-512 via Python hashlib", "value": round(k * ml / edt / 1e9, 3),
                         "unit": "GB/s (message bytes)", "cores": th, "kind": "external",
                         "digests_agree_with_gpu": "%d/%d" % (eagree, k)}}


def bench_certs(args, torch, dev, be, sp, stream, world, rank, barrier, max_over_ranks):
    """Config 3: Certificate::verify (primary/src/messages.rs:189-215) for 100k
    certificates of an n=100 committee, 2f+1 = 67 votes each, sharded over ranks.
    Per certificate on the GPU: SHA-512 of the header preimage (id check,
    messages.rs:70-84), SHA-512 of the certificate digest preimage (:226-234),
    verify_strict of the header signature, cofactorless verify of the 67 votes,
    group AND -- against the committee key cache (nt_keyset) and, for
    comparison, through the uncached verify path."""
    import hashlib
    import struct
    import ntcrypto

    nk = args.committee
    quorum = 2 * nk // 3 + 1                      # config/src/lib.rs:168-173 with stake 1
    from ntcrypto import dist as nd
    G_total = args.certs
    glo, ghi = nd.shard(G_total, world, rank)
    G = ghi - glo
    n_pay, n_par = 32, quorum                      # header_size 1,000 B / 32 B digests; 2f+1 parents
    hlen = 32 + 8 + 36 * n_pay + 32 * n_par
    seeds_h = np.stack([np.frombuffer(hashlib.sha512(b"nt-bench-key" + struct.pack("<Q", i)).digest()[:32], np.uint8)
                        for i in range(nk)])
    seeds = torch.from_numpy(seeds_h).to(dev)
    pks = be.sign_batch(seeds_h)
    t_ks = time.perf_counter()
    ks = be.keyset(pks)
    ks_build_s = time.perf_counter() - t_ks
    progress("cfg3 committee key cache built (%.1f s)" % ks_build_s)
    ks_bits, ks_bytes = ks.info()
    pks_d = torch.from_numpy(pks).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(777 + rank)
    author = torch.randint(0, nk, (G,), device=dev, generator=g)
    rnd = torch.randint(1, 1 << 20, (G,), device=dev, generator=g, dtype=torch.int64)
    hdr = torch.randint(0, 256, (G, hlen), dtype=torch.uint8, device=dev, generator=g)
    hdr[:, 0:32] = pks_d[author]
    hdr[:, 32:40] = rnd.view(-1, 1).bitwise_right_shift(torch.arange(0, 64, 8, device=dev)).bitwise_and(255).to(torch.uint8)
    wid = 40 + 36 * torch.arange(n_pay, device=dev).view(-1, 1) + 32 + torch.arange(4, device=dev).view(1, -1)
    hdr[:, wid.reshape(-1)] = 0                    # worker id 0
    hdr_flat = hdr.reshape(-1).contiguous()
    h_off = torch.arange(G, dtype=torch.int64, device=dev) * hlen
    h_len = torch.full((G,), hlen, dtype=torch.int64, device=dev)
    ids = torch.empty((G, 32), dtype=torch.uint8, device=dev)
    be.dev_sha512(0, sp, hdr_flat.data_ptr(), nbytes(hdr_flat), h_off.data_ptr(), h_len.data_ptr(), G, ids.data_ptr())
    # header signatures by the author over the id
    i_off = torch.arange(G, dtype=torch.int64, device=dev) * 32
    i_len = torch.full((G,), 32, dtype=torch.int64, device=dev)
    hsig = torch.empty((G, 64), dtype=torch.uint8, device=dev)
    tmp_pk = torch.empty((G, 32), dtype=torch.uint8, device=dev)
    be.dev_sign(0, sp, seeds[author].contiguous().data_ptr(), ids.data_ptr(), nbytes(ids), i_off.data_ptr(), i_len.data_ptr(), G,
                tmp_pk.data_ptr(), hsig.data_ptr())
    # certificate digest preimage: id || round_le || origin
    cpre = torch.cat([ids, hdr[:, 32:40], hdr[:, 0:32]], dim=1).contiguous()
    c_off = torch.arange(G, dtype=torch.int64, device=dev) * 72
    c_len = torch.full((G,), 72, dtype=torch.int64, device=dev)
    cdig = torch.empty((G, 32), dtype=torch.uint8, device=dev)
    be.dev_sha512(0, sp, cpre.data_ptr(), nbytes(cpre), c_off.data_ptr(), c_len.data_ptr(), G, cdig.data_ptr())
    # 67 distinct voters per certificate, signatures over the certificate digest
    voters = torch.rand((G, nk), device=dev, generator=g).argsort(dim=1)[:, :quorum].contiguous()
    V = G * quorum
    vkey = voters.reshape(-1).to(torch.int32).contiguous()
    v_off = (torch.arange(V, device=dev, dtype=torch.int64) // quorum) * 32
    v_len = torch.full((V,), 32, dtype=torch.int64, device=dev)
    vsig = torch.empty((V, 64), dtype=torch.uint8, device=dev)
    vpk = torch.empty((V, 32), dtype=torch.uint8, device=dev)
    be.dev_sign(0, sp, seeds[voters.reshape(-1)].contiguous().data_ptr(), cdig.data_ptr(), nbytes(cdig), v_off.data_ptr(),
                v_len.data_ptr(), V, vpk.data_ptr(), vsig.data_ptr())
    # 1 % of certificates carry one corrupted vote
    rng = np.random.default_rng(99 + rank)
    bad = np.sort(rng.choice(G, size=max(1, G // 100), replace=False)) if G else np.zeros(0, np.int64)
    if len(bad):
        rows = torch.from_numpy(bad * quorum + rng.integers(0, quorum, len(bad))).to(dev)
        vsig[rows, 40] ^= 0x01
    expect = np.ones(G, dtype=bool)
    expect[bad] = False
    torch.cuda.synchronize(dev)

    first = torch.arange(G, dtype=torch.int64, device=dev) * quorum
    cnt = torch.full((G,), quorum, dtype=torch.int32, device=dev)
    hkey = author.to(torch.int32).contiguous()
    # Consecutive steps (independent certificate batches) alternate between two
    # streams, each with its own digest / verdict buffers, for the fused key-cache
    # path (the device API alternates its two stashes, so the launches are
    # independent); NT_BENCH_STREAMS=1: one stream.  The uncached reference runs
    # on one stream.
    nst = 2 if os.environ.get("NT_BENCH_STREAMS", "2") != "1" else 1
    streams = pipeline_streams(torch, be, dev, stream, nst)
    side = side_streams(torch, dev, nst)

    def make_bufs():
        b = {"hd2": torch.empty((G, 32), dtype=torch.uint8, device=dev),
             # one message buffer for the fused key-cache launch: certificate digests, then header ids
             "msgbuf": torch.empty((2 * G, 32), dtype=torch.uint8, device=dev),
             "hbits": torch.zeros(((G + 63) // 64,), dtype=torch.int64, device=dev),
             "vbits": torch.zeros(((V + 63) // 64 + 1,), dtype=torch.int64, device=dev),
             "gbits": torch.zeros(((G + 63) // 64,), dtype=torch.int64, device=dev),
             "mbits": torch.zeros(((V + G + 63) // 64 + 1,), dtype=torch.int64, device=dev)}
        b["msgbuf"][G:] = ids
        b["cd2"] = b["msgbuf"][:G]
        return b
    bufs = [make_bufs() for _ in range(nst)]
    # NT_MODE_MIXED inputs: V vote signatures (cofactorless), then G header signatures
    # (strict: key index with bit 31 set) -- Certificate::verify's two checks in one launch
    mkey = torch.cat([vkey, hkey + torch.iinfo(torch.int32).min]).contiguous()
    msig = torch.cat([vsig, hsig]).contiguous()
    m_off = torch.cat([v_off, G * 32 + i_off]).contiguous()
    m_len = torch.cat([v_len, i_len]).contiguous()

    fused = os.environ.get("NT_BENCH_FUSED", "1") != "0"
    # layout experiment (A/B only): the fused launch sees the votes grouped by
    # committee key, so a wave's comb lookups stay within one key's table
    keysort = fused and os.environ.get("NT_BENCH_KEYSORT") == "1"
    perm = None
    if keysort:
        perm = torch.argsort(vkey, stable=True)
        mkey[:V] = vkey[perm]
        msig[:V] = vsig[perm]
        m_off[:V] = v_off[perm]
        m_len[:V] = v_len[perm]
        perm = perm.cpu().numpy()

    kev = []  # (start, end) events around the key-cache launch of each timed step
    probe = ClockProbe(torch, be, dev)

    mode_streams = {True: nst, False: 1}  # streams of the cached / uncached runs

    def slots(cached):
        return mode_streams[cached] if cached and fused else 1

    def step(cached, i, timed=False):
        k = i % slots(cached)
        st = streams[k]
        sq = st.cuda_stream
        b = bufs[k]
        # certificate digests first (the votes' message); the header-id digests
        # (3.3 KB serial chains, latency-bound) are only needed by the verdict, so
        # they go after the signature launch, where they overlap the other stream
        be.dev_sha512(0, sq, cpre.data_ptr(), nbytes(cpre), c_off.data_ptr(), c_len.data_ptr(), G, b["cd2"].data_ptr(), max_len=72)
        if not (cached and fused):
            be.dev_sha512(0, sq, hdr_flat.data_ptr(), nbytes(hdr_flat), h_off.data_ptr(), h_len.data_ptr(), G, b["hd2"].data_ptr(),
                          max_len=hlen)
        if cached and not fused:   # A/B reference: the header and vote launches separately
            ks.dev_verify(0, sq, ntcrypto.NT_MODE_STRICT, hkey.data_ptr(), hsig.data_ptr(), ids.data_ptr(), nbytes(ids),
                          i_off.data_ptr(), i_len.data_ptr(), G, b["hbits"].data_ptr())
            ks.dev_verify(0, sq, ntcrypto.NT_MODE_COFACTORLESS, vkey.data_ptr(), vsig.data_ptr(), b["cd2"].data_ptr(), nbytes(b["cd2"]),
                          v_off.data_ptr(), v_len.data_ptr(), V, b["vbits"].data_ptr())
            be.dev_group_and(0, sq, first.data_ptr(), cnt.data_ptr(), G, b["vbits"].data_ptr(), b["gbits"].data_ptr())
        elif cached:
            if timed:
                kev.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
                kev[-1][0].record(st)
            if side and slots(cached) > 1:
                # header ids beside the signature launch; the step's last kernel waits for them
                be.dev_sha512(0, side[k].cuda_stream, hdr_flat.data_ptr(), nbytes(hdr_flat), h_off.data_ptr(), h_len.data_ptr(), G,
                              b["hd2"].data_ptr(), max_len=hlen)
                hev = torch.cuda.Event()
                hev.record(side[k])
            # the votes' AND per certificate happens in the key-cache kernel's epilogue
            # (nt_dev_ed25519_verify_keyset_groups): no pack / group-AND launch follows
            ks.dev_verify_groups(0, sq, ntcrypto.NT_MODE_MIXED, mkey.data_ptr(), msig.data_ptr(), b["msgbuf"].data_ptr(),
                                 nbytes(b["msgbuf"]), m_off.data_ptr(), m_len.data_ptr(), V + G, first.data_ptr(),
                                 cnt.data_ptr(), G, b["mbits"].data_ptr(), b["gbits"].data_ptr())
            if timed:
                kev[-1][1].record(st)
            if side and slots(cached) > 1:
                if SIDE_JOIN:
                    st.wait_event(hev)
            else:
                be.dev_sha512(0, sq, hdr_flat.data_ptr(), nbytes(hdr_flat), h_off.data_ptr(), h_len.data_ptr(), G, b["hd2"].data_ptr(),
                              max_len=hlen)
        else:
            be.dev_verify(0, sq, ntcrypto.NT_MODE_STRICT, tmp_pk.data_ptr(), hsig.data_ptr(), ids.data_ptr(), nbytes(ids),
                          i_off.data_ptr(), i_len.data_ptr(), G, b["hbits"].data_ptr())
            be.dev_verify(0, sq, ntcrypto.NT_MODE_COFACTORLESS, vpk.data_ptr(), vsig.data_ptr(), b["cd2"].data_ptr(), nbytes(b["cd2"]),
                          v_off.data_ptr(), v_len.data_ptr(), V, b["vbits"].data_ptr())
            be.dev_group_and(0, sq, first.data_ptr(), cnt.data_ptr(), G, b["vbits"].data_ptr(), b["gbits"].data_ptr())

    def verdicts(cached, k):
        b = bufs[k]
        gb = np.unpackbits(b["gbits"].cpu().numpy().view(np.uint8), bitorder="little")[:G].astype(bool)
        if cached and keysort:   # un-permute the vote bits, AND per certificate on the host
            vb = np.unpackbits(b["mbits"].cpu().numpy().view(np.uint8), bitorder="little")[:V].astype(bool)
            orig = np.empty(V, bool)
            orig[perm] = vb
            gb = orig.reshape(G, quorum).all(axis=1)
        if cached and fused:   # header verdicts follow the V vote bits of the fused launch
            hb = np.unpackbits(b["mbits"].cpu().numpy().view(np.uint8), bitorder="little")[V:V + G].astype(bool)
        else:
            hb = np.unpackbits(b["hbits"].cpu().numpy().view(np.uint8), bitorder="little")[:G].astype(bool)
        idok = (b["hd2"] == ids).all(dim=1).cpu().numpy()
        return gb & hb & idok

    out = {}
    runs = [("keyset", True, nst)] + ([("keyset_one_stream", True, 1)] if nst > 1 and fused else []) + \
        [("uncached", False, 1)]
    for key, cached, ns in runs:
        # up to 20 pipelined key-cache steps (a 2-stream pipeline's fill and drain are
        # one step each); the uncached reference (~70 ms per step) keeps 5
        steps = max(1, min(args.steps, 20 if cached else 5))
        mode_streams[cached] = ns
        kev.clear()
        # the inputs and buffers were written on `stream`: the pipeline streams
        # (library streams on queues of their own) must not start before that work
        barrier()
        for i in range(max(1, args.warmup)):
            step(cached, i)
        clk = [probe.ghz(streams[0])] if key == "keyset" else []
        barrier()
        reg = Region(torch, streams[:slots(cached)] + (side if side and slots(cached) > 1 else []), stream)
        t0 = time.perf_counter()
        reg.start()
        for i in range(steps):
            step(cached, i, timed=True)
        reg.end()
        barrier()
        wall_r = time.perf_counter() - t0
        if clk:
            clk.append(probe.ghz(streams[0]))
        wall = max_over_ranks(wall_r)
        kms = reg.ms() / steps
        if key == "keyset":
            ranks3 = nd.gather_object({"rank": rank, "certificates": G, "signatures": G * (quorum + 1),
                                       "kernel_ms": round(kms, 3), "wall_ms_per_step": round(wall_r * 1e3 / steps, 3),
                                       "rate": round(G * steps / wall_r, 1)})
        bad = sum(int((verdicts(cached, k) != expect).sum()) for k in range(min(slots(cached), steps)))
        mism = int(max_over_ranks(bad))
        out[key] = {"certs_per_s": round(G_total * steps / wall, 1),
                    "sig_verifies_per_s": round(G_total * (quorum + 1) * steps / wall, 1),
                    "ms_per_step": round(wall * 1e3 / steps, 3), "gpu_ms_per_step": round(kms, 3),
                    "streams": slots(cached), "mismatches_vs_expected": mism}
        if key == "keyset" and fused and kev:
            out[key]["roofline"] = keyset_roofline(np.mean([a.elapsed_time(b) for a, b in kev]), kms, V + G, clk)
        if key == "keyset_one_stream" and kev and "keyset" in out and out["keyset"].get("roofline"):
            # launches strictly back to back: each one's own duration (sort + key-cache kernel +
            # byte pack, what rocprof sums per step) without the two-stream overlap
            own = float(np.mean([a.elapsed_time(b) for a, b in kev]))
            rf = out["keyset"]["roofline"]
            ach = rf["mads_per_signature"] * (V + G) / (own * 1e-3) / 1e12
            rf["launch_ms_one_stream"] = round(own, 3)
            rf["frac_one_stream_launch"] = round(ach / MAD_PEAK_TS, 4)
        progress("cfg3 %s: %.2f M certificates/s" % (key, out[key]["certs_per_s"] / 1e6))
    if os.environ.get("NT_BENCH_STREAM_AB") == "1" and fused and world == 1:
        # diagnosis: the same one-stream key-cache steps on each
        # candidate stream, interleaved twice, in one process
        saved = list(streams)
        lib = [torch.cuda.ExternalStream(be.dev_stream(0, k), device=dev) for k in range(2)]
        cands = [("lib0", lib[0]), ("torch_cur", stream)]
        ab = []
        mode_streams[True] = 1
        # variants (profiles/r05/ab_join.txt): "region" = the timed regions above (per-stream end
        # events); "gpujoin" = rounds 1-4's join (`stream` waits for the pipeline stream, a
        # cross-queue wait enqueued on idle `stream` that stays pending for the region);
        # "nokev" = region without the per-launch timing events
        for name, st in cands * 2:
            for var in ("region", "gpujoin", "nokev"):
                streams[0] = st
                barrier()
                for i in range(max(1, args.warmup)):
                    step(True, i)
                barrier()
                kev.clear()
                reg = Region(torch, [st], stream)
                t0 = time.perf_counter()
                reg.start()
                for i in range(20):
                    step(True, i, timed=(var != "nokev"))
                if var == "gpujoin" and st.cuda_stream != stream.cuda_stream:
                    j = torch.cuda.Event()
                    j.record(st)
                    stream.wait_event(j)
                reg.end()
                barrier()
                wall = time.perf_counter() - t0
                ab.append({"stream": name, "variant": var, "certs_per_s": round(G * 20 / wall, 1),
                           "launch_ms": round(float(np.mean([a.elapsed_time(b) for a, b in kev])), 3) if kev else None})
        streams[:] = saved
        mode_streams[True] = nst
        out["stream_ab"] = ab
        progress("cfg3 stream A/B")
    # -------- the same votes through the host entry point (what the crate's FFI binds)
    # nt_ed25519_verify_batch_groups_keyset: Certificate::verify's verify_batch of the
    # 67 votes per certificate (crypto/src/lib.rs:206-219), keys as committee indices,
    # inputs in nt_host_alloc (pinned) memory: PCIe-inclusive, never `value`
    if os.environ.get("NT_BENCH_HOST_CERTS", "1") != "0":
        out["host_api"] = bench_cert_host_api(be, ks, vkey, vsig, cdig, G, quorum, expect, barrier,
                                              max_over_ranks, world, G_total)
        progress("cfg3 host entry point: %.2f M certificates/s" % (out["host_api"]["certs_per_s"] / 1e6))
    if world == 1 and fused and os.environ.get("NT_BENCH_SHARDS", "1") != "0":
        out["shard_of"] = bench_cert_shards(args, torch, dev, ks, be, ntcrypto, streams, side, stream, barrier, G,
                                            quorum,
                                            dict(hdr_flat=hdr_flat, h_off=h_off, h_len=h_len, hlen=hlen, cpre=cpre,
                                                 c_off=c_off,
                                                 c_len=c_len, ids=ids, vkey=vkey, hkey=hkey, vsig=vsig, hsig=hsig,
                                                 v_off=v_off, v_len=v_len, i_off=i_off, i_len=i_len, first=first,
                                                 cnt=cnt),
                                            expect, out["keyset"]["certs_per_s"])
        progress("cfg3 shards")
        if os.environ.get("NT_BENCH_STREAM_AB") == "1":
            # the same shard steps on two torch streams (rounds 1-4's layout), same process
            tst = [stream, torch.cuda.Stream(dev)]
            out["shard_of_torch_streams"] = bench_cert_shards(
                args, torch, dev, ks, be, ntcrypto, tst, side, stream, barrier, G, quorum,
                dict(hdr_flat=hdr_flat, h_off=h_off, h_len=h_len, hlen=hlen, cpre=cpre, c_off=c_off, c_len=c_len,
                     ids=ids, vkey=vkey, hkey=hkey, vsig=vsig, hsig=hsig, v_off=v_off, v_len=v_len, i_off=i_off,
                     i_len=i_len, first=first, cnt=cnt),
                expect, out["keyset"]["certs_per_s"])
            out["shard_of_lib_again"] = bench_cert_shards(
                args, torch, dev, ks, be, ntcrypto, streams, side, stream, barrier, G, quorum,
                dict(hdr_flat=hdr_flat, h_off=h_off, h_len=h_len, hlen=hlen, cpre=cpre, c_off=c_off, c_len=c_len,
                     ids=ids, vkey=vkey, hkey=hkey, vsig=vsig, hsig=hsig, v_off=v_off, v_len=v_len, i_off=i_off,
                     i_len=i_len, first=first, cnt=cnt),
                expect, out["keyset"]["certs_per_s"])
            progress("cfg3 shards A/B")
    ks.close()
    # -------- the drop-in path: the same votes through nt_ed25519_verify_batch_groups
    # (what the unchanged crate's Signature::verify_batch binds) with raw 32-byte keys,
    # the committee keys in the context's key registry (nt_set_key_cache)
    if os.environ.get("NT_BENCH_HOST_CERTS", "1") != "0":
        out["host_api_plain"] = bench_cert_registry(be, pks, vpk, vsig, cdig, G, quorum, expect, barrier,
                                                    max_over_ranks, world, G_total)
        progress("cfg3 plain entry point + key registry: %.2f M certificates/s"
                 % (out["host_api_plain"]["certs_per_s"] / 1e6))
    if world == 1 and not getattr(args, "no_cpu", False):
        out["cpu_baseline"] = cert_cpu_baseline(args, hdr, hlen, ids, tmp_pk, hsig, cpre, vpk, vsig, quorum, expect)
    out["_ranks"] = nd.rank_summary(ranks3)
    return {"value": out["keyset"]["certs_per_s"], "unit": "certificates/s",
            "workload": "cfg3: %d certificates, committee n=%d, %d votes + 1 header signature each, "
                        "%d-byte header preimage" % (G_total, nk, quorum, hlen),
            "scaling": "strong (certificates sharded over ranks)",
            "pipelining": "keyset: consecutive steps re-verify the SAME 100k certificates (resident inputs), "
                          "alternating two streams, each with its own digest / verdict buffers (the device API "
                          "alternates its two key-cache stashes), every buffer's verdicts checked; "
                          "keyset_one_stream: the same launches strictly back to back on one stream",
            "key_cache": {"comb_bits": ks_bits, "gb_per_device": round(ks_bytes / 1e9, 2),
                          "build_s": round(ks_build_s, 3),
                          "note": "per-key wide combs of -A (%d comb additions per [k]A at %d bits%s; [s]B: 11 "
                                  "additions from the device's 24-bit comb of B), built once "
                                  "per committee on every device; not in the timed region"
                                  % ({21: 12, 20: 13, 18: 15, 16: 16}.get(ks_bits, 0), ks_bits,
                                     ", k taken as k or k - L" if ks_bits == 21 else ""),
                          "launches": "per step: SHA-512 of the certificate digests, 1 NT_MODE_MIXED key-cache verify "
                                      "(67 votes cofactorless + the header signature strict) whose kernel also ANDs "
                                      "the votes per certificate (nt_dev_ed25519_verify_keyset_groups: init, key "
                                      "sort, kernel), SHA-512 of the header ids on a side stream (only the verdict "
                                      "needs them)"},
            **out}


def bench_cert_host_api(be, ks, vkey, vsig, cdig, G, quorum, expect, barrier, max_over_ranks, world, G_total,
                        reps=3):
    """Config 3's votes through nt_ed25519_verify_batch_groups_keyset from pinned
    host buffers: G certificates x `quorum` votes, keys as
    committee indices, one 32-byte certificate digest per group.  The library
    DMAs keys and signatures straight from them (nt_host_alloc memory, densely
    packed; only the 32-B digests are memcpy'd into its pinned staging): chunk
    c+1's copies run under chunk c's key-cache launch on the library's two
    compute streams, chunks ramped R/8, R/4, R/2 ... R/2, R/4, R/8
    (pipe_plan.hpp).  Verdicts checked against the expected group results."""
    key_p = be.pinned((G * quorum,), np.uint32)
    sig_p = be.pinned((G * quorum, 64))
    key_p[...] = vkey.cpu().numpy().view(np.uint32)
    sig_p[...] = vsig.cpu().numpy()
    msg32 = cdig.cpu().numpy()
    first = np.arange(G, dtype=np.uint64) * quorum
    cnt = np.full(G, quorum, np.uint32)
    got = ks.verify_batch_groups(key_p, sig_p, first, cnt, msg32)   # warm-up (stash, staging)
    barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        got = ks.verify_batch_groups(key_p, sig_p, first, cnt, msg32)
    barrier()
    wall = max_over_ranks((time.perf_counter() - t0) / reps)
    mism = int(max_over_ranks(int((got != expect).sum())))
    del key_p, sig_p
    return {"certs_per_s": round(G_total / wall, 1), "sig_verifies_per_s": round(G_total * quorum / wall, 1),
            "ms_per_call": round(wall * 1e3, 3), "mismatches_vs_expected": mism,
            "bytes_per_call": int(G * quorum * 68 + G * 44),
            "note": "nt_ed25519_verify_batch_groups_keyset on %d certificates x %d votes per rank from nt_host_alloc "
                    "buffers (4-B key index + 64-B signature per vote over PCIe, no staging copy of them), the library's "
                    "chunk pipeline on its own streams; PCIe-inclusive, never `value`" % (G, quorum)}


def bench_cert_registry(be, pks, vpk, vsig, cdig, G, quorum, expect, barrier, max_over_ranks, world, G_total,
                        reps=3):
    """Config 3's votes through the PLAIN entry point nt_ed25519_verify_batch_groups
    (crypto/src/lib.rs:206-219, what INTEGRATION.md's unchanged verify_batch binds):
    raw 32-byte keys, no key-set handle.  The context's key registry holds the
    100 committee keys (nt_key_cache_add once, timed apart as a one-time cost --
    the same tables a first sighting builds in the background); every call looks
    each key up on host threads as its chunks are staged and sends 4-byte
    indices over PCIe (68 B per vote).  From nt_host_alloc (pinned) buffers and
    from ordinary numpy (pageable) arrays; PCIe-inclusive, never `value`."""
    t0 = time.perf_counter()
    be.set_key_cache(len(pks))   # the committee (config/src/lib.rs:140-143): its n keys
    be.key_cache_add(pks)
    build_s = time.perf_counter() - t0
    info = be.key_cache_info()
    vpk_h = vpk.cpu().numpy()
    vsig_h = vsig.cpu().numpy()
    msg32 = cdig.cpu().numpy()
    first = np.arange(G, dtype=np.uint64) * quorum
    cnt = np.full(G, quorum, np.uint32)
    res = {}
    for kind in ("pinned", "pageable"):
        if kind == "pinned":
            pk_a, sig_a = be.pinned((G * quorum, 32)), be.pinned((G * quorum, 64))
            pk_a[...] = vpk_h
            sig_a[...] = vsig_h
        else:
            pk_a, sig_a = vpk_h, vsig_h
        got = be.verify_batch_groups(pk_a, sig_a, first, cnt, msg32)   # warm-up (staging, stash)
        barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            got = be.verify_batch_groups(pk_a, sig_a, first, cnt, msg32)
        barrier()
        wall = max_over_ranks((time.perf_counter() - t0) / reps)
        res[kind] = {"certs_per_s": round(G_total / wall, 1), "ms_per_call": round(wall * 1e3, 3),
                     "mismatches_vs_expected": int(max_over_ranks(int((got != expect).sum())))}
        del pk_a, sig_a
    after = be.key_cache_info()
    be.set_key_cache(0)
    return {"certs_per_s": res["pinned"]["certs_per_s"], "ms_per_call": res["pinned"]["ms_per_call"],
            "mismatches_vs_expected": res["pinned"]["mismatches_vs_expected"], "pageable": res["pageable"],
            "sig_verifies_per_s": round(G_total * quorum / (res["pinned"]["ms_per_call"] * 1e-3), 1),
            "key_registry": {"keys": info["keys"], "comb_bits": info["comb_bits"],
                             "gb_per_device": round(info["bytes_per_device"] / 1e9, 2), "build_s": round(build_s, 3),
                             "alloc_s": round(info["alloc_us"] / 1e6, 3), "comb_build_s": round(info["build_us"] / 1e6, 3),
                             "alloc_note": "hipMalloc of the registry's tables right after the key set's 161 GB were "
                                           "freed waits for the driver to clear that memory; the combs themselves "
                                           "build in comb_build_s",
                             "lookups_hit": after["hits"], "lookups_missed": after["misses"]},
            "note": "nt_ed25519_verify_batch_groups (the plain entry point the crate's verify_batch binds) on %d "
                    "certificates x %d votes per rank, raw 32-byte keys looked up in the context's key registry on "
                    "host threads while the chunks are staged (4-B index + 64-B signature per vote over PCIe); "
                    "pinned: keys and signatures in nt_host_alloc memory; pageable: ordinary numpy arrays; "
                    "PCIe-inclusive, never `value`" % (G, quorum)}


def bench_cert_shards(args, torch, dev, ks, be, ntcrypto, streams, side, stream, barrier, G,
                                            quorum, t, expect,
                      rate1):
    """Config 3's 2/4/8-GPU shards rehearsed on this GPU (BASELINE configs[2] is
    strong-scaled: each of N GPUs verifies G/N certificates): the first G/N
    certificates through the same fused step (2 digests, one NT_MODE_MIXED
    key-cache launch, group AND; consecutive steps on two streams with their
    own buffers), timed the same way.  `per_gpu_vs_1gpu` = this shard's
    certificates/s on one GPU / the full batch's: what each GPU of an N-GPU run
    keeps of the 1-GPU rate (the key-cache launch plan, ks_stream_plan in
    ks_plan.hpp, sizes the persistent grid to the shard; its waves stream rows).
    `expected_aggregate_certs_per_s` = N x that rate: the strong-scaled N-GPU
    aggregate this GPU's shard rate implies (the 8-GPU run itself is the
    driver's)."""
    res = {}
    # the 1-GPU keyset run's step count: the two-stream pipeline's fill (the first
    # step runs without a neighbour) then weighs the same in both rates
    steps = max(1, min(args.steps, 20))
    nst = len(streams)
    for N in (2, 4, 8):
        Gs = G // N
        Vs = Gs * quorum
        mkey = torch.cat([t["vkey"][:Vs], t["hkey"][:Gs] + torch.iinfo(torch.int32).min]).contiguous()
        msig = torch.cat([t["vsig"][:Vs], t["hsig"][:Gs]]).contiguous()
        m_off = torch.cat([t["v_off"][:Vs], Gs * 32 + t["i_off"][:Gs]]).contiguous()
        m_len = torch.cat([t["v_len"][:Vs], t["i_len"][:Gs]]).contiguous()
        bufs = []
        for _ in range(nst):
            b = {"hd2": torch.empty((Gs, 32), dtype=torch.uint8, device=dev),
                 "msgbuf": torch.empty((2 * Gs, 32), dtype=torch.uint8, device=dev),
                 "gbits": torch.zeros(((Gs + 63) // 64,), dtype=torch.int64, device=dev),
                 "mbits": torch.zeros(((Vs + Gs + 63) // 64 + 1,), dtype=torch.int64, device=dev)}
            b["msgbuf"][Gs:] = t["ids"][:Gs]
            bufs.append(b)
        kev = []
        # mkey / msig / m_off / m_len and the buffers above were built on `stream`;
        # the pipeline streams read them (an unfinished m_off is a wild message
        # offset: the key-cache kernel reads out of bounds)
        barrier()

        def step(i, timed=False):
            st = streams[i % nst]
            sq = st.cuda_stream
            b = bufs[i % nst]
            be.dev_sha512(0, sq, t["cpre"].data_ptr(), nbytes(t["cpre"]), t["c_off"].data_ptr(), t["c_len"].data_ptr(), Gs,
                          b["msgbuf"].data_ptr(), max_len=72)
            if timed:
                kev.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
                kev[-1][0].record(st)
            if side:
                be.dev_sha512(0, side[i % nst].cuda_stream, t["hdr_flat"].data_ptr(), nbytes(t["hdr_flat"]), t["h_off"].data_ptr(),
                              t["h_len"].data_ptr(), Gs, b["hd2"].data_ptr(), max_len=t["hlen"])
                hev = torch.cuda.Event()
                hev.record(side[i % nst])
            ks.dev_verify_groups(0, sq, ntcrypto.NT_MODE_MIXED, mkey.data_ptr(), msig.data_ptr(), b["msgbuf"].data_ptr(),
                                 nbytes(b["msgbuf"]), m_off.data_ptr(), m_len.data_ptr(), Vs + Gs, t["first"].data_ptr(),
                                 t["cnt"].data_ptr(), Gs, b["mbits"].data_ptr(), b["gbits"].data_ptr())
            if timed:
                kev[-1][1].record(st)
            if side:
                if SIDE_JOIN:
                    st.wait_event(hev)
            else:
                be.dev_sha512(0, sq, t["hdr_flat"].data_ptr(), nbytes(t["hdr_flat"]), t["h_off"].data_ptr(), t["h_len"].data_ptr(), Gs,
                              b["hd2"].data_ptr(), max_len=t["hlen"])

        for i in range(max(1, args.warmup)):
            step(i)
        barrier()
        reg = Region(torch, streams + (side or []), stream)
        t0 = time.perf_counter()
        reg.start()
        for i in range(steps):
            step(i, timed=True)
        reg.end()
        barrier()
        wall = time.perf_counter() - t0
        bad = 0
        for k in range(min(nst, steps)):
            b = bufs[k]
            gb = np.unpackbits(b["gbits"].cpu().numpy().view(np.uint8), bitorder="little")[:Gs].astype(bool)
            hb = np.unpackbits(b["mbits"].cpu().numpy().view(np.uint8), bitorder="little")[Vs:Vs + Gs].astype(bool)
            idok = (b["hd2"] == t["ids"][:Gs]).all(dim=1).cpu().numpy()
            bad += int(((gb & hb & idok) != expect[:Gs]).sum())
        rate = Gs * steps / wall
        res[str(N)] = {"certificates": Gs, "signatures_per_launch": Vs + Gs, "steps": steps,
                       "certs_per_s": round(rate, 1),
                       "ms_per_step": round(wall * 1e3 / steps, 3),
                       "gpu_ms_per_step": round(reg.ms() / steps, 3),
                       "keyset_launch_ms": round(float(np.mean([a.elapsed_time(b) for a, b in kev])), 3),
                       "per_gpu_vs_1gpu": round(rate / rate1, 3),
                       "expected_aggregate_certs_per_s": round(N * rate, 1), "mismatches_vs_expected": bad}
    res["note"] = ("one GPU running the first G/N certificates of the same batch, as rank r of an N-GPU run would "
                   "(nd.shard); per_gpu_vs_1gpu >= 0.9 means the N-GPU aggregate stays within 10% of linear")
    return res


def keyset_roofline(launch_ms, step_ms, nsig, clk=None):
    """The config-3 key-cache launch (k_ed25519_verify_keyset, NT_MODE_MIXED) against
    the same v_mad_u64_u32 issue peak as the headline kernel; the instruction
    count, issue share and HBM traffic come from the committed PMC profile.
    With steps alternating between two streams the launches of consecutive
    batches overlap, so a launch's own start-to-end time (launch_ms, what rocprof
    reports per dispatch) exceeds the GPU time per batch; the kernel's rate is
    then taken over the smaller of the two (step_ms includes the step's digest
    and group-AND launches, so it understates the kernel's rate slightly)."""
    kernel_ms = min(launch_ms, step_ms)
    try:
        with open(os.path.join(ROOT, "profiles", "opcount.json")) as f:
            mads = float(json.load(f)["verify_cofactorless_keyset_mads"])
    except Exception:
        return None
    achieved = mads * nsig / (kernel_ms * 1e-3) / 1e12
    kprof = load_profile(PMC_KEYSET_PROFILE) or {}
    pk = kprof.get("kernels", {}).get("verify_keyset", {})
    ratio = probe_ratio(pk, kprof)
    pkl = pk.get("per_launch", {})
    grid = pk.get("grid")
    return {"bound": "valu", "kernel": "k_ed25519_verify_keyset<mixed>", "kernel_ms": round(kernel_ms, 3),
            "launch_ms": round(launch_ms, 3), "gpu_ms_per_step": round(step_ms, 3),
            "signatures_per_launch": nsig, "mads_per_signature": mads,
            "achieved": round(achieved, 3), "peak": round(MAD_PEAK_TS, 2), "unit": "Tmad/s",
            "frac": round(achieved / MAD_PEAK_TS, 4),
            "frac_vs_measured_mad_rate": round(achieved / MAD_MEASURED_TS, 4),
            # the profile's launch is the same 6.9M-signature config-3 launch (NT_BENCH_SHARDS=0 in the PMC pass)
            "valu_instr_per_signature": (round(pkl["SQ_INSTS_VALU"] * 64 / nsig) if "SQ_INSTS_VALU" in pkl else None),
            "effective_clock_ghz": round(pk["effective_clock_ghz"], 3) if "effective_clock_ghz" in pk else None,
            "valu_issue_share": round(pk["valu_issue_share_4cyc"], 3) if "valu_issue_share_4cyc" in pk else None,
            "traffic": pk.get("hbm_bytes_per_launch"),
            "traffic_note": "HBM bytes per launch (profiles/%s, FETCH_SIZE*2 + WRITE_SIZE): 23 random 128-B comb "
                            "lines (2.9 KB: 12 of the 21-bit key comb, 11 of the 24-bit comb of B) + ~250 B of "
                            "inputs + the 160-B stash round trip per signature" % PMC_KEYSET_PROFILE,
            "pmc_source": "traffic, valu_instr_per_signature, valu_issue_share and effective_clock_ghz come from "
                          "profiles/%s (a separate rocprofv3 --pmc run, another box); run_clock is this run's own"
                          % PMC_KEYSET_PROFILE,
            **({"run_clock": {"probe_ghz_before": round(clk[0], 3), "probe_ghz_after": round(clk[1], 3),
                              "probe_ghz": round(sum(clk) / 2, 3),
                              "kernel_over_probe_pmc": round(ratio, 4) if ratio else None,
                              "note": "the probe's clock around this run's key-cache region; kernel_over_probe_pmc = "
                                      "the key-cache launch's GRBM clock / the probe's in one profiled process "
                                      "(profiles/r06/clock_probe_calibration_r06p.txt): this kernel holds a lower "
                                      "clock than the probe while it streams its random comb lines"},
                "frac_at_run_clock": round(achieved / (MAD_PEAK_TS * sum(clk) / 2 / 2.4), 4)}
               if clk else {})}


def bench_latency(be, pk_h, sig_h, msg_h, L):
    """Per-call latency of the host entry points at the reference's call sizes
    (SURVEY H3): Header/Vote::verify = one verify_strict over a 32-byte digest
    (crypto/src/lib.rs:200-204), Certificate::verify's verify_batch = one group
    of 67 votes (:206-219, primary/src/core.rs:349-411), a Processor call = one
    508,052-B digest (worker/src/processor.rs:36-38).  p50 / p99 over repeated
    calls from ordinary host buffers through the Python binding (ctypes: a few
    us of the figure), with the small-call path off (every call on the GPU) and
    in AUTO mode (below the crossover on host threads: csrc/cpu_lane.cpp)."""
    import ntcrypto
    rng = np.random.default_rng(11)
    d = rng.integers(0, 256, 32, dtype=np.uint8)
    seeds = rng.integers(0, 256, (67, 32), dtype=np.uint8)
    pk67, sig67 = be.sign_batch(seeds, np.tile(d, 67), np.arange(67, dtype=np.uint64) * 32, np.full(67, 32, np.uint64))
    one = (pk67[:1], sig67[:1], d, np.zeros(1, np.uint64), np.full(1, 32, np.uint64))
    first, cnt = np.zeros(1, np.uint64), np.full(1, 67, np.uint32)
    big = [rng.integers(0, 256, 508052, dtype=np.uint8).tobytes()]
    cases = {
        "verify_strict_n1": (lambda: be.verify_strict(*one), 200),
        "verify_batch_1x67": (lambda: be.verify_batch_groups(pk67, sig67, first, cnt, d), 100),
        "sha512_one_508052B": (lambda: be.digest_many(big), 30),
        # the same lone calls through the PLAIN entry points with their keys in the
        # context's key registry (nt_set_key_cache): the key-cache kernel's floor
        "verify_strict_n1_key_cache": (lambda: be.verify_strict(*one), 200),
        "verify_batch_1x67_key_cache": (lambda: be.verify_batch_groups(pk67, sig67, first, cnt, d), 100),
    }
    out = {"note": "per-call wall time (us) through the Python binding; gpu = small-call path off, "
                   "auto = NT_SMALL_AUTO (calls below the crossover on host threads); *_key_cache: the same calls "
                   "with the 67 keys in the context's key registry (16-bit key combs: a lone call's floor is the "
                   "launch and one lane's chain, 27 vs 23 comb additions at 21 bits)"}

    def crossover(m, floor):
        T = m["threads"]
        nv = 0
        while nv < 100000:
            t = min(T, nv + 1)
            if -(-(nv + 1) // t) * m["cpu_verify_us"] + (m["spawn_us"] if t > 1 else 0) >= m[floor]:
                break
            nv += 1
        return nv

    def registry(on):
        if on:
            saved = os.environ.get("NT_KEYSET_COMB_BITS")
            os.environ["NT_KEYSET_COMB_BITS"] = "16"
            be.set_key_cache(128)
            be.key_cache_add(pk67)
            if saved is None:
                del os.environ["NT_KEYSET_COMB_BITS"]
            else:
                os.environ["NT_KEYSET_COMB_BITS"] = saved
        else:
            be.set_key_cache(0)

    for mode, name in ((ntcrypto.NT_SMALL_OFF, "gpu"), (ntcrypto.NT_SMALL_AUTO, "auto")):
        be.set_small_call_path(mode, 0)
        if mode == ntcrypto.NT_SMALL_AUTO:
            # the cost model AUTO routes by, calibrated on this context by the call above
            m = be.small_call_model()
            out["small_call_model"] = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in m.items()}
            out["small_call_model"]["verify_crossover_signatures"] = crossover(m, "gpu_verify_us")
            out["small_call_model"]["verify_crossover_signatures_key_cache"] = crossover(m, "gpu_keyset_us")
        for case, (fn, reps) in cases.items():
            cached = case.endswith("_key_cache")
            if cached:
                registry(True)
            h0, g0 = be.call_counts()
            fn()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                fn()
                ts.append((time.perf_counter() - t0) * 1e6)
            h1, g1 = be.call_counts()
            ts.sort()
            out.setdefault(case, {})[name] = {"p50_us": round(ts[len(ts) // 2], 1),
                                              "p99_us": round(ts[min(len(ts) - 1, int(len(ts) * 0.99))], 1),
                                              "reps": reps, "host_calls": h1 - h0, "gpu_calls": g1 - g0}
            if cached:
                ki = be.key_cache_info()
                out[case][name]["key_cache"] = {"keys": ki["keys"], "comb_bits": ki["comb_bits"], "hits": ki["hits"],
                                                "misses": ki["misses"]}
                registry(False)
    # host-lane throughput of one thread (the small-call cost model's constants)
    be.set_small_call_path(ntcrypto.NT_SMALL_ALWAYS, 1)
    n = 64
    offs = np.arange(n, dtype=np.uint64) * L
    t0 = time.perf_counter()
    be.verify_strict(pk_h[:n], sig_h[:n], msg_h[:n * L], offs, np.full(n, L, np.uint64))
    per512 = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    be.verify_strict(np.repeat(pk67[:1], n, 0), np.repeat(sig67[:1], n, 0), d, np.zeros(n, np.uint64),
                     np.full(n, 32, np.uint64))
    per32 = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    be.digest_many(big)
    sha_s = time.perf_counter() - t0
    be.set_small_call_path(ntcrypto.NT_SMALL_OFF, 0)
    out["host_lane_1thread"] = {"verify_us_msg32": round(per32 * 1e6, 1), "verify_us_msg512": round(per512 * 1e6, 1),
                                "sha512_mb_per_s": round(508052 / sha_s / 1e6, 1)}
    return out


def bench_batcher(per_stream=64, size=508052):
    """worker::DigestBatcher: the worker's two Processor streams
    (own batches / others' batches, worker/src/worker.rs:182-188, 227-233) each
    push `per_stream` real-size batches from their own thread, keeping them in
    flight and awaiting the results in order; the batcher hashes what is queued
    in one nt_sha512_trunc32 call per flush (1 ms age / 64 MB / 4096 batches).
    Per-batch latency = submit -> digest.  GPU vs the small-call path (AUTO)."""
    import hashlib
    import threading
    from ntcrypto import narwhal as N
    rng = np.random.default_rng(21)
    jobs = {own: [rng.integers(0, 256, size, dtype=np.uint8).tobytes() for _ in range(per_stream)]
            for own in (True, False)}
    out = {"workload": "2 Processor streams x %d batches of %d B, pipelined" % (per_stream, size)}
    for mode, name in ((0, "gpu"), (1, "auto")):
        N.set_small_call_path(mode, 0)
        b = N.DigestBatcher(max_bytes=64 << 20, max_batches=4096, max_delay_us=1000)
        lat, res = {True: [], False: []}, {}

        def stream(own):
            t_sub, tickets = [], []
            for x in jobs[own]:
                t_sub.append(time.perf_counter())
                tickets.append(b.submit(0, own, x))
            got = []
            for t0, t in zip(t_sub, tickets):
                got.append(b.wait(t)[0])
                lat[own].append(time.perf_counter() - t0)
            res[own] = got

        b.process(0, True, jobs[True][0])  # warm-up (contexts, pinned arenas)
        st0 = b.stats()
        t0 = time.perf_counter()
        th = [threading.Thread(target=stream, args=(own,)) for own in (True, False)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
        st = b.stats()
        b.close()
        ok = all(d == hashlib.sha512(x).digest()[:32] for own in (True, False) for x, d in zip(jobs[own], res[own]))
        ls = sorted(lat[True] + lat[False])
        nb = 2 * per_stream
        out[name] = {"batches_per_s": round(nb / wall, 1), "gb_per_s": round(nb * size / wall / 1e9, 3),
                     "latency_p50_ms": round(ls[len(ls) // 2] * 1e3, 3),
                     "latency_p99_ms": round(ls[min(len(ls) - 1, int(len(ls) * 0.99))] * 1e3, 3),
                     "flushes": st["flushes"] - st0["flushes"], "digests_match_hashlib": bool(ok)}
    N.set_small_call_path(0)
    return out


def bench_contention(ntcrypto, device, reps=40):
    """Device-lock contention (one context shared by a worker and a primary,
    SURVEY §3.5): a Core-shaped call -- verify_batch of a drained batch of 100
    certificates x 67 votes -- timed alone and while another thread keeps the
    same context busy with Processor-shaped digest flushes (64 x 508,052 B on
    the GPU).  NT_SLOTS=1: one execution slot per device (the call waits for the
    flush to finish); default NT_SLOTS=2: a second slot runs it concurrently."""
    import threading
    rng = np.random.default_rng(31)
    G, q = 100, 67
    seeds = rng.integers(0, 256, (q, 32), dtype=np.uint8)
    dig = rng.integers(0, 256, (G, 32), dtype=np.uint8)
    big = rng.integers(0, 256, 64 * 508052, dtype=np.uint8)
    boff = np.arange(64, dtype=np.uint64) * 508052
    blen = np.full(64, 508052, np.uint64)
    out = {"call": "verify_batch_groups: %d certificates x %d votes (GPU path)" % (G, q),
           "background": "nt_sha512_trunc32 of 64 x 508,052 B in a loop (GPU path)"}
    saved = os.environ.get("NT_SLOTS")
    for slots in (1, 2):
        os.environ["NT_SLOTS"] = str(slots)
        be = ntcrypto.Backend(device=device)
        try:
            msgs = np.repeat(dig, q, axis=0).reshape(-1)
            pk, sig = be.sign_batch(np.tile(seeds, (G, 1)), msgs, np.arange(G * q, dtype=np.uint64) * 32,
                                    np.full(G * q, 32, np.uint64))
            first = np.arange(G, dtype=np.uint64) * q
            cnt = np.full(G, q, np.uint32)

            def call():
                t0 = time.perf_counter()
                ok = be.verify_batch_groups(pk, sig, first, cnt, dig.reshape(-1))
                assert ok.all()
                return (time.perf_counter() - t0) * 1e3

            call()
            alone = sorted(call() for _ in range(reps))
            stop = threading.Event()

            def background():
                while not stop.is_set():
                    be.sha512_trunc32(big, boff, blen)

            th = threading.Thread(target=background)
            th.start()
            time.sleep(0.05)
            busy = sorted(call() for _ in range(reps))
            stop.set()
            th.join()
        finally:
            be.close()
        out["slots_%d" % slots] = {"alone_p50_ms": round(alone[reps // 2], 3), "alone_p99_ms": round(alone[-1], 3),
                                   "with_digests_p50_ms": round(busy[reps // 2], 3),
                                   "with_digests_p99_ms": round(busy[-1], 3)}
    if saved is None:
        os.environ.pop("NT_SLOTS", None)
    else:
        os.environ["NT_SLOTS"] = saved
    return out


def cert_cpu_baseline(args, hdr, hlen, ids, hpk, hsig, cpre, vpk, vsig, quorum, expect):
    """Config 3 on the host cores: Certificate::verify (primary/src/messages.rs:189-215)
    per certificate = SHA-512 of the header preimage (id check), verify_strict of
    the header signature, SHA-512 of the certificate digest preimage and dalek's
    verify_batch of the votes -- computed as dalek computes it (random z_i, one
    Straus multiscalar multiplication; oracle ntor_certificates_verify_many) --
    on a bounded sample of the same certificates, verdicts compared."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle
    orc = _oracle.load()
    th = cpu_threads(args)
    G = hdr.shape[0]

    def run(k, threads):
        h = hdr[:k].cpu().numpy()
        first = np.arange(k, dtype=np.uint64) * quorum
        t0 = time.perf_counter()
        r = orc.certificates_verify_many(h.reshape(-1), np.arange(k, dtype=np.uint64) * hlen,
                                         np.full(k, hlen, np.uint64), ids[:k].cpu().numpy(), hpk[:k].cpu().numpy(),
                                         hsig[:k].cpu().numpy(), cpre[:k].cpu().numpy(),
                                         vpk[:k * quorum].cpu().numpy(), vsig[:k * quorum].cpu().numpy(), first,
                                         np.full(k, quorum, np.uint32), nthreads=threads)
        return r, time.perf_counter() - t0

    _, one = run(4, 1)
    per = one / 4
    sample = int(min(G, max(th * 8, args.cpu_seconds / per)))
    dt, (res, _) = timed_median(lambda: run(sample, th))
    agree = int((res.astype(bool) == expect[:sample]).sum())
    host = host_cpu()
    return {"value": round(sample / dt, 1), "unit": "certificates/s", "cores": th, "kind": "port",
            "label": "dalek-equivalent CPU restatement: Certificate::verify's 2 SHA-512 digests, verify_strict of "
                     "the header and dalek's randomized verify_batch of the %d votes (Straus / NAF-5 multiscalar)"
                     % quorum,
            "sample": "first %d of the same cfg3 certificates, 1 warm-up + median of 5 runs (%.2f s wall each on %d threads)"
                      % (sample, dt, th),
            "single_thread_ms_per_certificate": round(per * 1e3, 3),
            "host": host, "full_host_estimate": full_host(sample / dt, th, host),
            "verdicts_agree_with_expected": "%d/%d" % (agree, sample)}


def bench_ingest(args, be, world, rank, local, max_over_ranks, barrier):
    """SURVEY §8(f).1 + (f).2: config 3's certificates as the primary receives
    them -- bincode PrimaryMessage::Certificate bytes (primary/src/primary.rs:230)
    -- through the C++ mirror's batched primary::Core::ingest: host decode
    straight into SoA buffers (16 threads), the Core's checks in the reference
    order, one SHA-512 + one verify_strict + one verify_batch launch against the
    committee key cache.  PCIe-inclusive host entry points: this is the
    wire-to-verdict rate, not the resident-data kernel rate of `certificates`."""
    import hashlib
    import struct
    from ntcrypto import dist as nd
    from ntcrypto import narwhal as N

    os.environ["NT_DEVICE"] = str(local)
    nk = args.committee
    quorum = 2 * nk // 3 + 1
    glo, ghi = nd.shard(args.certs, world, rank)
    G = ghi - glo
    n_pay, n_par = 32, quorum
    seeds = np.stack([np.frombuffer(hashlib.sha512(b"nt-bench-key" + struct.pack("<Q", i)).digest()[:32], np.uint8)
                      for i in range(nk)])
    pks = be.sign_batch(seeds)
    b64 = np.frombuffer(b"".join(__import__("base64").b64encode(p.tobytes()) for p in pks), np.uint8).reshape(nk, 44)
    rng = np.random.default_rng(4242 + rank)
    author = rng.integers(0, nk, G)
    rnd = rng.integers(1, 1 << 40, G, dtype=np.uint64)

    def sorted_digests(k):
        d = rng.integers(0, 256, (G, k, 32), dtype=np.uint8)
        key = d[:, :, :8].copy().view(">u8")[:, :, 0]     # BTreeMap/BTreeSet order (8-byte prefix)
        return np.take_along_axis(d, np.argsort(key, axis=1)[:, :, None], axis=1)

    pay = np.zeros((G, n_pay, 36), np.uint8)
    pay[:, :, :32] = sorted_digests(n_pay)               # worker id 0
    par = sorted_digests(n_par)
    rbytes = rnd.view(np.uint8).reshape(G, 8)
    pre = np.concatenate([pks[author], rbytes, pay.reshape(G, -1), par.reshape(G, -1)], axis=1)
    plen = pre.shape[1]
    ids = be.sha512_trunc32(pre.reshape(-1), np.arange(G, dtype=np.uint64) * plen, np.full(G, plen, np.uint64))
    _, hsig = be.sign_batch(seeds[author], ids.reshape(-1), np.arange(G, dtype=np.uint64) * 32,
                            np.full(G, 32, np.uint64))
    cpre = np.concatenate([ids, rbytes, pks[author]], axis=1)
    cdig = be.sha512_trunc32(cpre.reshape(-1), np.arange(G, dtype=np.uint64) * 72, np.full(G, 72, np.uint64))
    voters = np.argsort(rng.random((G, nk)), axis=1)[:, :quorum]
    V = G * quorum
    _, vsig = be.sign_batch(seeds[voters.reshape(-1)], cdig.reshape(-1),
                            np.repeat(np.arange(G, dtype=np.uint64) * 32, quorum), np.full(V, 32, np.uint64))
    vsig = vsig.reshape(G, quorum, 64)
    bad = np.sort(rng.choice(G, size=max(1, G // 100), replace=False))
    vsig[bad, rng.integers(0, quorum, len(bad)), 40] ^= 1

    def u64(x):
        return np.full((G, 8), 0, np.uint8) + np.frombuffer(struct.pack("<Q", x), np.uint8)

    votes = np.concatenate([np.broadcast_to(u64(44)[:, None, :], (G, quorum, 8)), b64[voters], vsig], axis=2)
    wire = np.concatenate([np.broadcast_to(np.array([2, 0, 0, 0], np.uint8), (G, 4)), u64(44), b64[author], rbytes,
                           u64(n_pay), pay.reshape(G, -1), u64(n_par), par.reshape(G, -1), ids, hsig, u64(quorum),
                           votes.reshape(G, -1)], axis=1)
    wlen = wire.shape[1]
    data = np.ascontiguousarray(wire).reshape(-1)
    off = np.arange(G, dtype=np.uint64) * wlen
    ln = np.full(G, wlen, np.uint64)
    expect = np.zeros(G, np.int32)
    expect[bad] = 1                                        # InvalidSignature
    core = N.Core(pks, np.ones(nk, np.uint32), np.ones(nk, np.uint32), 0, None, True)
    try:
        core.ingest(data, off, ln, args.ingest_threads)    # warm-up (key cache, allocations)
        steps = 3
        barrier()
        t0 = time.perf_counter()
        dec = 0.0
        for _ in range(steps):
            got, d = core.ingest(data, off, ln, args.ingest_threads)
            dec += d
        wall1 = max_over_ranks(time.perf_counter() - t0)
        phases = {k: round(v * 1e3, 2) for k, v in N.Core.last_stats().items()}
        # two chunks in flight: host decode/checks of one overlap the other's launches
        # 2 chunks (one per pipeline) measured best: 4 / 8 chunks pay the per-call
        # overheads more often (profiles/r02/ab_ingest/)
        nch = int(os.environ.get("NT_BENCH_INGEST_CHUNKS", "2"))
        chunk = max(1, (G + nch - 1) // nch)
        core.ingest_pipelined(data, off, ln, args.ingest_threads, chunk)
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            gotp = core.ingest_pipelined(data, off, ln, args.ingest_threads, chunk)
        wall = max_over_ranks(time.perf_counter() - t0)
        got = np.where(got == gotp, got, -1)
        # certificates parsed and checked on the GPU from the wire bytes
        # (Core::ingest_device -> nt_certificates_ingest): the bytes as received,
        # in pinned memory (a receiver that owns its buffers), DMA'd per chunk
        pdata = be.pinned(data.shape)
        pdata[...] = data
        core.ingest(pdata, off, ln, args.ingest_threads, device=True)   # warm-up (committee tables, buffers)
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            gotd, host_n = core.ingest(pdata, off, ln, args.ingest_threads, device=True)
        walld = max_over_ranks(time.perf_counter() - t0)
        gotdp, _ = core.ingest(data, off, ln, args.ingest_threads, device=True)  # pageable input, once
        del pdata
    finally:
        core.close()
    mism = int(max_over_ranks(int((got != expect).sum())))
    mismd = int(max_over_ranks(int((gotd != expect).sum()) + int((gotdp != expect).sum())))
    device = {"certs_per_s": round(args.certs * steps / walld, 1), "ms_per_step": round(walld * 1e3 / steps, 3),
              "host_decided": int(host_n), "mismatches_vs_expected": mismd,
              "note": "Core::ingest_device: wire bytes copied as-is (pinned), parsed / checked on the GPU "
                      "(k_cert_parse, k_cert_scatter, one SHA-512 + one NT_MODE_MIXED key-cache launch + group AND "
                      "per chunk of %s messages, chunks alternating two streams so the PCIe copy of one runs under "
                      "the previous one's kernels); PCIe-inclusive" % os.environ.get("NT_INGEST_CHUNK", "6250")}
    return {"value": device["certs_per_s"], "unit": "certificates/s",
            "path": "device parse (Core::ingest_device); host_decode = the host decoder path",
            "device_parse": device,
            "host_decode": {"certs_per_s": round(args.certs * steps / wall, 1)},
            "workload": "cfg3 as wire bytes: %d bincode PrimaryMessage::Certificate messages of %d B (n=%d "
                        "committee, %d votes), Core::ingest -> DagError per message" % (args.certs, wlen, nk, quorum),
            "ms_per_step": round(wall * 1e3 / steps, 3), "pipeline_chunk": chunk,
            "single_call": {"certs_per_s": round(args.certs * steps / wall1, 1),
                            "ms_per_step": round(wall1 * 1e3 / steps, 3)},
            "host_decode_ms": round(dec * 1e3 / steps, 3),
            "decode_threads": args.ingest_threads, "wire_bytes_per_step": int(G * wlen),
            "phase_ms_last_step": phases,
            "note": "host decode into SoA + reference-order checks + 1 SHA-512, 1 verify_strict, 1 verify_batch "
                    "launch (key cache) per chunk, %d chunks on 2 pipelines; PCIe-inclusive" % nch,
            "mismatches_vs_expected": mism}


def cpu_baseline(args, pk_h, sig_h, msg_h, L, got):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle
    orc = _oracle.load()
    th = cpu_threads(args)
    # calibrate: per-verify cost on one thread
    k = 256
    offs = (np.arange(k, dtype=np.uint64) * L)
    lens = np.full(k, L, np.uint64)
    t0 = time.perf_counter()
    orc.verify_strict_many(pk_h[:k], sig_h[:k], msg_h[:k * L], offs, lens, nthreads=1)
    per = (time.perf_counter() - t0) / k
    sample = int(min(len(pk_h), max(th * 64, args.cpu_seconds / per)))
    offs = (np.arange(sample, dtype=np.uint64) * L)
    lens = np.full(sample, L, np.uint64)
    # 1 warm-up + median of 5 timed runs (SURVEY §8(d) procedure)
    dt, res = timed_median(lambda: orc.verify_strict_many(pk_h[:sample], sig_h[:sample], msg_h[:sample * L], offs,
                                                          lens, nthreads=th))
    agree = int((res.astype(bool) == got[:sample]).sum())
    host = host_cpu()
    out = {"value": round(sample / dt, 1), "unit": "verifies/s", "cores": th, "kind": "port",
           "label": "dalek-equivalent CPU restatement (oracle/: curve25519-dalek u64-backend field arithmetic -- radix 2^51, dedicated square, lazy add -- and dalek's verify algorithms)",
           "sample": "first %d of the same 1M cfg2 verifies, 1 warm-up + median of 5 runs (%.1f s wall each on %d threads)"
                     % (sample, dt, th),
           "host": host, "full_host_estimate": full_host(sample / dt, th, host),
           "single_thread_us_per_verify": round(per * 1e6, 2),
           "verdicts_agree_with_gpu": "%d/%d" % (agree, sample)}
    progress("cfg2 CPU baseline")
    ext = sodium_baseline(orc, pk_h, sig_h, msg_h, L, got, th, args.cpu_seconds)
    if ext:
        out["external"] = ext
    return out


def sodium_baseline(orc, pk_h, sig_h, msg_h, L, got, th, seconds):
    """libsodium 1.0.18 crypto_sign_verify_detached (optimised C, ref10 arithmetic) on
    the same inputs and th threads (oracle/sodium_batch.c: a pthread loop, library
    dlopen'ed): an external comparator for the CPU baseline -- its verdicts coincide
    with verify_strict on this corpus, which is checked here too."""
    if not os.path.exists(SODIUM):
        return None
    k = 256
    offs = np.arange(k, dtype=np.uint64) * L
    lens = np.full(k, L, np.uint64)
    t0 = time.perf_counter()
    if orc.sodium_verify_many(SODIUM, pk_h[:k], sig_h[:k], msg_h[:k * L], offs, lens, 1) is None:
        return None
    per = (time.perf_counter() - t0) / k
    sample = int(min(len(pk_h), max(th * 64, seconds / per)))
    offs = np.arange(sample, dtype=np.uint64) * L
    lens = np.full(sample, L, np.uint64)
    dt, res = timed_median(lambda: orc.sodium_verify_many(SODIUM, pk_h[:sample], sig_h[:sample], msg_h[:sample * L],
                                                          offs, lens, th))
    agree = int((res.astype(bool) == got[:sample]).sum())
    return {"name": "libsodium 1.0.18 crypto_sign_verify_detached", "value": round(sample / dt, 1),
            "unit": "verifies/s", "cores": th, "kind": "external",
            "sample": "first %d of the same cfg2 verifies, 1 warm-up + median of 5 runs (%.1f s wall each)"
                      % (sample, dt),
            "single_thread_us_per_verify": round(per * 1e6, 2), "verdicts_agree_with_gpu": "%d/%d" % (agree, sample)}


def timed_median(fn, runs=5, warmup=1):
    """SURVEY §8(d) procedure: `warmup` untimed calls, then the median wall time
    of `runs` timed calls; returns (median seconds, result of the last call)."""
    res = None
    for _ in range(warmup):
        res = fn()
    times = []
    for _ in range(runs):
        t0 = time.perf_counter()
        res = fn()
        times.append(time.perf_counter() - t0)
    return sorted(times)[len(times) // 2], res


def expand(label: bytes, n: int) -> bytes:
    """Deterministic synthetic bytes (SHA-512 counter mode), the generator of
    tests/golden/make_golden.py's real-batch fixture."""
    import hashlib
    import struct
    out = bytearray()
    i = 0
    while len(out) < n:
        out += hashlib.sha512(label + struct.pack("<Q", i)).digest()
        i += 1
    return bytes(out[:n])


def mads_per_verify(msg_len):
    path = os.path.join(ROOT, "profiles", "opcount.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return int(d["verify_strict_mads"])
    except Exception:
        return None


def probe_ratio(kernel_entry, prof):
    """A kernel's GRBM clock / the clock probe's GRBM clock in one PMC profile
    (the same process), or None"""
    try:
        return kernel_entry["effective_clock_ghz"] / prof["kernels"]["clock_probe"]["effective_clock_ghz"]
    except (KeyError, TypeError, ZeroDivisionError):
        return None


def load_profile(name):
    try:
        with open(os.path.join(ROOT, "profiles", name)) as f:
            return json.load(f)
    except Exception:
        return None


if __name__ == "__main__":
    main()
