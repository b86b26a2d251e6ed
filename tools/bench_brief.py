#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (the last line of a log)."""
import json
import sys


def g(d, *path, default=None):
    for p in path:
        if not isinstance(d, dict) or p not in d:
            return default
        d = d[p]
    return d


def main(path):
    line = [x for x in open(path).read().splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    r = d["roofline"]
    c = d.get("certificates", {})
    print("cfg2 %.2f M/s (one stream %.2f)  kernel %.3f ms  frac %.4f  run clock %s GHz  frac@clock %s  cycles r05/now %s"
          % (d["value"] / 1e6, g(d, "one_stream", "value", default=0) / 1e6, r["kernel_ms"], r["frac"],
             g(r, "run_clock", "probe_ghz"), r.get("frac_at_run_clock"), g(r, "vs_r05", "cycle_ratio_r05_over_now")))
    print("host_api cfg2 pinned %.2f M/s, pageable %.2f M/s" % (g(d, "host_api", "pinned", "verify_strict_per_s", default=0) / 1e6,
                                                          g(d, "host_api", "verify_strict_per_s", default=0) / 1e6))
    if c:
        kr = g(c, "keyset", "roofline", default={})
        print("cfg3 %.3f M certs/s (one stream %.3f)  launch %.3f ms  frac %s  run clock %s  mism %s"
              % (c["value"] / 1e6, g(c, "keyset_one_stream", "certs_per_s", default=0) / 1e6, kr.get("launch_ms", 0),
                 kr.get("frac"), g(kr, "run_clock", "probe_ghz"), g(c, "keyset", "mismatches_vs_expected")))
        so = c.get("shard_of", {})
        print("shards " + " / ".join("%s" % g(so, k, "per_gpu_vs_1gpu") for k in ("2", "4", "8")))
        print("cfg3 host keyset %.3f M/s; plain+registry pinned %s pageable %s (mism %s, registry %s)"
              % (g(c, "host_api", "certs_per_s", default=0) / 1e6, g(c, "host_api_plain", "certs_per_s"),
                 g(c, "host_api_plain", "pageable", "certs_per_s"), g(c, "host_api_plain", "mismatches_vs_expected"),
                 g(c, "host_api_plain", "key_registry")))
    if "sha512" in d:
        print("cfg4 %.1f GB/s" % d["sha512"]["value"])
    lat = d.get("latency", {})
    for k in ("verify_strict_n1", "verify_batch_1x67", "verify_strict_n1_key_cache", "verify_batch_1x67_key_cache"):
        if k in lat:
            print("lat %-28s gpu p50 %s p99 %s | auto p50 %s" % (k, g(lat, k, "gpu", "p50_us"), g(lat, k, "gpu", "p99_us"),
                                                              g(lat, k, "auto", "p50_us")))
    if "small_call_model" in lat:
        print("model", lat["small_call_model"])
    if "ingest" in d:
        print("ingest", {k: v for k, v in d["ingest"].items() if not isinstance(v, (dict, list))})


if __name__ == "__main__":
    import signal
    signal.signal(signal.SIGPIPE, signal.SIG_DFL)  # `| head` ends the summary quietly
    main(sys.argv[1])
