"""Subprocess helper of test_gpu_parity.test_keyset_per_lane_counts (not a test
module): the corpus through the key cache in mixed mode with the per-lane
row cap and waves per SIMD the parent chose (NT_KEYSET_PER_LANE,
NT_KEYSET_WAVES, read once per process by libntcrypto), as the plain corpus
(input order), tiled to 72k signatures (key-grouped order, one row per
chunk) and to ~1M signatures (multi-row chunks, several rounds at small
caps).  Prints one JSON line: mismatches per launch."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "narwhal-tusk_amd"))
import ntcrypto  # noqa: E402

d = np.load(os.path.join(ROOT, "tests", "golden", "ed25519_corpus.npz"))
be = ntcrypto.Backend(0)
uniq, inv = np.unique(d["pk"], axis=0, return_inverse=True)
inv = inv.ravel().astype(np.uint32)
ks = be.keyset(uniq)
out = {"per_lane": os.environ.get("NT_KEYSET_PER_LANE"), "waves": os.environ.get("NT_KEYSET_WAVES")}
for reps in (1, 200, 2800):
    n0 = len(inv)
    idx = np.tile(inv, reps)
    unknown = (np.arange(n0 * reps) % 97) == 5
    idx[unknown] = len(uniq) + 3
    strict = (np.arange(n0 * reps) % 3) == 1
    midx = (idx | np.where(strict, np.uint32(ntcrypto.NT_KEY_STRICT_BIT), np.uint32(0))).astype(np.uint32)
    got = ks.verify(ntcrypto.NT_MODE_MIXED, midx, np.tile(d["sig"], (reps, 1)), d["msg"], np.tile(d["off"], reps),
                    np.tile(d["len"], reps))
    want = np.where(strict, np.tile(d["strict"], reps), np.tile(d["batch_rule"], reps)).astype(bool) & ~unknown
    out["mismatches_%d" % (n0 * reps)] = int((got != want).sum())
ks.close()
be.close()
print(json.dumps(out))
