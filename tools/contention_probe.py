"""Device-slot contention probe (bench.py bench_contention alone): run with
different HIP queue settings to see whether two execution slots of one device
actually run concurrently on the GPU.

    python tools/contention_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "narwhal-tusk_amd"))


def main():
    import bench
    import ntcrypto
    import torch
    # the bench's surroundings: a torch stream and a main context are alive
    st = torch.cuda.Stream(torch.device("cuda", 0))
    main_be = ntcrypto.Backend(device=0)
    res = bench.bench_contention(ntcrypto, 0, reps=20)
    main_be.close()
    del st
    res["GPU_MAX_HW_QUEUES"] = os.environ.get("GPU_MAX_HW_QUEUES")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
