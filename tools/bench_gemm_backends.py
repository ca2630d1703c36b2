"""The c3 acting forward's hipBLASLt GEMMs (F.linear fp16: QKV 557,056 x 512 -> 1,536, KV -> 1,024,
conv3 32,768 x 2,304 -> 500, the 512 x 512 layers at 32,768 rows) timed under torch's BLAS choices:
hipBLASLt default heuristic, rocBLAS (preferred_blas_library), and TunableOp (every candidate
solution benchmarked on first use).  One JSON line per (mode, shape)."""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

SHAPES = [("qkv", 557056, 512, 1536), ("kv", 557056, 512, 1024), ("conv3", 32768, 2304, 500),
          ("fc512", 32768, 512, 512)]


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="default", choices=["default", "rocblas", "tunable"])
    a = ap.parse_args()
    if a.mode == "rocblas":
        torch.backends.cuda.preferred_blas_library("cublas")
    if a.mode == "tunable":
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        torch.cuda.tunable.set_filename(os.path.join(os.environ.get("TUNE_DIR", "/tmp"), "tunableop_results.csv"))
        torch.cuda.tunable.set_max_tuning_duration(200)
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, M, K, N in SHAPES:
        x = torch.randn(M, K, device="cuda", generator=g).half()
        w = torch.randn(N, K, device="cuda", generator=g).half() / K ** 0.5
        b = torch.randn(N, device="cuda", generator=g).half()
        t0 = time.time()
        us = timeit(lambda: F.linear(x, w, b))
        print(json.dumps({"mode": a.mode, "shape": name, "M": M, "K": K, "N": N, "us": round(us, 1),
                          "pflops": round(2 * M * K * N / us / 1e9, 3), "wall_s": round(time.time() - t0, 1)}),
              flush=True)
    if a.mode == "tunable":
        torch.cuda.tunable.write_file()


if __name__ == "__main__":
    sys.exit(main())
