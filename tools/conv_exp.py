"""Times mapf_conv3x3_c128_9x9 (B = 32768 images, no pool) from one or more builds of
libmapf (diagnostic variants built by tools/conv_variants.sh), HIP events on the launch
stream.   python tools/conv_exp.py lib/libmapf.so lib/libmapf_cnomfma.so ..."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    B = 32768
    x = torch.randn(B, 128, 9, 9, device="cuda").half().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(9, 128, 128, device="cuda") / 24).half()
    b = torch.randn(128, device="cuda").half()
    out = torch.empty(B, 128, 9, 9, device="cuda", dtype=torch.float16).contiguous(memory_format=torch.channels_last)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    st = torch.cuda.current_stream()
    for path in sys.argv[1:]:
        lib = ctypes.CDLL(os.path.join(ROOT, "primal-ppo_amd", path))
        f = lib.mapf_conv3x3_c128_9x9
        f.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p]
        for _ in range(3):
            assert f(p(x), p(w), p(b), p(out), B, 0, ctypes.c_void_p(st.cuda_stream)) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            f(p(x), p(w), p(b), p(out), B, 0, ctypes.c_void_p(st.cuda_stream))
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"{path}: {ms * 1e3:.0f} us  ({2 * B * 81 * 128 * 1152 / ms / 1e9:.0f} TFLOP/s)", flush=True)


if __name__ == "__main__":
    main()
