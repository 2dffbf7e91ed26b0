"""Device -> pinned host copy rates on the box (host tool, no product code): torch's copy_ on its
stream, hipMemcpy on the null stream, hipMemcpyAsync on a non-blocking stream — the paths the
multi-GPU driver's text fetch can take.  Usage: python tools/d2h_probe.py [GB]"""
import ctypes
import sys
import time

import torch

n = int(float(sys.argv[1] if len(sys.argv) > 1 else 1.0) * (1 << 30))
d = torch.empty(n, dtype=torch.uint8, device="cuda:0")
d.fill_(7)
h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
hip = ctypes.CDLL("libamdhip64.so")
st = ctypes.c_void_p()
assert hip.hipStreamCreateWithFlags(ctypes.byref(st), 1) == 0
torch.cuda.synchronize()


def rate(name, fn, reps=5):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    dt = (time.perf_counter() - t) / reps
    print(f"{name:40s} {n / dt / 1e9:6.1f} GB/s ({dt * 1e3:.1f} ms per {n >> 20} MB)", flush=True)


def torch_copy():
    h.copy_(d)


def hip_sync():
    assert hip.hipMemcpy(ctypes.c_void_p(h.data_ptr()), ctypes.c_void_p(d.data_ptr()), ctypes.c_size_t(n), 2) == 0


def hip_async():
    assert hip.hipMemcpyAsync(ctypes.c_void_p(h.data_ptr()), ctypes.c_void_p(d.data_ptr()), ctypes.c_size_t(n), 2,
                              st) == 0
    assert hip.hipStreamSynchronize(st) == 0


rate("torch copy_ (device -> pinned)", torch_copy)
rate("hipMemcpy (null stream)", hip_sync)
rate("hipMemcpyAsync (non-blocking stream)", hip_async)
hp = torch.empty(n, dtype=torch.uint8)
hp.fill_(1)
rate("torch copy_ (device -> pageable, faulted)", lambda: hp.copy_(d))
