#!/usr/bin/env python3
"""Host-side cost of the copies the host-inclusive bench loop makes (diagnostic): torch copy_ of
page-locked host frames to the device (non_blocking), device-to-device copies, and the same H2D
through hipMemcpyAsync directly; per call, after warm-up, with the GPU otherwise idle."""
import ctypes as C
import time

import torch

S, H, W = 8, 512, 640
dev = torch.device("cuda", 0)
host = torch.empty((4, S, H, W, 3), dtype=torch.uint8, pin_memory=True)
host.random_(0, 255)
d0 = torch.empty((S, H, W, 3), dtype=torch.uint8, device=dev)
d1 = torch.empty_like(d0)
st = torch.cuda.Stream(dev)
hip = C.CDLL("libamdhip64.so")


def timed(fn, n=20):
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        fn(i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6


def h2d(i):
    with torch.cuda.stream(st):
        d0.copy_(host[i % 4], non_blocking=True)


def d2d(i):
    with torch.cuda.stream(st):
        d1.copy_(d0, non_blocking=True)


def raw(i):
    src = host[i % 4]
    hip.hipMemcpyAsync(C.c_void_p(d0.data_ptr()), C.c_void_p(src.data_ptr()), C.c_size_t(src.numel()), 1,
                       C.c_void_p(st.cuda_stream))


print("is_pinned", host.is_pinned(), host[1].is_pinned())
for name, fn in (("torch h2d pinned", h2d), ("torch d2d", d2d), ("hipMemcpyAsync h2d", raw)):
    hu, tu = timed(fn)
    print(f"{name:22s} host {hu:8.1f} us/call   host+device {tu:8.1f} us/call", flush=True)
