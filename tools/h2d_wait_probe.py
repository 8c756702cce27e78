#!/usr/bin/env python3
"""Does an H2D copy_ from page-locked memory block the host when its stream waits on an event
that has not completed yet (diagnostic)?  A compute stream runs ~2 ms of matmuls per step; the
copy stream (a) copies with no dependency, (b) first waits on an event recorded behind the
compute stream's pending work.  Host time per copy_ call is printed."""
import time

import torch

dev = torch.device("cuda", 0)
host = torch.empty((4, 8, 512, 640, 3), dtype=torch.uint8, pin_memory=True)
dst = torch.empty((8, 512, 640, 3), dtype=torch.uint8, device=dev)
a = torch.randn(4096, 4096, device=dev)
comp, cs = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
for mode in ("nodep", "dep", "dep-queried"):
    torch.cuda.synchronize()
    tc = 0.0
    t0 = time.perf_counter()
    for i in range(30):
        with torch.cuda.stream(comp):
            for _ in range(8):
                a = (a @ a).clamp_(-1, 1)
            ev = torch.cuda.Event()
            ev.record(comp)
        if mode == "dep" or (mode == "dep-queried" and not ev.query()):
            cs.wait_event(ev)
        h0 = time.perf_counter()
        with torch.cuda.stream(cs):
            dst.copy_(host[i % 4], non_blocking=True)
        tc += time.perf_counter() - h0
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{mode:12s} copy_ host {tc / 30 * 1e6:8.1f} us/call; loop host {(t1 - t0) / 30 * 1e6:8.1f} us/step, "
          f"wall {(t2 - t0) / 30 * 1e6:8.1f} us/step", flush=True)
