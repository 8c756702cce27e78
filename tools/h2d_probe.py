#!/usr/bin/env python3
"""Host -> HBM copy rate of the bench's frame batches (page-locked source, the DMA engine):
one batch of S frames per copy, back to back on one stream, and split over two / four streams.

usage: h2d_probe.py [--streams 8] [--hw 512x640] [--reps 200]
Prints one JSON line: GB/s per configuration, and the frames/s ceiling each implies."""
import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=8)
    ap.add_argument("--hw", default="512x640")
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    H, W = (int(v) for v in a.hw.split("x"))
    S = a.streams
    nb = S * H * W * 3
    host = [torch.empty(nb, dtype=torch.uint8, pin_memory=True) for _ in range(4)]
    for h in host:
        h.fill_(7)
    dev = [torch.empty(nb, dtype=torch.uint8, device="cuda") for _ in range(4)]
    out = {"bytes_per_copy": nb, "frames_per_copy": S}
    for ns in (1, 2, 4):
        sts = [torch.cuda.Stream() for _ in range(ns)]
        for i in range(8):  # warm-up (first DMA from a fresh page-locked page maps it)
            with torch.cuda.stream(sts[i % ns]):
                dev[i % 4].copy_(host[i % 4], non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.reps):
            with torch.cuda.stream(sts[i % ns]):
                dev[i % 4].copy_(host[i % 4], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        gbs = nb * a.reps / dt / 1e9
        out[f"h2d_{ns}_streams_GBps"] = round(gbs, 2)
        out[f"h2d_{ns}_streams_frames_per_s"] = round(S * a.reps / dt, 1)
    t0 = time.perf_counter()
    for i in range(a.reps):
        host[i % 4].copy_(dev[i % 4], non_blocking=True)
    torch.cuda.synchronize()
    out["d2h_1_stream_GBps"] = round(nb * a.reps / (time.perf_counter() - t0) / 1e9, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
