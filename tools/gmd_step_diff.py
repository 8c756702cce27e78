#!/usr/bin/env python3
"""Where the pipelined motion detector first departs from the serial one: the product
StreamPipeline (motion detection on the tracker stream) at --inflight D, with every step's device
motion records copied in stream order on the tracker stream (step_hook, no host sync), compared
step by step with the serial pipeline on test_pipeline_with_global_motion_matches_serial's scene;
prints the first differing step and field per repetition.

usage: gmd_step_diff.py [--inflight 6] [--reps 6]"""
import argparse
import ctypes as C
import importlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"
P = importlib.import_module(PKG)
pipeline = importlib.import_module(PKG + ".pipeline")
L = importlib.import_module(PKG + "._lib")


class IsolatedMotionPipeline(pipeline.StreamPipeline):
    """--isolate: the motion detector of step t waits for every detector slot stream (all forwards
    up to t done) and forward(t + 1) waits for it, so no forward overlaps the motion kernels."""

    def step(self):
        k = self._k
        s = self._slot(k)
        cur = self._stream(s)
        if self._trk_pending[k]:
            cur.wait_event(self._ev_trk[k])
            self._trk_pending[k] = False
        if getattr(self, "_ev_motion_done", None) is not None:
            cur.wait_event(self._ev_motion_done)
        with torch.cuda.stream(cur):
            self.models[s].detect(self.frame_slots[s], self.conf, self.iou, self.max_det, self._dets[k],
                                  self._counts[k], graph=bool(self.graph))
        self._ev_det[k].record(cur)
        for j in range(self.D):
            self.trk_stream.wait_stream(self._stream(j))
        with torch.cuda.stream(self.trk_stream):
            self.gmd.detect_device(self.frame_slots[s])
            self._ev_gmd[s].record(self.trk_stream)
            self._gmd_pending[s] = True
            ev = torch.cuda.Event()
            ev.record(self.trk_stream)
            self._ev_motion_done = ev
            self.tracker.step_device(self._dets[k], self._counts[k], motion=self.gmd.motion_ptr)
        if self.step_hook is not None:
            self.step_hook(self, k, cur, self.trk_stream)
        self._ev_trk[k].record(self.trk_stream)
        self._trk_pending[k] = True
        self._k = (k + 1) % self.nb


class PrivateFramePipeline(pipeline.StreamPipeline):
    """--private: the motion detector reads its own copy of the step's frames, made on the tracker
    stream from the caller's (never rewritten) source tensor instead of the detector slot."""

    def run(self, frames):
        self._src = frames
        super().run(frames)

    def _track(self, k, s):
        if getattr(self, "_gbuf", None) is None:
            self._gbuf = torch.empty_like(self.frames)
        self._gbuf.copy_(self._src, non_blocking=True)
        self.gmd.detect_device(self._gbuf)
        self.tracker.step_device(self._dets[k], self._counts[k], motion=self.gmd.motion_ptr)


def main():
    from gmd_helpers import camera_sequence
    from gpu_helpers import d2d_async

    ap = argparse.ArgumentParser()
    ap.add_argument("--inflight", type=int, default=6)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--isolate", action="store_true", help="no forward overlaps the motion kernels")
    ap.add_argument("--private", action="store_true", help="motion reads a tracker-stream copy of the frames")
    ap.add_argument("--serial", action="store_true", help="repetitions run the serial pipeline too (baseline noise)")
    ap.add_argument("--overlap", action="store_true",
                    help="the round-4 schedule: motion kernels beside the forwards (YK_MOTION_OVERLAP=1, no windows)")
    ap.add_argument("--beside", type=int, default=0,
                    help="MiB: a host thread keeps device-to-device torch copies of this size running on a stream of "
                         "its own during every run (no detector code beside the motion kernels: use with the serial "
                         "pipeline, --serial)")
    a = ap.parse_args()
    if a.overlap:
        os.environ["YK_MOTION_OVERLAP"] = "1"
    S, F = 3, 20
    seqs = [camera_sequence(80 + s, F, h=512, w=640, whip_at=(7, 14), n_targets=12)[0] for s in range(S)]
    frames = torch.from_numpy(np.stack(seqs, 1)).cuda()
    nbytes = S * L.MOTION_DTYPE.itemsize

    def run(pipelined, inflight, churn=False):
        cls = pipeline.StreamPipeline
        if pipelined and a.isolate:
            cls = IsolatedMotionPipeline
        elif pipelined and a.private:
            cls = PrivateFramePipeline
        pipe = cls("yolov8s-small.yaml", S, (512, 640), "bf16", seed=0, max_tracks=256,
                                       pipelined=pipelined, inflight=inflight, tracker_policy=1,
                                       motion_method="optical_flow")
        rec = torch.zeros((F, nbytes), dtype=torch.uint8, device="cuda")
        ptrs = [C.c_void_p() for _ in range(4)]
        M = C.c_int32()
        L.check(L.lib().yk_gmd_debug_buffers(pipe.gmd._h, *[C.byref(q) for q in ptrs], C.byref(M)), "debug buffers")
        M = M.value
        pp = [C.c_void_p() for _ in range(4)]
        per = C.c_int64()
        L.check(L.lib().yk_gmd_debug_pyramids(pipe.gmd._h, *[C.byref(q) for q in pp], C.byref(per)), "pyramids")
        per = per.value
        pyr = torch.zeros((F, 2, S * per), dtype=torch.uint8, device="cuda")
        der = torch.zeros((F, 2, S * per * 4), dtype=torch.uint8, device="cuda")
        cor = torch.zeros((F, S, M, 2), dtype=torch.float32, device="cuda")
        nxt = torch.zeros((F, S, M, 2), dtype=torch.float32, device="cuda")
        step = [0]

        def hook(p, k, det_stream, trk_stream):
            t = step[0]
            # (motion windows: each step's record is its own buffer; the debug buffers below then
            # hold the state after the wave's last motion call, so only the records are per step)
            src = p._motion_out[k].data_ptr() if getattr(p, "_windowed", False) else p.gmd.motion_ptr
            d2d_async(rec[t].data_ptr(), src, nbytes, trk_stream)
            d2d_async(cor[t].data_ptr(), ptrs[0].value, S * M * 8, trk_stream)
            d2d_async(nxt[t].data_ptr(), ptrs[1].value, S * M * 8, trk_stream)
            for j in range(2):
                d2d_async(pyr[t, j].data_ptr(), pp[j].value, S * per, trk_stream)
                d2d_async(der[t, j].data_ptr(), pp[2 + j].value, S * per * 4, trk_stream)
            step[0] += 1

        pipe.frames.copy_(frames[0])
        pipe.capture(tune=False)
        pipe.step_hook = hook
        side = None
        if a.beside and churn:
            import threading

            stop = threading.Event()
            sbuf = [torch.empty(a.beside << 18, dtype=torch.float32, device="cuda") for _ in range(2)]
            sst = torch.cuda.Stream()

            def spin():
                n = 0
                while not stop.is_set():
                    with torch.cuda.stream(sst):
                        sbuf[n & 1].copy_(sbuf[(n + 1) & 1])
                        sbuf[n & 1].add_(1.0)
                    n += 1
                    if n % 32 == 0:  # bound the queue (~32 x 2 kernels of a few tens of us each)
                        sst.synchronize()
                spin.n = n

            sys.setswitchinterval(1e-4)  # the side thread gets the GIL between the pipeline's calls

            spin.n = 0
            side = threading.Thread(target=spin)
            side.start()
        for t in range(F):
            pipe.run(frames[t])
        pipe.sync()
        if side is not None:
            stop.set()
            side.join()
            torch.cuda.synchronize()
            print(f"    beside: {spin.n} copy + add pairs of {a.beside} MiB ran on another stream", flush=True)
        info = np.zeros((S, 5), np.int32)  # diag builds (YK_GMD_DIAG 4 / 8): LK self-consistency counters
        L.check(L.lib().yk_gmc_info(pipe.gmd._h, L.ptr(info), L.current_stream(0)), "yk_gmc_info")
        if info[:, :2].any():
            print(f"    LK recompute mismatches: same wave {info[:, 0].tolist()}  second launch {info[:, 1].tolist()}",
                  flush=True)
        # every frame buffer must still hold the frame last copied into it
        held = [(f"slot{(F - 1 - j) % pipe.D if pipe.D > 1 else 0}", pipe.frame_slots[(F - 1 - j) % pipe.D], frames[F - 1 - j])
                for j in range(pipe.D)]
        if getattr(pipe, "_gbuf", None) is not None:
            held.append(("private", pipe._gbuf, frames[F - 1]))
        for name, buf, want in held:
            nbad = int((buf != want).sum())
            if nbad:
                idx = (buf != want).flatten().nonzero()[:4].flatten().tolist()
                print(f"    {name}: {nbad} bytes differ from the frame copied in, first at {idx}", flush=True)
        return (np.frombuffer(rec.cpu().numpy().tobytes(), dtype=L.MOTION_DTYPE).reshape(F, S), cor.cpu().numpy(),
                nxt.cpu().numpy(), pyr.cpu().numpy(), der.cpu().numpy())

    ref, rcor, rnxt, rpyr, rder = run(False, 1)
    bad = 0
    for r in range(a.reps):
        got, gcor, gnxt, gpyr, gder = run(False, 1, True) if a.serial else run(True, a.inflight, True)
        for t in range(1, F):  # first step whose pyramid / derivative buffers differ (both written)
            bp = [int((rpyr[t, j] != gpyr[t, j]).sum()) for j in range(2)]
            bd = [int((rder[t, j] != gder[t, j]).sum()) for j in range(2)]
            if any(bp) or any(bd):
                print(f"rep {r}: pyramid bytes differing at step {t}: pyr {bp} der {bd}", flush=True)
                break
        # first step whose corners / LK end points differ (any stream), before the motion record
        for t in range(F):
            # the first n_corners entries of each stream (the rest is not written by that step)
            live = np.arange(rcor.shape[2])[None, :, None] < ref[t]["n_corners"][:, None, None]
            dc = np.argwhere((rcor[t] != gcor[t]) & live)
            dn = np.argwhere((rnxt[t] != gnxt[t]) & live)
            if len(dc) or len(dn):
                what = "corners" if len(dc) else "lk_next"
                s_, i_ = (dc if len(dc) else dn)[0][:2]
                src = (rcor, gcor) if len(dc) else (rnxt, gnxt)
                print(f"rep {r}: first {what} difference at step {t} stream {s_} point {i_} "
                      f"({len(dc)} corner / {len(dn)} end-point values differ): serial {src[0][t, s_, i_].tolist()} "
                      f"pipelined {src[1][t, s_, i_].tolist()}", flush=True)
                break
        first = None
        for t in range(F):
            for f in ref.dtype.names:
                if ref[t][f].tobytes() != got[t][f].tobytes():
                    first = (t, f)
                    break
            if first:
                break
        if first:
            bad += 1
            t, f = first
            print(f"rep {r}: first difference at step {t}, field {f}", flush=True)
            for name in ("n_corners", "n_tracked", "n_inliers", "magnitude", "vector"):
                print(f"    {name:9s} serial {ref[t][name].tolist()}  pipelined {got[t][name].tolist()}", flush=True)
        else:
            print(f"rep {r}: identical", flush=True)
    print(f"inflight={a.inflight}{' isolated' if a.isolate else ''}{' private' if a.private else ''}{' serial' if a.serial else ''}"
          f"{' overlap' if a.overlap else ''}: {bad} of {a.reps} runs differ", flush=True)
    n = np.zeros(1, np.int64)
    L.check(L.lib().yk_store_check_count(L.ptr(n)), "yk_store_check_count")
    print("detector stores outside the detector's allocations:",
          "n/a (product library)" if n[0] < 0 else int(n[0]), flush=True)


if __name__ == "__main__":
    main()
