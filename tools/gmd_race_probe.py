#!/usr/bin/env python3
"""Probe of the round-4 motion-stream race: the motion detector on a stream of its own (one
yk_motion record per detection buffer; the variant withdrawn from pipeline.py), compared with the
serial pipeline --reps times in one process on test_pipeline_with_global_motion_matches_serial's
scene.  Run it under different GPU_MAX_HW_QUEUES to see whether the mismatches need two of the
pipeline's streams to share a hardware queue.

usage: gmd_race_probe.py [--reps 6] [--inflight 3]"""
import argparse
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


class MotionStreamPipeline(pipeline.StreamPipeline):
    """motion(t) on its own stream after forward(t), writing record t mod nb; tracker(t) waits for it."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        dev = torch.device("cuda", self.device)
        self.gmd_stream = torch.cuda.Stream(dev)
        self._motion = torch.zeros((self.nb, self.S * L.MOTION_DTYPE.itemsize), dtype=torch.uint8, device=dev)

    def step(self):
        k = self._k
        s = self._slot(k)
        cur = self._stream(s)
        trk_busy = self._trk_pending[k]
        if trk_busy:
            cur.wait_event(self._ev_trk[k])
            self._trk_pending[k] = False
        with torch.cuda.stream(cur):
            self.models[s].detect(self.frame_slots[s], self.conf, self.iou, self.max_det, self._dets[k],
                                  self._counts[k], graph=bool(self.graph))
        self._ev_det[k].record(cur)
        self.gmd_stream.wait_event(self._ev_det[k])
        if trk_busy:
            self.gmd_stream.wait_event(self._ev_trk[k])
        with torch.cuda.stream(self.gmd_stream):
            self.gmd.detect_device(self.frame_slots[s], out=self._motion[k].data_ptr())
        self._ev_gmd[s].record(self.gmd_stream)
        self._gmd_pending[s] = True
        self.trk_stream.wait_event(self._ev_det[k])
        self.trk_stream.wait_event(self._ev_gmd[s])
        with torch.cuda.stream(self.trk_stream):
            self.tracker.step_device(self._dets[k], self._counts[k], motion=self._motion[k].data_ptr())
        self._ev_trk[k].record(self.trk_stream)
        self._trk_pending[k] = True
        self._k = (k + 1) % self.nb


def main():
    from gmd_helpers import camera_sequence

    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--inflight", type=int, default=3)
    a = ap.parse_args()
    S, F = 3, 20
    seqs = [camera_sequence(80 + s, F, h=512, w=640, whip_at=(7, 14), n_targets=12)[0] for s in range(S)]
    frames = torch.from_numpy(np.stack(seqs, 1)).cuda()

    def run(cls, pipelined, inflight):
        pipe = cls("yolov8s-small.yaml", S, (512, 640), "bf16", seed=0, max_tracks=256, pipelined=pipelined,
                   inflight=inflight, tracker_policy=1, motion_method="optical_flow")
        pipe.frames.copy_(frames[0])
        pipe.capture(tune=False)
        for t in range(F):
            pipe.run(frames[t])
        pipe.sync()
        _, counts, stats = pipe.tracker.download()
        motion, mstats = pipe.gmd.download()
        return counts.copy(), stats.copy(), motion.copy(), mstats.copy()

    ref = run(pipeline.StreamPipeline, False, 1)
    bad = 0
    for r in range(a.reps):
        got = run(MotionStreamPipeline, True, a.inflight)
        diff = [n for n, x, y in zip(("counts", "stats", "motion", "gmd_stats"), ref, got) if x.tobytes() != y.tobytes()]
        bad += bool(diff)
        print(f"rep {r}: {'differs in ' + ','.join(diff) if diff else 'identical'}", flush=True)
    print(f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES', 'default')} inflight={a.inflight}: "
          f"{bad} of {a.reps} runs differ", flush=True)


if __name__ == "__main__":
    main()
