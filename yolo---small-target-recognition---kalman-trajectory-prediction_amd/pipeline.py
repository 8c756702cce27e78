"""End-to-end detect-and-track step for S independent video streams on one GPU.

One step = the reference driver's per-frame body (kalman/aircraft_detection_tracking.py:96-109)
for every stream at once: ``model(frame)`` for S frames as one batch (yk_detect), then one
``tracker.update(detections)`` per stream (yk_tracker_step, one workgroup per stream), with
the NMS output handed to the tracker in HBM (rows [x1, y1, x2, y2, conf, cls] float32, the
reference's np.float32 detections).  The driver's ``score > 0.1`` filter (:105) is a no-op
at conf >= 0.1 and is checked, not executed.  The detector (~90 launches) replays as one
native hipGraph (yk_detect_graph); the tracker is one more launch.

``pipelined=True`` runs the tracker on its own HIP stream: detector(t+1) does not depend on
tracker state, so it starts while tracker(t) is still running.  Detections are
double-buffered; detector(t+2) waits for tracker(t) to have read its buffer.  Results are
identical to the serial order (the tracker still sees frames in order on one stream).

``motion_method='optical_flow'`` (with ``tracker_policy=1``, the camera-motion-compensation
tracker) adds the global camera-motion branch of MotionCompensatedMultiTracker.update(dets,
frame) (motion_compensated_multi_tracker.py:94-121): GlobalMotionDetector on every stream's
frame (motion.BatchedMotionDetector, gmd.hip) on the tracker stream right before the tracker
step, which consumes its device results.  The frame slot is not refilled before that detector
has read it.

With the motion detector on a pipelined tracker stream, the motion kernels never overlap a
forward (motion windows): the D forwards of a wave (steps t .. t + D - 1) run concurrently, then
one window on the tracker stream -- which waits for every forward enqueued so far -- runs the
wave's motion + tracker steps in frame order, and the next wave's forwards wait for the window.
A step's tracker output therefore exists once its wave's window has been enqueued (the last step
of the wave, or flush() / sync()).  The window's motion calls run as one launch sequence
(yk_gmd_detect_window: its steps' frame pairs side by side, each stream's detector state stepped
in frame order; the per-call records bit for bit).  Round 5 traced run-to-run differences of the pipelined motion records to the Lucas-Kanade
kernel alone: one wave solving its corner twice in one launch read different J samples at the
same addresses in the two passes while forwards ran beside it (csrc/gmd.hip YK_GMD_DIAG 4),
with every pyramid producer wave provably complete before the launch (diag 16) and with the
pyramids in fine-grained or uncached memory (diag 32 / 64) -- not a stale cache line, not an
ordering fault of ours, not fixed by fences.  No overlap, no difference.

``inflight=D`` > 1 (needs ``pipelined``) keeps D detector forwards in flight: D DeviceModels
(same program and conv plan, each its own activation arena) replay their hipGraphs on D HIP
streams, step t on slot t % D with its own detection buffer.  Every forward is still one batch of the S streams' frames;
the tracker consumes the detections in frame order.  The detector's ~90 launches are each
bound by their own latency, not by the chip (op time is nearly flat in the batch), and the
parallel branches inside one captured graph execute one after the other, so a second
independent graph on another stream is what fills the idle CUs (tools/inflight.py: 1.45x).

``frames_per_forward=T`` > 1 (temporal batching; forwards in flight) makes
one forward of T consecutive steps' frames: run() t uploads step t's S frames into sub-batch
t % T of the forward's frame buffer, and the T-th run() launches one batch-(T S) forward and then
the T tracker steps in frame order.  Detections of one image do not depend on the other images
of the batch (same kernels, same plan), and the tracker still sees every stream's frames in
order, so the results are the T = 1 pipeline's; a step's tracker output exists once its forward
has been launched (its T-th run(), or flush()).  Measured: fp32 +4 %, bf16 +18 % at T = 2
(gpurun_out/r6a, BASELINE config 3).  With the motion detector the window runs each forward's T
steps (the motion detector on each step's sub-batch of the slot's frames, in frame order, then
the tracker steps), so a wave of D forwards covers D T steps.
"""
from __future__ import annotations

import numpy as np
import torch

from . import arch as A
from . import model as M
from . import tracker as T
from . import weights as Wt


class StreamPipeline:
    def __init__(self, model_cfg: str = "yolov8s-small.yaml", n_streams: int = 8, frame_hw=(512, 640),
                 dtype: str = "fp32", weights=None, seed: int = 0, conf: float = 0.25, iou: float = 0.7,
                 max_det: int = 300, max_lost_frames: int = 150, min_hits: int = 1, iou_threshold: float = 0.1,
                 max_tracks: int = 512, device: int = 0, pipelined: bool = False, imgsz=640, inflight: int = 1,
                 tracker_policy: int = 0, motion_method: str | None = None, frames_per_forward: int = 1):
        if conf < 0.1:
            raise ValueError("conf < 0.1 would need the driver's score > 0.1 filter on the device path")
        self.S, self.device = int(n_streams), int(device)
        self.T = int(frames_per_forward)
        if not 1 <= self.T <= 8:
            raise ValueError("frames_per_forward must be in [1, 8]")
        if self.T > 1 and (int(inflight) < 2 or not pipelined):
            raise ValueError("frames_per_forward > 1 needs inflight > 1 (pipelined)")
        if self.T > 1 and motion_method is not None and __import__("os").environ.get("YK_MOTION_OVERLAP") == "1":
            raise ValueError("frames_per_forward > 1 with a motion detector needs the motion windows")
        self.conf, self.iou, self.max_det = float(conf), float(iou), int(max_det)
        ar = A.parse_arch(A.load_model_dict(model_cfg))
        sd = weights if weights is not None else Wt.synthetic_state_dict(ar, seed)
        self.prog = M.Program(ar, sd, frame_hw[0], frame_hw[1], imgsz, self.T * self.S, dtype, self.max_det)
        self.model = M.DeviceModel(self.prog, self.device)
        self.tracker = T.MultiStreamTracker(self.S, max_lost_frames, min_hits, iou_threshold, max_tracks,
                                            self.max_det, self.device,
                                            policy=tracker_policy)
        dev = torch.device("cuda", self.device)
        BF = self.T * self.S  # images per forward
        # slot 0's frame buffer; `frames` is its first step's S images (the capture / autotune input)
        self.forward_frames = torch.zeros((BF, frame_hw[0], frame_hw[1], 3), dtype=torch.uint8, device=dev)
        self.frames = self.forward_frames[:self.S]
        # motion windows (see the header): with the motion detector on a pipelined tracker stream
        # (YK_MOTION_OVERLAP=1, diagnostics only: the round-4 schedule, motion kernels on the tracker
        # stream beside the forwards -- tools/gmd_step_diff.py --overlap)
        self._windowed = motion_method is not None and bool(pipelined) and \
            __import__("os").environ.get("YK_MOTION_OVERLAP") != "1"
        # detection buffers: 2 D when the tracker runs on its own stream, so the forward of step
        # t + D does not wait for the tracker step of step t (HBM-resident rate +6.6 % fp32, +11.5 %
        # bf16, profiles/r05_inflight_lanes_sweep.txt), and with motion windows the next wave's
        # forwards do not wait for this wave's tracker steps; D (at least 2) otherwise
        self.nb = max(2, int(inflight)) * (2 if pipelined else 1)
        self._dets = torch.zeros((self.nb, BF, self.max_det, 6), dtype=torch.float32, device=dev)
        self._counts = torch.zeros((self.nb, BF), dtype=torch.int32, device=dev)
        self._k = 0  # detection buffer the next step writes
        self._j = 0  # (frames_per_forward > 1) steps uploaded into the next forward's frame buffer
        self._last = (0, 0)  # (detection buffer, sub-batch) of the most recent tracker step
        self._hook_j = 0  # sub-batch of the step the step hook is called for
        self._dl_t = {}  # (frames_per_forward > 1) download_async requests by sub-batch, issued after its tracker step
        self._n_sub = self.T  # sub-batches the next step() tracks (fewer in a partial flush)
        self.pipelined = bool(pipelined)
        # default stream priorities: a high-priority tracker / motion stream halved the bf16 line
        # (12,301 -> 5,974 frames/s, profiles/r04_cmc_ab.txt).  The motion detector stays on the
        # tracker stream: moving it to a stream of its own (+13 % on the bf16 CMC line) made the
        # pipelined motion records differ from the serial ones in 3 of 5 runs of
        # test_pipeline_with_global_motion_matches_serial, a race not found in round 4
        self.trk_stream = torch.cuda.Stream(dev) if self.pipelined else None
        self._ev_det = [torch.cuda.Event() for _ in range(self.nb)]
        self._ev_trk = [torch.cuda.Event() for _ in range(self.nb)]
        self._trk_pending = [False] * self.nb
        self.graph = None
        self.step_hook = None  # callable(pipe, k, det_stream, trk_stream), see step()
        self.D = int(inflight)
        if not 1 <= self.D <= 8:
            raise ValueError("inflight must be in [1, 8]")
        if self.D > 1 and not self.pipelined:
            raise ValueError("inflight > 1 needs pipelined=True (the tracker runs on its own stream)")
        # slot s: detector model, input frames and launch stream (None = the caller's stream)
        self.models = [self.model] + [M.DeviceModel(self.prog, self.device) for _ in range(self.D - 1)]
        # frame buffers: one per detector slot; or, with forwards in flight and no motion detector, a
        # ring of 2 nb = 4 D that the step index walks (one graph per frame buffer), so a host-frame
        # upload lands in the buffer its forward reads -- no staging hop -- and rewrites a buffer 4 D
        # steps after its forward, which has long finished (bf16 +4-6 %, fp32 unchanged,
        # profiles/r05_inflight_lanes_sweep.txt; a 2 D ring made the copies wait, -15 %)
        self._ring = self.D > 1 and motion_method is None
        nf = 2 * self.nb if self._ring else self.D
        self.frame_slots = [self.forward_frames] + [torch.zeros_like(self.forward_frames) for _ in range(nf - 1)]
        self._ev_fread = [torch.cuda.Event() for _ in range(nf)] if self._ring else []  # its forward
        self._fread_pending = [False] * nf
        self._kf = 0  # (ring) frame buffer of the next step
        # one created stream per slot with forwards in flight (the caller's stream with one: the
        # serial order); slot 0 on the legacy null stream cost ~4 % of the host-frame rate
        self.det_streams = [None] if self.D == 1 else [torch.cuda.Stream(dev) for _ in range(self.D)]
        if self.D > 1:
            # forwards in flight are the concurrency: one lane per graph (bench.py's default too).
            # Multi-lane (forked) graphs of several in-flight slots plus other live models were
            # seen to crash the HIP runtime inside hipGraphLaunch (tools/graph_lanes_repro.py, round 4)
            self.set_schedule(1, 1)
        self.gmd = None
        if motion_method is not None:
            if tracker_policy != 1:
                raise ValueError("motion_method needs tracker_policy=1 (the camera-motion-compensation tracker)")
            from . import motion as Mo

            self.gmd = Mo.BatchedMotionDetector(self.S, frame_hw[0], frame_hw[1], motion_method, self.device)
        self._ev_gmd = [torch.cuda.Event() for _ in range(self.D)]  # slot's frames read by the motion detector
        self._gmd_pending = [False] * self.D
        # host-frame prefetch (run(..., next_frames=)): the next step's upload runs on its own copy
        # stream one step ahead, behind the forward that last read that slot
        # Uploads go to a staging ring, not to the slot: a slot is still being read by its forward
        # from D steps ago when the next upload is issued, and a copy stream made to wait for that
        # forward holds the host thread in hipMemcpyAsync (the runtime resolves an SDMA copy's
        # cross-stream wait on the host: ~1 ms per step, bench --io h2d).  A staging buffer is read
        # by the slot stream's staging -> slot copy in front of its forward; with D + 4 buffers the
        # buffer an upload reuses was read D + 4 steps earlier, which the host never outruns while
        # D forwards are in flight, so the copy stream waits for nothing in steady state.
        self.copy_stream = torch.cuda.Stream(dev) if self.D > 1 else None
        self.n_stage = self.D + 4 if self.D > 1 and not self._ring else 0
        self._stage = [torch.empty_like(self.frames) for _ in range(self.n_stage)]
        self._ev_stage_read = [torch.cuda.Event() for _ in range(self.n_stage)]  # slot stream's copy out of it
        self._stage_read_pending = [False] * self.n_stage
        self._ev_copy = [torch.cuda.Event() for _ in range(nf * self.T if self._ring else self.n_stage)]
        self._n_stage = 0
        self._prefetched = __import__("collections").deque()  # (data_ptr of the host frames, staging index), one per upcoming step
        self._ev_window = None  # end of the last motion window (the next wave's forwards wait for it)
        # a window's motion calls as one launch sequence (yk_gmd_detect_window); YK_GMD_WINDOW=0: one
        # yk_gmd_detect per step (the A/B of profiles/r06_sweeps.txt r6ac)
        self._gmd_window = __import__("os").environ.get("YK_GMD_WINDOW", "1") != "0"
        self.fw_events = None  # a list: step() appends (start, end, tracker start, tracker end) timing events of each forward
        self._wave = []  # detection buffers of the current wave's steps (forwards enqueued, window not yet)
        self._dl = {}  # download_async requests of the current wave's steps, issued in its window
        self._motion_out = None  # per detection buffer: its step's yk_motion[S] (motion windows)

    def step_outputs(self, k: int, j: int | None = None):
        """(detections [S, max_det, 6], counts [S]) of detection buffer k's sub-batch j (the step
        the step hook is being called for when j is None)."""
        j = self._hook_j if j is None else j
        S = self.S
        return self._dets[k][j * S:(j + 1) * S], self._counts[k][j * S:(j + 1) * S]

    @property
    def dets(self) -> torch.Tensor:
        """Detections [S, max_det, 6] of the most recent tracker step."""
        return self.step_outputs(*self._last)[0]

    @property
    def counts(self) -> torch.Tensor:
        return self.step_outputs(*self._last)[1]

    def set_schedule(self, groups: int, lanes: int):
        for m in self.models:
            m.set_schedule(groups, lanes)

    def sync_plan(self):
        """Give every detector slot model 0's conv plan (autotuned or loaded)."""
        b, plan = self.model.get_plan()
        if b:
            for m in self.models[1:]:
                m.load_plan(b, plan)

    def _slot(self, k: int) -> int:
        return k % self.D

    def _stream(self, s: int):
        st = self.det_streams[s]
        return torch.cuda.current_stream(self.device) if st is None else st

    def capture(self, tune: bool = True):
        """Autotune the conv kernels for this batch (on the current frames), then build and warm
        the detector's native hipGraph(s); later steps replay them."""
        for j in range(1, self.T):  # every sub-batch of the forward holds the current frames
            self.forward_frames[j * self.S:(j + 1) * self.S].copy_(self.frames)
        if tune:
            self.model.autotune(self.forward_frames, self.conf)
        self.sync_plan()
        for fs in self.frame_slots[1:]:
            fs.copy_(self.forward_frames)
        self.graph = True
        # one graph per (frame buffer, detection buffer) pair the steps use, in step order from the
        # current step: the ring's frame index and the detection buffer index advance together
        n = len(self.frame_slots) if self._ring else self.nb
        for j in range(n):
            k = (self._k + j) % self.nb
            s = self._slot(k)
            f = (self._kf + j) % len(self.frame_slots) if self._ring else s
            with torch.cuda.stream(self._stream(s)):
                self.models[s].detect(self.frame_slots[f], self.conf, self.iou, self.max_det, self._dets[k],
                                      self._counts[k], graph=True)
        torch.cuda.synchronize(self.device)
        return self.graph

    def step(self):
        k = self._k
        s = self._slot(k)
        cur = self._stream(s)
        if self._trk_pending[k]:  # tracker(t - nb) still reads buffer k
            cur.wait_event(self._ev_trk[k])
            self._trk_pending[k] = False
        if self._ev_window is not None:  # no forward beside a motion window
            cur.wait_event(self._ev_window)
        f = self._kf if self._ring else s
        if self.fw_events is not None:  # (diagnostics: each forward's start / end on its stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cur)
        with torch.cuda.stream(cur):
            self.models[s].detect(self.frame_slots[f], self.conf, self.iou, self.max_det, self._dets[k],
                                  self._counts[k], graph=bool(self.graph))
        if self.fw_events is not None:
            e1.record(cur)
            self.fw_events.append([e0, e1, None, None])
        if self._ring:
            self._ev_fread[f].record(cur)
            self._fread_pending[f] = True
            self._kf = (f + 1) % len(self.frame_slots)
        if self._windowed:
            self._ev_det[k].record(cur)
            self._wave.append((k, self._n_sub))
            for j, req in self._dl_t.items():  # (T > 1) requests of this forward's steps, issued in the window
                self._dl[(k, j)] = req
            self._dl_t = {}
            self._k = (k + 1) % self.nb
            if len(self._wave) == self.D:
                self._run_window()
            return
        if self.pipelined:
            self._ev_det[k].record(cur)
            self.trk_stream.wait_event(self._ev_det[k])
            if self.fw_events is not None:  # (diagnostics: its tracker steps' start / end)
                self.fw_events[-1][2] = torch.cuda.Event(enable_timing=True)
                self.fw_events[-1][2].record(self.trk_stream)
            for j in range(self._n_sub):  # the forward's steps, in frame order
                with torch.cuda.stream(self.trk_stream):
                    self._track(k, s, j)
                self._after_track(k, j, cur)
            if self.fw_events is not None:
                self.fw_events[-1][3] = torch.cuda.Event(enable_timing=True)
                self.fw_events[-1][3].record(self.trk_stream)
            self._ev_trk[k].record(self.trk_stream)
            self._trk_pending[k] = True
        else:
            self._track(k, s)
            self._after_track(k, 0, cur)
        self._k = (k + 1) % self.nb

    def _after_track(self, k: int, j: int, cur):
        """After the tracker step of detection buffer k's sub-batch j: the step hook and (T > 1)
        a download_async request of that step."""
        self._last = (k, j)
        if self.step_hook is not None:
            # harness hook (tests/recorders): enqueue work after this step's launches on the
            # detector stream (reads of detection buffer k) and the tracker stream (results)
            self._hook_j = j
            self.step_hook(self, k, cur, self.trk_stream if self.pipelined else cur)
        req = self._dl_t.pop(j, None)
        if req is not None:
            self.tracker.download_async(*req, stream=self.trk_stream.cuda_stream)

    def _track(self, k: int, s: int, j: int = 0):
        """Tracker step of detection buffer k's sub-batch j (frames of slot s) on the current stream."""
        if self.gmd is None:
            self.tracker.step_device(*self.step_outputs(k, j))
            return
        self.gmd.detect_device(self.frame_slots[s][j * self.S:(j + 1) * self.S])
        if self.pipelined:
            self._ev_gmd[s].record(torch.cuda.current_stream(self.device))
            self._gmd_pending[s] = True
        self.tracker.step_device(*self.step_outputs(k, j), motion=self.gmd.motion_ptr)

    def _run_window(self):
        """Motion window of the current wave (see the header): after every forward enqueued so far,
        each step's motion detector in frame order on the tracker stream, each into its own motion
        record; the next forwards wait for the window's end.  Then the wave's tracker steps (plus
        the step hook and any download_async request of each step), which may overlap them."""
        trk = self.trk_stream
        for j in range(self.D):
            trk.wait_stream(self._stream(j))
        if self._motion_out is None:  # the window's records, one row per step (yk_motion[S] each)
            from . import _lib as L

            self._motion_out = torch.zeros((self.D * self.T, self.S * L.MOTION_DTYPE.itemsize), dtype=torch.uint8,
                                           device=self.frames.device)
        S = self.S
        steps = [(k, j) for k, n in self._wave for j in range(n)]
        with torch.cuda.stream(trk):  # the exclusive part: the wave's motion detector calls, in frame order,
            # as one launch sequence (yk_gmd_detect_window: the steps' frame pairs side by side)
            fr = [self.frame_slots[self._slot(k)][j * S:(j + 1) * S] for k, j in steps]
            if self._gmd_window:
                self.gmd.detect_window(fr, out=self._motion_out.data_ptr())
            else:  # (diagnostics, YK_GMD_WINDOW=0: one call per step)
                for i, f in enumerate(fr):
                    self.gmd.detect_device(f, out=self._motion_out[i].data_ptr())
            for k, _ in self._wave:
                s = self._slot(k)
                self._ev_gmd[s].record(trk)
                self._gmd_pending[s] = True
        self._ev_window = torch.cuda.Event()
        self._ev_window.record(trk)  # the next wave's forwards may start: the tracker steps overlap them
        with torch.cuda.stream(trk):
            i = 0
            for k, n in self._wave:
                s = self._slot(k)
                for j in range(n):
                    self.tracker.step_device(*self.step_outputs(k, j), motion=self._motion_out[i].data_ptr())
                    i += 1
                    self._last = (k, j)
                    if self.step_hook is not None:
                        self._hook_j = j
                        self.step_hook(self, k, self._stream(s), trk)
                    req = self._dl.pop((k, j), None)
                    if req is not None:
                        self.tracker.download_async(*req, stream=trk.cuda_stream)
                self._ev_trk[k].record(trk)
                self._trk_pending[k] = True
        self._wave = []

    def flush(self):
        """Enqueue what run() has held back, so that after it every run() so far has its tracker
        step enqueued: the motion window of a partial wave, or (frames_per_forward > 1) the
        forward of a partly filled frame buffer.  A partial forward runs the whole batch (the
        same graph; the sub-batches not refilled hold older frames) and steps the tracker on the
        filled sub-batches only.  A no-op otherwise."""
        if self.T > 1 and self._j:
            if self._prefetched:
                raise ValueError("flush(): prefetched frames wait for steps not yet run")
            self._n_sub, self._j = self._j, 0
            self.step()
            self._n_sub = self.T
        if self._windowed and self._wave:
            self._run_window()

    def sync(self):
        """Wait for every launched step (detector and tracker streams)."""
        self.flush()
        torch.cuda.synchronize(self.device)

    def run(self, frames: torch.Tensor, next_frames: torch.Tensor | None = None):
        """frames [S, H, W, 3] uint8 (device, or page-locked host memory: the frame in host memory
        the driver loop starts from) -> one step.  The copy runs on the slot's detector stream,
        after that slot's previous forward has read its frames, and after whatever the caller's
        current stream enqueued before this call (the producer of `frames`); the forward that reads
        the slot follows it on the same stream.  A host source must stay unchanged until that copy
        has run (the caller's buffer; see download_async for the matching output side).

        next_frames (page-locked host, inflight > 1): the NEXT step's frames, already decoded (a
        video driver reads ahead).  Their upload is issued now, on the copy stream, into that step's
        frame buffer of the ring (with a motion detector: into a staging buffer that the slot
        stream copies to the slot); the next run() is handed the same tensor and its forward waits
        for that upload's event.  Every frame still crosses PCIe once,
        inside the caller's loop; the upload of step t + 1 overlaps step t.  Frames smaller than
        PULL_BYTES are not prefetched: the next run() pulls them onto the slot stream with a kernel
        (yk_upload_pinned_async), which holds neither the host nor a copy stream."""
        pre = next_frames is not None and next_frames.numel() * next_frames.element_size() >= self.PULL_BYTES
        if pre:  # refuse before anything of this step is enqueued
            self._check_prefetch(next_frames, extra=1 if self._prefetched else 0)
        s = self._slot(self._k)
        st = self._stream(s)
        cur = torch.cuda.current_stream(self.device)
        if self._ring:
            f, j = self._kf, self._j
            if self._prefetched:  # uploaded straight into this step's frame buffer
                ptr, i = self._prefetched[0]
                if frames.data_ptr() != ptr:
                    raise ValueError("run(): other frames were prefetched for this step (next_frames / prefetch)")
                self._prefetched.popleft()
                st.wait_event(self._ev_copy[i])
            else:
                if st != cur:
                    st.wait_stream(cur)
                    if frames.is_cuda:
                        frames.record_stream(st)  # the allocator keeps `frames` alive until the copy ran
                if self._fread_pending[f]:  # its last forward ran on another slot stream
                    st.wait_event(self._ev_fread[f])
                    self._fread_pending[f] = False
                with torch.cuda.stream(st):
                    self._upload(self.frame_slots[f][j * self.S:(j + 1) * self.S], frames)
            if self.T > 1:
                self._j = j + 1
                if self._j < self.T:  # the forward waits for its last step's frames
                    if pre:
                        self.prefetch(next_frames)
                    return
                self._j = 0
        else:
            # the slot's frame buffer: sub-batch j of its forward (T > 1), the whole buffer otherwise
            j = self._j
            dst = self.frame_slots[s][j * self.S:(j + 1) * self.S]
            staged = None
            if self._prefetched:
                ptr, i = self._prefetched[0]
                if frames.data_ptr() != ptr:
                    raise ValueError("run(): other frames were prefetched for this step (next_frames / prefetch)")
                self._prefetched.popleft()
                st.wait_event(self._ev_copy[i])
                staged = i
            elif st != cur:
                st.wait_stream(cur)
                if frames.is_cuda:
                    frames.record_stream(st)  # the allocator keeps `frames` alive until the copy ran
            if self._gmd_pending[s]:  # the motion detector (tracker stream) still reads this slot's frames
                st.wait_event(self._ev_gmd[s])
                self._gmd_pending[s] = False
            if self._ev_window is not None:  # (staging copies, device copies, pull kernels: not beside a motion window)
                st.wait_event(self._ev_window)
            with torch.cuda.stream(st):
                if staged is not None:
                    dst.copy_(self._stage[staged], non_blocking=True)
                else:
                    self._upload(dst, frames)
            if staged is not None:
                self._ev_stage_read[staged].record(st)
                self._stage_read_pending[staged] = True
            if self.T > 1:
                self._j = j + 1
                if self._j < self.T:  # the forward waits for its last step's frames
                    if pre:
                        self.prefetch(next_frames)
                    return
                self._j = 0
        self.step()
        if pre:
            # (frames below PULL_BYTES are pulled on the slot stream by the next run() instead: the
            # pull kernel costs the host nothing, and a copy-stream hop measured 26 % slower at
            # batch 1, bench.py --config 2 --no-prefetch)
            self.prefetch(next_frames)

    @property
    def n_prefetched(self) -> int:
        """Uploads issued by prefetch() that no run() has consumed yet."""
        return len(self._prefetched)

    def prefetch(self, frames: torch.Tensor):
        """Issue the upload of a FUTURE step's page-locked host frames now, on the copy stream, into
        that step's frame buffer (a staging buffer with a motion detector).  Prefetches queue in step order: the run() calls that follow must be
        handed the same tensors, in the same order.  At most 4 may be outstanding."""
        self._check_prefetch(frames)
        cs = self.copy_stream
        if self._ring:
            nf = len(self.frame_slots)
            q = self._kf * self.T + self._j + len(self._prefetched)  # that step's (frame buffer, sub-batch)
            f, j = (q // self.T) % nf, q % self.T
            # its previous reader: the forward of 4 D steps earlier (done in steady state; waiting for
            # it here would hold the host inside the copy call)
            if self._fread_pending[f] and not self._ev_fread[f].query():
                cs.wait_event(self._ev_fread[f])
            self._fread_pending[f] = False
            if frames.is_cuda:  # behind their producer; the allocator keeps them alive until the copy ran
                cs.wait_stream(torch.cuda.current_stream(self.device))
                frames.record_stream(cs)
            with torch.cuda.stream(cs):
                self._upload(self.frame_slots[f][j * self.S:(j + 1) * self.S], frames)
            self._ev_copy[f * self.T + j].record(cs)
            self._prefetched.append((frames.data_ptr(), f * self.T + j))
            return
        i = self._n_stage % self.n_stage
        self._n_stage += 1
        if self._stage_read_pending[i] and not self._ev_stage_read[i].query():
            cs.wait_event(self._ev_stage_read[i])  # (rare: its staging -> slot copy has not run yet)
        self._stage_read_pending[i] = False
        if frames.is_cuda:  # behind their producer; the allocator keeps them alive until the copy ran
            cs.wait_stream(torch.cuda.current_stream(self.device))
            frames.record_stream(cs)
        with torch.cuda.stream(cs):
            self._upload(self._stage[i], frames)
        self._ev_copy[i].record(cs)
        self._prefetched.append((frames.data_ptr(), i))

    def _check_prefetch(self, frames: torch.Tensor, extra: int = 0):
        """Raise ValueError if prefetch(frames) would be refused (after `extra` more steps have
        consumed theirs): no copy stream (inflight 1), frames neither page-locked nor on the
        device, or the prefetch queue full."""
        if self.copy_stream is None or not (frames.is_cuda or frames.is_pinned()):
            raise ValueError("prefetch: page-locked host (or device) frames and inflight > 1")
        cap = 4 if self._ring else self.n_stage - self.D
        if len(self._prefetched) - extra >= cap:
            raise ValueError(f"prefetch: at most {cap} steps ahead")

    # page-locked host frames below this size are pulled by a kernel (yk_upload_pinned_async):
    # the runtime copies small page-locked H2D transfers through the CPU, synchronously (one
    # 640x512 frame held the host ~170 us per step, tools/host_split_probe.py); larger ones go to
    # the DMA engine, which costs no CU time
    PULL_BYTES = int(__import__("os").environ.get("YK_PULL_BYTES", 4 << 20))

    def _upload(self, dst: torch.Tensor, src: torch.Tensor):
        """dst (device) <- src (device, or page-locked host) on the current stream."""
        n = src.numel() * src.element_size()
        if not src.is_cuda and n < self.PULL_BYTES and src.is_pinned() and src.is_contiguous() and n % 16 == 0:
            from . import _lib as L

            L.check(L.lib().yk_upload_pinned_async(L.ptr(dst), L.ptr(src), n, L.current_stream(self.device)),
                    "yk_upload_pinned_async")
        else:
            dst.copy_(src, non_blocking=True)

    def download_async(self, rows, counts, stats, rows_per_stream=None):
        """Enqueue the tracker output of the most recent step into page-locked host buffers
        (rows [S * max_tracks] yk_track_out bytes, counts int32 [S], stats [S] yk_tracker_stats)
        on the tracker stream, behind that step; no host wait.  The host reads them after
        sync() (or an event recorded on the tracker stream after this call).  With motion windows
        the copy is issued right after that step's tracker step, inside its wave's window."""
        if self.T > 1 and self._j:  # this step's forward (and tracker step) has not been launched yet
            self._dl_t[self._j - 1] = (rows, counts, stats, rows_per_stream)
            return
        if self._windowed and self._wave:  # this step's tracker step runs in its wave's window
            k, n = self._wave[-1]
            self._dl[(k, n - 1)] = (rows, counts, stats, rows_per_stream)
            return
        st = self.trk_stream if self.pipelined else torch.cuda.current_stream(self.device)
        self.tracker.download_async(rows, counts, stats, rows_per_stream, stream=st.cuda_stream)

    def download(self):
        """Tracker results of the most recent step (rows, counts, stats; host arrays).  Waits for
        the tracker stream first, so it is safe while steps are pipelined."""
        self.flush()
        if self.pipelined:
            torch.cuda.current_stream(self.device).wait_stream(self.trk_stream)
        return self.tracker.download()

    def stats(self):
        self.sync()
        _, counts, stats = self.tracker.download()
        return counts.copy(), stats.copy()

    def flops_per_frame(self) -> int:
        return int(sum(self.prog.op_flops(1)))
