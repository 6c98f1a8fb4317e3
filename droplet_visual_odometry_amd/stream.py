"""Batched frame stream on the GPU: the whole per-pair path of
VisualOdometry.visual_odometry_calculations (visual_odometry_v3.py:384-408) for
many device-resident frames per call.

A call with n frames runs ORB on every frame once, matches each consecutive
pair, runs findEssentialMat(RANSAC) + recoverPose per pair and writes n-1
256-byte pair records (PAIR_RECORD_DTYPE) to device memory.  Torch tensors are
only containers for device memory; all compute is in libdvo_hip.so.
"""
from __future__ import annotations

import collections
import contextlib
import ctypes

import numpy as np
import torch

from ._native import (DMATCH_DTYPE, KEYPOINT_DTYPE, PAIR_RECORD_DTYPE, Context, StreamConfig, _vp, orb_params, ptr)


class FrameStream:
    def __init__(self, width: int, height: int, K, nfeatures: int = 500, max_frames: int = 64, prob: float = 0.999,
                 threshold: float = 1.0, max_iters: int = 1000, cross_check: int | None = None,
                 dist_thresh: float = 50.0, device: int | None = None, ctx: Context | None = None, opencv="4.x"):
        """opencv: the OpenCV version whose semantics the path reproduces, "4.x"
        (default) or "3.2" (ORB pyramid / retainBest, and cross_check defaults
        to the 3.x reverse pass); see include/dvo.h DVO_OPENCV_*."""
        from ._native import opencv_semantics
        sem = opencv_semantics(opencv)
        if cross_check is None:
            cross_check = 2 if sem == 1 else 1
        if ctx is not None and device is not None and device != ctx.device:
            raise ValueError(f"device {device} != context device {ctx.device}")
        self.ctx = ctx if ctx is not None else Context(0 if device is None else device)
        self.device = torch.device("cuda", self.ctx.device)  # the library runs on the context's device
        cfg = StreamConfig()
        cfg.width, cfg.height, cfg.max_frames = int(width), int(height), int(max_frames)
        cfg.orb = orb_params(nfeatures=nfeatures, opencv=opencv)
        K = np.asarray(K, np.float64).reshape(9)
        for i in range(9):
            cfg.K[i] = float(K[i])
        cfg.prob, cfg.threshold, cfg.max_iters = float(prob), float(threshold), int(max_iters)
        cfg.cross_check, cfg.dist_thresh = int(cross_check), float(dist_thresh)
        h = _vp()
        self.ctx.check(self.ctx.lib.dvo_stream_create(self.ctx.h, ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h
        self._ext = torch.cuda.ExternalStream(self.hip_stream, device=self.device)
        self._held = collections.deque()  # (event, tensors) in flight on the library's stream
        # The last process() call's frames and records: the library keeps raw pointers to both
        # (dvo_stream_pose_tail reads the records, get_pyramid(blurred) re-reads level 0 of the
        # frames), so they stay referenced until the next process() or close(), whatever the
        # caller keeps and whether or not sync() has drained _held.
        self._last = ()
        self._pending = {}  # records of submitted, not yet retired batches (by device address)
        self.width, self.height, self.max_frames, self.nfeatures = width, height, max_frames, nfeatures
        self.K = K.reshape(3, 3)

    @property
    def hip_stream(self) -> int:
        return self.ctx.lib.dvo_stream_hip_stream(self.h) or 0

    def new_records(self, n_pairs: int) -> torch.Tensor:
        return torch.zeros(max(n_pairs, 1) * PAIR_RECORD_DTYPE.itemsize, dtype=torch.uint8, device=self.device)

    def process(self, frames: torch.Tensor, records: torch.Tensor | None = None, wait_torch: bool = True,
                undistort=None) -> torch.Tensor:
        """Enqueue the batch on the stream's HIP stream (asynchronous).  With
        wait_torch the batch is ordered after work queued on torch's current
        stream (the frames' producer); pass False for frames already resident."""
        if frames.dtype != torch.uint8 or frames.dim() != 3 or not frames.is_cuda:
            raise ValueError("frames must be a uint8 [n, H, W] device tensor")
        n, h, w = frames.shape
        if (h, w) != (self.height, self.width):
            raise ValueError(f"frame size {w}x{h} != stream {self.width}x{self.height}")
        if frames.stride(2) != 1 or frames.stride(1) < w:
            raise ValueError("frames rows must be contiguous")
        if records is None:
            records = self.new_records(n - 1)
            wait_torch = True  # the zero-fill runs on torch's stream: order the library's writes after it
        if wait_torch:
            self._after_torch()
        if n > 1:
            self._pending[records.data_ptr()] = records
        if undistort is not None:  # ops.Undistorter: frames are remapped into the stream's slab first
            self.ctx.check(self.ctx.lib.dvo_stream_process_undistorted(
                self.h, undistort.h_, frames.data_ptr(), n, frames.stride(0), frames.stride(1),
                records.data_ptr() if n > 1 else None))
        else:
            self.ctx.check(self.ctx.lib.dvo_stream_process(self.h, frames.data_ptr(), n, frames.stride(0),
                                                           frames.stride(1), records.data_ptr() if n > 1 else None))
        self._take_retired()  # this batch, and any submitted before it (drained)
        self._last = (frames, records)
        self._hold(frames, records)
        return records

    def process_pairs(self, frames: torch.Tensor, records: torch.Tensor | None = None,
                      wait_torch: bool = True) -> torch.Tensor:
        """The reference's schedule (dvo_stream_process_pairs): frames holds 2n
        frames and pair p is frames 2p, 2p+1, each detected on its own, as
        visual_odometry_calculations re-detects both frames of every pair
        (visual_odometry_v3.py:387-392).  Records / pose tail as process()."""
        if frames.dtype != torch.uint8 or frames.dim() != 3 or not frames.is_cuda:
            raise ValueError("frames must be a uint8 [2n, H, W] device tensor")
        n2, h, w = frames.shape
        if (h, w) != (self.height, self.width):
            raise ValueError(f"frame size {w}x{h} != stream {self.width}x{self.height}")
        if n2 % 2 or n2 == 0:
            raise ValueError("frames must hold an even, non-zero number of frames (pairs 2p, 2p+1)")
        if frames.stride(2) != 1 or frames.stride(1) < w:
            raise ValueError("frames rows must be contiguous")
        if records is None:
            records = self.new_records(n2 // 2)
            wait_torch = True
        if wait_torch:
            self._after_torch()
        self._pending[records.data_ptr()] = records
        self.ctx.check(self.ctx.lib.dvo_stream_process_pairs(self.h, frames.data_ptr(), n2 // 2, frames.stride(0),
                                                             frames.stride(1), records.data_ptr()))
        self._take_retired()
        self._last = (frames, records)
        self._hold(frames, records)
        return records

    # ---- pipelined batches (dvo_stream_submit): see include/dvo.h ------------------------------
    @staticmethod
    def pipeline_depth() -> int:
        from ._native import load_library
        return int(load_library().dvo_pipeline_depth())

    def _check_frames(self, frames, pairs_layout=False):
        if frames.dtype != torch.uint8 or frames.dim() != 3 or not frames.is_cuda:
            raise ValueError("frames must be a uint8 [n, H, W] device tensor")
        n, h, w = frames.shape
        if (h, w) != (self.height, self.width):
            raise ValueError(f"frame size {w}x{h} != stream {self.width}x{self.height}")
        if frames.stride(2) != 1 or frames.stride(1) < w:
            raise ValueError("frames rows must be contiguous")
        if pairs_layout and (n % 2 or n == 0):
            raise ValueError("frames must hold an even, non-zero number of frames (pairs 2p, 2p+1)")
        return n

    def submit(self, frames: torch.Tensor, records: torch.Tensor, wait_torch: bool = True) -> list:
        """Pipelined batch (dvo_stream_submit): detection and matching of these
        frames, then one merged RANSAC round of the pending batches.  `records`
        (n - 1 records) is complete once the batch retires, pipeline_depth() - 1
        submits later or at drain(); it is kept referenced until then.  Returns
        the batches this call retired, oldest first, as (records, pairs)."""
        n = self._check_frames(frames)
        if n < 2:
            raise ValueError("a submitted batch needs >= 2 frames")
        if records.numel() < (n - 1) * PAIR_RECORD_DTYPE.itemsize:
            raise ValueError("records too small")
        if wait_torch:
            self._after_torch()
        self.ctx.check(self.ctx.lib.dvo_stream_submit(self.h, frames.data_ptr(), n, frames.stride(0),
                                                      frames.stride(1), records.data_ptr()))
        self._pending[records.data_ptr()] = records
        self._hold(frames, records)
        return self._take_retired()

    def submit_pairs(self, frames: torch.Tensor, records: torch.Tensor, wait_torch: bool = True) -> list:
        """submit() with the reference's schedule (pair p = frames 2p, 2p+1; process_pairs)."""
        n2 = self._check_frames(frames, pairs_layout=True)
        if records.numel() < (n2 // 2) * PAIR_RECORD_DTYPE.itemsize:
            raise ValueError("records too small")
        if wait_torch:
            self._after_torch()
        self.ctx.check(self.ctx.lib.dvo_stream_submit_pairs(self.h, frames.data_ptr(), n2 // 2, frames.stride(0),
                                                            frames.stride(1), records.data_ptr()))
        self._pending[records.data_ptr()] = records
        self._hold(frames, records)
        return self._take_retired()

    def drain(self) -> list:
        """Run the pending batches' remaining rounds and retire them (oldest first)."""
        self.ctx.check(self.ctx.lib.dvo_stream_drain(self.h))
        return self._take_retired()

    def _take_retired(self) -> list:
        from ._native import _vp
        cap = 16
        recs = (_vp * cap)()
        pairs = (ctypes.c_int * cap)()
        n = self.ctx.lib.dvo_stream_retired(self.h, recs, pairs, cap)
        out = []
        for i in range(min(n, cap)):
            t = self._pending.pop(recs[i], None)
            if t is None:
                raise RuntimeError("retired records that were not submitted through this FrameStream")
            out.append((t, int(pairs[i])))
        if out:
            # the retire kernels (records_kernel) writing these records are queued on the library's
            # stream by the call that retired them: keep the tensors alive until they have run,
            # whether or not the caller keeps the returned list (process() drops it)
            self._hold(*[t for t, _ in out])
        return out

    def pose_tail_batch(self, records: torch.Tensor, pairs: int, corners_prev: torch.Tensor,
                        corners_cur: torch.Tensor, marker_length: float, T_rel: torch.Tensor,
                        T_abs: torch.Tensor, wait_torch: bool = False):
        """Device pose tail over a retired batch's records (dvo_stream_pose_tail_batch), on this
        stream's carry (shared with share_pose)."""
        k = corners_prev.shape[1]
        if corners_prev.shape[0] < pairs or corners_cur.shape[0] < pairs or T_rel.shape[0] < pairs \
                or T_abs.shape[0] < pairs:
            raise ValueError("corners / outputs hold fewer pairs than the batch")
        if wait_torch:
            self._after_torch()
        self.ctx.check(self.ctx.lib.dvo_stream_pose_tail_batch(
            self.h, records.data_ptr(), int(pairs), corners_prev.data_ptr(), corners_cur.data_ptr(), k,
            float(marker_length), T_rel.data_ptr(), T_abs.data_ptr()))
        self._hold(records, corners_prev, corners_cur, T_rel, T_abs)
        return T_rel, T_abs

    def _hold(self, *tensors):
        """Keep the tensors the library's stream reads or writes alive until that
        work has finished, so torch's caching allocator cannot hand their blocks
        to a new tensor meanwhile.  (Not record_stream: the allocator would then
        record events on this stream after close() destroyed it.)"""
        ev = torch.cuda.Event()
        ev.record(self._ext)
        self._held.append((ev, tensors))
        while self._held and self._held[0][0].query():
            self._held.popleft()

    def _after_torch(self):
        """Order the library's HIP stream after work already queued on torch's
        current stream (frames / corners produced by torch)."""
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._ext.wait_event(ev)

    def record_event(self) -> torch.cuda.Event:
        """An event on the library's stream after everything enqueued so far."""
        ev = torch.cuda.Event()
        ev.record(self._ext)
        return ev

    def wait_event(self, ev):
        """Order the library's HIP stream after a torch.cuda.Event (e.g. the
        all-gather that last read this stream's records buffer)."""
        if ev is not None:
            self._ext.wait_event(ev)

    def share_pose(self, owner: "FrameStream"):
        """Chain this stream's pose tails on `owner`'s carry (batches alternating
        between streams form one pose stream)."""
        self.ctx.check(self.ctx.lib.dvo_stream_share_pose(self.h, owner.h))

    def reset_pose(self, P0=None, T0=None):
        """Carry-in of the pose tail: P_prev (3x4, default K[I|0] as in controlled
        mode, v3:164-166) and the absolute pose (4x4, default identity)."""
        P0 = self.K @ np.hstack((np.eye(3), np.zeros((3, 1)))) if P0 is None else np.asarray(P0, np.float64)
        T0 = np.eye(4) if T0 is None else np.asarray(T0, np.float64)
        self.ctx.check(self.ctx.lib.dvo_stream_reset_pose(self.h, ptr(np.ascontiguousarray(P0)),
                                                          ptr(np.ascontiguousarray(T0))))

    def pose_tail(self, corners_prev: torch.Tensor, corners_cur: torch.Tensor, marker_length: float,
                  T_rel: torch.Tensor | None = None, T_abs: torch.Tensor | None = None, wait_torch: bool = True):
        """Device pose tail for the last processed batch (see dvo.h); corners are
        float64 [pairs, k, 2] device tensors.  Returns (T_rel, T_abs) [pairs, 4, 4]."""
        pairs, k = corners_prev.shape[0], corners_prev.shape[1]
        if T_rel is None or T_abs is None:
            # blocks fresh from torch's stream may still be in use by work queued there
            wait_torch = True
        if T_rel is None:
            T_rel = torch.empty((pairs, 4, 4), dtype=torch.float64, device=self.device)
        if T_abs is None:
            T_abs = torch.empty((pairs, 4, 4), dtype=torch.float64, device=self.device)
        if wait_torch:
            self._after_torch()
        self.ctx.check(self.ctx.lib.dvo_stream_pose_tail(self.h, corners_prev.data_ptr(), corners_cur.data_ptr(), k,
                                                         float(marker_length), T_rel.data_ptr(), T_abs.data_ptr()))
        self._hold(corners_prev, corners_cur, T_rel, T_abs, *self._last)
        return T_rel, T_abs

    def set_profiling(self, enable: bool = True):
        self.ctx.check(self.ctx.lib.dvo_stream_set_profiling(self.h, int(enable)))

    def stage_times(self):
        """{stage: accumulated device ms} over calls since set_profiling(True), plus call count."""
        from ._native import DVO_NSTAGES, STAGE_NAMES
        ms = np.zeros(DVO_NSTAGES, np.float64)
        calls = ctypes.c_int()
        self.ctx.check(self.ctx.lib.dvo_stream_stage_times(self.h, ptr(ms), ctypes.byref(calls)))
        return dict(zip(STAGE_NAMES, ms.tolist())), calls.value

    def sync(self):
        self.ctx.check(self.ctx.lib.dvo_stream_sync(self.h))
        self._held.clear()

    @staticmethod
    def records_numpy(records: torch.Tensor, n_pairs: int) -> np.ndarray:
        raw = records[: n_pairs * PAIR_RECORD_DTYPE.itemsize].cpu().numpy()
        return raw.view(PAIR_RECORD_DTYPE).copy()

    def features(self, frame: int):
        cap = self.nfeatures + 1024
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = ctypes.c_int()
        self.ctx.check(self.ctx.lib.dvo_stream_get_features(self.h, frame, ptr(kps), ptr(desc), cap, ctypes.byref(n)))
        return kps[:n.value].copy(), desc[:n.value].copy()

    def matches(self, pair: int) -> np.ndarray:
        cap = self.nfeatures + 1024
        out = np.zeros(cap, DMATCH_DTYPE)
        m = ctypes.c_int()
        self.ctx.check(self.ctx.lib.dvo_stream_get_matches(self.h, pair, ptr(out), cap, ctypes.byref(m)))
        return out[:m.value].copy()

    def pyramid(self, frame: int, level: int, blurred: bool = False) -> np.ndarray:
        from .plan import level_sizes
        lw, lh = level_sizes(self.width, self.height)[level]
        out = np.zeros(lw * lh, np.uint8)
        self.ctx.check(self.ctx.lib.dvo_stream_get_pyramid(self.h, frame, level, int(blurred), ptr(out), out.size))
        return out.reshape(lh, lw)

    def close(self):
        if getattr(self, "h", None):
            self.ctx.lib.dvo_stream_destroy(self.h)  # synchronises the stream first
            self.h = None
            if getattr(self, "_held", None):
                self._held.clear()
            self._last = ()
            self._pending = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_side_streams = {}


@contextlib.contextmanager
def ordered_side_stream(device):
    """A HIP stream handle for a library call that must behave as if it ran on
    torch's current stream.  The C API reads a NULL stream as "the context's
    stream" (non-blocking, unordered with torch's default stream), so calls
    are made on a per-device side stream that waits for torch's current stream
    before the call, and that torch's current stream waits for after it."""
    cur = torch.cuda.current_stream(device)
    side = _side_streams.get(device)
    if side is None:
        side = _side_streams[device] = torch.cuda.Stream(device)
    side.wait_stream(cur)
    yield side.cuda_stream
    cur.wait_stream(side)


class PoseChain:
    """Absolute-pose chain T_abs[p] = T_abs[p-1] . T_rel[p] (v3:367) on the
    device (dvo_pose_chain) with a persistent carry: the reassembly step of a
    sharded pose stream (dist.ShardedPoseStream).  Runs on torch's current
    stream, where the all-gather that produced T_rel ran (ordered_side_stream)."""

    def __init__(self, ctx: Context | None = None, device: int | None = None, T0=None):
        self.ctx = ctx if ctx is not None else Context(0 if device is None else device)
        self.device = torch.device("cuda", self.ctx.device)
        self.carry = torch.empty(16, dtype=torch.float64, device=self.device)
        self.reset(T0)

    def reset(self, T0=None):
        T0 = np.eye(4) if T0 is None else np.asarray(T0, np.float64)
        self.carry.copy_(torch.from_numpy(np.ascontiguousarray(T0).reshape(16)))

    def run(self, T_rel: torch.Tensor, T_abs: torch.Tensor | None = None) -> torch.Tensor:
        if T_rel.dtype != torch.float64 or not T_rel.is_cuda or not T_rel.is_contiguous():
            raise ValueError("T_rel must be a contiguous float64 [n, 4, 4] device tensor")
        n = T_rel.shape[0]
        if T_abs is None:
            T_abs = torch.empty((n, 4, 4), dtype=torch.float64, device=self.device)
        if T_abs.shape[0] < n or not T_abs.is_contiguous():
            raise ValueError("T_abs must be a contiguous float64 [>= n, 4, 4] device tensor")
        with ordered_side_stream(self.device) as st:
            self.ctx.check(self.ctx.lib.dvo_pose_chain(self.ctx.h, T_rel.data_ptr(), n, self.carry.data_ptr(),
                                                       T_abs.data_ptr(), st))
        return T_abs



class HostPoseChain:
    """The absolute chain T_abs[p] = T_abs[p-1] . T_rel[p] (v3:367) on a host thread
    (dvo_pose_chain_host, the device kernel's arithmetic bit for bit): rank 0 of a sharded stream
    (dist.ShardedStreamRunner).  submit(T_rel) copies the device T_rel into a pinned slot on
    torch's current stream and returns a Future of the window's T_abs (host, [n, 4, 4] float64);
    one worker thread chains the windows in submission order, waiting for each copy's event, while
    the GPU goes on with the next batches.  The carry (16 doubles) continues across windows."""

    def __init__(self, max_pairs: int, slots: int, device, T0=None):
        import concurrent.futures
        from ._native import load_library
        self.lib = load_library()
        self.device = torch.device(device)
        self.carry = np.ascontiguousarray(np.eye(4) if T0 is None else np.asarray(T0, np.float64)).reshape(16).copy()
        self.pinned = [torch.empty((max_pairs, 4, 4), dtype=torch.float64, pin_memory=True) for _ in range(slots)]
        self.pending = [None] * slots
        self.n = 0
        self.pool = concurrent.futures.ThreadPoolExecutor(max_workers=1)

    def reset(self, T0=None):
        """The absolute pose before the next submitted window (default identity); waits for the
        windows already submitted, which chain on the old carry."""
        self.wait()
        self.carry[:] = np.asarray(np.eye(4) if T0 is None else T0, np.float64).reshape(16)

    def submit(self, T_rel: torch.Tensor):
        n = T_rel.shape[0]
        k = self.n % len(self.pinned)
        self.n += 1
        if self.pending[k] is not None:
            self.pending[k].result()  # the slot's previous chain has read its pinned buffer
        buf = self.pinned[k]
        buf[:n].copy_(T_rel, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))

        def work():
            ev.synchronize()
            out = np.empty((n, 4, 4), np.float64)
            src = buf[:n].numpy()
            rc = self.lib.dvo_pose_chain_host(src.ctypes.data, n, self.carry.ctypes.data, out.ctypes.data)
            if rc != 0:
                raise RuntimeError(f"dvo_pose_chain_host failed ({rc})")
            return out

        fut = self.pool.submit(work)
        self.pending[k] = fut
        return fut

    def wait(self):
        """Block until every submitted window is chained (raises a chain's error)."""
        for f in self.pending:
            if f is not None:
                f.result()

    def close(self):
        self.pool.shutdown(wait=True)


class PoseTail:
    """Pose tail over pair records (dvo_pose_tail_records): the marker-scaled
    relative poses (v3:309-345) and the absolute chain (v3:367) for records
    that arrive from elsewhere -- the reassembly step of a sharded pose stream
    (dist.ShardedPoseStream), run by rank 0 over the whole window in pair order.
    Same kernels and record fields as FrameStream.pose_tail, so the result is
    bit-identical to one rank's stream.  The carry (P_prev | T_abs) persists
    across calls on the device.  Runs on torch's current stream, where the
    all-gather that produced the records ran (ordered_side_stream)."""

    def __init__(self, K, marker_length: float, ctx: Context | None = None, device: int | None = None):
        self.ctx = ctx if ctx is not None else Context(0 if device is None else device)
        self.device = torch.device("cuda", self.ctx.device)
        self.K = np.ascontiguousarray(np.asarray(K, np.float64).reshape(3, 3))
        self.marker_length = float(marker_length)
        self.carry = torch.empty(28, dtype=torch.float64, device=self.device)
        self.reset()

    def reset(self, P0=None, T0=None):
        """P_prev (3x4, default K[I|0] as in controlled mode, v3:164-166) and the
        absolute pose (4x4, default identity) before the next record."""
        P0 = self.K @ np.hstack((np.eye(3), np.zeros((3, 1)))) if P0 is None else np.asarray(P0, np.float64)
        T0 = np.eye(4) if T0 is None else np.asarray(T0, np.float64)
        c = np.concatenate([np.asarray(P0, np.float64).reshape(12), np.asarray(T0, np.float64).reshape(16)])
        self.carry.copy_(torch.from_numpy(c))

    def run(self, records: torch.Tensor, corners_prev: torch.Tensor, corners_cur: torch.Tensor,
            T_rel: torch.Tensor | None = None, T_abs: torch.Tensor | None = None):
        """records: uint8 device tensor of n x 256 B; corners: float64 [n, k, 2]
        device tensors.  Returns (T_rel, T_abs) [n, 4, 4]."""
        rb = PAIR_RECORD_DTYPE.itemsize
        if records.dtype != torch.uint8 or not records.is_cuda or not records.is_contiguous() or records.numel() % rb:
            raise ValueError("records must be a contiguous uint8 device tensor of whole 256-B records")
        n = records.numel() // rb
        for c in (corners_prev, corners_cur):
            if c.dtype != torch.float64 or not c.is_cuda or not c.is_contiguous() or c.dim() != 3 \
                    or c.shape[0] != n or c.shape[2] != 2:
                raise ValueError(f"corners must be contiguous float64 [{n}, k, 2] device tensors")
        k = corners_prev.shape[1]
        if corners_cur.shape[1] != k:
            raise ValueError("previous and current corners differ in k")
        if T_rel is None:
            T_rel = torch.empty((n, 4, 4), dtype=torch.float64, device=self.device)
        if T_abs is None:
            T_abs = torch.empty((n, 4, 4), dtype=torch.float64, device=self.device)
        for T in (T_rel, T_abs):
            if T.dtype != torch.float64 or not T.is_contiguous() or T.shape[0] < n:
                raise ValueError(f"T_rel / T_abs must be contiguous float64 [>= {n}, 4, 4] device tensors")
        with ordered_side_stream(self.device) as st:
            self.ctx.check(self.ctx.lib.dvo_pose_tail_records(
                self.ctx.h, records.data_ptr(), n, ptr(self.K), corners_prev.data_ptr(), corners_cur.data_ptr(), k,
                self.marker_length, self.carry.data_ptr(), T_rel.data_ptr(), T_abs.data_ptr(), st))
        return T_rel, T_abs

    def rel_range(self, records: torch.Tensor, corners_prev: torch.Tensor, corners_cur: torch.Tensor, p0: int,
                  n: int, T_rel: torch.Tensor) -> torch.Tensor:
        """The pair-parallel half over pairs [p0, p0 + n) of a gathered window (dvo_pose_rel_range):
        T_rel[0 .. n), then the P_prev carry advanced past the whole window.  Every rank of a sharded
        stream runs it over its own pairs; rank 0 chains the gathered T_rel with chain()."""
        rb = PAIR_RECORD_DTYPE.itemsize
        pairs = records.numel() // rb
        k = corners_prev.shape[1]
        if corners_prev.shape[0] != pairs or corners_cur.shape[0] != pairs:
            raise ValueError("corners must cover the window's pairs")
        if T_rel.shape[0] < n or not T_rel.is_contiguous() or T_rel.dtype != torch.float64:
            raise ValueError("T_rel must be a contiguous float64 [>= n, 4, 4] device tensor")
        with ordered_side_stream(self.device) as st:
            self.ctx.check(self.ctx.lib.dvo_pose_rel_range(
                self.ctx.h, records.data_ptr(), pairs, int(p0), int(n), ptr(self.K), corners_prev.data_ptr(),
                corners_cur.data_ptr(), k, self.marker_length, self.carry.data_ptr(), T_rel.data_ptr(), st))
        return T_rel

    def chain(self, T_rel: torch.Tensor, T_abs: torch.Tensor, detached: bool = False) -> torch.Tensor:
        """The serial absolute chain (dvo_pose_chain) on this tail's T_abs carry.  detached: on the
        tail's own chain stream, after the work queued on torch's current stream so far, WITHOUT
        ordering torch's stream after it -- the chain (one wave's dependency chain over the
        window) then stays off the path of the next collectives; chains still run in call
        order.  Read T_abs after torch.cuda.synchronize() (or chain_event())."""
        n = T_rel.shape[0]
        if not detached:
            with ordered_side_stream(self.device) as st:
                self.ctx.check(self.ctx.lib.dvo_pose_chain(self.ctx.h, T_rel.data_ptr(), n,
                                                           self.carry.data_ptr() + 12 * 8, T_abs.data_ptr(), st))
            return T_abs
        if getattr(self, "_chain_stream", None) is None:
            self._chain_stream = torch.cuda.Stream(self.device)
        cs = self._chain_stream
        cs.wait_stream(torch.cuda.current_stream(self.device))
        self.ctx.check(self.ctx.lib.dvo_pose_chain(self.ctx.h, T_rel.data_ptr(), n, self.carry.data_ptr() + 12 * 8,
                                                   T_abs.data_ptr(), cs.cuda_stream))
        T_rel.record_stream(cs)  # torch's allocator keeps T_rel / T_abs until the chain has read / written them
        T_abs.record_stream(cs)
        return T_abs

    def chain_event(self):
        """An event after the detached chains queued so far (None if there were none)."""
        cs = getattr(self, "_chain_stream", None)
        if cs is None:
            return None
        ev = torch.cuda.Event()
        ev.record(cs)
        return ev
