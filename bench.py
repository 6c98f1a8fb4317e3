#!/usr/bin/env python3
"""Benchmark: frames/sec of the visual-odometry front end (detect + match + pose).

Workload (BASELINE.json metric / configs[2]): a synthetic 1280x720 mono8
stream, 2000 ORB features, one MI355X per rank.  One "step" is one batch of B
new frames: the GPU runs ORB on B+1 device-resident frames (the first is the
previous batch's last frame), Hamming cross-check matching, findEssentialMat
(RANSAC, 5-point), recoverPose and the marker-scaled pose tail (triangulated
marker corners -> scale -> 4x4 relative pose -> chained absolute pose) for the B
consecutive pairs, and with N > 1 ranks all-gathers the B pair records over
RCCL (the pose stream reassembly of SURVEY.md §8e).  value = (B x steps x ranks) / max-over-ranks wall time.

Also reported:
  roofline      the dominant kernel group's algorithmic bytes / its HIP-event
                time on the library's stream, against 8 TB/s HBM
  cpu_baseline  the oracle (C++ restatement of the OpenCV path) on one host
                core over a bounded sample of the same stream (rank 0, N=1)

Run: python bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
PMC_TRAFFIC = "r01i_pmc_traffic.json"  # tools/profile_round.sh: FETCH_SIZE / WRITE_SIZE passes of the current kernels


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--batch", type=int, default=1024, help="new frames per step (pairs per step)")
    ap.add_argument("--max-iters", type=int, default=1000)
    ap.add_argument("--pool", type=int, default=0, help="distinct frames rendered per rank (default 2*batch+1)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-stage HIP-event timing")
    ap.add_argument("--streams", type=int, default=2,
                    help="batches in flight: each on its own dvo_stream / HIP stream, so one batch's "
                         "serial RANSAC tail overlaps the next batch's ORB")
    return ap.parse_args()


def stage_bytes(w, h, nfeatures, n_matches):
    """Algorithmic HBM bytes per frame for each kernel group."""
    from droplet_visual_odometry_amd.plan import level_sizes
    L = level_sizes(w, h)
    px = [a * b for a, b in L]
    n = nfeatures
    return {
        "pyramid": float(sum(px[l - 1] + px[l] for l in range(1, 8))),  # read l-1, write l
        "blur": float(2 * sum(px)),                                    # read + write every level
        "fast": float(sum(px)),                                        # read every level once
        "select_harris": float(8 * 2 * n + 81 * 2 * n),                 # keys + 9x9 Harris windows
        "describe": float(n * (749 + 512 + 28 + 32)),                  # angle disc + pattern + kp + desc
        "match": float(2 * 2 * n * 32 + 16 * n_matches),               # both directions read both sets
        "ransac": float(32 * n_matches),                               # normalised correspondences
        "recover_pose": float(32 * n_matches + 256),
        "pose_tail": float(96 + 16 + 2 * 64 + 2 * 128),                  # R|t, info, corners, T_rel + T_abs
    }


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # DVO_BENCH_BACKEND=gloo: rehearsal of the multi-rank path on fewer GPUs than
    # ranks (ranks share devices, records are gathered through host memory).
    backend = os.environ.get("DVO_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local_rank = local_rank % torch.cuda.device_count()
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        if backend == "gloo":
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)

    from droplet_visual_odometry_amd._native import Context, PAIR_RECORD_DTYPE
    from droplet_visual_odometry_amd.plan import algorithmic_bytes_per_frame
    from droplet_visual_odometry_amd.stream import FrameStream
    from droplet_visual_odometry_amd.synth import SceneStream

    W, H, N, B = args.width, args.height, args.nfeatures, args.batch
    scene = SceneStream(W, H, device=str(dev))
    pool_n = args.pool or (2 * B + 1)
    base = rank * 100_000  # each rank owns a disjoint stretch of the stream (weak scaling)
    pool = torch.stack([scene.render(base + i) for i in range(pool_n)]).contiguous()
    torch.cuda.synchronize()

    ctx = Context(local_rank)
    S = max(1, args.streams)
    fss = [FrameStream(W, H, scene.K, nfeatures=N, max_frames=B + 1, max_iters=args.max_iters, ctx=ctx)
           for _ in range(S)]
    for f in fss[1:]:
        f.share_pose(fss[0])  # one pose stream across the alternating batches
    recs_t = [f.new_records(B) for f in fss]
    from droplet_visual_odometry_amd.synth import MARKER_LEN
    corners = torch.tensor(np.stack([scene.marker_corners(base + i) for i in range(pool_n)]), dtype=torch.float64,
                           device=dev)
    T_rel = [torch.empty((B, 4, 4), dtype=torch.float64, device=dev) for _ in range(S)]
    T_abs = [torch.empty((B, 4, 4), dtype=torch.float64, device=dev) for _ in range(S)]
    fss[0].reset_pose()
    torch.cuda.synchronize()
    gdev = torch.device("cpu") if backend == "gloo" else dev
    gathered = [torch.empty(world * recs_t[0].numel(), dtype=torch.uint8, device=gdev) for _ in range(S)] \
        if world > 1 else None
    n_windows = max(1, (pool_n - 1) // B)

    def step(i):
        s = (i % n_windows) * B
        k = i % S
        fs = fss[k]
        fs.process(pool[s:s + B + 1], recs_t[k], wait_torch=False)
        fs.pose_tail(corners[s:s + B], corners[s + 1:s + B + 1], MARKER_LEN, T_rel[k], T_abs[k], wait_torch=False)
        if world > 1:
            if backend == "gloo":
                fs.sync()
                dist.all_gather_into_tensor(gathered[k], recs_t[k].cpu())
            else:
                # RCCL (on torch's stream) reads the records once the library's stream has written them
                torch.cuda.current_stream().wait_event(fs.record_event())
                dist.all_gather_into_tensor(gathered[k], recs_t[k])

    def sync_all():
        for f in fss:
            f.sync()
        torch.cuda.synchronize()

    for i in range(args.warmup):
        step(i)
    sync_all()
    if not args.no_profile:
        for f in fss:
            f.set_profiling(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    sync_all()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=gdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    recs = FrameStream.records_numpy(recs_t[(args.warmup + args.steps - 1) % S], B)
    stage_ms, calls = {}, 0
    if not args.no_profile:
        for f in fss:
            sm, c = f.stage_times()
            calls += c
            for kk, v in sm.items():
                stage_ms[kk] = stage_ms.get(kk, 0.0) + v
    frames_total = B * args.steps * world
    value = frames_total / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    m_avg = float(np.mean(recs["n_matches"])) if len(recs) else N / 2
    ok = int(np.sum(recs["status"] == 0))
    roofline = None
    if stage_ms and calls:
        sb = stage_bytes(W, H, N, m_avg)
        per_call = {k: v / calls for k, v in stage_ms.items()}
        # roofline of the dominant single-kernel stage (one launch per step, so the
        # HIP-event time on the library's stream is that kernel's duration)
        single = {"fast": "fast_strip_kernel", "blur": "blur_kernel", "describe": "describe_kernel"}
        dom = max(single, key=lambda k: per_call.get(k, 0.0))
        bytes_per_launch = sb[dom] * (B + 1)
        achieved = bytes_per_launch / (per_call[dom] * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(single[dom], W, H, N, B)
        roofline = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic, "traffic_source": traffic_src,
                    "kernel": single[dom], "algorithmic_bytes_per_launch": bytes_per_launch,
                    "kernel_ms_per_launch": round(per_call[dom], 4),
                    "stage_ms_per_step": {k: round(v, 4) for k, v in per_call.items()},
                    "path_algorithmic_bytes_per_frame": algorithmic_bytes_per_frame(W, H, N, m_avg),
                    "path_frac": round(value / world * algorithmic_bytes_per_frame(W, H, N, m_avg) / 1e9
                                       / HBM_PEAK_GBS, 8)}

    cpu = None
    pose_check = None
    if args.cpu_seconds > 0 and world == 1:
        cpu, ref = cpu_baseline(pool, scene.K, N, args.max_iters, args.cpu_seconds)
        # the same pairs on the GPU (window 0), compared with the oracle's R, t
        fss[0].process(pool[0:B + 1], recs_t[0], wait_torch=False)
        fss[0].sync()
        g = FrameStream.records_numpy(recs_t[0], B)
        n = min(len(ref), B)
        ident = 0
        err_r = err_t = 0.0
        for i in range(n):
            R_ref, t_ref = ref[i]
            if R_ref is None:
                ident += int(g["status"][i] != 0)
                continue
            Rg, tg = g["R"][i].reshape(3, 3), g["t"][i]
            ident += int(np.array_equal(Rg, R_ref) and np.array_equal(tg, t_ref.ravel()))
            err_r = max(err_r, float(np.max(np.abs(Rg - R_ref))))
            err_t = max(err_t, float(np.max(np.abs(tg - t_ref.ravel()))))
        ate = chained_ate(fss[0], pool, corners, scene.K, ref, B)
        pose_check = {"pairs": n, "bit_identical": ident, "max_abs_R_err": err_r, "max_abs_t_err": err_t,
                      "ate_m": ate, "reference": "oracle/ C++ restatement, same frames; ATE = RMS position "
                                                 "difference of the marker-scaled chained trajectories"}

    default_cfg = (W, H, N) == (1280, 720, 2000)
    out = {
        "metric": ("frames/sec (detect+match+pose) at 1280\u00d7720, 2000 feats; ATE vs reference" if default_cfg
                   else f"frames/sec (detect+match+pose) at {W}\u00d7{H}, {N} feats; ATE vs reference"),
        "value": round(value, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/f32/f64",
        "data": "synthetic (seeded ray-cast textured room, droplet_visual_odometry_amd/synth.py)",
        "config": {"workload": f"{W}x{H} mono8 stream, {N} ORB features, batch {B} new frames/step per GPU",
                   "width": W, "height": H, "nfeatures": N, "batch_frames": B, "max_iters": args.max_iters,
                   "parallelism": f"frame-sharded x{world}" + (
                       (" + RCCL all_gather" if backend != "gloo" else " + gloo all_gather (rehearsal)")
                       if world > 1 else ""),
                   "streams_in_flight": S,
                   "pairs_ok": f"{ok}/{len(recs)}", "mean_matches": round(m_avg, 1),
                   "mean_ransac_iters": round(float(np.mean(recs['ransac_iters'])), 1) if len(recs) else 0},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "pose_check": pose_check,
    }
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def chained_ate(fs, pool, corners, K, ref, B):
    """RMS position difference between the device pose tail's chained
    trajectory and the oracle's (restated host tail) over the sampled pairs."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from droplet_visual_odometry_amd.synth import MARKER_LEN
    fs.reset_pose()
    fs.process(pool[0:B + 1])  # fresh records: zero-filled on torch's stream, so the library waits for it
    _, T_abs = fs.pose_tail(corners[0:B], corners[1:B + 1], MARKER_LEN)
    fs.sync()
    T_abs = T_abs.cpu().numpy()
    c = corners.cpu().numpy()
    P = K @ np.hstack((np.eye(3), np.zeros((3, 1))))
    T = np.eye(4)
    err = []
    for i, (R, t) in enumerate(ref[:B]):
        if R is None:
            break
        P, _, T = oracle.pose_tail(K, R, t, c[i], c[i + 1], MARKER_LEN, P, T)
        err.append(float(np.sum((T_abs[i][:3, 3] - T[:3, 3]) ** 2)))
    return float(np.sqrt(np.mean(err))) if err else None


def pmc_traffic(kernel, W, H, N, B):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (profiles/PMC_TRAFFIC: FETCH_SIZE + WRITE_SIZE), when they were
    taken on this configuration; PMC counters cannot run inside the timed loop."""
    path = os.path.join(ROOT, "profiles", PMC_TRAFFIC)
    try:
        doc = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    c = doc.get("config", {})
    k = doc.get("kernels", {}).get(kernel)
    if k is None or (c.get("width"), c.get("height"), c.get("nfeatures")) != (W, H, N) or not c.get("batch"):
        return None, None
    # one launch covers B + 1 frames: the counted bytes scale per frame from the profiled batch
    scale = (B + 1) / (c["batch"] + 1)
    src = f"profiles/{PMC_TRAFFIC} (rocprofv3 --pmc FETCH_SIZE, WRITE_SIZE at batch {c['batch']}"
    src += ")" if c["batch"] == B else f", scaled per frame to batch {B})"
    return round((k["fetch_bytes"] + k["write_bytes"]) * scale), src


def cpu_baseline(pool, K, nfeatures, max_iters, seconds):
    """The oracle (restated OpenCV path, -O2 C++, one core) on the same stream:
    sequential pairs with the previous frame's features reused (streaming mode)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.build()
    t0 = time.perf_counter()
    kp_prev = oracle.detect_and_compute(pool[0].cpu().numpy(), nfeatures)
    n = 0
    i = 0
    ref = []
    while time.perf_counter() - t0 < seconds and i + 1 < len(pool):
        a, b = pool[i].cpu().numpy(), pool[i + 1].cpu().numpy()
        r = oracle.pair_pose(a, b, K, nfeatures, max_iters=max_iters, kp_prev=kp_prev)
        kp_prev = (r["kp_cur"], r["desc_cur"])
        ref.append((r["R"], r["t_unit"]))
        n += 1
        i += 1
    dt = time.perf_counter() - t0
    return ({"value": round(n / dt, 3), "unit": "frames/s", "cores": 1, "kind": "port",
             "sample": f"{n} consecutive pairs of the same {pool.shape[2]}x{pool.shape[1]} stream ({dt:.1f} s, "
                       f"first frame's detect included), oracle/ C++ restatement of the OpenCV path, streaming "
                       f"mode, one host core"}, ref)


if __name__ == "__main__":
    main()
