#!/usr/bin/env python3
"""Benchmark: frames/sec of the visual-odometry front end (detect + match + pose).

Workload (BASELINE.json metric / configs[2]): a synthetic 1280x720 mono8
stream, 2000 ORB features, one MI355X per rank.  One "step" is one batch of B
new frames per rank: the GPU runs ORB on B+1 device-resident frames (the first
is the previous batch's last frame), Hamming cross-check matching,
findEssentialMat (RANSAC, 5-point), recoverPose and the marker-scaled pose tail
(triangulated marker corners -> scale -> 4x4 relative pose -> chained absolute
pose) for the B consecutive pairs.  With N > 1 ranks (configs[3]) ONE stream is
sharded: each rank takes B consecutive pairs of a window of N x B, the ranks
all-gather their pair records and marker corners over RCCL, and rank 0 runs the
window's marker-scaled pose tail and absolute chain (SURVEY.md §8e;
main_sharded).
value = (B x steps x ranks) / max-over-ranks wall time.

Also reported:
  roofline      the dominant kernel group's algorithmic bytes / its HIP-event
                time on the library's stream, against 8 TB/s HBM
  cpu_baseline  the oracle (C++ restatement of the OpenCV path, -O3
                -march=native) over bounded samples of the same stream on all
                host threads (value) and on one core (rank 0, N=1)

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
# VALU issue: a SIMD issues one wave64 VALU instruction per 2 cycles; 256 CUs x 4 SIMDs at 2.4 GHz
VALU_PEAK_WIPS = 256 * 4 * 2.4e9 / 2
PMC_TRAFFIC = "r03z_pmc_traffic.json"  # tools/profile_round.sh: calibrated FETCH/WRITE_SIZE + SQ passes of the kernels
# FP64 vector peak: 78.6 TFLOP/s, AMD's MI355X data-sheet figure (MI355X_MICROARCH.md lists no f64 row).  It is
# the wave64 f64 FMA issue rate: 16 lanes per cycle per SIMD (a wave64 f64 instruction per 4 cycles) x 2 FLOP x
# 1024 SIMDs x 2.4 GHz.
F64_PEAK_TFLOPS = 78.6
PMC_F64 = "r03z_pmc_f64.json"  # tools/pmc_stall_f64.sh + tools/pmc_f64.py: f64 VALU instructions per kernel


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--batch", type=int, default=2048,
                    help="new frames per step (pairs per step); two streams, 1280x720: 1024 68.7 K frames/s, "
                         "1536 70.3 K, 2048 71.0 K, 3072 72.2 K (profiles/r02r_batch_sweep.txt)")
    ap.add_argument("--max-iters", type=int, default=1000)
    ap.add_argument("--pool", type=int, default=0, help="distinct frames rendered per rank (default 2*batch+1)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--no-profile", action="store_true", help="skip the per-stage HIP-event timing")
    ap.add_argument("--host-trace", action="store_true", help="print host-side enqueue times per step to stderr")
    ap.add_argument("--dropin-seconds", type=float, default=4.0,
                    help="bounded timing of the per-pair drop-in surface (0 = skip)")
    ap.add_argument("--sharded", action="store_true",
                    help="take the sharded path (main_sharded) even at N=1: rehearses the RCCL exchange and its "
                         "stream ordering on one GPU")
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
        "blur": 0.0,                                                   # no separate pass: describe blurs its windows
        "fast": float(sum(px)),                                        # read every level once
        "select_harris": float(8 * 2 * n + 81 * 2 * n),                 # keys + 9x9 Harris windows
        "describe": float(n * (749 + 45 * 52 + 28 + 32)),              # angle disc + raw 45x52 window + kp + desc
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
    if world > 1 or args.sharded:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
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
    if world > 1 or args.sharded:
        return main_sharded(args, world, rank, local_rank, backend, dev, scene)
    pool_n = args.pool or (2 * B + 1)
    pool = torch.stack([scene.render(i) for i in range(pool_n)]).contiguous()
    torch.cuda.synchronize()

    ctx = Context(local_rank)
    S = max(1, args.streams)
    fss = [FrameStream(W, H, scene.K, nfeatures=N, max_frames=B + 1, max_iters=args.max_iters, ctx=ctx)
           for _ in range(S)]
    for f in fss[1:]:
        f.share_pose(fss[0])  # one pose stream across the alternating batches
    recs_t = [f.new_records(B) for f in fss]
    from droplet_visual_odometry_amd.synth import MARKER_LEN
    corners = torch.tensor(np.stack([scene.marker_corners(i) for i in range(pool_n)]), dtype=torch.float64,
                           device=dev)
    T_rel = [torch.empty((B, 4, 4), dtype=torch.float64, device=dev) for _ in range(S)]
    T_abs = [torch.empty((B, 4, 4), dtype=torch.float64, device=dev) for _ in range(S)]
    fss[0].reset_pose()
    torch.cuda.synchronize()
    n_windows = max(1, (pool_n - 1) // B)

    host_log = []

    def step(i):
        s = (i % n_windows) * B
        k = i % S
        fs = fss[k]
        t_a = time.perf_counter()
        fs.process(pool[s:s + B + 1], recs_t[k], wait_torch=False)
        t_b = time.perf_counter()
        fs.pose_tail(corners[s:s + B], corners[s + 1:s + B + 1], MARKER_LEN, T_rel[k], T_abs[k], wait_torch=False)
        if args.host_trace:
            host_log.append((i, t_a, t_b, time.perf_counter()))

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
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    sync_all()
    elapsed = time.perf_counter() - t0
    for i, t_a, t_b, t_c in host_log:
        print(f"host step {i}: process enqueued at {1e3 * (t_a - t0):8.2f} ms, took {1e3 * (t_b - t_a):6.2f} ms; "
              f"pose_tail {1e3 * (t_c - t_b):6.2f} ms", file=sys.stderr)

    recs = FrameStream.records_numpy(recs_t[(args.warmup + args.steps - 1) % S], B)
    stage_ms, calls = {}, 0
    if not args.no_profile:
        for f in fss:
            sm, c = f.stage_times()
            calls += c
            for kk, v in sm.items():
                stage_ms[kk] = stage_ms.get(kk, 0.0) + v
    value = B * args.steps / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

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
        pmc = pmc_counts(single[dom], W, H, N, B)
        valu = None
        if pmc and pmc["valu_insts"]:
            va = pmc["valu_insts"] / (per_call[dom] * 1e-3)
            valu = {"achieved": round(va / 1e9, 3), "peak": VALU_PEAK_WIPS / 1e9, "unit": "G wave-instructions/s",
                    "frac": round(va / VALU_PEAK_WIPS, 6), "insts_per_launch": round(pmc["valu_insts"]),
                    "note": "SQ_INSTS_VALU per launch / the launch's HIP-event time; peak = one wave64 VALU "
                            "instruction per 2 cycles per SIMD x 1024 SIMDs x 2.4 GHz (MI355X_MICROARCH.md)"}
        roofline = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 6),
                    "traffic": pmc["traffic"] if pmc else None,
                    "traffic_raw": pmc["traffic_raw"] if pmc else None,
                    "traffic_calibrated": pmc["calibrated"] if pmc else None,
                    "traffic_source": pmc["source"] if pmc else None,
                    "valu": valu, "valu_frac": valu["frac"] if valu else None,
                    "kernel": single[dom], "algorithmic_bytes_per_launch": bytes_per_launch,
                    "kernel_ms_per_launch": round(per_call[dom], 4),
                    "stage_ms_per_step": {k: round(v, 4) for k, v in per_call.items()},
                    "path_algorithmic_bytes_per_frame": algorithmic_bytes_per_frame(W, H, N, m_avg),
                    "path_frac": round(value * algorithmic_bytes_per_frame(W, H, N, m_avg) / 1e9
                                       / HBM_PEAK_GBS, 8),
                    "ransac_f64": ransac_f64(per_call.get("ransac"), W, H, N, B)}

    cpu = None
    pose_check = None
    if args.cpu_seconds > 0:
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

    dropin = dropin_rate(pool, corners, scene.K, N, args.dropin_seconds) if args.dropin_seconds > 0 else None

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
                   "parallelism": "single GPU",
                   "streams_in_flight": S,
                   "pairs_ok": f"{ok}/{len(recs)}", "mean_matches": round(m_avg, 1),
                   "mean_ransac_iters": round(float(np.mean(recs['ransac_iters'])), 1) if len(recs) else 0,
                   "mean_ransac_hypotheses_solved": round(float(np.mean(recs['n_hypotheses'])), 1) if len(recs) else 0},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "pose_check": pose_check,
        "dropin": dropin,
    }
    print(json.dumps(out), flush=True)


def main_sharded(args, world, rank, local_rank, backend, dev, scene):
    """N > 1 (BASELINE configs[3]): ONE stream sharded across the ranks.  A step
    is a window of world x B consecutive pairs; rank r computes pairs
    [r B, (r+1) B) of it (frames r B .. (r+1) B, dist.shard_window) into the
    record slots of its send buffer, the ranks all-gather records and marker
    corners in one collective over RCCL (dist.ShardedPoseStream), and rank 0
    runs the window's pose tail -- marker scale against the previous
    successful pair, relative pose, absolute chain -- from the gathered
    records (stream.PoseTail), continuing across steps.  Weak scaling: B new
    pairs per rank per step; value = world x B x steps / max-over-ranks time.

    Stream ordering on the RCCL path (no host syncs in the loop): torch's
    stream waits for the library stream's records before the collective, and
    the library stream waits for the collective's `done` event before it
    rewrites the same send buffer S steps later."""
    import torch
    import torch.distributed as dist
    from droplet_visual_odometry_amd import dist as ddist
    from droplet_visual_odometry_amd._native import PAIR_RECORD_DTYPE, Context
    from droplet_visual_odometry_amd.synth import MARKER_LEN
    W, H, N, B = args.width, args.height, args.nfeatures, args.batch
    WP = world * B
    n_windows = 2
    wins = [ddist.shard_window(WP, world, rank, j * WP) for j in range(n_windows)]
    # each rank renders only the frames of its own runs (no scatter)
    pools = [torch.stack([scene.render(g) for g in range(f0, f1)]).contiguous() for (_, _, f0, f1) in wins]
    corners = [torch.tensor(np.stack([scene.marker_corners(g) for g in range(f0, f1)]), dtype=torch.float64,
                            device=dev) for (_, _, f0, f1) in wins]
    torch.cuda.synchronize()
    run = ddist.ShardedStreamRunner(W, H, scene.K, N, WP, world, rank, MARKER_LEN, ctx=Context(local_rank),
                                    max_iters=args.max_iters, streams=args.streams, host_gather=backend == "gloo")
    S = run.S
    torch.cuda.synchronize()

    def step(i):
        j = i % n_windows
        return run.step(pools[j], corners[j][:-1], corners[j][1:])[0]

    sync_all = run.sync
    for i in range(args.warmup):
        step(i)
    sync_all()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        recs = step(args.warmup + i)
    sync_all()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=torch.device("cpu") if run.host_gather else dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    recs = recs.cpu().numpy().view(PAIR_RECORD_DTYPE)
    value = WP * args.steps / elapsed
    if rank == 0:
        m_avg = float(np.mean(recs["n_matches"]))
        out = {
            "metric": ("frames/sec (detect+match+pose) at 1280\u00d7720, 2000 feats; ATE vs reference"
                       if (W, H, N) == (1280, 720, 2000)
                       else f"frames/sec (detect+match+pose) at {W}\u00d7{H}, {N} feats; ATE vs reference"),
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8/f32/f64",
            "data": "synthetic (seeded ray-cast textured room, droplet_visual_odometry_amd/synth.py)",
            "config": {"workload": f"{W}x{H} mono8 stream, {N} ORB features, one stream sharded over {world} "
                                   f"ranks, {B} new frames/step per rank",
                       "width": W, "height": H, "nfeatures": N, "batch_frames": B, "max_iters": args.max_iters,
                       "parallelism": f"one stream pair-sharded x{world} + "
                                      + ("gloo all_gather (rehearsal)" if run.host_gather else "RCCL all_gather")
                                      + " of records and marker corners, rank-0 device pose tail and chain",
                       "streams_in_flight": S,
                       "pairs_ok": f"{int(np.sum(recs['status'] == 0))}/{len(recs)}", "mean_matches": round(m_avg, 1),
                       "mean_ransac_iters": round(float(np.mean(recs['ransac_iters'])), 1)},
            "roofline": None,
            "cpu_baseline": None,
        }
        print(json.dumps(out), flush=True)
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


def pmc_counts(kernel, W, H, N, B):
    """Per-launch PMC figures of `kernel` from the committed round profile
    (profiles/PMC_TRAFFIC, tools/profile_round.sh): HBM bytes (FETCH_SIZE +
    WRITE_SIZE, corrected by the known-bytes calibration of the kernel's access
    widths) and SQ_INSTS_VALU, scaled per frame from the profiled batch to a
    launch over B + 1 frames.  PMC counters cannot run inside the timed loop."""
    path = os.path.join(ROOT, "profiles", PMC_TRAFFIC)
    try:
        doc = json.load(open(path))
    except (OSError, ValueError):
        return None
    c = doc.get("config", {})
    k = doc.get("kernels", {}).get(kernel)
    if k is None or (c.get("width"), c.get("height"), c.get("nfeatures")) != (W, H, N) or not c.get("batch"):
        return None
    scale = (B + 1) / (c["batch"] + 1)
    src = f"profiles/{PMC_TRAFFIC} (rocprofv3 --pmc passes at batch {c['batch']}"
    src += ")" if c["batch"] == B else f", scaled per frame to batch {B})"
    return {"traffic": round((k["fetch_bytes"] + k["write_bytes"]) * scale),
            "traffic_raw": round((k["fetch_bytes_raw"] + k["write_bytes_raw"]) * scale),
            "calibrated": bool(k.get("calibrated")), "widths": k.get("widths"),
            "valu_insts": k.get("SQ_INSTS_VALU", 0.0) * scale, "source": src}


def ransac_f64(ms_per_launch, W, H, N, B):
    """f64 issue fraction of the RANSAC kernel group (sampling, stage A, Durand-Kerner, stage C, score,
    replay, finish): its f64 VALU FLOPs per launch (profiles/PMC_F64: SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64,
    FMA = 2 FLOP, a wave64 instruction = 64 lanes; scaled per pair from the profiled batch) / the group's
    HIP-event time on the library stream / the FP64 vector peak.  The event time includes the waits for the
    other stream's kernels sharing the CUs, so this is the rate the stage achieves in the pipeline."""
    if not ms_per_launch:
        return None
    path = os.path.join(ROOT, "profiles", PMC_F64)
    try:
        doc = json.load(open(path))
    except (OSError, ValueError):
        return None
    c = doc.get("config", {})
    if (c.get("width"), c.get("height"), c.get("nfeatures")) != (W, H, N) or not c.get("batch"):
        return None
    scale = B / c["batch"]
    ks = {k: v for k, v in doc["kernels"].items() if "ransac_" in k}  # incl. "void ransac_score_kernel<16>"
    flops = sum(v["f64_flops_full_wave"] for v in ks.values()) * scale
    insts = sum(v["f64_wave_insts"] for v in ks.values()) * scale
    achieved = flops / (ms_per_launch * 1e-3) / 1e12
    # issue view: a wave64 f64 instruction holds a SIMD's f64 pipe 4 cycles (16 lanes per cycle)
    issue = insts * 4 / (ms_per_launch * 1e-3 * 1024 * 2.4e9)
    return {"bound": "f64 valu", "achieved": round(achieved, 3), "peak": F64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / F64_PEAK_TFLOPS, 5), "issue_frac": round(issue, 5),
            "f64_wave_insts_per_launch": round(insts),
            "f64_flops_per_launch": round(flops), "ms_per_launch": round(ms_per_launch, 4),
            "kernels": sorted(ks), "source": f"profiles/{PMC_F64} (batch {c['batch']}, scaled per pair to {B})"}


def dropin_rate(pool, corners, K, nfeatures, seconds, n_frames=48):
    """Pairs/s of the drop-in surface the ROS harness calls: the drop-in
    VisualOdometry.visual_odometry_calculations (visual_odometry_v3.py:384-408)
    one pair at a time, host mono8 frames in and 4x4 poses out, synchronous,
    chained as trajectory_evaluation_dual_process.py:151-166 does (previous
    absolute pose and both frames' marker corners per call).  ORB runs at the
    bench's nfeatures (the reference's ORB_create() default is 500)."""
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "droplet_visual_odometry_amd", "dropin"))
    try:
        import visual_odometry_v3 as v3
    finally:
        sys.path.pop(0)
    d = ", ".join(repr(float(v)) for v in np.asarray(K).ravel())
    with tempfile.NamedTemporaryFile("w", suffix=".yaml", delete=False) as fh:
        fh.write(f"camera_matrix:\n  rows: 3\n  cols: 3\n  data: [{d}]\n"
                 "distortion_coefficients:\n  rows: 1\n  cols: 5\n  data: [0.0, 0.0, 0.0, 0.0, 0.0]\n")
        cal = fh.name
    from droplet_visual_odometry_amd.synth import MARKER_LEN
    vo = v3.VisualOdometry(mode="orb", calibration_file_path=cal, controlled=True, real_marker_length=MARKER_LEN)
    os.unlink(cal)
    vo.feature_detector.setMaxFeatures(nfeatures)
    n = min(n_frames, len(pool))
    frames = [pool[i].cpu().numpy() for i in range(n)]
    cs = corners[:n].cpu().numpy()
    T = vo.robot_curr_position
    T, _ = vo.visual_odometry_calculations(frames[0], frames[1], T, cs[0], cs[1])  # warm-up (plans, scratch)
    lat = []
    t0 = time.perf_counter()
    i = 1
    while time.perf_counter() - t0 < seconds:
        a = i % (n - 1)
        t1 = time.perf_counter()
        T, _ = vo.visual_odometry_calculations(frames[a], frames[a + 1], T, cs[a], cs[a + 1])
        lat.append(time.perf_counter() - t1)
        i += 1
    dt = time.perf_counter() - t0
    lat = np.array(lat) * 1e3
    return {"dropin_pairs_per_s": round(len(lat) / dt, 2), "ms_per_pair_median": round(float(np.median(lat)), 3),
            "ms_per_pair_p90": round(float(np.percentile(lat, 90)), 3), "pairs": len(lat),
            "surface": "dropin/visual_odometry_v3.VisualOdometry.visual_odometry_calculations, one synchronous call "
                       "per pair (host frames in, poses out), as trajectory_evaluation_dual_process.py:151-166"}


def cpu_threads():
    """Host threads for the all-cores leg: the CPUs this process may run on,
    capped by OMP_NUM_THREADS (the GPU box sets it to the box's CPU share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        n = min(n, int(os.environ.get("OMP_NUM_THREADS", n)))
    except ValueError:
        pass
    return max(1, n)


def cpu_baseline(pool, K, nfeatures, max_iters, seconds):
    """The oracle (restated OpenCV path, C++ built -O3 -march=native for this
    host) on the same stream, in streaming mode (each frame detected once,
    its features reused by the next pair):
      single core   sequential pairs, the reference's execution model
                    (trajectory_evaluation_dual_process.py:172);
      all cores     the stream split into contiguous runs, one per thread
                    (ctypes releases the GIL inside the C++ calls), each run
                    sequential with feature reuse -- SURVEY.md §8d (2).
    Each leg runs about `seconds`.  value = the all-cores figure."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    lib_path = oracle.use_native_build()
    model, _ = oracle.host_cpu()
    host = lambda i: pool[i].cpu().numpy()  # noqa: E731

    t0 = time.perf_counter()
    kp_prev = oracle.detect_and_compute(host(0), nfeatures)
    i = 0
    ref = []
    while time.perf_counter() - t0 < seconds and i + 1 < len(pool):
        r = oracle.pair_pose(host(i), host(i + 1), K, nfeatures, max_iters=max_iters, kp_prev=kp_prev)
        kp_prev = (r["kp_cur"], r["desc_cur"])
        ref.append((r["R"], r["t_unit"]))
        i += 1
    dt1 = time.perf_counter() - t0
    n1 = i

    T = cpu_threads()
    run = max(2, (len(pool) - 1) // T)
    done = [0] * T
    deadline = time.perf_counter() + seconds

    def worker(t):
        a = t * run
        if a + 1 >= len(pool):
            return
        kp = oracle.detect_and_compute(host(a), nfeatures)
        j = a
        while j + 1 < min(len(pool), a + run + 1) and time.perf_counter() < deadline:
            r = oracle.pair_pose(host(j), host(j + 1), K, nfeatures, max_iters=max_iters, kp_prev=kp)
            kp = (r["kp_cur"], r["desc_cur"])
            done[t] += 1
            j += 1

    t1 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dtn = time.perf_counter() - t1
    nn = sum(done)
    W, H = pool.shape[2], pool.shape[1]
    return ({"value": round(nn / dtn, 3), "unit": "frames/s", "cores": T, "kind": "port",
             "sample": f"{nn} pairs of the same {W}x{H} stream in {dtn:.1f} s on {T} threads (the stream split into "
                       f"{T} contiguous runs, each sequential with feature reuse; each run's first detect included); "
                       f"oracle/ C++ restatement of the OpenCV path built -O3 -march=native "
                       f"({os.path.basename(lib_path)})",
             "single_core": {"value": round(n1 / dt1, 3), "cores": 1,
                             "sample": f"{n1} consecutive pairs in {dt1:.1f} s, first frame's detect included"},
             "host_cpus": os.cpu_count(), "cpu_model": model}, ref)


if __name__ == "__main__":
    main()
