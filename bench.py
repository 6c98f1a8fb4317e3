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
# HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default); streams that
# share a queue run in order, so the copy stream of the host-fed leg queued behind a library stream's
# kernels (host-fed 45.0 K -> 58.1 K frames/s with 8; the device-resident run is unchanged,
# profiles/r05h_queues.txt).  The bench runs two library streams, torch's stream, a side stream and a
# copy stream: 8 queues give each its own.  Set before the HIP runtime starts, over the environment's
# value (the GPU box exports HIP's default, 4); DVO_BENCH_HW_QUEUES chooses another count.
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("DVO_BENCH_HW_QUEUES", "8")

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
# VALU issue: a SIMD issues one wave64 VALU instruction per 2 cycles; 256 CUs x 4 SIMDs at 2.4 GHz
VALU_PEAK_WIPS = 256 * 4 * 2.4e9 / 2
# PMC documents (tools/profile_round.sh: calibrated FETCH/WRITE_SIZE + SQ passes; tools/pmc_stall_f64.sh +
# tools/pmc_f64.py: f64 VALU instructions per kernel) are looked up under profiles/ by the workload they were
# collected on: the newest round tag whose config matches (width, height, nfeatures) wins (pmc_doc).
PMC_TRAFFIC_GLOB = "r*_pmc_traffic*.json"
PMC_F64_GLOB = "r*_pmc_f64*.json"
# FP64 vector peak: 78.6 TFLOP/s, AMD's MI355X data-sheet figure (MI355X_MICROARCH.md lists no f64 row).  It is
# the wave64 f64 FMA issue rate: 16 lanes per cycle per SIMD (a wave64 f64 instruction per 4 cycles) x 2 FLOP x
# 1024 SIMDs x 2.4 GHz.
F64_PEAK_TFLOPS = 78.6
# The kernels of each HIP-event stage (include/dvo.h DVO_NSTAGES; api.cpp run_stream / launch_geometry).
STAGE_KERNELS = {
    "pyramid": ["resize_level_lds_kernel"],
    "blur": ["blur_kernel"],
    "fast": ["fast_strip_kernel"],
    "select_harris": ["select_fast_kernel", "harris_kernel", "select_harris_kernel"],
    "describe": ["describe_kernel"],
    "match": ["nn_mfma_kernel", "crosscheck_stream_kernel"],
    "ransac": ["normalize_kernel", "ransac_"],
    "recover_pose": ["pose_decompose_kernel", "pose_count_kernel", "pose_pick_kernel", "records_kernel"],
    "pose_tail": ["pose_tail_kernel", "pose_chain_kernel"],
}
PAIR_STAGES = ("match", "ransac", "recover_pose", "pose_tail")  # units are pairs (B), the rest frames (B + 1)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--batch", type=int, default=3072,
                    help="new frames per step (pairs per step); two streams, 1280x720: 1024 68.7 K frames/s, "
                         "1536 70.3 K, 2048 71.0 K, 3072 72.2 K (profiles/r02r_batch_sweep.txt); round 4 tree: "
                         "2048 90.3-90.4 K, 3072 91.4 K, 4096 91.5 K, 3 streams 83.4 K (profiles/r04u_sweep.txt)")
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
    ap.add_argument("--no-ref-equivalent", action="store_true",
                    help="skip the reference-equivalent leg (both frames of every pair detected, GPU and CPU)")
    ap.add_argument("--no-host-fed", action="store_true",
                    help="skip the host-fed leg (pinned host frames, async H2D on a copy stream)")
    ap.add_argument("--tail-world", type=int, default=8,
                    help="rehearse rank 0's reassembly load of a world-N window at N=1: the pose tail and absolute "
                         "chain over N x B gathered records on torch's stream beside the library streams (0 = skip)")
    ap.add_argument("--pose-check-32", type=int, default=256,
                    help="pairs of the OpenCV 3.2-semantics pose check against the oracle (0 = skip); run by the "
                         "c3_ocv32 config leg when it is enabled")
    ap.add_argument("--config-legs", default="c2,c5,c3_ocv32",
                    help="BASELINE configs timed after the headline, each with the headline's pipelined two-stream "
                         "schedule, roofline and an oracle pose check (comma list of c2, c5, c3_ocv32; 'none' skips)")
    ap.add_argument("--leg-steps", type=int, default=10, help="timed steps per run of a config leg")
    ap.add_argument("--leg-runs", type=int, default=3, help="timed runs of a config leg (value = the median)")
    ap.add_argument("--leg-pose-pairs", type=int, default=64,
                    help="pairs of a config leg's pose check against the oracle in the same semantics")
    ap.add_argument("--runs", type=int, default=5,
                    help="timed runs of exactly --steps steps each; value = the median run (BASELINE.md §3: "
                         "median of 5 runs), every run's rate reported under `runs`")
    ap.add_argument("--pose-check-per-rank", type=int, default=6,
                    help="N > 1: pairs at the start of every rank's run of the gathered window checked against "
                         "the oracle (0 = skip)")
    ap.add_argument("--spawn-check", action="store_true", help=argparse.SUPPRESS)  # tests/test_bench_launch.py
    return ap.parse_args()


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`--gpus N` (N > 1) run directly, without torch.distributed.run: one
    worker process per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on
    127.0.0.1), each re-running this script with the same arguments; only rank
    0 prints the JSON line.  The parent starts them before anything touches the
    GPU (torch.cuda.device_count() does not initialise a device on this image)
    and never replaces itself: it waits, stops the other ranks when one fails
    and exits with the first failure's status.  With RCCL (the default) N must
    not exceed the node's GPUs; DVO_BENCH_BACKEND=gloo rehearses more ranks
    than GPUs (ranks share devices, records gathered through host memory).
    Under a launcher (WORLD_SIZE set) this is skipped."""
    import subprocess
    n = args.gpus
    backend = os.environ.get("DVO_BENCH_BACKEND", "nccl")
    if backend != "gloo" and not args.spawn_check:
        import torch
        have = torch.cuda.device_count()
        if n > have:
            print(f"bench.py: --gpus {n} needs {n} GPUs for RCCL, this node has {have} "
                  f"(DVO_BENCH_BACKEND=gloo rehearses more ranks than GPUs)", file=sys.stderr, flush=True)
            return 2
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    alive = set(range(n))
    while alive:
        for r in sorted(alive):
            c = procs[r].poll()
            if c is None:
                continue
            alive.discard(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                print(f"bench.py: rank {r} exited with status {c}; stopping the other ranks", file=sys.stderr,
                      flush=True)
                for q in alive:
                    procs[q].terminate()
        time.sleep(0.1)
    return rc


def spawn_check():
    """The launcher rehearsal without a GPU (tests/test_bench_launch.py): every
    rank joins the gloo group; rank 0 prints what each rank saw."""
    import torch.distributed as dist
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seen = [None] * world
    dist.all_gather_object(seen, {"rank": rank, "local_rank": int(os.environ["LOCAL_RANK"]), "pid": os.getpid(),
                                  "world": dist.get_world_size()})
    if rank == 0:
        print(json.dumps({"spawn_check": seen}), flush=True)
    dist.destroy_process_group()


def timed_runs(args, step, sync_all, first, dist=None, device=None):
    """args.runs timed runs of exactly args.steps steps each, every run
    bracketed by a barrier (N > 1) and a device sync on both sides, its time
    the max over ranks.  Returns the per-run seconds."""
    import torch
    out = []
    i = first
    for _ in range(max(1, args.runs)):
        sync_all()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(i)
            i += 1
        sync_all()
        if dist is not None:
            dist.barrier()
        dt = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([dt], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        out.append(dt)
    return out


def runs_summary(per_run_s, units_per_run):
    rates = [units_per_run / s for s in per_run_s]
    med = float(np.median(rates))
    return med, {"n": len(rates), "frames_per_s": [round(r, 1) for r in rates], "median": round(med, 2),
                 "min": round(min(rates), 1), "max": round(max(rates), 1),
                 "spread_frac": round((max(rates) - min(rates)) / med, 4),
                 "note": "value = the median run; each run times exactly `steps` steps (BASELINE.md §3)"}


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
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.spawn_check:
        return spawn_check()
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
    from droplet_visual_odometry_amd.synth import MARKER_LEN
    corners = torch.tensor(np.stack([scene.marker_corners(i) for i in range(pool_n)]), dtype=torch.float64,
                           device=dev)
    T_rel = [torch.empty((B, 4, 4), dtype=torch.float64, device=dev) for _ in range(S)]
    T_abs = [torch.empty((B, 4, 4), dtype=torch.float64, device=dev) for _ in range(S)]
    fss[0].reset_pose()
    pipe = Pipeline(fss, B, corners, MARKER_LEN, T_rel, T_abs)
    torch.cuda.synchronize()
    n_windows = max(1, (pool_n - 1) // B)

    host_log = []

    def step(i):
        s = (i % n_windows) * B
        t_a = time.perf_counter()
        pipe.step(i % S, pool[s:s + B + 1], s)
        if args.host_trace:
            host_log.append((i, t_a, time.perf_counter(), time.perf_counter()))

    sync_all = pipe.sync
    prime = max(args.warmup, pipe.prime_steps)  # the pipeline is full: every timed step retires one batch
    for i in range(prime):
        step(i)
    sync_all()
    if not args.no_profile:
        for f in fss:
            f.set_profiling(True)
    torch.cuda.synchronize()
    t_origin = time.perf_counter()
    per_run = timed_runs(args, step, sync_all, prime)
    n_run = len(per_run)
    for i, t_a, t_b, t_c in host_log:
        print(f"host step {i}: submit enqueued at {1e3 * (t_a - t_origin):8.2f} ms, took {1e3 * (t_b - t_a):6.2f} ms",
              file=sys.stderr)
    value, runs = runs_summary(per_run, B * args.steps)
    elapsed = B * args.steps / value  # the median run's time
    stage_ms, calls = {}, 0
    if not args.no_profile:
        for f in fss:
            sm, c = f.stage_times()
            calls += c
            for kk, v in sm.items():
                stage_ms[kk] = stage_ms.get(kk, 0.0) + v
            f.set_profiling(False)
    t_d = time.perf_counter()
    pipe.drain()
    sync_all()
    drain_ms = 1e3 * (time.perf_counter() - t_d)
    recs = FrameStream.records_numpy(*pipe.last)
    pipe_depth, pipe_prime = pipe.D, pipe.prime_steps
    ms_per_step = 1000.0 * elapsed / args.steps

    m_avg = float(np.mean(recs["n_matches"])) if len(recs) else N / 2
    ok = int(np.sum(recs["status"] == 0))
    roofline = None
    if stage_ms and calls:
        per_call = {k: v / calls for k, v in stage_ms.items()}
        roofline = roofline_of(per_call, value, W, H, N, B, m_avg)
    # the other schedules of the same workload, on the GPU (never `value`)
    legs = {}
    def leg(name, fn, *a):
        # a leg that fails (e.g. out of device memory at an unusual batch) is reported, never the whole line
        try:
            legs[name] = fn(*a)
        except Exception as e:  # noqa: BLE001
            legs[name] = {"error": f"{type(e).__name__}: {e}"}
            torch.cuda.synchronize()
            torch.cuda.empty_cache()

    if not args.no_ref_equivalent:
        leg("reference_equivalent", ref_equivalent_leg, args, pool, corners, scene.K, ctx, value, recs,
            pipe.last_s0)
    cpu = None
    pose_check = None
    pose_check_32 = None
    if args.cpu_seconds > 0:
        cpu, ref = cpu_baseline(pool, scene.K, N, args.max_iters, args.cpu_seconds,
                                ref_equivalent=not args.no_ref_equivalent)
        if "value" in legs.get("reference_equivalent", {}) and cpu.get("reference_equivalent"):
            re = legs["reference_equivalent"]
            re["cpu_value"] = cpu["reference_equivalent"]["value"]
            re["speedup_vs_cpu_same_mode"] = round(re["value"] / max(re["cpu_value"], 1e-9), 1)
        # the same pairs on the GPU (window 0, through the pipelined submit), compared with the oracle's R, t
        rec0 = fss[0].new_records(B)
        torch.cuda.synchronize()
        fss[0].submit(pool[0:B + 1], rec0, wait_torch=False)
        fss[0].drain()
        fss[0].sync()
        g = FrameStream.records_numpy(rec0, B)
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
        leg_names = [x for x in args.config_legs.split(",") if x and x != "none"]
        if args.pose_check_32 > 0 and "c3_ocv32" not in leg_names:
            pose_check_32 = pose_check_opencv32(pool, scene.K, N, args.max_iters, args.pose_check_32, ctx)

    # BASELINE's other configs and the OpenCV 3.2 semantics, each on two new library streams beside the
    # headline's (never `value`).  They run before the legs that use torch side streams: torch creates its
    # stream pool (dozens of HIP streams) on first use, after which new library streams can share a hardware
    # queue with each other and run serialised
    leg_names = [x for x in args.config_legs.split(",") if x and x != "none"]
    if leg_names:
        cfg_legs = {}
        for name in leg_names:
            try:
                cfg_legs[name] = config_leg(args, ctx, dev, name)
            except Exception as e:  # noqa: BLE001
                import traceback
                traceback.print_exc()
                cfg_legs[name] = {"error": f"{type(e).__name__}: {e}"}
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        if "c3_ocv32" in cfg_legs and "pose_check" in cfg_legs["c3_ocv32"]:
            pose_check_32 = cfg_legs["c3_ocv32"]["pose_check"]
        legs["configs"] = cfg_legs

    if not args.no_host_fed:
        for f in fss:
            f.set_profiling(False)
        leg("host_fed", host_fed_leg, args, pool, pipe, n_windows, value)
    if args.tail_world > 1:
        for f in fss:
            f.set_profiling(False)
        leg(f"rank0_tail_world{args.tail_world}", rank0_tail_leg, args, pool, pipe, corners, n_windows,
            scene.K, ctx)

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
                   "mean_ransac_hypotheses_solved": round(float(np.mean(recs['n_hypotheses'])), 1) if len(recs) else 0,
                   "ransac_pipeline": {"depth": pipe_depth, "prime_steps": max(args.warmup, pipe_prime),
                                       "drain_ms": round(drain_ms, 3),
                                       "note": "RANSAC rounds of the last `depth` batches of a stream run as one "
                                               "merged round per submit (include/dvo.h dvo_stream_submit); after "
                                               "prime_steps untimed submits every timed step retires one complete "
                                               "batch (records + pose tail); records identical to one batch at a "
                                               "time (tests/test_gpu_pipeline.py)"}},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "pose_check": pose_check,
        "pose_check_opencv32": pose_check_32,
        "runs": runs,
        "dropin": dropin,
    }
    if cpu is not None:
        out["speedup_vs_cpu_same_mode"] = {"streaming": round(value / max(cpu["value"], 1e-9), 1)}
        if "reference_equivalent" in legs and "speedup_vs_cpu_same_mode" in legs["reference_equivalent"]:
            out["speedup_vs_cpu_same_mode"]["reference_equivalent"] = \
                legs["reference_equivalent"]["speedup_vs_cpu_same_mode"]
        out["speedup_vs_cpu_same_mode"]["cpu_threads"] = cpu["cores"]
    cfg_l = legs.pop("configs", None)
    if cfg_l is not None:
        legs["configs"] = cfg_l
    out["legs"] = legs  # last: the config legs' summaries end the line (the driver keeps the stdout tail)
    print(json.dumps(out), flush=True)


class Pipeline:
    """Batches in flight on S library streams (dvo_stream_submit, include/dvo.h): stream k takes
    steps k, k + S, ...; each submit runs detection + matching of its batch and one merged RANSAC
    round of the stream's last pipeline_depth() batches, and retires the oldest, whose pose tail
    (marker scale, relative and absolute poses, v3:309-345, :367) then runs on the shared carry in
    step order.  After prime_steps submits every step retires exactly one batch of B pairs.
    Each stream keeps pipeline_depth() record buffers in a ring (a batch's records stay pending
    until it retires)."""

    def __init__(self, fss, B, corners, marker_len, T_rel, T_abs, paired=False, tail=True):
        from droplet_visual_odometry_amd.stream import FrameStream
        import collections
        self.fss, self.B, self.corners, self.L = fss, B, corners, marker_len
        self.T_rel, self.T_abs, self.paired, self.tail = T_rel, T_abs, paired, tail
        self.D = FrameStream.pipeline_depth()
        self.recs = [[f.new_records(B) for _ in range(self.D)] for f in fss]
        self.fifo = [collections.deque() for _ in fss]  # (first frame, global submit number) per pending batch
        self.nsub = [0] * len(fss)
        self.gseq = 0
        self.last = None      # (records, pairs) of the last retired batch
        self.last_s0 = None   # its first frame in the pool
        self.prime_steps = len(fss) * (self.D - 1)
        self.on_retire = None  # optional hook(k, records, pairs, s0) instead of the pose tail

    def step(self, k, frames, s0, wait_torch=False):
        fs = self.fss[k]
        rec = self.recs[k][self.nsub[k] % self.D]
        self.nsub[k] += 1
        self.fifo[k].append((s0, self.gseq))
        self.gseq += 1
        ret = (fs.submit_pairs if self.paired else fs.submit)(frames, rec, wait_torch=wait_torch)
        for r, pairs in ret:
            self._retired(k, r, pairs, self.fifo[k].popleft()[0])

    def _retired(self, k, r, pairs, s0):
        if self.on_retire is not None:
            self.on_retire(k, r, pairs, s0)
        elif self.tail:
            c = self.corners
            self.fss[k].pose_tail_batch(r, pairs, c[s0:s0 + pairs], c[s0 + 1:s0 + pairs + 1], self.L, self.T_rel[k],
                                        self.T_abs[k])
        self.last, self.last_s0 = (r, pairs), s0

    def drain(self):
        # every stream's remaining rounds, then the pose tails in submission order (one carry)
        done = []
        for k, fs in enumerate(self.fss):
            for r, pairs in fs.drain():
                s0, g = self.fifo[k].popleft()
                done.append((g, k, r, pairs, s0))
        for g, k, r, pairs, s0 in sorted(done, key=lambda t: t[0]):
            self._retired(k, r, pairs, s0)

    def sync(self):
        import torch
        for f in self.fss:
            f.sync()
        torch.cuda.synchronize()


def ref_equivalent_leg(args, pool, corners, K, ctx, stream_value, stream_recs, stream_first_pair):
    """The reference's own schedule on the GPU: visual_odometry_calculations
    re-detects BOTH frames of every pair (visual_odometry_v3.py:387-392), so a
    step of B pairs detects 2B frames (FrameStream.submit_pairs /
    dvo_stream_submit_pairs: pair p = frames 2p, 2p+1), then matches, RANSAC,
    recoverPose and the pose tail as the streaming step (pipelined the same
    way).  The paired frame tensors are gathered from the same device pool
    before timing.  Its records must equal the streaming schedule's byte for
    byte (detection is a function of the frame), which is checked on the
    streaming run's last batch.  Steps carry min(batch, 1024) pairs (2 x that
    many frames per stream, beside the streaming run's streams, which stay
    allocated)."""
    import torch
    from droplet_visual_odometry_amd.stream import FrameStream
    from droplet_visual_odometry_amd.synth import MARKER_LEN
    W, H, N, S = args.width, args.height, args.nfeatures, max(1, args.streams)
    B = min(args.batch, 1024)
    n_windows = max(1, (len(pool) - 1) // B)
    dev = pool.device
    pp = [pool.index_select(0, torch.tensor([w * B + p + j for p in range(B) for j in (0, 1)], device=dev))
          .contiguous() for w in range(n_windows)]
    fss = [FrameStream(W, H, K, nfeatures=N, max_frames=2 * B, max_iters=args.max_iters, ctx=ctx) for _ in range(S)]
    for f in fss[1:]:
        f.share_pose(fss[0])
    T_rel = [torch.empty((B, 4, 4), dtype=torch.float64, device=dev) for _ in range(S)]
    T_abs = [torch.empty((B, 4, 4), dtype=torch.float64, device=dev) for _ in range(S)]
    fss[0].reset_pose()
    pipe = Pipeline(fss, B, corners, MARKER_LEN, T_rel, T_abs, paired=True)
    torch.cuda.synchronize()

    def step(i):
        w = i % n_windows
        pipe.step(i % S, pp[w], w * B)

    prime = max(args.warmup, pipe.prime_steps)
    for i in range(prime):
        step(i)
    pipe.sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(prime + i)
    pipe.sync()
    dt = time.perf_counter() - t0
    pipe.drain()
    pipe.sync()
    # the streaming run's last batch (its first B pairs) through the paired schedule: identical records
    chk = pool.index_select(0, torch.tensor([stream_first_pair + p + j for p in range(B) for j in (0, 1)],
                                            device=dev)).contiguous()
    rec = fss[0].process_pairs(chk, wait_torch=True)  # chk is written on torch's stream
    fss[0].sync()
    # every field the pair path defines (`reserved` carries pose-tail state of whichever window ran last)
    got = FrameStream.records_numpy(rec, B)
    differing = [k for k in got.dtype.names if not np.array_equal(got[k], stream_recs[:B][k])]
    same = not [k for k in differing if k not in ("reserved", "pad0")]
    for f in fss:
        f.close()
    del pp, fss, pipe
    torch.cuda.empty_cache()
    value = B * args.steps / dt
    return {"value": round(value, 2), "unit": "frames/s", "ms_per_step": round(1e3 * dt / args.steps, 3),
            "frames_detected_per_step": 2 * B, "pairs_per_step": B, "vs_streaming": round(value / stream_value, 4),
            "records_identical_to_streaming": same, "record_fields_differing": differing,
            "schedule": "reference-equivalent: both frames of every pair detected (v3:387-392), 2B detections "
                        "per B pairs, two batches in flight, RANSAC rounds pipelined as the streaming run; value "
                        "counts pairs (= new frames of the stream)"}


def host_fed_leg(args, pool, pipe, n_windows, stream_value):
    """Frames arriving from host memory, as the ROS harness hands them over
    (trajectory_evaluation_dual_process.py:154-164): the pool is held in
    pinned host memory, each step's B + 1 frames are copied host-to-device
    on a copy stream into a ring of device slots, and the library stream waits
    for the copy's event, so the H2D copies of the next steps overlap the
    compute of this one.  A slot is free again once the submit that read it
    has run its detection (the frames are read only there).  The link rate is
    the same copies timed alone.  Never `value`."""
    import torch
    B, S = args.batch, len(pipe.fss)
    R = S + 2  # copies run up to two steps ahead of the compute
    hpool = torch.empty(pool.shape, dtype=pool.dtype, pin_memory=True)
    hpool.copy_(pool)
    slots = [torch.empty((B + 1,) + tuple(pool.shape[1:]), dtype=pool.dtype, device=pool.device) for _ in range(R)]
    cs = torch.cuda.Stream(device=pool.device)
    used = [None] * R
    cev = []  # (start, end) timing events of the timed copies
    torch.cuda.synchronize()

    def step(i, timed=False):
        s0, k, r = (i % n_windows) * B, i % S, i % R
        with torch.cuda.stream(cs):
            if used[r] is not None:
                cs.wait_event(used[r])  # the detection that last read this slot has finished
            if timed:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record(cs)
            slots[r].copy_(hpool[s0:s0 + B + 1], non_blocking=True)
            ev = torch.cuda.Event(enable_timing=timed)
            ev.record(cs)
            if timed:
                cev.append((e0, ev))
        fs = pipe.fss[k]
        fs.wait_event(ev)
        pipe.step(k, slots[r], s0)
        used[r] = fs.record_event()

    prime = max(args.warmup, pipe.prime_steps)
    for i in range(prime):
        step(i)
    pipe.sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(prime + i, timed=True)
    pipe.sync()
    dt = time.perf_counter() - t0
    copy_ms = float(np.mean([a.elapsed_time(b) for a, b in cev])) if cev else None
    pipe.drain()
    pipe.sync()
    # the link alone: the same copies back to back on the copy stream
    nb = slots[0].numel()
    reps = max(3, min(args.steps, 10))
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    with torch.cuda.stream(cs):
        for i in range(reps):
            s0 = (i % n_windows) * B
            slots[i % R].copy_(hpool[s0:s0 + B + 1], non_blocking=True)
    cs.synchronize()
    dl = time.perf_counter() - t1
    link = nb * reps / dl / 1e9
    value = B * args.steps / dt
    del slots, hpool
    torch.cuda.empty_cache()
    return {"value": round(value, 2), "unit": "frames/s", "ms_per_step": round(1e3 * dt / args.steps, 3),
            "h2d_bytes_per_step": nb, "h2d_link_GBps": round(link, 2),
            "link_bound_frames_per_s": round(link * 1e9 / (nb / (B + 1)) * B / (B + 1), 1),
            "vs_device_resident": round(value / stream_value, 4),
            "copy_ms_during_compute": round(copy_ms, 3) if copy_ms else None,
            "copy_ms_alone": round(1e3 * dl / reps, 3),
            "schedule": "pinned host frames, async H2D on a copy stream into a ring of S+2 device slots overlapped "
                        "with compute; B+1 frames copied per B-pair step"}


def rank0_tail_leg(args, pool, pipe, corners, n_windows, K, ctx):
    """Rank 0's added load in a world-N run (bench.main_sharded, dist.ShardedStreamRunner), rehearsed on one
    GPU: per step the library streams submit B new pairs as every rank does, and torch's stream -- after
    waiting for the retired batch's records, as before the all-gather -- runs the pose tail and the serial
    absolute chain over a whole world-N window, N x B records (stream.PoseTail / dvo_pose_tail_records), as
    rank 0 does after the collective.  The gathered window is the retired batch's records and corners tiled
    N times (the tail's cost does not depend on their values).  Reported: ms per step with and without the
    rank-0 tail and the difference, against north_star's near-linear scaling (trajectory_evaluation_dual_
    process.py:172-252 is the single stream being reassembled)."""
    import torch
    from droplet_visual_odometry_amd._native import PAIR_RECORD_DTYPE
    from droplet_visual_odometry_amd.stream import HostPoseChain, PoseTail
    from droplet_visual_odometry_amd.synth import MARKER_LEN
    B, S, N = args.batch, len(pipe.fss), args.tail_world
    dev = pool.device
    rb = PAIR_RECORD_DTYPE.itemsize
    wrecs = [torch.zeros(N * B * rb, dtype=torch.uint8, device=dev) for _ in range(S)]
    cp = corners[:B].repeat(N, 1, 1).contiguous()
    cc = corners[1:B + 1].repeat(N, 1, 1).contiguous()
    tail = PoseTail(K, MARKER_LEN, ctx=ctx)
    hchain = HostPoseChain(N * B, 2 * S + 1, dev)
    T_rel = [torch.empty((N * B, 4, 4), dtype=torch.float64, device=dev) for _ in range(S)]
    T_abs = [torch.empty((N * B, 4, 4), dtype=torch.float64, device=dev) for _ in range(S)]
    cur = torch.cuda.current_stream(dev)
    torch.cuda.synchronize()
    done = {}  # record buffer -> the event after its last read (the stand-in collective)

    def on_retire(k, r, pairs, s0):
        fs = pipe.fss[k]
        cur.wait_event(fs.record_event())  # the records are final (before the collective)
        # stands in for the all-gather: it reads the records buffer, which the library rewrites only
        # pipeline_depth() submits later, after waiting for this copy (as the runner's per-slot wait,
        # dist.ShardedStreamRunner.step)
        wrecs[k][:pairs * rb].copy_(r[:pairs * rb])
        ev = torch.cuda.Event()
        ev.record(cur)
        done[r.data_ptr()] = ev
        # rank 0's half of the split tail (dist.ShardedStreamRunner): T_rel of its own B pairs, then
        # (after the T_rel all-gather, stood in for by the window's T_rel buffer) the serial chain on
        # a host thread
        tail.rel_range(wrecs[k], cp, cc, 0, pairs, T_rel[k])
        hchain.submit(T_rel[k])

    def run(with_tail):
        pipe.on_retire = on_retire if with_tail else (lambda *a: None)

        def step(i):
            s0, k = (i % n_windows) * B, i % S
            nxt = pipe.recs[k][pipe.nsub[k] % pipe.D]  # the buffer this submit writes
            if nxt.data_ptr() in done:
                pipe.fss[k].wait_event(done[nxt.data_ptr()])
            pipe.step(k, pool[s0:s0 + B + 1], s0)

        prime = max(args.warmup, pipe.prime_steps)
        for i in range(prime):
            step(i)
        pipe.sync()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(prime + i)
        pipe.sync()
        hchain.wait()  # every window chained
        dt = 1e3 * (time.perf_counter() - t0) / args.steps
        pipe.drain()
        pipe.sync()
        hchain.wait()
        return dt

    base = run(False)
    with_tail = run(True)
    pipe.on_retire = None
    # rank 0's tail alone: its pairs' T_rel on the idle GPU, the host chain over N x B
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(cur)
    tail.rel_range(wrecs[0], cp, cc, 0, B, T_rel[0])
    e1.record(cur)
    torch.cuda.synchronize()
    rel_alone = e0.elapsed_time(e1)
    th = time.perf_counter()
    hchain.submit(T_rel[0]).result()
    host_chain_ms = 1e3 * (time.perf_counter() - th)
    hchain.close()
    # the unsplit tail (every pair's T_rel on rank 0, round 4's schedule), for comparison
    e0.record(cur)
    tail.run(wrecs[0], cp, cc, T_rel[0], T_abs[0])
    e1.record(cur)
    torch.cuda.synchronize()
    alone_unsplit = e0.elapsed_time(e1)
    return {"world": N, "pairs_per_window": N * B, "ms_per_step_without_tail": round(base, 3),
            "ms_per_step_with_tail": round(with_tail, 3), "added_ms_per_step": round(with_tail - base, 3),
            "added_frac": round((with_tail - base) / base, 4), "rel_range_alone_ms": round(rel_alone, 3),
            "host_chain_ms": round(host_chain_ms, 3), "unsplit_device_tail_alone_ms": round(alone_unsplit, 3),
            "note": "rank 0's share of the split pose tail (dist.ShardedStreamRunner): T_rel of its own B pairs on "
                    "torch's stream beside the library streams, then the serial absolute chain over the world-N "
                    "window (N x B gathered T_rel) on a host thread (dvo_pose_chain_host); steps of B new pairs "
                    "per rank (weak scaling)"}


def oracle_pairs(host, K, nfeatures, max_iters, n_pairs, semantics):
    """The oracle's R, t for pairs 0 .. n_pairs-1 of a frame stream (host(i) = frame i as numpy), in
    streaming mode (each frame's features reused by the next pair), over all usable host threads: the
    pairs split into contiguous runs, each starting with a fresh detect of its first frame (detection is
    a function of the frame, so this equals one sequential pass).  ctypes releases the GIL inside the
    oracle's C++ calls.  Returns [(R or None, t_unit, n_matches)] in pair order."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.use_native_build()
    T = max(1, min(cpu_threads(), n_pairs))
    bounds = [(n_pairs * t // T, n_pairs * (t + 1) // T) for t in range(T)]
    frames = [host(i) for i in range(n_pairs + 1)]
    out = [None] * n_pairs
    errors = []

    def worker(a, b):
        try:
            kp = oracle.detect_and_compute(frames[a], nfeatures, semantics=semantics)
            for i in range(a, b):
                r = oracle.pair_pose(frames[i], frames[i + 1], K, nfeatures, max_iters=max_iters, kp_prev=kp,
                                     semantics=semantics)
                kp = (r["kp_cur"], r["desc_cur"])
                out[i] = (r["R"], r["t_unit"], len(r["q"]) if r.get("q") is not None else None)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ths = [threading.Thread(target=worker, args=ab) for ab in bounds if ab[1] > ab[0]]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    if errors:
        raise errors[0]
    return out, T


def compare_records(g, ref, check_matches=False):
    """Pairs whose device record equals the oracle's R and t bit for bit (a pair the oracle fails must fail
    on the device too); with check_matches the cross-checked match count as well."""
    ident = 0
    for i, (R, t, nm) in enumerate(ref):
        if R is None:
            ident += int(g["status"][i] != 0)
            continue
        ident += int(g["status"][i] == 0 and np.array_equal(g["R"][i].reshape(3, 3), R)
                     and np.array_equal(g["t"][i], np.asarray(t).ravel())
                     and (not check_matches or g["n_matches"][i] == nm))
    return ident


def pose_check_opencv32(pool, K, nfeatures, max_iters, n_pairs, ctx):
    """OpenCV 3.2 semantics (FrameStream(opencv="3.2"): INTER_LINEAR pyramid,
    3.2 retainBest, 3.x reverse-pass cross check) on the first n_pairs of the
    same stream, against the oracle in the same mode (streaming, features
    reused)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from droplet_visual_odometry_amd.stream import FrameStream
    W, H = pool.shape[2], pool.shape[1]
    n = min(n_pairs, len(pool) - 1)
    fs = FrameStream(W, H, K, nfeatures=nfeatures, max_frames=n + 1, max_iters=max_iters, ctx=ctx, opencv="3.2")
    rec = fs.process(pool[0:n + 1])
    fs.sync()
    g = FrameStream.records_numpy(rec, n)
    fs.close()
    ref, T = oracle_pairs(lambda i: pool[i].cpu().numpy(), K, nfeatures, max_iters, n, oracle.OCV32)
    return {"pairs": n, "bit_identical": compare_records(g, ref, check_matches=True),
            "reference": "oracle/ in OpenCV 3.2 mode (INTER_LINEAR pyramid, 3.2 retainBest, 3.x cross check), "
                         f"same frames, streaming ({T} threads)"}


# BASELINE.json configs timed as legs (north_star: 640x480 and 1280x720 numbers; configs[4] on one GPU) and the
# headline config in OpenCV 3.2 semantics, the version the reference most likely ran
CONFIG_LEGS = {
    "c2": dict(width=640, height=480, nfeatures=1000, batch=3072, max_iters=1000, opencv="4.x"),
    "c5": dict(width=1920, height=1080, nfeatures=4000, batch=1024, max_iters=4096, opencv="4.x"),
    # batch 2048: its two streams beside the headline's two fit the 288 GB (round 4 sweep: 2048 is within 1 % of
    # 3072 in frames/s, profiles/r04u_sweep.txt)
    "c3_ocv32": dict(width=1280, height=720, nfeatures=2000, batch=2048, max_iters=1000, opencv="3.2"),
}


def config_leg(args, ctx, dev, name):
    """One BASELINE config through the headline's schedule: S streams of pipelined submits
    (Pipeline), the pose tail on every retired batch, prime_steps untimed submits, then
    --leg-runs runs of exactly --leg-steps steps (value = the median run), HIP-event stage times
    -> the dominant stage's roofline, and the first pairs of window 0 (pipelined submit + drain)
    against the oracle in the same semantics, bit for bit."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from droplet_visual_odometry_amd.stream import FrameStream
    from droplet_visual_odometry_amd.synth import MARKER_LEN, SceneStream
    c = CONFIG_LEGS[name]
    W, H, N, B, it = c["width"], c["height"], c["nfeatures"], c["batch"], c["max_iters"]
    S = max(1, args.streams)
    t_leg = time.perf_counter()
    scene = SceneStream(W, H, device=str(dev))
    pool_n = 2 * B + 1
    pool = torch.stack([scene.render(i) for i in range(pool_n)]).contiguous()
    corners = torch.tensor(np.stack([scene.marker_corners(i) for i in range(pool_n)]), dtype=torch.float64,
                           device=dev)
    fss = [FrameStream(W, H, scene.K, nfeatures=N, max_frames=B + 1, max_iters=it, ctx=ctx, opencv=c["opencv"])
           for _ in range(S)]
    for f in fss[1:]:
        f.share_pose(fss[0])
    T_rel = [torch.empty((B, 4, 4), dtype=torch.float64, device=dev) for _ in range(S)]
    T_abs = [torch.empty((B, 4, 4), dtype=torch.float64, device=dev) for _ in range(S)]
    fss[0].reset_pose()
    pipe = Pipeline(fss, B, corners, MARKER_LEN, T_rel, T_abs)
    torch.cuda.synchronize()
    n_windows = 2

    trace = os.environ.get("DVO_BENCH_TRACE") == "1"  # diagnostics: every step synchronised and logged

    def step(i):
        s0 = (i % n_windows) * B
        pipe.step(i % S, pool[s0:s0 + B + 1], s0)
        if trace:
            pipe.sync()
            print(f"[{name}] step {i} ok ({time.perf_counter() - t_leg:.1f} s)", file=sys.stderr, flush=True)

    prime = max(args.warmup, pipe.prime_steps)
    for i in range(prime):
        step(i)
    pipe.sync()
    for f in fss:
        f.set_profiling(True)
    la = argparse.Namespace(runs=args.leg_runs, steps=args.leg_steps)
    per_run = timed_runs(la, step, pipe.sync, prime)
    value, runs = runs_summary(per_run, B * args.leg_steps)
    stage_ms, calls = {}, 0
    for f in fss:
        sm, cc = f.stage_times()
        calls += cc
        for kk, v in sm.items():
            stage_ms[kk] = stage_ms.get(kk, 0.0) + v
        f.set_profiling(False)
    pipe.drain()
    pipe.sync()
    recs = FrameStream.records_numpy(*pipe.last)
    m_avg = float(np.mean(recs["n_matches"]))
    roof = roofline_of({k: v / calls for k, v in stage_ms.items()}, value, W, H, N, B, m_avg) if calls else None
    # window 0's first pairs through the pipelined submit, against the oracle in the same semantics
    n = min(args.pose_check_32 if name == "c3_ocv32" else args.leg_pose_pairs, B)
    rec0 = fss[0].new_records(B)
    torch.cuda.synchronize()
    fss[0].submit(pool[0:B + 1], rec0, wait_torch=False)
    fss[0].drain()
    fss[0].sync()
    g = FrameStream.records_numpy(rec0, B)
    sem = oracle.OCV32 if c["opencv"] == "3.2" else oracle.OCV4
    t_o = time.perf_counter()
    ref, T = oracle_pairs(lambda i: pool[i].cpu().numpy(), scene.K, N, it, n, sem)
    oracle_s = time.perf_counter() - t_o
    ident = compare_records(g, ref, check_matches=True)
    for f in fss:
        f.close()
    del pipe, fss, pool, corners, T_rel, T_abs
    torch.cuda.empty_cache()
    out = {"value": round(value, 1), "unit": "frames/s", "config": f"{W}x{H} N{N} it{it} B{B} x{S} streams, OpenCV "
           f"{c['opencv']}", "ms_per_step": round(1e3 * B / value, 3), "runs": {"median": runs["median"],
           "spread_frac": runs["spread_frac"], "n": runs["n"], "steps": args.leg_steps},
           "mean_hypotheses_solved": round(float(np.mean(recs["n_hypotheses"])), 1),
           "mean_ransac_iters": round(float(np.mean(recs["ransac_iters"])), 1),
           "pairs_ok": f"{int(np.sum(recs['status'] == 0))}/{len(recs)}",
           "pose_check": {"pairs": n, "bit_identical": ident, "oracle_threads": T, "oracle_s": round(oracle_s, 1),
                          "semantics": c["opencv"]},
           "leg_s": round(time.perf_counter() - t_leg, 1)}
    if roof:
        hd = roof.get("hbm_dominant") or {}
        out["roofline"] = {"dominant_stage": roof["dominant_stage"], "bound": roof["bound"],
                           "frac": roof["frac"], "unit": roof["unit"], "achieved": roof["achieved"],
                           "path_frac": roof["path_frac"],
                           "hbm_dominant": {"stage": hd.get("stage"), "frac": hd.get("frac")} if hd else None,
                           "stage_ms_per_step": roof["stage_ms_per_step"]}
    return out


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
        run.step(pools[j], corners[j][:-1], corners[j][1:], wait_torch=False)  # frames resident

    sync_all = run.sync
    prime = max(args.warmup, run.prime_steps)  # the pipeline is full: every timed step retires one window
    for i in range(prime):
        step(i)
    sync_all()
    if not args.no_profile:
        for f in run.fss:
            f.set_profiling(True)
    per_run = timed_runs(args, step, sync_all, prime, dist=dist,
                         device=torch.device("cpu") if run.host_gather else dev)
    value, runs = runs_summary(per_run, WP * args.steps)
    elapsed = WP * args.steps / value
    stage_ms, calls = {}, 0
    if not args.no_profile:
        for f in run.fss:
            sm, c = f.stage_times()
            calls += c
            for kk, v in sm.items():
                stage_ms[kk] = stage_ms.get(kk, 0.0) + v
            f.set_profiling(False)
    run.drain()
    # window 0 once more, every rank: its gathered records are what rank 0 checks against the oracle
    outs = run.step(pools[0], corners[0][:-1], corners[0][1:], wait_torch=False) + run.drain()
    recs = outs[-1][0]
    sync_all()
    recs = recs.cpu().numpy().view(PAIR_RECORD_DTYPE).copy()
    if rank == 0:
        m_avg = float(np.mean(recs["n_matches"]))
        roofline = None
        if stage_ms and calls:
            per_call = {k: v / calls for k, v in stage_ms.items()}
            roofline = roofline_of(per_call, value / world, W, H, N, run.n_local, m_avg)
            roofline["rank"] = 0
            roofline["note_sharded"] = ("rank 0's HIP-event stages over its own runs (n_local + 1 frames, n_local "
                                        "pairs per launch); path_frac per GPU")
        cpu = pose_check = None
        if args.cpu_seconds > 0:
            cpu, ref = cpu_baseline(pools[0], scene.K, N, args.max_iters, args.cpu_seconds)
            pose_check = sharded_pose_check(args, scene, recs, ref, world, WP)
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
                       "streams_in_flight": S, "rccl_world": dist.get_world_size(),
                       "ransac_pipeline": {"depth": run.D, "prime_steps": prime},
                       "backend": "gloo" if run.host_gather else "nccl (RCCL)",
                       "pairs_per_rank": run.n_local, "window_pairs": WP,
                       "pairs_ok": f"{int(np.sum(recs['status'] == 0))}/{len(recs)}", "mean_matches": round(m_avg, 1),
                       "mean_ransac_iters": round(float(np.mean(recs['ransac_iters'])), 1),
                       "mean_ransac_hypotheses_solved": round(float(np.mean(recs['n_hypotheses'])), 1)},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "pose_check": pose_check,
            "runs": runs,
        }
        if cpu is not None:
            out["speedup_vs_cpu_same_mode"] = {"streaming": round(value / max(cpu["value"], 1e-9), 1),
                                               "cpu_threads": cpu["cores"]}
        print(json.dumps(out), flush=True)
    dist.barrier()  # the other ranks wait for rank 0's checks before the group goes away
    run.close()
    dist.destroy_process_group()


def sharded_pose_check(args, scene, recs, ref, world, WP):
    """R, t of the gathered window-0 records against the oracle: rank 0's
    pairs from cpu_baseline's sequential sample (`ref`), and the first
    --pose-check-per-rank pairs of every other rank's run, each run's oracle
    pass starting, as that rank does, from a fresh detect of its first frame."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from droplet_visual_odometry_amd import dist as ddist
    from droplet_visual_odometry_amd.synth import MARKER_LEN  # noqa: F401
    K, N = scene.K, args.nfeatures
    host = lambda g: scene.render(g).cpu().numpy()  # noqa: E731
    checked = []  # (global pair, R_ref, t_ref)
    for i, (R, t) in enumerate(ref[:max(1, args.pose_check_per_rank)]):
        checked.append((i, R, t))
    for r in range(1, world):
        p0, p1, _, _ = ddist.shard_window(WP, world, r, 0)
        n = min(args.pose_check_per_rank, p1 - p0)
        if n <= 0:
            continue
        kp = oracle.detect_and_compute(host(p0), N)
        for p in range(p0, p0 + n):
            o = oracle.pair_pose(host(p), host(p + 1), K, N, max_iters=args.max_iters, kp_prev=kp)
            kp = (o["kp_cur"], o["desc_cur"])
            checked.append((p, o["R"], o["t_unit"]))
    ident = 0
    err_r = err_t = 0.0
    for p, R_ref, t_ref in checked:
        if R_ref is None:
            ident += int(recs["status"][p] != 0)
            continue
        Rg, tg = recs["R"][p].reshape(3, 3), recs["t"][p]
        ident += int(np.array_equal(Rg, R_ref) and np.array_equal(tg, np.asarray(t_ref).ravel()))
        err_r = max(err_r, float(np.max(np.abs(Rg - R_ref))))
        err_t = max(err_t, float(np.max(np.abs(tg - np.asarray(t_ref).ravel()))))
    return {"pairs": len(checked), "bit_identical": ident, "max_abs_R_err": err_r, "max_abs_t_err": err_t,
            "ranks_checked": world, "pairs_checked": sorted({p for p, _, _ in checked}),
            "reference": "oracle/ C++ restatement, same frames, streaming with feature reuse from each rank's first "
                         "frame; records from the all-gathered window 0"}


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


def pmc_doc(pattern, W, H, N):
    """(path, document) of the committed PMC document under profiles/ collected on this workload:
    the newest (round tags sort by name) profiled on this tree if there is one, else the newest."""
    import glob
    best = same = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", pattern))):
        try:
            doc = json.load(open(path))
        except (OSError, ValueError):
            continue
        c = doc.get("config", {}) if isinstance(doc, dict) else {}
        if (c.get("width"), c.get("height"), c.get("nfeatures")) == (W, H, N) and c.get("batch") \
                and isinstance(doc.get("kernels"), dict):
            best = (path, doc)
            if pmc_tree(doc)["this_tree"]:
                same = best
    return same or best


def pmc_tree(doc):
    """The profiled tree a PMC document records (tools/profile_final.sh) and whether it is this one:
    the library sources' hash (build.source_hash, the build id the loaded library is checked against)."""
    t = doc.get("tree") if isinstance(doc, dict) else None
    if not t:
        return {"git": None, "this_tree": False}
    from droplet_visual_odometry_amd.build import source_hash
    return {"git": t.get("git"), "source_hash": t.get("source_hash"), "this_tree": t.get("source_hash") == source_hash()}


def kernels_of(stage, names):
    """The profiled kernel names (rocprofv3 spells templates "void k<...>") of a stage."""
    out = []
    for name in names:
        base = name.replace("void ", "").split("<")[0].strip()
        if any(base == k or (k.endswith("_") and base.startswith(k)) for k in STAGE_KERNELS[stage]):
            out.append(name)
    return sorted(out)


def pmc_counts(stage, W, H, N, B):
    """Per-launch PMC figures of a stage's kernels from the committed round
    profile (tools/profile_round.sh): HBM bytes (fetched bytes from the
    read-request-size counters, calibrated against kernels of known traffic,
    plus WRITE_SIZE) and SQ_INSTS_VALU, scaled from the profiled batch to a
    launch over this run's units (B + 1 frames, or B pairs).  PMC counters
    cannot run inside the timed loop."""
    found = pmc_doc(PMC_TRAFFIC_GLOB, W, H, N)
    if found is None:
        return None
    path, doc = found
    c = doc["config"]
    ks = kernels_of(stage, doc["kernels"])
    if not ks:
        return None
    scale = B / c["batch"] if stage in PAIR_STAGES else (B + 1) / (c["batch"] + 1)
    tot = lambda key: sum(doc["kernels"][k].get(key, 0.0) for k in ks)  # noqa: E731
    src = f"profiles/{os.path.basename(path)} (rocprofv3 --pmc passes at batch {c['batch']}, {c.get('streams', 1)} " \
          f"stream(s)"
    src += ")" if c["batch"] == B else f", scaled per unit to batch {B})"
    return {"traffic": round((tot("fetch_bytes") + tot("write_bytes")) * scale),
            "traffic_raw": round((tot("fetch_bytes_raw") + tot("write_bytes_raw")) * scale),
            "calibrated": all(bool(doc["kernels"][k].get("calibrated")) for k in ks),
            "valu_insts": tot("SQ_INSTS_VALU") * scale, "kernels": ks, "source": src, "tree": pmc_tree(doc)}


def ransac_f64(ms_per_launch, W, H, N, B):
    """f64 issue fraction of the RANSAC kernel group (sampling, stage A, Durand-Kerner, stage C, score,
    replay, finish): its f64 VALU FLOPs per launch (SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64, FMA = 2 FLOP, a
    wave64 instruction = 64 lanes; scaled per pair from the profiled batch) / the group's HIP-event time on
    the library stream / the FP64 vector peak.  The event time includes the waits for the other stream's
    kernels sharing the CUs, so this is the rate the stage achieves in the pipeline."""
    if not ms_per_launch:
        return None
    found = pmc_doc(PMC_F64_GLOB, W, H, N)
    if found is None:
        return None
    path, doc = found
    c = doc["config"]
    scale = B / c["batch"]
    ks = {k: v for k, v in doc["kernels"].items() if "ransac_" in k}  # incl. "void ransac_score_kernel<16>"
    flops = sum(v["f64_flops_full_wave"] for v in ks.values()) * scale
    insts = sum(v["f64_wave_insts"] for v in ks.values()) * scale
    achieved = flops / (ms_per_launch * 1e-3) / 1e12
    # issue view: a wave64 f64 instruction holds a SIMD's f64 pipe 4 cycles (16 lanes per cycle)
    issue = insts * 4 / (ms_per_launch * 1e-3 * 1024 * 2.4e9)
    per_kernel = {k: round(v["f64_wave_insts"] * scale) for k, v in sorted(ks.items())}
    # the lane pass (SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64) per kernel): FLOPs of active lanes only
    weighted = None
    if all("f64_flops_lane_weighted" in v for v in ks.values()):
        weighted = sum(v["f64_flops_lane_weighted"] for v in ks.values()) * scale / (ms_per_launch * 1e-3) / 1e12
    return {"bound": "f64 valu", "achieved": round(achieved, 3), "peak": F64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / F64_PEAK_TFLOPS, 5),
            "frac_counts": "issued lane slots: every lane of every issued f64 wave-instruction",
            "achieved_lane_weighted": round(weighted, 3) if weighted is not None else None,
            "frac_lane_weighted": round(weighted / F64_PEAK_TFLOPS, 5) if weighted is not None else None,
            "lane_util": {k: round(v["valu_lane_util"], 4) for k, v in sorted(ks.items()) if "valu_lane_util" in v},
            "issue_frac": round(issue, 5), "tree": pmc_tree(doc),
            "f64_wave_insts_per_launch": round(insts), "f64_wave_insts_per_kernel": per_kernel,
            "f64_flops_per_launch": round(flops), "ms_per_launch": round(ms_per_launch, 4),
            "kernels": sorted(ks), "source": f"profiles/{os.path.basename(path)} (batch {c['batch']}, scaled per "
                                             f"pair to {B})"}


def hbm_roofline(stage, ms, W, H, N, B, m_avg):
    """A stage priced against HBM: its algorithmic bytes per launch (stage_bytes x units) / its HIP-event time."""
    sb = stage_bytes(W, H, N, m_avg)
    units = B if stage in PAIR_STAGES else B + 1
    bytes_per_launch = sb[stage] * units
    achieved = bytes_per_launch / (ms * 1e-3) / 1e9
    pmc = pmc_counts(stage, W, H, N, B)
    valu = None
    if pmc and pmc["valu_insts"]:
        va = pmc["valu_insts"] / (ms * 1e-3)
        valu = {"achieved": round(va / 1e9, 3), "peak": VALU_PEAK_WIPS / 1e9, "unit": "G wave-instructions/s",
                "frac": round(va / VALU_PEAK_WIPS, 6), "insts_per_launch": round(pmc["valu_insts"]),
                "note": "SQ_INSTS_VALU per launch / the launch's HIP-event time; peak = one wave64 VALU "
                        "instruction per 2 cycles per SIMD x 1024 SIMDs x 2.4 GHz (MI355X_MICROARCH.md)"}
    return {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 6),
            "traffic": pmc["traffic"] if pmc else None,
            "traffic_raw": pmc["traffic_raw"] if pmc else None,
            "traffic_calibrated": pmc["calibrated"] if pmc else None,
            "traffic_source": pmc["source"] if pmc else None,
            "traffic_tree": pmc["tree"] if pmc else None,
            "valu": valu, "valu_frac": valu["frac"] if valu else None,
            "stage": stage, "kernel": ", ".join(pmc["kernels"]) if pmc else " / ".join(STAGE_KERNELS[stage]),
            "algorithmic_bytes_per_launch": bytes_per_launch, "kernel_ms_per_launch": round(ms, 4),
            "launch_note": "a launch = one batch (B + 1 frames or B pairs); detection stages run in frame groups of "
                           "<= 768 (csrc/orb.hip DVO_ORB_GROUP), so rocprofv3's per-dispatch average for these "
                           "kernels is this time divided by ceil((B + 1) / 768) dispatches"}


def roofline_of(per_call, value, W, H, N, B, m_avg):
    """The roofline of the dominant stage: the HIP-event stage with the most
    device time per step, whatever its bound.  The RANSAC group (scalar f64
    solver and scorer) is priced against the FP64 vector peak, every other
    stage against HBM with its algorithmic bytes.  The
    longest single-kernel HBM stage is reported beside it (`hbm_dominant`),
    and the f64 view of the RANSAC group always (`ransac_f64`)."""
    from droplet_visual_odometry_amd.plan import algorithmic_bytes_per_frame
    dom = max(per_call, key=lambda k: per_call.get(k, 0.0))
    rf = ransac_f64(per_call.get("ransac"), W, H, N, B)
    single = [k for k in ("fast", "blur", "describe") if per_call.get(k)]
    hdom = max(single, key=lambda k: per_call[k]) if single else None
    hbm_dom = hbm_roofline(hdom, per_call[hdom], W, H, N, B, m_avg) if hdom else None
    if dom == "ransac" and rf is not None:
        pmc = pmc_counts("ransac", W, H, N, B)
        roof = {"bound": "f64", "achieved": rf["achieved"], "peak": rf["peak"], "unit": "TFLOP/s",
                "frac": rf["frac"], "traffic": pmc["traffic"] if pmc else None,
                "traffic_source": pmc["source"] if pmc else None, "traffic_tree": pmc["tree"] if pmc else None,
                "frac_counts": rf["frac_counts"], "frac_lane_weighted": rf["frac_lane_weighted"], "stage": "ransac",
                "kernel": "RANSAC group: " + ", ".join(rf["kernels"]), "kernel_ms_per_launch": rf["ms_per_launch"],
                "note": "dominant stage = most HIP-event time per step; the RANSAC group is scalar f64 work "
                        "(5-point solve, Durand-Kerner, Sampson scoring), priced against the 78.6 TFLOP/s FP64 "
                        "vector peak; issue_frac in ransac_f64"}
    else:
        roof = hbm_roofline(dom, per_call[dom], W, H, N, B, m_avg) if dom != "ransac" else dict(hbm_dom or {})
    roof.update({"dominant_stage": dom,
                 "stage_ms_per_step": {k: round(v, 4) for k, v in per_call.items()},
                 "path_algorithmic_bytes_per_frame": algorithmic_bytes_per_frame(W, H, N, m_avg),
                 "path_frac": round(value * algorithmic_bytes_per_frame(W, H, N, m_avg) / 1e9 / HBM_PEAK_GBS, 8),
                 "hbm_dominant": hbm_dom, "ransac_f64": rf})
    return roof


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


def cpu_baseline(pool, K, nfeatures, max_iters, seconds, ref_equivalent=False):
    """The oracle (restated OpenCV path, C++ built -O3 -march=native for this
    host) on the same stream, in streaming mode (each frame detected once,
    its features reused by the next pair):
      single core   sequential pairs, the reference's execution model
                    (trajectory_evaluation_dual_process.py:172);
      all cores     the stream split into contiguous runs, one per thread
                    (ctypes releases the GIL inside the C++ calls), each run
                    sequential with feature reuse -- SURVEY.md §8d (2);
      reference-equivalent (ref_equivalent)  all cores again, but every pair
                    detects both of its frames, as visual_odometry_calculations
                    does (visual_odometry_v3.py:387-392).
    Each leg runs about `seconds`.  value = the all-cores streaming figure."""
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

    def worker(t, reuse):
        a = t * run
        if a + 1 >= len(pool):
            return
        kp = oracle.detect_and_compute(host(a), nfeatures) if reuse else None
        j = a
        while j + 1 < min(len(pool), a + run + 1) and time.perf_counter() < deadline:
            r = oracle.pair_pose(host(j), host(j + 1), K, nfeatures, max_iters=max_iters, kp_prev=kp)
            kp = (r["kp_cur"], r["desc_cur"]) if reuse else None
            done[t] += 1
            j += 1

    def all_threads(reuse):
        t1 = time.perf_counter()
        ths = [threading.Thread(target=worker, args=(t, reuse)) for t in range(T)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        return sum(done), time.perf_counter() - t1

    nn, dtn = all_threads(True)
    W, H = pool.shape[2], pool.shape[1]
    re = None
    if ref_equivalent:
        done[:] = [0] * T
        deadline = time.perf_counter() + seconds
        nr, dtr = all_threads(False)
        re = {"value": round(nr / dtr, 3), "cores": T,
              "sample": f"{nr} pairs in {dtr:.1f} s on {T} threads, both frames of every pair detected (v3:387-392)"}
    return ({"value": round(nn / dtn, 3), "unit": "frames/s", "cores": T, "kind": "port",
             "sample": f"{nn} pairs of the same {W}x{H} stream in {dtn:.1f} s on {T} threads (the stream split into "
                       f"{T} contiguous runs, each sequential with feature reuse; each run's first detect included); "
                       f"oracle/ C++ restatement of the OpenCV path built -O3 -march=native "
                       f"({os.path.basename(lib_path)})",
             "single_core": {"value": round(n1 / dt1, 3), "cores": 1,
                             "sample": f"{n1} consecutive pairs in {dt1:.1f} s, first frame's detect included"},
             "reference_equivalent": re,
             "host_cpus": os.cpu_count(), "cpu_model": model}, ref)


if __name__ == "__main__":
    main()
