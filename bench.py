"""bench.py — frames/s of integrate + global BA on a synthetic 640x480 stream at 4 mm voxels
(BASELINE.json metric), plus ms/GN-iter of the global solve.

A step is one submap (10 frames) of the reconstruction loop (bf_recon: per frame one integrate,
up to 10 re-integration queue ops and GC; per submap one local solve (11 frames, dense term on the
80x60 cache) and one global solve over all keyframes so far, with max-residual removal and the
trajectory update that feeds the queue). W warmup submaps run untimed, then K submaps are timed.
Every input (frames, cache frames, correspondences) is resident in HBM before timing starts.

Multi-GPU (torchrun, one process per GPU): the TSDF is sharded by 1 m chunk ownership
(every GPU sees every frame and integrates only the blocks it owns, no
collective); local BA solves run round-robin by submap with an RCCL broadcast of the solved poses;
the global solve shards its image-pair normal-equation blocks and all-reduces them over RCCL once
per GN iteration (§8(e)3). The host-side barrier / max-over-ranks uses gloo.

roofline: the dominant kernel is k_apply_ops, the op-batch voxel pass that applies a frame's
re-integration fixes (up to 10 de-integrate + integrate pairs = 20 voxel ops) with one read and one
write per voxel; its launches are timed with dispatch-stamped HIP events on the scene stream inside
the timed region. achieved = SURVEY.md §8(d)'s per-op algorithmic bytes of the integrate kernel
(8 B per pixel: depth + colour; 16 B per visible-list block; 24 B per voxel updated inside the
truncation band) x the ops one launch applies, from the device counters of the same launches, /
the average launch time. Because the batch reads and writes each voxel once for all its ops, the
pass itself moves far fewer bytes (alg_bytes_pass_per_launch: 20 B per work-list block + 24 B per
voxel read + written + 8 B per pixel per op) and the measured HBM traffic (PMC) sits between the
two. The kernel is VALU-issue bound (projection + band test of every voxel for every op of its
block); roofline.valu reports that bound from the SQ_INSTS_VALU pass of the same command.
cpu_baseline: the CPU oracle (oracle/, serial C++ restatement) timed on a bounded sample of the
same workload on this host, scaled by the GPU run's op counts to frames/s.
"""
from __future__ import annotations

import argparse
import ctypes as C
import glob
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
# VALU issue peak: 256 CUs x 4 SIMD-32 x 2.4 GHz / 2 cycles per wave64 instruction (MI355X_MICROARCH.md
# "Wave scheduling": a SIMD issues a wave64 VALU instruction over 2 cycles; one wave alone needs 4)
VALU_PEAK_WAVE_INSTS_PER_US = 256 * 4 * 2400 / 2


# revision of k_apply_ops' memory behaviour: a PMC profile (profiles/apply_pass_pmc*.json) describes the
# kernel only for the revision it recorded (2: z-halves no op reaches are not loaded; 3: work-list entries
# through scalar loads one block ahead, issue priority in the op steps)
APPLY_PASS_REV = 3

def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def host_info() -> dict:
    """nproc, CPU model, OMP threads and measured memory GB/s of this host."""
    import ctypes as C_
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_lib import lib as olib
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    L = olib()
    L.or_host_membw.restype = C_.c_double
    L.or_host_membw.argtypes = [C_.c_size_t, C_.c_int, C_.c_void_p]
    thr = C_.c_int()
    gbs = L.or_host_membw(1 << 30, 4, C_.byref(thr))
    return {"nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)), "cpu_model": model,
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS"), "omp_threads": thr.value,
            "host_mem_copy_GBps": gbs}


SHARD_CHUNK = 0.25  # metres: edge of the ownership chunks of the multi-GPU TSDF sharding (balance: DESIGN §6)
# The CPU oracle's loop prefix (500 frames): it runs whole 10-frame steps until
# PREFIX_FRAMES frames or the time budget, whichever comes first. At the north-star shape the oracle
# costs ~2 s per steady-state frame on the box's 16-thread CPU share (21 TSDF ops of 640x480 per frame),
# so 500 frames take ~15 min: the default bench caps the prefix by --cpu-prefix-budget (the bench must
# finish within minutes); `--cpu-prefix-budget 0` runs all 500. The GPU's time for the same prefix
# comes from synchronized checkpoints every PREFIX_STEP frames of the (untimed) fill.
PREFIX_FRAMES = 500
PREFIX_STEP = 10
PREFIX_BUDGET_S = 45.0


def oracle_threads() -> tuple[int, str]:
    """The thread count the CPU oracle runs with, set explicitly: the CPU share the pool gives this
    process (OMP_NUM_THREADS, which the GPU boxes export as their share), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.strip().isdigit() and int(env) > 0:
        return int(env), "OMP_NUM_THREADS (the box's CPU share)"
    return len(os.sched_getaffinity(0)), "sched_getaffinity"


def cpu_loop_prefix(stream, params, n_frames=PREFIX_FRAMES, budget_s=PREFIX_BUDGET_S):
    """The CPU oracle running the reconstruction loop itself on the stream's first frames: the
    OnlineBundler state machine + TrajectoryManager restatement (oracle/recon.cpp: local solves with the
    dense term, verification, global solves, max-residual removal, queue) with every scene call it
    issues applied to the oracle TSDF (integrate / de-integrate / GC, OpenMP), over the first n_frames
    or the whole PREFIX_STEP-frame steps that fit in budget_s (0: no budget)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_lib import OracleScene
    from oracle_recon import OracleRecon
    P = stream.cam.imageWidth * stream.cam.imageHeight
    H = stream.cam.imageHeight
    n_max = min(stream.F - 1, n_frames)
    K = stream.K
    ora = OracleRecon(stream.F, stream.gt[0], stream.cache_intrinsics, max_keyframes=K + 1,
                      max_global_corr=max(1000, 25 * (K + 1) * K // 2))
    local = stream.local_corr.download()
    for s in range(min(stream.num_submaps, n_max // stream.S + 2)):
        ora.set_local_corr(s, local[stream.local_off[s]:stream.local_off[s] + stream.local_n[s]])
    ora.set_global_corr(stream.global_host, stream.global_prefix)
    scene = OracleScene(params)
    depth, color = {}, {}

    raw = getattr(stream, "raw_input", False)
    if raw:
        from oracle_lib import preprocess
        from bundlefusion_amd.io import preprocess_options
        popt = preprocess_options()
        W = stream.cam.imageWidth

    def frame(f):
        if f not in depth:
            if raw:  # the loop's per-frame CUDAImageManager::process, restated by the oracle (oracle/frames.cpp)
                du = stream.depth_u16.download_range(f * P * 2, P * 2).view(np.uint16).reshape(H, -1)
                cx = stream.rgbx.download_range(f * P * 4, P * 4).reshape(H, -1, 4)
                depth[f], color[f] = preprocess(popt, du, cx, (W, H))
            else:
                depth[f] = stream.depth.download_range(f * P * 4, P * 4).view(np.float32).reshape(H, -1)
                color[f] = stream.color.download_range(f * P * 4, P * 4).reshape(H, -1, 4)
        return depth[f], color[f]

    for f in range(n_max + 1):
        ora.set_frame(f, stream.tinc[f], stream.cache_store.download(f))
    done, ops = 0, 0
    t0 = time.perf_counter()
    last = t0
    while done < n_max:
        if budget_s > 0 and done % PREFIX_STEP == 0 and done > 0 and time.perf_counter() - t0 > budget_s:
            break
        if time.perf_counter() - last > 20.0:
            log(f"  cpu oracle loop frame {done}")
            last = time.perf_counter()
        if raw:
            frame(done)  # preprocessing of the frame the loop takes in
        ora.process_frame(done)
        log_ = ora.op_log()
        for kind, f, oldT, newT in log_[ops:]:
            if kind == 1:
                scene.integrate(oldT.reshape(4, 4), *frame(f), stream.cam, deintegrate=True)
            elif kind == 2:
                scene.integrate(newT.reshape(4, 4), *frame(f), stream.cam)
            else:
                scene.garbageCollect()
        ops = len(log_)
        done += 1
    t = time.perf_counter() - t0
    st = ora.stats()
    n_tsdf = sum(1 for k, *_ in ora.op_log() if k in (1, 2))
    return {"frames": done, "s": t, "frames_per_s": done / t, "tsdf_ops": n_tsdf, "ops_per_frame": n_tsdf / done,
            "local_solves": st["localSolves"], "global_solves": st["globalSolves"], "frame_cap": n_max,
            "budget_s": budget_s,
            "cap_reason": None if done >= n_max else
            f"time budget {budget_s:.0f} s (the bench must finish within minutes; 500 frames take ~15 min of "
            f"oracle time on this CPU share; run bench.py --cpu-prefix-budget 0 for all {n_max})"}


def cpu_baseline(stream, params, gpu, prefix_frames=PREFIX_FRAMES, prefix_budget_s=PREFIX_BUDGET_S):
    """The CPU oracle (oracle/, C++ restatement built -O3 -fopenmp) on the box's host cores: TSDF
    integrate / de-integrate / GC on frames of the same stream, and one full global GN iteration
    (150 PCG iterations, the reference's global schedule) at the same (K, Nc) as the GPU's global
    solve. Frames/s = per-frame work at the GPU run's measured op mix (ops per frame, GN iterations
    per global solve)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_ba import matrix_to_pose, max_corr_per_image, solve
    from oracle_lib import OracleScene

    from oracle_lib import lib as olib
    nthr, thr_src = oracle_threads()
    L = olib()
    L.or_set_threads.restype = C.c_int
    L.or_set_threads.argtypes = [C.c_int]
    threads = L.or_set_threads(nthr)
    hi = host_info()
    t_start = time.perf_counter()
    prefix = cpu_loop_prefix(stream, params, prefix_frames, prefix_budget_s)
    gpu_t = gpu.get("prefix_times", {}).get(prefix["frames"])
    prefix["gpu_s"] = gpu_t
    prefix["gpu_frames_per_s"] = prefix["frames"] / gpu_t if gpu_t else None
    P = stream.cam.imageWidth * stream.cam.imageHeight
    ora = OracleScene(params)
    n = min(6, stream.F)
    depth = [stream.depth.download_range(f * P * 4, P * 4).view(np.float32).reshape(stream.cam.imageHeight, -1)
             for f in range(n)]
    color = [stream.color.download_range(f * P * 4, P * 4).reshape(stream.cam.imageHeight, -1, 4) for f in range(n)]
    t0 = time.perf_counter()
    for f in range(n):
        ora.integrate(stream.gt[f], depth[f], color[f], stream.cam)
    t_int = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    for f in range(2):
        ora.integrate(stream.gt[n - 1 - f], depth[n - 1 - f], color[n - 1 - f], stream.cam, deintegrate=True)
    t_deint = (time.perf_counter() - t0) / 2
    t0 = time.perf_counter()
    ora.garbageCollect()
    t_gc = time.perf_counter() - t0
    del ora
    # one global GN iteration with the full 150-iteration PCG at the GPU solve's (K, Nc)
    K = gpu["keyframes"]
    ncorr = int(stream.global_prefix[K - 1])
    corr = stream.global_host[:ncorr]
    rot = np.zeros((K, 3), np.float32)
    trans = np.zeros((K, 3), np.float32)
    for k in range(K):
        rot[k], trans[k] = matrix_to_pose(stream.gt[k * stream.S])
    maxc = max_corr_per_image(K + 1, 25 * (K + 1) * K // 2)
    t0 = time.perf_counter()
    _, _, _, res = solve(corr, np.ones(K, np.int32), rot, trans, 1, 150, [1.0], max_corr_per_img=maxc)
    t_gn = time.perf_counter() - t0
    per_solve = gpu["gn_per_solve"] * t_gn * (gpu["pcg_per_solve"] / max(gpu["gn_per_solve"], 1e-9)) / \
        max(1, res["pcgIterations"])
    ops_per_frame = gpu["ops_per_frame"]
    frame_s = ops_per_frame * (t_int + t_deint) / 2.0 + t_gc + per_solve / stream.S
    sample = (f"the oracle loop (bundling state machine + queue + TSDF, oracle/recon.cpp + tsdf.cpp) over the "
              f"stream's first {prefix['frames']} frames ({prefix['ops_per_frame']:.1f} TSDF ops/frame, "
              f"{'cap: ' + prefix['cap_reason'] if prefix['cap_reason'] else 'uncapped'}): "
              f"{prefix['frames_per_s']:.3f} frames/s = value; the GPU loop over the same prefix: "
              f"{(prefix['gpu_frames_per_s'] or 0):.0f} frames/s; steady-state estimate: oracle TSDF: {n} integrates + 2 de-integrates + 1 GC at {stream.cam.imageWidth}x"
              f"{stream.cam.imageHeight} @ {params.virtualVoxelSize * 1000:.0f} mm ({t_int * 1e3:.0f} / "
              f"{t_deint * 1e3:.0f} / {t_gc * 1e3:.0f} ms per call); oracle global GN iteration at K={K}, "
              f"Nc={ncorr}: {t_gn * 1e3:.0f} ms for {res['pcgIterations']} PCG iterations; frames/s at the GPU "
              f"run's {ops_per_frame:.2f} ops/frame and {gpu['pcg_per_solve']:.1f} PCG iterations per global solve "
              f"(local solves not counted); {time.perf_counter() - t_start:.0f} s of CPU work")
    return {"value": prefix["frames_per_s"], "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": sample, "loop_prefix": prefix, "steady_state_frames_per_s": 1.0 / frame_s,
            "gpu_prefix_frames_per_s": prefix["gpu_frames_per_s"],
            "ms_per_gn_iter": t_gn * 1e3, "host": hi, "threads": threads, "threads_source": thr_src,
            "threading": "set explicitly (or_set_threads); TSDF integrate / de-integrate / GC: OpenMP over "
                         "blocks; BA: OpenMP over correspondences and images with order-preserving reductions "
                         "(bit-identical to the serial oracle)"}


def global_solve_timing(stream, K, reps=3):
    """ms per GN iteration of a standalone global solve (3 GN x 150 PCG, the reference's global
    schedule) over the final K keyframes and their correspondences, timed with HIP events on the
    solver stream (no TSDF work competing for the CUs)."""
    import bundlefusion_amd as bfa
    from bundlefusion_amd.solver import SolverBundling
    rng = np.random.default_rng(7)
    kf = stream.gt[::stream.S][:K].astype(np.float64)
    T = np.empty((K, 4, 4), np.float32)
    D = np.eye(4)
    for k in range(K):  # GT with a random-walk drift (0.05 deg, 2 mm per keyframe), SURVEY §8(d)
        if k:
            w = rng.normal(size=3) * np.deg2rad(0.05)
            th = np.linalg.norm(w)
            A = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]]) / th
            step = np.eye(4)
            step[:3, :3] = np.eye(3) + np.sin(th) * A + (1 - np.cos(th)) * A @ A
            step[:3, 3] = rng.normal(size=3) * 0.002
            D = D @ step
        T[k] = (kf[k] @ D).astype(np.float32)
    n = int(stream.global_prefix[K - 1])
    S = SolverBundling(K + 1, max(1000, 25 * (K + 1) * K // 2))
    dT = bfa.DeviceArray.from_host(T)
    dv = bfa.DeviceArray.from_host(np.ones(K, np.int32))
    dr = bfa.DeviceArray((K, 3), np.float32)
    dt = bfa.DeviceArray((K, 3), np.float32)
    corr = bfa.DeviceArray.from_host(stream.global_host[:n])
    L = bfa.lib()
    timer = C.c_void_p()
    bfa.check(L.bf_timer_create(C.byref(timer)))
    pcg_ms, pcg_n = C.c_double(), C.c_uint64()
    ms_tot, gn_tot, pcg_tot = 0.0, 0, 0
    for r in range(reps + 1):
        corr.upload(stream.global_host[:n])
        S.matrices_to_poses(dT, K, dr, dt, dv)
        S.synchronize()
        ms = C.c_float()
        if r == 1 and hasattr(L, "bf_solver_pcg_time"):  # the persistent PCG launches' own device time
            bfa.check(L.bf_solver_pcg_time(S.h, 1, None, None))
        bfa.check(L.bf_solver_timer_start(S.h, timer))
        S.solve(corr, n, dv, K, 3, 150, [1.0, 1.0, 1.0], rot=dr, trans=dt)
        bfa.check(L.bf_solver_timer_stop(S.h, timer, C.byref(ms)))
        res = S.result()
        if r:  # first solve is warmup
            ms_tot += ms.value
            gn_tot += res["gnIterations"]
            pcg_tot += res["pcgIterations"]
    if hasattr(L, "bf_solver_pcg_time"):
        bfa.check(L.bf_solver_pcg_time(S.h, 0, C.byref(pcg_ms), C.byref(pcg_n)))
    bfa.check(L.bf_timer_destroy(timer))
    S.close()
    g = stream.global_host[:n]
    ok = (g["i"] < K) & (g["j"] < K)
    pairs = int(np.unique(np.minimum(g["i"][ok], g["j"][ok]).astype(np.int64) * K + np.maximum(g["i"][ok], g["j"][ok])).size)
    return {"ms_per_gn_iter": ms_tot / max(1, gn_tot), "keyframes": K, "correspondences": n, "image_pairs": pairs,
            "gn_iters": gn_tot / reps, "pcg_iters": pcg_tot / reps, "ms_per_solve": ms_tot / reps,
            "pcg_kernel_us_per_iter": pcg_ms.value * 1e3 / max(1, pcg_tot) if pcg_n.value else None}


def roofline_ba(solo):
    """The global PCG against HBM: SURVEY / VERDICT's matrix-free per-iteration bytes (140 B per
    correspondence: its two 32-B row entries, T_i p_i / T_j p_j and p gathers of the reference's
    applyJ + applyJT; 288 B per image of vector traffic) and the bytes the assembled path moves per
    iteration (k_pcg_persist: each pair orientation's partner p, 32 B — pair statistics and row entries
    stay in registers across iterations — plus 160 B per image: own p, Ap out and in as granules, new p),
    each divided by the standalone solve's time per PCG iteration (GN-step overheads included)."""
    N, Nc, Np = solo["keyframes"], solo["correspondences"], solo.get("image_pairs", 0)
    per_iter_s = solo["ms_per_solve"] / max(1e-9, solo["pcg_iters"]) * 1e-3
    b_mf = 140.0 * Nc + 288.0 * N
    b_asm = 2.0 * Np * 32.0 + 160.0 * N
    return {"bound": "latency", "kernel": "k_pcg_persist (all PCG iterations of a GN step in one launch)",
            "us_per_pcg_iter": per_iter_s * 1e6, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "bytes_assembled": b_asm, "achieved_assembled": b_asm / per_iter_s / 1e9,
            "frac_assembled": b_asm / per_iter_s / 1e9 / HBM_PEAK_GBS,
            "matrix_free_equivalent": {"bytes": b_mf, "GBps": b_mf / per_iter_s / 1e9,
                                       "note": "SURVEY 8(d)'s matrix-free bytes per iteration over the same time: an "
                                               "equivalent rate only (the assembled path does not move these bytes), "
                                               "so no fraction of peak"},
            "note": "the assembled normal equations move ~50x fewer bytes per iteration than the matrix-free "
                    "formula: the iteration is bound by its two hand-offs (Ap to the finisher, p back), not HBM"}


def sens_main(args):
    """FriedLiver over a .sens (BASELINE configs 2 / 3 when copyroom.sens / apt0.sens are present). Multi-GPU
    (torchrun, one app per GPU, every rank on the same .sens and parameters): the TSDF is chunk-sharded over
    the ranks, local solves run round-robin by submap with an RCCL broadcast of their poses, the global solve
    all-reduces its pair statistics; frames/s = frames / max over ranks of the loop time."""
    import tempfile

    import bundlefusion_amd as bfa
    from bundlefusion_amd.app import FriedLiver
    from bundlefusion_amd.dist import Comm, HostGroup, env_rank, input_digest
    from bundlefusion_amd.io import SensorData
    from bundlefusion_amd.params import NORTH_STAR_APP, write_parameter_files
    rank, world, local_rank = env_rank()
    group = HostGroup(rank, world)
    bfa.check(bfa.lib().bf_set_device(local_rank % max(1, bfa.device_count())))
    tmp = tempfile.mkdtemp(prefix="bf_sens_")
    pa, pb = args.app_params, args.bundling_params
    n = len(SensorData(args.sens))
    if not (pa and pb):
        pa, pb = write_parameter_files(tmp, NORTH_STAR_APP, {"s_maxNumImages": max(1200, n // 10 + 2)}, sens=args.sens)
    group.agree("the .sens and parameter files", input_digest([args.sens, pa, pb]))
    app = FriedLiver(pa, pb, args.sens, output_dir=tmp, skip_outputs=True, enable_timing=True, shard=(world, rank),
                     shard_chunk=args.shard_chunk if world > 1 else 0.0, result_lag=args.result_lag)
    comm = None
    if world > 1:
        comm = Comm(group)
        app.set_comm(comm)
    log(f"{args.sens}: {app.num_frames} frames, rank {rank} of {world}")
    group.barrier()
    t0 = time.perf_counter()
    done, last = 0, t0
    while app.step():
        done += 1
        if time.perf_counter() - last > 20.0:
            log(f"  frame {done}")
            last = time.perf_counter()
    rc = app.recon
    rc.synchronize()
    dt = time.perf_counter() - t0
    group.barrier()
    dt = group.max(dt)
    st = rc.stats()
    cap = rc.scene_capacity()
    tm = app.timing()
    res = app.finish()
    out = {"metric": f"frames/s FriedLiver pipeline on {os.path.basename(args.sens)}",
           "value": done / dt if cap["errorFlags"] == 0 else None,
           "unit": "frames/s", "n_gpus": world, "steps": done, "warmup": 0, "ms_per_step": dt / max(1, done) * 1e3,
           "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
           "data": f"{args.sens} (.sens input; EntryJ from the stand-in producer)",
           "config": {"workload": f"FriedLiver over {os.path.basename(args.sens)}: {done} frames, parameters {pa}, {pb}",
                      "parallelism": (f"tsdf-chunk-shard{world}+local-round-robin+ba-pair-shard{world}-rccl"
                                      if world > 1 else "single"),
                      "note": "whole pipeline per frame: .sens decode (prefetch threads), H2D, preprocessing, cache, "
                              "EntryJ stand-in, re-integration queue + integrate, local/global BA; not HBM-resident"},
           "loop": {k: st[k] for k in ("frames", "integrations", "deintegrations", "localSolves", "globalSolves",
                                       "globalGnIterations", "globalPcgIterations", "removedPairs", "invalidLocals")},
           "end_phase": {k: res["end"][k] for k in ("pastEndFrames", "globalSolves", "localSolved", "denseSolve",
                                                     "queueDrained", "denseSolveMs")},
           "host": {"decode_wait_ms_per_frame": tm["decodeWaitSeconds"] * 1e3 / max(1, done),
                    "upload_preprocess_ms_per_frame": tm["uploadSeconds"] * 1e3 / max(1, done),
                    "entryj_ms_per_frame": tm["corrSeconds"] * 1e3 / max(1, done),
                    "loop_ms_per_frame": tm["loopSeconds"] * 1e3 / max(1, done),
                    "decode_ms_per_frame_per_thread": tm["decodeSeconds"] * 1e3 / max(1, done),
                    "decode_threads": tm["decodeThreads"],
                    "upload_GBps": tm["uploadBytes"] / max(1e-9, tm["uploadSeconds"]) / 1e9,
                    "loop_host_ms_per_frame": st["hostMs"] / max(1, st["frames"]),
                    "loop_host_wait_ms_per_frame": st["hostWaitMs"] / max(1, st["frames"]),
                    "note": "host time per frame inside bf_app_step by section (bf_app_timing); decode runs on "
                            "prefetch threads beside the loop, so only decode_wait is on the critical path"},
           "gpu": {"scene_kernel_ms_per_frame": (st["reintegrateKernelMs"] + st["integrateKernelMs"]) / max(1, done),
                   "scene_stream_busy": (st["reintegrateKernelMs"] + st["integrateKernelMs"]) / 1e3 / dt,
                   "apply_us_per_launch": st["reintegrateKernelMs"] * 1e3 / max(1, st["reintegrateLaunches"]),
                   "global_ms_per_gn_iter_in_loop": st["globalSolveMs"] / max(1, st["globalGnIterations"])},
           "scene_capacity": {"error_flags": cap["errorFlags"], "peak_candidates": cap["peakCandidates"],
                              "candidate_capacity": cap["candidateCapacity"], "heap_free": cap["heapFree"]},
           "end_phase_s": res["endSeconds"], "heap_free": res["heapFreeCount"],
           "valid_transforms": [res["numValidTransforms"], res["numTransforms"]], "mesh_triangles": res["meshTriangles"]}
    if rank == 0:
        print(json.dumps(out), flush=True)
    app.close()
    if comm is not None:
        comm.close()
    group.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--frames", type=int, default=None,
                    help="stream length (BASELINE north star: 5000 frames; --preset config5: 10000, config 5's length); "
                         "independent of --steps")
    ap.add_argument("--steps", type=int, default=50, help="timed submaps (10 frames each) at the stream's tail")
    ap.add_argument("--warmup", type=int, default=5, help="untimed submaps right before the timed ones")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--voxel", type=float, default=None)
    ap.add_argument("--buckets", type=int, default=None)
    ap.add_argument("--blocks", type=int, default=None)
    ap.add_argument("--preset", choices=["config1", "config5"], default="config1",
                    help="config1: BASELINE north star (640x480, 4 mm, 2^23 buckets, 2^21 blocks); config5: "
                         "1280x960 depth at 2 mm voxels over 10 000 frames (2^24 buckets, 2^23 blocks: a heap beyond the "
                         "reference's 2^22-block int32 voxel index); explicit size flags override")
    ap.add_argument("--rehearse-shards", type=int, default=0,
                    help="single process: run rank 0's share of a G-way TSDF-sharded job (scene chunk shard 0 "
                         "of G, bundling replicated) to measure one rank's per-frame cost without G GPUs")
    ap.add_argument("--shard-chunk", type=float, default=SHARD_CHUNK,
                    help="edge (m) of the TSDF ownership chunks when sharded over ranks")
    ap.add_argument("--async-bundling", type=int, default=1, choices=[1, 2],
                    help="1: solves issued from the frame loop onto their own streams; 2: from a bundling thread")
    ap.add_argument("--no-preprocess", action="store_true",
                    help="feed the rendered float depth straight into the loop instead of raw sensor frames "
                         "(ushort depth, RGBX) preprocessed per frame inside it (CUDAImageManager::process: erode x2, "
                         "bilateral filter, resample; DepthSensing.cpp:986)")
    ap.add_argument("--result-lag", type=int, default=20,
                    help="frames after its issue at which a submap's solved poses are applied (waiting if needed): "
                         "the run's op sequence is then repeatable; 0: picked up by polling as soon as done "
                         "(timing-dependent, like the reference's bundling thread)")
    ap.add_argument("--sens", default=None,
                    help="run the FriedLiver application (bf_app_*) over this .sens instead of the synthetic stream "
                         "(copyroom / apt0: BASELINE configs 2 and 3): decode, preprocessing, cache, EntryJ stand-in, "
                         "the loop, the end-of-sequence phase; frames/s of the whole pipeline")
    ap.add_argument("--app-params", default=None, help="with --sens: zParametersDefault.txt-style file (default: the "
                    "reference defaults at the north-star 640x480 / 4 mm, 2^23 buckets, 2^21 blocks)")
    ap.add_argument("--bundling-params", default=None, help="with --sens: zParametersBundlingDefault.txt-style file")
    ap.add_argument("--apply-xcd-run", type=int, default=0,
                    help="BFSceneOptions.applyXcdRun: work-list positions per XCD run of the voxel pass (0: the library's 64)")
    ap.add_argument("--apply-rounds", type=int, default=0,
                    help="BFSceneOptions.applyRounds: resident rounds of the voxel pass's grid (0: the library's 4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-prefix-frames", type=int, default=PREFIX_FRAMES,
                    help="cpu_baseline: frames of the oracle loop prefix (SURVEY.md §8(d): 500)")
    ap.add_argument("--cpu-prefix-budget", type=float, default=PREFIX_BUDGET_S,
                    help="cpu_baseline: seconds after which the oracle prefix stops at a 10-frame boundary (0: none)")
    ap.add_argument("--traffic", default=None,
                    help="JSON with per-launch HBM bytes of k_apply_ops from the PMC passes of "
                         "tools/profile_bench.sh (committed under profiles/); used only when its "
                         "workload equals this run's, else traffic is null. Default: the first "
                         "profiles/apply_pass_pmc*.json whose workload matches")
    args = ap.parse_args()
    preset = {"config1": dict(width=640, height=480, voxel=0.004, buckets=1 << 23, blocks=1 << 21, frames=5000),
              "config5": dict(width=1280, height=960, voxel=0.002, buckets=1 << 24, blocks=1 << 23, frames=10000)}[args.preset]
    for k, v in preset.items():
        if getattr(args, k) is None:
            setattr(args, k, v)

    if args.sens:
        return sens_main(args)

    from bundlefusion_amd.dist import HostGroup, env_rank
    rank, world, local_rank = env_rank()
    group = HostGroup(rank, world)  # host-side barrier / max only (gloo)

    import bundlefusion_amd as bfa
    from bundlefusion_amd.abi import BFSceneOptions
    from bundlefusion_amd.recon import Recon, recon_options
    from bundlefusion_amd.stream import SyntheticStream

    # one rank per GPU; more ranks than GPUs (a rehearsal of the multi-rank path on a smaller box)
    # share them round-robin
    bfa.check(bfa.lib().bf_set_device(local_rank % max(1, bfa.device_count())))
    S = 10
    # The stream is the BASELINE workload whatever --steps says: `frames` frames (+1 so that the
    # last submap has its S+1-th local frame). The untimed prefix ("fill": everything before the
    # timed submaps, warmup included) builds the scene and the keyframe set; the timed submaps are
    # the stream's tail, where the global solve runs at its largest K.
    frames_total = max(args.frames, S * (args.warmup + args.steps))
    F = frames_total + 1
    fill = frames_total - S * args.steps
    t_setup = time.perf_counter()
    # the dense-term cache frames are built inside the loop as each frame is processed
    # (Bundler::storeCachedFrame in OnlineBundler::processInput, OnlineBundler.cpp:199-204), so the
    # timed region includes CUDACache::storeFrame
    stream = SyntheticStream(F, width=args.width, height=args.height, submap=S, log=log, cache_source="loop",
                             raw_input=not args.no_preprocess)
    params = bfa.hash_params(voxel_size=args.voxel, num_buckets=args.buckets, num_blocks=args.blocks)
    K = stream.K
    opts = recon_options(F, enableTiming=1, asyncBundling=args.async_bundling, cacheWidth=80, cacheHeight=60, cacheIntrinsics=stream.cache_intrinsics,
                         maxKeyframes=K + 1, maxGlobalCorr=max(1000, 25 * (K + 1) * K // 2), resultLag=args.result_lag)
    so = BFSceneOptions()
    so.shardCount, so.shardIndex, so.shardChunk = world, rank, args.shard_chunk
    if world == 1 and args.rehearse_shards > 1:
        so.shardCount, so.shardIndex = args.rehearse_shards, 0
    so.applyXcdRun, so.applyRounds = args.apply_xcd_run, args.apply_rounds
    rc = Recon(params, stream.cam, opts, so)
    comm = None
    if world > 1 and os.environ.get("BF_BA_SHARD", "1") != "0":
        # global BA: image-pair normal-equation blocks sharded over the ranks, one RCCL all-reduce
        # per GN iteration; the PCG then runs replicated on every GPU
        from bundlefusion_amd.dist import Comm
        try:
            comm = Comm(group)
        except Exception as e:  # keep the job alive: bundling replicated on every rank instead
            log(f"rank {rank}: RCCL communicator failed ({e!r}); global BA replicated")
            comm = None
        # every rank must take the same path (one order of collectives)
        if group.max(0.0 if comm is not None else 1.0):
            if comm is not None:
                comm.close()
            comm = None
        if comm is not None:
            rc.set_comm(comm)
    stream.attach(rc)
    log(f"setup {time.perf_counter() - t_setup:.1f}s: {F} frames, {K} keyframes, "
        f"{len(stream.global_host)} global correspondences")

    def barrier():
        group.barrier()

    # visualizeFrame's render every frame (DepthSensing.cpp:790-793: compactify + CUDARayCastSDF::render after each
    # integration), off the metric per SURVEY 8(d) but part of the reference's frame body: the last frames of the
    # fill (as many as the timed tail, up to 200) run with it, between synchronizations -> frames_per_s_with_render
    render_frames = min(fill, S * min(args.steps, 20)) if world == 1 else 0
    render_from = fill - render_frames
    # the same number of frames right before it, without the render: the comparison rate for the window
    plain_from = max(0, render_from - render_frames) if render_frames else -1
    t_pw = None
    rp_loop = bfa.raycast_params(args.width, args.height, fx=stream.cam.fx, fy=stream.cam.fy)
    t_rw = None
    barrier()
    t_fill = time.perf_counter()
    last = t_fill
    prefix_times = {}
    for f in range(fill):
        if render_frames and f == plain_from:
            rc.synchronize()
            t_pw = time.perf_counter()
        if render_frames and f == render_from:
            rc.synchronize()
            t_rw = time.perf_counter()
            if t_pw is not None:
                t_pw = t_rw - t_pw
            rc.set_render(rp_loop)
        rc.process_frame(f)
        if (f + 1) % PREFIX_STEP == 0 and f + 1 <= PREFIX_FRAMES:
            # the prefixes the CPU loop baseline may run (untimed region): synchronized checkpoints
            rc.synchronize()
            prefix_times[f + 1] = time.perf_counter() - t_fill
        if time.perf_counter() - last > 20.0:
            log(f"  fill frame {f}")
            last = time.perf_counter()
    rc.synchronize()
    t_fill = time.perf_counter() - t_fill
    if t_rw is not None:
        t_rw = time.perf_counter() - t_rw
        rc.set_render(None)
    fill_stats = rc.stats()
    rc.reset_stats()
    barrier()
    rc.synchronize()
    t0 = time.perf_counter()
    for f in range(fill, frames_total):
        rc.process_frame(f)
    rc.synchronize()
    dt = time.perf_counter() - t0
    barrier()
    dt = group.max(dt)
    t_fill = group.max(t_fill)
    st = rc.stats()
    ss = rc.scene_stats()
    # a dropped block would have failed the loop (BF_ERR_CAPACITY); the line states the headroom it had
    cap = rc.scene_capacity()
    frames = S * args.steps
    P = args.width * args.height
    workload = (f"{frames_total}-frame {args.width}x{args.height} stream, {args.voxel * 1000:.0f} mm voxels, "
                f"2^{args.buckets.bit_length() - 1} buckets, 2^{args.blocks.bit_length() - 1} blocks; "
                f"local 2x100 + global 3x150 GN x PCG per submap; cache frames built in the loop; "
                f"{'rendered depth fed directly' if args.no_preprocess else 'raw frames preprocessed in the loop'}; "
                f"timed: last {args.steps} submaps")
    # a profile's counters describe one scheduling: a sharded rehearsal or another bundling mode is a
    # different workload (a rehearsal must not pick up the unsharded profile's counters)
    if world > 1 or args.rehearse_shards > 1:
        workload += f"; tsdf shard {so.shardIndex} of {so.shardCount} (chunk {so.shardChunk:g} m)"
    if args.async_bundling != 1:
        workload += f"; asyncBundling {args.async_bundling}"
    workload += (f"; solved poses applied {args.result_lag} frames after issue" if args.result_lag
                 else "; solved poses applied when polled ready (timing-dependent)")
    # dominant kernel: k_apply_ops, the op-batch voxel pass that applies a frame's re-integration
    # fixes (<= 10 x de-integrate + integrate) in one read + write per voxel. Per launch, from the
    # device counters of the same launches:
    #   the fused pass's own bytes (roofline.achieved / frac): 20 B per work-list block (16 B entry + 4 B op
    #     mask) + 12 B per voxel of every block z-half the pass loads (a half some op's mask reaches; 256
    #     voxels) + 12 B per voxel written back + 8 B per pixel per op (the op's {depth, colour} image)
    #   SURVEY §8(d) per-op bytes of the integrate kernel, summed over the launch's ops (what the reference's
    #     one pass per op moves; an equivalent rate only, so no fraction of peak):
    #     8 B per pixel per op + 16 B per visible-list block per op + 24 B per in-band voxel update
    launches = max(1, st["reintegrateLaunches"])
    kernel_ms = st["reintegrateKernelMs"]
    survey_bytes = 8 * P * ss["batchOps"] + 16 * ss["batchBlocks"] * (ss["batchOps"] / launches) + 24 * ss["batchUpdates"]
    pass_bytes = (20 * ss["batchBlocks"] + 12 * 256 * ss["batchHalves"] + 12 * ss["batchVoxelsRMW"]
                  + 8 * P * ss["batchOps"])
    per_launch_s = kernel_ms / 1e3 / launches
    achieved = pass_bytes / launches / per_launch_s / 1e9
    traffic = None
    valu = None
    traffic_src = None
    cands = [args.traffic] if args.traffic else sorted(glob.glob(os.path.join(REPO, "profiles", "apply_pass_pmc*.json")))
    tj = {}
    for c in cands:
        if c and os.path.exists(c):
            tj = json.load(open(c))
            if tj.get("workload") == workload and tj.get("pass_rev") == APPLY_PASS_REV:
                args.traffic = c
                break
    # counters are taken only from a profile of this same workload (tools/profile_bench.sh records
    # the workload string of the bench run it profiled and averages over its timed launches)
    evals_pl = ss["batchEvals"] / launches
    rmw_pl = ss["batchVoxelsRMW"] / launches
    traffic_units = None
    if tj.get("workload") == workload and tj.get("pass_rev") == APPLY_PASS_REV and world == 1 and args.rehearse_shards <= 1:
        traffic_src = os.path.relpath(args.traffic, REPO)
        if "fetch_bytes_per_evaluation" in tj:
            # the profile's per-unit rates x this run's own per-launch counts (identical to the profiled
            # run's when the hand-off is repeatable: --result-lag)
            traffic = tj["fetch_bytes_per_evaluation"] * evals_pl + tj["write_bytes_per_voxel_rmw"] * rmw_pl
            traffic_units = {"fetch_bytes_per_evaluation": tj["fetch_bytes_per_evaluation"],
                             "write_bytes_per_voxel_rmw": tj["write_bytes_per_voxel_rmw"],
                             "profiled_units_per_launch": tj.get("units_per_launch"),
                             "profiled_bytes_per_launch": tj.get("bytes_per_launch")}
        else:
            traffic = tj.get("bytes_per_launch")
        if "valu_insts_per_launch" in tj:  # VALU-issue bound of the same kernel (SQ_INSTS_VALU pass)
            us = per_launch_s * 1e6
            vpl = tj["valu_insts_per_evaluation"] * evals_pl if "valu_insts_per_evaluation" in tj else tj["valu_insts_per_launch"]
            valu = {"wave_insts_per_launch": vpl, "wave_insts_per_evaluation": tj.get("valu_insts_per_evaluation"),
                    "peak_wave_insts_per_us": VALU_PEAK_WAVE_INSTS_PER_US,
                    "frac": vpl / (us * VALU_PEAK_WAVE_INSTS_PER_US), "source": traffic_src}
    hbm_cnt = traffic / per_launch_s / 1e9 / HBM_PEAK_GBS if traffic else None
    bound = ("valu-issue/latency" if valu and hbm_cnt is not None and valu["frac"] > hbm_cnt else
             "latency" if hbm_cnt is None or hbm_cnt < 0.7 else "hbm")
    gn = max(1, st["globalGnIterations"])
    ms_gn_loop = st["globalSolveMs"] / gn
    solo = global_solve_timing(stream, K - 1)
    # end of sequence (after the timed region): the render loop past the last frame — the last submap,
    # s_numSolveFramesBeforeExit (30) global solves, the last with the dense depth term at weight 15
    # (USE_GLOBAL_DENSE_AT_END, OnlineBundler.cpp:167-196), re-integration until the queue is empty
    # (DepthSensing.cpp:1114-1126)
    t_end = time.perf_counter()
    end = rc.end_sequence(30)
    t_end = time.perf_counter() - t_end
    # the end phase's re-integration batches run k_apply_ops after the timed region: trace / PMC tools take
    # the timed region's dispatches as the `launches` before the last `launches_after` ones
    launches_after = rc.stats()["reintegrateLaunches"] - st["reintegrateLaunches"]
    dres = end["last"]
    dense_end = {"ms": end["denseSolveMs"], "keyframes": K - 1, "dense_pairs": dres["numDensePairs"],
                 "gn_iters": dres["gnIterations"], "pcg_iters": dres["pcgIterations"],
                 "ms_per_gn_iter": end["denseSolveMs"] / max(1, dres["gnIterations"]),
                 "end_phase": {k: end[k] for k in ("pastEndFrames", "globalSolves", "localSolved", "denseSolve",
                                                   "queueDrained")},
                 "end_phase_s": t_end,
                 "note": "bf_recon_end_sequence(30): 31 past-the-end global solves, the last with sparse weight 1 + "
                         "dense depth 15 (3 x 150 GN x PCG) over every keyframe's 80x60 cache frame, then re-integration "
                         "until the queue drains; untimed, after the timed tail"}
    out = {
        "metric": f"frames/s integrate+global-BA on {args.width}x{args.height} @{args.voxel * 1000:g}mm voxels",
        "value": frames / dt if cap["errorFlags"] == 0 else None,
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if world > 1 else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded analytic room, GPU-rendered depth/colour with the sensor noise model, "
                "EntryJ stand-in correspondences)",
        "config": {"workload": workload, "frames": frames_total, "frames_fill": fill, "frames_timed": frames,
                   "keyframes_final": K,
                   "parallelism": (f"tsdf-chunk-shard{world}+ba-pair-shard{world}-rccl" if comm is not None
                                   else f"tsdf-chunk-shard{world}+ba-replicated") if world > 1 else
                                  (f"rehearsal: rank 0 of tsdf-chunk-shard{args.rehearse_shards}, ba-replicated"
                                   if args.rehearse_shards > 1 else "single"),
                   **({"apply_xcd_run": args.apply_xcd_run} if args.apply_xcd_run else {}),
                   **({"apply_rounds": args.apply_rounds} if args.apply_rounds else {})},
        "stream": {"frames_per_s_whole_stream": frames_total / (t_fill + dt), "fill_s": t_fill, "timed_s": dt,
                   "fill_frames_per_s": fill / t_fill if fill else None,
                   "fill_global_gn_iters": fill_stats["globalGnIterations"],
                   "note": "whole stream = fill + timed tail, same loop; value is the tail (largest K, largest scene)"},
        "frames_per_s_with_render": (render_frames / t_rw) if t_rw else None,
        "render_in_loop": {"frames": render_frames, "frames_window": [render_from, fill], "s": t_rw,
                           "frames_per_s_window_before_without_render": ((render_from - plain_from) / t_pw) if t_pw else None,
                           "renders": fill_stats["renders"],
                           "note": "the fill's last frames with visualizeFrame's render after each frame's batch "
                                   "(bf_recon_set_render: compactify + splat + renderKernel + computeNormals at "
                                   f"{args.width}x{args.height}), between synchronizations; compare with "
                                   "frames_per_s_window_before_without_render (the as many frames right before it, "
                                   "no render), not with value (the timed tail: larger K and scene); the reference "
                                   "renders every frame for display, which SURVEY 8(d) keeps out of the metric"} if render_frames else None,
        "scene_capacity": {"error_flags": cap["errorFlags"], "peak_candidates": cap["peakCandidates"],
                           "candidate_capacity": cap["candidateCapacity"],
                           "candidate_headroom": cap["candidateCapacity"] / max(1, cap["peakCandidates"]),
                           "heap_free": cap["heapFree"], "num_sdf_blocks": cap["numSDFBlocks"],
                           "high_water": cap["highWater"],
                           "note": "peak alloc candidates of one batch over the whole stream vs the candidate "
                                   "buffer; nonzero error_flags (a dropped block) fail the loop and void value"},
        "ms_per_gn_iter": solo["ms_per_gn_iter"],
        "global_solve": dict(solo, ms_per_gn_iter_in_loop=ms_gn_loop,
                             pcg_kernel_us_per_iter_in_loop=(st["globalPcgKernelMs"] * 1e3 / max(1, st["globalPcgIterations"])
                                                             if st["globalPcgLaunches"] else None),
                             pcg_launches_in_loop=st["globalPcgLaunches"],
                             note="ms_per_gn_iter*: whole solves (table build, GN steps, per-solve overheads) per GN "
                                  "iteration; pcg_kernel_us_per_iter*: the persistent PCG launches' own device time per "
                                  "PCG iteration (dispatch-stamped events), standalone vs inside the loop"),
        "roofline_ba": roofline_ba(solo),
        "global_dense_end_solve": dense_end,
        "roofline": {"bound": bound, "kernel": "k_apply_ops (op-batch voxel pass)", "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_src, "traffic_units": traffic_units,
                     "hbm_frac_counters": (traffic / per_launch_s / 1e9 / HBM_PEAK_GBS) if traffic else None,
                     "launches": launches, "launches_after": launches_after,
                     "avg_launch_us": per_launch_s * 1e6, "pass_rev": APPLY_PASS_REV,
                     "alg_bytes_per_launch": pass_bytes / launches,
                     "alg_bytes_source": "the fused pass's own bytes: 20 B per work-list block + 12 B per voxel of each "
                                         "block z-half loaded (256 voxels; halves no op reaches are skipped) + 12 B per "
                                         "voxel written + 8 B per pixel per op",
                     "equivalent_GBps": survey_bytes / launches / per_launch_s / 1e9,
                     "survey_bytes_per_launch": survey_bytes / launches,
                     "survey_bytes_source": "SURVEY 8(d) per-op integrate bytes (8 P + 16 Nv + 24 V) x ops per launch: "
                                            "what one reference pass per op would move; the batch reads and writes each "
                                            "voxel once for all of its ops, so this is an equivalent rate, not a roofline "
                                            "position",
                     "note": "frac is the pass's own bytes against HBM peak (traffic / hbm_frac_counters: the PMC bytes "
                             "of the same launches); bound names the resource that binds: VALU issue and dependency "
                             "latency (valu.frac above the counters' HBM fraction), not HBM",
                     "per_launch": {"work_list_blocks": ss["batchBlocks"] / launches,
                                    "halves_loaded": ss["batchHalves"] / launches,
                                    "voxels_rmw": ss["batchVoxelsRMW"] / launches,
                                    "voxel_op_updates": ss["batchUpdates"] / launches,
                                    "voxel_op_evaluations": ss["batchEvals"] / launches,
                                    "ops": ss["batchOps"] / launches},
                     "valu": valu,
                     "k_integrate": {"launches": st["integrateLaunches"],
                                     "avg_us": st["integrateKernelMs"] * 1e3 / max(1, st["integrateLaunches"])}},
        "loop": {"ops_per_frame": (st["integrations"] + st["deintegrations"]) / max(1, st["frames"]),
                 "fix_ops": st["fixOps"], "local_solves": st["localSolves"], "global_solves": st["globalSolves"],
                 "global_gn_iters": st["globalGnIterations"], "global_pcg_iters": st["globalPcgIterations"],
                 "removed_pairs": st["removedPairs"], "global_solve_ms": st["globalSolveMs"],
                 "local_solve_ms": st["localSolveMs"], "integrate_kernel_ms": st["integrateKernelMs"],
                 "apply_kernel_ms": st["reintegrateKernelMs"],
                 "host_ms_per_frame": st["hostMs"] / max(1, st["frames"]),
                 "host_wait_ms_per_frame": st["hostWaitMs"] / max(1, st["frames"]),
                 "heap_free": rc.heap_free_count(),
                 "allocated_blocks_scanned_per_compactify": ss["scanned"] / max(1, ss["integrateOps"])},
    }
    # multi-GPU TSDF sharding: how evenly 1 m chunk ownership spreads the final
    # scene's blocks and the timed frames' in-frustum blocks over G = 2 / 4 / 8 ranks (host mirror)
    if world == 1:
        from bundlefusion_amd.dist import shard_balance
        blk = rc.export_blocks()
        blk = blk[blk[:, 3] != 0]
        poses_t = stream.gt[fill:frames_total:10]
        out["shard_balance"] = shard_balance(blk[:, :3], args.voxel, poses_t, stream.cam, chunk=args.shard_chunk)
        # max / mean over ranks of (stored blocks, in-frustum block-frames) for other ownership chunk sizes
        out["shard_balance"]["by_chunk"] = {
            f"{c:g}m": {g: [round(v["stored_max_over_mean"], 3), round(v["visible_max_over_mean"], 3)]
                        for g, v in shard_balance(blk[:, :3], args.voxel, poses_t, stream.cam, chunk=c).items()
                        if g.startswith("G")}
            for c in (1.0, 0.5, 0.25, 0.125)}
    # raycast (visualizeFrame's render, reported beside the metric): 20 renders from the last pose
    W_, H_ = args.width, args.height
    rpr = bfa.raycast_params(W_, H_, fx=stream.cam.fx, fy=stream.cam.fy)
    routs = [bfa.DeviceArray((H_, W_), np.float32)] + [bfa.DeviceArray((H_, W_, 4), np.float32) for _ in range(3)]
    Tlast = stream.gt[frames_total - 1]
    rc.render_time()  # enables the render clock
    rc.raycast_device(Tlast, rpr, routs)
    rc.synchronize()
    ms0, n0 = rc.render_time()
    rs0 = rc.render_stats()
    t_r = time.perf_counter()
    for _ in range(20):
        rc.raycast_device(Tlast, rpr, routs)
    rc.synchronize()
    t_r = (time.perf_counter() - t_r) / 20
    ms1, n1 = rc.render_time()
    rs1 = rc.render_stats()
    rdepth = routs[0].download()
    # SURVEY.md §8(d) raycast bytes: 96 B per trilinear sample (8 corner voxels x 12 B) + 52 B of output per
    # pixel (depth 4 + depth4 16 + normal 16 + colour 16), from the device counters of the same 20 renders
    nr = max(1, rs1["renders"] - rs0["renders"])
    samples = (rs1["samples"] - rs0["samples"]) / nr
    loads = (rs1["voxelLoads"] - rs0["voxelLoads"]) / nr
    k_render_us = (ms1 - ms0) / max(1, n1 - n0) * 1e3
    splat_us = (rs1["splatMs"] - rs0["splatMs"]) / max(1, rs1["timedRenders"] - rs0["timedRenders"]) * 1e3
    rbytes = 96.0 * samples + 52.0 * W_ * H_
    atomics = (rs1["splatAtomics"] - rs0["splatAtomics"]) / nr
    out["raycast"] = {"ms_per_render": t_r * 1e3, "k_render_us": k_render_us,
                      "valid_fraction": float(np.isfinite(rdepth).mean()),
                      "per_render": {"samples": samples, "voxel_loads": loads,
                                     "hash_probes": (rs1["hashProbes"] - rs0["hashProbes"]) / nr,
                                     "rays": (rs1["rays"] - rs0["rays"]) / nr,
                                     "splat_blocks": (rs1["splatBlocks"] - rs0["splatBlocks"]) / nr,
                                     "splat_atomics": atomics, "k_splat_us": splat_us,
                                     "march_lane_efficiency": (rs1["samples"] - rs0["samples"]) /
                                                              max(1, rs1["waveSamples"] - rs0["waveSamples"]),
                                     "long_waves": (rs1["longWaves"] - rs0["longWaves"]) / nr,
                                     "wave_samples_max": rs1["waveSamplesMax"]},
                      "roofline": {"bound": "latency", "kernel": "k_render (renderKernel)", "unit": "GB/s",
                                   "alg_bytes_per_render": rbytes, "achieved": rbytes / (k_render_us * 1e-6) / 1e9,
                                   "peak": HBM_PEAK_GBS, "frac": rbytes / (k_render_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                                   "loaded_bytes_per_render": 12.0 * loads + 52.0 * W_ * H_,
                                   "note": "SURVEY 8(d): 96 B per trilinear sample + 52 B per pixel; a sample's voxels "
                                           "are dependent loads of one ray (hash probe -> 8 corners -> next step), so "
                                           "the march is bound by load latency, not bandwidth"},
                      "splat_roofline": {"kernel": "k_splat_quads + k_splat_tiles (ray-interval splat)",
                                         "pixel_updates_per_render": atomics,
                                         "pixel_updates_per_us": atomics / max(1e-9, splat_us),
                                         "note": "per covered pixel one min (near pass) and one max (far pass), folded in "
                                                 "registers per 64x8 tile from the block rectangles that overlap it "
                                                 "(no global atomics)"},
                      "note": f"compactify + interval splat + renderKernel + computeNormals at {W_}x{H_} from the last pose"}
    # marching cubes over the final scene (StopScanningAndExtractIsoSurfaceMC, reported beside the metric)
    mcp = bfa.mc_params(params.virtualVoxelSize)
    mbuf = bfa.DeviceArray((mcp.maxNumTriangles, 3, 6), np.float32)
    rc.extract_mesh_device(mcp, mbuf)  # warm
    t_m = time.perf_counter()
    nt, tt = rc.extract_mesh_device(mcp, mbuf)
    t_m = time.perf_counter() - t_m
    out["mesh"] = {"ms_extract": t_m * 1e3, "triangles": nt, "triangles_total": tt,
                   "allocated_blocks": int(params.numSDFBlocks - rc.heap_free_count()),
                   "note": "marching cubes over every allocated block (count + scan + emit), 3M-triangle cap"}
    del mbuf
    # the metric's config, rank 0 of a one-GPU run only (the multi-GPU lines carry no CPU leg)
    if world == 1 and rank == 0 and not args.no_cpu_baseline and args.preset == "config1":
        gpu = {"keyframes": K - 1, "global_corr": solo["correspondences"],
               "gn_per_solve": st["globalGnIterations"] / max(1, st["globalSolves"]),
               "pcg_per_solve": st["globalPcgIterations"] / max(1, st["globalSolves"]),
               "ops_per_frame": out["loop"]["ops_per_frame"],
               "prefix_times": prefix_times}
        try:
            out["cpu_baseline"] = cpu_baseline(stream, params, gpu, args.cpu_prefix_frames, args.cpu_prefix_budget)
        except Exception as e:  # the baseline is reported, not the target: keep the GPU line
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    rc.close()
    if comm is not None:
        comm.close()
    group.close()


if __name__ == "__main__":
    main()
