"""GPU: the reconstruction loop (bf_recon_*: integrate + re-integration queue + local/global BA).

* Replay parity: every scene call the loop issued (integrate / de-integrate / GC, with the exact
  transforms the queue chose) is replayed through the CPU oracle scene on the same frames; the final
  voxel hash must be bit-identical (block set, buckets, heap, sdf/weight/colour bits).
* Queue invariants: a frame is only de-integrated with the transform it was last integrated with,
  and never integrated twice without a de-integration in between (TrajectoryManager.cpp:117-170).
* The loop's poses beat the front end's dead reckoning against ground truth (local + global BA
  with re-integration actually corrects the trajectory).
"""
import ctypes as C

import numpy as np
import pytest

import bundlefusion_amd as bfa
from bundlefusion_amd.recon import FIX_DEINTEGRATE, FIX_INTEGRATE, OP_GC, Recon, recon_options
from bundlefusion_amd.stream import SyntheticStream
from oracle_lib import OracleScene, blocks_of
from tsdf_compare import compare_states

pytestmark = pytest.mark.gpu


def run_loop(F=40, W=160, H=120, voxel=0.01, record=True, drift=(0.05, 0.002), async_ba=0, outliers=0.0):
    # outlier-free correspondences: with 4 keyframes a single solve cannot yet have removed the
    # 0.1-0.3 m outliers of the newest pairs, and this loop checks drift removal, not robustness
    st = SyntheticStream(F, width=W, height=H, drift=drift, outliers=outliers)
    params = bfa.hash_params(voxel_size=voxel, num_buckets=1 << 16, num_blocks=1 << 15)
    K = st.K
    opts = recon_options(F, recordOps=int(record), cacheWidth=80, cacheHeight=60, cacheIntrinsics=st.cache_intrinsics,
                         maxGlobalCorr=max(1000, 25 * K * (K - 1) // 2), maxKeyframes=K + 1, asyncBundling=async_ba)
    rc = Recon(params, st.cam, opts)
    st.attach(rc)
    for f in range(F):
        rc.process_frame(f)
    rc.finish()  # last submap's solves; then let the queue catch up as the render loop would
    for _ in range(30):
        rc.reintegrate()
    rc.synchronize()
    return st, params, rc


@pytest.fixture(scope="module", params=[0, 1, 2], ids=["sync", "async", "thread"])
def loop(request):
    return run_loop(async_ba=request.param)


def test_replay_parity_bit_exact(loop):
    st, params, rc = loop
    ops = rc.op_log()
    kinds = [k for k, _, _, _ in ops]
    assert kinds.count(FIX_DEINTEGRATE) > 0 and kinds.count(OP_GC) == st.F + 30
    depth = st.depth.download()
    color = st.color.download()
    ora = OracleScene(params)
    for kind, f, oldT, newT in ops:
        if kind == FIX_DEINTEGRATE:
            ora.integrate(oldT.reshape(4, 4), depth[f], color[f], st.cam, deintegrate=True)
        elif kind == FIX_INTEGRATE:
            ora.integrate(newT.reshape(4, 4), depth[f], color[f], st.cam)
        elif kind == OP_GC:
            ora.garbageCollect()
    n = compare_states(params, rc, ora)
    assert n > 100


def test_queue_invariants(loop):
    st, _, rc = loop
    current = {}
    for kind, f, oldT, newT in rc.op_log():
        if kind == FIX_INTEGRATE:
            assert f not in current, f"frame {f} integrated twice"
            current[f] = newT
        elif kind == FIX_DEINTEGRATE:
            assert f in current, f"frame {f} de-integrated while not integrated"
            np.testing.assert_array_equal(current.pop(f), oldT)
    traj = rc.trajectory(st.F)
    for f in range(st.F):
        np.testing.assert_array_equal(traj[f].reshape(16), current[f])


def test_loop_corrects_drift(loop):
    st, _, rc = loop
    s = rc.stats()
    assert s["localSolves"] == st.num_submaps
    assert s["globalSolves"] >= st.num_submaps - 1
    assert s["fixOps"] > 0 and s["deintegrations"] > 0
    # dead reckoning of the front end vs the poses the volume holds now
    dr = [st.gt[0].astype(np.float64)]
    for f in range(1, st.F):
        dr.append(dr[-1] @ st.tinc[f].astype(np.float64))
    traj = rc.trajectory(st.F)
    err_dr = np.array([np.linalg.norm(dr[f][:3, 3] - st.gt[f][:3, 3]) for f in range(st.F)])
    err_loop = np.array([np.linalg.norm(traj[f][:3, 3] - st.gt[f][:3, 3]) for f in range(st.F)])
    settled = st.F
    assert np.mean(err_loop[:settled]) < 0.5 * np.mean(err_dr[:settled]), (err_loop[:settled], err_dr[:settled])


def test_loop_redoes_timed_out_persistent_pcg():
    """The loop never consumes a timed-out persistent PCG solve. With every wait of the persistent launch
    bounded by 1 us (BFSolverOptions.pcgSpinLimitUs) each global solve above 64 keyframes times out and
    its GN steps are redone in stream order (pcg_recover in k_gn_end): the loop counts them (pcgRecoveries) and its
    scene calls, trajectory and submap poses are bit-identical to a loop that runs one launch per PCG
    iteration (pcgLaunch = 1)."""
    F, S = 216, 3  # 72 keyframes: the global solves from keyframe 65 on take the persistent route
    st = SyntheticStream(F, width=80, height=60, submap=S, drift=(0.05, 0.002), outliers=0.0, cache_w=40,
                         cache_h=30)
    params = bfa.hash_params(voxel_size=0.02, num_buckets=1 << 14, num_blocks=1 << 13)
    K = st.K
    runs = []
    for launch, spin in ((1, 0), (0, 1)):
        opts = recon_options(F, recordOps=1, submapSize=S, cacheWidth=40, cacheHeight=30,
                             cacheIntrinsics=st.cache_intrinsics, maxGlobalCorr=max(1000, 25 * K * (K - 1) // 2),
                             maxKeyframes=K + 1, asyncBundling=0)
        opts.solver.pcgLaunch = launch
        opts.solver.pcgSpinLimitUs = spin
        rc = Recon(params, st.cam, opts)
        st.attach(rc)
        for f in range(F):
            rc.process_frame(f)
        rc.finish()
        rc.synchronize()
        runs.append((rc.stats(), rc.trajectory(F), rc.op_log(),
                     [rc.submap_poses(s, K + 1, S)[1] for s in range(st.num_submaps - 1)]))
        rc.close()
    (s1, t1, o1, g1), (s0, t0, o0, g0) = runs
    assert s1["pcgRecoveries"] == 0
    assert s0["pcgRecoveries"] >= K - 66, s0["pcgRecoveries"]  # every global solve above 64 keyframes
    assert s0["globalSolves"] == s1["globalSolves"] and s0["globalPcgIterations"] == s1["globalPcgIterations"]
    np.testing.assert_array_equal(t0, t1)
    assert len(o0) == len(o1)
    for a, b in zip(o0, o1):
        assert a[0] == b[0] and a[1] == b[1]
        np.testing.assert_array_equal(a[2], b[2])
        np.testing.assert_array_equal(a[3], b[3])
    for a, b in zip(g0, g1):
        np.testing.assert_array_equal(a, b)


def test_loop_preprocesses_raw_frames_in_order():
    """CUDAImageManager::process inside the loop (bf_recon_attach_preproc + bf_recon_set_frame_raw): each raw
    sensor frame (ushort depth, RGBX) is preprocessed into its frame-store slot when the loop reaches it, on
    the preprocessor's stream, with the scene stream ordered after it. The loop must then do exactly what a
    loop over frames preprocessed beforehand does: the same scene calls, trajectory and voxels, bit for bit,
    in the synchronous and the asynchronous bundling modes. Mode "ready": each frame preprocessed outside the
    loop right before it is processed, on the preprocessor's own stream with no host wait, the loop ordered
    after it by bf_recon_frame_ready alone (the FriedLiver app's input path). With cache_source "loop" the
    attached cache (its own stream) builds each cache frame from the frame store inside process_frame: in
    "ready" mode its stream must wait for the caller's preprocessing too (the cache frames feed the local
    solves, so a cache that read a frame early changes the local poses)."""
    from bundlefusion_amd.io import Preprocessor, preprocess_options
    F, W, H = 40, 160, 120
    results = []
    runs = [(m, a, "synth") for m in ("in_loop", "before", "ready") for a in (0, 1)]
    runs += [("before", 1, "loop"), ("ready", 1, "loop")]
    for mode, async_ba, cache_source in runs:
        st = SyntheticStream(F, width=W, height=H, drift=(0.05, 0.002), outliers=0.0, cache_source=cache_source,
                             raw_input=True)
        if mode == "before":  # preprocess every frame up front into the frame store
            pre = Preprocessor((W, H), (W, H), (W, H), preprocess_options())
            P = W * H
            for f in range(F):
                lib_ = bfa.lib()
                bfa.check(lib_.bf_preproc_run(pre.h, C.c_void_p(st.depth_u16.ptr.value + 2 * P * f),
                                              C.c_void_p(st.rgbx.ptr.value + 4 * P * f),
                                              C.c_void_p(st.depth.ptr.value + 4 * P * f),
                                              C.c_void_p(st.color.ptr.value + 4 * P * f)))
            bfa.check(bfa.lib().bf_preproc_synchronize(pre.h))
            st.raw_input = False  # attach() then registers no raw frames
        pre_async = None
        if mode == "ready":  # preprocessed outside the loop, frame by frame, ordered by bf_recon_frame_ready only
            pre_async = Preprocessor((W, H), (W, H), (W, H), preprocess_options())
            st.raw_input = False
        params = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 16, num_blocks=1 << 15)
        K = st.K
        opts = recon_options(F, recordOps=1, cacheWidth=80, cacheHeight=60, cacheIntrinsics=st.cache_intrinsics,
                             maxGlobalCorr=max(1000, 25 * K * (K - 1) // 2), maxKeyframes=K + 1,
                             asyncBundling=async_ba, resultLag=10 if async_ba else 0)
        rc = Recon(params, st.cam, opts)
        st.attach(rc)
        P = W * H
        for f in range(F):
            if pre_async is not None:
                pre_async.run_async(st.depth_u16.ptr.value + 2 * P * f, st.rgbx.ptr.value + 4 * P * f,
                                    st.depth.ptr.value + 4 * P * f, st.color.ptr.value + 4 * P * f)
                rc.frame_ready(f, pre_async.stream)
            rc.process_frame(f)
        rc.finish()
        rc.synchronize()
        hash_, heap, hc, vox = rc.export()
        subs = [rc.submap_poses(s, K + 1) for s in range(K - 1)]
        results.append(((mode, async_ba, cache_source), rc.op_log(), rc.trajectory(F), hash_, heap, hc, vox, subs))
        rc.close()
    res = {r[0]: r[1:] for r in results}
    for async_ba, other, cache_source in ((0, "in_loop", "synth"), (1, "in_loop", "synth"), (0, "ready", "synth"),
                                          (1, "ready", "synth"), (1, "ready", "loop")):
        a, b = res[(other, async_ba, cache_source)], res[("before", async_ba, cache_source)]
        assert len(a[0]) == len(b[0]) and len(a[0]) > F
        for x, y in zip(a[0], b[0]):
            assert x[0] == y[0] and x[1] == y[1]
            np.testing.assert_array_equal(x[2], y[2])
            np.testing.assert_array_equal(x[3], y[3])
        np.testing.assert_array_equal(a[1], b[1])
        for x, y in zip(a[6], b[6]):  # per-submap local / global poses (the cache feeds the local solves)
            for u, v in zip(x, y):
                np.testing.assert_array_equal(u, v)
        # the scenes: same block set and heap count, voxels bit for bit (the heap's free-list order and so
        # the blocks' heap slots depend on the GC's atomic push order, not on the inputs)
        assert a[4] == b[4]
        ba, bb = blocks_of(a[2]), blocks_of(b[2])
        assert set(ba) == set(bb) and len(ba) > 100
        for k, p in ba.items():
            x, y = a[5][p:p + 512], b[5][bb[k]:bb[k] + 512]
            assert x["sdf"].view(np.uint32).tobytes() == y["sdf"].view(np.uint32).tobytes(), k
            assert np.array_equal(x["weight"], y["weight"]) and np.array_equal(x["color"], y["color"]), k


def test_loop_fails_when_the_scene_drops_blocks():
    """The reference drops an allocation silently when its heap runs out (VoxelUtilHashSDF.h:535-540); the loop
    must not: a scene whose alloc candidate buffer is far too small for a frame (BFSceneOptions.candidateCapacity
    64 at 160x120 / 1 cm) sets error bit 1 in the batch that integrates frame 0, and the loop fails with
    BF_ERR_CAPACITY (at a later bf_recon_process_frame, through the GC kernel's host mirror, or at the latest at
    bf_recon_finish's exact check) instead of carrying on with holes. A loop with the default capacity runs the
    same frames with zero error bits and reports its peak candidates against the capacity."""
    from bundlefusion_amd.abi import BFSceneOptions
    ERR_CAPACITY = -3  # BF_ERR_CAPACITY
    F, W, H = 30, 160, 120
    st = SyntheticStream(F, width=W, height=H, outliers=0.0, cache_source="synth")
    params = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 16, num_blocks=1 << 15)
    K = st.K
    for cap in (64, 0):
        opts = recon_options(F, cacheWidth=80, cacheHeight=60, cacheIntrinsics=st.cache_intrinsics,
                             maxGlobalCorr=max(1000, 25 * K * (K - 1) // 2), maxKeyframes=K + 1)
        so = BFSceneOptions()
        so.candidateCapacity = cap
        rc = Recon(params, st.cam, opts, so)
        st.attach(rc)
        if cap:
            with pytest.raises(bfa.BFError, match="scene capacity exceeded.*candidate buffer overflow") as ei:
                for f in range(F):
                    rc.process_frame(f)
                rc.finish()
            assert ei.value.code == ERR_CAPACITY
            c = rc.scene_capacity()
            assert c["errorFlags"] & 1 and c["peakCandidates"] > c["candidateCapacity"] == 64, c
        else:
            for f in range(F):
                rc.process_frame(f)
            rc.finish()
            c = rc.scene_capacity()
            assert c["errorFlags"] == 0 and 0 < c["peakCandidates"] < c["candidateCapacity"] == 1 << 21, c
        rc.close()


def test_loop_renders_every_frame_like_visualize_frame():
    """bf_recon_set_render: visualizeFrame (DepthSensing.cpp:790-793) after every frame's batch, at the pose of
    the frame that batch integrated. The render must (a) not change what the loop does (the same scene calls,
    trajectory and voxels as the loop without it, bit for bit) and (b) show the scene as it stood: the last
    render equals the oracle's ray cast of the loop's own scene calls replayed up to that frame's garbage
    collection (>= 99.9 % bit-identical pixels, the ray-cast bar)."""
    import test_raycast_gpu as trg
    F, W, H = 30, 160, 120
    st = SyntheticStream(F, width=W, height=H, drift=(0.05, 0.002), outliers=0.0, cache_source="synth")
    params = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 16, num_blocks=1 << 15)
    K = st.K
    rp = bfa.raycast_params(W, H, fx=st.cam.fx, fy=st.cam.fy)
    runs = []
    for render in (True, False):
        opts = recon_options(F, recordOps=1, cacheWidth=80, cacheHeight=60, cacheIntrinsics=st.cache_intrinsics,
                             maxGlobalCorr=max(1000, 25 * K * (K - 1) // 2), maxKeyframes=K + 1, asyncBundling=0)
        rc = Recon(params, st.cam, opts)
        st.attach(rc)
        if render:
            rc.set_render(rp)
        for f in range(F):
            rc.process_frame(f)
        ops = rc.op_log()  # before synchronize (which integrates the pending frame)
        rc.synchronize()
        out = None
        if render:
            def d2h(ptr, shape):
                a = np.empty(shape, np.float32)
                bfa.check(bfa.lib().bf_memcpy_d2h(a.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), C.c_size_t(a.nbytes)))
                return a
            ptrs = rc.render_output()
            out = (d2h(ptrs[0], (H, W)),) + tuple(d2h(p, (H, W, 4)) for p in ptrs[1:])
            assert rc.stats()["renders"] == F - 1
        runs.append((ops, rc.trajectory(F), rc.export(), out))
        rc.close()
    (o1, t1, e1, img), (o0, t0, e0, _) = runs
    assert len(o1) == len(o0)
    for a, b in zip(o1, o0):
        assert a[0] == b[0] and a[1] == b[1]
        np.testing.assert_array_equal(a[2], b[2])
        np.testing.assert_array_equal(a[3], b[3])
    np.testing.assert_array_equal(t1, t0)
    assert e1[2] == e0[2]
    b1, b0 = blocks_of(e1[0]), blocks_of(e0[0])
    assert set(b1) == set(b0)
    for k, p in b1.items():
        assert e1[3][p:p + 512].tobytes() == e0[3][b0[k]:b0[k] + 512].tobytes(), k
    # the last render: after frame F-1's batch (it integrated frame F-2) and its GC
    # the log ends with frame F-1's pending integration (logged at process_frame, applied later): drop it
    assert o1[-1][0] == FIX_INTEGRATE and o1[-1][1] == F - 1 and o1[-2][0] == OP_GC
    depth, color = st.depth.download(), st.color.download()
    ora = OracleScene(params)
    last_T = None
    for kind, f, oldT, newT in o1[:-1]:
        if kind == FIX_DEINTEGRATE:
            ora.integrate(oldT.reshape(4, 4), depth[f], color[f], st.cam, deintegrate=True)
        elif kind == FIX_INTEGRATE:
            ora.integrate(newT.reshape(4, 4), depth[f], color[f], st.cam)
            if f == F - 2 and last_T is None:  # the render pose: frame F-2's own integration (first in its batch)
                last_T = newT.reshape(4, 4).copy()
        elif kind == OP_GC:
            ora.garbageCollect()
    o = ora.raycast(last_T, st.cam, rp)
    hit = trg.compare(img, o)
    assert hit > 0.5
