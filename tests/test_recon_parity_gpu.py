"""GPU: loop-level pose parity of the reconstruction loop against the oracle's restatement of the
OnlineBundler local -> global state machine (oracle/recon.cpp; Source/OnlineBundler.cpp:242-416,
Source/OnlineBundler.cu:73-140, Source/SBA.cpp:106-109, Source/Bundler.cpp:259-274).

The BASELINE config-2 shape: 640x480 frames, 4 mm voxels, 200 frames = 20 submaps, local 2x100 and
global 3x150 GN x PCG, dense local term on the 80x60 caches the GPU built from the rendered frames,
synchronous bundling. Per submap the local trajectory, the keyframe poses after its global solve and
its verification outcome are compared; then the integrated trajectory, the re-integration queue's op
sequence and the end-of-sequence phase (30 past-the-end global solves, the last with the dense term of
USE_GLOBAL_DENSE_AT_END, weight 15; then re-integration until the queue is empty).
Poses: SURVEY.md §8(c) bars, 1e-3 rad / 1 mm. Integer outcomes (valid flags, verification, the op
kinds and frames) exact; the queue itself bit-exact given the loop's poses (test_queue_bit_exact_given_the_
loop_poses). The TSDF replay of the ops is covered bit-exactly by test_recon_gpu.py (160x120) and, at
640x480 / 4 mm, by the window replay of test_app_gpu.py.
"""
import numpy as np
import pytest

import bundlefusion_amd as bfa
from ba_problem import pose_diff
from bundlefusion_amd.recon import Recon, recon_options
from bundlefusion_amd.stream import SyntheticStream
from oracle_ba import matrix_to_pose
from oracle_recon import OracleRecon

pytestmark = pytest.mark.gpu

ROT_TOL, TRANS_TOL = 1e-3, 1e-3


def mat_diff(A, B):
    """max rotation / translation difference between two stacks of 4x4 camera -> world matrices"""
    ra = np.zeros((len(A), 3), np.float32)
    ta = np.zeros((len(A), 3), np.float32)
    rb, tb = ra.copy(), ta.copy()
    for k in range(len(A)):
        ra[k], ta[k] = matrix_to_pose(A[k])
        rb[k], tb[k] = matrix_to_pose(B[k])
    return pose_diff(ra, ta, rb, tb)


def corrupt_submap(st, s, seed=7):
    """Replace submap s's local correspondences by ones drawn from a wrong trajectory (frames 5.. of the
    submap moved by 4 deg / 6 cm) with 30 % outliers: the solve keeps >5 % high residuals, so
    useVerification runs the dense check, and the cache frames (rendered from the true poses) fail it."""
    from bundlefusion_amd.abi import ENTRYJ_DTYPE
    from bundlefusion_amd.solver import synth_correspondences
    from ba_problem import rodrigues
    base = s * st.S
    poses = st.gt[base:base + st.S + 1].copy()
    D = np.eye(4)
    D[:3, :3] = rodrigues(np.array([0.2, 0.9, -0.4]) / np.linalg.norm([0.2, 0.9, -0.4]) * np.deg2rad(4.0))
    D[:3, 3] = [0.06, 0.0, -0.04]
    for i in range(5, len(poses)):
        poses[i] = (poses[i].astype(np.float64) @ D).astype(np.float32)
    bad = synth_correspondences(st.scene, poses, st.cam, max_per_pair=25, min_covis=0.3, noise=0.0015,
                                outlier_frac=0.3, seed=seed)
    locs = [st.local_corr.download()[st.local_off[k]:st.local_off[k] + st.local_n[k]] for k in range(st.num_submaps)]
    locs[s] = bad
    off = 0
    for k in range(st.num_submaps):
        st.local_off[k] = off
        st.local_n[k] = len(locs[k])
        off += len(locs[k])
    st.local_corr = bfa.DeviceArray.from_host(np.concatenate(locs) if off else np.zeros(1, ENTRYJ_DTYPE))


def run_pair(F=200, corrupt=None, end_dense=15.0):
    st = SyntheticStream(F, width=640, height=480, outliers=0.02)
    if corrupt is not None:
        corrupt_submap(st, corrupt)
    K = st.K
    max_global = max(1000, 25 * K * (K - 1) // 2)
    params = bfa.hash_params(voxel_size=0.004, num_buckets=1 << 21, num_blocks=1 << 19)
    opts = recon_options(F, recordOps=1, cacheWidth=80, cacheHeight=60, cacheIntrinsics=st.cache_intrinsics,
                         maxGlobalCorr=max_global, maxKeyframes=K + 1, asyncBundling=0)
    rc = Recon(params, st.cam, opts)
    # host copies before the GPU loop modifies its lists in place (cap / pair invalidation)
    glob = st.global_host.copy()
    local = st.local_corr.download()
    caches = [st.cache_store.download(i) for i in range(F)]
    st.attach(rc)
    ora = OracleRecon(F, st.gt[0], st.cache_intrinsics, max_keyframes=K + 1, max_global_corr=max_global)
    for f in range(F):
        ora.set_frame(f, st.tinc[f], caches[f])
    for s in range(st.num_submaps):
        ora.set_local_corr(s, local[st.local_off[s]:st.local_off[s] + st.local_n[s]])
    ora.set_global_corr(glob, st.global_prefix)
    for f in range(F):
        rc.process_frame(f)
        ora.process_frame(f)
    out = dict(st=st, rc=rc, ora=ora, K=K)
    if end_dense is not None:
        # the render loop past the last frame (OnlineBundler.cpp:167-196, DepthSensing.cpp:1114-1126):
        # the last submap, s_numSolveFramesBeforeExit global solves (the last with the dense term), then
        # re-integration until the queue is empty
        out["end_gpu"] = rc.end_sequence(30, dense_depth_weight=end_dense)
        out["end_ora"] = ora.end_sequence(30, dense_depth_weight=end_dense)
    else:
        rc.finish()
        ora.finish()
    rc.synchronize()
    return out


@pytest.fixture(scope="module")
def clean():
    return run_pair()


def _check_submaps(run, upto=None, loose_after=None):
    """Per submap: verification outcome and keyframe valid flags exact, poses within ROT_TOL / TRANS_TOL
    (submaps after `loose_after`: within 1e-2, see test_invalid_local_submap_is_dropped)."""
    st, rc, ora = run["st"], run["rc"], run["ora"]
    worst = [0.0, 0.0, 0.0, 0.0]
    for s in range(st.num_submaps if upto is None else upto):
        rt = tt = 1e-2 if loose_after is not None and s > loose_after else ROT_TOL
        if rt == ROT_TOL:
            tt = TRANS_TOL
        gl, gg, gv, gok = rc.submap_poses(s, run["K"] + 1)
        ol, og, ov, ook = ora.submap_poses(s)
        assert gok == ook, f"submap {s}: verification GPU {gok} oracle {ook}"
        np.testing.assert_array_equal(gv, ov, err_msg=f"submap {s} keyframe valid flags")
        er, et = mat_diff(gl, ol)
        worst[0], worst[1] = max(worst[0], er), max(worst[1], et)
        assert er <= rt and et <= tt, (s, "local", er, et)
        sel = gv.astype(bool)
        er, et = mat_diff(gg[sel], og[sel])
        worst[2], worst[3] = max(worst[2], er), max(worst[3], et)
        print(f"submap {s}: global diff rot {er:.2e} trans {et:.2e}")
        assert er <= rt and et <= tt, (s, "global", er, et)
    return worst


def test_loop_submap_poses_parity(clean):
    worst = _check_submaps(clean)
    print(f"max diff local rot {worst[0]:.2e} trans {worst[1]:.2e}; global rot {worst[2]:.2e} trans {worst[3]:.2e}")
    s = clean["rc"].stats()
    o = clean["ora"].stats()
    assert s["localSolves"] == o["localSolves"] == clean["st"].num_submaps
    assert s["globalSolves"] == o["globalSolves"] and s["endSolves"] == o["endSolves"] == 30
    assert s["removedPairs"] == o["removedPairs"] and s["invalidLocals"] == o["invalidLocals"] == 0
    assert s["localVerifications"] == o["localVerifications"]


def test_loop_trajectory_and_queue_parity(clean):
    st, rc, ora = clean["st"], clean["rc"], clean["ora"]
    tg, to = rc.trajectory(st.F), ora.trajectory(st.F)
    fin = np.isfinite(tg[:, 0, 0])
    np.testing.assert_array_equal(fin, np.isfinite(to[:, 0, 0]))
    er, et = mat_diff(tg[fin], to[fin])
    assert er <= ROT_TOL and et <= TRANS_TOL, (er, et)
    # informational: per-call op multisets of the two loops (their BA poses differ in the last bits, which
    # may swap near-tied frames across a 10-fix cut); the queue itself is held bit-exact given the loop's
    # own poses (test_queue_bit_exact_given_the_loop_poses)
    same, total = compare_queues(rc.op_log(), ora.op_log())
    print(f"re-integration queue: {same}/{total} reintegrate() calls with the same ops")


def compare_queues(lg, lo, t_tol=2e-3):
    """The queue sorts frames by pose change (TrajectoryManager.cpp:45-109); frames of one submap move
    together when its keyframe moves, so their distances nearly tie and float differences of ~1e-5 in
    the poses may swap two of them across the 10-fix cut of one reintegrate() call. Compare per call
    (ops between GC markers): the multiset of (kind, frame), and the transforms of identical calls."""
    from collections import Counter

    def groups(log):
        out, cur = [], []
        for k, f, o, n in log:
            if k == 4:
                out.append(cur)
                cur = []
            else:
                cur.append((k, f, o, n))
        return out

    gg, go = groups(lg), groups(lo)
    assert len(gg) == len(go)
    tot_g = Counter(k for k, *_ in lg)
    tot_o = Counter(k for k, *_ in lo)
    for k in (1, 2):
        assert abs(tot_g[k] - tot_o[k]) <= max(2, 0.01 * tot_o[k]), (k, tot_g, tot_o)
    same = 0
    for a, b in zip(gg, go):
        if Counter((k, f) for k, f, _, _ in a) != Counter((k, f) for k, f, _, _ in b):
            continue
        same += 1
        for (k, f, og, ng), (_, _, oo, no) in zip(sorted(a, key=lambda x: (x[0], x[1])), sorted(b, key=lambda x: (x[0], x[1]))):
            x, y = (og, oo) if k == 1 else (ng, no)
            assert np.max(np.abs(x - y)) <= t_tol, (k, f)
    return same, len(gg)


def test_end_of_sequence_phase(clean):
    e, o = clean["end_gpu"], clean["end_ora"]
    for k in ("pastEndFrames", "globalSolves", "localSolved", "denseSolve", "queueDrained"):
        assert e[k] == o[k], (k, e[k], o[k])
    assert e["localSolved"] == 1 and e["globalSolves"] == 31 and e["denseSolve"] == 1 and e["queueDrained"] == 1
    res = e["last"]
    assert res["skipped"] == 0 and res["numDensePairs"] > 0 and e["denseSolveMs"] > 0
    print(f"end phase: {e['pastEndFrames']} iterations; dense solve {e['denseSolveMs']:.2f} ms, "
          f"{res['numDensePairs']} overlapping keyframe pairs, gn {res['gnIterations']}")


def test_queue_bit_exact_given_the_loop_poses(clean):
    """The GPU loop's TrajectoryManager call sequence (its own optimized poses included) through the oracle
    TrajectoryManager: every fix list identical, transforms bit for bit (TrajectoryManager.cpp:45-200,
    DepthSensing.cpp:854-902). This separates the queue logic from the BA's float drift, which is what the
    per-call multiset comparison above tolerates."""
    from test_traj import replay_queue_trace
    calls, ops = replay_queue_trace(clean["rc"].queue_trace(), clean["st"].F)
    print(f"queue: {calls} fix loops, {ops} ops identical")
    assert calls >= clean["st"].F and ops > 1000


def test_invalid_local_submap_is_dropped():
    """Submap 6's local correspondences come from a wrong trajectory: both sides run the dense check,
    reject the submap, mark keyframe 6 invalid (no global solve for it) and de-integrate its frames.

    Up to submap 6 the poses meet the 1 mm / 1e-3 rad bar. After it, keyframe 7 starts from keyframe
    6's pose (initializeNextTransformUnknown, Bundler.h:75-79), ~20 cm from where it belongs; the
    3 x 150 schedule has not converged it when it stops, and from there the two float32 CG summation
    orders end at different points: measured on MI355X 2.7-2.9e-3 rad / 4.1-4.4 mm at submap 7, shrinking
    with every later solve to 1.5e-3 rad / 2.6 mm at submap 11 (the same
    chaotic divergence profiles/r2_ba_parity_scan.txt shows for unconverged small chains). Those
    submaps are held to 1e-2 and to the same valid flags and verification outcomes."""
    run = run_pair(F=120, corrupt=6, end_dense=None)
    st, rc, ora = run["st"], run["rc"], run["ora"]
    _, _, gv, gok = rc.submap_poses(6, run["K"] + 1)
    _, _, ov, ook = ora.submap_poses(6)
    assert not gok and not ook and gv[6] == 0 and ov[6] == 0
    _check_submaps(run, loose_after=6)
    s, o = rc.stats(), ora.stats()
    assert s["invalidLocals"] == o["invalidLocals"] == 1
    for _ in range(5):
        rc.reintegrate()
        ora.reintegrate()
    traj = rc.trajectory(st.F)
    assert not np.isfinite(traj[60:70, 0, 0]).any()  # frames of the invalid submap are no longer in the volume
    same, total = compare_queues(rc.op_log(), ora.op_log(), t_tol=2e-2)
    print(f"re-integration queue: {same}/{total} reintegrate() calls with the same ops (informational)")
    # the queue logic bit-exact given the loop's own poses, the invalid submap's de-integrations included
    from test_traj import replay_queue_trace
    calls, ops = replay_queue_trace(rc.queue_trace(), st.F)
    print(f"queue: {calls} fix loops, {ops} ops identical")
    assert calls >= st.F and ops > 100
