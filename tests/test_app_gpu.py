"""GPU: the FriedLiver application (bf_app_*, bundlefusion_amd/csrc/app.cpp) on a `.sens` in the copyroom /
apt0 layout — JPEG colour, zlib depth, 640x480, a camera trajectory — written by the repo's .sens writer
from the seeded synthetic room, run through zParameters files as FriedLiver's main() reads them
(Source/FriedLiver.cpp:184-320): preprocessing, per-frame cache, the EntryJ stand-in, the loop, the
end-of-sequence phase (OnlineBundler.cpp:167-196; DepthSensing.cpp:1114-1126) and StopScanningAndExit's
outputs (DepthSensing.cpp:904-953).

The oracle (tests/oracle_app.py) reads the same file with Python + PIL and runs the oracle's restatements
frame by frame. Bars:
  * derived parameters and the front end's estimates: bit-exact;
  * per-submap local / global poses: 1e-3 rad / 1 mm; verification outcomes, valid flags, solve and removal
    counts, the end-of-sequence outcome: exact;
  * the re-integration queue: the loop's recorded TrajectoryManager call sequence replayed through the
    oracle TrajectoryManager gives every fix list bit for bit (queue logic separated from BA float drift);
  * the voxels: the GPU loop's scene calls over three windows — frames 0..50 from an empty scene, frames
    141..170 and the whole end-of-sequence phase from the GPU's own state at the window's start — replayed
    through the oracle TSDF give a bit-identical scene;
  * the outputs: the trajectory .sens carries the optimized trajectory, processed.txt its verdict."""
import os

import numpy as np
import pytest

import bundlefusion_amd as bfa
from bundlefusion_amd.app import FriedLiver
from bundlefusion_amd.params import APP_DEFAULTS, BUNDLING_DEFAULTS, NORTH_STAR_APP, write_parameter_files
from bundlefusion_amd.stream import write_synthetic_sens
from oracle_app import OracleFriedLiver
from oracle_lib import OracleScene
from test_recon_parity_gpu import mat_diff
from test_traj import replay_queue_trace
from tsdf_compare import compare_states, replay_ops

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

F = 205            # 20 full submaps + a 5-frame partial one
START = 50         # the first window: frames 0..START from an empty scene
SNAP, WINDOW = 140, 30
ROT_TOL, TRANS_TOL = 1e-3, 1e-3
DRIFT = (float(np.deg2rad(0.05)), 0.002)
APP = dict(NORTH_STAR_APP, s_hashNumBuckets=1 << 20, s_hashNumSDFBlocks=1 << 18)


class _Snapshot:
    def __init__(self, state):
        self.state = state

    def export(self):
        return self.state


@pytest.fixture(scope="module")
def run(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("friedliver"))
    sens = os.path.join(d, "synthetic.sens")
    write_synthetic_sens(sens, F, 640, 480)
    pa, pb = write_parameter_files(d, APP, {}, sens=sens)
    app = FriedLiver(pa, pb, output_dir=d, async_bundling=0, record_ops=True, front_end_drift=DRIFT)
    rc = app.recon
    ora = OracleFriedLiver(sens, dict(APP_DEFAULTS, **APP), dict(BUNDLING_DEFAULTS), drift=DRIFT)
    snaps = {}
    for f in range(F):
        assert app.step()
        ora.step()
        if f in (START, SNAP, SNAP + WINDOW, F - 1):
            snaps[f] = (rc.export(), len(rc.op_log()))
    assert not app.step()
    res = app.finish()
    ores = ora.finish(APP_DEFAULTS["s_numSolveFramesBeforeExit"])
    snaps["end"] = (rc.export(), len(rc.op_log()))
    return dict(dir=d, sens=sens, app=app, rc=rc, ora=ora, res=res, ores=ores, snaps=snaps)


def test_derived_parameters_and_front_end(run):
    app, ora = run["app"], run["ora"]
    info = app.info
    assert info.numFrames == F and info.submapSize == 10 and info.maxKeyframes == ora.K
    for k in ("fx", "fy", "mx", "my", "sensorDepthWorldMin", "sensorDepthWorldMax"):
        assert np.float32(getattr(info.integrationCamera, k)) == np.float32(getattr(ora.cam, k)), k
    np.testing.assert_array_equal(np.float32(list(info.cacheIntrinsics)), np.float32(ora.cache_intrinsics))
    np.testing.assert_array_equal(np.float32(list(info.corr.intrinsicsInv)), np.float32(list(ora.corr_opts.intrinsicsInv)))
    assert info.corr.minPerPair == ora.corr_opts.minPerPair == 5
    assert (info.preprocess.erode, info.preprocess.depthFilter) == (1, 1)
    for f in range(F):
        assert app.front_end_pose(f).tobytes() == ora.tinc[f].tobytes(), f


def test_submap_poses_and_counts(run):
    rc, ora = run["rc"], run["ora"].ora
    nsub = (F + 9) // 10
    worst = np.zeros(4)
    for s in range(nsub):
        gl, gg, gv, gok = rc.submap_poses(s, run["ora"].K)
        ol, og, ov, ook = ora.submap_poses(s)
        assert gok == ook, s
        np.testing.assert_array_equal(gv, ov, err_msg=f"submap {s} valid flags")
        er, et = mat_diff(gl, ol)
        assert er <= ROT_TOL and et <= TRANS_TOL, (s, "local", er, et)
        sel = gv.astype(bool)
        gr, gt = mat_diff(gg[sel], og[sel])
        assert gr <= ROT_TOL and gt <= TRANS_TOL, (s, "global", gr, gt)
        worst = np.maximum(worst, [er, et, gr, gt])
    print(f"max diff local rot {worst[0]:.2e} trans {worst[1]:.2e}; global rot {worst[2]:.2e} trans {worst[3]:.2e}")
    s, o = rc.stats(), ora.stats()
    assert s["localSolves"] == o["localSolves"] == nsub
    for k in ("globalSolves", "removedPairs", "invalidLocals", "localVerifications", "endSolves"):
        assert s[k] == o[k], (k, s[k], o[k])


def test_end_of_sequence_phase(run):
    e, o = run["res"]["end"], run["ores"]
    for k in ("pastEndFrames", "globalSolves", "localSolved", "denseSolve", "queueDrained"):
        assert e[k] == o[k], (k, e[k], o[k])
    # the last submap (5 frames) is solved at p = 0, 30 more global solves follow, the 30th with the dense term
    assert e["localSolved"] == 1 and e["globalSolves"] == 31 and e["denseSolve"] == 1 and e["queueDrained"] == 1
    assert e["denseSolveMs"] > 0 and e["last"]["numDensePairs"] > 0
    print(f"end phase: {e['pastEndFrames']} frames past the end, dense solve {e['denseSolveMs']:.1f} ms, "
          f"{e['last']['numDensePairs']} pairs")


def test_final_trajectory(run):
    rc, ora = run["rc"], run["ora"]
    tg, to = rc.trajectory(F), ora.ora.trajectory(F)
    fin = np.isfinite(tg[:, 0, 0])
    np.testing.assert_array_equal(fin, np.isfinite(to[:, 0, 0]))
    er, et = mat_diff(tg[fin], to[fin])
    assert er <= ROT_TOL and et <= TRANS_TOL, (er, et)
    # the queue has drained: every optimized transform is the integrated one
    opt = rc.optimized_trajectory()
    assert len(opt) == F
    np.testing.assert_array_equal(opt[fin], tg[fin])
    # against the .sens trajectory (ground truth of the synthetic room): the drift of the front end is removed
    gt = np.stack(ora.poses)
    ate = np.sqrt(np.mean(np.sum((opt[fin][:, :3, 3] - gt[fin][:, :3, 3]) ** 2, axis=1)))
    dead = np.eye(4)
    for f in range(1, F):
        dead = dead @ ora.tinc[f].astype(np.float64)
    print(f"ATE {ate * 1000:.2f} mm over {fin.sum()} frames (front-end dead reckoning ends "
          f"{np.linalg.norm(dead[:3, 3] - (np.linalg.inv(gt[0]) @ gt[-1])[:3, 3]) * 1000:.1f} mm off)")
    assert ate < 0.02


def test_queue_bit_exact(run):
    calls, ops = replay_queue_trace(run["rc"].queue_trace(), F)
    print(f"queue: {calls} reintegrate() fix loops, {ops} ops, identical")
    assert calls >= F and ops > 500


def test_tsdf_window_replay(run):
    rc, ora = run["rc"], run["ora"]
    (s0, i0), (s1, i1) = run["snaps"][SNAP], run["snaps"][SNAP + WINDOW]
    log = rc.op_log()
    kind, frame, _, newT = log[i0 - 1]
    assert kind == 2 and frame == SNAP  # the snapshot follows frame SNAP's integration
    params = rc.params
    sc = OracleScene(params)
    sc.import_state(*s0)
    sc.compactify(newT.reshape(4, 4), ora.cam)  # the last op's frustum list (what the next GC walks)
    n = replay_ops(sc, log[i0:i1], ora.integration_image, ora.cam, "window")
    blocks = compare_states(params, _Snapshot(s1), sc)
    print(f"TSDF window frames {SNAP + 1}..{SNAP + WINDOW}: {n} scene ops replayed, {blocks} blocks bit-identical")
    assert n >= 4 * WINDOW


def test_tsdf_first_frames_replay(run):
    """The scene calls of frames 0..START through the oracle TSDF from an empty scene: bit for bit."""
    rc, ora = run["rc"], run["ora"]
    s1, i1 = run["snaps"][START]
    sc = OracleScene(rc.params)
    n = replay_ops(sc, rc.op_log()[:i1], ora.integration_image, ora.cam, "first frames")
    blocks = compare_states(rc.params, _Snapshot(s1), sc)
    print(f"TSDF frames 0..{START} from empty: {n} scene ops, {blocks} blocks bit-identical")


def test_tsdf_end_phase_replay(run):
    """The end-of-sequence phase's scene calls (the last submap's and 30 more solves' re-integrations
    until the queue drains) from the GPU's state after the last frame: bit for bit."""
    rc, ora = run["rc"], run["ora"]
    (s0, i0), (s1, i1) = run["snaps"][F - 1], run["snaps"]["end"]
    log = rc.op_log()
    assert len(log) == i1 and log[i0 - 1][0] == 2 and log[i0 - 1][1] == F - 1
    sc = OracleScene(rc.params)
    sc.import_state(*s0)
    sc.compactify(log[i0 - 1][3].reshape(4, 4), ora.cam)
    n = replay_ops(sc, log[i0:i1], ora.integration_image, ora.cam, "end phase")
    blocks = compare_states(rc.params, _Snapshot(s1), sc)
    print(f"TSDF end phase: {n} scene ops, {blocks} blocks bit-identical")
    assert n > 100


def test_outputs(run):
    d, res, rc = run["dir"], run["res"], run["rc"]
    txt = open(os.path.join(d, "processed.txt")).read().split("\n")
    assert txt[0] == "valid = true" and res["valid"] == 1
    assert txt[1] == f"heapFreeCount = {res['heapFreeCount']}"
    assert txt[2] == f"numValidOptTransforms = {res['numValidTransforms']}" and txt[3] == f"numTransforms = {F}"
    from bundlefusion_amd.io import SensorData
    out = SensorData(os.path.join(d, "synthetic.optimized.sens"))
    src = SensorData(run["sens"])
    opt = rc.optimized_trajectory()
    assert len(out) == F
    for f in range(0, F, 7):
        np.testing.assert_array_equal(out.pose(f), opt[f])
        np.testing.assert_array_equal(out.depth_u16(f), src.depth_u16(f))
    head = open(os.path.join(d, "synthetic.ply"), "rb").read(400).split(b"end_header")[0].decode()
    assert f"element vertex {res['meshVertices']}" in head and res["meshVertices"] > 1000
    assert res["meshTriangles"] > 1000
