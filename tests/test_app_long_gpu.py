"""GPU: the FriedLiver application over BASELINE config 3's length — an 8 000-frame 640x480 .sens (JPEG colour,
zlib depth, the apt0 layout) of the seeded synthetic room at 4 mm, written on the box by the repo's writer —
through the whole program: decode threads, H2D, preprocessing, the cache, the EntryJ stand-in, the loop with
asynchronous bundling (results applied 20 frames after issue, so the run is repeatable), the end-of-sequence
phase and the exit outputs (FriedLiver.cpp:184-320, SensorDataReader.cpp:38-124, CUDAImageManager.cpp:22-158,
DepthSensing.cpp:854-902, 966-1129). Config 2 (copyroom, ~4k frames) is the first half of the same run.

Size-independent checks at full length:
  * the re-integration queue: the loop's whole TrajectoryManager call sequence replayed through the oracle
    TrajectoryManager, every fix list and transform bit for bit (TrajectoryManager.cpp:44-200);
  * debugHash's invariants of the final scene (CUDASceneRepHashSDF.h:179-314) and the heap accounting;
  * the voxels over a window of frames near the end: the app's scene calls replayed through the oracle TSDF
    from the GPU's own state, with the integration images recomputed independently (PIL / zlib decode, the
    oracle's preprocessing), bit for bit;
  * the optimized trajectory against the .sens ground truth (ATE): the front end's drift is removed."""
import os
import struct
import sys
import time
import zlib

import numpy as np
import pytest

from bundlefusion_amd import abi
from bundlefusion_amd.app import FriedLiver
from bundlefusion_amd.params import BUNDLING_DEFAULTS, NORTH_STAR_APP, write_parameter_files
from bundlefusion_amd.stream import write_synthetic_sens
from oracle_app import preprocess2
from oracle_lib import OracleScene, check_hash_invariants
from test_traj import replay_queue_trace
from tsdf_compare import compare_states, replay_ops

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

F = 8000
SNAP, WINDOW = 7960, 8
# the north-star stream at 640x480 / 4 mm; a 2^19-block heap (the room's final scene holds ~400 k blocks) keeps
# the exported snapshots small
APP = dict(NORTH_STAR_APP, s_hashNumBuckets=1 << 21, s_hashNumSDFBlocks=1 << 19)


class _Snapshot:
    def __init__(self, state):
        self.state = state

    def export(self):
        return self.state


class SensFrames:
    """Random access to a v4 .sens's frames by seeking (SensorData layout), decoded with
    zlib / PIL: the images the app decodes, recomputed off the product path."""

    def __init__(self, path):
        self.f = open(path, "rb")
        rd = self.f.read
        version, nlen = struct.unpack("<IQ", rd(12))
        assert version == 4
        rd(nlen)
        mats = np.frombuffer(rd(256), "<f4").reshape(4, 4, 4)
        self.depth_intrinsic = mats[2].copy()
        self.cc, self.dc = struct.unpack("<ii", rd(8))
        self.cw, self.ch, self.dw, self.dh, self.shift, self.n = struct.unpack("<IIIIfQ", rd(28))
        self.offsets, self.poses = [], []
        for _ in range(self.n):
            pose = np.frombuffer(rd(64), "<f4").reshape(4, 4).copy()
            _, _, cb, db = struct.unpack("<QQQQ", rd(32))
            self.offsets.append((self.f.tell(), cb, db))
            self.poses.append(pose)
            self.f.seek(cb + db, 1)

    def frame(self, i):
        import io

        from PIL import Image
        o, cb, db = self.offsets[i]
        self.f.seek(o)
        col, dep = self.f.read(cb), self.f.read(db)
        d = np.frombuffer(zlib.decompress(dep), "<u2").reshape(self.dh, self.dw)
        rgb = np.asarray(Image.open(io.BytesIO(col)).convert("RGB"))
        rgbx = np.empty(rgb.shape[:2] + (4,), np.uint8)
        rgbx[..., :3], rgbx[..., 3] = rgb, 255
        return d, rgbx


@pytest.fixture(scope="module")
def run(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("friedliver_long"))
    sens = os.path.join(d, "apt0_synthetic.sens")
    t0 = time.perf_counter()
    write_synthetic_sens(sens, F, 640, 480, threads=12)
    t1 = time.perf_counter()
    pa, pb = write_parameter_files(d, APP, {"s_maxNumImages": F // 10 + 2}, sens=sens)
    app = FriedLiver(pa, pb, output_dir=d, record_ops=True, enable_timing=True, result_lag=20)
    rc = app.recon
    snaps = {}
    f = 0
    while app.step():
        if f % 1000 == 0:
            print(f"  frame {f}", file=sys.stderr, flush=True)
        if f in (SNAP, SNAP + WINDOW):
            snaps[f] = (rc.export(), len(rc.op_log()))
        f += 1
    t2 = time.perf_counter()
    tm = app.timing()
    res = app.finish()
    t3 = time.perf_counter()
    print(f"{F} frames: .sens written in {t1 - t0:.1f} s; app loop {t2 - t1:.1f} s ({tm['frames'] / tm['stepSeconds']:.0f} "
          f"frames/s inside bf_app_step, snapshots included); end phase + outputs {t3 - t2:.1f} s")
    return dict(dir=d, sens=sens, app=app, rc=rc, res=res, snaps=snaps)


def test_app_ran_the_whole_stream(run):
    res, rc = run["res"], run["rc"]
    s = rc.stats()
    assert res["frames"] == F and s["frames"] == F
    assert s["localSolves"] == F // 10 and s["globalSolves"] >= F // 10 - 2
    assert s["deintegrations"] > 10 * F  # the queue re-integrates continuously
    e = res["end"]
    assert e["queueDrained"] == 1 and e["denseSolve"] == 1 and e["globalSolves"] == 31
    assert res["valid"] == 1 and res["numValidTransforms"] == res["numTransforms"] == F
    assert open(os.path.join(run["dir"], "processed.txt")).readline().strip() == "valid = true"
    # no block was dropped over the whole run (the loop would have failed with BF_ERR_CAPACITY), with headroom
    cap = rc.scene_capacity()
    assert cap["errorFlags"] == 0 and cap["peakCandidates"] < cap["candidateCapacity"] // 2, cap
    print(f"scene capacity: {cap}")
    print(f"{s['integrations']} integrations, {s['deintegrations']} de-integrations, {s['globalSolves']} global solves "
          f"({s['globalGnIterations']} GN, {s['globalPcgIterations']} PCG iterations), {s['removedPairs']} pair removals; "
          f"end phase: {e['pastEndFrames']} frames, dense solve {e['denseSolveMs']:.1f} ms")


def test_queue_bit_exact(run):
    calls, ops = replay_queue_trace(run["rc"].queue_trace(), F)
    print(f"queue: {calls} reintegrate() fix loops, {ops} ops identical")
    assert calls >= F and ops > 10 * F


def test_hash_and_heap_invariants(run):
    rc = run["rc"]
    params = rc.params
    h, heap, hc, _ = rc.export()
    check_hash_invariants(params, h, heap, hc)
    used = int(np.count_nonzero(h["ptr"] != abi.FREE_ENTRY))
    assert used == params.numSDFBlocks - rc.heap_free_count() == params.numSDFBlocks - (hc + 1)
    assert used == params.numSDFBlocks - run["res"]["heapFreeCount"]
    print(f"final scene: {used} blocks, heap free {hc + 1}")


def test_tsdf_window_replay(run):
    rc = run["rc"]
    params = rc.params
    (s0, i0), (s1, i1) = run["snaps"][SNAP], run["snaps"][SNAP + WINDOW]
    log = rc.op_log()
    kind, frame, _, newT = log[i0 - 1]
    assert kind == 2 and frame == SNAP
    info = run["app"].info
    cam = info.integrationCamera
    sens = SensFrames(run["sens"])
    B = BUNDLING_DEFAULTS
    pre = abi.BFPreprocessOptions(1 if B["s_erodeSIFTdepth"] else 0, 3, 0.05, 0.3, 1 if B["s_depthFilter"] else 0,
                                  B["s_depthSigmaD"], B["s_depthSigmaR"], sens.shift)
    images = {}

    def image(f):
        if f not in images:
            du, rgbx = sens.frame(f)
            od, oc, _, _ = preprocess2(pre, du, rgbx, cam.imageWidth, cam.imageHeight)
            images[f] = (od, oc)
        return images[f]

    sc = OracleScene(params)
    sc.import_state(*s0)
    sc.compactify(newT.reshape(4, 4), cam)
    n = replay_ops(sc, log[i0:i1], image, cam, "window")
    blocks = compare_states(params, _Snapshot(s1), sc)
    print(f"TSDF window frames {SNAP + 1}..{SNAP + WINDOW}: {n} scene ops over {len(images)} frames, {blocks} blocks "
          f"bit-identical")
    assert n >= 10 * WINDOW


def test_trajectory_against_ground_truth(run):
    rc = run["rc"]
    opt = rc.optimized_trajectory()
    gt = np.stack(SensFrames(run["sens"]).poses)
    assert len(opt) == F
    fin = np.isfinite(opt[:, 0, 0])
    assert fin.all()
    ate = np.sqrt(np.mean(np.sum((opt[:, :3, 3] - gt[:, :3, 3]) ** 2, axis=1)))
    print(f"ATE {ate * 1000:.2f} mm over {F} frames")
    assert ate < 0.02
