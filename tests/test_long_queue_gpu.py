"""GPU: the reconstruction loop over a long stream at the north-star shape (BASELINE config 3's regime:
the on-the-fly re-integration queue running for thousands of frames, apt0 ~8k frames at 640x480 / 4 mm).

2 001 frames of the seeded synthetic room at 640x480 / 4 mm (201 keyframes, loop closures every ~1 000
frames), synchronous bundling, the end-of-sequence phase. Checked:
  * the queue: the loop's whole TrajectoryManager call sequence replayed through the oracle
    TrajectoryManager, every fix list bit for bit (TrajectoryManager.cpp:45-200, DepthSensing.cpp:854-902);
  * heap accounting and hash invariants of the final scene (debugHash, CUDASceneRepHashSDF.h:179-314):
    every heap slot either free or owned by exactly one entry, buckets per computeHashPos;
  * the voxels over a window of frames near the end: the GPU's scene calls replayed through the oracle
    TSDF from the GPU's own state, bit for bit;
  * the trajectory against the ground truth: the front end's drift is removed (ATE)."""
import numpy as np
import pytest

import bundlefusion_amd as bfa
from bundlefusion_amd.recon import Recon, recon_options
from bundlefusion_amd.stream import SyntheticStream
from oracle_lib import OracleScene, check_hash_invariants
from test_traj import replay_queue_trace
from tsdf_compare import compare_states, replay_ops

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(1200)]

F = 2001
SNAP, WINDOW = 1960, 12


class _Snapshot:
    def __init__(self, state):
        self.state = state

    def export(self):
        return self.state


def test_long_stream_queue_heap_voxels():
    import time
    t0 = time.perf_counter()
    st = SyntheticStream(F, width=640, height=480, cache_source="loop")
    params = bfa.hash_params(voxel_size=0.004, num_buckets=1 << 21, num_blocks=1 << 19)
    K = st.K
    opts = recon_options(F, recordOps=1, cacheWidth=80, cacheHeight=60, cacheIntrinsics=st.cache_intrinsics,
                         maxGlobalCorr=max(1000, 25 * (K + 1) * K // 2), maxKeyframes=K + 1, asyncBundling=0)
    rc = Recon(params, st.cam, opts)
    st.attach(rc)
    t1 = time.perf_counter()
    snaps = {}
    import sys
    for f in range(F):
        rc.process_frame(f)
        if f % 250 == 0:
            print(f"  frame {f}", file=sys.stderr, flush=True)
        if f in (SNAP, SNAP + WINDOW):
            snaps[f] = (rc.export(), len(rc.op_log()))
    end = rc.end_sequence(30)
    t2 = time.perf_counter()
    s = rc.stats()
    print(f"{F} frames: stream {t1 - t0:.0f} s, loop + end phase {t2 - t1:.0f} s; {s['integrations']} integrations, "
          f"{s['deintegrations']} de-integrations, {s['globalSolves']} global solves, {s['removedPairs']} removals; "
          f"end: {end['pastEndFrames']} iterations, queue drained {end['queueDrained']}")
    assert end["queueDrained"] == 1 and end["denseSolve"] == 1
    assert s["deintegrations"] > 10 * F  # the queue re-integrates continuously

    # the queue, bit for bit
    calls, ops = replay_queue_trace(rc.queue_trace(), F)
    assert calls >= F
    print(f"queue: {calls} fix loops, {ops} ops identical")

    # heap accounting + hash invariants of the final scene
    h, heap, hc, vox = rc.export()
    check_hash_invariants(params, h, heap, hc)
    used = int(np.count_nonzero(h["ptr"] != bfa.abi.FREE_ENTRY))
    assert used == params.numSDFBlocks - rc.heap_free_count() == params.numSDFBlocks - (hc + 1)
    print(f"final scene: {used} blocks; heap free {hc + 1}")

    # voxels over the window, from the GPU's own state
    (s0, i0), (s1, i1) = snaps[SNAP], snaps[SNAP + WINDOW]
    log = rc.op_log()
    kind, frame, _, newT = log[i0 - 1]
    assert kind == 2 and frame == SNAP
    sc = OracleScene(params)
    sc.import_state(*s0)
    sc.compactify(newT.reshape(4, 4), st.cam)
    P = st.cam.imageWidth * st.cam.imageHeight
    H = st.cam.imageHeight
    def image(f):
        d = st.depth.download_range(f * P * 4, P * 4).view(np.float32).reshape(H, -1)
        return d, st.color.download_range(f * P * 4, P * 4).reshape(H, -1, 4)

    n = replay_ops(sc, log[i0:i1], image, st.cam, "window")
    blocks = compare_states(params, _Snapshot(s1), sc)
    print(f"TSDF window frames {SNAP + 1}..{SNAP + WINDOW}: {n} scene ops, {blocks} blocks bit-identical")
    assert n >= 10 * WINDOW

    # drift removal against the ground truth
    traj = rc.trajectory(F)
    fin = np.isfinite(traj[:, 0, 0])
    assert fin.mean() > 0.95
    ate = np.sqrt(np.mean(np.sum((traj[fin][:, :3, 3] - st.gt[fin][:, :3, 3]) ** 2, axis=1)))
    print(f"ATE {ate * 1000:.2f} mm over {fin.sum()} frames")
    assert ate < 0.01
    rc.close()
