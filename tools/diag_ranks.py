"""Diagnostics for the multi-rank loop on one GPU (tests/test_config4_gpu.py's setup at a chosen length): two
ranks of a loopback group, each a bf_recon on its own thread; every `every` frames both ranks synchronise
(a host barrier) and print heap use and whether their integrated trajectories still agree bit for bit.
Usage: python tools/diag_ranks.py FRAMES [EVERY] [BLOCKS_LOG2]"""
import os
import sys
import threading
import time

import numpy as np

# before anything initialises HIP (as tests/conftest.py): one hardware queue per stream of every rank
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 24:
    os.environ["GPU_MAX_HW_QUEUES"] = "24"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bundlefusion_amd as bfa  # noqa: E402
from bundlefusion_amd.abi import BFSceneOptions  # noqa: E402
from bundlefusion_amd.dist import LoopbackComm  # noqa: E402
from bundlefusion_amd.recon import Recon, recon_options  # noqa: E402
from bundlefusion_amd.stream import SyntheticStream  # noqa: E402


def main():
    frames = int(sys.argv[1])
    every = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    blocks = 1 << (int(sys.argv[3]) if len(sys.argv) > 3 else 20)
    F = frames + 1
    st = SyntheticStream(F, width=640, height=480, cache_source="loop", log=lambda *a: print(*a, flush=True))
    params = bfa.hash_params(voxel_size=0.004, num_buckets=1 << 22, num_blocks=blocks)
    K = st.K
    max_corr = max(1000, 25 * (K + 1) * K // 2)
    caches = [st.cache_store, st.loop_cache()]
    loops = []
    for r in range(2):
        opts = recon_options(F, recordOps=0, cacheWidth=80, cacheHeight=60, cacheIntrinsics=st.cache_intrinsics,
                             maxKeyframes=K + 1, maxGlobalCorr=max_corr, asyncBundling=1, resultLag=20)
        so = BFSceneOptions()
        so.shardCount, so.shardIndex, so.shardChunk = 2, r, 0.25
        rc = Recon(params, st.cam, opts, so)
        st.attach(rc, cache_store=caches[r], own_corr=True)
        loops.append(rc)
    comms = LoopbackComm.group(2, timeout_ms=60000, capacity_bytes=128 << 20)
    for rc, c in zip(loops, comms):
        rc.set_comm(c)
    bar = threading.Barrier(2)
    errors = []

    def rank(i, rc):
        try:
            for f in range(F):
                rc.process_frame(f)
                if (f + 1) % every == 0:
                    cap = rc.scene_capacity()
                    bar.wait()
                    print(f"rank {i} frame {f + 1}: heap used {cap['numSDFBlocks'] - cap['heapFree']} high water "
                          f"{cap['highWater']} err {cap['errorFlags']} peak cand {cap['peakCandidates']}", flush=True)
                    bar.wait()
            rc.synchronize()
        except Exception as e:  # noqa: BLE001
            errors.append((i, repr(e)))
            print(f"rank {i} failed: {e!r}", flush=True)
            bar.abort()

    t0 = time.perf_counter()
    th = [threading.Thread(target=rank, args=(i, rc)) for i, rc in enumerate(loops)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    print(f"{F} frames in {time.perf_counter() - t0:.0f} s; errors {errors}", flush=True)
    t = [rc.trajectory(F) for rc in loops]
    same = np.array_equal(t[0].view(np.uint32), t[1].view(np.uint32))
    fin = np.isfinite(t[0][:, 0, 0])
    ate = [float(np.sqrt(np.mean(np.sum((x[fin][:, :3, 3] - st.gt[fin][:, :3, 3]) ** 2, axis=1)))) for x in t]
    print(f"trajectories identical: {same}; ATE per rank (m): {ate}", flush=True)
    for rc in loops:
        rc.close()
    for c in comms:
        c.close()


if __name__ == "__main__":
    main()
