"""Quick timing probe: integrate a synthetic 640x480 stream at 4 mm on the GPU and print
per-op times and the device counters (development tool; bench.py is the contract)."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bundlefusion_amd as bfa  # noqa: E402


def main(n=60, buckets=1 << 23, blocks=1 << 21):
    L = bfa.lib()
    cam = bfa.depth_camera(640, 480)
    p = bfa.hash_params(voxel_size=0.004, num_buckets=buckets, num_blocks=blocks)
    scene = bfa.SceneRepHashSDF(p)
    sc = bfa.synth_scene(0)
    frames = []
    for f in range(n):
        T = bfa.synth_pose(f * 2)
        d = bfa.DeviceArray((480, 640), "f4")
        c = bfa.DeviceArray((480, 640, 4), "u1")
        bfa.synth_render(sc, T, cam, 1, f, d, c)
        frames.append((T, d, c))
    t = C.c_void_p()
    bfa.check(L.bf_timer_create(C.byref(t)))
    ms = C.c_float()
    # warm
    for T, d, c in frames[:5]:
        scene.integrate(T, d, c, cam)
    scene.synchronize()
    scene.reset()
    scene.resetStats()
    bfa.check(L.bf_scene_timer_start(scene.h, t))
    for T, d, c in frames:
        scene.integrate(T, d, c, cam)
    bfa.check(L.bf_scene_timer_stop(scene.h, t, C.byref(ms)))
    st = scene.stats()
    print(f"integrate: {ms.value / n:.3f} ms/op over {n} frames; stats {st}")
    # steady-state ops (no new allocation): re-integrate the last frame repeatedly
    T, d, c = frames[-1]
    scene.resetStats()
    bfa.check(L.bf_scene_timer_start(scene.h, t))
    for _ in range(20):
        scene.deIntegrate(T, d, c, cam)
        scene.integrate(T, d, c, cam)
    bfa.check(L.bf_scene_timer_stop(scene.h, t, C.byref(ms)))
    st = scene.stats()
    print(f"deint+int steady: {ms.value / 40:.3f} ms/op; stats {st}")
    bfa.check(L.bf_scene_timer_start(scene.h, t))
    for _ in range(20):
        scene.garbageCollect()
    bfa.check(L.bf_scene_timer_stop(scene.h, t, C.byref(ms)))
    print(f"gc: {ms.value / 20:.3f} ms; heap free {scene.getHeapFreeCount()} err {scene.errorFlags()}")
    vis = scene.numVisible()
    print("visible", vis)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
