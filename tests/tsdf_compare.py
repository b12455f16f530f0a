"""Shared driver for TSDF parity: run one op sequence on the HIP scene and the CPU oracle
and compare the resulting voxel-hash states block by block."""
from __future__ import annotations

import numpy as np

import bundlefusion_amd as bfa
from oracle_lib import OracleScene, block_voxels, blocks_of, bucket_of, check_hash_invariants


def render_frames(scene, cam, frames, noise_seed=1):
    out = []
    for f in frames:
        T = bfa.synth_pose(f)
        d, c = bfa.synth_render_host(scene, T, cam, noise_seed, f)
        out.append((T, d, c))
    return out


def compare_states(params, gpu: bfa.SceneRepHashSDF, ora: OracleScene, check_voxels=True):
    gh, gheap, ghc, gvox = gpu.export()
    oh, oheap, ohc, ovox = ora.export()
    check_hash_invariants(params, gh, gheap, ghc)
    check_hash_invariants(params, oh, oheap, ohc)
    gb, ob = blocks_of(gh), blocks_of(oh)
    missing = set(ob) - set(gb)
    extra = set(gb) - set(ob)
    if missing or extra:
        nb = params.hashNumBuckets
        info = []
        for k in sorted(missing)[:6] + sorted(extra)[:6]:
            b = bucket_of(k, nb)
            info.append((k, "missing" if k in missing else "extra", b,
                         int((gh["ptr"][b * 4:b * 4 + 4] != -2).sum()), int((oh["ptr"][b * 4:b * 4 + 4] != -2).sum()),
                         int(gh[b * 4 + 3]["offset"]), int(oh[b * 4 + 3]["offset"])))
        raise AssertionError(f"block sets differ: {len(missing)} missing, {len(extra)} extra; "
                             f"(key, kind, bucket, gpu slots used, oracle slots used, gpu/oracle last offset): {info}")
    assert ghc == ohc, f"heap counter {ghc} != {ohc}"
    # bucket index of every entry (slot // 4 for in-bucket entries) is computeHashPos exactly
    occ = np.nonzero(gh["ptr"] != bfa.abi.FREE_ENTRY)[0]
    for i in occ[:2000]:
        e = gh[i]
        key = (int(e["x"]), int(e["y"]), int(e["z"]))
        h = bucket_of(key, params.hashNumBuckets)
        assert i // 4 == h or int(gh[h * 4 + 3]["offset"]) != 0
    if check_voxels and ob:
        keys = sorted(ob)
        gptr = np.array([gb[k] for k in keys])
        optr = np.array([ob[k] for k in keys])
        idx = np.arange(512)
        gv = gvox[(gptr[:, None] + idx[None, :]).ravel()]
        ov = ovox[(optr[:, None] + idx[None, :]).ravel()]
        bad_sdf = np.nonzero(gv["sdf"].view(np.uint32) != ov["sdf"].view(np.uint32))[0]
        bad_w = np.nonzero(gv["weight"] != ov["weight"])[0]
        bad_c = np.nonzero(np.any(gv["color"] != ov["color"], axis=1))[0]
        if len(bad_w):
            det = [(keys[i // 512], int(i % 512), float(gv["weight"][i]), float(ov["weight"][i]), float(gv["sdf"][i]),
                    float(ov["sdf"][i])) for i in bad_w[:8]]
            raise AssertionError(f"{len(bad_w)} weights differ; (block, voxel, gpu w, oracle w, gpu sdf, oracle sdf): {det}")
        assert len(bad_c) == 0, f"{len(bad_c)} colours differ"
        assert len(bad_sdf) == 0, (f"{len(bad_sdf)} sdf differ, max |d| = "
                                   f"{np.max(np.abs(gv['sdf'][bad_sdf] - ov['sdf'][bad_sdf]))}")
    return len(ob)


class Pair:
    """HIP scene + oracle scene driven with identical operations."""

    def __init__(self, params, cam, **scene_opts):
        self.params, self.cam = params, cam
        self.gpu = bfa.SceneRepHashSDF(params, **scene_opts)
        self.ora = OracleScene(params)
        self._dev = {}

    def _upload(self, key, d, c):
        if key not in self._dev:
            dd = bfa.DeviceArray.from_host(np.ascontiguousarray(d, np.float32))
            cc = bfa.DeviceArray.from_host(np.ascontiguousarray(c, np.uint8)) if c is not None else None
            self._dev[key] = (dd, cc)
        return self._dev[key]

    def integrate(self, key, T, d, c, deint=False):
        dd, cc = self._upload(key, d, c)
        if deint:
            self.gpu.deIntegrate(T, dd, cc, self.cam)
        else:
            self.gpu.integrate(T, dd, cc, self.cam)
        self.ora.integrate(T, d, c, self.cam, deintegrate=deint)

    def gc(self):
        self.gpu.garbageCollect()
        self.ora.garbageCollect()

    def compare(self, **kw):
        return compare_states(self.params, self.gpu, self.ora, **kw)


def replay_ops(scene, ops, image, cam, label="replay"):
    """Apply a loop's op log (kind 1 de-integrate oldT, 2 integrate newT, 4 GC) to an oracle scene;
    image(f) -> (depth, colour). Prints a progress line every 30 s (long replays must not look hung).
    Returns the number of integrate / de-integrate calls."""
    import sys
    import time
    n, t0, last = 0, time.perf_counter(), time.perf_counter()
    for kind, f, oldT, newT in ops:
        if kind == 4:
            scene.garbageCollect()
            continue
        d, c = image(f)
        scene.integrate((oldT if kind == 1 else newT).reshape(4, 4), d, c, cam, deintegrate=(kind == 1))
        n += 1
        if time.perf_counter() - last > 30.0:
            last = time.perf_counter()
            print(f"  {label}: {n} ops in {last - t0:.0f} s", file=sys.stderr, flush=True)
    return n
