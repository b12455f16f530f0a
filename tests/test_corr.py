"""EntryJ correspondences: the Bundler::saveSparseCorrsToFile dump format (Bundler.cpp:396-409) and
the depth + pose producer standing in for the SiftGPU front end (pos = intrinsicsInv * (d * (u, v, 1))
as AddCurrToResidualsCU, SIFTImageManager.cu:610-686).

CPU: dump round trip and layout; a known-answer test of the oracle restatement (a wall seen from two
camera positions 5 cm apart). GPU: bf_corr_from_depth against the oracle, bit for bit, on rendered
frames, and a global solve fed by its output."""
import os

import numpy as np
import pytest

import bundlefusion_amd as bfa
from bundlefusion_amd.abi import ENTRYJ_DTYPE
from bundlefusion_amd.corr import corr_from_depth, corr_load, corr_options, corr_save
from oracle_lib import corr_from_depth as or_corr

FX = 577.87


def test_corr_dump_roundtrip_and_layout(tmp_path):
    rng = np.random.default_rng(0)
    c = np.zeros(37, ENTRYJ_DTYPE)
    c["i"] = rng.integers(0, 100, 37)
    c["j"] = c["i"] + 1
    c["pos_i"] = rng.normal(size=(37, 3))
    c["pos_j"] = rng.normal(size=(37, 3))
    p = str(tmp_path / "corrs.bin")
    corr_save(p, c)
    raw = open(p, "rb").read()
    assert len(raw) == 8 + 32 * 37 and int.from_bytes(raw[:8], "little") == 37
    assert raw[8:] == c.tobytes()
    back = corr_load(p)
    assert back.tobytes() == c.tobytes()
    corr_save(p, c[:0])
    assert len(corr_load(p)) == 0
    open(p, "wb").write(raw[:8 + 32 * 10])  # truncated
    with pytest.raises(bfa.BFError):
        corr_load(p)


def test_oracle_corr_wall_known_answer():
    W, H = 160, 120
    f = FX * W / 640
    cx, cy = (W - 1) / 2, (H - 1) / 2
    o = corr_options(W, H, f, f, cx, cy, stride=8, max_per_pair=25)
    d = np.full((H, W), 2.0, np.float32)
    T = np.stack([np.eye(4, dtype=np.float32)] * 3)
    T[1, 0, 3] = 0.05   # camera 1: 5 cm to the right
    T[2, 0, 3] = 2.00   # camera 2: the wall region it sees does not overlap frame 0's samples much
    Tinv = np.linalg.inv(T.astype(np.float64)).astype(np.float32)
    e, total = or_corr([d, d, d], T, Tinv, 1, 0, o, 100)
    assert total == len(e) == 25
    assert np.all(e["i"] == 0) and np.all(e["j"] == 1)
    assert np.all(e["pos_i"][:, 2] == 2.0) and np.all(e["pos_j"][:, 2] == 2.0)
    # pos_j is the frame-1 point re-sampled at the rounded pixel: within half a pixel at 2 m
    err = e["pos_i"] - np.float32([0.05, 0, 0]) - e["pos_j"]
    assert np.max(np.abs(err[:, :2])) <= 0.5 * 2.0 / f + 1e-6
    # frames (0, 2) and (1, 2): the pair order, then candidate order; cap truncates the list
    e2, t2 = or_corr([d, d, d], T, Tinv, 2, 0, o, 100)
    assert list(e2["i"]) == sorted(e2["i"]) and set(e2["i"]) <= {0, 1} and np.all(e2["j"] == 2)
    e3, t3 = or_corr([d, d, d], T, Tinv, 2, 0, o, 7)
    assert t3 == t2 and len(e3) == 7 and e3.tobytes() == e2[:7].tobytes()
    # invalid depth in the current frame: no matches
    bad = np.full((H, W), -np.inf, np.float32)
    e4, t4 = or_corr([d, bad], T[:2], Tinv[:2], 1, 0, o, 100)
    assert t4 == 0


@pytest.mark.gpu
def test_corr_gpu_matches_oracle_bitwise():
    sc = bfa.synth_scene(0)
    W, H = 640, 480
    cam = bfa.depth_camera(W, H, fx=FX, fy=FX)
    frames = list(range(0, 60, 10))
    T = np.stack([bfa.synth_pose(f) for f in frames]).astype(np.float32)
    Tinv = np.linalg.inv(T.astype(np.float64)).astype(np.float32)
    depths = [bfa.synth_render_host(sc, T[k], cam, 1, f)[0] for k, f in enumerate(frames)]
    dd = [bfa.DeviceArray.from_host(d) for d in depths]
    dT, dTi = bfa.DeviceArray.from_host(T), bfa.DeviceArray.from_host(Tinv)
    o = corr_options(W, H, FX, FX, cam.mx, cam.my)
    for cur, start in ((5, 0), (3, 1), (1, 0), (2, 2)):
        g, gt = corr_from_depth([a.ptr.value for a in dd], dT, dTi, cur, start, o, 1000)
        r, rt = or_corr(depths, T, Tinv, cur, start, o, 1000)
        assert gt == rt and g.tobytes() == r.tobytes(), (cur, start)
    assert len(corr_from_depth([a.ptr.value for a in dd], dT, dTi, 5, 0, o, 1000)[0]) > 50
    g, gt = corr_from_depth([a.ptr.value for a in dd], dT, dTi, 5, 0, o, 10)
    assert len(g) == 10 and gt > 10
