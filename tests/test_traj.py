"""Host logic (CPU): the product's re-integration queue (bf_traj_*, csrc/trajectory.cpp) against the
oracle's transcription (oracle/traj.cpp) of TrajectoryManager + reintegrate()
(Source/TrajectoryManager.cpp:8-200, Source/DepthSensing/DepthSensing.cpp:854-902).

Op lists, frame states and pose distances must be identical (bit-exact: both sides evaluate the
same float32 expressions)."""
import ctypes as C

import numpy as np
import pytest

from bundlefusion_amd.recon import TrajectoryManager, pose_helper_matrix_to_pose
from ba_problem import rodrigues
from oracle_lib import lib as _olib


class OracleTM:
    def __init__(self, max_frames, top_n=30, min_dist=0.0):
        L = _olib()
        L.or_traj_create.restype = C.c_void_p
        L.or_traj_create.argtypes = [C.c_uint, C.c_uint, C.c_float]
        L.or_traj_add_frame.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_uint]
        L.or_traj_update_optimized.argtypes = [C.c_void_p, C.c_void_p, C.c_uint]
        L.or_traj_next_fixes.argtypes = [C.c_void_p, C.c_uint] + [C.c_void_p] * 4
        L.or_traj_next_fixes.restype = C.c_uint
        L.or_traj_frame_info.argtypes = [C.c_void_p, C.c_uint, C.c_void_p, C.c_void_p]
        L.or_traj_destroy.argtypes = [C.c_void_p]
        L.or_pose_helper_matrix_to_pose.argtypes = [C.c_void_p, C.c_void_p]
        L.or_traj_generate_and_count.argtypes = [C.c_void_p]
        L.or_traj_generate_and_count.restype = C.c_uint
        self.L = L
        self.h = L.or_traj_create(max_frames, top_n, min_dist)

    def __del__(self):
        self.L.or_traj_destroy(self.h)

    def add_frame(self, typ, T, idx):
        T = np.ascontiguousarray(np.asarray(T if T is not None else np.zeros(16), np.float32).reshape(16))
        self.L.or_traj_add_frame(self.h, typ, T.ctypes.data, idx)

    def update_optimized(self, T):
        T = np.ascontiguousarray(np.asarray(T, np.float32).reshape(-1, 16))
        self.L.or_traj_update_optimized(self.h, T.ctypes.data, T.shape[0])

    def next_fixes(self, max_fixes=10):
        kinds = np.zeros(max_fixes, np.int32)
        frames = np.zeros(max_fixes, np.uint32)
        old = np.zeros((max_fixes, 16), np.float32)
        new = np.zeros((max_fixes, 16), np.float32)
        n = self.L.or_traj_next_fixes(self.h, max_fixes, kinds.ctypes.data, frames.ctypes.data, old.ctypes.data,
                                      new.ctypes.data)
        return [(int(kinds[i]), int(frames[i]), old[i], new[i]) for i in range(n)]

    def generate_and_count(self):
        """generateUpdateLists + getNumActiveOperations (the past-the-end exit check)"""
        return self.L.or_traj_generate_and_count(self.h)

    def frame_info(self, idx):
        t = C.c_int()
        d = C.c_float()
        self.L.or_traj_frame_info(self.h, idx, C.byref(t), C.byref(d))
        return t.value, d.value


def pose_mat(rng, scale_r=0.5, scale_t=1.0):
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = rodrigues(rng.normal(size=3) * scale_r)
    T[:3, 3] = rng.normal(size=3) * scale_t
    return T


def assert_same_ops(a, b):
    assert [(k, f) for k, f, _, _ in a] == [(k, f) for k, f, _, _ in b]
    for (k, f, o1, n1), (_, _, o2, n2) in zip(a, b):
        if k in (1, 3):
            np.testing.assert_array_equal(o1, o2)
        if k in (2, 3):
            np.testing.assert_array_equal(n1, n2)


def test_pose_helper_matrix_to_pose_matches_oracle_and_inverts():
    rng = np.random.default_rng(0)
    L = OracleTM(1).L
    for scale in (1e-5, 1e-3, 0.3, 1.5, 3.0):
        for _ in range(20):
            T = pose_mat(rng, scale_r=scale)
            p = pose_helper_matrix_to_pose(T)
            o = np.zeros(6, np.float32)
            Tc = np.ascontiguousarray(T.reshape(16))
            L.or_pose_helper_matrix_to_pose(Tc.ctypes.data, o.ctypes.data)
            np.testing.assert_array_equal(p, o)
            # omega part is the rotation vector of R
            th = np.linalg.norm(p[3:])
            if 1e-4 < th < 3.0:
                np.testing.assert_allclose(rodrigues(p[3:].astype(np.float64)), T[:3, :3], atol=3e-5)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_queue_matches_oracle(seed):
    """Random stream: frames added (some without transform), optimized trajectories arriving every
    10 frames with drift corrections and invalidations; compare every reintegrate() op list."""
    rng = np.random.default_rng(seed)
    F = 160
    prod, orc = TrajectoryManager(F), OracleTM(F)
    traj = np.stack([pose_mat(rng) for _ in range(F)])
    for f in range(F):
        if f % 10 == 0 and f > 0:
            opt = traj[:f].copy()
            for g in range(f):  # pose corrections of varying size (ties included: unchanged frames)
                if rng.random() < 0.7:
                    opt[g] = opt[g] @ pose_mat(rng, scale_r=rng.choice([1e-4, 1e-2, 0.05]), scale_t=0.02)
            for g in rng.choice(f, size=2, replace=False):  # invalid frames (-inf)
                opt[g] = -np.inf
            if rng.random() < 0.3:  # a re-validated frame
                g = int(rng.integers(f))
                opt[g] = traj[g]
            traj[:f] = np.where(np.isfinite(opt), opt, traj[:f])
            prod.update_optimized(opt)
            orc.update_optimized(opt)
        a = prod.next_fixes(10)
        b = orc.next_fixes(10)
        assert_same_ops(a, b)
        typ = 1 if rng.random() < 0.05 else 0
        prod.add_frame(typ, traj[f] if typ == 0 else None, f)
        orc.add_frame(typ, traj[f] if typ == 0 else None, f)
    for _ in range(40):  # drain
        assert_same_ops(prod.next_fixes(10), orc.next_fixes(10))
    for f in range(F):
        assert prod.frame_info(f) == orc.frame_info(f)


@pytest.mark.parametrize("seed", [5, 6])
def test_queue_ties_match_oracle(seed):
    """Equal non-zero distances in bulk: frames share one of a few poses and get one of a few
    corrections, so whole groups tie. The product sorts by a radix sort of {class, distance,
    position} keys and caches MatrixToPose per frame; the order among equal keys must stay the
    oracle's stable_sort order over the persistent permutation, across many regenerations."""
    rng = np.random.default_rng(seed)
    F = 400
    prod, orc = TrajectoryManager(F, 30), OracleTM(F, 30)
    base = [pose_mat(rng) for _ in range(3)]
    corr = [pose_mat(rng, scale_r=s, scale_t=0.01) for s in (1e-3, 1e-2, 3e-2)]
    traj = np.stack([base[int(rng.integers(3))] for _ in range(F)])
    for f in range(F):
        if f % 10 == 0 and f > 0:
            opt = traj[:f].copy()
            for g in range(f):
                if rng.random() < 0.8:
                    opt[g] = opt[g] @ corr[int(rng.integers(3))]
            if f % 30 == 0:
                opt[int(rng.integers(f))] = -np.inf
            prod.update_optimized(opt)
            orc.update_optimized(opt)
        assert_same_ops(prod.next_fixes(10), orc.next_fixes(10))
        prod.add_frame(0, traj[f], f)
        orc.add_frame(0, traj[f], f)
    for _ in range(60):
        assert_same_ops(prod.next_fixes(10), orc.next_fixes(10))
    for f in range(F):
        assert prod.frame_info(f) == orc.frame_info(f)


def test_queue_long_stream_matches_oracle():
    """1 600 frames with every frame's optimized pose changed by each update: the product converts the
    changed poses on its host pool (more than 1 024 stale poses), the oracle serially; op lists and
    per-frame distances must agree."""
    rng = np.random.default_rng(9)
    F = 1600
    prod, orc = TrajectoryManager(F), OracleTM(F)
    ang = rng.uniform(-np.pi, np.pi, F)
    traj = np.tile(np.eye(4, dtype=np.float32), (F, 1, 1))
    traj[:, 0, 0], traj[:, 0, 1], traj[:, 1, 0], traj[:, 1, 1] = np.cos(ang), -np.sin(ang), np.sin(ang), np.cos(ang)
    traj[:, :3, 3] = rng.normal(size=(F, 3))
    for f in range(F):
        if f % 10 == 0 and f > 0:
            a = rng.normal(0, 1e-3, f).astype(np.float32)
            corr = np.tile(np.eye(4, dtype=np.float32), (f, 1, 1))
            corr[:, 0, 0], corr[:, 0, 1], corr[:, 1, 0], corr[:, 1, 1] = np.cos(a), -np.sin(a), np.sin(a), np.cos(a)
            corr[:, :3, 3] = rng.normal(0, 5e-3, (f, 3))
            opt = np.einsum("nij,njk->nik", traj[:f], corr).astype(np.float32)
            prod.update_optimized(opt)
            orc.update_optimized(opt)
        assert_same_ops(prod.next_fixes(10), orc.next_fixes(10))
        prod.add_frame(0, traj[f], f)
        orc.add_frame(0, traj[f], f)
    for f in range(F):
        assert prod.frame_info(f) == orc.frame_info(f)


def test_queue_semantics_by_hand():
    """Reference behaviour spelled out: integrated frames whose optimized pose moved are re-integrated
    largest distance first (top 30, dist > 0); -inf frames are de-integrated; a re-validated frame is
    integrated again."""
    tm = TrajectoryManager(8)
    I = np.eye(4, dtype=np.float32)
    for f in range(6):
        tm.add_frame(0, I, f)
    opt = np.stack([I] * 6)
    opt[1] = I.copy()
    opt[1][0, 3] = 0.01
    opt[3] = I.copy()
    opt[3][0, 3] = 0.05
    opt[4] = -np.inf
    tm.update_optimized(opt)
    ops = tm.next_fixes(10)
    # de-integrate list first (frame 4), then re-integrations by distance: 3 (5 cm) before 1 (1 cm)
    assert [(k, f) for k, f, _, _ in ops] == [(1, 4), (3, 3), (3, 1)]
    assert tm.frame_info(4)[0] == 3  # Invalid
    # frame 4 comes back -> integrate op with its new pose
    opt[4] = I
    tm.update_optimized(opt)
    ops = tm.next_fixes(10)
    assert [(k, f) for k, f, _, _ in ops] == [(2, 4)]
    assert tm.next_fixes(10) == []


def replay_queue_trace(trace, max_frames, max_fixes=10, top_n=30, min_dist=0.0):
    """Drive the oracle TrajectoryManager through a loop's recorded call sequence (bf_recon_queue_trace)
    and require every fix list and exit-check count to be identical, transforms bit for bit. Returns the
    number of fix-loop calls checked and of ops compared."""
    tm = OracleTM(max_frames, top_n, min_dist)
    calls = ops = 0
    for kind, a, payload in trace:
        if kind == 0:
            tm.add_frame(0, payload, a)
        elif kind == 1:
            tm.update_optimized(payload)
        elif kind == 2:
            got = tm.next_fixes(max_fixes)
            assert len(got) == len(payload), (calls, len(got), len(payload))
            for (k1, f1, o1, n1), (k2, f2, o2, n2) in zip(got, payload):
                assert (k1, f1) == (k2, f2), (calls, (k1, f1), (k2, f2))
                if k1 in (1, 3):
                    assert o1.tobytes() == o2.tobytes(), (calls, f1, "oldT")
                if k1 in (2, 3):
                    assert n1.tobytes() == n2.tobytes(), (calls, f1, "newT")
                ops += 1
            calls += 1
        elif kind == 3:
            assert tm.generate_and_count() == a
    return calls, ops
