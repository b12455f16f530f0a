"""Seeded synthetic bundle-adjustment problems (SURVEY.md §8(d) "BA inputs")."""
from __future__ import annotations

import numpy as np

import bundlefusion_amd as bfa
from bundlefusion_amd import solver as bs
from oracle_ba import matrix_to_pose


def rodrigues(w):
    th = np.linalg.norm(w)
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


def drifted(gt: np.ndarray, seed=3, rot_deg=0.05, trans_m=0.002) -> np.ndarray:
    """GT poses composed with a random-walk drift (frame 0 is fixed and keeps its pose)."""
    rng = np.random.default_rng(seed)
    out = gt.copy()
    D = np.eye(4)
    for k in range(1, len(gt)):
        step = np.eye(4)
        step[:3, :3] = rodrigues(rng.normal(size=3) * np.deg2rad(rot_deg))
        step[:3, 3] = rng.normal(size=3) * trans_m
        D = D @ step
        out[k] = (gt[k].astype(np.float64) @ D).astype(np.float32)
    return out


def make_problem(K=12, stride=10, start=0, max_per_pair=25, outliers=0.0, noise=0.0015, seed=2, cam=None,
                 with_cache=False, cache_cam=None, drift=(0.5, 0.01)):
    scene = bfa.synth_scene(0)
    cam = cam or bfa.depth_camera(640, 480)
    gt = np.stack([bfa.synth_pose(start + stride * k) for k in range(K)]).astype(np.float32)
    corr = bs.synth_correspondences(scene, gt, cam, max_per_pair=max_per_pair, min_covis=0.3, noise=noise,
                                    outlier_frac=outliers, seed=seed)
    init = drifted(gt, rot_deg=drift[0], trans_m=drift[1])
    rot = np.zeros((K, 3), np.float32)
    trans = np.zeros((K, 3), np.float32)
    for k in range(K):
        rot[k], trans[k] = matrix_to_pose(init[k])
    prob = dict(scene=scene, gt=gt, init=init, corr=corr, rot=rot, trans=trans, valid=np.ones(K, np.int32), K=K)
    if with_cache:
        cc = cache_cam or bfa.depth_camera(80, 60, fx=577.87 / 8, fy=577.87 / 8, mx=39.5, my=29.5)
        prob["cache"] = bs.synth_cache_frames(scene, gt, cc)
        prob["cache_cam"] = cc
        prob["intrinsics"] = (cc.fx, cc.fy, cc.mx, cc.my)
    return prob


def pose_errors(rot, trans, gt):
    """max rotation (rad) / translation (m) error of each pose relative to frame 0 (gauge)."""
    from oracle_ba import pose_to_matrix, rotation_angle
    T0 = pose_to_matrix(rot[0], trans[0])
    er, et = 0.0, 0.0
    for k in range(len(gt)):
        Tk = pose_to_matrix(rot[k], trans[k])
        rel = np.linalg.inv(T0) @ Tk
        rel_gt = np.linalg.inv(gt[0]) @ gt[k]
        er = max(er, rotation_angle(rel, rel_gt))
        et = max(et, float(np.linalg.norm(rel[:3, 3] - rel_gt[:3, 3])))
    return er, et


def pose_diff(rot_a, trans_a, rot_b, trans_b):
    """max per-pose rotation (rad) and translation (m) difference between two solutions.

    The angle is taken from the chord ||Ra - Rb||_F = 2 sqrt(2) sin(theta / 2) in float64, which
    resolves ~1e-7 rad (arccos of the float32 trace bottoms out near 3e-4 rad)."""
    from oracle_ba import pose_to_matrix
    er, et = 0.0, 0.0
    for k in range(len(rot_a)):
        A = pose_to_matrix(rot_a[k], trans_a[k]).astype(np.float64)
        B = pose_to_matrix(rot_b[k], trans_b[k]).astype(np.float64)
        chord = np.linalg.norm(A[:3, :3] - B[:3, :3]) / (2.0 * np.sqrt(2.0))
        er = max(er, float(2.0 * np.arcsin(min(1.0, chord))))
        et = max(et, float(np.linalg.norm(A[:3, 3] - B[:3, 3])))
    return er, et
