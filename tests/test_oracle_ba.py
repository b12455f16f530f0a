"""CPU tests of the BA oracle: Lie maps against closed forms, Jacobian identities, convergence
of the sparse solve to the synthetic ground truth, the dense term, and the residual analysis."""
import numpy as np
import pytest

import bundlefusion_amd as bfa
from ba_problem import make_problem, pose_diff, pose_errors, rodrigues
from oracle_ba import dense_system, matrix_to_pose, pose_to_matrix, rotation_angle, solve


def test_pose_to_matrix_is_se3_exp():
    """poseToMatrix (LieDerivUtil.h:160-207): rotation = Rodrigues(omega), translation = V(omega) t."""
    rng = np.random.default_rng(0)
    for _ in range(50):
        w = rng.normal(size=3) * rng.choice([1e-5, 1e-3, 0.3, 2.0])
        t = rng.normal(size=3)
        M = pose_to_matrix(w, t)
        np.testing.assert_allclose(M[:3, :3], rodrigues(w), atol=3e-6)
        th = np.linalg.norm(w)
        Wx = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
        if th > 1e-3:
            V = np.eye(3) + (1 - np.cos(th)) / th ** 2 * Wx + (th - np.sin(th)) / th ** 3 * Wx @ Wx
        else:
            V = np.eye(3) + 0.5 * Wx
        np.testing.assert_allclose(M[:3, 3], V @ t, rtol=1e-4, atol=5e-5)  # float32 arithmetic
        np.testing.assert_array_equal(M[3], [0, 0, 0, 1])


def test_matrix_to_pose_roundtrip():
    """matrixToPose (:135-158) inverts poseToMatrix, including the > 3pi/4 symmetric branch."""
    rng = np.random.default_rng(1)
    for scale in (1e-4, 0.1, 1.0, 2.8):
        for _ in range(20):
            w = rng.normal(size=3)
            w = w / np.linalg.norm(w) * scale
            t = rng.normal(size=3)
            r2, t2 = matrix_to_pose(pose_to_matrix(w, t))
            np.testing.assert_allclose(pose_to_matrix(r2, t2), pose_to_matrix(w, t), atol=2e-5)


def test_sparse_solve_converges_to_ground_truth():
    prob = make_problem(K=12, outliers=0.0, max_per_pair=60)
    assert len(prob["corr"]) > 2000
    e0 = pose_errors(prob["rot"], prob["trans"], prob["gt"])
    rot, trans, _, res = solve(prob["corr"], prob["valid"], prob["rot"], prob["trans"], 3, 150, [1, 1, 1])
    er, et = pose_errors(rot, trans, prob["gt"])
    assert e0[0] > 0.04 and e0[1] > 0.03  # the drift is real
    # 1.5 mm correspondence noise chained over 12 keyframes: a few mm / mrad is the noise floor
    assert er < 4e-3 and et < 7e-3, (er, et)
    assert res["gnIterations"] >= 2 and res["pcgIterations"] >= 10
    assert res["maxResidual"] < 0.02


def test_max_residual_finds_outlier():
    """computeMaxResidual (CUDASolverBundling.cpp:313-427): an injected 0.25 m outlier is the argmax."""
    prob = make_problem(K=8, outliers=0.0)
    corr = prob["corr"].copy()
    k = len(corr) // 3
    corr["pos_j"][k] += np.float32([0.25, 0.0, 0.0])
    rot, trans, c2, res = solve(corr, prob["valid"], prob["rot"], prob["trans"], 3, 100, [1, 1, 1])
    assert res["maxResidualIndex"] == k
    assert res["maxResidual"] > 0.08  # above s_optMaxResThresh -> the pair would be invalidated


def test_per_image_cap_invalidates_in_index_order():
    """BuildVariablesToCorrespondencesTableDevice (SolverBundling.cu:1226-1248): correspondences past
    maxCorrPerImage in either row are invalidated (serial replay: highest indices go)."""
    prob = make_problem(K=6, outliers=0.0, max_per_pair=40)
    corr = prob["corr"]
    counts = np.bincount(np.concatenate([corr["i"], corr["j"]]), minlength=6)
    cap = int(counts.max()) - 10
    _, _, c2, _ = solve(corr, prob["valid"], prob["rot"], prob["trans"], 1, 5, [1], max_corr_per_img=cap)
    inval = c2["i"] == 0xFFFFFFFF
    assert inval.sum() > 0
    # replay the serial rule
    cnt = np.zeros(6, int)
    expect = np.zeros(len(corr), bool)
    for x, e in enumerate(corr):
        o0, o1 = cnt[e["i"]], cnt[e["j"]]
        cnt[e["i"]] += 1
        cnt[e["j"]] += 1
        expect[x] = not (o0 < cap and o1 < cap)
    np.testing.assert_array_equal(inval, expect)


def _left_perturbed(rot, trans, k, c, h):
    """exp(h e_c) * T_k (left perturbation, computeLieUpdate order); c indexes [trans|rot]."""
    r, t = rot.copy(), trans.copy()
    d = np.zeros(6, np.float32)
    d[c] = h
    M = pose_to_matrix(d[3:], d[:3]) @ pose_to_matrix(r[k], t[k])
    r[k], t[k] = matrix_to_pose(M)
    return r, t


@pytest.fixture(scope="module")
def dense_problem():
    return make_problem(K=3, stride=2, outliers=0.0, with_cache=True, max_per_pair=10, drift=(0.2, 0.005))


def test_dense_jtr_is_energy_gradient(dense_problem):
    """BuildDenseSystem (SolverBundling.cu:182-306): Jtr = 1/2 dE/d(delta) for the point-to-plane energy
    E = sum w r^2, checked by central differences of the oracle's own energy."""
    prob = dense_problem
    sysf = lambda r, t: dense_system(prob["valid"], r, t, prob["cache"], prob["intrinsics"])
    _, jtr, E, npairs = sysf(prob["rot"], prob["trans"])
    assert npairs >= 2 and E > 0
    for k in (1, 2):
        g = np.zeros(6)
        for c in range(6):
            e_p = sysf(*_left_perturbed(prob["rot"], prob["trans"], k, c, 1e-3))[2]
            e_m = sysf(*_left_perturbed(prob["rot"], prob["trans"], k, c, -1e-3))[2]
            g[c] = (e_p - e_m) / 4e-3
        a = jtr[6 * k:6 * k + 6].astype(np.float64)
        # correspondences are re-searched per evaluation (pixel rounding), so compare direction and size
        assert a @ g / (np.linalg.norm(a) * np.linalg.norm(g)) > 0.98
        assert abs(np.linalg.norm(a) / np.linalg.norm(g) - 1.0) < 0.15
    np.testing.assert_array_equal(jtr[:6], 0)  # image 0 is fixed


def test_dense_jtj_is_jtr_jacobian(dense_problem):
    """JtJ (FlipJtJ-symmetrised) matches the finite-difference Jacobian of Jtr (Gauss-Newton, small residuals)."""
    prob = dense_problem
    sysf = lambda r, t: dense_system(prob["valid"], r, t, prob["cache"], prob["intrinsics"])
    jtj, _, _, _ = sysf(prob["rot"], prob["trans"])
    np.testing.assert_array_equal(jtj, jtj.T)
    H = np.zeros((12, 12))
    for k in (1, 2):
        for c in range(6):
            jp = sysf(*_left_perturbed(prob["rot"], prob["trans"], k, c, 1e-3))[1]
            jm = sysf(*_left_perturbed(prob["rot"], prob["trans"], k, c, -1e-3))[1]
            H[:, 6 * (k - 1) + c] = (jp[6:] - jm[6:]) / 2e-3
    np.testing.assert_allclose(jtj[6:, 6:], H, atol=0.06 * np.abs(H).max())


def test_dense_plus_sparse_local_solve():
    """Local solve (SBA.cpp:28-33 schedule shape): sparse + dense depth on the 80x60 cache converges."""
    prob = make_problem(K=6, stride=2, outliers=0.0, with_cache=True, max_per_pair=10, drift=(0.2, 0.005))
    rot, trans, _, res = solve(prob["corr"], prob["valid"], prob["rot"], prob["trans"], 3, 100, [1, 1, 1],
                               [1000, 1000, 1000], [0, 0, 0], cache=prob["cache"], intrinsics=prob["intrinsics"])
    er, et = pose_errors(rot, trans, prob["gt"])
    assert er < 3e-3 and et < 5e-3, (er, et)


def test_oracle_verify_trajectory_known_answers():
    """VerifyTrajectoryCU restated (SIFTImageManager.cu:1036-1127): the ground-truth trajectory of an
    11-frame submap passes with every pair overlapping; one frame moved by 6 deg / 8 cm fails."""
    from oracle_ba import verify_trajectory
    prob = make_problem(K=11, stride=1, outliers=0.0, with_cache=True, max_per_pair=10, drift=(0.2, 0.004))
    ok, st = verify_trajectory(prob["valid"], prob["gt"], prob["cache"], prob["intrinsics"])
    iu = np.triu_indices(11, 1)
    assert ok and np.all(st[iu][:, 2] > 0)
    err = st[iu][:, 0] / st[iu][:, 1]
    assert np.all(err < 0.05)
    T = prob["gt"].copy()
    D = np.eye(4)
    D[:3, :3] = rodrigues(np.array([0.3, -0.8, 0.5]) / np.linalg.norm([0.3, -0.8, 0.5]) * np.deg2rad(6.0))
    D[:3, 3] = [0.08, -0.08, 0.04]
    T[6] = (T[6].astype(np.float64) @ D).astype(np.float32)
    ok2, st2 = verify_trajectory(prob["valid"], T, prob["cache"], prob["intrinsics"])
    assert not ok2
    # pairs without frame 6 are unchanged
    for i, j in zip(*iu):
        if 6 not in (i, j):
            np.testing.assert_array_equal(st2[i, j], st[i, j])


def test_oracle_count_high_residuals():
    from oracle_ba import count_high_residuals
    prob = make_problem(K=6, outliers=0.3, max_per_pair=20)
    gt_rot = np.zeros((6, 3), np.float32)
    gt_trans = np.zeros((6, 3), np.float32)
    for k in range(6):
        gt_rot[k], gt_trans[k] = matrix_to_pose(prob["gt"][k])
    n = count_high_residuals(prob["corr"], gt_rot, gt_trans, 1.0, 0.02)
    # at the ground truth only the 0.1-0.3 m outliers exceed 2 cm
    assert 0.2 * len(prob["corr"]) < n < 0.4 * len(prob["corr"])
    assert count_high_residuals(prob["corr"], gt_rot, gt_trans, 1.0, 1.0) == 0
