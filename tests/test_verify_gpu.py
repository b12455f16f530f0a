"""GPU: local-submap verification (useVerification + VerifyTrajectoryCU) against the oracle.

Reference chain: SBA::align (SBA.cpp:106-109) -> CUDASolverBundling::useVerification
(Solver/CUDASolverBundling.cpp:454-476) -> Bundler::optimize (Bundler.cpp:259-274) ->
SIFTImageManager::VerifyTrajectoryCU (SiftGPU/SIFTImageManager.cu:1036-1159). The kernel and the
oracle sum in the same fixed order, so the per-pair sums and the decision are compared bit-exact.
"""
import numpy as np
import pytest

import bundlefusion_amd as bfa
from ba_problem import make_problem, rodrigues
from oracle_ba import count_high_residuals, verify_trajectory

pytestmark = pytest.mark.gpu


def _submap(seed=0, start=0):
    return make_problem(K=11, stride=1, start=start, max_per_pair=25, outliers=0.0, with_cache=True, drift=(0.2, 0.004))


def _gpu_verify(prob, T, always=True, n_corr=0, solver=None, valid=None):
    from bundlefusion_amd.solver import DeviceCache, SolverBundling
    K = prob["K"]
    S = solver or SolverBundling(K, 4000)
    cache = DeviceCache(prob["cache"])
    d_T = bfa.DeviceArray.from_host(np.ascontiguousarray(np.asarray(T, np.float32).reshape(K, 16)))
    d_valid = bfa.DeviceArray.from_host(prob["valid"] if valid is None else valid)
    stats = bfa.DeviceArray.from_host(np.zeros((K, K, 3), np.float32))
    ok = S.verify_trajectory(d_T, d_valid, K, n_corr, cache.table, cache.W, cache.H, prob["intrinsics"], always=always,
                             pair_stats=stats)
    return ok, stats.download(), S.result()


def _perturb(T, k, deg=6.0, trans=0.08):
    T = T.copy()
    D = np.eye(4)
    D[:3, :3] = rodrigues(np.array([0.3, -0.8, 0.5]) / np.linalg.norm([0.3, -0.8, 0.5]) * np.deg2rad(deg))
    D[:3, 3] = [trans, -trans, 0.5 * trans]
    T[k] = (T[k].astype(np.float64) @ D).astype(np.float32)
    return T


def test_verify_ground_truth_valid_bit_exact():
    prob = _submap()
    ok_g, st_g, res = _gpu_verify(prob, prob["gt"])
    ok_o, st_o = verify_trajectory(prob["valid"], prob["gt"], prob["cache"], prob["intrinsics"])
    assert res["verifyUsed"] == 1
    assert ok_g and ok_o and res["verifyOk"] == 1
    iu = np.triu_indices(prob["K"], 1)
    assert np.all(st_o[iu][:, 2] > 0)  # every pair of an 11-frame submap overlaps
    np.testing.assert_array_equal(st_g[iu], st_o[iu])


def test_verify_perturbed_frame_invalid_bit_exact():
    prob = _submap()
    T = _perturb(prob["gt"], 6)
    ok_g, st_g, res = _gpu_verify(prob, T)
    ok_o, st_o = verify_trajectory(prob["valid"], T, prob["cache"], prob["intrinsics"])
    assert not ok_o and not ok_g and res["verifyOk"] == 0
    iu = np.triu_indices(prob["K"], 1)
    np.testing.assert_array_equal(st_g[iu], st_o[iu])


def test_verify_skips_invalid_images():
    prob = _submap()
    T = _perturb(prob["gt"], 6)
    valid = np.ones(prob["K"], np.int32)
    valid[6] = 0  # the bad frame is already invalid: no pair with it is checked
    ok_g, st_g, _ = _gpu_verify(prob, T, valid=valid)
    ok_o, st_o = verify_trajectory(valid, T, prob["cache"], prob["intrinsics"])
    assert ok_g and ok_o
    assert np.all(st_g[6] == 0) and np.all(st_g[:, 6] == 0)


@pytest.mark.parametrize("outliers", [0.0, 0.3])
def test_use_verification_gate(outliers):
    """After a local solve: the high-residual count equals the oracle's at the solved poses, and the
    pair check runs iff count / nCorr >= 0.05 (CUDASolverBundling.cpp:472-475)."""
    from bundlefusion_amd.solver import DeviceCache, SolverBundling
    prob = make_problem(K=11, stride=1, max_per_pair=25, outliers=outliers, with_cache=True, drift=(0.2, 0.004))
    K, corr = prob["K"], prob["corr"]
    S = SolverBundling(K, 4000)
    d_corr = bfa.DeviceArray.from_host(corr)
    d_valid = bfa.DeviceArray.from_host(prob["valid"])
    d_rot = bfa.DeviceArray.from_host(prob["rot"])
    d_trans = bfa.DeviceArray.from_host(prob["trans"])
    cache = DeviceCache(prob["cache"])
    S.solve(d_corr, len(corr), d_valid, K, 2, 100, [1, 1], [1, 2], [0, 0], cache=cache.table, cache_w=cache.W,
            cache_h=cache.H, intrinsics=prob["intrinsics"], rot=d_rot, trans=d_trans, find_max_residual=True)
    res = S.result()
    rot, trans = d_rot.download(), d_trans.download()
    high = count_high_residuals(d_corr.download()[:len(corr)], rot, trans, 1.0, 0.02)
    assert res["highResidualCount"] == high
    d_T = bfa.DeviceArray.from_host(np.zeros((K, 16), np.float32))
    S.poses_to_matrices(d_rot, d_trans, K, d_T, d_valid)
    ok = S.verify_trajectory(d_T, d_valid, K, len(corr), cache.table, cache.W, cache.H, prob["intrinsics"])
    r2 = S.result()
    used = np.float32(high) / np.float32(len(corr)) >= np.float32(0.05)
    assert r2["verifyUsed"] == int(used)
    if used:
        ok_o, _ = verify_trajectory(prob["valid"], d_T.download(), prob["cache"], prob["intrinsics"])
        assert ok == ok_o
    else:
        assert ok
    if outliers > 0:
        assert used  # 30 % outliers leave far more than 5 % of the residuals above 2 cm
