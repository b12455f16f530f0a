"""CPU checks of the assembled (per image pair) normal equations used by the global solve
(csrc/ba.hip k_pair_stats / k_pair_init / k_pcg_pairs): the operator and right-hand side rebuilt
from the 28 per-pair statistics equal the reference's matrix-free J^T J p and J^T F
(SolverBundlingEquationsLie.h:63-228) on seeded problems with outliers."""
import numpy as np
import pytest

from ba_problem import make_problem
from oracle_ba import pose_to_matrix
from oracle_pairs import matrix_free_apply, matrix_free_jtr, pair_apply, pair_jtr, pair_stats


def _problem(K, seed):
    prob = make_problem(K=K, max_per_pair=12, outliers=0.02, seed=seed)
    T = np.stack([pose_to_matrix(prob["rot"][k], prob["trans"][k]) for k in range(K)])
    return prob["corr"], T


@pytest.mark.parametrize("K,seed", [(6, 1), (10, 4)])
def test_pair_operator_equals_matrix_free(K, seed):
    corr, T = _problem(K, seed)
    rng = np.random.default_rng(seed)
    pr, pt = rng.normal(size=(K, 3)) * 1e-3, rng.normal(size=(K, 3)) * 1e-3
    stats = pair_stats(corr, T)
    a = pair_apply(stats, pr, pt, 1.0, K)
    b = matrix_free_apply(corr, T, pr, pt, 1.0, K)
    np.testing.assert_allclose(a, b, rtol=1e-9, atol=1e-12 * np.abs(b).max())


@pytest.mark.parametrize("K,seed", [(6, 2), (10, 5)])
def test_pair_rhs_equals_matrix_free(K, seed):
    corr, T = _problem(K, seed)
    a = pair_jtr(pair_stats(corr, T), K)
    b = matrix_free_jtr(corr, T, K)
    np.testing.assert_allclose(a, b, rtol=1e-9, atol=1e-12 * np.abs(b).max())


def test_smooth_mode_cancellation_is_resolved_in_fp64():
    """p equal on every image (a rigid motion of the whole trajectory): the reference operator maps it
    to ~0 by cancellation; the fp64 pair statistics resolve that cancellation (|Ap| ~ 1e-12 |D||p|)."""
    corr, T = _problem(8, 7)
    K = 8
    pr = np.tile([1e-3, -2e-3, 5e-4], (K, 1))
    pt = np.tile([1e-3, 1e-3, -1e-3], (K, 1))
    stats = pair_stats(corr, T)
    a = pair_apply(stats, pr, pt, 1.0, K)
    b = matrix_free_apply(corr, T, pr, pt, 1.0, K)
    np.testing.assert_allclose(a[2:], b[2:], atol=1e-9)
