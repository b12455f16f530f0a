"""Test infrastructure (checker only): numpy restatement of the bundle adjuster's sparse operator in
its two forms, used to pin the assembled (per image pair) normal equations of csrc/ba.hip against the
reference's matrix-free products.

matrix_free_*: applyJDevice / applyJTDevice and evalMinusJTFDevice
    (Source/Solver/SolverBundlingEquationsLie.h:63-148, :154-228): per correspondence c = (i, j),
    P_i = T_i p_i, P_j = T_j p_j, Jp_c = w (omega_i x P_i + t_i - omega_j x P_j - t_j) over images > 0,
    (J^T Jp)_v = sum_c (P_v x g, g) with g = Jp_c from v's side (no second w), J^T F with r = P_v - P_u.
pair_*: the same operator from per-pair sufficient statistics (k_pair_stats / k_pair_init /
    k_pcg_pairs): M = sum P_b P_a^T, s_a, s_b, n, Q_a, Q_b for a < b.
Everything here is float64 numpy; inputs are the float32 world points.
"""
import numpy as np

PSTAT = 28


def world_points(corr, T):
    """(P_i, P_j) float32 world points of every valid EntryJ (the k_entries / xf arithmetic order)."""
    Ti, Tj = T[corr["i"]], T[corr["j"]]
    pi = corr["pos_i"].astype(np.float32)
    pj = corr["pos_j"].astype(np.float32)

    def xf(Tm, p):  # row-major float4x4 * (p, 1), ((m0 x + m1 y) + m2 z) + m3 in float32
        out = np.empty_like(p)
        for r in range(3):
            out[:, r] = ((Tm[:, r, 0] * p[:, 0] + Tm[:, r, 1] * p[:, 1]) + Tm[:, r, 2] * p[:, 2]) + Tm[:, r, 3]
        return out
    return xf(Ti, pi), xf(Tj, pj)


def matrix_free_apply(corr, T, p_rot, p_trans, w, N):
    """A p of the reference (JTJ p), float64."""
    Pi, Pj = (x.astype(np.float64) for x in world_points(corr, T))
    out = np.zeros((N, 6))
    wr, wt = p_rot.astype(np.float64).copy(), p_trans.astype(np.float64).copy()
    wr[0] = 0.0
    wt[0] = 0.0
    for k, e in enumerate(corr):
        i, j = int(e["i"]), int(e["j"])
        g = w * (np.cross(wr[i], Pi[k]) + wt[i] - np.cross(wr[j], Pj[k]) - wt[j])
        out[i, :3] += np.cross(Pi[k], g)
        out[i, 3:] += g
        out[j, :3] += np.cross(Pj[k], -g)
        out[j, 3:] += -g
    out[0] = 0.0
    return out


def matrix_free_jtr(corr, T, N):
    """sum_c J_v^T r_c with r = P_v - P_u (before the -w of PCGInit)."""
    Pi, Pj = (x.astype(np.float64) for x in world_points(corr, T))
    out = np.zeros((N, 6))
    for k, e in enumerate(corr):
        i, j = int(e["i"]), int(e["j"])
        r = Pi[k] - Pj[k]
        out[i, :3] += np.cross(Pi[k], r)
        out[i, 3:] += r
        out[j, :3] += np.cross(Pj[k], -r)
        out[j, 3:] += -r
    return out


def pair_stats(corr, T):
    """{(a, b): 28 float64 statistics} in the layout of bf_solver_export_pairs."""
    Pi, Pj = (x.astype(np.float64) for x in world_points(corr, T))
    stats = {}
    for k, e in enumerate(corr):
        i, j = int(e["i"]), int(e["j"])
        if i == j:
            continue
        a, b = (i, j) if i < j else (j, i)
        A, B = (Pi[k], Pj[k]) if i == a else (Pj[k], Pi[k])
        s = stats.setdefault((a, b), np.zeros(PSTAT))
        s[0:9] += np.outer(B, A).ravel()
        s[9:12] += A
        s[12:15] += B
        s[15] += 1.0
        s[16:22] += [A[0] * A[0], A[0] * A[1], A[0] * A[2], A[1] * A[1], A[1] * A[2], A[2] * A[2]]
        s[22:28] += [B[0] * B[0], B[0] * B[1], B[0] * B[2], B[1] * B[1], B[1] * B[2], B[2] * B[2]]
    return stats


def _cross_mat(s):
    return np.array([[0.0, -s[2], s[1]], [s[2], 0.0, -s[0]], [-s[1], s[0], 0.0]])


def pair_blocks(stats, N):
    """Dense 6N x 6N operator sum_c J^T J (rot | trans per image) built from the pair statistics."""
    H = np.zeros((6 * N, 6 * N))
    for (a, b), s in stats.items():
        M = s[0:9].reshape(3, 3)
        sa, sb, n = s[9:12], s[12:15], s[15]
        Bab = np.zeros((6, 6))
        Bab[:3, :3] = np.trace(M) * np.eye(3) - M
        Bab[:3, 3:] = _cross_mat(sa)
        Bab[3:, :3] = -_cross_mat(sb)
        Bab[3:, 3:] = n * np.eye(3)
        H[6 * a:6 * a + 6, 6 * b:6 * b + 6] -= Bab
        H[6 * b:6 * b + 6, 6 * a:6 * a + 6] -= Bab.T
        for v, off, sv in ((a, 16, sa), (b, 22, sb)):
            q = s[off:off + 6]
            Q = np.array([[q[0], q[1], q[2]], [q[1], q[3], q[4]], [q[2], q[4], q[5]]])
            D = np.zeros((6, 6))
            D[:3, :3] = np.trace(Q) * np.eye(3) - Q
            D[:3, 3:] = _cross_mat(sv)
            D[3:, :3] = -_cross_mat(sv)
            D[3:, 3:] = n * np.eye(3)
            H[6 * v:6 * v + 6, 6 * v:6 * v + 6] += D
    return H


def pair_apply(stats, p_rot, p_trans, w, N):
    H = pair_blocks(stats, N)
    p = np.concatenate([p_rot.astype(np.float64), p_trans.astype(np.float64)], axis=1)
    p[0] = 0.0
    out = w * (H @ p.ravel()).reshape(N, 6)
    out[0] = 0.0
    return out


def pair_jtr(stats, N):
    """J^T r per image from the statistics: rot -/+ sum P_a x P_b (antisymmetric part of M), trans s_v - s_u."""
    out = np.zeros((N, 6))
    for (a, b), s in stats.items():
        M = s[0:9].reshape(3, 3)
        X = np.array([M[2, 1] - M[1, 2], M[0, 2] - M[2, 0], M[1, 0] - M[0, 1]])
        out[a, :3] -= X
        out[b, :3] += X
        out[a, 3:] += s[9:12] - s[12:15]
        out[b, 3:] += s[12:15] - s[9:12]
    return out
