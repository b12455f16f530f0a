"""Per-PCG-iteration divergence trace between the HIP solver and the oracle (development tool)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]

from ba_problem import make_problem, pose_diff  # noqa: E402
from test_ba_gpu import gpu_solve, oracle_solve  # noqa: E402

for K, outl in ((6, 0.01), (6, 0.0), (32, 0.01)):
    prob = make_problem(K=K, max_per_pair=30, outliers=outl)
    print(f"K={K} outliers={outl} ncorr={len(prob['corr'])}")
    for n in list(range(1, 12)) + [20, 40]:
        g = gpu_solve(prob, 1, n, [1])
        o = oracle_solve(prob, 1, n, [1])
        er, et = pose_diff(g[0], g[1], o[0], o[1])
        print(f"  nlin={n:3d} rot={er:.3e} trans={et:.3e} pcg g/o={g[3]['pcgIterations']}/{o[3]['pcgIterations']} "
              f"E g/o={g[3]['energy']:.6g}/{o[3]['finalEnergy']:.6g}")
