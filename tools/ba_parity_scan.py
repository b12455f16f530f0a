"""BA parity scan (development/measurement tool): pose difference between the HIP solver (both
normal-equation modes) and the oracle on the bench-shaped K=400 problem and on the small chains
of tests/test_ba_gpu.py, for growing PCG schedules. Prints one line per run; the summary is
committed under profiles/ as the measured justification of each test's tolerance."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]

import bundlefusion_amd as bfa  # noqa: E402
from ba_problem import make_problem, pose_diff, pose_errors  # noqa: E402
from test_ba_gpu import gpu_solve, oracle_solve  # noqa: E402

MODES = {"matrix_free": bfa.abi.NORMAL_EQ_MATRIX_FREE, "assembled": bfa.abi.NORMAL_EQ_ASSEMBLED}
problems = {
    "K400_stride10_out2": dict(K=400, stride=10, max_per_pair=25, outliers=0.02, drift=(0.05, 0.002)),
    "K12_chain": dict(K=12, max_per_pair=60, outliers=0.0),
    "K16_chain_out2": dict(K=16, max_per_pair=40, outliers=0.02, seed=5),
}
which = sys.argv[1:] or list(problems)
out = []
for name in which:
    prob = make_problem(**problems[name])
    sched = [(1, 10), (1, 50), (1, 150), (3, 150)] if prob["K"] >= 100 else [(1, 5), (1, 10), (1, 20), (1, 50), (1, 150), (3, 150)]
    sched = [(nn, nl, True) for nn, nl in sched] + [(3, 50, False), (3, 150, False), (1, 150, False)]
    for nn, nl, eo in sched:
        t = time.time()
        o = oracle_solve(prob, nn, nl, [1.0] * nn, early_out=eo)
        to = time.time() - t
        for mname, m in MODES.items():
            g = gpu_solve(prob, nn, nl, [1.0] * nn, mode=m, early_out=eo)
            er, et = pose_diff(g[0], g[1], o[0], o[1])
            rec = dict(problem=name, K=prob["K"], ncorr=len(prob["corr"]), gn=nn, pcg=nl, early_out=eo, mode=mname, rot_diff=er,
                       trans_diff=et, gn_g=g[3]["gnIterations"], gn_o=o[3]["gnIterations"],
                       pcg_g=g[3]["pcgIterations"], pcg_o=o[3]["pcgIterations"], energy_g=g[3]["energy"],
                       energy_o=o[3]["finalEnergy"], gt_err_g=pose_errors(g[0], g[1], prob["gt"]),
                       gt_err_o=pose_errors(o[0], o[1], prob["gt"]), oracle_s=to)
            out.append(rec)
            print(json.dumps(rec), flush=True)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(REPO, "gpurun_out", "ba_parity_scan.json"), "w"), indent=1)
