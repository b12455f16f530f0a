import os
import sys

import pytest

# The loopback communicator's ranks (tests/test_recon_comm_gpu.py, test_app_shards_gpu.py) share this process and
# one GPU, and their collectives wait on the device for each other, as RCCL's kernels do across processes. A rank's
# streams must then not share a hardware queue with another rank's (a collective spinning in a shared queue would
# hold back the other rank's arrival behind it), so the process gets more hardware queues than HIP's default 4
# before anything initialises HIP. One process per GPU (bench.py, the app) keeps the default.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 24:
    os.environ["GPU_MAX_HW_QUEUES"] = "24"

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: longer CPU tests")


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    oracle_lib.lib()
    return oracle_lib
