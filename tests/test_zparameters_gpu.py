"""GPU: bf_app_create on the reference's own parameter settings (tests/golden/zparameters_reference.json, the
two zParameters*.txt files key for key) with only the sensor file overridden (FriedLiver.cpp:228-250 reads
s_binaryDumpSensorFile; BFAppOptions.sensFile replaces it): the app comes up with the parameters bf_app_resolve
derives, runs a 25-frame .sens through the loop and the end-of-sequence phase, and writes its outputs."""
import os

import pytest

from bundlefusion_amd.app import FriedLiver
from bundlefusion_amd.stream import write_synthetic_sens
from test_zparameters import FILES, _fields, _resolved, _write_fixture_files

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def test_app_runs_on_the_reference_settings(tmp_path):
    d = str(tmp_path)
    sens = os.path.join(d, "input.sens")
    write_synthetic_sens(sens, 25, 640, 480)
    pa, pb = _write_fixture_files(d)
    assert [os.path.basename(p) for p in (pa, pb)] == list(FILES)
    app = FriedLiver(pa, pb, sens_file=sens, output_dir=d)
    info, _ = _resolved(pa, pb, sens)
    assert _fields(app.info) == info
    res = app.run()
    assert res["frames"] == 25 and res["end"]["globalSolves"] > 0
    assert res["numTransforms"] == 25 and res["numValidTransforms"] == 25
    assert res["meshTriangles"] > 0
    assert open(os.path.join(d, "processed.txt")).readline().strip() == "valid = " + ("true" if res["valid"] else "false")
    assert os.path.exists(os.path.join(d, "input.optimized.sens")) and os.path.exists(os.path.join(d, "input.ply"))
    app.close()
