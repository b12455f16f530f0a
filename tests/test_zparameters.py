"""CPU: the zParameters entry point pinned to the reference's own two parameter files
(FriedLiver/zParametersDefault.txt, zParametersBundlingDefault.txt: the only inputs of the boundary the reference
holds). GlobalAppState / GlobalBundlingState read them with mLib's ParameterFile (GlobalAppState.h:128-136,
GlobalBundlingState.h:15-65, FriedLiver.cpp:228-250).

* the committed fixture (tests/golden/zparameters_reference.json) equals the files, read independently
  (container only: /root/reference does not exist on the GPU box);
* the C++ parameter path (bf_params_*) reads the files verbatim to the same values, key by key;
* params.py's APP_DEFAULTS / BUNDLING_DEFAULTS equal the files, except the documented s_sensorIdx 7 -> 8
  (SensorDataReader, the offline .sens reader the path runs; the file's 7 is the StructureSensor);
* bf_app_resolve (the parameter half of bf_app_create) accepts the verbatim files with only the sensor file
  overridden, derives the values the reference code derives from them, and derives bit-identical structs
  from the files params.py writes."""
import json
import os

import numpy as np
import pytest

from bundlefusion_amd.app import resolve
from bundlefusion_amd.io import ParameterFile
from bundlefusion_amd.params import APP_DEFAULTS, BUNDLING_DEFAULTS, write_parameter_files
from golden.make_zparameters_fixture import FILES, read_parameter_text

REF = "/root/reference/FriedLiver"
HAVE_REF = all(os.path.exists(os.path.join(REF, f)) for f in FILES)
needs_ref = pytest.mark.skipif(not HAVE_REF, reason="the reference tree exists only in the build container")
FIXTURE = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "zparameters_reference.json")))
APP_FILE, BUNDLING_FILE = FILES
DEVIATIONS = {"s_sensorIdx": (7, 8)}  # app file: StructureSensor in the file, SensorDataReader on this path


def typed(raw: str):
    """The raw value text as ParameterFile's typed reads see it: bool, string, number or list of numbers."""
    if raw in ("true", "false"):
        return raw == "true"
    if raw.startswith('"'):
        return raw.strip('"')
    parts = [float(p.rstrip("f")) for p in raw.split()]
    return parts[0] if len(parts) == 1 else tuple(parts)


def same(a, b) -> bool:
    if isinstance(a, bool) or isinstance(b, bool) or isinstance(a, str) or isinstance(b, str):
        return a == b
    return np.array_equal(np.float32(a), np.float32(b))


@needs_ref
def test_fixture_equals_reference_files():
    for f in FILES:
        with open(os.path.join(REF, f), encoding="latin-1") as fh:
            assert read_parameter_text(fh.read()) == FIXTURE[f], f


@needs_ref
@pytest.mark.parametrize("name", FILES)
def test_cpp_parser_reads_reference_files_verbatim(name):
    pf = ParameterFile(os.path.join(REF, name))
    for key, raw in FIXTURE[name].items():
        assert key in pf, key
        v = typed(raw)
        if isinstance(v, bool):
            assert pf.boolean(key) == v, key
        elif isinstance(v, str):
            assert pf.string(key) == v, key
        else:
            np.testing.assert_array_equal(pf.floats(key), np.float32(np.atleast_1d(v)), err_msg=key)
            if not isinstance(v, tuple):
                assert np.float32(pf.number(key)) == np.float32(v), key


@pytest.mark.parametrize("defaults,name", [(APP_DEFAULTS, APP_FILE), (BUNDLING_DEFAULTS, BUNDLING_FILE)])
def test_param_defaults_equal_reference_files(defaults, name):
    ref = FIXTURE[name]
    checked = 0
    for key, val in defaults.items():
        assert key in ref, f"{key} is not a key of {name}"
        r = typed(ref[key])
        if key in DEVIATIONS:
            assert (r, val) == DEVIATIONS[key], key
            continue
        assert same(r, val), (key, r, val)
        checked += 1
    assert checked == len(defaults) - sum(k in defaults for k in DEVIATIONS)


def _write_fixture_files(d):
    """The two files rebuilt from the fixture (the reference's settings, key for key)."""
    paths = []
    for f in FILES:
        p = os.path.join(d, f)
        with open(p, "w") as fh:
            for k, v in FIXTURE[f].items():
                fh.write(f"{k} = {v};\n")
        paths.append(p)
    return paths


@pytest.fixture(scope="module")
def sens(tmp_path_factory):
    from bundlefusion_amd.stream import write_synthetic_sens
    p = str(tmp_path_factory.mktemp("zp") / "input.sens")
    write_synthetic_sens(p, 3, 640, 480, device=False)
    return p


def _fields(s, prefix=""):
    import ctypes as C
    out = {}
    for name, t in s._fields_:
        v = getattr(s, name)
        if isinstance(v, C.Structure):
            out.update(_fields(v, prefix + name + "."))
        elif isinstance(v, C.Array):
            out[prefix + name] = tuple(v)
        else:
            out[prefix + name] = v
    return out


def _resolved(app, bundling, sens):
    info, loop = resolve(app, bundling, sens)
    return _fields(info), _fields(loop)


@needs_ref
def test_app_accepts_reference_files_with_only_the_sensor_override(sens):
    info, loop = _resolved(os.path.join(REF, APP_FILE), os.path.join(REF, BUNDLING_FILE), sens)
    A = {k: typed(v) for k, v in FIXTURE[APP_FILE].items()}
    B = {k: typed(v) for k, v in FIXTURE[BUNDLING_FILE].items()}
    f32 = np.float32
    # GlobalAppState -> HashParams (CUDASceneRepHashSDF.h:39-59)
    assert f32(info["hashParams.virtualVoxelSize"]) == f32(A["s_SDFVoxelSize"])
    assert info["hashParams.hashNumBuckets"] == A["s_hashNumBuckets"]
    assert info["hashParams.numSDFBlocks"] == A["s_hashNumSDFBlocks"]
    assert info["hashParams.hashMaxCollisionLinkedListSize"] == A["s_hashMaxCollisionLinkedListSize"]
    assert f32(info["hashParams.truncation"]) == f32(A["s_SDFTruncation"])
    assert f32(info["hashParams.truncScale"]) == f32(A["s_SDFTruncationScale"])
    assert f32(info["hashParams.maxIntegrationDistance"]) == f32(A["s_SDFMaxIntegrationDistance"])
    assert info["hashParams.integrationWeightSample"] == A["s_SDFIntegrationWeightSample"]
    assert info["hashParams.integrationWeightMax"] == A["s_SDFIntegrationWeightMax"]
    # the integration camera: the sensor intrinsics resampled to s_integrationWidth x Height
    # (CUDAImageManager.h:160-166), depth range from s_renderDepthMin / Max (DepthSensing.cpp:636-643)
    cam_w, cam_h = int(A["s_integrationWidth"]), int(A["s_integrationHeight"])
    assert (info["integrationCamera.imageWidth"], info["integrationCamera.imageHeight"]) == (cam_w, cam_h)
    fx = f32(577.87) * (f32(cam_w) / f32(640))
    assert f32(info["integrationCamera.fx"]) == f32(fx)
    assert f32(info["integrationCamera.sensorDepthWorldMin"]) == f32(A["s_renderDepthMin"])
    assert f32(info["integrationCamera.sensorDepthWorldMax"]) == f32(A["s_renderDepthMax"])
    # preprocessing from the BUNDLING file (its s_depthFilter / s_depthSigma* win; the app file's are unused)
    assert info["preprocess.erode"] == int(B["s_erodeSIFTdepth"])
    assert info["preprocess.depthFilter"] == int(B["s_depthFilter"]) == 1
    assert f32(info["preprocess.sigmaD"]) == f32(B["s_depthSigmaD"])
    assert f32(info["preprocess.sigmaR"]) == f32(B["s_depthSigmaR"]) != f32(A["s_depthSigmaR"])
    # CUDACache (Bundler.cpp:33-38)
    assert (info["cache.width"], info["cache.height"]) == (B["s_downsampledWidth"], B["s_downsampledHeight"])
    assert f32(info["cache.colorSigma"]) == f32(B["s_colorDownSigma"])
    assert f32(info["cache.depthSigmaD"]) == f32(B["s_depthDownSigmaD"])
    assert f32(info["cache.depthSigmaR"]) == f32(B["s_depthDownSigmaR"])
    assert info["submapSize"] == B["s_submapSize"]
    assert info["numSolveFramesBeforeExit"] == A["s_numSolveFramesBeforeExit"]
    # the loop: TrajectoryManager + OnlineBundler schedules and thresholds
    assert loop["maxFrameFixes"] == A["s_maxFrameFixes"] and loop["topNActive"] == A["s_topNActive"]
    assert f32(loop["minPoseDistSqrt"]) == f32(A["s_minPoseDistSqrt"])
    assert (loop["localNonLin"], loop["localLin"]) == (B["s_numLocalNonLinIterations"], B["s_numLocalLinIterations"])
    assert (loop["globalNonLin"], loop["globalLin"]) == (B["s_numGlobalNonLinIterations"], B["s_numGlobalLinIterations"])
    assert f32(loop["maxResidualThresh"]) == f32(B["s_optMaxResThresh"])
    assert loop["useLocalDense"] == int(B["s_useLocalDense"])
    assert loop["disableLocalVerify"] == int(not B["s_useLocalVerify"])
    assert f32(loop["verify.verifyOptErrThresh"]) == f32(B["s_verifyOptErrThresh"])
    assert f32(loop["verify.verifyOptCorrThresh"]) == f32(B["s_verifyOptCorrThresh"])
    assert f32(loop["solver.denseDistThresh"]) == f32(B["s_denseDistThresh"])
    assert f32(loop["solver.denseNormalThresh"]) == f32(B["s_denseNormalThresh"])
    assert loop["solver.denseOverlapSubsample"] == B["s_denseOverlapCheckSubsampleFactor"]


@needs_ref
def test_fixture_files_resolve_like_the_reference_files(sens, tmp_path):
    got = _resolved(*_write_fixture_files(str(tmp_path)), sens)
    ref = _resolved(os.path.join(REF, APP_FILE), os.path.join(REF, BUNDLING_FILE), sens)
    assert got == ref


def test_params_py_files_resolve_like_the_reference_settings(sens, tmp_path):
    """The files params.py writes (its defaults) give bf_app_resolve the same structs as the reference's own
    settings (rebuilt from the fixture): every key the path reads agrees."""
    ref = _resolved(*_write_fixture_files(str(tmp_path)), sens)
    d = tmp_path / "ours"
    d.mkdir()
    got = _resolved(*write_parameter_files(str(d), {}, {}, sens=sens), sens)
    assert got == ref


def test_resolve_rejects_what_bf_app_create_rejects(sens, tmp_path):
    """The parameter stage's checks (FriedLiver.cpp / SensorDataReader): a stream longer than s_maxNumImages x
    s_submapSize, a missing sensor file, a stream without colour."""
    import bundlefusion_amd as bfa
    pa, pb = write_parameter_files(str(tmp_path), {}, {"s_maxNumImages": 1, "s_submapSize": 2}, sens=sens)
    with pytest.raises(bfa.BFError, match="please change param file"):
        resolve(pa, pb, sens)  # 3 frames > 1 x 2
    pa, pb = write_parameter_files(str(tmp_path), {}, {}, sens=sens)
    with pytest.raises(bfa.BFError):
        resolve(pa, pb, str(tmp_path / "missing.sens"))
    info, loop = resolve(pa, pb, sens, max_frames=2)  # maxFrames caps the stream
    assert info.numFrames == 2 and loop.maxFrames == 2
