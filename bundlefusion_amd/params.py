"""Parameter files in the zParameters*.txt format (mLib ParameterFile: `name = value;`, `//` comments) for
the keys the north-star path reads, with the values of FriedLiver's own zParametersDefault.txt /
zParametersBundlingDefault.txt (SURVEY.md §5 "Config / flag system", Appendix B) unless overridden —
what the bench's `--sens` mode and the application tests hand bf_app_create when the user brings no
parameter files of their own."""
from __future__ import annotations

# GlobalAppState keys of the path (zParametersDefault.txt:1-117)
APP_DEFAULTS = {
    "s_sensorIdx": 8,
    "s_numSolveFramesBeforeExit": 30,
    "s_integrationWidth": 320, "s_integrationHeight": 240,
    "s_rayCastWidth": 320, "s_rayCastHeight": 240,
    "s_maxFrameFixes": 10, "s_topNActive": 30, "s_minPoseDistSqrt": 0.0,
    "s_sensorDepthMax": 4.0, "s_sensorDepthMin": 0.1, "s_renderDepthMax": 4.0, "s_renderDepthMin": 0.1,
    "s_SDFVoxelSize": 0.010, "s_SDFMarchingCubeThreshFactor": 10.0, "s_SDFTruncation": 0.06,
    "s_SDFTruncationScale": 0.02, "s_SDFMaxIntegrationDistance": 3.0, "s_SDFIntegrationWeightSample": 1,
    "s_SDFIntegrationWeightMax": 99999999,
    "s_hashNumBuckets": 800000, "s_hashNumSDFBlocks": 200000, "s_hashMaxCollisionLinkedListSize": 7,
    "s_SDFRayIncrementFactor": 0.8, "s_SDFRayThresSampleDistFactor": 50.5, "s_SDFRayThresDistFactor": 50.0,
    "s_SDFUseGradients": False,
    "s_binaryDumpSensorFile": "../data/sequence.sens",
    "s_marchingCubesMaxNumTriangles": 3000000,
    "s_streamingEnabled": False, "s_streamingVoxelExtents": (1.0, 1.0, 1.0),
    "s_streamingGridDimensions": (257, 257, 257), "s_streamingMinGridPos": (-128, -128, -128),
    "s_streamingInitialChunkListSize": 2000,
    # the app file's own (unused on the path) filter keys: the bundling file's win for preprocessing
    "s_depthSigmaD": 2.0, "s_depthSigmaR": 0.1, "s_depthFilter": False,
}

# GlobalBundlingState keys of the path (zParametersBundlingDefault.txt)
BUNDLING_DEFAULTS = {
    "s_erodeSIFTdepth": True,
    "s_widthSIFT": 640, "s_heightSIFT": 480,
    "s_optMaxResThresh": 0.08, "s_denseDistThresh": 0.15, "s_denseNormalThresh": 0.97, "s_denseColorThresh": 0.1,
    "s_denseColorGradientMin": 0.005, "s_denseDepthMin": 0.5, "s_denseDepthMax": 4.0,
    "s_denseOverlapCheckSubsampleFactor": 4,
    "s_maxNumImages": 1200, "s_submapSize": 10, "s_maxNumKeysPerImage": 1024,
    "s_useLocalDense": True, "s_numOptPerResidualRemoval": 1,
    "s_numLocalNonLinIterations": 2, "s_numLocalLinIterations": 100,
    "s_numGlobalNonLinIterations": 3, "s_numGlobalLinIterations": 150,
    "s_downsampledWidth": 80, "s_downsampledHeight": 60,
    "s_colorDownSigma": 2.5, "s_depthDownSigmaD": 1.0, "s_depthDownSigmaR": 0.05,
    "s_projCorrDistThres": 0.15, "s_projCorrNormalThres": 0.97, "s_projCorrColorThresh": 0.1,
    "s_useLocalVerify": True, "s_verifyOptErrThresh": 0.05, "s_verifyOptCorrThresh": 0.001,
    "s_minNumMatchesLocal": 5, "s_minNumMatchesGlobal": 5,
    "s_depthSigmaD": 2.0, "s_depthSigmaR": 0.05, "s_depthFilter": True,
}

# BASELINE.json's north-star stream: 640x480 integration at 4 mm voxels (SURVEY.md §8(d) "Parameters")
NORTH_STAR_APP = {"s_integrationWidth": 640, "s_integrationHeight": 480, "s_rayCastWidth": 640,
                  "s_rayCastHeight": 480, "s_SDFVoxelSize": 0.004, "s_hashNumBuckets": 1 << 23,
                  "s_hashNumSDFBlocks": 1 << 21}


def _fmt(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, str):
        return f'"{v}"'
    if isinstance(v, (tuple, list)):
        return " ".join(_fmt(x) for x in v)
    if isinstance(v, float):
        return f"{v!r}f"
    return str(v)


def write_zparameters(path: str, values: dict, header: str = "") -> str:
    with open(path, "w") as f:
        if header:
            f.write(f"// {header}\n")
        for k, v in values.items():
            f.write(f"{k} = {_fmt(v)};\n")
    return path


def write_parameter_files(directory: str, app: dict | None = None, bundling: dict | None = None, sens: str | None = None):
    """zParametersDefault-style app file + bundling file in `directory`; returns their paths."""
    import os
    a = dict(APP_DEFAULTS, **(app or {}))
    if sens is not None:
        a["s_binaryDumpSensorFile"] = sens
    b = dict(BUNDLING_DEFAULTS, **(bundling or {}))
    pa = write_zparameters(os.path.join(directory, "zParametersApp.txt"), a, "GlobalAppState")
    pb = write_zparameters(os.path.join(directory, "zParametersBundling.txt"), b, "GlobalBundlingState")
    return pa, pb
