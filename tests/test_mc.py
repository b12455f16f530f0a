"""Marching-cubes mesh extraction (CUDAMarchingCubesHashSDF::extractIsoSurface + saveMesh,
/root/reference/FriedLiver/Source/DepthSensing/CUDAMarchingCubesHashSDF.cpp:48-118,
MarchingCubesSDFUtil.h:119-227).

CPU: the compiled case tables against the reference's own Tables.h (golden fixture), an analytic
known-answer test of the oracle restatement (a fronto-parallel wall: the projective SDF is linear in
z, so every vertex lies on the wall), and the host mesh merge / PLY writer of the C ABI.
GPU: bf_scene_extract_mesh against the oracle on identical volumes, bit for bit (as multisets: heap
block numbering follows the allocation schedule); the GPU's fixed output order run to run; the
maxNumTriangles cap and the box filter."""
import json
import os
import struct

import numpy as np
import pytest

import bundlefusion_amd as bfa
from oracle_lib import OracleScene, mc_tables

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "mc_tables.json")
# corner pairs of the 12 edges in cubeindex-bit order (vertexInterp calls, MarchingCubesSDFUtil.h:181-192)
EDGE_A = [0, 1, 2, 3, 4, 5, 6, 7, 0, 1, 2, 3]
EDGE_B = [1, 2, 3, 0, 5, 6, 7, 4, 4, 5, 6, 7]


def test_case_tables_match_reference_tables():
    g = json.load(open(GOLDEN))
    edges, ntri, tri = mc_tables()
    # edgeTable: derived from the edge topology in mc_tables.h, equal to the reference's literal table
    assert edges.tolist() == g["edgeTable"]
    for c in range(256):
        ref = [int(ch, 16) for ch in g["triTableCases"][c]]
        assert ntri[c] * 3 == len(ref)
        assert tri[c, : len(ref)].tolist() == ref
        # every triangle edge crosses the iso level, and every crossing edge is used
        used = 0
        for e in ref:
            used |= 1 << e
        assert used == int(edges[c]), c
        for e in range(12):
            assert bool(edges[c] >> e & 1) == (((c >> EDGE_A[e]) & 1) != ((c >> EDGE_B[e]) & 1))


def wall_scene(vs=0.01, W=64, H=48, depth=1.0, rgb=(200, 100, 50)):
    f = 577.87 * W / 640.0
    cam = bfa.depth_camera(W, H, fx=f, fy=f)
    p = bfa.hash_params(voxel_size=vs, num_buckets=1 << 14, num_blocks=1 << 13)
    d = np.full((H, W), depth, np.float32)
    c = np.zeros((H, W, 4), np.uint8)
    c[..., 0], c[..., 1], c[..., 2], c[..., 3] = rgb[0], rgb[1], rgb[2], 255
    return p, cam, d, c


def test_oracle_wall_known_answer():
    """A wall at z = 1 m seen from the origin: sdf = 1 - z at every voxel of the band, trilinear
    samples of a linear field are exact, so every vertex has z = 1 (to float rounding) and the
    colour of the wall."""
    vs = 0.01
    p, cam, d, c = wall_scene(vs)
    o = OracleScene(p)
    T = np.eye(4, dtype=np.float32)
    o.integrate(T, d, c, cam)
    o.integrate(T, d, c, cam)
    tris, total = o.extract_mesh(bfa.mc_params(vs))
    assert total == len(tris) > 100
    xyz, rgb = tris[..., :3], tris[..., 3:]
    assert np.max(np.abs(xyz[..., 2] - 1.0)) < 2e-5
    assert np.allclose(rgb.reshape(-1, 3), np.float32([200, 100, 50]) / np.float32(255), atol=0)
    # flat triangles: each normal is along z
    n = np.cross(xyz[:, 1] - xyz[:, 0], xyz[:, 2] - xyz[:, 0])
    n /= np.linalg.norm(n, axis=1, keepdims=True)
    assert np.min(np.abs(n[:, 2])) > 0.999
    # the cap keeps the first triangles of the same order
    cap = bfa.mc_params(vs, max_triangles=37)
    part, tot2 = o.extract_mesh(cap)
    assert tot2 == total and len(part) == 37 and np.array_equal(part, tris[:37])


def test_mesh_merge_and_ply_roundtrip(tmp_path):
    """saveMesh's host side (bf_mesh_merge / bf_mesh_save_ply, no GPU needed): shared corners merge
    (within 1e-5), duplicate faces (same vertex set) and degenerate faces go, transform applies."""
    def tri(a, b, c, col=(1.0, 0.5, 0.25)):
        return np.array([list(a) + list(col), list(b) + list(col), list(c) + list(col)], np.float32)
    t = np.stack([
        tri((0, 0, 0), (1, 0, 0), (0, 1, 0)),
        tri((1, 0, 0), (1, 1, 0), (0, 1, 0)),            # shares an edge with the first
        tri((0, 1, 0), (0, 0, 0), (1, 0, 0)),            # the first again, rotated: duplicate face
        tri((0, 0, 0), (0.000001, 0, 0), (0, 1, 0)),     # two corners merge: degenerate
        tri((2, 2, 2), (3, 2, 2), (2, 3, 2.000001)),     # separate; last corner snaps onto its own cell
    ])
    v, c, f = bfa.mesh_merge(t)
    assert len(v) == 7 and len(f) == 3
    assert f.tolist() == [[0, 1, 2], [1, 3, 2], [4, 5, 6]]
    assert np.allclose(c[:, 3], 1.0)
    T = np.eye(4, dtype=np.float32)
    T[:3, 3] = (10, 20, 30)
    v2, _, f2 = bfa.mesh_merge(t, T)
    assert np.allclose(v2, v + np.float32([10, 20, 30])) and np.array_equal(f2, f)
    path = str(tmp_path / "mesh.ply")
    nv, nf = bfa.mesh_save_ply(path, t)
    assert (nv, nf) == (7, 3)
    raw = open(path, "rb").read()
    head, body = raw.split(b"end_header\n", 1)
    assert b"format binary_little_endian 1.0" in head and b"element vertex 7" in head and b"element face 3" in head
    verts = [struct.unpack_from("<3f4B", body, 16 * i) for i in range(7)]
    assert np.allclose([vv[:3] for vv in verts], v)
    assert verts[0][3:] == (255, 128, 64, 255)
    off = 16 * 7
    faces = [struct.unpack_from("<B3i", body, off + 13 * i) for i in range(3)]
    assert [list(fc[1:]) for fc in faces] == f.tolist() and all(fc[0] == 3 for fc in faces)
    assert len(body) == off + 13 * 3
    assert bfa.mesh_merge(np.zeros((0, 3, 6), np.float32))[2].shape == (0, 3)


# ---- GPU parity ------------------------------------------------------------------------------
def canon(tris):
    """Triangles as rows of 18 raw float bits, sorted: the GPU emits in heap-block order, and which
    heap block a hash entry received depends on the allocation schedule (the reference's too), so
    the comparison is of the multiset of triangles, bit for bit."""
    u = np.ascontiguousarray(tris).view(np.uint32).reshape(len(tris), 18)
    return u[np.lexsort(u.T[::-1])]


def gpu_pair(W=160, H=120, vs=0.01, frames=(0, 3, 6, 9)):
    from tsdf_compare import Pair, render_frames
    sc = bfa.synth_scene(0)
    f = 577.87 * W / 640.0
    cam = bfa.depth_camera(W, H, fx=f, fy=f)
    p = bfa.hash_params(voxel_size=vs, num_buckets=1 << 16, num_blocks=1 << 15)
    pair = Pair(p, cam)
    for k, (T, d, c) in enumerate(render_frames(sc, cam, list(frames))):
        pair.integrate(k, T, d, c)
    pair.gc()
    return pair


@pytest.mark.gpu
def test_mc_gpu_matches_oracle_bitwise():
    pair = gpu_pair()
    mc = bfa.mc_params(0.01)
    g, gt = pair.gpu.extract_mesh(mc)
    o, ot = pair.ora.extract_mesh(mc)
    assert gt == ot == len(o) > 1000
    assert np.array_equal(canon(g), canon(o))
    g2, _ = pair.gpu.extract_mesh(mc)  # deterministic order run to run
    assert np.array_equal(g2.view(np.uint32), g.view(np.uint32))


@pytest.mark.gpu
def test_mc_gpu_cap_box_and_deintegrated_scene():
    pair = gpu_pair(frames=(0, 5))
    mc = bfa.mc_params(0.01)
    full, total = pair.gpu.extract_mesh(mc)
    cap = bfa.mc_params(0.01, max_triangles=total // 3)
    part, t2 = pair.gpu.extract_mesh(cap)
    assert t2 == total and len(part) == total // 3 and np.array_equal(part, full[: total // 3])
    c = full[..., :3].reshape(-1, 3).mean(0)
    box = bfa.mc_params(0.01, box=(c - 0.5, c + 0.5))
    gb, gbt = pair.gpu.extract_mesh(box)
    ob, obt = pair.ora.extract_mesh(box)
    assert 0 < gbt == obt < total and np.array_equal(canon(gb), canon(ob))
    # de-integrate everything: weights return to 0 and no surface is left
    from tsdf_compare import render_frames
    sc = bfa.synth_scene(0)
    for k, (T, d, cc) in enumerate(render_frames(sc, pair.cam, [0, 5])):
        pair.integrate(k, T, d, cc, deint=True)
    g0, t0 = pair.gpu.extract_mesh(mc)
    o0, u0 = pair.ora.extract_mesh(mc)
    assert t0 == u0 == 0 and len(g0) == 0
