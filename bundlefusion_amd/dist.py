"""Host-side multi-process plumbing for one process per GPU (torchrun): rank discovery, a gloo
group for barriers, max-over-ranks timing and the RCCL id hand-off, and the TSDF shard assignment.
The TSDF data path has no collective: each rank integrates only the 1 m chunks it owns (SURVEY.md
§8(e)1). The global bundle adjustment shards its image-pair normal-equation blocks over the ranks
and sums them with one RCCL all-reduce per Gauss-Newton iteration (Comm)."""
from __future__ import annotations

import os


def env_rank():
    """(rank, world_size, local_rank) from the torchrun environment (1 process when unset)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


class HostGroup:
    """gloo process group used only for host synchronisation (barrier, max of a float)."""

    def __init__(self, rank: int, world: int):
        self.rank, self.world = rank, world
        self.dist = None
        if world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max(self, value: float) -> float:
        if self.dist is None:
            return value
        import torch
        t = torch.tensor([value], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, value: float) -> float:
        if self.dist is None:
            return value
        import torch
        t = torch.tensor([value], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def broadcast_bytes(self, data: bytes | None, n: int) -> bytes:
        """rank 0's n bytes on every rank (the RCCL unique id hand-off)."""
        if self.dist is None:
            return data
        import torch
        t = torch.zeros(n, dtype=torch.uint8)
        if self.rank == 0:
            t[:] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        self.dist.broadcast(t, src=0)
        return bytes(t.numpy().tobytes())

    def agree(self, what: str, digest: bytes) -> None:
        """Every rank must run on the same inputs (replicated bundling, one order of collectives): rank 0's
        digest is broadcast and any rank holding another fails on every rank."""
        if self.dist is None:
            return
        ref = self.broadcast_bytes(digest if self.rank == 0 else None, len(digest))
        bad = self.max(0.0 if ref == digest else 1.0)
        if bad:
            raise RuntimeError(f"ranks disagree on {what}" + (" (this rank differs from rank 0)" if ref != digest else ""))

    def close(self):
        if self.dist is not None and self.dist.is_initialized():
            self.dist.destroy_process_group()


def input_digest(paths, head_bytes: int = 1 << 20) -> bytes:
    """32-byte digest of input files: size and first head_bytes of each (a .sens header and its first
    frames, parameter files whole)."""
    import hashlib
    h = hashlib.sha256()
    for p in paths:
        h.update(str(os.path.getsize(p)).encode())
        with open(p, "rb") as f:
            h.update(f.read(head_bytes))
    return h.digest()


class Comm:
    """RCCL communicator of the C library (bf_comm_*): rank 0 draws the unique id, the host group
    broadcasts it, every rank joins. Used by the sharded global solve (bf_recon_set_comm /
    SolverBundling.set_shard)."""

    ID_BYTES = 128

    def __init__(self, group: HostGroup):
        import ctypes as C
        from . import check, lib
        self.rank, self.world = group.rank, group.world
        uid = None
        if group.rank == 0:
            buf = (C.c_uint8 * self.ID_BYTES)()
            check(lib().bf_comm_unique_id(buf))
            uid = bytes(buf)
        uid = group.broadcast_bytes(uid, self.ID_BYTES)
        self.h = C.c_void_p()
        idbuf = (C.c_uint8 * self.ID_BYTES).from_buffer_copy(uid)
        check(lib().bf_comm_create(idbuf, C.c_int(group.world), C.c_int(group.rank), C.byref(self.h)))

    def allreduce_sum_f64(self, d_array) -> None:
        import ctypes as C
        from . import check, lib
        check(lib().bf_comm_allreduce_sum_f64(self.h, d_array.ptr, C.c_size_t(d_array.nbytes // 8)))

    def close(self):
        from . import lib
        if self.h:
            lib().bf_comm_destroy(self.h)
            self.h = None


class LoopbackComm:
    """One rank of an in-process loopback group (bf_comm_create_loopback): the multi-rank loop's
    collectives for ranks driven from threads of one process sharing one GPU, each a one-workgroup kernel
    on the caller's stream that waits on the device for every rank (RCCL's asynchronous, stream-ordered
    semantics; tests, no RCCL). Same .h / .rank / .world / .close() as Comm."""

    def __init__(self, h, rank: int, world: int):
        self.h, self.rank, self.world = h, rank, world

    # streams one rank of a loop or FriedLiver app keeps busy (scene, bundling, local solve, result copies, input
    # preprocessing, cache): each needs a hardware queue of its own, or a collective spinning in a queue another
    # rank shares would hold that rank's arrival behind it (a 30-s stall, then the group's error)
    STREAMS_PER_RANK = 6

    @staticmethod
    def group(world: int, timeout_ms: int = 30000, capacity_bytes: int = 0) -> list["LoopbackComm"]:
        """The ranks' collectives wait on the device for each other, so the process needs at least
        world x STREAMS_PER_RANK hardware queues (GPU_MAX_HW_QUEUES, read by HIP at its initialisation: set it
        before the first HIP call, as tests/conftest.py does); fails fast otherwise. A spinning collective also
        holds one workgroup slot while it waits; another rank's persistent PCG grid that then cannot become
        resident times out and is redone in stream order, so the loop stays correct."""
        import ctypes as C
        import os
        from . import check, lib
        queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
        need = world * LoopbackComm.STREAMS_PER_RANK
        if world > 1 and queues < need:
            raise RuntimeError(f"loopback group of {world} ranks needs GPU_MAX_HW_QUEUES >= {need} "
                               f"(is {queues}); set it before HIP initialises")
        hs = (C.c_void_p * world)()
        check(lib().bf_comm_create_loopback(C.c_int(world), C.c_int(timeout_ms), C.c_size_t(capacity_bytes), hs))
        return [LoopbackComm(C.c_void_p(hs[r]), r, world) for r in range(world)]

    def allreduce_sum_f64(self, d_array) -> None:
        """In-place sum over the group's ranks (bf_comm_allreduce_sum_f64; synchronizes, checks the group)."""
        import ctypes as C
        from . import check, lib
        check(lib().bf_comm_allreduce_sum_f64(self.h, d_array.ptr, C.c_size_t(d_array.nbytes // 8)))

    def close(self):
        from . import lib
        if self.h:
            lib().bf_comm_destroy(self.h)
            self.h = None


def chunk_owner_array(blocks, voxel_size: float, shard_count: int, chunk: float = 1.0):
    """chunk_owner over an int array of block coordinates [n, 3] (same float32 / int32 arithmetic)."""
    import numpy as np
    b = np.asarray(blocks, np.int64)[:, :3]
    w = (b * 8).astype(np.float32) * np.float32(voxel_size)
    q = (w / np.float32(chunk)).astype(np.float32)
    c = np.trunc((q + np.sign(q).astype(np.float32) * np.float32(0.5)).astype(np.float32)).astype(np.int64)
    h = ((c[:, 0] * 73856093) ^ (c[:, 1] * 19349669) ^ (c[:, 2] * 83492791)) & 0xFFFFFFFF
    h = np.where(h >= (1 << 31), h - (1 << 32), h)
    r = np.abs(h) % shard_count
    r = np.where(h < 0, -r, r)
    return np.where(r < 0, r + shard_count, r).astype(np.int32)


def shard_balance(blocks, voxel_size: float, poses, cam, shard_counts=(2, 4, 8), chunk: float = 1.0) -> dict:
    """Load balance of the chunk-ownership TSDF sharding for a final scene: per shard
    count G, the allocated blocks each rank stores and, over the given camera poses, the in-frustum
    allocated blocks each rank scans and updates (the per-frame voxel work, isInCameraFrustumApprox at
    the block centre, DepthCameraUtil.h:95-107); max / mean over ranks."""
    import numpy as np
    b = np.asarray(blocks, np.int64)[:, :3]
    ctr = (b * 8).astype(np.float64) * voxel_size + voxel_size * 0.5 * 7.0
    vis = np.zeros(len(b), np.int64)
    for T in poses:
        Ti = np.linalg.inv(np.asarray(T, np.float64))
        p = ctr @ Ti[:3, :3].T + Ti[:3, 3]
        z = p[:, 2]
        with np.errstate(divide="ignore", invalid="ignore"):
            u = p[:, 0] * cam.fx / z + cam.mx
            v = p[:, 1] * cam.fy / z + cam.my
        nx = (2.0 * u - (cam.imageWidth - 1.0)) / (cam.imageWidth - 1.0) * 0.95
        ny = ((cam.imageHeight - 1.0) - 2.0 * v) / (cam.imageHeight - 1.0) * 0.95
        nz = (z - cam.sensorDepthWorldMin) / (cam.sensorDepthWorldMax - cam.sensorDepthWorldMin) * 0.95
        vis += ((z > 0) & (np.abs(nx) <= 1) & (np.abs(ny) <= 1) & (nz >= 0) & (nz <= 1)).astype(np.int64)
    out = {"blocks": int(len(b)), "frames": len(poses), "chunk_m": chunk}
    for G in shard_counts:
        own = chunk_owner_array(b, voxel_size, G, chunk=chunk)
        stored = np.bincount(own, minlength=G)
        work = np.bincount(own, weights=vis, minlength=G)
        out[f"G{G}"] = {"stored_max_over_mean": float(stored.max() / max(stored.mean(), 1e-9)),
                        "visible_max_over_mean": float(work.max() / max(work.mean(), 1e-9)),
                        "stored": stored.tolist(), "visible_block_frames": work.astype(int).tolist()}
    return out


def chunk_owner(bx: int, by: int, bz: int, voxel_size: float, shard_count: int, chunk: float = 1.0) -> int:
    """Shard owning block (bx, by, bz): computeHashPos of its 1 m chunk (worldToChunks rounding,
    CUDASceneRepHashSDF.cu:136-150) mod shard_count — the host mirror of owned() in csrc/tsdf.hip."""
    import numpy as np
    w = np.float32(bx * 8) * np.float32(voxel_size), np.float32(by * 8) * np.float32(voxel_size), \
        np.float32(bz * 8) * np.float32(voxel_size)
    c = []
    for v in w:
        q = np.float32(v / np.float32(chunk))
        s = np.float32(np.sign(q)) * np.float32(0.5)
        c.append(int(np.trunc(np.float32(q + s))))
    x, y, z = c
    # int32 products with wrap-around, done on Python ints (no numpy overflow warnings)
    h = ((x * 73856093) ^ (y * 19349669) ^ (z * 83492791)) & 0xFFFFFFFF
    h = h - (1 << 32) if h >= (1 << 31) else h
    r = abs(h) % shard_count          # C's fmod/% truncates toward zero
    r = -r if h < 0 else r
    return r + shard_count if r < 0 else r
