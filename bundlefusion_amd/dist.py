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

    def close(self):
        if self.dist is not None and self.dist.is_initialized():
            self.dist.destroy_process_group()


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
