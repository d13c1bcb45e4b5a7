"""One-rank RCCL transport check (run by tests/test_gpu_distributed.py::test_rccl_one_rank_transport).

A single process creates the RCCL communicator exactly as a rank of bench.py --gpus N does (unique id broadcast over
the gloo control plane, ncclCommInitRank) and runs the transport's operations through the C-ABI
(sx_comm_alltoallv, sx_comm_allreduce) on device buffers of the context stream.
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sph-exa_amd", "python"))


def main():
    import torch.distributed as dist

    dist.init_process_group("gloo")
    import sphexa_amd as sx

    ctx = sx.Context(0)
    comm = sx.Comm("rccl")
    stream = ctx.L.sx_get_stream(ctx.h)
    rng = np.random.default_rng(5)

    payload = rng.integers(0, 255, 1000, dtype=np.uint8)
    src = ctx.upload(payload)
    dst = ctx.alloc(1200, np.uint8)
    ctx.L.sx_memset(ctx.h, dst.ptr, 0, 1200)
    comm.alltoallv(src.ptr, [1000], [0], C.c_void_p(dst.ptr + 100).value, [1000], [0], stream)
    ctx.sync()
    got = dst.get()
    assert np.array_equal(got[100:1100], payload) and not got[:100].any() and not got[1100:].any()

    u = rng.integers(0, 1 << 20, 4096).astype(np.uint32)
    du = ctx.upload(u)
    comm.allreduce(du.ptr, u.size, "sum_u32", stream)
    f = rng.standard_normal(33)
    df = ctx.upload(f)
    comm.allreduce(df.ptr, f.size, "min_f64", stream)
    dg = ctx.upload(f)
    comm.allreduce(dg.ptr, f.size, "sum_f64", stream)
    ctx.sync()
    assert np.array_equal(du.get(), u) and np.array_equal(df.get(), f) and np.array_equal(dg.get(), f)

    # a zero-byte exchange (every peer empty: the sync's "nothing moves" case) must leave the RCCL group closed, and
    # an allreduce on a stream other than the context's must not leave one open either: the operations after each
    # run normally
    comm.alltoallv(src.ptr, [0], [0], dst.ptr, [0], [0], stream)
    comm.allreduce(du.ptr, u.size, "sum_u32", stream)
    hip = C.CDLL("libamdhip64.so")
    other = C.c_void_p()
    assert hip.hipStreamCreate(C.byref(other)) == 0
    dh = ctx.upload(u)
    comm.allreduce(dh.ptr, u.size, "sum_u32", other.value)
    assert hip.hipStreamSynchronize(other) == 0
    ctx.L.sx_memset(ctx.h, dst.ptr, 0, 1200)
    comm.alltoallv(src.ptr, [1000], [0], dst.ptr, [1000], [0], stream)
    comm.allreduce(df.ptr, f.size, "min_f64", stream)
    ctx.sync()
    assert hip.hipStreamDestroy(other) == 0
    assert np.array_equal(dh.get(), u) and np.array_equal(du.get(), u) and np.array_equal(df.get(), f)
    assert np.array_equal(dst.get()[:1000], payload)
    comm.close()
    ctx.close()
    dist.destroy_process_group()
    print("RCCL one-rank OK: alltoallv (self segment, zero bytes) and allreduce sum_u32/min_f64/sum_f64 through "
          "RcclTransport, on the context stream and another stream")


if __name__ == "__main__":
    main()
