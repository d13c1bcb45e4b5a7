/*! @file sx_comm.hpp
 * @brief Inter-GPU transport of the SFC domain decomposition.
 *
 * Replaces the reference's MPI point-to-point halo / particle exchange and MPI_Allreduce
 * (halos/exchange_halos_gpu.cuh:51-143, domain/domaindecomp_mpi_gpu.cuh:86-171, tree/update_mpi_gpu.cuh:75,
 * sph/ts_global.hpp:106) with two operations on device buffers:
 *   alltoallv  -- every rank sends sendBytes[q] from send+sendOff[q] to rank q, receiving recvBytes[q] at
 *                 recv+recvOff[q] (recv may be a field array: halos land in place, no unpack pass);
 *   allreduce  -- u32 sum (global key histogram), f64 min (time-step), u32 min/max (displacement grid of the skin
 *                 lists).
 * Backends: RCCL (one communicator per node, grouped ncclSend/ncclRecv per peer over xGMI, collectives on device
 * buffers, all on the compute stream) and a host-staged backend that calls back into the caller (used with
 * torch.distributed/gloo to run several ranks on one GPU in the tests).
 */
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace sx
{

class Transport
{
public:
    virtual ~Transport()                   = default;
    virtual int  rank() const              = 0;
    virtual int  size() const              = 0;
    virtual bool alltoallv(const void* send, const uint64_t* sendBytes, const uint64_t* sendOff, void* recv,
                           const uint64_t* recvBytes, const uint64_t* recvOff, hipStream_t s) = 0;
    virtual bool allreduceSumU32(uint32_t* dev, size_t count, hipStream_t s)                  = 0;
    virtual bool allreduceMinF64(double* dev, size_t count, hipStream_t s)                    = 0;
    virtual bool allreduceSumF64(double* dev, size_t count, hipStream_t s)                    = 0;
    //! u32 min / max (the skin lists' displacement grid: per cell the component ranges of every rank's particles)
    virtual bool allreduceMinU32(uint32_t* dev, size_t count, hipStream_t s)                  = 0;
    virtual bool allreduceMaxU32(uint32_t* dev, size_t count, hipStream_t s)                  = 0;

    //! host-count convenience: exchange one u64 per peer (counts), synchronous
    bool exchangeCounts(const std::vector<uint64_t>& send, std::vector<uint64_t>& recv, hipStream_t s, uint64_t* devBuf);
};

} // namespace sx
