/*! @file sx_comm.cpp
 * @brief RCCL and host-staged transports (sx_comm.hpp) and their C-ABI constructors.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "../../include/sphexa_hip.h"
#include "sx_comm.hpp"

namespace sx
{

bool Transport::exchangeCounts(const std::vector<uint64_t>& send, std::vector<uint64_t>& recv, hipStream_t s,
                               uint64_t* devBuf)
{
    int P = size();
    recv.assign(P, 0);
    std::vector<uint64_t> bytes(P, 8), off(P);
    for (int q = 0; q < P; ++q)
        off[q] = 8 * q;
    // devBuf: 2*P u64 (send | recv)
    if (hipMemcpyAsync(devBuf, send.data(), 8 * P, hipMemcpyHostToDevice, s) != hipSuccess) return false;
    if (!alltoallv(devBuf, bytes.data(), off.data(), devBuf + P, bytes.data(), off.data(), s)) return false;
    if (hipMemcpyAsync(recv.data(), devBuf + P, 8 * P, hipMemcpyDeviceToHost, s) != hipSuccess) return false;
    return hipStreamSynchronize(s) == hipSuccess;
}

//! RCCL over xGMI: grouped point-to-point per peer (no ring; each peer message rides its own link)
class RcclTransport : public Transport
{
public:
    RcclTransport(int rank, int size, const ncclUniqueId& id)
        : rank_(rank)
        , size_(size)
    {
        ok_ = ncclCommInitRank(&comm_, size, id, rank) == ncclSuccess;
    }
    ~RcclTransport() override
    {
        if (ok_) ncclCommDestroy(comm_);
    }
    bool ok() const { return ok_; }
    int  rank() const override { return rank_; }
    int  size() const override { return size_; }

    bool alltoallv(const void* send, const uint64_t* sendBytes, const uint64_t* sendOff, void* recv,
                   const uint64_t* recvBytes, const uint64_t* recvOff, hipStream_t s) override
    {
        const char* sb = static_cast<const char*>(send);
        char*       rb = static_cast<char*>(recv);
        if (sendBytes[rank_] &&
            hipMemcpyAsync(rb + recvOff[rank_], sb + sendOff[rank_], sendBytes[rank_], hipMemcpyDeviceToDevice, s) !=
                hipSuccess)
            return false;
        if (ncclGroupStart() != ncclSuccess) return false;
        // a failed enqueue stops issuing further peers, but the group is always closed: returning between
        // ncclGroupStart and ncclGroupEnd would leave the thread's group open and poison every later RCCL call
        bool ok = true;
        for (int q = 0; q < size_ && ok; ++q)
        {
            if (q == rank_) continue;
            if (sendBytes[q]) ok = ncclSend(sb + sendOff[q], sendBytes[q], ncclUint8, q, comm_, s) == ncclSuccess;
            if (ok && recvBytes[q])
                ok = ncclRecv(rb + recvOff[q], recvBytes[q], ncclUint8, q, comm_, s) == ncclSuccess;
        }
        bool closed = ncclGroupEnd() == ncclSuccess;
        return ok && closed;
    }
    bool allreduceSumU32(uint32_t* dev, size_t count, hipStream_t s) override
    {
        return ncclAllReduce(dev, dev, count, ncclUint32, ncclSum, comm_, s) == ncclSuccess;
    }
    bool allreduceMinF64(double* dev, size_t count, hipStream_t s) override
    {
        return ncclAllReduce(dev, dev, count, ncclFloat64, ncclMin, comm_, s) == ncclSuccess;
    }
    bool allreduceSumF64(double* dev, size_t count, hipStream_t s) override
    {
        return ncclAllReduce(dev, dev, count, ncclFloat64, ncclSum, comm_, s) == ncclSuccess;
    }
    bool allreduceMinU32(uint32_t* dev, size_t count, hipStream_t s) override
    {
        return ncclAllReduce(dev, dev, count, ncclUint32, ncclMin, comm_, s) == ncclSuccess;
    }
    bool allreduceMaxU32(uint32_t* dev, size_t count, hipStream_t s) override
    {
        return ncclAllReduce(dev, dev, count, ncclUint32, ncclMax, comm_, s) == ncclSuccess;
    }

private:
    int          rank_, size_;
    ncclComm_t   comm_{};
    bool         ok_{false};
};

//! host-staged: device -> pinned host -> caller's collective (e.g. gloo) -> device
class HostTransport : public Transport
{
public:
    HostTransport(int rank, int size, sx_alltoallv_cb a2a, sx_allreduce_cb ar, void* user)
        : rank_(rank)
        , size_(size)
        , a2a_(a2a)
        , ar_(ar)
        , user_(user)
    {
    }
    int rank() const override { return rank_; }
    int size() const override { return size_; }

    bool alltoallv(const void* send, const uint64_t* sendBytes, const uint64_t* sendOff, void* recv,
                   const uint64_t* recvBytes, const uint64_t* recvOff, hipStream_t s) override
    {
        uint64_t ts = 0, tr = 0;
        for (int q = 0; q < size_; ++q)
            ts += sendBytes[q], tr += recvBytes[q];
        hs_.resize(ts + 1);
        hr_.resize(tr + 1);
        uint64_t o = 0;
        for (int q = 0; q < size_; ++q)
        {
            if (sendBytes[q] &&
                hipMemcpyAsync(hs_.data() + o, static_cast<const char*>(send) + sendOff[q], sendBytes[q],
                               hipMemcpyDeviceToHost, s) != hipSuccess)
                return false;
            o += sendBytes[q];
        }
        if (hipStreamSynchronize(s) != hipSuccess) return false;
        if (a2a_(user_, hs_.data(), sendBytes, hr_.data(), recvBytes) != 0) return false;
        o = 0;
        for (int q = 0; q < size_; ++q)
        {
            if (recvBytes[q] && hipMemcpyAsync(static_cast<char*>(recv) + recvOff[q], hr_.data() + o, recvBytes[q],
                                               hipMemcpyHostToDevice, s) != hipSuccess)
                return false;
            o += recvBytes[q];
        }
        return hipStreamSynchronize(s) == hipSuccess;
    }
    bool allreduce(void* dev, size_t count, size_t es, int op, hipStream_t s)
    {
        hs_.resize(count * es);
        if (hipMemcpyAsync(hs_.data(), dev, count * es, hipMemcpyDeviceToHost, s) != hipSuccess) return false;
        if (hipStreamSynchronize(s) != hipSuccess) return false;
        if (ar_(user_, hs_.data(), count, op) != 0) return false;
        if (hipMemcpyAsync(dev, hs_.data(), count * es, hipMemcpyHostToDevice, s) != hipSuccess) return false;
        return hipStreamSynchronize(s) == hipSuccess;
    }
    bool allreduceSumU32(uint32_t* dev, size_t count, hipStream_t s) override { return allreduce(dev, count, 4, 0, s); }
    bool allreduceMinF64(double* dev, size_t count, hipStream_t s) override { return allreduce(dev, count, 8, 1, s); }
    bool allreduceSumF64(double* dev, size_t count, hipStream_t s) override { return allreduce(dev, count, 8, 2, s); }
    bool allreduceMinU32(uint32_t* dev, size_t count, hipStream_t s) override { return allreduce(dev, count, 4, 3, s); }
    bool allreduceMaxU32(uint32_t* dev, size_t count, hipStream_t s) override { return allreduce(dev, count, 4, 4, s); }

private:
    int               rank_, size_;
    sx_alltoallv_cb   a2a_;
    sx_allreduce_cb   ar_;
    void*             user_;
    std::vector<char> hs_, hr_;
};

} // namespace sx

struct sx_comm
{
    sx::Transport* t{nullptr};
};

extern "C"
{
    sx::Transport* sx_comm_transport_internal(sx_comm* c) { return c ? c->t : nullptr; }

    int sx_comm_unique_id(void* out)
    {
        ncclUniqueId id;
        if (ncclGetUniqueId(&id) != ncclSuccess) return SX_ERR_HIP;
        std::memcpy(out, &id, sizeof(id));
        return SX_OK;
    }

    int sx_comm_create_rccl(sx_comm** out, int rank, int size, const void* id128)
    {
        ncclUniqueId id;
        std::memcpy(&id, id128, sizeof(id));
        auto* t = new sx::RcclTransport(rank, size, id);
        if (!t->ok())
        {
            delete t;
            return SX_ERR_HIP;
        }
        *out = new sx_comm{t};
        return SX_OK;
    }

    int sx_comm_create_host(sx_comm** out, int rank, int size, sx_alltoallv_cb a2a, sx_allreduce_cb ar, void* user)
    {
        *out = new sx_comm{new sx::HostTransport(rank, size, a2a, ar, user)};
        return SX_OK;
    }

    int sx_comm_alltoallv(sx_comm* c, const void* send, const uint64_t* sendBytes, const uint64_t* sendOff,
                          void* recv, const uint64_t* recvBytes, const uint64_t* recvOff, void* hipStream)
    {
        if (!c || !c->t) return SX_ERR_ARG;
        return c->t->alltoallv(send, sendBytes, sendOff, recv, recvBytes, recvOff, static_cast<hipStream_t>(hipStream)) ? SX_OK : SX_ERR_HIP;
    }

    int sx_comm_allreduce(sx_comm* c, void* dev, uint64_t count, int op, void* hipStream)
    {
        if (!c || !c->t) return SX_ERR_ARG;
        bool ok;
        switch (op)
        {
            case 0: ok = c->t->allreduceSumU32(static_cast<uint32_t*>(dev), count, static_cast<hipStream_t>(hipStream)); break;
            case 1: ok = c->t->allreduceMinF64(static_cast<double*>(dev), count, static_cast<hipStream_t>(hipStream)); break;
            case 2: ok = c->t->allreduceSumF64(static_cast<double*>(dev), count, static_cast<hipStream_t>(hipStream)); break;
            case 3: ok = c->t->allreduceMinU32(static_cast<uint32_t*>(dev), count, static_cast<hipStream_t>(hipStream)); break;
            case 4: ok = c->t->allreduceMaxU32(static_cast<uint32_t*>(dev), count, static_cast<hipStream_t>(hipStream)); break;
            default: return SX_ERR_ARG;
        }
        return ok ? SX_OK : SX_ERR_HIP;
    }

    void sx_comm_destroy(sx_comm* c)
    {
        if (!c) return;
        delete c->t;
        delete c;
    }
}
