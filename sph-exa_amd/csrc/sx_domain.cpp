/*! @file sx_domain.cpp
 * @brief Host-side decisions of the multi-GPU SFC domain decomposition (sx_sim.cpp distributedSync), exported
 *        through the C ABI so the same code drives the GPU path and the CPU (gloo) decomposition tests.
 *
 *   sx_domain_splitters   global key histogram -> P+1 SFC splitter keys with equal particle counts per rank;
 *                         replaces cstone::makeSfcAssignment (domain/include/cstone/domain/domaindecomp.hpp:120),
 *                         which equalises counts over the global cornerstone tree's leaves (here: 2^bits bins of
 *                         the key space, all ranks computing identical splitters from the all-reduced histogram)
 *   sx_domain_halo_layout received halo counts per peer -> receive offsets [lower ranks | locals | higher ranks],
 *                         the reference's layout of halos around the assigned range (domain.hpp:196-244,
 *                         halos.hpp:138-227): key-sorted by construction, so one tree covers locals + halos
 */
#include <cstdint>

#include "../../include/sphexa_hip.h"

extern "C"
{
    int sx_domain_splitters(const uint32_t* hist, uint32_t histBits, int nranks, uint64_t* split)
    {
        if (!hist || !split || nranks < 1 || histBits == 0 || histBits > 30) return SX_ERR_ARG;
        const uint64_t nb    = uint64_t(1) << histBits;
        uint64_t       total = 0;
        for (uint64_t b = 0; b < nb; ++b)
            total += hist[b];
        split[0]      = 0;
        split[nranks] = uint64_t(1) << 63; // one past the last 63-bit Hilbert key
        uint64_t acc  = 0;
        int      q    = 1;
        for (uint64_t b = 0; b < nb && q < nranks; ++b)
        {
            // rank q starts at the first bin boundary where the running count reaches q/P of the total
            while (q < nranks && acc >= (total * (uint64_t)q) / (uint64_t)nranks)
                split[q++] = b << (63 - histBits);
            acc += hist[b];
        }
        while (q < nranks)
            split[q++] = uint64_t(1) << 63;
        return SX_OK;
    }

    int sx_domain_halo_layout(const uint64_t* recvCounts, int nranks, int rank, uint64_t numLocal,
                              uint64_t* recvOff, uint64_t out[3])
    {
        if (!recvCounts || !recvOff || !out || rank < 0 || rank >= nranks) return SX_ERR_ARG;
        uint64_t nLow = 0, nHigh = 0;
        for (int q = 0; q < nranks; ++q)
        {
            if (q < rank) nLow += recvCounts[q];
            else if (q > rank) nHigh += recvCounts[q];
        }
        uint64_t lo = 0, hi = nLow + numLocal;
        for (int q = 0; q < nranks; ++q)
        {
            recvOff[q] = 0;
            if (q < rank) { recvOff[q] = lo, lo += recvCounts[q]; }
            else if (q > rank) { recvOff[q] = hi, hi += recvCounts[q]; }
        }
        out[0] = nLow;                    // first local
        out[1] = nLow + numLocal;         // last local
        out[2] = nLow + numLocal + nHigh; // locals + halos
        return SX_OK;
    }
}
