/*! @file fetch_calib.hip
 * @brief Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access shapes of this library's
 *        kernels (MI355X_MICROARCH.md, HBM: "FETCH_SIZE reports exactly 1/2 of the bytes of a wide coalesced
 *        streaming read ... other access widths are uncalibrated: calibrate on a known byte count").
 *
 * Every kernel touches a known number of UNIQUE bytes, each byte once, in buffers of 1 GiB (4x the 256 MiB
 * Infinity Cache, so the memory-side counters see HBM traffic):
 *   rd16      dwordx4 streaming read, 16 B per lane, coalesced                      (own packed records)
 *   rd4       dword streaming read, 4 B per lane, coalesced 256-B rows              (u16-pair list words, union ids)
 *   rd8       dwordx2 streaming read, 8 B per lane                                  (f64 coordinates, search stream)
 *   gat32run  32-B records gathered through an index list of leaf-order runs       (union record staging, RecX)
 *   gat16rnd  16-B records gathered in a random permutation                         (RecV/RecT/RecC staging)
 *   gat4rnd   4-B words gathered in a random permutation                           (gather kernels, sort reorder)
 *   wr16      dwordx4 streaming store                                               (record packing)
 *   wr4       dword streaming store, coalesced                                      (outputs, list rewrite)
 *   wr4lane   dword stores of lane-interleaved rows written at per-lane positions   (search list append)
 *   wr2       2-B stores, coalesced                                                 (u16 tables)
 * The index reads of the gathers are part of the known bytes (4 B per record).
 *
 *   hipcc --offload-arch=gfx950 -O3 scripts/fetch_calib.hip -o scripts/fetch_calib
 *   rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d out/f -o f -- scripts/fetch_calib
 *   rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d out/w -o w -- scripts/fetch_calib
 *   python scripts/fetch_calib.py out   (factor = known bytes / counter bytes, per shape)
 * The program prints the known bytes per kernel as JSON (one line) for fetch_calib.py.
 */
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                                                         \
    do                                                                                                                \
    {                                                                                                                 \
        hipError_t e_ = (x);                                                                                          \
        if (e_ != hipSuccess)                                                                                         \
        {                                                                                                             \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                                 \
            exit(1);                                                                                                  \
        }                                                                                                             \
    } while (0)

constexpr size_t kBytes = size_t(1) << 30;

__global__ void rd16(const float4* __restrict__ a, size_t n, float* out)
{
    float s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1.2345f) out[0] = s;
}
__global__ void rd4(const uint32_t* __restrict__ a, size_t n, uint32_t* out)
{
    uint32_t s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s ^= a[i];
    if (s == 0x12345u) out[0] = s;
}
__global__ void rd8(const double* __restrict__ a, size_t n, double* out)
{
    double s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += a[i];
    if (s == 1.2345) out[0] = s;
}
struct Rec32
{
    float4 a, b;
};
__global__ void gat32(const Rec32* __restrict__ r, const uint32_t* __restrict__ idx, size_t n, float* out)
{
    float s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    {
        const Rec32 v = r[idx[i]];
        s += v.a.x + v.a.y + v.b.z + v.b.w;
    }
    if (s == 1.2345f) out[0] = s;
}
__global__ void gat16(const float4* __restrict__ r, const uint32_t* __restrict__ idx, size_t n, float* out)
{
    float s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    {
        const float4 v = r[idx[i]];
        s += v.x + v.w;
    }
    if (s == 1.2345f) out[0] = s;
}
__global__ void gat4(const uint32_t* __restrict__ r, const uint32_t* __restrict__ idx, size_t n, uint32_t* out)
{
    uint32_t s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s ^= r[idx[i]];
    if (s == 0x12345u) out[0] = s;
}
__global__ void wr16(float4* a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_float4(i, 1, 2, 3);
}
__global__ void wr4(uint32_t* a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = (uint32_t)i;
}
__global__ void wr2(uint16_t* a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = (uint16_t)i;
}
//! the search's append shape: wave w owns rows [w*R, (w+1)*R) of 64 dwords (256 B); lane l writes its column
//! word by word, each lane stepping at its own pace (lane l writes one word every 1 + (l & 3) iterations), so a
//! store instruction touches several rows and a row is completed by many instructions
__global__ void wr4lane(uint32_t* a, size_t rows, int R)
{
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const int    lane = threadIdx.x & 63;
    if ((wave + 1) * R > rows) return;
    uint32_t* col  = a + wave * R * 64 + lane;
    int       k    = 0;
    const int step = 1 + (lane & 3);
    for (int it = 0; k < R; ++it)
        if (it % step == 0) col[(size_t)(k++) * 64] = (uint32_t)it;
}

int main()
{
    std::vector<std::pair<const char*, double>> known;
    void *a, *b, *idx;
    CK(hipMalloc(&a, kBytes));
    CK(hipMalloc(&b, kBytes));
    CK(hipMalloc(&idx, kBytes / 2));
    CK(hipMemset(a, 0, kBytes));
    float* out;
    CK(hipMalloc(&out, 64));
    const int grid = 256 * 16, block = 256;

    // index lists: 32-B records in runs of 12 consecutive records starting at random leaf offsets (every record of
    // the first half of the buffer exactly once), and a random permutation for the 16-B / 4-B gathers
    const size_t n32 = kBytes / 2 / sizeof(Rec32); // 16M records: 512 MiB
    std::vector<uint32_t> h(n32);
    {
        const size_t nrun = (n32 + 11) / 12;
        std::vector<uint32_t> runs(nrun);
        std::iota(runs.begin(), runs.end(), 0u);
        std::shuffle(runs.begin(), runs.end(), std::mt19937(7));
        size_t k = 0;
        for (size_t r : runs)
            for (size_t q = r * 12; q < std::min(n32, r * 12 + 12); ++q)
                h[k++] = (uint32_t)q;
    }
    CK(hipMemcpy(idx, h.data(), n32 * 4, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 2; ++rep) // the second repetition is the one to read (first touch aside)
    {
        rd16<<<grid, block>>>((const float4*)a, kBytes / 16, out);
        rd4<<<grid, block>>>((const uint32_t*)a, kBytes / 4, (uint32_t*)out);
        rd8<<<grid, block>>>((const double*)a, kBytes / 8, (double*)out);
        gat32<<<grid, block>>>((const Rec32*)a, (const uint32_t*)idx, n32, out);
    }
    known.push_back({"rd16", (double)kBytes});
    known.push_back({"rd4", (double)kBytes});
    known.push_back({"rd8", (double)kBytes});
    known.push_back({"gat32", (double)n32 * (32 + 4)});

    const size_t n16 = kBytes / 2 / 16; // 32M records of the first 512 MiB
    h.resize(n16);
    std::iota(h.begin(), h.end(), 0u);
    std::shuffle(h.begin(), h.end(), std::mt19937(9));
    CK(hipMemcpy(idx, h.data(), n16 * 4, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 2; ++rep)
        gat16<<<grid, block>>>((const float4*)a, (const uint32_t*)idx, n16, out);
    known.push_back({"gat16", (double)n16 * (16 + 4)});

    const size_t n4 = kBytes / 2 / 4 / 4; // 32M words of the first 128 MiB... spread: word q*4 (stride 16 B)
    h.resize(n4);
    std::iota(h.begin(), h.end(), 0u);
    std::shuffle(h.begin(), h.end(), std::mt19937(11));
    for (auto& v : h)
        v *= 4;
    CK(hipMemcpy(idx, h.data(), n4 * 4, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 2; ++rep)
        gat4<<<grid, block>>>((const uint32_t*)a, (const uint32_t*)idx, n4, (uint32_t*)out);
    known.push_back({"gat4", (double)n4 * (4 + 4)}); // 4 useful B per 16-B stride: the sector granularity shows

    for (int rep = 0; rep < 2; ++rep)
    {
        wr16<<<grid, block>>>((float4*)b, kBytes / 16);
        wr4<<<grid, block>>>((uint32_t*)b, kBytes / 4);
        wr2<<<grid, block>>>((uint16_t*)b, kBytes / 2);
    }
    known.push_back({"wr16", (double)kBytes});
    known.push_back({"wr4", (double)kBytes});
    known.push_back({"wr2", (double)kBytes});
    const int    R    = 64;
    const size_t rows = kBytes / 256;
    for (int rep = 0; rep < 2; ++rep)
        wr4lane<<<(unsigned)(rows / R * 64 / 256), 256>>>((uint32_t*)b, rows, R);
    known.push_back({"wr4lane", (double)kBytes});
    CK(hipDeviceSynchronize());
    printf("{");
    for (size_t k = 0; k < known.size(); ++k)
        printf("%s\"%s\": %.0f", k ? ", " : "", known[k].first, known[k].second);
    printf("}\n");
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(idx));
    CK(hipFree(out));
    return 0;
}
