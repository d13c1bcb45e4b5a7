// Radix-sort variants for the per-step local sort (sortLocals): 64M nearly sorted SFC keys, stable sort of the top
// 30 key bits with the input positions as values.  Times the variants with HIP events and checks they agree.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 scripts/sort_bench.hip -o scripts/sort_bench && scripts/sort_bench
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                                                                          \
    do {                                                                                                               \
        hipError_t e_ = (x);                                                                                           \
        if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); }      \
    } while (0)

__global__ void iota(uint32_t* v, size_t n)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}
__global__ void top32(const uint64_t* k, uint32_t* o, size_t n, int shift)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) o[i] = (uint32_t)(k[i] >> shift);
}

template<unsigned Bits, unsigned BS, unsigned IPT>
using OneCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                          rocprim::radix_sort_onesweep_config<rocprim::kernel_config<BS, IPT>,
                                                                              rocprim::kernel_config<BS, IPT>, Bits,
                                                                              rocprim::block_radix_rank_algorithm::match>>;

template<class F>
float timeIt(F&& f, int reps = 5)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv)
{
    const size_t n    = argc > 1 ? std::stoull(argv[1]) : (size_t)64000000;
    const int    bits = 30, begin = 63 - bits;
    std::vector<uint64_t> h(n);
    std::mt19937_64       rng(7);
    for (auto& v : h)
        v = rng() >> 1;
    std::sort(h.begin(), h.end());
    // ~10 % displaced: small local swaps plus a few far moves
    for (size_t i = 0; i + 1 < n; i += 20)
        std::swap(h[i], h[i + 1]);
    for (size_t i = 0; i < n; i += 1000)
        h[i] = rng() >> 1;
    uint64_t *k, *kOut;
    uint32_t *k32, *k32Out, *vIn, *order, *ref;
    CK(hipMalloc(&k, n * 8)); CK(hipMalloc(&kOut, n * 8));
    CK(hipMalloc(&k32, n * 4)); CK(hipMalloc(&k32Out, n * 4));
    CK(hipMalloc(&vIn, n * 4)); CK(hipMalloc(&order, n * 4)); CK(hipMalloc(&ref, n * 4));
    CK(hipMemcpy(k, h.data(), n * 8, hipMemcpyHostToDevice));
    const unsigned g = (unsigned)((n + 255) / 256);
    iota<<<g, 256>>>(vIn, n);
    top32<<<g, 256>>>(k, k32, n, begin);
    void*  tmp      = nullptr;
    size_t tmpBytes = 0, need = 0;
    auto   ensure   = [&](size_t b) {
        if (b > tmpBytes)
        {
            if (tmp) CK(hipFree(tmp));
            CK(hipMalloc(&tmp, b));
            tmpBytes = b;
        }
    };
    std::vector<uint32_t> hr(n), ho(n);
    auto check = [&](const char* name, float ms) {
        CK(hipMemcpy(ho.data(), order, n * 4, hipMemcpyDeviceToHost));
        const bool ok = ho == hr;
        printf("{\"variant\": \"%s\", \"ms\": %.3f, \"same_order\": %s}\n", name, ms, ok ? "true" : "false");
        fflush(stdout);
    };
    // baseline: hipcub u64 keys, bits [33, 63)
    CK(hipcub::DeviceRadixSort::SortPairs(nullptr, need, k, kOut, vIn, order, (int)n, begin, 63));
    ensure(need);
    float ms = timeIt([&] { CK(hipcub::DeviceRadixSort::SortPairs(tmp, need, k, kOut, vIn, order, (int)n, begin, 63)); });
    CK(hipMemcpy(hr.data(), order, n * 4, hipMemcpyDeviceToHost));
    printf("{\"variant\": \"hipcub u64 keys 30 bits (current)\", \"ms\": %.3f}\n", ms);
    // u32 keys, default config
    CK(hipMemset(order, 0, n * 4));
    need = 0;
    CK(hipcub::DeviceRadixSort::SortPairs(nullptr, need, k32, k32Out, vIn, order, (int)n, 0, bits));
    ensure(need);
    ms = timeIt([&] { CK(hipcub::DeviceRadixSort::SortPairs(tmp, need, k32, k32Out, vIn, order, (int)n, 0, bits)); });
    check("hipcub u32 keys 30 bits", ms);
    ms = timeIt([&] {
        top32<<<g, 256>>>(k, k32, n, begin);
        CK(hipcub::DeviceRadixSort::SortPairs(tmp, need, k32, k32Out, vIn, order, (int)n, 0, bits));
    });
    check("hipcub u32 keys 30 bits + key extraction", ms);
    auto variant = [&](auto cfgTag, const char* name) {
        using Cfg = decltype(cfgTag);
        CK(hipMemset(order, 0, n * 4));
        size_t nb = 0;
        CK(rocprim::radix_sort_pairs<Cfg>(nullptr, nb, k32, k32Out, vIn, order, n, 0, bits));
        ensure(nb);
        float t = timeIt([&] { CK(rocprim::radix_sort_pairs<Cfg>(tmp, nb, k32, k32Out, vIn, order, n, 0, bits)); });
        check(name, t);
    };
    variant(OneCfg<8, 512, 12>{}, "rocprim u32 8 bits 512x12");
    variant(OneCfg<10, 512, 12>{}, "rocprim u32 10 bits 512x12");
    variant(OneCfg<10, 1024, 12>{}, "rocprim u32 10 bits 1024x12");
    variant(OneCfg<10, 512, 16>{}, "rocprim u32 10 bits 512x16");
    variant(OneCfg<11, 1024, 12>{}, "rocprim u32 11 bits 1024x12");
    variant(OneCfg<10, 1024, 16>{}, "rocprim u32 10 bits 1024x16");
    variant(OneCfg<8, 1024, 16>{}, "rocprim u32 8 bits 1024x16");
    return 0;
}
