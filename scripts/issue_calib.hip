// VALU issue calibration on gfx950: FP32 FMA throughput vs waves per SIMD, scalar v_fma_f32 and packed
// v_pk_fma_f32, with 8 independent chains per lane (ILP) or 1 dependent chain.  Occupancy is pinned by dynamic LDS
// (a workgroup of 256 threads = one wave per SIMD; LDS per workgroup = 160 KiB / W gives W workgroups per CU).
//   hipcc --offload-arch=gfx950 -O3 scripts/issue_calib.hip -o scripts/issue_calib && scripts/issue_calib
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float v2f __attribute__((ext_vector_type(2)));

template<int CHAINS, bool PACKED>
__global__ __launch_bounds__(256) void fmaKernel(float* out, int iters, float a, float b)
{
    extern __shared__ float lds[];
    if (PACKED)
    {
        v2f x[CHAINS];
        for (int c = 0; c < CHAINS; ++c)
            x[c] = v2f{(float)threadIdx.x + c, (float)c};
        const v2f A = {a, a}, B = {b, b};
        for (int i = 0; i < iters; ++i)
#pragma unroll
            for (int c = 0; c < CHAINS; ++c)
                x[c] = __builtin_elementwise_fma(x[c], A, B);
        float s = 0;
        for (int c = 0; c < CHAINS; ++c)
            s += x[c].x + x[c].y;
        if (s == 1.2345f) lds[threadIdx.x] = s, out[blockIdx.x] = lds[threadIdx.x ^ 1];
    }
    else
    {
        float x[CHAINS];
        for (int c = 0; c < CHAINS; ++c)
            x[c] = (float)threadIdx.x + c;
        for (int i = 0; i < iters; ++i)
#pragma unroll
            for (int c = 0; c < CHAINS; ++c)
                x[c] = __builtin_fmaf(x[c], a, b);
        float s = 0;
        for (int c = 0; c < CHAINS; ++c)
            s += x[c];
        if (s == 1.2345f) lds[threadIdx.x] = s, out[blockIdx.x] = lds[threadIdx.x ^ 1];
    }
}

template<int CHAINS, bool PACKED>
void run(int wavesPerSimd, float* out)
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const size_t lds   = (160 * 1024) / wavesPerSimd - 1024;
    const int    grid  = cus * wavesPerSimd * 4; // four rounds of full occupancy
    const int    iters = 4096;
    hipFuncSetAttribute((const void*)fmaKernel<CHAINS, PACKED>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1;
    hipEventCreate(&e0), hipEventCreate(&e1);
    fmaKernel<CHAINS, PACKED><<<grid, 256, lds>>>(out, 16, 1.0001f, 0.5f);
    hipEventRecord(e0);
    fmaKernel<CHAINS, PACKED><<<grid, 256, lds>>>(out, iters, 1.0001f, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double instrs = (double)grid * 4 /*waves*/ * iters * CHAINS;     // wave64 FMA instructions
    const double flops  = instrs * 64 * 2 * (PACKED ? 2 : 1);
    // per SIMD: instructions / (cycles at 2.4 GHz)
    const double perSimdCycles = ms * 1e-3 * 2.4e9;
    const double instrPerSimd  = instrs / (cus * 4.0);
    printf("{\"chains\": %d, \"packed\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"tflops\": %.1f, "
           "\"cycles_per_wave64_instr_per_simd\": %.2f}\n",
           CHAINS, PACKED ? 1 : 0, wavesPerSimd, ms, flops / (ms * 1e-3) / 1e12, perSimdCycles / instrPerSimd);
}

int main()
{
    float* out;
    hipMalloc(&out, 1 << 20);
    for (int w : {1, 2, 3, 4, 8})
    {
        run<8, false>(w, out);
        run<1, false>(w, out);
        run<8, true>(w, out);
    }
    hipFree(out);
    return 0;
}
