// ubench_valu.hip -- VALU rate microbenchmark for the roofline record (bench.py "roofline").
//
// MI355X_MICROARCH.md quotes the FP32 vector peak (157.3 TF/s) but no FP64 figure, so the FP64 peak the
// roofline uses is measured here: many independent fused-multiply-add chains per lane, full occupancy
// (8 waves per SIMD), timed with HIP events. The one-wave-per-SIMD rows give the issue cost the solve kernel
// sees (it runs one wave per SIMD at the headline batch): cycles per instruction from s_memtime.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o build/ubench_valu
// run:   build/ubench_valu  -> one JSON line
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                                   \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                         \
            std::exit(1);                                                                        \
        }                                                                                        \
    } while (0)

constexpr int kChains = 8;

__device__ __forceinline__ float fma_t(float x, float a, float b) { return __builtin_fmaf(x, a, b); }
__device__ __forceinline__ double fma_t(double x, double a, double b) { return __builtin_fma(x, a, b); }

template <class T>
__global__ __launch_bounds__(256) void k_fma(T* out, int iters, T a, T b, unsigned long long* cyc)
{
    T c[kChains];
#pragma unroll
    for (int j = 0; j < kChains; j++) c[j] = (T)(threadIdx.x + j);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int j = 0; j < kChains; j++) c[j] = fma_t(c[j], a, b);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    T s = 0;
#pragma unroll
    for (int j = 0; j < kChains; j++) s += c[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && cyc) cyc[blockIdx.x] = t1 - t0;
}

template <class T>
static void run(const char* name, int blocks, int iters, bool last)
{
    T* out;
    unsigned long long* cyc;
    CHK(hipMalloc(&out, sizeof(T) * blocks * 256));
    CHK(hipMalloc(&cyc, sizeof(unsigned long long) * blocks));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const T a = (T)0.999999, b = (T)1e-7;
    hipLaunchKernelGGL(k_fma<T>, dim3(blocks), dim3(256), 0, nullptr, out, iters / 8, a, b, cyc);  // warm
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_fma<T>, dim3(blocks), dim3(256), 0, nullptr, out, iters, a, b, cyc);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0.0f;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long* h = (unsigned long long*)std::malloc(sizeof(unsigned long long) * blocks);
    CHK(hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost));
    double cmean = 0.0;
    for (int i = 0; i < blocks; i++) cmean += (double)h[i];
    cmean /= blocks;
    const double fmas = (double)blocks * 256 * iters * 16 * kChains;
    const double tflops = 2.0 * fmas / (ms * 1e-3) / 1e12;
    // per-wave instruction count: iters * 16 * kChains FMAs; cycles from s_memtime (shader clock ticks)
    const double cyc_per_inst = cmean / ((double)iters * 16 * kChains);
    std::printf("\"%s\": {\"blocks\": %d, \"ms\": %.4f, \"tflops\": %.2f, \"cycles_per_fma_per_wave\": %.3f}%s", name,
                blocks, ms, tflops, cyc_per_inst, last ? "" : ", ");
    std::free(h);
    CHK(hipFree(out));
    CHK(hipFree(cyc));
}

int main()
{
    int dev = 0;
    hipDeviceProp_t p;
    CHK(hipGetDevice(&dev));
    CHK(hipGetDeviceProperties(&p, dev));
    const int cus = p.multiProcessorCount;
    std::printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d, ", p.name, cus, p.clockRate);
    // full occupancy: 8 blocks of 4 waves per CU = 8 waves per SIMD
    run<float>("fp32_full", cus * 8, 4096, false);
    run<double>("fp64_full", cus * 8, 2048, false);
    // one 256-thread block per CU = one wave per SIMD (the solve kernel's occupancy at the headline batch)
    run<float>("fp32_one_wave_per_simd", cus, 4096, false);
    run<double>("fp64_one_wave_per_simd", cus, 2048, false);
    // two waves per SIMD
    run<float>("fp32_two_waves_per_simd", cus * 2, 4096, false);
    run<double>("fp64_two_waves_per_simd", cus * 2, 2048, true);
    std::printf("}\n");
    return 0;
}
