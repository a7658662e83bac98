// ubench_mall.hip -- calibration of the L2 memory-side request counters for bench.py's roofline.hbm block.
//
// The solve kernel's records stream between the XCDs' L2 and the memory side. MI355X_MICROARCH.md ("HBM") says
// FETCH_SIZE / WRITE_SIZE come from the L2's fabric request counters and appear to include Infinity-Cache (MALL)
// hits. gfx950 also exposes TCC_EA0_RDREQ_DRAM / TCC_EA0_WRREQ_DRAM ("requests destined for DRAM"). This program
// streams a read-only table of `mb` MiB with 16-B loads `reps` times per launch; run it under
// `rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum ...` once with a table that stays resident in the
// 256 MiB Infinity Cache (64 MiB: every rep after the first is an L3 hit, the 4 MiB L2s cannot hold it) and once
// with one that cannot (2 GiB). If the DRAM-destined count per byte is the same in both, the counter does not
// separate MALL hits from HBM reads and the bench reports L2-miss traffic only (an upper bound on HBM bytes).
//
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench_mall.hip -o build/ubench_mall
// run:   build/ubench_mall <MiB> <reps> [launches]  -> one JSON line (bytes read per launch, GB/s)
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

// grid-stride 16-B loads over n4 float4 entries, reps passes; one float per thread out (keeps the loads live)
__global__ __launch_bounds__(256) void k_stream(const float4* __restrict__ a, size_t n4, int reps, float* out)
{
    float s = 0.0f;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (int r = 0; r < reps; r++)
        for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
            const float4 v = a[i];
            s += v.x + v.y + v.z + v.w;
        }
    out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fill(float4* a, size_t n4)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
        a[i] = make_float4(1.0f, 2.0f, 3.0f, (float)(i & 1023));
}

int main(int argc, char** argv)
{
    const size_t mb = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 64;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 8;
    const int launches = argc > 3 ? std::atoi(argv[3]) : 3;
    if (mb < 1 || mb > 8192 || reps < 1 || reps > 64 || launches < 1 || launches > 16) {
        std::fprintf(stderr, "usage: ubench_mall <MiB 1..8192> <reps 1..64> [launches 1..16]\n");
        return 2;
    }
    const size_t n4 = mb * 1024 * 1024 / sizeof(float4);
    const int grid = 256 * 8, block = 256;  // 8 blocks per CU
    float4* a;
    float* out;
    CHK(hipMalloc(&a, n4 * sizeof(float4)));
    CHK(hipMalloc(&out, sizeof(float) * grid * block));
    hipLaunchKernelGGL(k_fill, dim3(grid), dim3(block), 0, nullptr, a, n4);
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    float ms_sum = 0.0f;
    for (int l = 0; l < launches; l++) {
        CHK(hipEventRecord(e0, nullptr));
        hipLaunchKernelGGL(k_stream, dim3(grid), dim3(block), 0, nullptr, a, n4, reps, out);
        CHK(hipEventRecord(e1, nullptr));
        CHK(hipEventSynchronize(e1));
        float ms = 0.0f;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        ms_sum += ms;
    }
    const double bytes = (double)n4 * sizeof(float4) * reps;
    const double ms = ms_sum / launches;
    std::printf("{\"table_mib\": %zu, \"reps\": %d, \"launches\": %d, \"bytes_read_per_launch\": %.0f, "
                "\"ms_per_launch\": %.4f, \"GBs\": %.1f}\n",
                mb, reps, launches, bytes, ms, bytes / (ms * 1e-3) / 1e9);
    CHK(hipFree(a));
    CHK(hipFree(out));
    return 0;
}
