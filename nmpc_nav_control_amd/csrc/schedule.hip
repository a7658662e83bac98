// schedule.hip -- difficulty-ordered team placement for launches with more waves than SIMDs.
//
// The team kernel's time is the busiest SIMD's: a wave iterates until its slowest team converges, and when
// a SIMD holds two or more waves they share its issue slots. A robot's IPM iteration count persists from
// tick to tick (DESIGN.md "Scheduling"), so the previous tick's count (iter_key, written by the kernel)
// predicts the next one. k_team_order sorts the robots by that key (stable counting sort, hardest first)
// and lays the sorted list out over the team slots:
//   sorted      slot s <- rank s: waves hold robots of like difficulty, the hard half of the blocks is
//               dispatched first;
//   interleaved even blocks take ranks from the hard end, odd blocks from the easy end, so neighbouring
//               blocks (which share CUs) pair a hard block with an easy one;
//   spread      the first wave of every block (one block = one CU at one wave per SIMD) takes the 4 x blocks
//               hardest robots, the other three waves the rest in order: the kernel ends with the slowest
//               wave, and a hard wave whose CU-mates finish early runs its last iterations alone on the CU
//               (memory pipeline and L1 no longer shared).
// Every robot keeps its own arithmetic whatever slot it lands in, so the order changes no result.
#include "nmpc_kernels.hpp"

namespace nmpc {

namespace {

constexpr int kOrderThreads = 1024;
constexpr int kOrderBins = 32;  // keys clamp to [0, 31] (IPM iterations; iter_max reaches 50 only on failures)

__global__ __launch_bounds__(kOrderThreads) void k_team_order(const int* __restrict__ key, int B, int layout,
                                                               int* __restrict__ sorted, int* __restrict__ order,
                                                               int H = 0, int cap = 0, int* __restrict__ nhard = nullptr)
{
    // cnt[bin][thread]: private column per thread, then one exclusive scan in (bin descending, thread) order
    __shared__ unsigned cnt[kOrderBins][kOrderThreads];
    __shared__ unsigned part[kOrderThreads];
    __shared__ unsigned hcnt;
    const int t = threadIdx.x;
    if (t == 0) hcnt = 0;
    const int E = (B + kOrderThreads - 1) / kOrderThreads;
    const int i0 = min(B, t * E), i1 = min(B, i0 + E);
    for (int b = 0; b < kOrderBins; b++) cnt[b][t] = 0;
    for (int i = i0; i < i1; i++) {
        const int k = min(max(key[i], 0), kOrderBins - 1);
        cnt[kOrderBins - 1 - k][t]++;
    }
    __syncthreads();
    // flattened index f = bin * T + thread; thread t scans f in [32 t, 32 t + 32)
    unsigned loc[kOrderBins];
    unsigned s = 0;
#pragma unroll
    for (int j = 0; j < kOrderBins; j++) {
        const int f = t * kOrderBins + j;
        loc[j] = s;
        s += cnt[f / kOrderThreads][f % kOrderThreads];
    }
    part[t] = s;
    __syncthreads();
    // Hillis-Steele inclusive scan of the partial sums
    for (int d = 1; d < kOrderThreads; d <<= 1) {
        const unsigned v = (t >= d) ? part[t - d] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    const unsigned base = part[t] - s;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kOrderBins; j++) {
        const int f = t * kOrderBins + j;
        cnt[f / kOrderThreads][f % kOrderThreads] = base + loc[j];
    }
    __syncthreads();
    int* dst = (layout == NMPC_SCHED_SORTED) ? order : sorted;
    unsigned nh = 0;
    for (int i = i0; i < i1; i++) {
        const int k = min(max(key[i], 0), kOrderBins - 1);
        dst[cnt[kOrderBins - 1 - k][t]++] = i;
        nh += (nhard && key[i] >= H) ? 1u : 0u;
    }
    if (nhard) {  // the hybrid split: how many of the hardest ranks go to the segmented kernel
        if (nh) atomicAdd(&hcnt, nh);
        __syncthreads();
        if (t == 0) nhard[0] = min((int)hcnt, cap);
    }
    if (layout == NMPC_SCHED_SORTED) return;
    __threadfence_block();
    __syncthreads();
    if (layout == NMPC_SCHED_SPREAD) {
        // wave-0 slots (s % 16 < 4) of block j take ranks 4 j .. 4 j + 3; every other slot follows in slot
        // order after the n0 wave-0 slots (only the last block can be partial)
        const int nb = (B + 15) >> 4;
        const int n0 = 4 * (nb - 1) + min(4, B - 16 * (nb - 1));
        for (int sl = t; sl < B; sl += kOrderThreads) {
            const int j = sl >> 4, w = sl & 15;
            order[sl] = sorted[(w < 4) ? 4 * j + w : n0 + sl - 4 * (j + 1)];
        }
        return;
    }
    // interleaved: slot s in block j = s / 16 (16 teams per block); even blocks count up from the hardest
    // rank, odd blocks down from the easiest (only the last block can be partial, so both runs are dense)
    for (int sl = t; sl < B; sl += kOrderThreads) {
        const int j = sl >> 4, w = sl & 15;
        const int q = (j >> 1) * 16 + w;
        order[sl] = sorted[(j & 1) ? B - 1 - q : q];
    }
}

}  // namespace

hipError_t launch_team_order(const int* key, int B, int layout, int* sorted, int* order, hipStream_t stream)
{
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_team_order, dim3(1), dim3(kOrderThreads), 0, stream, key, B, layout, sorted, order, 0, 0,
                       nullptr);
    return hipGetLastError();
}

#ifdef NMPC_HYBRID
hipError_t launch_hybrid_order(const int* key, int B, int H, int cap, int* order, int* nhard, hipStream_t stream)
{
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_team_order, dim3(1), dim3(kOrderThreads), 0, stream, key, B, (int)NMPC_SCHED_SORTED, order,
                       order, H, cap, nhard);
    return hipGetLastError();
}
#endif

}  // namespace nmpc
