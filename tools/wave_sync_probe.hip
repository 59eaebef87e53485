/*
 * wave_sync_probe.hip — what a multi-wave config-4 workgroup would pay to hand data between its waves (VERDICT r5
 * "Next round" #3: a measured A/B of splitting a document's event across waves). One workgroup per CU as
 * k_replay_tiled runs (256 workgroups), W waves each; per workgroup, in cycles (s_memtime):
 *   barrier:   an s_barrier round (__syncthreads) with every wave arriving together;
 *   handoff:   wave 0 writes 64 dwords to LDS, barrier, wave 1 reads them and writes 64 back, barrier, wave 0 reads
 *              them — the exchange a split phase needs (its partial results one way, the merged ones back);
 *   flag:      the same exchange through an LDS flag the other wave polls (s_sleep 1 between polls), no barrier;
 *   ldsread:   one dependent LDS read round trip (a wave reading what it wrote), for scale;
 *   hbmread:   one dependent global read round trip (a pointer chase over 64 MB, mostly HBM misses), for scale.
 * Every loop has a fixed trip count and every wave runs the same number of barriers, so the grid always drains.
 * Built here: hipcc --offload-arch=gfx950 -O3 -o tools/bin/wave_sync_probe tools/wave_sync_probe.hip; run on the GPU.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define ITERS 256

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memtime(); }

/* out[blockIdx.x * 8 + k]: total cycles of test k over ITERS rounds, measured by wave 0 */
__global__ __launch_bounds__(256) void k_probe(uint64_t* out, const uint32_t* chase, uint32_t mask, int waves) {
    __shared__ int32_t buf[2][64];
    __shared__ volatile int32_t flag[2];
    const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
    if (wv >= waves) return; /* a block of `waves` waves: blockDim.x = 64 * waves */
    uint64_t t0, acc = 0;
    int32_t sink = 0;
    /* barrier */
    __syncthreads();
    t0 = now();
    for (int i = 0; i < ITERS; i++) __syncthreads();
    if (wv == 0 && lane == 0) out[blockIdx.x * 8 + 0] = now() - t0;
    /* handoff through barriers */
    __syncthreads();
    t0 = now();
    for (int i = 0; i < ITERS; i++) {
        if (wv == 0) buf[0][lane] = i + lane;
        __syncthreads();
        if (wv == 1) buf[1][lane] = buf[0][lane] + 1;
        __syncthreads();
        if (wv == 0) sink += buf[1][lane];
    }
    if (wv == 0 && lane == 0) out[blockIdx.x * 8 + 1] = now() - t0;
    /* handoff through a polled LDS flag (waves >= 2): wave 0 publishes round i, wave 1 answers it */
    if (threadIdx.x == 0) flag[0] = flag[1] = -1;
    __syncthreads();
    t0 = now();
    if (waves >= 2) {
        for (int i = 0; i < ITERS; i++) {
            if (wv == 0) {
                buf[0][lane] = i + lane;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) flag[0] = i;
                int spins = 0;
                while (flag[1] != i && ++spins < 100000) __builtin_amdgcn_s_sleep(1);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                sink += buf[1][lane];
            } else if (wv == 1) {
                int spins = 0;
                while (flag[0] != i && ++spins < 100000) __builtin_amdgcn_s_sleep(1);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                buf[1][lane] = buf[0][lane] + 1;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) flag[1] = i;
            }
        }
    }
    if (wv == 0 && lane == 0) out[blockIdx.x * 8 + 2] = now() - t0;
    __syncthreads();
    /* one dependent LDS round trip */
    if (wv == 0) {
        int32_t x = lane;
        buf[0][lane] = lane;
        t0 = now();
        for (int i = 0; i < ITERS; i++) {
            buf[0][lane] = x + 1;
            x = buf[0][(x + 1) & 63];
        }
        acc = now() - t0;
        sink += x;
        if (lane == 0) out[blockIdx.x * 8 + 3] = acc;
    }
    /* one dependent global round trip (pointer chase, one lane's chain broadcast by the wave) */
    if (wv == 0) {
        uint32_t p = (blockIdx.x * 7919u + (uint32_t)lane * 64u) & mask; /* a chain per lane: vector loads */
        t0 = now();
        for (int i = 0; i < ITERS; i++) p = (chase[p] + (uint32_t)lane * 64u) & mask;
        acc = now() - t0;
        sink += (int32_t)p;
        if (lane == 0) out[blockIdx.x * 8 + 4] = acc;
    }
    if (sink == 0x7fffffff && lane == 0) out[blockIdx.x * 8 + 7] = 1; /* keeps the loads */
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 256;
    const uint32_t n = 1u << 24, mask = n - 1; /* 64 MB chase table */
    uint32_t* h = (uint32_t*)malloc(sizeof(uint32_t) * n);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (uint32_t i = 0; i < n; i++) {
        s ^= s << 13, s ^= s >> 7, s ^= s << 17;
        h[i] = (uint32_t)(s >> 20) & mask & ~63u; /* 256-byte strides: one miss per step */
    }
    uint32_t* d;
    uint64_t* dout;
    if (hipMalloc(&d, sizeof(uint32_t) * n) != hipSuccess || hipMalloc(&dout, 8 * 8 * blocks) != hipSuccess) return 2;
    hipMemcpy(d, h, sizeof(uint32_t) * n, hipMemcpyHostToDevice);
    uint64_t* ho = (uint64_t*)malloc(8 * 8 * blocks);
    printf("{\"blocks\": %d, \"iters\": %d, \"cycles_per_round\": {", blocks, ITERS);
    for (int waves = 1; waves <= 4; waves *= 2) {
        hipMemset(dout, 0, 8 * 8 * blocks);
        hipLaunchKernelGGL(k_probe, dim3(blocks), dim3(64 * waves), 0, 0, dout, d, mask, waves);
        if (hipDeviceSynchronize() != hipSuccess) return 3;
        hipMemcpy(ho, dout, 8 * 8 * blocks, hipMemcpyDeviceToHost);
        const char* names[5] = {"barrier", "handoff_barrier", "handoff_flag", "lds_read", "global_read"};
        printf("%s\"waves_%d\": {", waves > 1 ? ", " : "", waves);
        for (int k = 0; k < 5; k++) {
            double m = 0;
            for (int b = 0; b < blocks; b++) m += (double)ho[b * 8 + k];
            m /= (double)blocks * ITERS;
            printf("%s\"%s\": %.1f", k ? ", " : "", names[k], (waves < 2 && (k == 1 || k == 2)) ? -1.0 : m);
        }
        printf("}");
    }
    printf("}, \"clock\": \"s_memtime (shader clock)\"}\n");
    return 0;
}
