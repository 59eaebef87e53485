/*
 * mt_wave.h — wavefront primitives used by mt_core.h.
 *   WaveHost: one lane; the serial host build (generator model, CPU spec tests).
 *   WaveGPU : one 64-lane CDNA wavefront; DPP/permute shuffles via __shfl_*, 64-bit ballots.
 */
#pragma once
#include <stdint.h>

namespace mt {

struct WaveHost {
    static constexpr int N = 1;
    int lane() const { return 0; }
    int32_t excl_scan(int32_t v, int32_t* tot) const {
        *tot = v;
        return 0;
    }
    int32_t sum(int32_t v) const { return v; }
    uint64_t ballot(bool p) const { return p ? 1ull : 0ull; }
    int32_t bcast(int32_t v, int) const { return v; }
    static int ffs(uint64_t m) { return __builtin_ctzll(m); }
    void sync() const {}
};

#ifdef __HIPCC__
struct WaveGPU {
    static constexpr int N = 64;
    __device__ int lane() const { return (int)(threadIdx.x & 63); }
    /* exclusive prefix sum across the wave (Hillis-Steele over __shfl_up) */
    __device__ int32_t excl_scan(int32_t v, int32_t* tot) const {
        int32_t x = v;
        int l = lane();
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            int32_t y = __shfl_up(x, o, 64);
            if (l >= o) x += y;
        }
        *tot = __shfl(x, 63, 64);
        return x - v;
    }
    __device__ int32_t sum(int32_t v) const {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        return v;
    }
    __device__ uint64_t ballot(bool p) const { return __ballot(p); }
    __device__ int32_t bcast(int32_t v, int l) const { return __shfl(v, l, 64); }
    __device__ static int ffs(uint64_t m) { return __builtin_ctzll(m); }
    __device__ void sync() const {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
};
#endif

} /* namespace mt */
