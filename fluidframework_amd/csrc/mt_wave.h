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
    int32_t max(int32_t v) const { return v; }
    uint64_t ballot(bool p) const { return p ? 1ull : 0ull; }
    int32_t bcast(int32_t v, int) const { return v; }
    int32_t shfl(int32_t v, int) const { return v; }
    int32_t shfl_xor(int32_t v, int) const { return v; }
    static int32_t uniform(int32_t v) { return v; }
    int32_t writelane(int32_t v, int, int32_t) const { return v; }
    static int ffs(uint64_t m) { return __builtin_ctzll(m); }
    void sync() const {}
    static void atomic_add(int32_t* p, int32_t v) { *p += v; }
};

#ifdef __HIPCC__
/* DPP control codes (GFX9 family, gfx950 included) */
#define MT_DPP_ROW_SHR(n) (0x110 + (n))
#define MT_DPP_ROW_BCAST15 0x142
#define MT_DPP_ROW_BCAST31 0x143

struct WaveGPU {
    static constexpr int N = 64;
    __device__ __attribute__((always_inline)) int lane() const { return (int)(threadIdx.x & 63); }
    /* inclusive prefix sum over the 64 lanes: 4 row_shr steps inside each 16-lane row, then
     * row_bcast:15 / row_bcast:31 carry the row totals (the GFX9 wave64 scan sequence).
     * Lanes without a source keep the identity (old = 0). Six VALU ops, no LDS traffic. */
    __device__ __attribute__((always_inline)) int32_t incl_scan(int32_t v) const {
        int32_t x = v;
        x += __builtin_amdgcn_update_dpp(0, x, MT_DPP_ROW_SHR(1), 0xf, 0xf, false);
        x += __builtin_amdgcn_update_dpp(0, x, MT_DPP_ROW_SHR(2), 0xf, 0xf, false);
        x += __builtin_amdgcn_update_dpp(0, x, MT_DPP_ROW_SHR(4), 0xf, 0xf, false);
        x += __builtin_amdgcn_update_dpp(0, x, MT_DPP_ROW_SHR(8), 0xf, 0xf, false);
        x += __builtin_amdgcn_update_dpp(0, x, MT_DPP_ROW_BCAST15, 0xa, 0xf, false);
        x += __builtin_amdgcn_update_dpp(0, x, MT_DPP_ROW_BCAST31, 0xc, 0xf, false);
        return x;
    }
    __device__ __attribute__((always_inline)) int32_t excl_scan(int32_t v, int32_t* tot) const {
        int32_t x = incl_scan(v);
        *tot = __builtin_amdgcn_readlane(x, 63);
        return x - v;
    }
    __device__ __attribute__((always_inline)) int32_t sum(int32_t v) const {
        return __builtin_amdgcn_readlane(incl_scan(v), 63);
    }
    /* maximum over the 64 lanes (butterfly over ds_bpermute; off the per-event path) */
    __device__ __attribute__((always_inline)) int32_t max(int32_t v) const {
        for (int o = 32; o > 0; o >>= 1) {
            int32_t u = __shfl_xor(v, o);
            v = u > v ? u : v;
        }
        return __builtin_amdgcn_readfirstlane(v);
    }
    __device__ __attribute__((always_inline)) uint64_t ballot(bool p) const { return __ballot(p); }
    /* a value every lane holds equally, moved to an SGPR */
    __device__ __attribute__((always_inline)) static int32_t uniform(int32_t v) {
        return __builtin_amdgcn_readfirstlane(v);
    }
    /* lane l (wave-uniform) of the result takes v; other lanes keep old */
    __device__ __attribute__((always_inline)) int32_t writelane(int32_t v, int l, int32_t old) const {
        return lane() == l ? v : old;
    }
    /* l is wave-uniform: v_readlane, no LDS round trip */
    __device__ __attribute__((always_inline)) int32_t bcast(int32_t v, int l) const {
        return __builtin_amdgcn_readlane(v, l);
    }
    __device__ __attribute__((always_inline)) static int ffs(uint64_t m) { return __builtin_ctzll(m); }
    /* every lane takes v of lane src (per-lane source: ds_bpermute) */
    __device__ __attribute__((always_inline)) int32_t shfl(int32_t v, int src) const { return __shfl(v, src); }
    /* every lane takes v of lane (lane ^ m) */
    __device__ __attribute__((always_inline)) int32_t shfl_xor(int32_t v, int m) const { return __shfl_xor(v, m); }
    /* per-lane add into wave-shared scratch (LDS in the tiled replay kernel) */
    __device__ __attribute__((always_inline)) static void atomic_add(int32_t* p, int32_t v) { atomicAdd(p, v); }
    /* Order the wave's memory accesses between lanes. One wavefront replays one document, so every
     * hand-off is between lanes of the same wave: its LDS operations execute in program order and so
     * do its vector-memory operations to one address, so only the compiler has to be kept from
     * moving accesses across this point. (A workgroup-scope fence would also wait for every
     * outstanding global store, s_waitcnt vmcnt(0), at each call.) */
    __device__ __attribute__((always_inline)) void sync() const {
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __builtin_amdgcn_wave_barrier();
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
};
#endif

} /* namespace mt */
