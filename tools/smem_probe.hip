/*
 * smem_probe.hip — isolates the k_digest mismatch of round 1.
 *
 * Without a compiler barrier, k_digest read the leaf-line columns with a scalar load of the form
 *     s_load_dword sD, s[base:base+1], sOFF offset:IMM      (SGPR offset AND immediate offset)
 * which no other kernel uses. This probe checks, on the GPU, whether that addressing form and plain
 * scalar loads return what vector loads return:
 *   k_fill   : vector stores of a pattern (salted, so a second fill changes every word)
 *   k_soe    : uniform load p[j + 80] for a kernel-argument j (compiler emits soffset + imm)
 *   k_soe_asm: the same addressing form written as inline asm
 *   k_imm    : uniform loads p[80] with p advanced per j on the scalar side (imm only)
 *   k_vec    : the same words through vector loads
 * Run order: fill(1), all four reads, fill(2), all four reads again (staleness across kernels).
 * Prints the mismatch count of each read against the host-computed pattern.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CHK(x)                                                                 \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            return 2;                                                          \
        }                                                                      \
    } while (0)

static __host__ __device__ inline uint32_t pat(uint32_t i, uint32_t salt) {
    uint32_t x = i * 0x9E3779B1u ^ salt * 0x85EBCA77u;
    x ^= x >> 15;
    x *= 0x2C1B3C6Du;
    return x ^ (x >> 12);
}

__global__ void k_fill(uint32_t* p, int64_t n, uint32_t salt) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = pat((uint32_t)i, salt);
}

/* one wave per block; block b reads the 128-byte "line" at word offset 64*b + 64 (like lf[n]); the
 * word index j is a kernel argument, so the compiler addresses it as base + soffset(4j) + imm(320) */
__global__ __launch_bounds__(64) void k_soe(const uint32_t* __restrict__ p, uint32_t* __restrict__ out, int j) {
    const uint32_t* line = p + 64 * (int64_t)blockIdx.x;
    uint32_t v = line[j + 80];
    if (threadIdx.x == 0) out[8 * (int64_t)blockIdx.x + j] = v;
}
/* the same addressing form written out explicitly */
__global__ __launch_bounds__(64) void k_soe_asm(const uint32_t* __restrict__ p, uint32_t* __restrict__ out, int j) {
    const uint32_t* line = p + 64 * (int64_t)blockIdx.x;
    uint32_t v;
    uint32_t off = 4u * (uint32_t)j;
    __asm__ volatile("s_load_dword %0, %1, %2 offset:0x140\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(line), "s"(off));
    if (threadIdx.x == 0) out[8 * (int64_t)blockIdx.x + j] = v;
}

__global__ __launch_bounds__(64) void k_imm(const uint32_t* __restrict__ p, uint32_t* __restrict__ out, int nj) {
    uint32_t acc[8];
    for (int j = 0; j < 8; j++) acc[j] = 0;
#pragma unroll
    for (int j = 0; j < 8; j++)
        if (j < nj) acc[j] = p[64 * (int64_t)blockIdx.x + 80 + j]; /* constant offsets only */
    if (threadIdx.x == 0)
        for (int j = 0; j < 8; j++) out[8 * (int64_t)blockIdx.x + j] = acc[j];
}

__global__ __launch_bounds__(64) void k_vec(const uint32_t* p, uint32_t* out, int nj) {
    int j = threadIdx.x & 7;
    uint32_t v = 0;
    if (j < nj) v = __builtin_nontemporal_load(&p[64 * (int64_t)blockIdx.x + 80 + j]);
    if (threadIdx.x < 8) out[8 * (int64_t)blockIdx.x + j] = v;
}

int main(int argc, char** argv) {
    int64_t nblk = argc > 1 ? atoll(argv[1]) : (1 << 20);
    int64_t nwords = 64 * nblk + 256;
    uint32_t *p, *o;
    CHK(hipMalloc(&p, 4 * nwords));
    CHK(hipMalloc(&o, 4 * 8 * nblk));
    std::vector<uint32_t> h(8 * nblk);
    const char* names[4] = {"soe (compiler)", "soe (asm)", "imm", "vector"};
    int bad_total = 0;
    for (uint32_t salt = 1; salt <= 2; salt++) {
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, p, nwords, salt);
        CHK(hipDeviceSynchronize());
        for (int k = 0; k < 4; k++) {
            CHK(hipMemset(o, 0xff, 4 * 8 * nblk));
            for (int j = 0; j < 8 && k < 2; j++) {
                if (k == 0) hipLaunchKernelGGL(k_soe, dim3((unsigned)nblk), dim3(64), 0, 0, p, o, j);
                if (k == 1) hipLaunchKernelGGL(k_soe_asm, dim3((unsigned)nblk), dim3(64), 0, 0, p, o, j);
            }
            if (k == 2) hipLaunchKernelGGL(k_imm, dim3((unsigned)nblk), dim3(64), 0, 0, p, o, 8);
            if (k == 3) hipLaunchKernelGGL(k_vec, dim3((unsigned)nblk), dim3(64), 0, 0, p, o, 8);
            CHK(hipDeviceSynchronize());
            CHK(hipMemcpy(h.data(), o, 4 * 8 * nblk, hipMemcpyDeviceToHost));
            int64_t bad = 0, first = -1;
            for (int64_t b = 0; b < nblk; b++)
                for (int j = 0; j < 8; j++)
                    if (h[8 * b + j] != pat((uint32_t)(64 * b + 80 + j), salt)) {
                        if (first < 0) first = 8 * b + j;
                        bad++;
                    }
            printf("salt %u %-18s mismatches %lld / %lld", salt, names[k], (long long)bad, (long long)(8 * nblk));
            if (first >= 0)
                printf("  first at block %lld word %lld: got %08x want %08x", (long long)(first / 8),
                       (long long)(first % 8), h[first], pat((uint32_t)(64 * (first / 8) + 80 + first % 8), salt));
            printf("\n");
            bad_total += bad != 0;
        }
    }
    CHK(hipFree(p));
    CHK(hipFree(o));
    return bad_total ? 1 : 0;
}
