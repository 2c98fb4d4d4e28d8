// Microbenchmark: how much do MFMAs of one wave and f32 VALU FMAs of another wave on the SAME SIMD
// interfere?  Workgroup of 8 waves = 2 per SIMD.  For each MFMA flavour (f32 32x32x2, f32 16x16x4,
// f16 32x32x16): all-MFMA, MFMA wave + VALU wave pairs, MFMA alone; plus all-VALU.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int KIND>
__device__ __forceinline__ void mfma_block(float a, float b, f16x8 ha, f16x8 hb, f32x16& c0, f32x16& c1, f32x16& c2,
                                           f32x16& c3, f32x4& d0, f32x4& d1, f32x4& d2, f32x4& d3) {
    if (KIND == 0) {   // 32 cycles of issue per 4 = 256 cyc/block (64 each)
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c3, 0, 0, 0);
    } else if (KIND == 1) {  // 8 x 32 cycles = 256
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            d0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, d0, 0, 0, 0);
            d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, d1, 0, 0, 0);
            d2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, d2, 0, 0, 0);
            d3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, d3, 0, 0, 0);
        }
    } else {  // f16 32x32x16: 8 passes = 32 cycles -> 8 per block = 256
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ha, hb, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ha, hb, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ha, hb, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ha, hb, c3, 0, 0, 0);
        }
    }
}

// mode 0: all waves MFMA; 1: all waves VALU; 2: waves 0-3 MFMA + 4-7 VALU; 3: waves 0-3 MFMA only
template <int KIND>
__global__ void __launch_bounds__(512) kern(int mode, int iters, float* out) {
    const int w = threadIdx.x >> 6;
    const bool do_mfma = (mode == 0) || ((mode == 2 || mode == 3) && w < 4);
    const bool do_valu = (mode == 1) || (mode == 2 && w >= 4);
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    f16x8 ha, hb;
    for (int i = 0; i < 8; ++i) { ha[i] = (_Float16)(a + i); hb[i] = (_Float16)b; }
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    f32x4 d0 = {}, d1 = {}, d2 = {}, d3 = {};
    float v[16];
    for (int i = 0; i < 16; ++i) v[i] = threadIdx.x * 1e-4f + i;
    if (do_mfma)
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int u = 0; u < 8; ++u) mfma_block<KIND>(a, b, ha, hb, c0, c1, c2, c3, d0, d1, d2, d3);
    if (do_valu)
        for (int it = 0; it < iters; ++it)
            for (int u = 0; u < 64; ++u)
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = fmaf(v[i], b, a);
    float s = 0;
    for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i] + v[i];
    for (int i = 0; i < 4; ++i) s += d0[i] + d1[i] + d2[i] + d3[i];
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <int KIND>
void run(const char* kname, float* out, hipEvent_t e0, hipEvent_t e1) {
    const int iters = 2000;
    const char* names[] = {"all MFMA (2 waves/SIMD)", "all VALU (2 waves/SIMD)", "MFMA wave + VALU wave per SIMD",
                           "MFMA 1 wave/SIMD only"};
    for (int mode = 0; mode < 4; ++mode) {
        if (KIND > 0 && mode == 1) continue;
        hipLaunchKernelGGL(kern<KIND>, dim3(256), dim3(512), 0, 0, mode, 10, out);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(kern<KIND>, dim3(256), dim3(512), 0, 0, mode, iters, out);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-18s mode %d %-34s %8.3f ms\n", kname, mode, names[mode], ms);
    }
}

int main() {
    float* out;
    (void)hipMalloc(&out, 4096);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    run<0>("f32_32x32x2", out, e0, e1);
    run<1>("f32_16x16x4", out, e0, e1);
    run<2>("f16_32x32x16", out, e0, e1);
    return 0;
}
