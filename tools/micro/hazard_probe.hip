// Hazard probe (developer tool): which instruction pair of the fp16x3 split -> MFMA sequence gives
// timing-dependent wrong values on MI355X?  Every test runs its sequence inside ONE asm statement on fixed
// registers (hipcc pads nothing inside asm, so each gap is exactly the one written) and compares it, lane by lane,
// with the same sequence padded far beyond any documented requirement; mismatches are counted with vector-memory
// atomics.  G = s_nop wait states in the gap under test.
//   T1 v_cvt_pk_f16_f32 -> v_cvt_f32_f16 / v_cvt_f32_f16_sdwa WORD_1 reading it     (the split's lo = x - f32(hi))
//   T2 v_cvt_pk_f16_f32 -> v_mfma_f32_32x32x16_f16 reading it as B                   (a layer's first MFMA)
//   T3 three MFMAs chained on one accumulator, then ds_read_b128 into the LAST one's A (WAR: LDS return)
//   T4 three MFMAs chained on one accumulator, then v_mov_b32 into the LAST one's B (WAR: VALU)
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/hazard_probe.hip -o /tmp/hazard_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CLOB16 "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15"
#define CLOBF "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39"
#define PAD16 "s_nop 7\n\ts_nop 7\n\t"
#define PAD64 PAD16 PAD16 PAD16 PAD16
// zero the accumulator, A fragment from a0..a3, B fragment from b0..b2 (+ v39 set by the test)
#define SETUP                                                                                      \
    "v_mov_b32 v0, 0\n\tv_mov_b32 v1, 0\n\tv_mov_b32 v2, 0\n\tv_mov_b32 v3, 0\n\t"                \
    "v_mov_b32 v4, 0\n\tv_mov_b32 v5, 0\n\tv_mov_b32 v6, 0\n\tv_mov_b32 v7, 0\n\t"                \
    "v_mov_b32 v8, 0\n\tv_mov_b32 v9, 0\n\tv_mov_b32 v10, 0\n\tv_mov_b32 v11, 0\n\t"              \
    "v_mov_b32 v12, 0\n\tv_mov_b32 v13, 0\n\tv_mov_b32 v14, 0\n\tv_mov_b32 v15, 0\n\t"            \
    "v_mov_b32 v32, %1\n\tv_mov_b32 v33, %2\n\tv_mov_b32 v34, %3\n\tv_mov_b32 v35, %4\n\t"        \
    "v_mov_b32 v36, %5\n\tv_mov_b32 v37, %6\n\tv_mov_b32 v38, %7\n\tv_mov_b32 v39, %5\n\t" PAD16
// sum of the 16 accumulator registers -> %0 (after the MFMA -> VALU read wait)
#define SUM16                                                                                      \
    PAD64 "v_add_f32 %0, v0, v1\n\tv_add_f32 %0, %0, v2\n\tv_add_f32 %0, %0, v3\n\t"              \
    "v_add_f32 %0, %0, v4\n\tv_add_f32 %0, %0, v5\n\tv_add_f32 %0, %0, v6\n\tv_add_f32 %0, %0, v7\n\t" \
    "v_add_f32 %0, %0, v8\n\tv_add_f32 %0, %0, v9\n\tv_add_f32 %0, %0, v10\n\tv_add_f32 %0, %0, v11\n\t" \
    "v_add_f32 %0, %0, v12\n\tv_add_f32 %0, %0, v13\n\tv_add_f32 %0, %0, v14\n\tv_add_f32 %0, %0, v15\n\t"
#define MF "v_mfma_f32_32x32x16_f16 v[0:15], v[32:35], v[36:39], v[0:15]\n\t"
// the 16 accumulators summed with no wait in front (the caller writes the MFMA -> VALU gap)
#define SUMRAW                                                                                     \
    "v_add_f32 %0, v0, v1\n\tv_add_f32 %0, %0, v2\n\tv_add_f32 %0, %0, v3\n\t"                    \
    "v_add_f32 %0, %0, v4\n\tv_add_f32 %0, %0, v5\n\tv_add_f32 %0, %0, v6\n\tv_add_f32 %0, %0, v7\n\t" \
    "v_add_f32 %0, %0, v8\n\tv_add_f32 %0, %0, v9\n\tv_add_f32 %0, %0, v10\n\tv_add_f32 %0, %0, v11\n\t" \
    "v_add_f32 %0, %0, v12\n\tv_add_f32 %0, %0, v13\n\tv_add_f32 %0, %0, v14\n\tv_add_f32 %0, %0, v15\n\t"
// T9: MFMA x N (one accumulator) -> VALU reads of the accumulator after GAP (hipcc: 12 states for this 8-pass MFMA)
#define T9_ASM(MFS, GAP)                                                                           \
    asm volatile(SETUP MFS GAP SUMRAW                                                              \
                 : "=&v"(r) : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2)            \
                 : CLOB16, CLOBF)

#define T2_ASM(GAP)                                                                                \
    asm volatile(SETUP "v_cvt_pk_f16_f32 v39, %8, %9\n\t" GAP MF SUM16                            \
                 : "=&v"(r) : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(x), "v"(y) \
                 : CLOB16, CLOBF)
#define T3_ASM(GAP)                                                                                \
    asm volatile(SETUP MF MF MF GAP "ds_read_b128 v[32:35], %8\n\ts_waitcnt lgkmcnt(0)\n\t" SUM16 \
                 : "=&v"(r) : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(addr) \
                 : CLOB16, CLOBF, "memory")
// T7: as T3 with the ds_read_b128 into the last MFMA's B register; T8: a global_load_dwordx4 into it
#define T7_ASM(GAP)                                                                                \
    asm volatile(SETUP MF MF MF GAP "ds_read_b128 v[36:39], %8\n\ts_waitcnt lgkmcnt(0)\n\t" SUM16 \
                 : "=&v"(r) : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(addr) \
                 : CLOB16, CLOBF, "memory")
#define T8_ASM(GAP)                                                                                \
    asm volatile(SETUP MF MF MF GAP "global_load_dwordx4 v[36:39], %8, off\n\ts_waitcnt vmcnt(0)\n\t" SUM16 \
                 : "=&v"(r) : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(gp) \
                 : CLOB16, CLOBF, "memory")
// T12: EIGHT chained MFMAs, then ds_read_b128 into the last one's B register right away (a long MFMA queue)
#define MF8 MF MF MF MF MF MF MF MF
#define T12_ASM(GAP)                                                                               \
    asm volatile(SETUP MF8 GAP "ds_read_b128 v[36:39], %8\n\ts_waitcnt lgkmcnt(0)\n\t" SUM16      \
                 : "=&v"(r) : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(addr) \
                 : CLOB16, CLOBF, "memory")
// T13: as T12 with v_cvt_pk_f16_f32 writes into the last MFMA's B register (the next layer's split)
#define T13_ASM(GAP)                                                                               \
    asm volatile(SETUP MF8 GAP "v_cvt_pk_f16_f32 v36, %8, %8\n\tv_cvt_pk_f16_f32 v37, %8, %8\n\t"   \
                 "v_cvt_pk_f16_f32 v38, %8, %8\n\tv_cvt_pk_f16_f32 v39, %8, %8\n\t" SUM16              \
                 : "=&v"(r) : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(x)    \
                 : CLOB16, CLOBF)
#define T4_ASM(GAP)                                                                                \
    asm volatile(SETUP MF MF MF GAP "v_mov_b32 v36, %8\n\tv_mov_b32 v37, %8\n\t" SUM16          \
                 : "=&v"(r) : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(z)    \
                 : CLOB16, CLOBF)

// T5: the split chain on fixed registers: hi = cvt_pk(x, y); (ta, tb) = f32(hi); d = (x, y) - (ta, tb) on
// v_pk_add_f32 [gap G1]; lo = cvt_pk(d) [gap G2 after the v_pk_add]; r = f32 sum of hi, lo halves (one value)
#define CLOBS "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47"
#define T5_ASM(G1, G2)                                                                             \
    asm volatile("v_mov_b32 v40, %1\n\tv_mov_b32 v41, %2\n\t" PAD16                               \
                 "v_cvt_pk_f16_f32 v44, v40, v41\n\tv_cvt_f32_f16_e32 v42, v44\n\t"                   \
                 "v_cvt_f32_f16_sdwa v43, v44 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1\n\t" G1 \
                 "v_pk_add_f32 v[40:41], v[40:41], v[42:43] neg_lo:[0,1] neg_hi:[0,1]\n\t" G2          \
                 "v_cvt_pk_f16_f32 v45, v40, v41\n\t" PAD16                                           \
                 "v_cvt_f32_f16_e32 v46, v45\n\tv_cvt_f32_f16_sdwa v47, v45 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1\n\t" \
                 PAD16 "v_add_f32 %0, v46, v42\n\tv_fmac_f32 %0, 4.0, v47\n\tv_fmac_f32 %0, 16.0, v43\n\t" \
                 : "=&v"(r) : "v"(x), "v"(y) : CLOBS)
// T6: v_pk_mul_f32 (the layer input scaled by 2^k) -> v_cvt_pk_f16_f32 reading it, gap G
#define T6_ASM(G)                                                                                  \
    asm volatile("v_mov_b32 v40, %1\n\tv_mov_b32 v41, %2\n\tv_mov_b32 v42, %3\n\tv_mov_b32 v43, %3\n\t" PAD16 \
                 "v_pk_mul_f32 v[40:41], v[40:41], v[42:43]\n\t" G "v_cvt_pk_f16_f32 v45, v40, v41\n\t" PAD16 \
                 "v_cvt_f32_f16_e32 v46, v45\n\tv_cvt_f32_f16_sdwa v47, v45 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1\n\t" \
                 PAD16 "v_fma_f32 %0, v47, 4.0, v46\n\t"                                            \
                 : "=&v"(r) : "v"(x), "v"(y), "v"(sc) : CLOBS)

// T11: a 64-bit address written by v_lshl_add_u64 (a 64-bit VALU op) -> global_load_dword through it, gap G.
// The pair first holds a valid address into bufA; the new address points into bufB (different values), so a
// load through a stale address returns bufA's value instead of bufB's (no wild access either way).
#define T11_ASM(GAP)                                                                               \
    asm volatile("v_mov_b32 v40, %1\n\tv_mov_b32 v41, %2\n\tv_mov_b32 v44, %3\n\tv_mov_b32 v45, 0\n\t" \
                 "v_mov_b32 v46, %4\n\tv_mov_b32 v47, %5\n\t" PAD16                                   \
                 "v_lshl_add_u64 v[40:41], v[44:45], 2, v[46:47]\n\t" GAP                             \
                 "global_load_dword v42, v[40:41], off\n\ts_waitcnt vmcnt(0)\n\tv_mov_b32 %0, v42\n\t"   \
                 : "=&v"(r) : "v"(alo), "v"(ahi), "v"(li), "v"(blo), "v"(bhi) : CLOBS, "memory")

__device__ __forceinline__ uint32_t hsh(uint32_t v) {
    v ^= v >> 16; v *= 0x7feb352dU; v ^= v >> 15; v *= 0x846ca68bU; v ^= v >> 16;
    return v;
}
// a random fp16 pair in [-1, 1) as a packed register
__device__ __forceinline__ uint32_t rnd_h2(uint32_t s) {
    const float f0 = (float)(hsh(s) & 0xffff) / 32768.0f - 1.0f, f1 = (float)(hsh(s ^ 0x9e3779b9U) & 0xffff) / 32768.0f - 1.0f;
    const _Float16 h0 = (_Float16)f0, h1 = (_Float16)f1;
    return (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
}

template <int TEST, int G>
__global__ void __launch_bounds__(256) probe(int iters, unsigned long long* bad, const float* gsrc) {
    __shared__ float lds[256 * 4];
    const int tid = threadIdx.x;
    for (int i = tid; i < 256 * 4; i += 256) lds[i] = (float)(i % 7) - 3.0f;   // NOT the A values
    __syncthreads();
    const uint32_t addr = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) float*)(lds + 4 * tid));
    unsigned long long nbad = 0;
    const float* gp = gsrc + 4 * ((blockIdx.x * 256 + tid) & 4095);
    for (int it = 0; it < iters; ++it) {
        const uint32_t s = hsh((uint32_t)(blockIdx.x * 256 + tid) * 7919u + (uint32_t)it * 104729u);
        const uint32_t a0 = rnd_h2(s), a1 = rnd_h2(s + 1), a2 = rnd_h2(s + 2), a3 = rnd_h2(s + 3);
        const uint32_t b0 = rnd_h2(s + 4), b1 = rnd_h2(s + 5), b2 = rnd_h2(s + 6);
        const float x = (float)(hsh(s + 7) & 0xffff) / 16384.0f - 2.0f, y = (float)(hsh(s + 8) & 0xffff) / 16384.0f - 2.0f;
        const uint32_t z = rnd_h2(s + 9);
        float r, ref;
        if constexpr (TEST == 1) {
            uint32_t hi;
            float ta, tb;
            if constexpr (G == 0)
                asm volatile("v_cvt_pk_f16_f32 %0, %3, %4\n\tv_cvt_f32_f16_e32 %1, %0\n\t"
                             "v_cvt_f32_f16_sdwa %2, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1\n\t"
                             : "=&v"(hi), "=&v"(ta), "=&v"(tb) : "v"(x), "v"(y));
            else
                asm volatile("v_cvt_pk_f16_f32 %0, %3, %4\n\ts_nop 0\n\tv_cvt_f32_f16_e32 %1, %0\n\t"
                             "v_cvt_f32_f16_sdwa %2, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1\n\t"
                             : "=&v"(hi), "=&v"(ta), "=&v"(tb) : "v"(x), "v"(y));
            asm volatile("" ::: "memory");
            r = ta * 3.0f + tb;
            const _Float16 hx = (_Float16)x, hy = (_Float16)y;
            ref = (float)hx * 3.0f + (float)hy;
        } else if constexpr (TEST == 2) {
            if constexpr (G == 0) T2_ASM("");
            else if constexpr (G == 1) T2_ASM("s_nop 0\n\t");
            else if constexpr (G == 2) T2_ASM("s_nop 1\n\t");
            else T2_ASM("s_nop 3\n\t");
            const float rr = r;
            T2_ASM(PAD16);
            ref = r;
            r = rr;
        } else if constexpr (TEST == 3) {
            if constexpr (G == 0) T3_ASM("");
            else if constexpr (G == 1) T3_ASM("s_nop 0\n\t");
            else if constexpr (G == 2) T3_ASM("s_nop 1\n\t");
            else T3_ASM("s_nop 7\n\t");
            const float rr = r;
            T3_ASM(PAD64 PAD64);
            ref = r;
            r = rr;
        } else if constexpr (TEST == 12) {
            if constexpr (G == 0) T12_ASM("");
            else T12_ASM(PAD64);
            const float rr = r;
            T12_ASM(PAD64 PAD64 PAD64 PAD64);
            ref = r;
            r = rr;
        } else if constexpr (TEST == 13) {
            if constexpr (G == 0) T13_ASM("");
            else T13_ASM(PAD64);
            const float rr = r;
            T13_ASM(PAD64 PAD64 PAD64 PAD64);
            ref = r;
            r = rr;
        } else if constexpr (TEST == 11) {
            const uint32_t li = (uint32_t)((blockIdx.x * 256 + tid) & 4095);
            const uint64_t pa = (uint64_t)(uintptr_t)(gsrc + li), pb = (uint64_t)(uintptr_t)(gsrc + 4096);
            const uint32_t alo = (uint32_t)pa, ahi = (uint32_t)(pa >> 32), blo = (uint32_t)pb, bhi = (uint32_t)(pb >> 32);
            if constexpr (G == 0) T11_ASM("");
            else if constexpr (G == 1) T11_ASM("s_nop 0\n\t");
            else T11_ASM("s_nop 1\n\t");
            const float rr = r;
            T11_ASM(PAD16);
            ref = r;
            r = rr;
        } else if constexpr (TEST == 9) {        // one MFMA, gap G (in wait states: s_nop G-1)
            if constexpr (G == 8) T9_ASM(MF, "s_nop 7\n\t");
            else if constexpr (G == 12) T9_ASM(MF, "s_nop 7\n\ts_nop 3\n\t");
            else if constexpr (G == 16) T9_ASM(MF, "s_nop 7\n\ts_nop 7\n\t");
            else T9_ASM(MF, "s_nop 7\n\ts_nop 7\n\ts_nop 3\n\t");
            const float rr = r;
            T9_ASM(MF, PAD64);
            ref = r;
            r = rr;
        } else if constexpr (TEST == 10) {       // three chained MFMAs, gap G after the last
            if constexpr (G == 8) T9_ASM(MF MF MF, "s_nop 7\n\t");
            else if constexpr (G == 12) T9_ASM(MF MF MF, "s_nop 7\n\ts_nop 3\n\t");
            else if constexpr (G == 16) T9_ASM(MF MF MF, "s_nop 7\n\ts_nop 7\n\t");
            else T9_ASM(MF MF MF, "s_nop 7\n\ts_nop 7\n\ts_nop 3\n\t");
            const float rr = r;
            T9_ASM(MF MF MF, PAD64);
            ref = r;
            r = rr;
        } else if constexpr (TEST == 7) {
            if constexpr (G == 0) T7_ASM("");
            else if constexpr (G == 1) T7_ASM("s_nop 0\n\t");
            else T7_ASM("s_nop 7\n\t");
            const float rr = r;
            T7_ASM(PAD64 PAD64);
            ref = r;
            r = rr;
        } else if constexpr (TEST == 8) {
            if constexpr (G == 0) T8_ASM("");
            else T8_ASM("s_nop 7\n\t");
            const float rr = r;
            T8_ASM(PAD64 PAD64);
            ref = r;
            r = rr;
        } else if constexpr (TEST == 5) {
            if constexpr (G == 0) T5_ASM("", "");
            else if constexpr (G == 1) T5_ASM("", "s_nop 0\n\t");
            else if constexpr (G == 2) T5_ASM("s_nop 0\n\t", "s_nop 1\n\t");
            else T5_ASM("s_nop 3\n\t", "s_nop 3\n\t");
            const float rr = r;
            T5_ASM(PAD16, PAD16);
            ref = r;
            r = rr;
        } else if constexpr (TEST == 6) {
            const float sc = 0.125f;
            if constexpr (G == 0) T6_ASM("");
            else if constexpr (G == 1) T6_ASM("s_nop 0\n\t");
            else T6_ASM("s_nop 1\n\t");
            const float rr = r;
            T6_ASM(PAD16);
            ref = r;
            r = rr;
        } else {
            if constexpr (G == 0) T4_ASM("");
            else if constexpr (G == 1) T4_ASM("s_nop 0\n\t");
            else if constexpr (G == 2) T4_ASM("s_nop 1\n\t");
            else T4_ASM("s_nop 7\n\t");
            const float rr = r;
            T4_ASM(PAD64 PAD64);
            ref = r;
            r = rr;
        }
        if (__float_as_uint(r) != __float_as_uint(ref)) ++nbad;
    }
    if (nbad) atomicAdd(bad, nbad);
}

template <int TEST, int G>
void run(const char* name, int blocks, int iters, unsigned long long* d) {
    hipMemset(d, 0, 8);
    static float* g = nullptr;
    if (!g) {
        hipMalloc(&g, 4096 * 16);
        static float h[4096 * 4];
        for (int i = 0; i < 4096 * 4; ++i) h[i] = i < 4096 ? 1.0f : (i < 8192 ? 2.0f : (float)(i % 5) - 2.0f);
        hipMemcpy(g, h, sizeof(h), hipMemcpyHostToDevice);
    }
    hipLaunchKernelGGL((probe<TEST, G>), dim3(blocks), dim3(256), 0, 0, iters, d, (const float*)g);
    unsigned long long h = 0;
    hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    printf("%-58s gap %d: %llu / %llu lane-iterations differ from the padded sequence\n", name, G, h,
           (unsigned long long)blocks * 256ull * (unsigned long long)iters);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 4096;
    const int iters = argc > 2 ? atoi(argv[2]) : 200;
    unsigned long long* d;
    hipMalloc(&d, 8);
    if (argc > 3 && argv[3][0] == 'q') {   // T12 / T13: WAR on B behind a long MFMA queue
        run<12, 0>("T12 mfma x8 (one acc) -> ds_read_b128 into last B", blocks, iters, d);
        run<13, 0>("T13 mfma x8 (one acc) -> v_cvt_pk into last B", blocks, iters, d);
        run<12, 1>("T12 mfma x8 (one acc) -> ds_read_b128 into last B", blocks, iters, d);
        return 0;
    }
    if (argc > 3 && argv[3][0] == 'a') {   // only T11 (64-bit VALU address -> VMEM)
        run<11, 0>("T11 v_lshl_add_u64 address -> global_load", blocks, iters, d);
        run<11, 1>("T11 v_lshl_add_u64 address -> global_load", blocks, iters, d);
        run<11, 2>("T11 v_lshl_add_u64 address -> global_load", blocks, iters, d);
        return 0;
    }
    if (argc > 3 && argv[3][0] == 'r') {   // only T9 / T10 (MFMA result -> VALU read)
        run<9, 8>("T9 mfma -> VALU read of its result", blocks, iters, d);
        run<9, 12>("T9 mfma -> VALU read of its result", blocks, iters, d);
        run<9, 16>("T9 mfma -> VALU read of its result", blocks, iters, d);
        run<9, 20>("T9 mfma -> VALU read of its result", blocks, iters, d);
        run<10, 8>("T10 mfma x3 (one acc) -> VALU read of the result", blocks, iters, d);
        run<10, 12>("T10 mfma x3 (one acc) -> VALU read of the result", blocks, iters, d);
        run<10, 16>("T10 mfma x3 (one acc) -> VALU read of the result", blocks, iters, d);
        run<10, 20>("T10 mfma x3 (one acc) -> VALU read of the result", blocks, iters, d);
        return 0;
    }
    if (argc > 3 && argv[3][0] == 'b') {   // only T7 / T8 (WAR on B by memory returns)
        run<7, 0>("T7 mfma x3 (one acc) -> ds_read_b128 into last B", blocks, iters, d);
        run<7, 1>("T7 mfma x3 (one acc) -> ds_read_b128 into last B", blocks, iters, d);
        run<7, 8>("T7 mfma x3 (one acc) -> ds_read_b128 into last B", blocks, iters, d);
        run<8, 0>("T8 mfma x3 (one acc) -> global_load_dwordx4 into last B", blocks, iters, d);
        run<8, 8>("T8 mfma x3 (one acc) -> global_load_dwordx4 into last B", blocks, iters, d);
        return 0;
    }
    if (argc > 3) {   // only T5 / T6
        run<5, 0>("T5 split chain: sdwa cvt -> v_pk_add [g] -> cvt_pk [g]", blocks, iters, d);
        run<5, 1>("T5 split chain: sdwa cvt -> v_pk_add [g] -> cvt_pk [g]", blocks, iters, d);
        run<5, 2>("T5 split chain: sdwa cvt -> v_pk_add [g] -> cvt_pk [g]", blocks, iters, d);
        run<6, 0>("T6 v_pk_mul_f32 -> cvt_pk_f16_f32", blocks, iters, d);
        run<6, 1>("T6 v_pk_mul_f32 -> cvt_pk_f16_f32", blocks, iters, d);
        return 0;
    }
    run<1, 0>("T1 cvt_pk_f16_f32 -> cvt_f32_f16 (+sdwa WORD_1)", blocks, iters, d);
    run<1, 1>("T1 cvt_pk_f16_f32 -> cvt_f32_f16 (+sdwa WORD_1)", blocks, iters, d);
    run<2, 0>("T2 cvt_pk_f16_f32 -> mfma B", blocks, iters, d);
    run<2, 1>("T2 cvt_pk_f16_f32 -> mfma B", blocks, iters, d);
    run<2, 2>("T2 cvt_pk_f16_f32 -> mfma B", blocks, iters, d);
    run<2, 4>("T2 cvt_pk_f16_f32 -> mfma B", blocks, iters, d);
    run<3, 0>("T3 mfma x3 (one acc) -> ds_read_b128 into last A", blocks, iters, d);
    run<3, 1>("T3 mfma x3 (one acc) -> ds_read_b128 into last A", blocks, iters, d);
    run<3, 2>("T3 mfma x3 (one acc) -> ds_read_b128 into last A", blocks, iters, d);
    run<3, 8>("T3 mfma x3 (one acc) -> ds_read_b128 into last A", blocks, iters, d);
    run<5, 0>("T5 split chain: sdwa cvt -> v_pk_add [g] -> cvt_pk [g]", blocks, iters, d);
    run<5, 1>("T5 split chain: sdwa cvt -> v_pk_add [g] -> cvt_pk [g]", blocks, iters, d);
    run<5, 2>("T5 split chain: sdwa cvt -> v_pk_add [g] -> cvt_pk [g]", blocks, iters, d);
    run<5, 4>("T5 split chain: sdwa cvt -> v_pk_add [g] -> cvt_pk [g]", blocks, iters, d);
    run<6, 0>("T6 v_pk_mul_f32 -> cvt_pk_f16_f32", blocks, iters, d);
    run<6, 1>("T6 v_pk_mul_f32 -> cvt_pk_f16_f32", blocks, iters, d);
    run<6, 2>("T6 v_pk_mul_f32 -> cvt_pk_f16_f32", blocks, iters, d);
    run<4, 0>("T4 mfma x3 (one acc) -> v_mov into last B", blocks, iters, d);
    run<4, 1>("T4 mfma x3 (one acc) -> v_mov into last B", blocks, iters, d);
    run<4, 2>("T4 mfma x3 (one acc) -> v_mov into last B", blocks, iters, d);
    run<4, 8>("T4 mfma x3 (one acc) -> v_mov into last B", blocks, iters, d);
    hipFree(d);
    return 0;
}
