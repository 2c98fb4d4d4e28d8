// Transcendental-forwarding probe (developer tool).  hipcc pads a trans VALU result (v_rcp_f32,
// v_sqrt_f32, v_exp_f32, ...) read by the next VALU with ONE wait state (s_nop 0, LLVM's gfx940 "trans forwarding"
// rule).  Is one enough on MI355X when the SIMD is busy?  Each test runs `trans dst <- x`, a gap of G wait states,
// and a consumer reading dst, inside ONE asm statement on fixed registers whose dst held a different value before
// (so a stale read shows), and compares lane by lane with the same sequence padded by 16 states.  Mismatches are
// counted per 16-lane quarter of the wave.  MIX = 1: odd waves of every workgroup run back-to-back MFMA chains
// meanwhile (the render's other wave on the SIMD is often in its MLP), so the trans unit and the matrix core are
// busy at the same time.
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/trans_probe.hip -o tools/micro/trans_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define PAD16 "s_nop 7\n\ts_nop 7\n\t"
#define CLOBT "v40", "v41", "v42"
// v40 <- stale value, then v40 <- TRANS(x), GAP, consumer r = fma(-x, v40, 1.0) (the fdiv Newton step) or
// r = v40 + 1 (integer, the sqrt correction step), all on fixed registers
#define TRANS_ASM(OP, GAP, CONS)                                                                   \
    asm volatile("v_mov_b32 v40, %2\n\tv_mov_b32 v41, %1\n\t" PAD16 OP " v40, v41\n\t" GAP CONS     \
                 "\n\t" PAD16 "v_mov_b32 %0, v42\n\t"                                             \
                 : "=&v"(r) : "v"(x), "v"(stale) : CLOBT)
// OPI 5 / 6: a 32-bit VALU writes the low half of a 64-bit index pair, then v_lshl_add_u64 (a 64-bit VALU op)
// reads the pair as the hash-row address (v98 <- v_bitop3_b32 / v_xor_b32; v_lshl_add_u64 v[..], v[98:99], 3, base)
#define CLOBU "v40", "v41", "v42", "v43", "v44", "v45"
#define U64_ASM(OP, GAP)                                                                           \
    asm volatile("v_mov_b32 v40, %2\n\tv_mov_b32 v41, 0\n\tv_mov_b32 v44, %3\n\tv_mov_b32 v45, 0\n\t" PAD16 \
                 OP "\n\t" GAP "v_lshl_add_u64 v[42:43], v[40:41], 3, v[44:45]\n\t" PAD16          \
                 "v_mov_b32 %0, v42\n\t"                                                          \
                 : "=&v"(r) : "v"(__float_as_uint(x)), "v"(__float_as_uint(stale)), "v"(0x1000u) : CLOBU)
#define C_FMA "v_fma_f32 v42, -v41, v40, 1.0"
#define C_ADD "v_add_u32_e32 v42, -1, v40"
#define C_MUL "v_mul_f32_e32 v42, v40, v41"

template <int OPI, int G>
__device__ __forceinline__ float one(float x, float stale) {
    float r;
#define GAPSEL(OP, CONS)                                                                           \
    if constexpr (G == 0) TRANS_ASM(OP, "", CONS);                                                 \
    else if constexpr (G == 1) TRANS_ASM(OP, "s_nop 0\n\t", CONS);                                 \
    else if constexpr (G == 2) TRANS_ASM(OP, "s_nop 1\n\t", CONS);                                 \
    else TRANS_ASM(OP, PAD16, CONS);
    if constexpr (OPI == 0) { GAPSEL("v_rcp_f32_e32", C_FMA) }
    else if constexpr (OPI == 1) { GAPSEL("v_sqrt_f32_e32", C_ADD) }
    else if constexpr (OPI == 2) { GAPSEL("v_exp_f32_e32", C_MUL) }
    else if constexpr (OPI == 3) { GAPSEL("v_rsq_f32_e32", C_MUL) }
#define U64SEL(OP)                                                                                 \
    if constexpr (G == 0) U64_ASM(OP, "");                                                         \
    else if constexpr (G == 1) U64_ASM(OP, "s_nop 0\n\t");                                         \
    else if constexpr (G == 2) U64_ASM(OP, "s_nop 1\n\t");                                         \
    else U64_ASM(OP, PAD16);
    else if constexpr (OPI == 5) { U64SEL("v_xor_b32_e32 v40, %1, v40") }
    else if constexpr (OPI == 6) { U64SEL("v_bitop3_b32 v40, %1, v40, %3 bitop3:0x48") }
    else { GAPSEL("v_log_f32_e32", C_MUL) }
    return r;
}

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t hsh(uint32_t v) {
    v ^= v >> 16; v *= 0x7feb352dU; v ^= v >> 15; v *= 0x846ca68bU; v ^= v >> 16;
    return v;
}

template <int OPI, int G, int MIX>
__global__ void __launch_bounds__(256) probe(int iters, unsigned long long* bad, float* sink) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (MIX && (wave & 1)) {   // MFMA load on the same SIMD (waves w and w+4 of a 256-thread block share none;
                               // with 8 resident blocks per CU every SIMD holds trans and MFMA waves)
        f16x8 a, b;
        for (int e = 0; e < 8; ++e) { a[e] = (_Float16)(0.001f * (lane + e)); b[e] = (_Float16)(0.002f * (e - lane)); }
        f32x16 c0 = {}, c1 = {};
        for (int it = 0; it < iters * 2; ++it) {
            c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, c1, 0, 0, 0);
        }
        float s = 0.0f;
        for (int i = 0; i < 16; ++i) s += c0[i] + c1[i];
        if (s == 12345.0f) sink[0] = s;
        return;
    }
    unsigned long long nb[4] = {0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
        const uint32_t h = hsh((uint32_t)(blockIdx.x * 256 + threadIdx.x) * 7919u + (uint32_t)it * 104729u);
        float x = 0.5f + (float)(h & 0xffffff) / 16777216.0f * 4.0f;      // (0.5, 4.5)
        const float stale = -1.0f - (float)(hsh(h) & 0xffff) / 65536.0f;   // a different value in dst before
        const float r = one<OPI, G>(x, stale);
        const float ref = one<OPI, 16>(x, stale);
        if (__float_as_uint(r) != __float_as_uint(ref)) ++nb[lane >> 4];
    }
    for (int q = 0; q < 4; ++q)
        if (nb[q]) atomicAdd(bad + q, nb[q]);
}

static const char* kName[] = {"v_rcp_f32 -> v_fma (fdiv Newton step)", "v_sqrt_f32 -> v_add_u32 (sqrt fixup)",
                              "v_exp_f32 -> v_mul", "v_rsq_f32 -> v_mul", "v_log_f32 -> v_mul",
                              "v_xor_b32 -> v_lshl_add_u64 (64-bit index)", "v_bitop3_b32 -> v_lshl_add_u64"};

template <int OPI, int G, int MIX>
void run(int blocks, int iters, unsigned long long* d, float* sink) {
    hipMemset(d, 0, 32);
    hipLaunchKernelGGL((probe<OPI, G, MIX>), dim3(blocks), dim3(256), 0, 0, iters, d, sink);
    unsigned long long h[4];
    hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
    const unsigned long long n = (unsigned long long)blocks * (MIX ? 128ull : 256ull) * (unsigned long long)iters;
    printf("%-40s gap %d %s: lanes 0-15 %llu, 16-31 %llu, 32-47 %llu, 48-63 %llu differ / %llu lane-iterations\n",
           kName[OPI], G, MIX ? "(MFMA waves beside)" : "(alone)            ", h[0], h[1], h[2], h[3], n);
    fflush(stdout);
}

template <int OPI>
void all(int blocks, int iters, unsigned long long* d, float* sink) {
    run<OPI, 0, 0>(blocks, iters, d, sink);
    run<OPI, 1, 0>(blocks, iters, d, sink);
    run<OPI, 2, 0>(blocks, iters, d, sink);
    run<OPI, 0, 1>(blocks, iters, d, sink);
    run<OPI, 1, 1>(blocks, iters, d, sink);
    run<OPI, 2, 1>(blocks, iters, d, sink);
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 4096;
    const int iters = argc > 2 ? atoi(argv[2]) : 200;
    unsigned long long* d;
    float* sink;
    hipMalloc(&d, 32);
    hipMalloc(&sink, 4);
    if (argc > 3 && argv[3][0] == 'u') {   // only the 64-bit index tests
        all<5>(blocks, iters, d, sink);
        all<6>(blocks, iters, d, sink);
        return 0;
    }
    all<0>(blocks, iters, d, sink);
    all<1>(blocks, iters, d, sink);
    all<2>(blocks, iters, d, sink);
    all<3>(blocks, iters, d, sink);
    all<4>(blocks, iters, d, sink);
    hipFree(d);
    hipFree(sink);
    return 0;
}
