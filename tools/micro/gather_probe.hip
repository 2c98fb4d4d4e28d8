// Hash-gather sequence probe (developer tool).  The self-check builds show lanes 48-63 of ONE
// hash level receiving wrong corner data now and then when the level's rows are fetched with global_load_dwordx2
// through 64-bit addresses built by v_lshl_add_u64 (as hipcc emits for hash_issue), and never when the same rows
// come through buffer_load with 32-bit offsets.  This replays the emitted shape on fixed registers: per corner
// v_xor (row index) -> v_lshl_add_u64 (row address = base + 8 * index) -> global_load_dwordx2 whose destination
// IS its address pair (DST=1, hipcc's choice under register pressure) or a separate pair (DST=0), 8 corners per
// level, two levels in flight, then s_waitcnt and every row checked (row i of the table holds (i, ~i)).  Wrong rows
// are counted per quarter of the wave.  MODE 2: the same rows through buffer_load_dwordx2 with a 32-bit offset.
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/gather_probe.hip -o tools/micro/gather_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr uint32_t kLog2 = 22;              // rows per level table
constexpr uint32_t kRows = 1u << kLog2;     // 32 MiB

__device__ __forceinline__ uint32_t hsh(uint32_t v) {
    v ^= v >> 16; v *= 0x7feb352dU; v ^= v >> 15; v *= 0x846ca68bU; v ^= v >> 16;
    return v;
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// one corner: index = (a ^ b) & mask; address = base + 8 * index; load; the address pair is the destination
#define CORNER_DST(D)                                                                              \
    "v_xor_b32 v40, %[a" #D "], %[b]\n\t"                                                           \
    "v_and_b32 v40, %[m], v40\n\t"                                                                  \
    "v_lshl_add_u64 v[" #D ":" #D "+1], v[40:41], 3, v[42:43]\n\t"                                  \
    "global_load_dwordx2 v[" #D ":" #D "+1], v[" #D ":" #D "+1], off\n\t"

template <int MODE>
__global__ void __launch_bounds__(256) probe(int iters, const uint2* __restrict__ tab, unsigned long long* bad) {
    const int lane = threadIdx.x & 63;
    unsigned long long nb[4] = {0, 0, 0, 0};
    const uint64_t base = (uint64_t)(uintptr_t)tab;
    for (int it = 0; it < iters; ++it) {
        const uint32_t s = hsh((uint32_t)(blockIdx.x * 256 + threadIdx.x) * 7919u + (uint32_t)it * 104729u);
        uint32_t a[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) a[c] = hsh(s + 17u * c);
        const uint32_t b = hsh(s ^ 0x5bd1e995u), m = kRows - 1;
        u32x2 r[16];
        if constexpr (MODE == 1) {
            asm volatile(
                "v_mov_b32 v41, 0\n\tv_mov_b32 v42, %[blo]\n\tv_mov_b32 v43, %[bhi]\n\ts_nop 4\n\t"
                CORNER_DST(44) CORNER_DST(46) CORNER_DST(48) CORNER_DST(50)
                CORNER_DST(52) CORNER_DST(54) CORNER_DST(56) CORNER_DST(58)
                "s_nop 0\n\t"
                CORNER_DST(60) CORNER_DST(62) CORNER_DST(64) CORNER_DST(66)
                CORNER_DST(68) CORNER_DST(70) CORNER_DST(72) CORNER_DST(74)
                "s_waitcnt vmcnt(8)\n\t"
                "v_mov_b32 %[r0], v44\n\tv_mov_b32 %[r1], v46\n\tv_mov_b32 %[r2], v48\n\tv_mov_b32 %[r3], v50\n\t"
                "v_mov_b32 %[r4], v52\n\tv_mov_b32 %[r5], v54\n\tv_mov_b32 %[r6], v56\n\tv_mov_b32 %[r7], v58\n\t"
                "s_waitcnt vmcnt(0)\n\t"
                "v_mov_b32 %[r8], v60\n\tv_mov_b32 %[r9], v62\n\tv_mov_b32 %[r10], v64\n\tv_mov_b32 %[r11], v66\n\t"
                "v_mov_b32 %[r12], v68\n\tv_mov_b32 %[r13], v70\n\tv_mov_b32 %[r14], v72\n\tv_mov_b32 %[r15], v74\n\t"
                : [r0] "=&v"(r[0].x), [r1] "=&v"(r[1].x), [r2] "=&v"(r[2].x), [r3] "=&v"(r[3].x),
                  [r4] "=&v"(r[4].x), [r5] "=&v"(r[5].x), [r6] "=&v"(r[6].x), [r7] "=&v"(r[7].x),
                  [r8] "=&v"(r[8].x), [r9] "=&v"(r[9].x), [r10] "=&v"(r[10].x), [r11] "=&v"(r[11].x),
                  [r12] "=&v"(r[12].x), [r13] "=&v"(r[13].x), [r14] "=&v"(r[14].x), [r15] "=&v"(r[15].x)
                : [a44] "v"(a[0]), [a46] "v"(a[1]), [a48] "v"(a[2]), [a50] "v"(a[3]), [a52] "v"(a[4]),
                  [a54] "v"(a[5]), [a56] "v"(a[6]), [a58] "v"(a[7]), [a60] "v"(a[8]), [a62] "v"(a[9]),
                  [a64] "v"(a[10]), [a66] "v"(a[11]), [a68] "v"(a[12]), [a70] "v"(a[13]), [a72] "v"(a[14]),
                  [a74] "v"(a[15]), [b] "v"(b), [m] "v"(m), [blo] "s"((uint32_t)base), [bhi] "s"((uint32_t)(base >> 32))
                : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53",
                  "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67",
                  "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "memory");
        } else {
            // the compiler's own code for the same gathers (MODE 0: global loads from 64-bit addresses; MODE 2:
            // buffer loads with 32-bit byte offsets)
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)tab, (short)0,
                                                                                 (int)(kRows * 8u), 0x00020000);
#pragma unroll
            for (int c = 0; c < 16; ++c) {
                const uint32_t i = (a[c] ^ b) & m;
                if constexpr (MODE == 2) r[c] = __builtin_amdgcn_raw_buffer_load_b64(rs, i << 3, 0, 0);
                else r[c] = *reinterpret_cast<const u32x2*>(tab + i);
            }
        }
#pragma unroll
        for (int c = 0; c < 16; ++c)
            if (r[c].x != ((a[c] ^ b) & m)) ++nb[lane >> 4];
    }
    for (int q = 0; q < 4; ++q)
        if (nb[q]) atomicAdd(bad + q, nb[q]);
}

__global__ void fill(uint2* t) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < kRows) t[i] = make_uint2(i, ~i);
}

template <int MODE>
void run(int blocks, int iters, const uint2* tab, unsigned long long* d) {
    (void)hipMemset(d, 0, 32);
    hipLaunchKernelGGL((probe<MODE>), dim3(blocks), dim3(256), 0, 0, iters, tab, d);
    const hipError_t e = hipDeviceSynchronize();
    unsigned long long h[4];
    (void)hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
    static const char* nm[] = {"hipcc global_load_dwordx2 (64-bit address)",
                               "asm: xor -> lshl_add_u64 -> global_load dst==addr",
                               "hipcc buffer_load_dwordx2 (32-bit offset)"};
    printf("%-50s %s: lanes 0-15 %llu, 16-31 %llu, 32-47 %llu, 48-63 %llu wrong rows / %llu\n", nm[MODE],
           hipGetErrorString(e), h[0], h[1], h[2], h[3], (unsigned long long)blocks * 256ull * iters * 16ull);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 4096;
    const int iters = argc > 2 ? atoi(argv[2]) : 50;
    const int reps = argc > 3 ? atoi(argv[3]) : 3;
    uint2* tab;
    unsigned long long* d;
    (void)hipMalloc(&tab, (size_t)kRows * 8);
    (void)hipMalloc(&d, 32);
    hipLaunchKernelGGL(fill, dim3(kRows / 256), dim3(256), 0, 0, tab);
    for (int r = 0; r < reps; ++r) {
        run<0>(blocks, iters, tab, d);
        run<1>(blocks, iters, tab, d);
        run<2>(blocks, iters, tab, d);
    }
    (void)hipFree(tab);
    (void)hipFree(d);
    return 0;
}
