// VMEM address write-after-read probe (developer tool).  hipcc reuses the address registers of a
// global_load the very next instruction after the load issues (547 such sites at 0 wait states in
// render_slots_kernel).  Does a gather always read all 64 lanes' addresses at issue, or can a VALU write that
// follows it change the address some lanes load from when the vector-memory path is backed up?
// Each lane gathers 8-byte rows of a 64 MiB table (row value = its index, so a wrong row shows) in a burst of
// B independent global_load_dwordx2, then the tested load whose address pair is overwritten by v_mov right after
// it issues (GAP wait states), then s_waitcnt.  Mismatches (tested load's value != its original row) per quarter.
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/vmem_war_probe.hip -o tools/micro/vmem_war_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define PAD16 "s_nop 7\n\ts_nop 7\n\t"
// v[40:41] = tested address, v[44:45] = other address; burst loads into v[50..] from v[46:47] + offsets
#define BURST8                                                                                     \
    "global_load_dwordx2 v[50:51], v[46:47], off\n\t"                                               \
    "global_load_dwordx2 v[52:53], v[46:47], off offset:2048\n\t"                                   \
    "global_load_dwordx2 v[54:55], v[46:47], off offset:-2048\n\t"                                  \
    "global_load_dwordx2 v[56:57], v[46:47], off offset:4088\n\t"                                   \
    "global_load_dwordx2 v[58:59], v[48:49], off\n\t"                                               \
    "global_load_dwordx2 v[60:61], v[48:49], off offset:2048\n\t"                                   \
    "global_load_dwordx2 v[62:63], v[48:49], off offset:-2048\n\t"                                  \
    "global_load_dwordx2 v[64:65], v[48:49], off offset:4088\n\t"
#define CLOBW "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", \
              "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65"
#define WAR_ASM(PRE, GAP)                                                                          \
    asm volatile("v_mov_b32 v40, %1\n\tv_mov_b32 v41, %2\n\tv_mov_b32 v44, %3\n\tv_mov_b32 v45, %4\n\t" \
                 "v_mov_b32 v46, %5\n\tv_mov_b32 v47, %6\n\tv_mov_b32 v48, %7\n\tv_mov_b32 v49, %8\n\t" PAD16 \
                 PRE "global_load_dwordx2 v[42:43], v[40:41], off\n\t" GAP                           \
                 "v_mov_b32 v40, v44\n\tv_mov_b32 v41, v45\n\t"                                     \
                 "s_waitcnt vmcnt(0)\n\tv_mov_b32 %0, v42\n\t"                                      \
                 : "=&v"(r)                                                                         \
                 : "v"((uint32_t)pa), "v"((uint32_t)(pa >> 32)), "v"((uint32_t)pb), "v"((uint32_t)(pb >> 32)), \
                   "v"((uint32_t)p1), "v"((uint32_t)(p1 >> 32)), "v"((uint32_t)p2), "v"((uint32_t)(p2 >> 32)) \
                 : CLOBW, "memory")

__device__ __forceinline__ uint32_t hsh(uint32_t v) {
    v ^= v >> 16; v *= 0x7feb352dU; v ^= v >> 15; v *= 0x846ca68bU; v ^= v >> 16;
    return v;
}

constexpr uint32_t kRows = 1u << 23;   // 64 MiB of 8-byte rows

template <int B, int G>
__global__ void __launch_bounds__(256) probe(int iters, const uint2* __restrict__ tab, unsigned long long* bad) {
    const int lane = threadIdx.x & 63;
    unsigned long long nb[4] = {0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
        const uint32_t s = hsh((uint32_t)(blockIdx.x * 256 + threadIdx.x) * 7919u + (uint32_t)it * 104729u);
        const uint32_t ia = s & (kRows - 1), ib = hsh(s) & (kRows - 1);
        const uint32_t i1 = (hsh(s + 1) & (kRows - 1)) | 512u, i2 = (hsh(s + 2) & (kRows - 1)) | 512u;
        const uint64_t pa = (uint64_t)(uintptr_t)(tab + ia), pb = (uint64_t)(uintptr_t)(tab + ib);
        const uint64_t p1 = (uint64_t)(uintptr_t)(tab + (i1 < kRows - 512 ? i1 : kRows - 512));
        const uint64_t p2 = (uint64_t)(uintptr_t)(tab + (i2 < kRows - 512 ? i2 : kRows - 512));
        uint32_t r;
        if constexpr (B == 0) {
            if constexpr (G == 0) WAR_ASM("", "");
            else WAR_ASM("", PAD16);
        } else if constexpr (B == 8) {
            if constexpr (G == 0) WAR_ASM(BURST8, "");
            else WAR_ASM(BURST8, PAD16);
        } else {
            if constexpr (G == 0) WAR_ASM(BURST8 BURST8, "");
            else WAR_ASM(BURST8 BURST8, PAD16);
        }
        if (r != ia) ++nb[lane >> 4];
    }
    for (int q = 0; q < 4; ++q)
        if (nb[q]) atomicAdd(bad + q, nb[q]);
}

template <int B, int G>
void run(int blocks, int iters, const uint2* tab, unsigned long long* d) {
    hipMemset(d, 0, 32);
    hipLaunchKernelGGL((probe<B, G>), dim3(blocks), dim3(256), 0, 0, iters, tab, d);
    unsigned long long h[4];
    hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
    printf("burst %2d loads, address overwritten %2d states after the load: lanes 0-15 %llu, 16-31 %llu, 32-47 %llu, "
           "48-63 %llu wrong / %llu lane-iterations\n", B, G ? 16 : 0, h[0], h[1], h[2], h[3],
           (unsigned long long)blocks * 256ull * (unsigned long long)iters);
    fflush(stdout);
}

__global__ void fill(uint2* t) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < kRows) t[i] = make_uint2(i, ~i);
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 4096;
    const int iters = argc > 2 ? atoi(argv[2]) : 100;
    uint2* tab;
    unsigned long long* d;
    hipMalloc(&tab, (size_t)kRows * 8);
    hipMalloc(&d, 32);
    hipLaunchKernelGGL(fill, dim3(kRows / 256), dim3(256), 0, 0, tab);
    run<0, 0>(blocks, iters, tab, d);
    run<0, 1>(blocks, iters, tab, d);
    run<8, 0>(blocks, iters, tab, d);
    run<8, 1>(blocks, iters, tab, d);
    run<16, 0>(blocks, iters, tab, d);
    run<16, 1>(blocks, iters, tab, d);
    hipFree(tab);
    hipFree(d);
    return 0;
}
