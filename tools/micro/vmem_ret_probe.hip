// VMEM return probe (developer tool): is every lane of a gather visible to the VALU right after a
// PARTIAL s_waitcnt vmcnt(N) that covers it, while later gathers are still in flight?  The hash encoding issues
// two levels of 8 gathers (16 in flight), waits vmcnt(8) for the first level and copies its data at once.  Here:
// the tested gather first, then M more (random rows of a 64 MiB table whose row i holds i), s_waitcnt vmcnt(M),
// and the tested data read by a v_mov in the next instruction (GAP wait states).  Wrong values per quarter.
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/vmem_ret_probe.hip -o tools/micro/vmem_ret_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define PAD16 "s_nop 7\n\ts_nop 7\n\t"
#define LD(D, OFF) "global_load_dwordx2 v[" #D ":" #D "+1], v[46:47], off offset:" #OFF "\n\t"
#define BURST7 "global_load_dwordx2 v[50:51], v[46:47], off\n\tglobal_load_dwordx2 v[52:53], v[46:47], off offset:2048\n\t" \
    "global_load_dwordx2 v[54:55], v[46:47], off offset:-2048\n\tglobal_load_dwordx2 v[56:57], v[46:47], off offset:4088\n\t" \
    "global_load_dwordx2 v[58:59], v[48:49], off\n\tglobal_load_dwordx2 v[60:61], v[48:49], off offset:2048\n\t" \
    "global_load_dwordx2 v[62:63], v[48:49], off offset:-2048\n\t"
#define BURST8B "global_load_dwordx2 v[64:65], v[48:49], off offset:4088\n\t" \
    "global_load_dwordx2 v[66:67], v[46:47], off offset:1024\n\tglobal_load_dwordx2 v[68:69], v[46:47], off offset:3072\n\t" \
    "global_load_dwordx2 v[70:71], v[46:47], off offset:-1024\n\tglobal_load_dwordx2 v[72:73], v[46:47], off offset:-3072\n\t" \
    "global_load_dwordx2 v[74:75], v[48:49], off offset:1024\n\tglobal_load_dwordx2 v[76:77], v[48:49], off offset:3072\n\t" \
    "global_load_dwordx2 v[78:79], v[48:49], off offset:-1024\n\t"
#define CLOBR "v40", "v41", "v42", "v43", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", \
              "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", \
              "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81"
// the tested gather into v[42:43] first; M later gathers; wait vmcnt(M); copy at once (or after 16 states)
#define RET_ASM(LATER, WAIT, GAP)                                                                  \
    asm volatile("v_mov_b32 v40, %1\n\tv_mov_b32 v41, %2\n\tv_mov_b32 v46, %3\n\tv_mov_b32 v47, %4\n\t" \
                 "v_mov_b32 v48, %5\n\tv_mov_b32 v49, %6\n\tv_mov_b32 v42, -1\n\tv_mov_b32 v43, -1\n\t" PAD16 \
                 "global_load_dwordx2 v[42:43], v[40:41], off\n\t" LATER WAIT GAP                   \
                 "v_mov_b32 v80, v42\n\tv_mov_b32 v81, v43\n\ts_waitcnt vmcnt(0)\n\tv_mov_b32 %0, v80\n\t" \
                 : "=&v"(r)                                                                         \
                 : "v"((uint32_t)pa), "v"((uint32_t)(pa >> 32)), "v"((uint32_t)p1), "v"((uint32_t)(p1 >> 32)), \
                   "v"((uint32_t)p2), "v"((uint32_t)(p2 >> 32))                                       \
                 : CLOBR, "memory")

__device__ __forceinline__ uint32_t hsh(uint32_t v) {
    v ^= v >> 16; v *= 0x7feb352dU; v ^= v >> 15; v *= 0x846ca68bU; v ^= v >> 16;
    return v;
}

constexpr uint32_t kRows = 1u << 23;   // 64 MiB of 8-byte rows

template <int M, int G>
__global__ void __launch_bounds__(256) probe(int iters, const uint2* __restrict__ tab, unsigned long long* bad) {
    const int lane = threadIdx.x & 63;
    unsigned long long nb[4] = {0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
        const uint32_t s = hsh((uint32_t)(blockIdx.x * 256 + threadIdx.x) * 7919u + (uint32_t)it * 104729u);
        const uint32_t ia = s & (kRows - 1);
        const uint32_t i1 = (hsh(s + 1) & (kRows - 1)) | 512u, i2 = (hsh(s + 2) & (kRows - 1)) | 512u;
        const uint64_t pa = (uint64_t)(uintptr_t)(tab + ia);
        const uint64_t p1 = (uint64_t)(uintptr_t)(tab + (i1 < kRows - 512 ? i1 : kRows - 512));
        const uint64_t p2 = (uint64_t)(uintptr_t)(tab + (i2 < kRows - 512 ? i2 : kRows - 512));
        uint32_t r;
        if constexpr (M == 7) {
            if constexpr (G == 0) RET_ASM(BURST7, "s_waitcnt vmcnt(7)\n\t", "");
            else RET_ASM(BURST7, "s_waitcnt vmcnt(7)\n\t", PAD16);
        } else if constexpr (M == 15) {
            if constexpr (G == 0) RET_ASM(BURST7 BURST8B, "s_waitcnt vmcnt(15)\n\t", "");
            else RET_ASM(BURST7 BURST8B, "s_waitcnt vmcnt(15)\n\t", PAD16);
        } else {
            if constexpr (G == 0) RET_ASM("", "s_waitcnt vmcnt(0)\n\t", "");
            else RET_ASM("", "s_waitcnt vmcnt(0)\n\t", PAD16);
        }
        if (r != ia) ++nb[lane >> 4];
    }
    for (int q = 0; q < 4; ++q)
        if (nb[q]) atomicAdd(bad + q, nb[q]);
}

template <int M, int G>
void run(int blocks, int iters, const uint2* tab, unsigned long long* d) {
    hipMemset(d, 0, 32);
    hipLaunchKernelGGL((probe<M, G>), dim3(blocks), dim3(256), 0, 0, iters, tab, d);
    unsigned long long h[4];
    hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
    printf("%2d later gathers, s_waitcnt vmcnt(%2d), data read %2d states after: lanes 0-15 %llu, 16-31 %llu, "
           "32-47 %llu, 48-63 %llu wrong / %llu lane-iterations\n", M, M, G ? 16 : 0, h[0], h[1], h[2], h[3],
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
    for (int rep = 0; rep < 3; ++rep) {
        run<0, 0>(blocks, iters, tab, d);
        run<7, 0>(blocks, iters, tab, d);
        run<7, 1>(blocks, iters, tab, d);
        run<15, 0>(blocks, iters, tab, d);
        run<15, 1>(blocks, iters, tab, d);
    }
    hipFree(tab);
    hipFree(d);
    return 0;
}
