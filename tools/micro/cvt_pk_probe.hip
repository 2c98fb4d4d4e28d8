// Semantics probe (developer tool): v_cvt_pk_f16_f32 vs (_Float16) casts and v_cvt_pkrtz_f16_f32.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
__global__ void k(const float* x, uint32_t* pk, uint32_t* rtz, uint32_t* ref, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float a = x[2 * i], b = x[2 * i + 1];
    uint32_t r;
    asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    pk[i] = r;
    rtz[i] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(a, b));
    _Float16 ha = (_Float16)a, hb = (_Float16)b;
    ref[i] = (uint32_t)__builtin_bit_cast(uint16_t, ha) | ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}
int main() {
    const int n = 1 << 20;
    std::vector<float> x(2 * n);
    srand(1);
    for (int i = 0; i < 2 * n; ++i) {
        float m = (float)rand() / RAND_MAX * 2 - 1;
        int e = rand() % 40 - 30;
        x[i] = ldexpf(m, e);
    }
    float* dx; uint32_t *a, *b, *c;
    hipMalloc(&dx, 8 * n); hipMalloc(&a, 4 * n); hipMalloc(&b, 4 * n); hipMalloc(&c, 4 * n);
    hipMemcpy(dx, x.data(), 8 * n, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dx, a, b, c, n);
    std::vector<uint32_t> A(n), B(n), Cc(n);
    hipMemcpy(A.data(), a, 4 * n, hipMemcpyDeviceToHost);
    hipMemcpy(B.data(), b, 4 * n, hipMemcpyDeviceToHost);
    hipMemcpy(Cc.data(), c, 4 * n, hipMemcpyDeviceToHost);
    long pk_ne = 0, rtz_ne = 0, swapped = 0;
    for (int i = 0; i < n; ++i) {
        pk_ne += A[i] != Cc[i];
        rtz_ne += B[i] != Cc[i];
        swapped += ((A[i] >> 16) | (A[i] << 16)) == Cc[i] && A[i] != Cc[i];
    }
    printf("cvt_pk != RNE casts: %ld / %d (swapped halves: %ld); pkrtz != RNE casts: %ld\n", pk_ne, n, swapped, rtz_ne);
    for (int i = 0; i < n && pk_ne; ++i)
        if (A[i] != Cc[i]) { printf("example a=%g b=%g pk=%08x ref=%08x\n", x[2 * i], x[2 * i + 1], A[i], Cc[i]); break; }
    return 0;
}
