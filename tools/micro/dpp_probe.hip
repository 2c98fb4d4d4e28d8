// DPP probe (developer tool): the wave64 inclusive scan (row_shr + row_bcast) and the row-DPP +
// readlane reductions used by ray_order_kernel / mlp_train, checked against the host.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
__global__ void k(const int* x, int* scan, float* sum, float* mx, const float* f) {
    const int g = blockIdx.x * 64 + threadIdx.x;
    int incl = x[g];
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x111, 0xF, 0xF, true);
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x112, 0xF, 0xF, true);
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x114, 0xF, 0xF, true);
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x118, 0xF, 0xF, true);
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x142, 0xA, 0xF, false);
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x143, 0xC, 0xF, false);
    scan[g] = incl;
    float v = f[g], m = f[g];
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
    m = fmaxf(m, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(m), 0xB1, 0xF, 0xF, false)));
    m = fmaxf(m, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(m), 0x4E, 0xF, 0xF, false)));
    m = fmaxf(m, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(m), 0x141, 0xF, 0xF, false)));
    m = fmaxf(m, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(m), 0x140, 0xF, 0xF, false)));
    float s = 0.0f, M = -1e30f;
    for (int r = 0; r < 4; ++r) {
        s += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16 * r));
        M = fmaxf(M, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m), 16 * r)));
    }
    sum[g] = s;
    mx[g] = M;
}
int main() {
    const int W = 256, n = W * 64;
    std::vector<int> x(n);
    std::vector<float> f(n);
    srand(3);
    for (int i = 0; i < n; ++i) { x[i] = rand() % 100; f[i] = (float)(rand() % 1000) - 500.0f; }
    int *dx, *ds; float *dsum, *dmx, *df;
    (void)hipMalloc(&dx, 4 * n); (void)hipMalloc(&ds, 4 * n); (void)hipMalloc(&dsum, 4 * n);
    (void)hipMalloc(&dmx, 4 * n); (void)hipMalloc(&df, 4 * n);
    (void)hipMemcpy(dx, x.data(), 4 * n, hipMemcpyHostToDevice);
    (void)hipMemcpy(df, f.data(), 4 * n, hipMemcpyHostToDevice);
    k<<<W, 64>>>(dx, ds, dsum, dmx, df);
    std::vector<int> s(n); std::vector<float> su(n), mx(n);
    (void)hipMemcpy(s.data(), ds, 4 * n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(su.data(), dsum, 4 * n, hipMemcpyDeviceToHost);
    (void)hipMemcpy(mx.data(), dmx, 4 * n, hipMemcpyDeviceToHost);
    long bad_scan = 0, bad_sum = 0, bad_max = 0;
    for (int w = 0; w < W; ++w) {
        int run = 0; float tot = 0.0f, M = -1e30f;
        for (int l = 0; l < 64; ++l) { tot += f[w * 64 + l]; M = f[w * 64 + l] > M ? f[w * 64 + l] : M; }
        for (int l = 0; l < 64; ++l) {
            run += x[w * 64 + l];
            bad_scan += s[w * 64 + l] != run;
            bad_sum += su[w * 64 + l] != tot;  // integers in float: exact in any order
            bad_max += mx[w * 64 + l] != M;
        }
    }
    printf("scan mismatches %ld, sum mismatches %ld, max mismatches %ld (of %d)\n", bad_scan, bad_sum, bad_max, n);
    return (bad_scan || bad_sum || bad_max) ? 1 : 0;
}
