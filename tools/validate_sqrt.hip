// validate_sqrt.hip — exhaustive test of the hardware square root (v_sqrt_f32) against
// the correctly rounded sqrtf that hipcc emits under -fhip-fp32-correctly-rounded-divide-sqrt,
// over all 2^31 non-negative bit patterns, by input class.  If v_sqrt_f32 alone is
// correctly rounded on a class, the render kernel may use it there (rtx_fastdiv.h).
// Build+run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         tools/validate_sqrt.hip -o /tmp/vs && /tmp/vs
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#ifndef FAST
#define FAST 0   // 1: validate sqrt_fast instead of the bare v_sqrt_f32
#endif

// classes: 0 zero, 1 denormal, 2 normal < 2^-96, 3 normal in [2^-96, 2^64), 4 normal >= 2^64, 5 inf
__device__ int cls(uint32_t u) {
    if (u == 0) return 0;
    if (u < 0x00800000u) return 1;
    if (u < (31u << 23)) return 2;        // 2^-96 = exponent field 31
    if (u < (191u << 23)) return 3;       // 2^64  = exponent field 191
    if (u < 0x7f800000u) return 4;
    return 5;
}

// The render kernel's fast path (rtx_fastdiv.h sqrt_rn): v_sqrt_f32 plus one residual
// correction, no scaling, valid where claimed below.
__device__ float sqrt_fast(float x) {
    float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = fmaf(-sm, s, x), rp = fmaf(-sp, s, x);
    s = (rm <= 0.f) ? sm : s;
    s = (rp > 0.f) ? sp : s;
    return s;
}

__global__ void k(unsigned long long* bad, unsigned long long* tested, unsigned* first) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long nb[6] = {0, 0, 0, 0, 0, 0}, nt[6] = {0, 0, 0, 0, 0, 0};
    for (uint64_t u = tid; u <= 0x7f800000ull; u += nthreads) {
        const float x = __uint_as_float(static_cast<uint32_t>(u));
        const int c = cls(static_cast<uint32_t>(u));
        const float ref = sqrtf(x);
        const float got = FAST ? sqrt_fast(x) : __builtin_amdgcn_sqrtf(x);
        ++nt[c];
        if (__float_as_uint(ref) != __float_as_uint(got)) {
            ++nb[c];
            atomicMin(first + c, static_cast<uint32_t>(u));
        }
    }
    for (int c = 0; c < 6; ++c) {
        if (nb[c]) atomicAdd(bad + c, nb[c]);
        if (nt[c]) atomicAdd(tested + c, nt[c]);
    }
}

int main() {
    // device memory (atomics on managed/host memory cross PCIe: far too slow here)
    unsigned long long *d_bad, *d_tested, bad[6], tested[6];
    unsigned *d_first, first[6];
    if (hipMalloc(&d_bad, 6 * 8) != hipSuccess || hipMalloc(&d_tested, 6 * 8) != hipSuccess ||
        hipMalloc(&d_first, 6 * 4) != hipSuccess || hipMemset(d_bad, 0, 48) != hipSuccess ||
        hipMemset(d_tested, 0, 48) != hipSuccess || hipMemset(d_first, 0xff, 24) != hipSuccess)
        return 1;
    hipLaunchKernelGGL(k, dim3(4096), dim3(256), 0, 0, d_bad, d_tested, d_first);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(bad, d_bad, 48, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(tested, d_tested, 48, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(first, d_first, 24, hipMemcpyDeviceToHost) != hipSuccess)
        return 1;
    const char* names[6] = {"zero", "denormal", "normal < 2^-96", "normal [2^-96, 2^64)", "normal >= 2^64", "inf"};
    for (int c = 0; c < 6; ++c)
        std::printf("%s %-22s tested %12llu  mismatches %12llu  first 0x%08x\n", FAST ? "sqrt_fast" : "v_sqrt_f32",
                    names[c], tested[c], bad[c],
                    first[c]);
    return 0;
}
