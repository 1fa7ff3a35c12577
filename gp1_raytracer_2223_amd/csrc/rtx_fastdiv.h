// rtx_fastdiv.h — cheap correctly rounded binary32 reciprocal / quotient for gfx950.
//
// hipcc's IEEE division a/b expands to ~11 VALU ops (v_div_scale x2, v_rcp, 4-5 FMAs,
// v_div_fmas, v_div_fixup) because it must handle every range.  Inside a checked domain
// the classic Markstein sequence gives the same correctly rounded result in 3 + 3 ops:
//   y  = v_rcp_f32(b);  e = fma(-b, y, 1);  y = fma(e, y, y)   -> RN(1/b)
//   q  = a * y;         r = fma(-b, q, a);  q = fma(r, y, q)    -> RN(a/b)
// RN(1/b) is verified EXHAUSTIVELY on the hardware for every b in the domain
// (tools/validate_fastdiv.hip, all 2^32 inputs), and the quotient step is Markstein's
// theorem (y = RN(1/b), q0 within 1 ulp, exact residual by FMA) — additionally checked
// on 2^33 random and near-halfway pairs by the same tool.  Lanes outside the domain
// (zeros, tiny or huge magnitudes, inf, NaN) take the IEEE `/` in a divergent branch that
// is skipped whenever no lane needs it.
#pragma once
#include <hip/hip_runtime.h>

namespace rtxd {

// |b| in [2^-60, 2^60]: RN(1/b) and every intermediate stay normal.
__device__ __forceinline__ bool fast_rcp_ok(float b) {
    const float ab = fabsf(b);
    return ab >= 0x1p-60f && ab <= 0x1p60f;
}

__device__ __forceinline__ float rcp_rn(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float e = fmaf(-b, y0, 1.0f);
    return fmaf(e, y0, y0);
}

// a == 0 or |a| in [2^-60, 2^60], and fast_rcp_ok(b): quotient in [2^-120, 2^120] and the
// residual a - b*q is exactly representable (granularity >= 2^-106).
__device__ __forceinline__ bool fast_num_ok(float a) {
    const float aa = fabsf(a);
    return (aa >= 0x1p-60f && aa <= 0x1p60f) || a == 0.0f;
}

__device__ __forceinline__ bool fast_div_ok(float a, float b) { return fast_num_ok(a) && fast_rcp_ok(b); }

// RN(a/b) given y = rcp_rn(b), inside the domain above.
__device__ __forceinline__ float div_rn(float a, float b, float y) {
    const float q = a * y;
    const float r = fmaf(-b, q, a);
    return fmaf(r, y, q);
}

// RN(1/b) for every b.
__device__ __forceinline__ float rcp_exact(float b) {
    float y = rcp_rn(b);
    if (__builtin_expect(!fast_rcp_ok(b), 0)) y = 1.f / b;
    return y;
}

// RN(1/x), RN(1/y), RN(1/z) with ONE domain test for the three: the IEEE fallback runs
// only in lanes where some component is outside.  Returns the ballot of those lanes.  In
// the domain every reciprocal is finite and non-zero, which is what the FAST slab path
// needs, so the ballot doubles as its (conservative) exclusion mask.  The magnitude sum
// carries a NaN or inf component into the test (v_min3 would drop a NaN).
__device__ __forceinline__ unsigned long long rcp3_exact(float x, float y, float z, float& rx, float& ry, float& rz) {
    rx = rcp_rn(x); ry = rcp_rn(y); rz = rcp_rn(z);
    const float lo = fminf(fminf(fabsf(x), fabsf(y)), fabsf(z));
    const float sum = (fabsf(x) + fabsf(y)) + fabsf(z);
    const bool in = lo >= 0x1p-60f && sum <= 0x1p60f;
    const unsigned long long out = __builtin_amdgcn_ballot_w64(!in);
    if (__builtin_expect(!in, 0)) {
        rx = 1.f / x; ry = 1.f / y; rz = 1.f / z;
    }
    return out;
}

// (x, y, z) / m, each correctly rounded, for m = |(x, y, z)| as computed by the caller.
__device__ __forceinline__ void div3_exact(float& x, float& y, float& z, float m) {
    const float r = rcp_rn(m);
    const float qx = div_rn(x, m, r), qy = div_rn(y, m, r), qz = div_rn(z, m, r);
    // a NaN component (dropped by v_min) gives NaN on both paths; inf makes m inf -> IEEE
    const float lo = fminf(fminf(fabsf(x), fabsf(y)), fabsf(z));
    if (__builtin_expect(!(fast_rcp_ok(m) && lo >= 0x1p-60f), 0)) {
        x = x / m; y = y / m; z = z / m;
    } else {
        x = qx; y = qy; z = qz;
    }
}

}  // namespace rtxd
