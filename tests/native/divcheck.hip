// Test-only: exhaustive check of rc::div_rn (raft-stereo_amd/csrc/common.h)
// against IEEE fp32 division on the device.  For every integer divisor b in
// [b_lo, b_hi] and every fp32 numerator a with 2^e_lo <= |a| < 2^e_hi (both
// signs, every mantissa), counts the a for which div_rn(a, b) differs bitwise
// from a / b and records the first such (b, a).  Built by the Makefile next to
// this file into _build/libdivcheck.so; driven by tests/test_div_rn.py.
#include "../../raft-stereo_amd/csrc/common.h"

namespace {

__global__ __launch_bounds__(256) void divcheck_kernel(int b_lo, int e_lo, int e_hi,
                                                       unsigned long long *count,
                                                       unsigned int *first) {
    const float b = (float)(b_lo + (int)blockIdx.y);
    const rc::DivRN d = rc::div_prep(b);
    // numerator bits: exponent field 127+e_lo .. 127+e_hi-1, every mantissa, both signs
    const unsigned int lo = (unsigned int)(127 + e_lo) << 23, hi = (unsigned int)(127 + e_hi) << 23;
    const unsigned int stride = gridDim.x * blockDim.x;
    unsigned int bad = 0;
    for (unsigned int m = lo + blockIdx.x * blockDim.x + threadIdx.x; m < hi; m += stride) {
#pragma unroll
        for (int sgn = 0; sgn < 2; ++sgn) {
            const unsigned int bits = m | ((unsigned int)sgn << 31);
            const float a = __builtin_bit_cast(float, bits);
            const float q_ieee = a / b;
            const float q_fast = rc::div_rn(a, d);
            if (__builtin_bit_cast(unsigned int, q_ieee) != __builtin_bit_cast(unsigned int, q_fast)) {
                if (bad == 0 && atomicCAS(&first[0], 0u, 1u) == 0u) {
                    first[1] = (unsigned int)(b_lo + (int)blockIdx.y);
                    first[2] = bits;
                }
                ++bad;
            }
        }
    }
    if (bad) atomicAdd(count, (unsigned long long)bad);
}

}  // namespace

// Returns 0 or a hipError_t; count[0] = mismatches, first = {flag, b, a bits}.
extern "C" int divcheck(int b_lo, int b_hi, int e_lo, int e_hi, unsigned long long *count,
                        unsigned int *first) {
    if (b_hi < b_lo || e_hi <= e_lo || e_lo < -126 || e_hi > 127) return (int)hipErrorInvalidValue;
    unsigned long long *dc;
    unsigned int *df;
    hipError_t e = hipMalloc(&dc, sizeof(*dc));
    if (e != hipSuccess) return (int)e;
    e = hipMalloc(&df, 3 * sizeof(*df));
    if (e != hipSuccess) { (void)hipFree(dc); return (int)e; }
    (void)hipMemset(dc, 0, sizeof(*dc));
    (void)hipMemset(df, 0, 3 * sizeof(*df));
    hipLaunchKernelGGL(divcheck_kernel, dim3(1024, b_hi - b_lo + 1), dim3(256), 0, 0, b_lo, e_lo,
                       e_hi, dc, df);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(count, dc, sizeof(*dc), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(first, df, 3 * sizeof(*df), hipMemcpyDeviceToHost);
    (void)hipFree(dc);
    (void)hipFree(df);
    return (int)e;
}
