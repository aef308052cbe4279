// One standalone pyramid step (model.py:294, F.avg_pool2d([1,2],[1,2])):
// out[p][j] = (in[p][2j] + in[p][2j+1]) / 2 for j < floor(W_in/2).
// Used for levels beyond the build kernel's fused epilogue and for A/B runs.
// HBM-bound: one thread per output element, grid-stride.
#include "common.h"

namespace rc {

template <bool BF16>
__global__ __launch_bounds__(256) void pool_kernel(const void *in, long long ld_in, void *out,
                                                   long long ld_out, long long rows, int W_in) {
    const int Wo = W_in >> 1;
    const long long n = rows * Wo;
    for (long long k = (long long)blockIdx.x * 256 + threadIdx.x; k < n;
         k += (long long)gridDim.x * 256) {
        const long long p = k / Wo, j = k - p * Wo;
        const long long src = p * ld_in + 2 * j, dst = p * ld_out + j;
        if constexpr (BF16) {
            const uint16_t *ip = reinterpret_cast<const uint16_t *>(in);
            const float s = bf16_to_f32(ip[src]) + bf16_to_f32(ip[src + 1]);
            reinterpret_cast<uint16_t *>(out)[dst] = f32_to_bf16(s * 0.5f);
        } else {
            const float *ip = reinterpret_cast<const float *>(in);
            const float s = ip[src] + ip[src + 1];
            reinterpret_cast<float *>(out)[dst] = s * 0.5f;
        }
    }
}

}  // namespace rc

hipError_t rc_launch_pool(const void *in, long long ld_in, void *out, long long ld_out, long rows,
                          int W_in, int bf16, hipStream_t s) {
    const long long n = (long long)rows * (W_in >> 1);
    if (n <= 0) return hipSuccess;
    long long blocks = (n + 255) / 256;
    if (blocks > 256 * 8) blocks = 256 * 8;
    if (bf16)
        hipLaunchKernelGGL(rc::pool_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, in, ld_in,
                           out, ld_out, (long long)rows, W_in);
    else
        hipLaunchKernelGGL(rc::pool_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, in, ld_in,
                           out, ld_out, (long long)rows, W_in);
    return hipGetLastError();
}
