// Convex upsampling of the low-resolution flow (gfx950), SURVEY.md §8f rank 3.
//
// The reference's update block already produces the upsampling mask
// (model.py:238-241, scaled by 0.25 at :264): (f^2)*9 channels per
// low-resolution pixel, f = 2^n_downsample (:236).  Its truncated forward
// never consumes it.  RAFT-Stereo's convex upsampler
// turns the mask into softmax weights over the 3x3 neighbourhood of every
// low-resolution pixel and combines f * flow there:
//     up[n][c][f h + i][f w + j] =
//         sum_k softmax_k(mask[n][k f^2 + i f + j][h][w]) * f * flow[n][c][h + dy_k][w + dx_k]
// with k = 3 (dy + 1) + (dx + 1) (F.unfold's row-major 3x3 order) and zeros
// outside the image.  Parity is checked against oracle/torch_ref.py's
// restatement (F.unfold + softmax); the reference has no upsampler to pin it.
//
// One lane per output pixel: consecutive lanes walk the output row, so the
// stores are coalesced and each mask plane is read in runs of w at fixed
// (i, j).  Every mask element is read by exactly one lane; the 3x3 flow
// neighbourhood is shared by f^2 lanes through the L1/L2.  HBM-bound:
// 4 (9 f^2 + C + f^2 C) bytes per low-resolution pixel.
#include "common.h"

namespace rc {

template <int F>
__global__ __launch_bounds__(256) void convex_upsample_kernel(const float *__restrict__ flow,
                                                              const float *__restrict__ mask,
                                                              float *__restrict__ out, int N, int C,
                                                              int H, int W, long long total) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;   // no barriers in this kernel
    const int WO = W * F, HO = H * F;
    const long long per_img = (long long)HO * WO;
    const int n = (int)(idx / per_img);
    const long long rem = idx - (long long)n * per_img;
    const int Y = (int)(rem / WO), X = (int)(rem - (long long)Y * WO);
    const int h = Y / F, i = Y - h * F, w = X / F, j = X - w * F;
    const long long HW = (long long)H * W;
    const float *m = mask + ((long long)n * 9 * F * F + i * F + j) * HW + (long long)h * W + w;
    float e[9];
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        e[k] = m[(long long)k * F * F * HW];
        mx = fmaxf(mx, e[k]);
    }
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        e[k] = expf(e[k] - mx);
        sum += e[k];
    }
    const float inv = 1.0f / sum;
    for (int c = 0; c < C; ++c) {
        const float *fl = flow + ((long long)n * C + c) * HW;
        float acc = 0.0f;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int yy = h + k / 3 - 1, xx = w + k % 3 - 1;
            const float v = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? fl[(long long)yy * W + xx] : 0.0f;
            acc = fmaf(e[k] * inv, (float)F * v, acc);
        }
        out[((long long)n * C + c) * per_img + rem] = acc;
    }
}

}  // namespace rc

hipError_t rc_launch_convex_upsample(const float *flow, const float *mask, int N, int C, int H,
                                     int W, int factor, float *out, hipStream_t s) {
    const long long total = (long long)N * H * W * factor * factor;
    if (total <= 0) return hipSuccess;
    const unsigned nblk = (unsigned)((total + 255) / 256);
    switch (factor) {
        case 1: hipLaunchKernelGGL(rc::convex_upsample_kernel<1>, dim3(nblk), dim3(256), 0, s, flow, mask, out, N, C, H, W, total); break;
        case 2: hipLaunchKernelGGL(rc::convex_upsample_kernel<2>, dim3(nblk), dim3(256), 0, s, flow, mask, out, N, C, H, W, total); break;
        case 4: hipLaunchKernelGGL(rc::convex_upsample_kernel<4>, dim3(nblk), dim3(256), 0, s, flow, mask, out, N, C, H, W, total); break;
        case 8: hipLaunchKernelGGL(rc::convex_upsample_kernel<8>, dim3(nblk), dim3(256), 0, s, flow, mask, out, N, C, H, W, total); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
