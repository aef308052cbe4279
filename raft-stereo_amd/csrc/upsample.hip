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
// One lane per (n, h, i, w): the f outputs of sub-row i of low-resolution
// pixel (h, w).  Consecutive lanes take consecutive w, so each of the 9 f
// mask loads of a lane is part of one contiguous 256-B wave access, every
// mask element is read once, and the f outputs go out as one vector store
// (f = 4: 16 B per lane, 1 KB per wave).  The 3x3 flow neighbourhood is
// loaded once per lane.  HBM-bound: 4 (9 f^2 + C + f^2 C) bytes per
// low-resolution pixel.
#include "common.h"

namespace rc {

template <int F>
__device__ __forceinline__ void store_row(float *dst, const float (&v)[F]) {
    if constexpr (F == 4) {
        *reinterpret_cast<f32x4 *>(dst) = f32x4{v[0], v[1], v[2], v[3]};
    } else if constexpr (F == 8) {
        *reinterpret_cast<f32x4 *>(dst) = f32x4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4 *>(dst + 4) = f32x4{v[4], v[5], v[6], v[7]};
    } else if constexpr (F == 2) {
        *reinterpret_cast<f32x2 *>(dst) = f32x2{v[0], v[1]};
    } else {
        dst[0] = v[0];
    }
}

template <int F>
__global__ __launch_bounds__(256) void convex_upsample_kernel(const float *__restrict__ flow,
                                                              const float *__restrict__ mask,
                                                              float *__restrict__ out, int N, int C,
                                                              int H, int W, long long total) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;   // no barriers in this kernel
    const int w = (int)(idx % W);
    long long t = idx / W;
    const int i = (int)(t % F);
    t /= F;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    const long long HW = (long long)H * W;
    const long long WO = (long long)W * F, per_img = (long long)H * F * WO;
    const float *m = mask + ((long long)n * 9 * F * F + i * F) * HW + (long long)h * W + w;
    // softmax weights of the f sub-pixels (i, j), j = 0..f-1
    float wt[F][9];
#pragma unroll
    for (int j = 0; j < F; ++j) {
        float mx = -INFINITY;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            wt[j][k] = m[((long long)k * F * F + j) * HW];
            mx = fmaxf(mx, wt[j][k]);
        }
        float sum = 0.0f;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            wt[j][k] = expf(wt[j][k] - mx);
            sum += wt[j][k];
        }
        const float inv = 1.0f / sum;
#pragma unroll
        for (int k = 0; k < 9; ++k) wt[j][k] *= inv;
    }
    for (int c = 0; c < C; ++c) {
        const float *fl = flow + ((long long)n * C + c) * HW;
        float nb[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int yy = h + k / 3 - 1, xx = w + k % 3 - 1;
            nb[k] = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? (float)F * fl[(long long)yy * W + xx] : 0.0f;
        }
        float o[F];
#pragma unroll
        for (int j = 0; j < F; ++j) {
            float acc = 0.0f;
#pragma unroll
            for (int k = 0; k < 9; ++k) acc = fmaf(wt[j][k], nb[k], acc);
            o[j] = acc;
        }
        store_row<F>(out + ((long long)n * C + c) * per_img + (long long)(h * F + i) * WO + (long long)w * F, o);
    }
}

}  // namespace rc

hipError_t rc_launch_convex_upsample(const float *flow, const float *mask, int N, int C, int H,
                                     int W, int factor, float *out, hipStream_t s) {
    const long long total = (long long)N * H * W * factor;   // lanes: (n, h, i, w)
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
