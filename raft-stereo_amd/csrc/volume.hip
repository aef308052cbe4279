// Correlation volume + fused pyramid epilogue, fp32 MFMA (gfx950).
//
// Replaces CorrBlock1D.corr (/root/reference/model.py:318-326) and the
// avg_pool2d loop of CorrBlock1D.__init__ (:284-295).
//
// Per (b,h) image row the volume is a GEMM  C[w1][w2] = sum_d F1[d][w1] F2[d][w2]
// with K = D.  F1/F2 are NCHW, so for a fixed row both operands are "K-major":
// row d of the operand is W contiguous floats.  v_mfma_f32_16x16x4_f32 takes
// one f32 per lane for A and for B: lane l supplies A[i=l&15][k=l>>4] and
// B[k=l>>4][j=l&15].  A lane loads one float4 along w (16 B, so 16 lanes cover
// 256 contiguous bytes of one d-row and the wave 4 d-rows): component c of that
// float4 is the operand of the c-th of four 16-wide fragments whose rows are
// w = w0 + 4*i + c.  The output is therefore "4-interleaved": fragment (ma,nb)
// register r of lane l holds C[m0 + 4*((l>>4)*4+r) + ma][n0 + 4*(l&15) + nb].
// Each lane thus owns 4 consecutive w2 of a row, which makes the first two
// pooling steps lane-local and the next ones xor-shuffles (l^1, l^2, ...).
//
// Workgroup: 256 threads = 4 waves in a 2x2 arrangement of 64x64 wave tiles
// (a 128x128 tile of one row's volume).  Workgroups are remapped so that all
// tiles of one (b,h) row run on one XCD (blocks b, b+8, ... share an XCD) and
// share that XCD's L2 copy of the row's feature maps.
#include "common.h"

namespace rc {

// Fragment loads: float4 along w at (d, w) of one (b) image, or zero when
// d >= D (offset pushed out of the buffer's range).
template <bool VEC>
__device__ __forceinline__ f32x4 load_frag(__amdgpu_buffer_rsrc_t r, int d, int D, int H, int h,
                                           int W, int w) {
    uint32_t off = (uint32_t)(((long long)(d * H + h) * W + w) * 4);
    if (d >= D) off = 0xFFFFFFF0u;
    if constexpr (VEC) {
        return ld4(r, off);
    } else {
        f32x4 v;
        v.x = ld1(r, off);
        v.y = ld1(r, off + 4);
        v.z = ld1(r, off + 8);
        v.w = ld1(r, off + 12);
        return v;
    }
}

__device__ __forceinline__ void store_level(void *lvl, int bf16, long long idx, float v) {
    if (bf16)
        reinterpret_cast<uint16_t *>(lvl)[idx] = f32_to_bf16(v);
    else
        reinterpret_cast<float *>(lvl)[idx] = v;
}

template <bool VEC>
__global__ __launch_bounds__(256) void build_f32_kernel(BuildArgs a) {
    // XCD-aware bijective remap (cdna_hip_programming.md §5, "XCD swizzle").
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
    const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
    const int T = a.tiles_m * a.tiles_n;
    const int row = wgid / T, tile = wgid - row * T;
    const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
    const int b = row / a.H, h = row - b * a.H;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int m0 = tm * 128 + (wave >> 1) * 64;
    const int n0 = tn * 128 + (wave & 1) * 64;
    if (m0 >= a.W1 || n0 >= a.W2) return;  // wave-uniform; no barriers below

    const int D = a.D, H = a.H, W1 = a.W1, W2 = a.W2;
    const long long img1 = (long long)D * H * W1, img2 = (long long)D * H * W2;
    const auto r1 = make_rsrc(reinterpret_cast<const float *>(a.f1) + b * img1, clamp_bytes(img1 * 4));
    const auto r2 = make_rsrc(reinterpret_cast<const float *>(a.f2) + b * img2, clamp_bytes(img2 * 4));

    const int kd = lane >> 4;                  // d offset inside a k-step
    const int wa = m0 + 4 * (lane & 15);       // this lane's w1 quad
    const int wb = n0 + 4 * (lane & 15);       // this lane's w2 quad

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    constexpr int U = 4;  // k-steps (of 4) per pipeline stage
    const int ksteps = (D + 3) >> 2;
    f32x4 An[U], Bn[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        An[u] = load_frag<VEC>(r1, 4 * u + kd, D, H, h, W1, wa);
        Bn[u] = load_frag<VEC>(r2, 4 * u + kd, D, H, h, W2, wb);
    }
    for (int ks = 0; ks < ksteps; ks += U) {
        f32x4 Ac[U], Bc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { Ac[u] = An[u]; Bc[u] = Bn[u]; }
        if (ks + U < ksteps) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                An[u] = load_frag<VEC>(r1, 4 * (ks + U + u) + kd, D, H, h, W1, wa);
                Bn[u] = load_frag<VEC>(r2, 4 * (ks + U + u) + kd, D, H, h, W2, wb);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (ks + u < ksteps) {
#pragma unroll
                for (int ma = 0; ma < 4; ++ma)
#pragma unroll
                    for (int nb = 0; nb < 4; ++nb)
                        acc[ma][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(Ac[u][ma], Bc[u][nb],
                                                                           acc[ma][nb], 0, 0, 0);
            }
        }
    }

    // ---- epilogue: scale, level 0, fused pooling (model.py:294) ----
    const long long rowbase = (long long)row * W1;  // pyramid row of w1 = 0
    const int col = lane & 15;
    const bool bf = a.pyr_bf16 != 0;
#pragma unroll
    for (int ma = 0; ma < 4; ++ma) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int w1 = m0 + 4 * ((lane >> 4) * 4 + r) + ma;
            const bool rv = w1 < W1;
            const long long p = rowbase + w1;
            float c[4];
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) {
                const float v = acc[ma][nb][r];
                c[nb] = a.pow2 ? v * a.scale : v / a.sq;
            }
            // level 0
            if (rv) {
                if (!bf && VEC && wb + 3 < W2) {
                    *reinterpret_cast<f32x4 *>(reinterpret_cast<float *>(a.lvl[0]) + p * W2 + wb) =
                        f32x4{c[0], c[1], c[2], c[3]};
                } else {
#pragma unroll
                    for (int nb = 0; nb < 4; ++nb)
                        if (wb + nb < W2) store_level(a.lvl[0], bf, p * W2 + wb + nb, c[nb]);
                }
            }
            if (a.nfused < 2) continue;
            // level 1: lane-local pairs
            const float e0 = (c[0] + c[1]) * 0.5f, e1 = (c[2] + c[3]) * 0.5f;
            {
                const int Wl = W2 >> 1, j = wb >> 1;
                if (rv) {
                    if (j < Wl) store_level(a.lvl[1], bf, p * Wl + j, e0);
                    if (j + 1 < Wl) store_level(a.lvl[1], bf, p * Wl + j + 1, e1);
                }
            }
            if (a.nfused < 3) continue;
            // level 2: lane-local
            float f = (e0 + e1) * 0.5f;
            {
                const int Wl = W2 >> 2, j = wb >> 2;
                if (rv && j < Wl) store_level(a.lvl[2], bf, p * Wl + j, f);
            }
            // levels 3..6: xor-shuffle across the 16 lanes of this row group
#pragma unroll
            for (int l = 3; l < 7; ++l) {
                if (a.nfused <= l) break;                 // wave-uniform
                const int m = 1 << (l - 3);               // lane distance
                const float o = __shfl_xor(f, m);
                f = (f + o) * 0.5f;
                const int Wl = W2 >> l, j = wb >> l;
                if (rv && (col & (2 * m - 1)) == 0 && j < Wl)
                    store_level(a.lvl[l], bf, p * Wl + j, f);
            }
        }
    }
}

}  // namespace rc

hipError_t rc_launch_build_f32(const rc::BuildArgs &a, hipStream_t s) {
    const long long nwg = (long long)a.B * a.H * a.tiles_m * a.tiles_n;
    if (nwg <= 0) return hipSuccess;
    if (nwg > 0x7FFFFFFF) return hipErrorInvalidValue;
    const bool vec = (a.W1 % 4 == 0) && (a.W2 % 4 == 0);
    if (vec)
        hipLaunchKernelGGL(rc::build_f32_kernel<true>, dim3((unsigned)nwg), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(rc::build_f32_kernel<false>, dim3((unsigned)nwg), dim3(256), 0, s, a);
    return hipGetLastError();
}
