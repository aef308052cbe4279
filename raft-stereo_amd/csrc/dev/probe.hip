// Dev-only memory-pipeline probe (libraftcorr_dev.so only, tools/gather_probe.py).
//
// The lookup reads, per pixel, a few 16-B chunks at a random position of the
// pixel's own pyramid row: every lane of a wave instruction hits a different
// 128-B line.  This kernel reproduces that access shape without any tap math
// so its cost can be split into parts: per wave instruction, per lane request,
// per distinct line, per out-of-range (predicated-off) lane, and by where the
// lines are served from.
//
// Lane i of the grid (one "pixel") owns row i of a table of rows of `row`
// floats.  It issues K 16-B buffer loads:
//   mode 0 (span):   chunks start, start+1, ..., start+K-1 of its row (start
//                    a pseudo-random chunk index), like the chain lookup's span;
//   mode 1 (scatter): K chunks at pseudo-random positions of its row;
//   mode 2 (shared): lanes in groups of G read consecutive chunks of ONE row
//                    (row = i / G), so a group covers G*16 contiguous bytes
//                    per load (G = 8: one whole 128-B line per load);
// `oob` of the K loads get an out-of-range offset (the lookup's exact-span
// predication).  The lane writes the xor of everything it loaded, so no load
// is dead.  Rows are taken modulo `nrows` (nrows < lanes re-reads rows: a
// small table is cache-served).
#include "../common.h"

namespace rc {

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

template <int K>
__global__ __launch_bounds__(256) void gather_probe_kernel(const float *__restrict__ table, long long nrows,
                                                           int row, int mode, int G, int oob,
                                                           uint32_t seed, long long lanes,
                                                           float *__restrict__ out) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    const bool active = i < lanes;
    const long long li = active ? i : lanes - 1;
    const int cpr = row / 4;                                  // chunks per row
    long long r = (mode == 2 ? li / G : li) % nrows;
    const long long wbase = (long long)blockIdx.x * 256;      // block-relative rows keep offsets < 4 GB
    const long long rbase = (mode == 2 ? wbase / G : wbase) % nrows;
    if (r < rbase) r += nrows;                                // (r - rbase) >= 0
    const char *base = reinterpret_cast<const char *>(table) + rbase * (long long)row * 4;
    const long long span_rows = nrows - rbase;
    const auto rs = make_rsrc(base, clamp_bytes(span_rows * (long long)row * 4));
    const uint32_t h = hash32((uint32_t)li * 2654435761u + seed);
    int start = (int)(h % (uint32_t)(cpr - K + 1));
    if (mode == 2) start = (int)(hash32((uint32_t)(li / G) + seed) % (uint32_t)(cpr - K * G + 1)) + (int)(li % G);
    uint32_t acc = 0;
    f32x4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        int c;
        if (mode == 1) c = (int)(hash32(h + 77u * k) % (uint32_t)cpr);
        else if (mode == 2) c = start + k * G;
        else c = start + k;
        uint32_t off = (uint32_t)((((r - rbase) * (long long)row) + 4LL * c) * 4);
        if (k >= K - oob) off = 0xFFFFFF00u;
        v[k] = ld4(rs, off);
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc ^= __builtin_bit_cast(uint32_t, v[k][c]);
    if (active) out[i] = __builtin_bit_cast(float, acc);
}

}  // namespace rc

extern "C" int rc_dev_gather_probe(const float *table, long long nrows, int row, int mode, int G,
                                   int K, int oob, unsigned seed, long long lanes, float *out,
                                   void *stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const unsigned nblk = (unsigned)((lanes + 255) / 256);
    switch (K) {
        case 4: hipLaunchKernelGGL(rc::gather_probe_kernel<4>, dim3(nblk), dim3(256), 0, s, table, nrows, row, mode, G, oob, seed, lanes, out); break;
        case 8: hipLaunchKernelGGL(rc::gather_probe_kernel<8>, dim3(nblk), dim3(256), 0, s, table, nrows, row, mode, G, oob, seed, lanes, out); break;
        case 12: hipLaunchKernelGGL(rc::gather_probe_kernel<12>, dim3(nblk), dim3(256), 0, s, table, nrows, row, mode, G, oob, seed, lanes, out); break;
        case 16: hipLaunchKernelGGL(rc::gather_probe_kernel<16>, dim3(nblk), dim3(256), 0, s, table, nrows, row, mode, G, oob, seed, lanes, out); break;
        default: return 1;
    }
    return hipGetLastError() == hipSuccess ? 0 : 3;
}

// Alignment probe (dev only): what a 16-B buffer load returns at byte offsets
// 0, 2, 4, 6, 8 -- into VGPRs (mode 0), by LDS DMA (mode 1), and 4-B LDS DMA
// (mode 2).  One wave; lane l loads at offset 64*l + shift; out[l][4] dwords
// per shift.
namespace {
__global__ __launch_bounds__(64) void align_probe_kernel(const char *src, unsigned *out, int mode) {
    __shared__ __attribute__((aligned(16))) unsigned lds[5][64 * 4];
    typedef __attribute__((address_space(3))) void lds_void;
    const int lane = threadIdx.x;
    const auto r = rc::make_rsrc(src, 64 * 64 + 64);
    for (int s = 0; s < 5; ++s) {
        const int off = 64 * lane + 2 * s;
        if (mode == 0) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
            for (int k = 0; k < 4; ++k) lds[s][4 * lane + k] = v[k];
        } else if (mode == 1) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)&lds[s][0], 16, off, 0, 0, 0);
        } else {
            for (int k = 0; k < 4; ++k)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void *)&lds[s][64 * k], 4, off + 4 * k, 0, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    for (int s = 0; s < 5; ++s)
        for (int k = 0; k < 4; ++k) {
            // mode 2 wrote dword k of every lane contiguously per k
            const unsigned v = mode == 2 ? lds[s][64 * k + lane] : lds[s][4 * lane + k];
            out[(s * 64 + lane) * 4 + k] = v;
        }
}
}  // namespace

extern "C" int rc_dev_align_probe(const void *src, void *out, int mode, void *stream) {
    hipLaunchKernelGGL(align_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                       (const char *)src, (unsigned *)out, mode);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
