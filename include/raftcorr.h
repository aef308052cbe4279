/*
 * raftcorr.h -- C-ABI of the MI355X (gfx950) correlation path for RAFT-Stereo.
 *
 * Drop-in boundary for the reference's CorrBlock1D (/root/reference/model.py):
 *   rc_corr_build   replaces CorrBlock1D.__init__ + CorrBlock1D.corr
 *                   (model.py:284-295 and :318-326): all-pairs per-row volume
 *                   / sqrt(D) plus the avg-pooled pyramid, in one launch.
 *   rc_corr_pool    replaces one F.avg_pool2d([1,2]) pyramid step (model.py:294);
 *                   used for levels beyond the fused epilogue (and for A/B runs).
 *   rc_corr_lookup  replaces CorrBlock1D.__call__ + bilinear_sampler
 *                   (model.py:297-316 and :267-281).
 *   rc_corr_lookup_conv  the lookup fused with BasicMotionEncoder.convc1 +
 *                   ReLU (model.py:199, :206), SURVEY.md §8f rank 1.
 *   rc_corr_lookup_chain  rc_corr_lookup for a pool-chain fp32 pyramid,
 *                   reading levels 0-1 only (the default of CorrBlock1D).
 *   rc_corr_lookup_step  coords update + flow + lookup of one loop
 *                   iteration in one launch.
 *   rc_convex_upsample  the convex upsampler for the mask the update block
 *                   produces.
 *   rc_corr_lookup_backward, rc_corr_build_backward  the gradient of the
 *                   path to the feature maps (autograd of model.py:267-326),
 *                   SURVEY.md §8f rank 2.
 *
 * The reference has no FFI; its "operator API" is the duck-typed class bound
 * at model.py:366-367 and called at :376.  raft-stereo_amd/corr.py mirrors that
 * class on top of these entry points (ctypes).
 *
 * Conventions: plain pointers and sizes, device pointers from any allocator
 * (PyTorch's caching allocator in practice), stream = hipStream_t passed as
 * void* (NULL = default stream).  Nothing is allocated, nothing synchronises,
 * nothing throws across the ABI.  Return 0 on success, else an RC_E* code;
 * rc_last_error() then describes the failure (thread-local).
 */
#ifndef RAFTCORR_H
#define RAFTCORR_H

#ifdef __cplusplus
extern "C" {
#endif

#define RC_ABI_VERSION 10

/* element types */
#define RC_F32  0
#define RC_BF16 1

/* Flags OR-ed into a pyr_dtype argument (ABI v5): RC_SHADOW_LEVEL(l) says
 * stored pyramid level l has a line-phase SHADOW copy (RC_SHADOW: every
 * stored level) -- the same rows, at byte offset
 * RC_SHADOW_OFFSET(rows, ld, esize) from the level's base (rows = B*H*W1,
 * ld = its row stride in elements, esize = 4 for RC_F32, 2 for RC_BF16), so
 * the allocation holds rows*ld*esize bytes, a gap, then the copy, shifted by
 * half a 128-byte line against the primary when the base is 128-B aligned.
 * rc_corr_build writes both copies; the pair kernel of rc_corr_lookup_chain /
 * rc_corr_lookup_step reads each pixel's span from the copy in which it
 * touches fewer 128-B lines (bit-identical results, fewer HBM lines per
 * pixel).  The other entry points accept the flag and read the primary copy.
 * A level and its copy must fit in 4 GiB (RC_EUNSUPPORTED otherwise).  The
 * copies cost build-time writes; which levels pay for themselves depends on
 * the level's size and how often it is read. */
#define RC_SHADOW_LEVEL(l) (0x100 << (l))
#define RC_SHADOW 0xFF00
#define RC_SHADOW_OFFSET(rows, ld, esize) \
    ((((long long)(rows) * (long long)(ld) * (long long)(esize) + 127) / 128) * 128 + 64)

/* Flag OR-ed into the pyr_dtype of rc_corr_lookup_chain / rc_corr_lookup_step
 * (ABI v5): write the lookup output channels-last, out[((b*H + h)*W1 + w)*C + c]
 * with C = levels*(2r+1) -- the (B, C, H, W1) tensor in NHWC memory order
 * (torch.channels_last), the same values.  Pair kernel only (2 levels, or 4
 * with level 2 given); RC_EUNSUPPORTED otherwise. */
#define RC_OUT_CHANNELS_LAST 0x10000

/* Flag OR-ed into the pyr_dtype of rc_corr_build (ABI v6): run the exact fp32
 * MFMA kernel (v_mfma_f32_16x16x4_f32) for fp32 fmaps and an fp32 pyramid.
 * Without it such a build runs the split-bf16 kernel: every fp32 operand is
 * the exact sum of three bf16 pieces and each product the sum of the six
 * leading piece products on v_mfma_f32_16x16x32_bf16 with fp32 accumulation
 * -- fp32 accuracy (measured at or below the fp32 MFMA chain's error against
 * an fp64 volume) at a third of the MFMA time.  Non-finite fmap values are
 * the exception: an inf operand gives NaN in its row's volume where the fp32
 * GEMM gives +-inf; pass this flag for such inputs.  Ignored by bf16 builds. */
#define RC_BUILD_EXACT_F32 0x20000

/* Flag OR-ed into the pyr_dtype of rc_corr_build and rc_corr_lookup_chain
 * (ABI v9): the pair layout's stored levels -- level 0, and level 2 of a
 * 4-level pyramid (pyr[1] == NULL) -- are DISPARITY-MAJOR.  Level l of row
 * block r = b*H + h is an array S of RC_SHEAR_ROWS(W2, W1, l) rows of
 * pyr_ld[l] fp32 elements (pyr_ld[l] >= W1, a multiple of 4), at
 * pyr[l] + r * RC_SHEAR_ROWS(W2, W1, l) * pyr_ld[l], with
 *     S[k][w1] = C_l[(r, w1)][j],   k = (w1 >> l) - j + (W2 >> l) - 1,
 * so the pixels of an image row that look at the same disparity read one
 * contiguous run of a row of S.  Entries with j outside [0, W2 >> l) are
 * neither written nor read.  The values are the row layout's bit for bit and
 * so are the lookups (rc_corr_lookup_chain with the flag: the pair kernel's
 * arithmetic); it pays where neighbouring pixels' coords agree (the
 * network's fields), and loses on independent random coords (DESIGN.md
 * §3.2h).  Requires fp32 fmaps and pyramid on the split-bf16 build (W1, W2
 * multiples of 4, no RC_BUILD_EXACT_F32, no shadow copies), nbuf 1 (2 levels)
 * or 3 with pyr[1] == NULL (4 levels), radius 1..4, NCHW output, each level
 * under 4 GiB; RC_EUNSUPPORTED otherwise.  The other entry points refuse it. */
#define RC_LAYOUT_DISPARITY 0x80000
#define RC_SHEAR_ROWS(W2, W1, l) (((W2) >> (l)) + (((W1) - 1) >> (l)))

/* Flag OR-ed into the pyr_dtype of rc_corr_build, rc_corr_lookup_chain and
 * rc_corr_lookup_step (ABI v10): the 4-level bf16 pair layout's stored levels
 * 0 and 2 as RECORDS -- one 128-byte line per pixel per lookup instead of two
 * (DESIGN.md §3.2i).  pyr[0] is the record buffer: B*H*W1 pixel rows of
 * RC_REC_COUNT(W2) records of RC_REC_SLOTS bf16 (RC_REC_BYTES each, pixel
 * row p at pyr[0] + p * RC_REC_COUNT(W2) * RC_REC_BYTES, 16-byte aligned),
 * record r holding
 *     slots  0..25   level-2 elements 4r - 14 .. 4r + 11,
 *     slots 26..63   level-0 elements 16r - 26 .. 16r + 11
 * (zeros outside the level's width), so a pixel whose floor(x/2) lies in
 * [8r - 8, 8r) reads every tap of all four levels (radius <= 4) from record
 * r.  The values are the row layout's bit for bit, and so are the lookups.
 * rc_corr_build: bf16 fmaps and pyramid, nbuf 3 with pyr[1] == pyr[2] ==
 * NULL (pyr_ld ignored), 64 < W2 <= 320, D > 224, no shadow copies;
 * rc_corr_lookup_chain / _step (chain != 0): RC_BF16, levels 4, radius 1..4,
 * pyr[0] the records and pyr[1..3] NULL, widths[0] = W2; channels-last output
 * allowed.  RC_EUNSUPPORTED otherwise; the other entry points refuse it.
 * A pixel row's records take RC_REC_COUNT(W2) * 128 bytes, against about
 * 2 * 2 * (W2 + W2 / 4) for the shadowed rows (2816 vs 1556 at W2 = 311):
 * the build writes more, and each lookup reads half the lines. */
#define RC_LAYOUT_RECORDS 0x100000
#define RC_REC_SLOTS 64
#define RC_REC_BYTES 128
#define RC_REC_COUNT(W2) (((((W2) >> 1) + 15) >> 3) + 1)

/* return codes */
#define RC_OK            0
#define RC_EINVAL        1  /* bad shape / pointer / alignment / parameter */
#define RC_EUNSUPPORTED  2  /* valid request this build does not implement */
#define RC_EHIP          3  /* HIP runtime error (launch / device) */

/* Maximum pyramid buffers one rc_corr_build call writes (num_levels + 1). */
#define RC_MAX_LEVELS 8

int rc_abi_version(void);
const char *rc_last_error(void);

/* Volume + pyramid (model.py:284-295, :318-326).
 *   fmap1: [B][D][H][W1], fmap2: [B][D][H][W2], contiguous, element type
 *          fmap_dtype (RC_F32, or RC_BF16 for the bf16 MFMA path).
 *   pyr[l], l < nbuf: device buffers of B*H*W1 rows of W2 >> l elements of
 *          pyr_dtype, row stride pyr_ld[l] elements (>= W2 >> l; NULL pyr_ld =
 *          dense rows).  Level 0 is the volume divided by sqrtf(D), level l+1
 *          the pairwise mean of level l along w2 (floor width).  The
 *          reference builds num_levels+1 buffers (model.py:293); pass
 *          nbuf = num_levels + 1.  Padding rows to a multiple of 16 bytes lets
 *          every store be a full aligned vector (the padding is written with
 *          don't-care values and never read).
 *   Requires (W2 >> (nbuf-1)) >= 1 (the reference raises otherwise) and
 *   16-byte aligned pointers.
 *   Arithmetic: fmap_dtype == pyr_dtype == RC_F32 runs the split-bf16 fp32
 *   kernel (ABI v6; see RC_BUILD_EXACT_F32, which selects the exact fp32 MFMA
 *   kernel v_mfma_f32_16x16x4_f32 instead).  Any bf16 operand (bf16 fmaps, or a
 *   bf16 pyramid requested for fp32 fmaps, which are rounded to bf16 on
 *   load) runs the bf16 MFMA kernel (v_mfma_f32_16x16x32_bf16, fp32
 *   accumulation); pooling is done on the fp32 accumulators either way. */
int rc_corr_build(const void *fmap1, const void *fmap2, int fmap_dtype,
                  int B, int D, int H, int W1, int W2,
                  void *const *pyr, const long *pyr_ld, int nbuf, int pyr_dtype,
                  void *stream);

/* One pooling step (model.py:294): out[p][j] = (in[p][2j] + in[p][2j+1]) / 2,
 * j < W_in/2, for p < rows; row strides ld_in / ld_out elements.  dtype
 * RC_F32 or RC_BF16 (bf16 rounds once). */
int rc_corr_pool(const void *in, long ld_in, void *out, long ld_out, long rows,
                 int W_in, int dtype, void *stream);

/* Lookup (model.py:297-316, :267-281).
 *   pyr[i], i < levels: B*H*W1 rows of widths[i] elements of pyr_dtype, row
 *          stride pyr_ld[i] elements (NULL = dense), 16-byte aligned base.
 *   coords_x: x channel of the (B,2,H,W1) fp32 coords, element (b,h,w) at
 *          coords_x[b*coord_batch_stride + h*W1 + w] (the y channel is
 *          ignored, model.py:299/:308).
 *   out:   [B][levels*(2*radius+1)][H][W1] fp32, channel = level*(2r+1)+(t+r).
 *   radius in 1..8, levels in 1..RC_MAX_LEVELS. */
int rc_corr_lookup(const void *const *pyr, const int *widths, const long *pyr_ld,
                   int pyr_dtype, int levels, int radius, const float *coords_x,
                   long coord_batch_stride, int B, int H, int W1, float *out,
                   void *stream);

/* Lookup fused with the motion encoder's first conv (model.py:199, :206):
 *   out[b][c][h][w] = act(bias[c] + sum_k weight[c][k] * corr[b][k][h][w]),
 *   corr = the rc_corr_lookup result (k = level*(2r+1) + tap, never written),
 *   weight: [cout][levels*(2r+1)] fp32 (a 1x1 Conv2d weight), bias: [cout] or
 *   NULL, act = ReLU when relu != 0.  out: [B][cout][H][W1] fp32.
 *   levels 2..4, radius 1..4. */
int rc_corr_lookup_conv(const void *const *pyr, const int *widths, const long *pyr_ld,
                        int pyr_dtype, int levels, int radius, const float *coords_x,
                        long coord_batch_stride, int B, int H, int W1,
                        const float *weight, const float *bias, int cout, int relu,
                        float *out, void *stream);

/* Lookup over a pool-chain fp32 pyramid (what rc_corr_build writes), same
 * arguments and bit-identical results as rc_corr_lookup with RC_F32, but
 * some levels are recomputed from others (level l+1 = pairwise mean of level
 * l, the fp32 ops of model.py:294) instead of read.  pyr[i], i >= 1, may be
 * NULL (not stored); the kernel is chosen from what is given:
 *   levels 2, or levels 4 with pyr[2] != NULL: the pair kernel reads levels 0
 *     and 2 (one span of each serves two levels); level-0 width <= 65536;
 *   otherwise levels 3..4 with pyr[1] != NULL: the level-1 chain kernel reads
 *     levels 0 and 1 (one level-1 span serves levels 1..L-1).
 * Requires widths[i] == widths[i-1] / 2, the read levels' row strides whole
 * 16-B chunks, radius 1..4.  Levels given but not read must still hold the
 * pool chain for the results to equal rc_corr_lookup's.  pyr_dtype RC_BF16
 * (pair layout only): every level is the bf16-rounded pool of the level below
 * as stored -- what rc_corr_build and rc_corr_pool write for a bf16 pyramid,
 * and what avg_pool2d gives on bf16 tensors.  (ABI v4 added pyr_dtype.) */
int rc_corr_lookup_chain(const void *const *pyr, const int *widths, const long *pyr_ld,
                         int pyr_dtype, int levels, int radius, const float *coords_x,
                         long coord_batch_stride, int B, int H, int W1, float *out,
                         void *stream);

/* One iteration of the forward loop's corr step in one launch: the
 * coordinate update that ends the previous iteration (coords1 + delta_flow
 * with delta_flow[:,1] = 0, the loop tail SURVEY Appendix A D8), then
 * flow = coords1 - coords0 (model.py:377, coords0 = coords_grid :329-332),
 * then the lookup at the new coords1 (:376).  coords1, delta, coords1_out,
 * flow_out: (B,2,H,W1) fp32 contiguous; delta NULL = no update (first
 * iteration); coords1_out may alias coords1.  chain != 0 runs
 * rc_corr_lookup_chain's kernel (its preconditions apply), else
 * rc_corr_lookup's.  The lookup output is bit-identical to theirs at the
 * updated coordinates; coords1_out and flow_out are bit-identical to the
 * PyTorch ops they replace.  SURVEY.md §8f rank 4. */
int rc_corr_lookup_step(const void *const *pyr, const int *widths, const long *pyr_ld,
                        int pyr_dtype, int levels, int radius, int chain,
                        const float *coords1, const float *delta, float *coords1_out,
                        float *flow_out, int B, int H, int W1, float *out, void *stream);

/* Backward of rc_corr_lookup (model.py:297-316 through grid_sample's input
 * gradient, :275): for every pixel p, level i and tap t, adds
 * (x0+1-x')*g to grad_pyr[i][p][x0] and (x'-x0)*g to grad_pyr[i][p][x0+1]
 * (zero-padded taps add nothing), g = grad_out[b][i*(2r+1)+t][h][w].
 *   grad_pyr[i]: fp32, B*H*W1 rows of widths[i], row stride grad_ld[i]
 *          (multiple of 4; NULL grad_ld = dense, then widths must be
 *          multiples of 4), 16-byte aligned.  Accumulates: zero the buffers
 *          once, then call once per lookup call.
 *   grad_out: [B][levels*(2r+1)][H][W1] fp32 contiguous.  Other arguments as
 *          rc_corr_lookup.  No atomics: pixel p owns row p.
 *   Pair layout: with levels 2 or 4, grad_pyr[1] (and grad_pyr[3]) NULL and
 *          radius <= 4, the gradients of levels 1 and 3 are added, already
 *          through avg_pool2d's backward (/2 to both children), to levels 0
 *          and 2; pass such buffers to rc_corr_build_backward with levels = 3
 *          and grad_pyr[1] = NULL.
 *   levels | RC_SHADOW_LEVEL(0) / RC_SHADOW_LEVEL(2) (4-level pair layout
 *          only, else RC_EUNSUPPORTED): the allocation of grad_pyr[l] also
 *          holds a zeroed copy at RC_SHADOW_OFFSET(B*H*W1, grad_ld[l], 4)
 *          bytes; each pixel's span goes to the copy in which it touches
 *          fewer 128-B lines.  Pass the same bits to rc_corr_build_backward,
 *          which sums the copies.  Measured not to pay at config 2
 *          (DESIGN.md §3.4b); off by default. */
int rc_corr_lookup_backward(void *const *grad_pyr, const int *widths, const long *grad_ld,
                            int levels, int radius, const float *coords_x,
                            long coord_batch_stride, int B, int H, int W1,
                            const float *grad_out, void *stream);

/* The gradients of n_calls lookups into the same gradient buffers, summed in
 * one pass (ABI v7; model.py:376 runs the lookup `iters` times, and autograd
 * adds every call's grid_sample input gradient, :275, into the levels):
 * equal to n_calls rc_corr_lookup_backward calls up to the association of
 * the fp32 sums.  coords_x[c], coord_batch_stride[c], grad_out[c]: call c's
 * arguments as in rc_corr_lookup_backward (all calls share B, H, W1, levels,
 * radius).  levels | RC_GRAD_OVERWRITE: the buffers receive the sum instead
 * of having it added (they need not be zeroed first; row padding up to the
 * next multiple of 4 columns is written as zeros).  With the pair layout each
 * lane keeps the union of its calls' windows of its pixel's rows on chip
 * (compact rows: any level-0 width whose LDS budget max(5120, 2(W + 8r + 24))
 * floats fits 64 KB, i.e. W up to about 8K), so each call's inputs are read
 * once and each row written once, in launches of up to 32
 * calls.  Wider rows, per-call coords or grad_out extents past the kernel's
 * 32-bit offsets, and the per-level layout run a loop over
 * rc_corr_lookup_backward instead -- chosen for the whole request before the
 * first launch.  RC_SHADOW_LEVEL bits are RC_EUNSUPPORTED here; other flag
 * bits than RC_GRAD_OVERWRITE are RC_EINVAL.  RC_GRAD_OVERWRITE with
 * n_calls == 0 is RC_EINVAL; n_calls == 0 otherwise does nothing. */
#define RC_GRAD_OVERWRITE 0x40000
int rc_corr_lookup_backward_calls(void *const *grad_pyr, const int *widths, const long *grad_ld,
                                  int levels, int radius, int n_calls,
                                  const float *const *coords_x, const long *coord_batch_stride,
                                  int B, int H, int W1, const float *const *grad_out,
                                  void *stream);

/* Backward of rc_corr_build (model.py:284-295 pooling, :318-326 volume):
 *   Dl_{L-1} = grad_pyr[L-1], Dl_i[k] = grad_pyr[i][k] + Dl_{i+1}[k/2] / 2
 *   (avg_pool2d's backward, floor widths), G = Dl_0 / sqrtf(D), and
 *   grad_fmap1[b][d][h][w1] = sum_w2 G[b,h,w1,w2] * fmap2[b][d][h][w2]
 *   grad_fmap2[b][d][h][w2] = sum_w1 G[b,h,w1,w2] * fmap1[b][d][h][w1]
 *   (overwritten, fp32).  grad_pyr[l], l < levels: fp32 B*H*W1 rows of
 *   W2 >> l, row stride grad_ld[l] (grad_ld[0] % 4 == 0).  fmap_dtype RC_F32
 *   only.  When B*H*W1 == 0 nothing is written.
 *   ABI v8: the two GEMMs run on bf16 MFMA with every fp32 operand split
 *   exactly into three bf16 pieces (six products per fp32 product, fp32
 *   accuracy, as rc_corr_build's default) when W1 % 4 == W2 % 4 == 0 and the
 *   gradients are pair-folded or 1-2 levels; otherwise, or with
 *   fmap_dtype | RC_BUILD_EXACT_F32 (needed only for non-finite values), on
 *   exact fp32 MFMA.
 *   levels == 3 with grad_pyr[1] == NULL: pair-folded gradients from
 *   rc_corr_lookup_backward's pair layout, Dl_0[k] = g_0[k] + g_2[k>>2] / 4;
 *   with levels | RC_SHADOW_LEVEL(0) / (2) each g_l is primary + shadow copy. */
int rc_corr_build_backward(const void *fmap1, const void *fmap2, int fmap_dtype,
                           int B, int D, int H, int W1, int W2,
                           const void *const *grad_pyr, const long *grad_ld, int levels,
                           float *grad_fmap1, float *grad_fmap2, void *stream);

/* Convex upsampling with the update block's mask
 * (model.py:238-241, 0.25-scaled at :264; f = 2^n_downsample, :236):
 *   out[n][c][f h + i][f w + j] = sum_k softmax_k(mask[n][k f^2 + i f + j][h][w])
 *                                 * f * flow[n][c][h + dy_k][w + dx_k]
 *   k = 3 (dy+1) + (dx+1), zeros outside the image (RAFT-Stereo's upsampler,
 *   F.unfold + softmax; the reference builds the mask but never applies it).
 *   flow (N,C,H,W), mask (N,9f^2,H,W), out (N,C,fH,fW): fp32 contiguous.
 *   factor 1, 2, 4 or 8. */
int rc_convex_upsample(const float *flow, const float *mask, int N, int C, int H, int W,
                       int factor, float *out, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* RAFTCORR_H */
