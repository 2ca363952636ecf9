/*
 * advpatch.h — C ABI of libadvpatch_hip.so, the MI355X (gfx950) hot path of the
 * adversarial-patch training loop (reference: train_patch.py batch body,
 * train_patch.py:157-330).
 *
 * The reference is pure Python over PyTorch (no FFI of its own);
 * each entry below replaces the ATen kernels that one reference Python op
 * invokes, and is bound from Python with ctypes.
 *
 * Conventions
 *  - All tensor pointers are DEVICE pointers owned by the caller; the library
 *    never allocates on the hot path.  float = IEEE fp32.
 *  - Every entry is stream-ordered on the caller's hipStream_t (passed as
 *    po_stream_t, an opaque pointer so this header needs no HIP headers) and
 *    returns 0 on success or a negative PO_E* code; po_last_error() returns a
 *    thread-local message for the last failure.
 *  - Activations inside the network are NHWC with the channel stride padded
 *    to a multiple of 16 ("Cp"); patch/image tensors are NCHW as in the
 *    reference.
 */
#ifndef ADVPATCH_H
#define ADVPATCH_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* po_stream_t;

#define PO_OK 0
#define PO_EINVAL -1   /* bad argument (shape, null pointer, unsupported config) */
#define PO_EHIP -2     /* HIP runtime error */
#define PO_EDEVICE -3  /* device is not gfx950 */

#define PO_ABI_VERSION 30
#define PO_AMAX_SUB 64  /* sub-slots per max|x| slot (see po_conv_desc) */

int po_abi_version(void);
const char* po_last_error(void);
/* Select the device and verify it is gfx950.  Returns PO_EDEVICE otherwise. */
int po_device_check(int device);

/* ---------------- patch-side ops (reference load_data.py / median_pool.py) ---------------- */

/* MedianPool2d(7, same=True).forward: reflect pad 3, 7x7 window median.
 * Replaces median_pool.py:46-52.  x,y [C,H,W]; argidx [C,H,W] = flat source
 * index (c*H*W + r*W + q, reflection resolved) of the selected element:
 * the first window position (row-major) holding the median value. */
int po_median7_fwd(const float* x, int C, int H, int W, float* y, int32_t* argidx, po_stream_t s);
/* dx = scatter-add of dy through argidx (deterministic gather form). */
int po_median7_bwd(const float* dy, const int32_t* argidx, int C, int H, int W, float* dx, po_stream_t s);
/* MedianPool2d for any kernel (kh, kw), stride (sh, sw) and reflect padding
 * (pl, pr, pt, pb) (median_pool.py:8-52; the 'same' rule is the caller's):
 * y [C,Ho,Wo] = the lower median (rank (n-1)/2) of each window, argidx = the
 * flat source index of the first window position holding it; bwd: dx [C,H,W]
 * = sum of dy over the outputs whose argument is each pixel. */
int po_median_fwd(const float* x, int C, int H, int W, int kh, int kw, int sh, int sw, int pl, int pr, int pt,
                  int pb, float* y, int32_t* argidx, po_stream_t s);
int po_median_bwd(const float* dy, const int32_t* argidx, int C, int H, int W, int kh, int kw, int sh, int sw,
                  int pl, int pr, int pt, int pb, float* dx, po_stream_t s);

/* Per-image patch placement (load_data.py:453-509 lab_transform,
 * 654-743 target_size/scale/theta, 693-715 target_x/y and patch_center).
 * lab [B,L,5]; angle,ux,uy [B]; theta out [B,6]; center out [B,2]
 * (column,row) pixels, fp32 exactly as the reference (the loss cell index is
 * derived from it); target_size out [B] (may be NULL); roi out [B,4] int32
 * (may be NULL) = {x0,y0,x1,y1} bounding box (+2 px margin, clipped to the
 * image) of the output pixels the warped patch can touch; affine out [B,6]
 * float64 rows (may be NULL) for po_warp_*.
 * geometry 1 or 2 (ABI 27; the trainer's default): the reference's fp32
 * arithmetic -- theta (load_data.py:738-743), affine_grid (745) and
 * grid_sample (748-749) as PyTorch-CPU computes them, op by op (pinned by
 * tests/test_geometry_ref.py); affine_grid's K = 3 dot product in the order
 * of the host's MKL sgemm: 1 = fl(fl(bx*t0) + fl(by*t1)) + t2 (AMD EPYC
 * hosts), 2 = fl(fma(by, t1, fl(bx*t0))) + t2 (Intel AVX-512); theta and
 * target_size are those fp32 values, and each affine row holds the fp32
 * theta as float[6] in its first 24 bytes with a tag in row[3]
 * (warp_geom.h), so the warp kernels sample exactly where the reference
 * samples.  sin/cos of angles on po_draws' lattice come
 * from sincos_lut [2^24][2] fp32 (8-byte aligned; may be NULL): PyTorch-CPU's
 * own torch.sin/torch.cos of the lattice angle k at [k] (MKL VML is not
 * correctly rounded, so the values are tabulated, not restated); other angles
 * get correctly rounded values.  sqrt_lut [2^24] fp32 (may be NULL): the
 * host's torch.sqrt (MKL VML, not correctly rounded either) of the floats
 * with bits 0x3F800000 + i, i.e. one period [1, 4) of a function that scales
 * exactly with powers of 4; the target size's sqrt reads it.
 * geometry 0: the same formulas in float64 from the same fp32 inputs; each
 * affine row is the pixel-space sampling map of affine_grid + grid_sample
 * (align_corners=False): output pixel (i,j) samples the padded patch at
 * column ix = a0*j + a1*i + a2, row iy = a3*j + a4*i + a5 (theta rounded to
 * fp32 on output). */
int po_patch_params(const float* lab, int B, int L, const float* angle, const float* ux,
                    const float* uy, int do_rotate, int S, int P, int geometry, const float* sincos_lut,
                    const float* sqrt_lut, float* theta, float* center, float* target_size, int32_t* roi,
                    double* affine, po_stream_t s);

/* Random draws of the patch transformer for images b0 .. b0+B-1 of a global
 * batch (load_data.py:548-574 contrast U(0.8,1.2), brightness U(-0.1,0.1),
 * noise U(-1,1) [B,3,P,P]; 607-614 angle U(-pi,pi); 693-707 ux, uy U(0,1)).
 * Counter-based (Philox4x32-10, key = seed, counter = {element group, global
 * image index, step counter}): a rank drawing its shard gets exactly the rows a
 * single process draws for the whole batch.  Any output may be NULL. */
int po_draws(uint64_t seed, uint64_t counter, int b0, int B, int P, float* contrast, float* bright,
             float* noise, float* angle, float* ux, float* uy, po_stream_t s);

/* NaN/Inf guard (replaces torch.autograd.detect_anomaly, train_patch.py:158):
 * flags[0] |= bit if any of x[0..n) is not finite.  No host synchronisation. */
int po_check_finite(const float* x, int64_t n, int32_t bit, int32_t* flags, po_stream_t s);

/* po_check_finite, then *found_inf = (flags[0] & bit) ? 1.0f : 0.0f: the
 * found_inf operand of PyTorch's fused Adam follows the flag word (set by
 * this or an earlier check, cleared only when the caller clears the flags),
 * so a non-finite step is skipped with no host code (ABI 21). */
int po_check_finite_inf(const float* x, int64_t n, int32_t bit, int32_t* flags, float* found_inf, po_stream_t s);

/* (ABI 30) Adam(amsgrad) + clamp of one parameter tensor in one launch
 * (replaces torch.optim.Adam(amsgrad=True).step() + adv_patch.data.clamp_(0, 1),
 * train_patch.py:131-136, 327-330; weight decay 0, not maximize).  The
 * arithmetic is torch's single-tensor Adam (the reference's CPU form):
 * exp_avg = fma(1 - beta1, grad - exp_avg, exp_avg) (ATen's lerp),
 * exp_avg_sq = exp_avg_sq * beta2 + ((1 - beta2) * grad) * grad,
 * max_exp_avg_sq = maximum(max_exp_avg_sq, exp_avg_sq) (NaN propagating),
 * param += (-lr / (1 - beta1^t)) * exp_avg / (sqrt(max_exp_avg_sq) /
 * sqrt(1 - beta2^t) + eps), the scalars in float64 with t = *step_in + 1,
 * rounded to fp32 where torch rounds them; then, if clamp, param =
 * min(max(param, lo), hi) (NaN kept).  *step_out = t, or *step_in when the
 * update is skipped: found_inf (if not NULL) nonzero or flags[0] & bit (if
 * flags not NULL) -- the update, the moments and the count then stay as they
 * were.  step_in and step_out are two different device floats (the caller
 * alternates them).  n may be 0. */
int po_adam_amsgrad(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, float* max_exp_avg_sq,
                    int64_t n, const float* step_in, float* step_out, double lr, double beta1, double beta2,
                    double eps, const float* found_inf, const int32_t* flags, int32_t bit, int clamp, float lo,
                    float hi, po_stream_t s);

/* Augment (contrast/brightness/noise/clamp, load_data.py:548-574) + affine
 * bilinear warp of patch and mask (affine_grid + grid_sample, align_corners
 * False, zeros, load_data.py:745-749) + clamp*mask (791-792).
 * mode 0: write adv_t [B,3,S,S] (PatchTransformer output, dim 1 squeezed).
 * mode 1: also composite, out = where(adv_t==0, img, adv_t) (PatchApplier,
 *         load_data.py:820) into `out` [B,3,S,S]; `img` required.
 * patch_mp [3,P,P] (median-pooled patch), noise [B,3,P,P] U(-1,1) (x0.1 inside),
 * contrast/bright [B], affine [B,6] float64 (po_patch_params). */
int po_warp_fwd(const float* img, const float* patch_mp, const float* noise, const float* contrast,
                const float* bright, const double* affine, int B, int S, int P, int mode,
                float* out, po_stream_t s);
/* Backward of po_warp_fwd w.r.t. patch_mp: d_patch_mp [3,P,P] (overwritten).
 * d_out [B,3,S,S] is dL/d(out).  mode as in fwd (mode 1 applies the where()
 * routing).  Deterministic: one thread per patch element gathers over images
 * and over the output pixels whose bilinear footprint covers it. */
int po_warp_bwd(const float* d_out, const float* patch_mp, const float* noise, const float* contrast,
                const float* bright, const double* affine, int B, int S, int P, int mode,
                float* work /* [B,3,S,S] scratch, may alias d_out */, float* d_patch_mp,
                po_stream_t s);
/* po_warp_fwd / po_warp_bwd with the noise regenerated in the kernels instead
 * of read from a [B,3,P,P] tensor: element e (flat over [3][P][P]) of image b
 * is po_draws(seed, counter, b0, ...)'s noise value of global image b0 + b,
 * bit for bit (lane e % 4 of Philox group e / 4).  The B*3*P*P*4 bytes of
 * noise are then neither written by po_draws nor gathered by the warp. */
int po_warp_fwd_keyed(const float* img, const float* patch_mp, uint64_t seed, uint64_t counter, int b0,
                      const float* contrast, const float* bright, const double* affine, int B, int S, int P,
                      int mode, float* out, po_stream_t s);
int po_warp_bwd_keyed(const float* d_out, const float* patch_mp, uint64_t seed, uint64_t counter, int b0,
                      const float* contrast, const float* bright, const double* affine, int B, int S, int P,
                      int mode, float* work, float* d_patch_mp, po_stream_t s);
/* The augmentation half of PatchTransformer (load_data.py:548-571) for the
 * keyed draws, before the clamp: pre [B,3,P,P] = patch_mp * contrast[b] +
 * bright[b] + 0.1 * noise, the noise being po_draws(seed, counter, b0, ...)'s
 * value of global image b0 + b (as po_warp_*_keyed).  po_warp_fwd_pre /
 * po_warp_bwd_pre then gather these values: the same outputs and patch
 * gradient as po_warp_*_keyed bit for bit, with one Philox call per 4 patch
 * elements instead of one per bilinear corner read.  po_warp_bwd_pre still
 * takes contrast (the gradient's factor).  roi [B][4] = po_patch_params' footprint
 * boxes {x0, y0, x1, y1}: the pixels outside an image's box are written as
 * 16-byte copies of img (mode 1) or zeros (mode 0) without per-pixel geometry,
 * the box's pixels one per thread; the backward's per-pixel phase runs over the
 * boxes only (`work`: >= 4*B*S*S floats, 16-byte aligned, not aliasing d_out:
 * the per-pixel factors interleaved [B][S][S][4]). */
int po_augment_patch(const float* patch_mp, uint64_t seed, uint64_t counter, int b0, const float* contrast,
                     const float* bright, int B, int P, float* pre, po_stream_t s);
int po_warp_fwd_pre(const float* img, const float* pre, const double* affine, const int32_t* roi, int B, int S,
                    int P, int mode, float* out, po_stream_t s);
int po_warp_bwd_pre(const float* d_out, const float* pre, const float* contrast, const double* affine,
                    const int32_t* roi, int B, int S, int P, int mode, float* work, float* d_patch_mp, po_stream_t s);
/* The footprint-box warp with the keyed noise formed at each bilinear corner
 * (mp * contrast + bright + 0.1 * Philox noise, as po_warp_*_keyed) instead of
 * gathered from po_augment_patch's [B,3,P,P] buffer: no augment pass and no
 * pre-augmented patches in HBM (a down-scaled patch is sampled at ~4 corners
 * per footprint pixel, far fewer than its 3*P*P elements).  Same values and
 * gradient as po_warp_*_pre / _keyed bit for bit.  fill = 1: `out` is the whole
 * composite (outside the boxes 16-byte copies of img / zeros, as
 * po_warp_fwd_pre); fill = 0: only the quad-widened boxes {x0 & ~3, y0,
 * (x1 + 3) & ~3, y1} are written -- the training step's form, consumed by
 * po_conv_first_fwd_cmp / po_conv_first_pool_fwd_cmp, which read img outside
 * them (S % 4 == 0).  The backward gathers only images with a bilinear
 * candidate per patch element. */
int po_warp_box_fwd_keyed(const float* img, const float* patch_mp, uint64_t seed, uint64_t counter, int b0,
                          const float* contrast, const float* bright, const double* affine, const int32_t* roi,
                          int B, int S, int P, int mode, int fill, float* out, po_stream_t s);
int po_warp_box_bwd_keyed(const float* d_out, const float* patch_mp, uint64_t seed, uint64_t counter, int b0,
                          const float* contrast, const float* bright, const double* affine, const int32_t* roi,
                          int B, int S, int P, int mode, float* work, float* d_patch_mp, po_stream_t s);
/* (ABI 26) The same pair with the backward's per-pixel factors saved by the
 * forward: po_warp_box_fwd_fac also writes fac [B][S][S][4] (16-byte aligned;
 * per box pixel and channel msk where the gradient passes -- clamp in range and,
 * mode 1, the patch value not replaced by the frame -- else -1), and
 * po_warp_box_bwd_fac turns them into the gradient factors in place (d_out *
 * fac, +0 at -1) instead of re-evaluating the warp at every box pixel, then
 * runs the same gather as po_warp_box_bwd_keyed.  fac must hold the forward's
 * values (nothing may write it in between); outputs equal po_warp_box_*_keyed
 * bit for bit. */
int po_warp_box_fwd_fac(const float* img, const float* patch_mp, uint64_t seed, uint64_t counter, int b0,
                        const float* contrast, const float* bright, const double* affine, const int32_t* roi, int B,
                        int S, int P, int mode, int fill, float* out, float* fac, po_stream_t s);
int po_warp_box_bwd_fac(const float* d_out, const float* patch_mp, uint64_t seed, uint64_t counter, int b0,
                        const float* contrast, const float* bright, const double* affine, const int32_t* roi, int B,
                        int S, int P, float* fac, float* d_patch_mp, po_stream_t s);

/* PatchApplier for an explicit adv tensor: out = where(adv==0, img, adv)
 * (load_data.py:820); n elements. bwd: d_img = d_out*(adv==0), d_adv = d_out*(adv!=0). */
int po_apply_fwd(const float* img, const float* adv, int64_t n, float* out, po_stream_t s);
int po_apply_bwd(const float* d_out, const float* adv, int64_t n, float* d_img, float* d_adv,
                 po_stream_t s);

/* NPS (load_data.py:357-367), TV (404-411) and HasSusRGB colourfulness
 * (1729-1754) of the raw patch [3,P,P], and the gradient
 *   d_patch = g3[0] * dNPS/dp + g3[1] * dTV/dp + g3[2] * dCOL/dp
 * g3 = DEVICE pointer to the upstream gradients of the three terms (so no
 * host sync is needed; the train_patch.py:280-314 weights and
 * torch.max(tv_loss, 0.1) are applied by the caller's autograd).
 * colors [ncol,3].  out3 [3] = {nps, tv, colour};
 * d_patch [3,P,P] is OVERWRITTEN (may be NULL: forward only). */
int po_regularisers(const float* patch, int P, const float* colors, int ncol, const float* g3,
                    float* out3, float* d_patch,
                    float* workspace /* >= 16384 floats */, po_stream_t s);
/* Its gradient in one launch: d_patch = g3[0] dNPS/dp + g3[1] dTV/dp + g3[2]
 * dCOL/dp from the statistics a po_regularisers call left in `workspace`
 * (that call's patch and colours; any g3), the same values bit for bit as
 * po_regularisers with d_patch.  accumulate = 1: d_patch += the gradient
 * (one fp32 add of the complete value: autograd's sum of two contributions). */
int po_regularisers_grad(const float* patch, int P, const float* colors, int ncol, const float* g3,
                         const float* workspace, int accumulate, float* d_patch, po_stream_t s);

/* Loss head (train_patch.py:428-548 + 230-253):
 * for each head h (map side hw_h, NHWC, Cp>=60, channel a*20+f), each image b:
 *   cell = floor(center/ (S/hw)) ; index = ix*hw + iy  (transposed)
 *   obj[b, h*3+a] = sigmoid(head[b, index, a*20+4]); cls[b,h*3+a,c] = sigmoid(.. a*20+5+c)
 * no_obj = 4*(1 - mean_b max_k obj)          (max: first index on ties)
 * no_cls = objective 0: mean_b mean_k CE(cls[b,k,:], target)  (CE on probabilities)
 *          objective 1: sum_b mean_k (max_c cls - cls[target])  (noCLS_loss_targeted,
 *                       train_patch.py:550-577; max: first index on ties)
 *          objective 2: 0 (untargeted)
 * Head buffers are either the full map [B,hw,hw,Cp] (org == NULL or org[h] ==
 * NULL) or a window [B,win[h],win[h],Cp] whose per-image origin (row, col) in
 * map coordinates is org[h][2b..2b+1] (po_cell_windows); win may be NULL when
 * every head is a full map.
 * out2 [2] = {no_obj, no_cls}; obj_out [B,3*nheads], cls_out [B,3*nheads,15], cells [nheads,B]
 * (each may be NULL).  d_heads (may be NULL, same layout as heads): gradient of
 * g2[0]*no_obj + g2[1]*no_cls (g2: DEVICE pointer, 2 floats)
 * written at the selected cells only (other elements untouched — caller zeroes).
 * flags (may be NULL): OR-ed with bit0 if any cell index was out of range
 * (clamped), bit1 if a cell fell outside its head window (clamped; a
 * planning error) — an accumulator the caller checks when it chooses.
 * scratch (may be NULL): 2*B floats; with it the images run on one workgroup
 * per 16 (the same results, bit for bit), without it on one workgroup. */
int po_cell_loss(const float* const* heads, const int* hw, const int* win, const int32_t* const* org,
                 int nheads, int Cp, int B, int S, const float* center, int target, int objective,
                 const float* g2, float* const* d_heads, float* out2, float* obj_out, float* cls_out,
                 int32_t* cells, int32_t* flags, float* scratch /* >= 2*B floats, or NULL */, po_stream_t s);

/* The iteration's loss (train_patch.py:230-314) from out2 = {no_obj_loss,
 * no_cls_loss} (po_cell_loss) and reg = {nps, tv, colour} (po_regularisers):
 *   loss = 0.01 nps + max(2.5 tv, 0.1) + no_obj + colour [+ no_cls if with_cls]
 * with, when `weighted` (a data-parallel rank, train_patch.shard_weights),
 * no_obj * w_img, no_cls * w_cls and the three patch terms * w_patch.
 * terms[0..5] = {loss, nps_loss, tv_loss, no_obj_loss, no_cls_loss,
 * colorful_loss} as train_patch.combine_terms returns them (same fp32
 * operations, same order); *loss_out (optional) = the loss.  One thread. */
int po_loss_combine(const float* out2, const float* reg, float w_img, float w_cls, float w_patch, int weighted,
                    int with_cls, float* terms, float* loss_out, po_stream_t s);

/* Its gradient for dL = g_loss[0]: d_out2[2] and d_reg[3], the values and
 * rounding of PyTorch's autograd of combine_terms (maximum's backward gives a
 * tie half the gradient). */
int po_loss_combine_bwd(const float* reg, const float* g_loss, float w_img, float w_cls, float w_patch, int weighted,
                        int with_cls, float* d_out2, float* d_reg, po_stream_t s);

/* MaxProbExtractor.forward (load_data.py:125-311; bbox_decode 63-122 rewrites
 * only the box fields, so it is not run): per image b, the max over every head
 * h, anchor a (3 per head) and cell p of
 *   q = 0: objectness logit (field 4),  q = 1: class cls_id logit (field 5+cls_id)
 * (sigmoid of the logit when sigmoid_mode), field f of anchor a at channel
 * a*(5+num_cls)+f.  Head h is h[h] x w[h] pixels at element strides
 * strides[3h..3h+2] = {image, channel, pixel} (NCHW: {C*hw, hw, 1}; an NHWC
 * buffer: {hw*Cp, 1, Cp}).  out [2][B] = maxima; idx [2][B] = flat index of
 * the reference's output_cat [B,5+C,sum 3hw]: sum_{h'<h} 3hw' + a*hw + p.
 * Ties: the first index (torch.max); NaN wins.  heads/h/w/strides are HOST arrays
 * of nheads (<= 4) entries. */
int po_max_prob(const float* const* heads, const int* h, const int* w, const int64_t* strides, int nheads, int B,
                int num_cls, int cls_id, int sigmoid_mode, float* out, int32_t* idx, po_stream_t s);
/* Its backward: d_heads[h] (same strides, caller-zeroed) += g[q][b] *
 * d(value)/d(logit) at the element idx[q][b] selected (g: DEVICE [2][B]). */
int po_max_prob_bwd(const float* const* heads, const int* h, const int* w, const int64_t* strides, int nheads,
                    int B, int num_cls, int cls_id, int sigmoid_mode, const int32_t* idx, const float* g,
                    float* const* d_heads, po_stream_t s);

/* Receptive-field windows of the loss (SURVEY Q1 cells): the loss reads each
 * head at one cell per image, so every block downstream of the last
 * full-map block is only needed on a small box around that cell.  For window
 * w and image b:
 *   cell_h = the head-h cell of po_cell_loss (row = index / hw, col = index % hw)
 *   lo = min_h lut[w][h][cell_h][0], hi = max_h lut[w][h][cell_h][1]   (per axis)
 *   org[w][b] = clamp(lo, 0, ext[w][1] - ext[w][0])  for rows and columns
 * lut [nwin][nheads][maxhw][2] int32 (lo > hi: head h does not reach w),
 * ext [nwin][2] = {window side, map side} (DEVICE), hw [nheads] (HOST).
 * flags bit2 is set if a needed box did not fit its static window. */
int po_cell_windows(const float* center, int B, int S, int nheads, const int* hw, int nwin,
                    const int32_t* lut, int maxhw, const int32_t* ext, int32_t* org, int32_t* flags,
                    po_stream_t s);

/* Gradient cones of the input-gradient path.  The patch gradient needs
 * dL/d(image) only inside the patch footprint roi (po_patch_params), so the
 * gradient of block j is only needed on the forward influence cone of roi at
 * j: the pixels of j that depend on an roi pixel.  This evaluates that cone
 * (a box per image and block) by interval arithmetic over `prog`, nprog rows
 * of 8 int32 (DEVICE) {dst, src, kind, k, stride, pad, Hdst, Wdst}, in order
 * (every dst index < nbox, a src's rows before any row reading it):
 *   src -1 = roi; kind 0 conv (k, stride, pad), 1 identity (route/shortcut/
 *   yolo), 2 maxpool size 2 stride 2, 3 maxpool size 2 stride 1 (window
 *   [o, o+1]), 4 nearest 2x upsample.  Rows with the same dst are unioned.
 * roi [B,4] {x0, y0, x1, y1} (NULL: the whole S x S image); boxes [nbox][B][4]
 * int32 {r0, c0, r1, c1} half-open, clipped to [0,Hdst) x [0,Wdst); an empty
 * cone is {0,0,0,0}.  Boxes of blocks no row writes are left untouched. */
int po_grad_boxes(const int32_t* roi, int B, int S, const int32_t* prog, int nprog, int nbox, int32_t* boxes,
                  po_stream_t s);
/* Support boxes of the windowed dgrad launches' compact grids, all entries in
 * one launch.  org [nwin][B][2] window origins (po_cell_windows), cones
 * [nblk][B][4] po_grad_boxes output (NULL when no entry uses a cone), prog
 * [E][12] int32 rows {win, b0, nb, dh1, dh0, dw1, dw0, H, W, w, cone or -1, 0},
 * dst [E] device addresses of the entries' int32 [nb][4] box arrays: box i =
 * {clamp(oy - dh1), clamp(ox - dw1), clamp(oy + w - dh0), clamp(ox + w - dw0)}
 * (rows to [0, H], columns to [0, W]; (oy, ox) = org[win][b0 + i]), then
 * intersected with cones[cone][b0 + i]. */
int po_support_boxes(const int32_t* org, const int32_t* cones, const int32_t* prog, const unsigned long long* dst,
                     int E, int B, po_stream_t s);

/* ---------------- patch evaluation (reference utils.py:93-245, 450-519) ---------------- */

/* get_region_boxes (utils.py:125-245) for one YOLO head, NCHW [B, A*(5+C), h, w]:
 * candidates enumerated per image in the reference's loop order (cy, cx,
 * anchor i); a candidate is kept when conf = sigmoid(obj) * max_c sigmoid(cls_c)
 * (only_objectness: sigmoid(obj)) > conf_thresh, as the 8-float record
 *   {cx, cy, w, h, det_conf, cls_max_conf, cls_max_id, src}
 * (src: the int32 bits of i*h*w + cy*w + cx, the record's head element --
 * get_region_boxes(validation=True) reads the other classes there; ABI 20)
 * with cx = (sigmoid(tx) + x) * stride_w, w = (exp(tw) * anchor_w) * stride_w
 * (anchors_scaled = HOST [A][2] fp32 anchor / stride), divided by norm_w /
 * norm_h unless 1 (do_detect's normalisation, utils.py:511-515).  Records are
 * appended in order at boxes[b][counts[b] ...] and counts[b] advanced (so the
 * heads of do_detect append one after another); records past `cap` are
 * dropped and *overflow is set to 1. */
int po_region_boxes(const float* head, int B, int A, int C, int h, int w, const float* anchors_scaled,
                    float stride_w, float stride_h, float norm_w, float norm_h, float conf_thresh,
                    int only_objectness, int cap, float* boxes, int32_t* counts, int32_t* overflow, po_stream_t s);
/* nms (utils.py:93-112) per image over boxes[b][0 .. min(counts[b], cap)):
 * sort by fp32(1 - det_conf) ascending (ties: record index), then keep a box
 * unless a kept box before it has bbox_iou (centre form, fp32, utils.py:37-57)
 * > nms_thresh with it, and only if det_conf > 0.  keep [B][cap] = record
 * indices in kept order, nkeep [B].  nmax >= every counts[b] (<= cap, <= 65536);
 * workspaces keys / mask sized by po_nms_workspace(B, nmax).  An image with
 * counts[b] > nmax is processed on its first nmax records only (the
 * workspaces hold nmax), never beyond. */
int po_nms(const float* boxes, const int32_t* counts, int B, int cap, int nmax, float nms_thresh, uint64_t* keys,
           uint64_t* mask, int32_t* keep, int32_t* nkeep, po_stream_t s);
int po_nms_workspace(int B, int nmax, int64_t* key_words, int64_t* mask_words);

/* ---------------- test-time placement (reference load_data.py:985-1722) ---------------- */

/* PatchTransformer_test_mode.forward (load_data.py:1432-1722) for B images at
 * once (the reference runs one image; lab_batch [1, n, 7]):
 *   lab [B, L, 7] fp32 rows {x, y, w, h, obj_conf, cls_conf, id} (normalised),
 *   nlab [B] (DEVICE int32) rows in use per image (1 <= nlab[b] <= L);
 *   patch_mp [3,P,P] the median-pooled patch (clamped to [0,1] here; the
 *   contrast/brightness/noise the reference draws are not applied there);
 *   angle [B] (DEVICE, radians; NULL = 0), upick [B] (DEVICE, U[0,1)) the
 *   draw behind random.randint(0, len(position_available)).
 * Steps: lab_transform (1262-1320: (max-area row + min-area row)/2 over cols
 * 2,3; 0.25 when nlab == 1 or max area > 0.99); theta1 = rotation + scale
 * sqrt((w S/sf)^2 + (h S/sf)^2)/P about the centre, warp of the padded patch
 * and its mask (1617-1635); semi_edge = (max - min)/2 of the rows holding
 * mask == 1 (1650-1664); inter_axis_cal's occupancy map (1322-1430: border
 * of int(semi_edge), label boxes grown by semi_edge in area order, the early
 * exit and its temp_lab[0:i-1] sum, Python slice semantics of the int()
 * bounds; the map is indexed [x][y]); position = the upick-th free cell in
 * torch.nonzero order (1678-1687); theta2 = translation to it and a second
 * bilinear resampling of the warped patch and mask (1689-1706); out =
 * clamp(adv) * msk (1714-1715).  Sampling geometry in float64, each resampled
 * value rounded once to fp32; msk == 1 is tested on that fp32 value.
 *   out [B,3,S,S]; info [B,8] int32 (DEVICE) = {flags, x, y, semi_edge*2,
 *   M, n_free, pick, rows_eq1}; flags bit 1: fewer than two mask==1 pixels
 *   (the reference fails in torch.min / the squeeze), 2: no free cell (its
 *   position_available[0] raises), 4: the pick equals n_free (its randint's
 *   inclusive bound: IndexError).  Flagged images get a zero output.
 * Workspace (po_place_workspace): fwork >= 4*B*S*S + 16*B floats (8-byte
 * aligned), iwork >= B*(S*S + 5*L + 16) int32 (16-byte aligned). */
int po_place_test_mode(const float* patch_mp, int P, const float* lab, const int32_t* nlab, int B, int L, int S,
                       float scale_factor, const float* angle, const float* upick, float* fwork, int32_t* iwork,
                       float* out, int32_t* info, po_stream_t s);
int po_place_workspace(int B, int L, int S, int64_t* fwords, int64_t* iwords);
/* inter_axis_cal alone (load_data.py:1322-1430) for a given semi_edge [B]
 * (DEVICE fp32): layout [B,S,S] int32 indexed [x][y] as the reference's map,
 * 0 where its returned sum is 0 (the free cells), 1 elsewhere (the layer
 * count itself is not reproduced; the reference only reads its zeros).
 * Workspaces as po_place_test_mode. */
int po_place_free_map(const float* lab, const int32_t* nlab, int B, int L, int S, const float* semi_edge,
                      float* fwork, int32_t* iwork, int32_t* layout, po_stream_t s);

/* PatchTransformer_vanishing placement (load_data.py:1095-1180): one patch
 * per label row, lab [B, L, 5] {cls, x, y, w, h}; target size
 * sqrt((w S/pre)^2 + (h S/pre)^2) (pre_scale 8, 1116-1120), centre (x, y)
 * (+ w*offx, h*offy with rand_loc, 1131-1147; x -/+ w/6 for orient 1 left /
 * 2 right, 1158-1162), rotation angle[B*L] (NULL = 0); single-stage theta
 * (1164-1178).  affine [B*L, 6] float64 pixel-space sampling maps for
 * po_warp_fwd / po_warp_composite_multi; roi [B*L, 4] footprint boxes. */
int po_vanishing_params(const float* lab, int B, int L, int S, int P, float pre_scale, const float* angle,
                        const float* offx, const float* offy, int orient, double* affine, int32_t* roi,
                        po_stream_t s);
/* Fused po_warp_fwd (mode 0) of L patches per image + PatchApplier's
 * sequential composite (load_data.py:808-833): out[b] = img[b] with, per
 * element, the value of the LAST patch l whose clamp(adv)*msk there is
 * non-zero.  noise [B*L,3,P,P], contrast/bright [B*L], affine/roi from
 * po_vanishing_params; noise == NULL: no augmentation (test_real). */
int po_warp_composite_multi(const float* img, const float* patch_mp, const float* noise, const float* contrast,
                            const float* bright, const double* affine, const int32_t* roi, int B, int L, int S,
                            int P, float* out, po_stream_t s);

/* ---------------- network ops (reference darknet_v3.py:37-100, 195-220) ---------------- */

/* Tap list of an implicit-GEMM convolution launch.  For output pixel (b,i,j)
 * of the launch grid and tap t the source pixel is
 *   (b, i*in_step + dh[t], j*in_step + dw[t])  (zero outside [0,Hin)x[0,Win))
 * and the destination is (b, i*out_step + out_oy, j*out_step + out_ox).
 * Window buffers (in_org / out_org non-NULL, [B,2] int32 DEVICE, the
 * per-image (row, col) map position of the buffer's pixel (0,0)): the source
 * pixel becomes (i + out_org[b] + dh[t] - in_org[b]) in the source buffer's
 * own coordinates (zero outside it); requires in_step = out_step = 1 and
 * out_oy = out_ox = 0. */
typedef struct po_conv_desc {
  int B;
  int Hin, Win, Cin_p;        /* source tensor (NHWC, channel stride Cin_p) */
  int Hout, Wout, Cout_p;     /* destination tensor (NHWC, channel stride Cout_p) */
  int Hg, Wg;                 /* launch grid (output pixels computed per image) */
  int in_step, out_step, out_oy, out_ox;
  int ntaps;
  int dh[9], dw[9];
  int N;                      /* output channels computed (<= Cout_p, multiple of 16) */
  int act;                    /* 0 linear, 1 leaky(0.1) */
  int accumulate;             /* 1: out = acc + out_prev (dst read) */
  int tile;                   /* 0: built-in heuristic; 1..PO_CONV_NTILES: fixed tile
                                 (po_conv_tile_info), chosen by the caller's autotuner */
  const int32_t* in_org;      /* NULL: full-map source */
  const int32_t* out_org;     /* NULL: full-map destination */
  int ksplit;                 /* <= 1: one pass over K; > 1: the k-steps are split over
                                 ksplit workgroups per tile whose partial sums (workspace,
                                 >= ksplit*M*N floats, M = B*Hg*Wg) are reduced in split
                                 order by a second kernel that applies the epilogue,
                                 or inside the launch (tile_ctr below) */
  float* workspace;
  /* Operand precision.  0: exact fp32 MFMA (v_mfma_f32_32x32x2_f32); W is fp32
   * [N][ntaps][Cin_p].  1: split fp16 ("fp16x3"): every operand x is scaled by
   * a power of two s and written as x*s = hi + lo with hi = fp16(x*s),
   * lo = fp16(x*s - hi); the product uses hi*hi' + hi*lo' + lo*hi' on
   * v_mfma_f32_32x32x16_f16 with fp32 accumulation and is scaled back
   * exactly (relative error per product <= ~3*2^-22).
   * W is then fp16 [2][N][ntaps][Cin_p] (hi plane, lo plane) of the fp32
   * weights times 2^w_shift, and in_amax must point at the max|in| slot. */
  int prec;
  int w_shift;
  /* Per-tensor max|x| slots (DEVICE): a slot is PO_AMAX_SUB uint32 holding float
   * bits, atomicMax'd by writers spread over the sub-slots; the tensor's bound
   * is the max over them.  The caller zeroes a slot before its tensor is
   * first written.  in_amax:
   * an upper bound of max|in| (required for prec 1, written by the kernels that
   * produced `in`); y_amax / sum_amax / y2_amax (each may be NULL): receive
   * max|y_out| / max|sum_out| / max|y2_out| of the values this launch writes. */
  const uint32_t* in_amax;
  uint32_t* y_amax;
  uint32_t* sum_amax;
  uint32_t* y2_amax;
  /* Leaky masks as sign bits ([pixel][Cout_p/32] uint32 words, bit c%32 of word
   * c/32 = (value of channel c > 0); need N % 32 == 0 and Cout_p % 32 == 0).
   * ybits: written with the signs of y_out (each launch writes whole words of
   * the pixels/channels it computes).  mbits / m2bits (each may be NULL):
   * replace mask_y / mask2 (leaky'(v) = bit ? 1 : 0.1), 1/32 of their bytes. */
  uint32_t* ybits;
  const uint32_t* mbits;
  const uint32_t* m2bits;
  /* Gradient cones (optional, DEVICE [B][4] int32 = {r0, c0, r1, c1} per image,
   * half-open, destination-map coordinates; po_grad_boxes): only the grid
   * points whose destination pixel lies in the image's box are computed, the
   * rest of the destination is left untouched.  Needs a full-map destination
   * (out_org = NULL). */
  const int32_t* gbox;
  /* Optional (prec 1, tiles 57..60): the split fp16 weights W in MFMA fragment
   * order, [2][N/32][ntaps][Cin_p/16][64][8] halves: element (lane l, e) of
   * block (nb, tap, c) is W[32 nb + (l & 31)][tap][16 c + 8 (l >> 5) + e].
   * Needs N % 32 == 0; NULL: those tiles do not apply. */
  const void* Wfrag;
  /* Optional (prec 0, tile 61): Winograd F(2x2,3x3) weights of this launch,
   * U = G g G^T in float64 rounded to fp32 (g = the launch's 3x3 taps mapped
   * onto the canonical offsets -1..1), stored in MFMA fragment order
   * [N/32][Cin_p/16][16 components][2][64 lanes][4]: element (lane l, s) of
   * block (nb, kc, xi), U[xi][16 kc + 8 (l >> 5) + s][32 nb + (l & 31)], sits
   * at [nb][kc][xi][s >> 2][l][s & 3].  NULL: the Winograd tiles do not apply. */
  const float* Wwino;
  /* GEMM rows per image (0: Hg*Wg).  With gbox, mrows < Hg*Wg enumerates each
   * image's box compactly when every box holds at most mrows grid points: a
   * dgrad from a receptive-field window (nonzero only on the window dilated by
   * the taps) runs over that box instead of the whole map.  Generic tiles only
   * (staging 0/1). */
  int mrows;
  /* Optional fused k=2 stride-2 max pool of a plain forward conv (y_out NULL,
   * full even grid, no split-K; generic tiles, or Winograd tiles 61/66/67/68/70/71/72/73
   * without gbox -- the windows lie inside their output tiles): pool_y [B,Hout/2,Wout/2,Cout_p]
   * and pool_argmax (int8, same shape) as po_maxpool2_fwd writes them, the
   * argmax bytes of a leaky conv also carrying its LeakyReLU slope (bit 3
   * set, bit 2 = max <= 0; see po_conv_first_pool_fwd); the conv output
   * itself is not stored (darknet_v3.py:61-69 conv + maxpool pairs). */
  float* pool_y;
  int8_t* pool_argmax;
  /* Optional (prec 0, tile 71, ABI 23): Winograd F(4x4,3x3) weights of this
   * launch, U = G g G^T (Lavin's G for the points 0, +-1, +-2, inf) in
   * float64 rounded to fp32, in MFMA fragment order [N/32][Cin_p/16][36
   * components][2][64 lanes][4] (Wwino's order with 36 components).  NULL:
   * tile 71 does not apply. */
  const float* Wwino6;
  /* Optional (tile 72, ABI 24): DEVICE workspace of winov_floats floats for the
   * transformed input V = B^T d B the tile writes before its GEMM:
   * ceil(B*ceil(Hout/4)*ceil(Wout/4)/32) * (Cin_p/16) * 18432 floats.  NULL:
   * tile 72 does not apply. */
  float* winov;
  int64_t winov_floats;
  /* Optional (ABI 28): DEVICE int32 arrival counters, tile_ctr_n of them, all
   * zero between launches (the caller zeroes them once; every launch leaves
   * them zero).  With ksplit > 1 on the generic exact-fp32 tiles (1..20, 27)
   * and at most tile_ctr_n output tiles, the split-K reduction runs inside the
   * launch: each slice publishes its partial sums (agent-scope release, then
   * an agent-scope arrival count on its tile's counter) and the tile's last
   * arriving workgroup sums the slices in split order and applies the
   * epilogue -- the same arithmetic, in the same order, as the separate
   * reduction kernel (bit-identical), one kernel boundary fewer.  NULL (or
   * too few counters, or other tiles): the separate reduction kernel.  Two
   * launches that may run concurrently need separate counter arrays. */
  int32_t* tile_ctr;
  int tile_ctr_n;
} po_conv_desc;

#define PO_CONV_NTILES 73
/* Tile `t` (1-based): block rows BM (output pixels), block columns BN (output
 * channels), k-step BK (input channels).  Tiles 1..10 stage operands through
 * registers, 11..20 are the same shapes staged by LDS-DMA, 27 a 128x256
 * LDS-DMA block; these are the exact-fp32 (prec 0) tiles.  29..54 are fp16x3
 * (prec 1) tiles: register staging, LDS-DMA multi-stage (46..52) and the row
 * halo kernel for stride-1 3x3 convs (53..54); 55..56 are the 2-D tile halo
 * kernel (8 x 16 output pixels per tile) for 3x3 convs of input step 1 or 2 on
 * full maps without split-K or boxes; 57..60 the same 2-D tiles (and 16 x
 * 16-pixel ones at input step 1) reading the weights as MFMA fragments from
 * Wfrag.  61, 65..68 are the exact-fp32 Winograd F(2x2,3x3) kernels (61: 64
 * 2x2-tiles x 32 channels; 65/66: 32 tiles x 64 channels with LDS-DMA input,
 * 65 in 8 scheduled waves, 66 in 4-wave workgroups with 64 KB of LDS, two per
 * CU, bit-identical to 65; 67: 64 tiles x 64 channels per 512-thread
 * workgroup, register-staged input and a pipelined k-loop, bit-identical to
 * 65/66; 68: 67 with the two waves of every SIMD staggered; 16 input channels
 * per k-step) for stride-1 3x3 convs and their input gradients on full maps,
 * without split-K except on 66/67/68 (needs Wwino; 65..68 need N % 64 == 0).
 * 69 (exact fp32, ABI 19) is a persistent direct kernel for a stride-1 3x3
 * conv with Cin_p = 16, N = 32 and pool_y set (full even maps, no split-K, no
 * boxes, only the pooled outputs): 8 x 16-pixel tiles whose input patch is
 * staged once, weights held in registers, pool in registers; bit-identical
 * to the generic tiles.
 * 70 (exact fp32, ABI 21) is tile 68 as a persistent kernel: one 512-thread
 * workgroup per CU walks the launch's (64 tiles x 64 channels x split-K
 * slice) units and issues each unit's stores after the next unit's first
 * input rows, so they drain under its k-loop; full maps without boxes, at
 * least two k-steps per slice, leaky masks as sign bits, no max|x| slots;
 * bit-identical to 68.
 * 71 (exact fp32, ABI 23) is the Winograd F(4x4,3x3) form of tile 70 (needs
 * Wwino6): 32 4x4-tiles x 64 channels per unit, one 512-thread workgroup per
 * CU walking the units; the same requirements as tile 70; since round 6 (no
 * ABI change) also the fused pool (pool_y on a plain full-map forward, even
 * map, no split-K: each 4x4 tile's four windows pooled in the epilogue).
 * Not bit-identical to the F(2x2) tiles (a different exact-arithmetic
 * factorisation); its error against float64 is tested per layer.
 * 72 (exact fp32, ABI 24) is tile 71 with its input transform as a separate
 * pass into winov: the GEMM kernel then loads its A fragments like its B
 * fragments (no gathers, transform or LDS in its k-loop); the same
 * requirements as tile 71 plus winov; the same results as tile 71 bit for bit.
 * 73 (exact fp32, ABI 29) is tile 69's launch (stride-1 3x3, Cin_p = 16, N =
 * Cout_p = 32, pool_y, full even maps, no split-K or boxes) as Winograd
 * F(2x2,3x3) (needs Wwino): a persistent kernel whose 2x2 output tiles are the
 * pool windows, the component GEMMs on v_mfma_f32_16x16x4_f32 with the
 * inverse transform, bias, LeakyReLU and pool in registers; bit-identical to
 * tile 61 on the same launch.
 * Retired tiles (21..26, 28, 62..64: never selected by a tuner run) keep their
 * numbers; po_conv_tile_info reports them with *prec = -1 and po_conv refuses
 * them.  A tile that does not apply to a launch makes po_conv return
 * PO_EINVAL.  Returns PO_EINVAL for a bad index. */
int po_conv_tile_info(int t, int* bm, int* bn, int* bk, int* prec);

/* v[m][n] = act(sum_k A[m][k] * W[n][k] + bias[n]) (+ y_out[m][n] if accumulate);
 * W [N][ntaps][Cin_p] (BN folded on the host).
 *   y_out[m][n]  = mask_y ? v * leaky'(mask_y[m][n]) : v
 *   sum_out      = v + res            (fused shortcut, darknet_v3.py:205-207;
 *                                      res/sum_out both NULL or both set)
 *   y2_out       = v * leaky'(mask2)  (dgrad dual output: the gradient of the
 *                                      conv feeding a shortcut, taken from the
 *                                      completed shortcut gradient; y2_out and
 *                                      mask2 both NULL or both set)
 * All outputs share the destination layout (pixel-major, stride Cout_p).
 * y_out may be NULL for a forward launch (no accumulate, mask_y, mbits or
 * y2_out) that writes sum_out or ybits: an activation read only as a LeakyReLU
 * mask need not be stored. */
int po_conv(const po_conv_desc* d, const float* in, const float* W, const float* bias,
            float* y_out, const float* res, float* sum_out, const float* mask_y,
            float* y2_out, const float* mask2, po_stream_t s);

/* First layer, 3 input channels NCHW image -> NHWC Cout_p (VALU direct conv):
 * y = leaky(conv3x3(img, W[Cout][27]) + bias). */
int po_conv_first_fwd(const float* img, int B, int H, int W, int stride, const float* Wt,
                      const float* bias, int Cout, int Cout_p, int act, float* y, uint32_t* amax,
                      po_stream_t s);
/* po_conv_first_fwd (stride 1) followed by the k=2 stride-2 max pool, fused
 * (yolov3-tiny's conv 3->16 + maxpool, darknet_v3.py:61-69; reference ops
 * nn.Conv2d + nn.LeakyReLU + nn.MaxPool2d).  y [B,H/2,W/2,Cout_p] is the pool
 * output and argmax [B,H/2,W/2,Cout_p] its window position (bits 0-1) as in
 * po_maxpool2_fwd, plus (act = leaky) bit 3 set and bit 2 = (max <= 0): the conv output is
 * not stored, and po_maxpool2_bwd / _bwd_box with mask_y == NULL apply the
 * LeakyReLU slope encoded there (valid when the pool is the conv's only
 * consumer).  Cout_p 16 or 32. */
int po_conv_first_pool_fwd(const float* img, int B, int H, int W, const float* Wt, const float* bias, int Cout,
                           int Cout_p, int act, float* y, int8_t* argmax, uint32_t* amax, po_stream_t s);
/* The two first-layer forwards on the training step's sparse composite: the
 * input is img except inside each image's quad-widened footprint box of roi
 * (po_warp_box_fwd_keyed, fill = 0), where it is pimg.  A wave whose taps all
 * miss the boxes runs the plain loads; results equal po_conv_first_fwd /
 * _pool_fwd on the materialised composite bit for bit, without the B*3*S*S
 * composite copy.  Square images; po_conv_first_fwd_cmp needs Cout_p <= 32. */
int po_conv_first_fwd_cmp(const float* img, const float* pimg, const int32_t* roi, int B, int H, int W, int stride,
                          const float* Wt, const float* bias, int Cout, int Cout_p, int act, float* y, uint32_t* amax,
                          po_stream_t s);
int po_conv_first_pool_fwd_cmp(const float* img, const float* pimg, const int32_t* roi, int B, int H, int W,
                               const float* Wt, const float* bias, int Cout, int Cout_p, int act, float* y,
                               int8_t* argmax, uint32_t* amax, po_stream_t s);
/* (ABI 25) po_conv_first_pool_fwd / _cmp with the conv as Winograd F(2x2,3x3):
 * each pooled pixel's 2x2 conv window is one F(2x2) output tile.  U [Cout][3][16]
 * = G g G^T of the [Cout][3][3][3] weights (row-major 4x4, G = {{1,0,0},
 * {.5,.5,.5},{.5,-.5,.5},{0,0,1}}; darknet_v3.first_wino_u computes it in
 * float64).  Same outputs, argmax codes and conditions as the direct form; the
 * conv sums differ from it by fp32 rounding only (tests/test_gpu_first_conv.py). */
int po_conv_first_pool_wino_fwd(const float* img, int B, int H, int W, const float* U, const float* bias, int Cout,
                                int Cout_p, int act, float* y, int8_t* argmax, uint32_t* amax, po_stream_t s);
int po_conv_first_pool_wino_fwd_cmp(const float* img, const float* pimg, const int32_t* roi, int B, int H, int W,
                                    const float* U, const float* bias, int Cout, int Cout_p, int act, float* y,
                                    int8_t* argmax, uint32_t* amax, po_stream_t s);
/* Its input gradient: d_img[b,c,h,w] (NCHW) from D [B,Ho,Wo,Cout_p] (already
 * multiplied by leaky'), W [Cout][27].  roi (may be NULL) [B,4] int32
 * {x0,y0,x1,y1}: only pixels x0<=w<x1, y0<=h<y1 of image b are computed (the
 * rest of d_img is left untouched) — the training step only consumes the
 * image gradient inside the patch footprint. */
int po_conv_first_dgrad(const float* D, int B, int H, int W, int stride, const float* Wt,
                        int Cout, int Cout_p, const int32_t* roi, float* d_img, po_stream_t s);

/* dst[m, 0:C] (=|+=) src[m, off:off+C] (optionally * leaky'(y[m,0:C])).
 * strides are channel strides; M pixels. */
int po_slice_accum(const float* src, int src_stride, int src_off, float* dst, int dst_stride,
                   int dst_off, int64_t M, int C, int accumulate, const float* mask_y,
                   int mask_stride, uint32_t* amax, po_stream_t s);
/* Spatially-aware copy between full-map and window buffers (NHWC).  Over
 * every pixel (b,i,j) of dst [B,Hd,Wd] (map position p = (i,j) + dst_org[b]):
 *   mode 0: v = src[p - src_org[b]]                  (route slice)
 *   mode 1: v = src[p/2 - src_org[b]]                (nearest 2x upsample fwd)
 *   mode 2: v = sum_{a,c in {0,1}} src[2p + (a,c) - src_org[b]]  (its backward)
 * src pixels outside the src buffer read 0; channels src[off_s + c], dst[off_d + c];
 * dst (=|+=) v, optionally * leaky'(mask_y) (mask in dst's pixel layout).
 * NULL org = full map.
 * The data-movement entries below and po_conv_first_fwd take an optional
 * `amax` slot (see po_conv_desc): max|value written| is atomicMax'd into it. */
int po_view_move(const float* src, int Hs, int Ws, int src_stride, int src_off, const int32_t* src_org,
                 float* dst, int Hd, int Wd, int dst_stride, int dst_off, const int32_t* dst_org, int B,
                 int C, int mode, int accumulate, const float* mask_y, int mask_stride, uint32_t* amax,
                 po_stream_t s);
/* nearest 2x upsample fwd (darknet_v3.py:103-113): dst[b,2h+y,2w+x, off+c] = src[b,h,w,c]. */
int po_upsample2_fwd(const float* src, int B, int H, int W, int C, int src_stride, float* dst,
                     int dst_stride, int dst_off, uint32_t* amax, po_stream_t s);
/* its backward: dst[b,h,w,c] (=|+=) sum of the 4 src pixels (src at 2H x 2W,
 * channel offset src_off), optionally * leaky'(mask_y). */
int po_upsample2_bwd(const float* src, int src_stride, int src_off, int B, int H, int W, int C,
                     float* dst, int dst_stride, int accumulate, const float* mask_y,
                     int mask_stride, uint32_t* amax, po_stream_t s);
/* max pool k=2 (stride 2, or stride 1 after ZeroPad2d((0,1,0,1)), darknet_v3.py:61-69);
 * argmax [B,Ho,Wo,C] int8 window position. */
int po_maxpool2_fwd(const float* src, int B, int H, int W, int C, int Cp, int stride, float* dst,
                    int8_t* argmax, uint32_t* amax, po_stream_t s);
int po_maxpool2_bwd(const float* d_dst, const int8_t* argmax, int B, int H, int W, int C, int Cp,
                    int stride, float* d_src, int accumulate, const float* mask_y,
                    uint32_t* amax, po_stream_t s);
/* po_maxpool2_bwd restricted to each image's gradient-cone box (boxes[4 b ..]
 * = r0, c0, r1, c1 half-open in the d_src map, from po_grad_boxes); pixels
 * outside the box are not written.  boxes == NULL: the full map. */
int po_maxpool2_bwd_box(const float* d_dst, const int8_t* argmax, int B, int H, int W, int C, int Cp,
                        int stride, float* d_src, int accumulate, const float* mask_y,
                        const int32_t* boxes, uint32_t* amax, po_stream_t s);

/* NCHW [B,C,H,W] <-> NHWC [B,H,W,Cp] layout conversion (heads in and out of
 * the drop-in Darknet.forward API). */
int po_nhwc_to_nchw(const float* src, int B, int H, int W, int C, int Cp, float* dst, po_stream_t s);
int po_nchw_to_nhwc(const float* src, int B, int H, int W, int C, int Cp, float* dst, po_stream_t s);

#ifdef __cplusplus
}
#endif
#endif /* ADVPATCH_H */
