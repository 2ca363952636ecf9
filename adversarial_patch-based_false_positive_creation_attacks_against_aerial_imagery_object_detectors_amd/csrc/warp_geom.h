// Float64 placement geometry shared by the training placement (po_patch_params)
// and the test-time placements (po_place_test_mode, po_vanishing_params).
// Include after `#pragma clang fp contract(off)`: the expressions are the
// reference formulas evaluated in float64, operation by operation.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace po {

// Pixel-space form of affine_grid + grid_sample (align_corners=False) on an
// S x S output: output pixel (i, j) samples the input at column
// ix = af0 j + af1 i + af2 and row iy = af3 j + af4 i + af5.
__device__ __forceinline__ void theta_pixel_affine(const double th[6], double dS, double af[6]) {
  const double half = 0.5 - 0.5 * dS;
  af[0] = th[0];
  af[1] = th[1];
  af[2] = (th[0] + th[1]) * half + 0.5 * dS * th[2] + 0.5 * (dS - 1.0);
  af[3] = th[3];
  af[4] = th[4];
  af[5] = (th[3] + th[4]) * half + 0.5 * dS * th[5] + 0.5 * (dS - 1.0);
}

// The single-stage theta of PatchTransformer (load_data.py:733-743) and
// PatchTransformer_vanishing (1171-1178): rotation by `a`, scale 1/scale,
// translation (tx, ty) in affine_grid units.
__device__ __forceinline__ void placement_theta(double a, double scale, double tx, double ty, double th[6]) {
  const double sn = sin(a), cs = cos(a);
  th[0] = cs / scale;
  th[1] = sn / scale;
  th[2] = tx * cs / scale + ty * sn / scale;
  th[3] = -sn / scale;
  th[4] = cs / scale;
  th[5] = -tx * sn / scale + ty * cs / scale;
}

// Bounding box {x0, y0, x1, y1} (+2 px margin, clipped to the image) of the
// output pixels whose bilinear sample can touch the padded patch region
// [pad-1, pad+P)^2: the preimage of its corners under the pixel-space affine.
__device__ __forceinline__ void footprint_roi(const double af[6], int S, int P, int32_t* roi) {
  const double A00 = af[0], A01 = af[1], A02 = af[2], A10 = af[3], A11 = af[4], A12 = af[5];
  const double det = A00 * A11 - A01 * A10;
  const int padL = (int)((S - P) / 2.0 + 0.5);
  double jlo = 1e30, jhi = -1e30, ilo = 1e30, ihi = -1e30;
  for (int k = 0; k < 4; ++k) {
    const double X = (double)((k & 1) ? padL + P : padL - 1) - A02;
    const double Y = (double)((k & 2) ? padL + P : padL - 1) - A12;
    const double jj = (A11 * X - A01 * Y) / det, ii = (-A10 * X + A00 * Y) / det;
    jlo = fmin(jlo, jj); jhi = fmax(jhi, jj);
    ilo = fmin(ilo, ii); ihi = fmax(ihi, ii);
  }
  if (!(det != 0.0) || !(jlo <= jhi) || !(ilo <= ihi)) {    // degenerate or non-finite map: empty box
    roi[0] = roi[1] = roi[2] = roi[3] = 0;
    return;
  }
  const double dS = (double)S, lo = -4.0, hi = dS + 4.0;      // clamp before the int conversion
  jlo = fmin(fmax(jlo, lo), hi); jhi = fmin(fmax(jhi, lo), hi);
  ilo = fmin(fmax(ilo, lo), hi); ihi = fmin(fmax(ihi, lo), hi);
  roi[0] = max(0, (int)floor(jlo) - 2);
  roi[1] = max(0, (int)floor(ilo) - 2);
  roi[2] = min(S, (int)ceil(jhi) + 3);
  roi[3] = min(S, (int)ceil(ihi) + 3);
}

// ---------------------------------------------------------------------------
// Reference geometry (po_patch_params geometry 1; ABI 27): the placement as
// the reference computes it on PyTorch-CPU in fp32 (load_data.py:726-749),
// every rounding restated from ATen / MKL and pinned bit for bit against the
// installed torch by tests/test_geometry_ref.py (oracle/geometry_ref.py):
//   theta        cos/scale, sin/scale, tx*cos/scale + ty*sin/scale, ...   738-743
//   affine_grid  base b(k) = fl(fl(linspace_k * (S-1)) / S), linspace_k =
//                fma(step, k, -1) (k < S/2) or fma(-step, S-1-k, 1), step =
//                fl(2/(S-1)); x = bx*t0 + by*t1 + t2 through MKL's sgemm,
//                whose code path depends on the host CPU: on AMD EPYC (the
//                MI355X hosts) fl(fl(fl(bx*t0) + fl(by*t1)) + t2) -- geometry 1;
//                on Intel AVX-512 fl(fma(by, t1, fl(bx*t0)) + t2) -- geometry 2
//                (load_data.reference_bmm_form() asks the host's torch) 745
//   grid_sample  ix = fma(x + 1, S/2, -0.5); bilinear weights s*e, s*w, n*e,
//                n*w; value = fma chain over the corners nw, ne, sw, se   748-749
// An affine row [6] float64 in this form holds the six fp32 theta values as
// float[6] in its first 24 bytes and a tag in row[3] -- AFFINE_REF_TAG + 1 or
// + 2 (the geometry), signalling-NaN bit patterns, which no arithmetic
// produces, so a float64-form row (the pixel-space map of theta_pixel_affine)
// never carries one.
// ---------------------------------------------------------------------------
constexpr unsigned long long AFFINE_REF_TAG = 0x7FF4A0F3E5F32000ull;

// Per-image placement of the warp kernels: the form, the fp32 theta (reference
// form) and a float64 pixel-space map (the map itself in the float64 form; in
// the reference form its float64 evaluation, used only for footprint boxes and
// candidate searches, whose margins cover the fp32 rounding).
struct Geo {
  double af[6];
  float th[6];
  int ref;      // 0: float64 pixel-space map; 1 / 2: the reference's fp32 arithmetic, sgemm form 1 / 2
};

// the geometry of a row: 0 (float64 form), 1 or 2 (reference forms)
__device__ __forceinline__ int affine_row_form(const double* row) {
  const unsigned long long t = (unsigned long long)__double_as_longlong(row[3]);
  return (t == AFFINE_REF_TAG + 1) ? 1 : (t == AFFINE_REF_TAG + 2) ? 2 : 0;
}

__device__ __forceinline__ Geo load_geo(const double* row, int S) {
  Geo G;
  G.ref = affine_row_form(row);
  if (G.ref) {
    const float* t = reinterpret_cast<const float*>(row);
    double th[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      G.th[k] = t[k];
      th[k] = (double)t[k];
    }
    theta_pixel_affine(th, (double)S, G.af);
  } else {
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      G.af[k] = row[k];
      G.th[k] = 0.f;
    }
  }
  return G;
}

__device__ __forceinline__ void store_ref_row(const float th[6], int form, double* row) {
  float* t = reinterpret_cast<float*>(row);
#pragma unroll
  for (int k = 0; k < 6; ++k) t[k] = th[k];
  row[3] = __longlong_as_double((long long)(AFFINE_REF_TAG + (unsigned long long)form));
  row[4] = 0.0;
  row[5] = 0.0;
}

// The reference-form functions below spell out every rounding: plain fp32
// operators under a block-scope `fp contract(off)` (HIP's __fmul_rn and
// friends are plain operators in a header compiled with contraction allowed,
// so an __fadd_rn(__fmul_rn(..)) pair may still fuse -- measured: it did in
// one kernel and not in another) and __builtin_fmaf where the reference fuses.

// affine_grid's base coordinate k of an S-point axis (align_corners=False):
// fl(fl(lin * (S-1)) / S), lin = fma(step, k, -1) (k < S/2) or fma(-step,
// S-1-k, 1), step = fl(2/(S-1)).  The division is formed from the correctly
// rounded reciprocal rcp = fl(1/S) with one Markstein step, q = fl(x rcp),
// r = fma(-q, S, x), fma(r, rcp, q), which equals fl(x / S) for every k < S
// of every axis S <= 32768 (checked exhaustively: tests/test_geometry_ref.py,
// oracle/geometry_ref.py base32_markstein): five operations per coordinate
// instead of a correctly rounded division.  step and rcp are per-launch
// constants (RefAxis, formed once on the host).
struct RefAxis {
  float step, rcp;
  int S;
};
__host__ __device__ inline RefAxis ref_axis(int S) {
  RefAxis a;
  a.S = S;
  a.step = S > 1 ? 2.0f / (float)(S - 1) : 0.0f;
  a.rcp = 1.0f / (float)S;
  return a;
}
__device__ __forceinline__ float ref_base(int k, const RefAxis& a) {
#pragma clang fp contract(off)
  const int S = a.S;
  const float fS = (float)S, fS1 = (float)(S - 1);
  const float lin = k < (S >> 1) ? __builtin_fmaf(a.step, (float)k, -1.0f) : __builtin_fmaf(-a.step, (float)(S - 1 - k), 1.0f);
  const float x = lin * fS1;
  if (S > 32768) return x / fS;
  const float q = x * a.rcp;
  return __builtin_fmaf(__builtin_fmaf(-q, fS, x), a.rcp, q);
}

// grid_sample's source coordinate (column ix, row iy) of output pixel (i, j);
// form: the host sgemm's order of the K = 3 dot product (see above)
__device__ __forceinline__ void ref_sample_coord(const float th[6], int form, const RefAxis& a, int i, int j,
                                                 float& ix, float& iy) {
#pragma clang fp contract(off)
  const float bx = ref_base(j, a), by = ref_base(i, a);
  float gx, gy;
  if (form == 2) {
    gx = __builtin_fmaf(by, th[1], bx * th[0]) + th[2];
    gy = __builtin_fmaf(by, th[4], bx * th[3]) + th[5];
  } else {
    gx = (bx * th[0] + by * th[1]) + th[2];
    gy = (bx * th[3] + by * th[4]) + th[5];
  }
  const float half = (float)a.S * 0.5f;
  ix = __builtin_fmaf(gx + 1.0f, half, -0.5f);
  iy = __builtin_fmaf(gy + 1.0f, half, -0.5f);
}

// the reference theta from its fp32 inputs (load_data.py:738-743)
__device__ __forceinline__ void ref_theta(float sn, float cs, float sc, float tx, float ty, float th[6]) {
#pragma clang fp contract(off)
  th[0] = cs / sc;
  th[1] = sn / sc;
  th[2] = (tx * cs) / sc + (ty * sn) / sc;
  th[3] = (-sn) / sc;
  th[4] = cs / sc;
  th[5] = ((-tx) * sn) / sc + (ty * cs) / sc;
}

// The composite's written box of image b (po_warp_fwd_pre, po_warp_box_fwd_keyed):
// the footprint box widened to whole 4-pixel quads, [qx0, qx1) x [y0, y1) (all
// zero when empty).  Outside it the composite equals the image (mode 1), so a
// consumer given both tensors (po_conv_first_fwd_cmp) reads the composite only
// inside this box.
struct QBox {
  int qx0, qx1, y0, y1;
};
__device__ __forceinline__ QBox quad_box(const int32_t* roi, int b, int S) {
  const int4 r = reinterpret_cast<const int4*>(roi)[b];
  QBox q;
  q.qx0 = r.x & ~3;
  q.qx1 = min(S, (r.z + 3) & ~3);
  q.y0 = r.y;
  q.y1 = r.w;
  if (q.qx1 <= q.qx0 || q.y1 <= q.y0) q.qx0 = q.qx1 = q.y0 = q.y1 = 0;
  return q;
}

}  // namespace po
