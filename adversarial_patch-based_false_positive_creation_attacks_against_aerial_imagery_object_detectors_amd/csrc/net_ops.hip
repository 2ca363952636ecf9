// Data-movement ops of the Darknet graph (route / upsample / maxpool / layout),
// forward and backward, NHWC fp32 with padded channel strides.
// Reference: darknet_v3.py:61-113 (maxpool, upsample), 202-207 (route, shortcut).
#include "common.h"

namespace {
__global__ __launch_bounds__(256) void slice_accum_k(const float* __restrict__ src, int ss, int so,
                                                     float* __restrict__ dst, int ds, int doff,
                                                     int64_t M, int C, int acc,
                                                     const float* __restrict__ my, int ms,
                                                     uint32_t* __restrict__ amax) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  float v = 0.f;
  if (t < M * C) {
    const int64_t m = t / C;
    const int c = (int)(t - m * C);
    v = src[m * ss + so + c];
    float* d = dst + m * ds + doff + c;
    if (acc) v += *d;
    if (my) v *= po::leaky_grad(my[m * ms + c]);
    *d = v;
  }
  if (amax) po::amax_commit(amax, fabsf(v));
}

// window <-> full-map moves (po_view_move): one thread per dst element
__global__ __launch_bounds__(256) void view_move_k(const float* __restrict__ src, int Hs, int Ws, int ss, int so,
                                                   const int32_t* __restrict__ sorg, float* __restrict__ dst,
                                                   int Hd, int Wd, int ds, int doff,
                                                   const int32_t* __restrict__ dorg, int B, int C, int mode,
                                                   int acc, const float* __restrict__ my, int ms,
                                                   uint32_t* __restrict__ amax) {
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t tot = (int64_t)B * Hd * Wd * C;
  const bool live = t0 < tot;
  const int64_t t = live ? t0 : 0;
  const int c = (int)(t % C);
  const int64_t p = t / C;
  const int x = (int)(p % Wd);
  const int y = (int)((p / Wd) % Hd);
  const int b = (int)(p / ((int64_t)Wd * Hd));
  const int py = y + (dorg ? dorg[2 * b] : 0), px = x + (dorg ? dorg[2 * b + 1] : 0);   // map position
  const int oy = sorg ? sorg[2 * b] : 0, ox = sorg ? sorg[2 * b + 1] : 0;
  auto at = [&](int my_, int mx_) -> float {      // src at map position, 0 outside the buffer
    const int ly = my_ - oy, lx = mx_ - ox;
    if (ly < 0 || ly >= Hs || lx < 0 || lx >= Ws) return 0.f;
    return src[(((int64_t)b * Hs + ly) * Ws + lx) * ss + so + c];
  };
  float v = 0.f;
  if (live) {
    if (mode == 0) v = at(py, px);
    else if (mode == 1) v = at(py >> 1, px >> 1);
    else v = (at(2 * py, 2 * px) + at(2 * py, 2 * px + 1)) + (at(2 * py + 1, 2 * px) + at(2 * py + 1, 2 * px + 1));
    float* d = dst + p * ds + doff + c;
    if (acc) v += *d;
    if (my) v *= po::leaky_grad(my[p * ms + c]);
    *d = v;
  }
  if (amax) po::amax_commit(amax, fabsf(v));
}

__global__ __launch_bounds__(256) void up2_fwd_k(const float* __restrict__ src, int B, int H, int W,
                                                 int C, int ss, float* __restrict__ dst, int ds,
                                                 int doff, uint32_t* __restrict__ amax) {
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t tot = (int64_t)B * 2 * H * 2 * W * C;
  const bool live = t0 < tot;
  const int64_t t = live ? t0 : 0;
  const int c = (int)(t % C);
  int64_t p = t / C;                       // output pixel (b, y, x) at 2H x 2W
  const int x = (int)(p % (2 * W));
  p /= 2 * W;
  const int y = (int)(p % (2 * H));
  const int b = (int)(p / (2 * H));
  float v = 0.f;
  if (live) {
    v = src[(((int64_t)b * H + y / 2) * W + x / 2) * ss + c];   // nearest: floor(dst/2)
    dst[(((int64_t)b * 2 * H + y) * 2 * W + x) * ds + doff + c] = v;
  }
  if (amax) po::amax_commit(amax, fabsf(v));
}

__global__ __launch_bounds__(256) void up2_bwd_k(const float* __restrict__ src, int ss, int so, int B,
                                                 int H, int W, int C, float* __restrict__ dst, int ds,
                                                 int acc, const float* __restrict__ my, int ms,
                                                 uint32_t* __restrict__ amax) {
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t tot = (int64_t)B * H * W * C;
  const bool live = t0 < tot;
  const int64_t t = live ? t0 : 0;
  const int c = (int)(t % C);
  const int64_t p = t / C;
  const int x = (int)(p % W);
  const int y = (int)((p / W) % H);
  const int b = (int)(p / ((int64_t)W * H));
  const float* s0 = src + (((int64_t)b * 2 * H + 2 * y) * 2 * W + 2 * x) * ss + so + c;
  const int64_t rs = (int64_t)2 * W * ss;
  float v = 0.f;
  if (live) {
    v = (s0[0] + s0[ss]) + (s0[rs] + s0[rs + ss]);
    float* d = dst + p * ds + c;
    if (acc) v += *d;
    if (my) v *= po::leaky_grad(my[p * ms + c]);
    *d = v;
  }
  if (amax) po::amax_commit(amax, fabsf(v));
}

// k=2 max pool; stride 2 (no padding) or stride 1 over ZeroPad2d((0,1,0,1)).
// Grid: x = one output row (b, y), y = 256-thread slices of that row's
// (pixel, 4-channel group) pairs: each thread moves 16 bytes per pixel and
// needs one 32-bit division for its indices.
__global__ __launch_bounds__(256) void maxpool2_fwd_k(const float* __restrict__ src, int B, int H, int W,
                                                      int C, int Cp, int stride, int Ho, int Wo,
                                                      float* __restrict__ dst, int8_t* __restrict__ am,
                                                      uint32_t* __restrict__ amax) {
  const int row = blockIdx.x, b = row / Ho, y = row - b * Ho;
  const int c4n = Cp >> 2;
  const int q = blockIdx.y * 256 + threadIdx.x;
  float vmax = 0.f;
  if (q < Wo * c4n) {
    const int x = q / c4n, c = (q - x * c4n) * 4;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    int arg[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int yy = y * stride + (k >> 1), xx = x * stride + (k & 1);
      // outside the source = the zero padding of ZeroPad2d (stride-1 case)
      const float4 v4 = (yy < H && xx < W)
                            ? *reinterpret_cast<const float4*>(src + (((int64_t)b * H + yy) * W + xx) * Cp + c)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
      const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (k == 0 || v[u] > bv[u] || isnan(v[u])) { bv[u] = v[u]; arg[u] = k; }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (c + u >= C) { bv[u] = 0.f; arg[u] = 0; }
    const int64_t o = ((int64_t)row * Wo + x) * Cp + c;
    *reinterpret_cast<float4*>(dst + o) = make_float4(bv[0], bv[1], bv[2], bv[3]);
    *reinterpret_cast<char4*>(am + o) = make_char4((char)arg[0], (char)arg[1], (char)arg[2], (char)arg[3]);
    vmax = fmaxf(fmaxf(fabsf(bv[0]), fabsf(bv[1])), fmaxf(fabsf(bv[2]), fabsf(bv[3])));
  }
  if (amax) po::amax_commit(amax, vmax);
}

// gather form: each source pixel sums, in window-position order, the outputs
// whose argmax selected it
// One (pixel, 4 channels) of the max-pool input gradient: the window
// positions k of the (up to 4) outputs whose window holds the pixel.
__device__ __forceinline__ float mp_bwd_px(const float* __restrict__ dd, const int8_t* __restrict__ am, int b, int y,
                                           int x, int c, int H, int W, int C, int Cp, int stride, int Ho, int Wo,
                                           float* __restrict__ ds, int acc, const float* __restrict__ my) {
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  // argmax bytes of po_conv_first_pool_fwd carry the LeakyReLU slope of the
  // (unstored) pool input at the argmax: bit 3 set, bit 2 = slope 0.1
  float lg[4] = {1.f, 1.f, 1.f, 1.f};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int ty = y - (k >> 1), tx = x - (k & 1);
    if (ty < 0 || tx < 0 || ty % stride || tx % stride) continue;
    const int oy = ty / stride, ox = tx / stride;
    if (oy >= Ho || ox >= Wo) continue;
    const int64_t o = (((int64_t)b * Ho + oy) * Wo + ox) * Cp + c;
    const char4 a = *reinterpret_cast<const char4*>(am + o);
    const float4 g = *reinterpret_cast<const float4*>(dd + o);
    const int ak[4] = {a.x, a.y, a.z, a.w};
    const float gk[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if ((ak[u] & 3) == k) {
        v[u] += gk[u];
        if (ak[u] & 8) lg[u] = (ak[u] & 4) ? 0.1f : 1.f;
      }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (c + u >= C) v[u] = 0.f;
  const int64_t t = (((int64_t)b * H + y) * W + x) * Cp + c;
  if (acc) {
    const float4 p = *reinterpret_cast<const float4*>(ds + t);
    v[0] += p.x; v[1] += p.y; v[2] += p.z; v[3] += p.w;
  }
  if (my) {
    const float4 m = *reinterpret_cast<const float4*>(my + t);
    v[0] *= po::leaky_grad(m.x); v[1] *= po::leaky_grad(m.y);
    v[2] *= po::leaky_grad(m.z); v[3] *= po::leaky_grad(m.w);
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] *= lg[u];
  }
  *reinterpret_cast<float4*>(ds + t) = make_float4(v[0], v[1], v[2], v[3]);
  return fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
}

__global__ __launch_bounds__(256) void maxpool2_bwd_k(const float* __restrict__ dd,
                                                      const int8_t* __restrict__ am, int B, int H, int W,
                                                      int C, int Cp, int stride, int Ho, int Wo,
                                                      float* __restrict__ ds, int acc,
                                                      const float* __restrict__ my,
                                                      uint32_t* __restrict__ amax) {
  const int row = blockIdx.x, b = row / H, y = row - b * H;
  const int c4n = Cp >> 2;
  const int q = blockIdx.y * 256 + threadIdx.x;
  float vmax = 0.f;
  if (q < W * c4n) {
    const int x = q / c4n, c = (q - x * c4n) * 4;
    vmax = mp_bwd_px(dd, am, b, y, x, c, H, W, C, Cp, stride, Ho, Wo, ds, acc, my);
  }
  if (amax) po::amax_commit(amax, vmax);
}

// Gradient-cone form: only the pixels of each image's box (boxes[4 b ..] =
// r0, c0, r1, c1, half-open, from po_grad_boxes) are written; the rest of
// d_src is left as it is (nothing downstream of the cone reads it).  Grid
// (B, rows): workgroup (b, r) walks rows r0 + r, r0 + r + gridDim.y, ... of the
// box, its threads the box's columns x channel quads.
__global__ __launch_bounds__(256) void maxpool2_bwd_box_k(const float* __restrict__ dd,
                                                          const int8_t* __restrict__ am, int B, int H, int W,
                                                          int C, int Cp, int stride, int Ho, int Wo,
                                                          float* __restrict__ ds, int acc,
                                                          const float* __restrict__ my,
                                                          const int32_t* __restrict__ boxes,
                                                          uint32_t* __restrict__ amax) {
  const int b = blockIdx.x;
  const int4 bx = reinterpret_cast<const int4*>(boxes)[b];
  const int r0 = max(bx.x, 0), c0 = max(bx.y, 0), r1 = min(bx.z, H), c1 = min(bx.w, W);
  const int c4n = Cp >> 2;
  const int nq = (c1 - c0) * c4n;
  float vmax = 0.f;
  if (c1 > c0) {
    for (int y = r0 + (int)blockIdx.y; y < r1; y += (int)gridDim.y)
      for (int q = threadIdx.x; q < nq; q += 256) {
        const int xr = q / c4n;
        vmax = fmaxf(vmax, mp_bwd_px(dd, am, b, y, c0 + xr, (q - xr * c4n) * 4, H, W, C, Cp, stride, Ho, Wo, ds,
                                     acc, my));
      }
  }
  if (amax) po::amax_commit(amax, vmax);
}

// Stride-2 form on even maps (H = 2 Ho, W = 2 Wo): every source pixel lies in
// exactly one window, so one thread per (pooled pixel, 4 channels) reads that
// output's gradient and argmax bytes once and writes its window's (up to) four
// source pixels inside the box -- instead of four gathering threads re-reading
// them.  Per pixel the arithmetic is mp_bwd_px's (0 + g at the argmax, channel
// mask, accumulate, slope): bit-identical, same pixels written.
__global__ __launch_bounds__(256) void maxpool2_bwd_box_s2_k(const float* __restrict__ dd,
                                                             const int8_t* __restrict__ am, int H, int W,
                                                             int C, int Cp, int Ho, int Wo,
                                                             float* __restrict__ ds, int acc,
                                                             const float* __restrict__ my,
                                                             const int32_t* __restrict__ boxes,
                                                             uint32_t* __restrict__ amax) {
  const int b = blockIdx.x;
  const int4 bx = reinterpret_cast<const int4*>(boxes)[b];
  const int r0 = max(bx.x, 0), c0 = max(bx.y, 0), r1 = min(bx.z, H), c1 = min(bx.w, W);
  const int c4n = Cp >> 2;
  float vmax = 0.f;
  if (c1 > c0 && r1 > r0) {
    const int oy0 = r0 >> 1, oy1 = (r1 + 1) >> 1;       // pooled rows / columns whose windows meet the box
    const int ox0 = c0 >> 1, ox1 = (c1 + 1) >> 1;
    const int nq = (ox1 - ox0) * c4n;
    for (int oy = oy0 + (int)blockIdx.y; oy < oy1; oy += (int)gridDim.y)
      for (int q = threadIdx.x; q < nq; q += 256) {
        const int oxr = q / c4n, c = (q - oxr * c4n) * 4, ox = ox0 + oxr;
        const uint32_t o = ((uint32_t)(b * Ho + oy) * Wo + ox) * Cp + c;     // < 2^31 (host check)
        const char4 a = *reinterpret_cast<const char4*>(am + o);
        const float4 g = *reinterpret_cast<const float4*>(dd + o);
        const int ak[4] = {a.x, a.y, a.z, a.w};
        const float gk[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int y = 2 * oy + (k >> 1), x = 2 * ox + (k & 1);
          if (y < r0 || y >= r1 || x < c0 || x >= c1) continue;
          float v[4], lg[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const bool sel = (ak[u] & 3) == k;
            v[u] = sel ? 0.f + gk[u] : 0.f;
            lg[u] = (sel && (ak[u] & 8)) ? ((ak[u] & 4) ? 0.1f : 1.f) : 1.f;
            if (c + u >= C) v[u] = 0.f;
          }
          const uint32_t t = ((uint32_t)(b * H + y) * W + x) * Cp + c;
          if (acc) {
            const float4 p = *reinterpret_cast<const float4*>(ds + t);
            v[0] += p.x; v[1] += p.y; v[2] += p.z; v[3] += p.w;
          }
          if (my) {
            const float4 m = *reinterpret_cast<const float4*>(my + t);
            v[0] *= po::leaky_grad(m.x); v[1] *= po::leaky_grad(m.y);
            v[2] *= po::leaky_grad(m.z); v[3] *= po::leaky_grad(m.w);
          } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] *= lg[u];
          }
          *reinterpret_cast<float4*>(ds + t) = make_float4(v[0], v[1], v[2], v[3]);
          vmax = fmaxf(vmax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
        }
      }
  }
  if (amax) po::amax_commit(amax, vmax);
}

__global__ __launch_bounds__(256) void nhwc2nchw_k(const float* __restrict__ s, int B, int H, int W, int C,
                                                   int Cp, float* __restrict__ d) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t tot = (int64_t)B * C * H * W;
  if (t >= tot) return;
  const int x = (int)(t % W);
  const int y = (int)((t / W) % H);
  const int c = (int)((t / ((int64_t)W * H)) % C);
  const int b = (int)(t / ((int64_t)W * H * C));
  d[t] = s[(((int64_t)b * H + y) * W + x) * Cp + c];
}

// po_view_move with every channel offset and stride a multiple of 4: one
// thread per 4 channels (16-byte loads/stores), 32-bit index math (host check)
__device__ __forceinline__ float4 vm_at4(const float* __restrict__ src, int b, int Hs, int Ws, int ss, int so, int c,
                                         int ly, int lx) {
  if (ly < 0 || ly >= Hs || lx < 0 || lx >= Ws) return make_float4(0.f, 0.f, 0.f, 0.f);
  return *reinterpret_cast<const float4*>(src + ((size_t)(b * Hs + ly) * Ws + lx) * ss + so + c);
}

__global__ __launch_bounds__(256) void view_move4_k(const float* __restrict__ src, int Hs, int Ws, int ss, int so,
                                                    const int32_t* __restrict__ sorg, float* __restrict__ dst,
                                                    int Hd, int Wd, int ds, int doff,
                                                    const int32_t* __restrict__ dorg, int B, int C4, int mode,
                                                    int acc, const float* __restrict__ my, int ms,
                                                    uint32_t* __restrict__ amax) {
  const int t0 = (int)blockIdx.x * 256 + (int)threadIdx.x;
  const int tot = B * Hd * Wd * C4;
  const bool live = t0 < tot;
  const int t = live ? t0 : 0;
  const int p = t / C4;
  const int c = (t - p * C4) * 4;
  const int b = p / (Hd * Wd);
  const int r = p - b * Hd * Wd;
  const int y = r / Wd, x = r - y * Wd;
  const int py = y + (dorg ? dorg[2 * b] : 0), px = x + (dorg ? dorg[2 * b + 1] : 0);
  const int oy = sorg ? sorg[2 * b] : 0, ox = sorg ? sorg[2 * b + 1] : 0;
  float vm = 0.f;
  if (live) {
    float4 v;
    if (mode == 0) {
      v = vm_at4(src, b, Hs, Ws, ss, so, c, py - oy, px - ox);
    } else if (mode == 1) {
      v = vm_at4(src, b, Hs, Ws, ss, so, c, (py >> 1) - oy, (px >> 1) - ox);
    } else {
      const float4 a0 = vm_at4(src, b, Hs, Ws, ss, so, c, 2 * py - oy, 2 * px - ox);
      const float4 a1 = vm_at4(src, b, Hs, Ws, ss, so, c, 2 * py - oy, 2 * px + 1 - ox);
      const float4 a2 = vm_at4(src, b, Hs, Ws, ss, so, c, 2 * py + 1 - oy, 2 * px - ox);
      const float4 a3 = vm_at4(src, b, Hs, Ws, ss, so, c, 2 * py + 1 - oy, 2 * px + 1 - ox);
      v = make_float4((a0.x + a1.x) + (a2.x + a3.x), (a0.y + a1.y) + (a2.y + a3.y),
                      (a0.z + a1.z) + (a2.z + a3.z), (a0.w + a1.w) + (a2.w + a3.w));
    }
    float4* d = reinterpret_cast<float4*>(dst + (size_t)p * ds + doff + c);
    if (acc) {
      const float4 o = *d;
      v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
    }
    if (my) {
      const float4 m = *reinterpret_cast<const float4*>(my + (size_t)p * ms + c);
      v.x *= po::leaky_grad(m.x); v.y *= po::leaky_grad(m.y); v.z *= po::leaky_grad(m.z); v.w *= po::leaky_grad(m.w);
    }
    *d = v;
    vm = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
  }
  if (amax) po::amax_commit(amax, vm);
}

__global__ __launch_bounds__(256) void nchw2nhwc_k(const float* __restrict__ s, int B, int H, int W, int C,
                                                   int Cp, float* __restrict__ d) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t tot = (int64_t)B * H * W * Cp;
  if (t >= tot) return;
  const int c = (int)(t % Cp);
  const int64_t p = t / Cp;
  const int x = (int)(p % W);
  const int y = (int)((p / W) % H);
  const int b = (int)(p / ((int64_t)W * H));
  d[t] = c < C ? s[(((int64_t)b * C + c) * H + y) * W + x] : 0.f;
}
}  // namespace

extern "C" int po_slice_accum(const float* src, int src_stride, int src_off, float* dst, int dst_stride,
                              int dst_off, int64_t M, int C, int accumulate, const float* mask_y,
                              int mask_stride, uint32_t* amax, po_stream_t s) {
  PO_REQUIRE(src && dst && M >= 0 && C >= 0, "po_slice_accum: bad argument");
  PO_REQUIRE(src_off + C <= src_stride && dst_off + C <= dst_stride, "po_slice_accum: slice exceeds stride");
  if (M * C == 0) return PO_OK;
  hipLaunchKernelGGL(slice_accum_k, dim3(po::ceil_div(M * C, 256)), dim3(256), 0, po::stream_of(s), src,
                     src_stride, src_off, dst, dst_stride, dst_off, M, C, accumulate, mask_y, mask_stride, amax);
  return po::check_launch("po_slice_accum");
}

extern "C" int po_view_move(const float* src, int Hs, int Ws, int src_stride, int src_off,
                            const int32_t* src_org, float* dst, int Hd, int Wd, int dst_stride, int dst_off,
                            const int32_t* dst_org, int B, int C, int mode, int accumulate,
                            const float* mask_y, int mask_stride, uint32_t* amax, po_stream_t s) {
  PO_REQUIRE(src && dst && B > 0 && C >= 0 && Hs > 0 && Ws > 0 && Hd > 0 && Wd > 0, "po_view_move: bad argument");
  PO_REQUIRE(mode >= 0 && mode <= 2, "po_view_move: mode %d", mode);
  PO_REQUIRE(src_off + C <= src_stride && dst_off + C <= dst_stride, "po_view_move: slice exceeds stride");
  PO_REQUIRE(!mask_y || C <= mask_stride, "po_view_move: mask stride");
  const int64_t tot = (int64_t)B * Hd * Wd * C;
  if (!tot) return PO_OK;
  const bool v4 = C % 4 == 0 && src_stride % 4 == 0 && src_off % 4 == 0 && dst_stride % 4 == 0 && dst_off % 4 == 0 &&
                  (!mask_y || mask_stride % 4 == 0) && ((uintptr_t)src | (uintptr_t)dst | (uintptr_t)mask_y) % 16 == 0 &&
                  tot + 1024 < (1LL << 31) && (int64_t)B * Hs * Ws * src_stride < (1LL << 31);
  if (v4) {
    hipLaunchKernelGGL(view_move4_k, dim3(po::ceil_div(tot / 4, 256)), dim3(256), 0, po::stream_of(s), src, Hs, Ws,
                       src_stride, src_off, src_org, dst, Hd, Wd, dst_stride, dst_off, dst_org, B, C / 4, mode,
                       accumulate, mask_y, mask_stride, amax);
    return po::check_launch("po_view_move");
  }
  hipLaunchKernelGGL(view_move_k, dim3(po::ceil_div(tot, 256)), dim3(256), 0, po::stream_of(s), src, Hs, Ws,
                     src_stride, src_off, src_org, dst, Hd, Wd, dst_stride, dst_off, dst_org, B, C, mode,
                     accumulate, mask_y, mask_stride, amax);
  return po::check_launch("po_view_move");
}

extern "C" int po_upsample2_fwd(const float* src, int B, int H, int W, int C, int src_stride, float* dst,
                                int dst_stride, int dst_off, uint32_t* amax, po_stream_t s) {
  PO_REQUIRE(src && dst && C <= src_stride && dst_off + C <= dst_stride, "po_upsample2_fwd: bad argument");
  const int64_t tot = (int64_t)B * 4 * H * W * C;
  hipLaunchKernelGGL(up2_fwd_k, dim3(po::ceil_div(tot, 256)), dim3(256), 0, po::stream_of(s), src, B, H, W,
                     C, src_stride, dst, dst_stride, dst_off, amax);
  return po::check_launch("po_upsample2_fwd");
}

extern "C" int po_upsample2_bwd(const float* src, int src_stride, int src_off, int B, int H, int W, int C,
                                float* dst, int dst_stride, int accumulate, const float* mask_y,
                                int mask_stride, uint32_t* amax, po_stream_t s) {
  PO_REQUIRE(src && dst && src_off + C <= src_stride && C <= dst_stride, "po_upsample2_bwd: bad argument");
  const int64_t tot = (int64_t)B * H * W * C;
  hipLaunchKernelGGL(up2_bwd_k, dim3(po::ceil_div(tot, 256)), dim3(256), 0, po::stream_of(s), src,
                     src_stride, src_off, B, H, W, C, dst, dst_stride, accumulate, mask_y, mask_stride, amax);
  return po::check_launch("po_upsample2_bwd");
}

static inline void pool_out(int H, int W, int stride, int& Ho, int& Wo) {
  if (stride == 2) { Ho = H / 2; Wo = W / 2; }       // MaxPool2d(2,2,padding=0)
  else { Ho = H; Wo = W; }                            // ZeroPad2d((0,1,0,1)) + MaxPool2d(2,1)
}

extern "C" int po_maxpool2_fwd(const float* src, int B, int H, int W, int C, int Cp, int stride, float* dst,
                               int8_t* argmax, uint32_t* amax, po_stream_t s) {
  PO_REQUIRE(src && dst && argmax && (stride == 1 || stride == 2) && C <= Cp, "po_maxpool2_fwd: bad argument");
  int Ho, Wo;
  pool_out(H, W, stride, Ho, Wo);
  PO_REQUIRE(Cp % 4 == 0 && (int64_t)B * Ho < (1LL << 31) && (int64_t)Wo * Cp < (1LL << 30),
             "po_maxpool2_fwd: Cp %d must be a multiple of 4 (sizes within 32-bit grids)", Cp);
  if ((int64_t)B * Ho * Wo == 0) return PO_OK;
  hipLaunchKernelGGL(maxpool2_fwd_k, dim3(B * Ho, po::ceil_div((int64_t)Wo * (Cp / 4), 256)), dim3(256), 0,
                     po::stream_of(s), src, B, H, W, C, Cp, stride, Ho, Wo, dst, argmax, amax);
  return po::check_launch("po_maxpool2_fwd");
}

extern "C" int po_maxpool2_bwd(const float* d_dst, const int8_t* argmax, int B, int H, int W, int C, int Cp,
                               int stride, float* d_src, int accumulate, const float* mask_y,
                               uint32_t* amax, po_stream_t s) {
  PO_REQUIRE(d_dst && argmax && d_src && (stride == 1 || stride == 2), "po_maxpool2_bwd: bad argument");
  int Ho, Wo;
  pool_out(H, W, stride, Ho, Wo);
  PO_REQUIRE(Cp % 4 == 0 && (int64_t)B * H < (1LL << 31) && (int64_t)W * Cp < (1LL << 30),
             "po_maxpool2_bwd: Cp %d must be a multiple of 4 (sizes within 32-bit grids)", Cp);
  if ((int64_t)B * H * W == 0) return PO_OK;
  hipLaunchKernelGGL(maxpool2_bwd_k, dim3(B * H, po::ceil_div((int64_t)W * (Cp / 4), 256)), dim3(256), 0,
                     po::stream_of(s), d_dst, argmax, B, H, W, C, Cp, stride, Ho, Wo, d_src, accumulate, mask_y,
                     amax);
  return po::check_launch("po_maxpool2_bwd");
}

extern "C" int po_maxpool2_bwd_box(const float* d_dst, const int8_t* argmax, int B, int H, int W, int C, int Cp,
                                   int stride, float* d_src, int accumulate, const float* mask_y,
                                   const int32_t* boxes, uint32_t* amax, po_stream_t s) {
  if (!boxes)
    return po_maxpool2_bwd(d_dst, argmax, B, H, W, C, Cp, stride, d_src, accumulate, mask_y, amax, s);
  PO_REQUIRE(d_dst && argmax && d_src && (stride == 1 || stride == 2), "po_maxpool2_bwd_box: bad argument");
  int Ho, Wo;
  pool_out(H, W, stride, Ho, Wo);
  PO_REQUIRE(Cp % 4 == 0 && B < 65536 && (int64_t)W * Cp < (1LL << 30),
             "po_maxpool2_bwd_box: Cp %d must be a multiple of 4 (sizes within 32-bit grids)", Cp);
  if ((int64_t)B * H * W == 0) return PO_OK;
  if (stride == 2 && H == 2 * Ho && W == 2 * Wo && (int64_t)B * H * W * Cp < (1LL << 31)) {
    const int prow = Ho < 32 ? Ho : 32;
    hipLaunchKernelGGL(maxpool2_bwd_box_s2_k, dim3(B, prow), dim3(256), 0, po::stream_of(s), d_dst, argmax, H, W, C,
                       Cp, Ho, Wo, d_src, accumulate, mask_y, boxes, amax);
    return po::check_launch("po_maxpool2_bwd_box");
  }
  const int rows = H < 32 ? H : 32;
  hipLaunchKernelGGL(maxpool2_bwd_box_k, dim3(B, rows), dim3(256), 0, po::stream_of(s), d_dst, argmax, B, H, W, C,
                     Cp, stride, Ho, Wo, d_src, accumulate, mask_y, boxes, amax);
  return po::check_launch("po_maxpool2_bwd_box");
}

extern "C" int po_nhwc_to_nchw(const float* src, int B, int H, int W, int C, int Cp, float* dst,
                               po_stream_t s) {
  PO_REQUIRE(src && dst && C <= Cp, "po_nhwc_to_nchw: bad argument");
  const int64_t tot = (int64_t)B * C * H * W;
  if (!tot) return PO_OK;
  hipLaunchKernelGGL(nhwc2nchw_k, dim3(po::ceil_div(tot, 256)), dim3(256), 0, po::stream_of(s), src, B, H, W,
                     C, Cp, dst);
  return po::check_launch("po_nhwc_to_nchw");
}

extern "C" int po_nchw_to_nhwc(const float* src, int B, int H, int W, int C, int Cp, float* dst,
                               po_stream_t s) {
  PO_REQUIRE(src && dst && C <= Cp, "po_nchw_to_nhwc: bad argument");
  const int64_t tot = (int64_t)B * H * W * Cp;
  if (!tot) return PO_OK;
  hipLaunchKernelGGL(nchw2nhwc_k, dim3(po::ceil_div(tot, 256)), dim3(256), 0, po::stream_of(s), src, B, H, W,
                     C, Cp, dst);
  return po::check_launch("po_nchw_to_nhwc");
}
