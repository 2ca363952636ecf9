// Test-time patch placement for gfx950 (§8f row 4):
//  - PatchTransformer_test_mode (load_data.py:1233-1722): rotation + scale about
//    the centre, the occupancy map of inter_axis_cal (free cells away from the
//    border and from every detection box), a random free cell, translation there;
//  - PatchTransformer_vanishing's placement parameters (load_data.py:985-1230),
//    whose warp and composite run on po_warp_fwd / po_warp_composite_multi.
//
// po_place_test_mode, per image b (grid dimension y = image):
//   tm_select_k   one wave: lab_transform's row, theta1, the area order
//   tm_warp1_k    patch + mask warped to the image centre (float64 sampling),
//                 the row extent of mask == 1 (wave-reduced atomics)
//   tm_rects_k    semi_edge, the label boxes grown by it (Python slice bounds)
//   tm_cover_k    per cell (x, y) of the [x][y] map: the first box (area order)
//                 covering it; M = max over non-border cells
//   tm_pick_k     the free set of the reference's early-exit rule, its size, the
//                 pick-th free cell in torch.nonzero order (block scan)
//   tm_warp2_k    translation + second bilinear resampling, clamp * mask
// Nothing is read back to the host; error conditions of the reference (its
// exceptions) are reported in info[b].flags and give a zero output.
#pragma clang fp contract(off)
#include "common.h"
#include "warp_geom.h"
#include <math.h>

namespace {
constexpr int TM_ST = 16;      // int32 state words per image
// state word indices
enum { ST_RMIN = 0, ST_RMAX, ST_CNT1, ST_M, ST_K, ST_SEMI2, ST_FLAGS };
enum { F_MASK = 1, F_NOFREE = 2, F_PICK = 4 };

struct TmWork {
  float* adv1;      // [B,3,S,S]
  float* msk1;      // [B,S,S]
  double* aff;      // [B,8]
  int32_t* cover;   // [B,S*S]
  int32_t* order;   // [B,L]
  int32_t* rect;    // [B,L,4] {x0, x1, y0, y1}
  int32_t* st;      // [B,TM_ST]
};

// int32 sub-buffer offsets rounded up to 4 words: every sub-buffer of the
// (16-byte aligned) int workspace starts 16-byte aligned, so tm_cover_k's int4
// loads of w.rect are aligned for any B, L, S
__host__ __device__ constexpr size_t up4(size_t n) { return (n + 3) & ~(size_t)3; }

TmWork carve(float* fwork, int32_t* iwork, int B, int L, int S) {
  TmWork w;
  const size_t plane = (size_t)S * S;
  w.adv1 = fwork;
  w.msk1 = fwork + (size_t)B * 3 * plane;
  w.aff = reinterpret_cast<double*>(fwork + (size_t)B * 4 * plane);
  w.cover = iwork;
  w.order = iwork + up4((size_t)B * plane);
  w.rect = w.order + up4((size_t)B * L);
  w.st = w.rect + (size_t)B * L * 4;
  return w;
}

// rows in use (the caller guarantees 1 <= nlab[b] <= L; clamped so a bad
// count cannot index out of the label buffer)
__device__ __forceinline__ int rows_of(const int32_t* nlab, int b, int L) { return min(max(nlab[b], 0), L); }

// Python slice bound normalisation (step 1) of an int() bound into [0, n]
__device__ __forceinline__ int py_slice_bound(int v, int n) {
  if (v < 0) v += n;
  return v < 0 ? 0 : (v > n ? n : v);
}

// int() of a float tensor: truncation toward zero (clamped before the cast)
__device__ __forceinline__ int py_int(float v) { return (int)fminf(fmaxf(v, -1e9f), 1e9f); }

// One wave per image: lab_transform (load_data.py:1295-1320), target size and
// theta1 (1576-1629), the ascending area order of inter_axis_cal (1336-1342).
__global__ __launch_bounds__(64) void tm_select_k(const float* __restrict__ lab, const int32_t* __restrict__ nlab,
                                                  int L, int S, int P, float sf, const float* __restrict__ angle,
                                                  TmWork w) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int n = rows_of(nlab, b, L);
  const float* lb = lab + (size_t)b * L * 7;
  // torch.max / torch.min of area = w*h over the rows, first index on ties
  float vmax = -INFINITY, vmin = INFINITY;
  int imax = 0x7fffffff, imin = 0x7fffffff;
  for (int l = lane; l < n; l += 64) {
    const float a = lb[l * 7 + 2] * lb[l * 7 + 3];        // load_data.py:1298
    if (a > vmax) { vmax = a; imax = l; }
    if (a < vmin) { vmin = a; imin = l; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(vmax, o), nv = __shfl_xor(vmin, o);
    const int oi = __shfl_xor(imax, o), ni = __shfl_xor(imin, o);
    if (ov > vmax || (ov == vmax && oi < imax)) { vmax = ov; imax = oi; }
    if (nv < vmin || (nv == vmin && ni < imin)) { vmin = nv; imin = ni; }
  }
  // stable ascending rank of the scaled area (lab*S)[:,2] * (lab*S)[:,3]
  const float fS = (float)S;
  for (int l = lane; l < n; l += 64) {
    const float al = (lb[l * 7 + 2] * fS) * (lb[l * 7 + 3] * fS);
    int r = 0;
    for (int m = 0; m < n; ++m) {
      const float am = (lb[m * 7 + 2] * fS) * (lb[m * 7 + 3] * fS);
      r += (am < al) || (am == al && m < l);
    }
    w.order[(size_t)b * L + r] = l;
  }
  if (lane != 0) return;
  double sel2, sel3;
  if (n <= 1 || vmax > 0.99f) {                           // load_data.py:1306-1313
    sel2 = 0.25; sel3 = 0.25;
  } else {                                                // 1315-1317
    sel2 = ((double)lb[imax * 7 + 2] + (double)lb[imin * 7 + 2]) / 2.0;
    sel3 = ((double)lb[imax * 7 + 3] + (double)lb[imin * 7 + 3]) / 2.0;
  }
  const double dS = (double)S;
  const double h2 = sel2 * dS / (double)sf, h3 = sel3 * dS / (double)sf;   // 1587-1596
  const double ts = sqrt(h2 * h2 + h3 * h3);
  const double scale = ts / (double)P;                    // 1605
  double th[6], af[6];
  po::placement_theta(angle ? (double)angle[b] : 0.0, scale, 0.0, 0.0, th);   // theta1, 1624-1629
  po::theta_pixel_affine(th, dS, af);
  for (int k = 0; k < 6; ++k) w.aff[8 * b + k] = af[k];
  int32_t* st = w.st + TM_ST * b;
  st[ST_RMIN] = 0x7fffffff;
  st[ST_RMAX] = -1;
  st[ST_CNT1] = 0;
  st[ST_M] = -1;
  st[ST_FLAGS] = 0;
}

// Bilinear sample (zeros outside) of an S x S single plane at (ix, iy), float64
__device__ __forceinline__ double bilin_plane(const float* __restrict__ p, int S, double ix, double iy) {
  const double fx = floor(ix), fy = floor(iy);
  const int x0 = (int)fx, y0 = (int)fy;
  const double ex = ix - fx, ey = iy - fy;
  const double wt[4] = {(1.0 - ex) * (1.0 - ey), ex * (1.0 - ey), (1.0 - ex) * ey, ex * ey};
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int x = x0 + (k & 1), y = y0 + (k >> 1);
    if (x >= 0 && x < S && y >= 0 && y < S) acc += wt[k] * (double)p[(size_t)y * S + x];
  }
  return acc;
}

// theta1 warp of the padded clamp(patch) and of its all-ones mask
// (load_data.py:1490, 1523-1535, 1631-1635), one output pixel per thread.
__global__ __launch_bounds__(256) void tm_warp1_k(const float* __restrict__ mp, int P, int S, TmWork w) {
  const int b = blockIdx.y;
  const int q = blockIdx.x * 256 + threadIdx.x;
  const bool live = q < S * S;
  const int i = live ? q / S : 0, j = live ? q - i * S : 0;
  const double* af = w.aff + 8 * b;
  const double ix = af[0] * (double)j + af[1] * (double)i + af[2];
  const double iy = af[3] * (double)j + af[4] * (double)i + af[5];
  const int pad = (int)((S - P) / 2.0 + 0.5);            // ConstantPad2d((int(pad+.5), int(pad), ...))
  double a[3] = {0.0, 0.0, 0.0}, m = 0.0;
  // a tap can be inside the padded patch only for ix, iy in [pad-1, pad+P)
  if (live && ix >= (double)(pad - 1) && ix < (double)(pad + P) && iy >= (double)(pad - 1) &&
      iy < (double)(pad + P)) {
    const double fx = floor(ix), fy = floor(iy);
    const int x0 = (int)fx, y0 = (int)fy;
    const double ex = ix - fx, ey = iy - fy;
    const double wt[4] = {(1.0 - ex) * (1.0 - ey), ex * (1.0 - ey), (1.0 - ex) * ey, ex * ey};
    const size_t pp = (size_t)P * P;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int pc = x0 + (k & 1) - pad, pr = y0 + (k >> 1) - pad;
      if (pr >= 0 && pr < P && pc >= 0 && pc < P) {
        const size_t o = (size_t)pr * P + pc;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) a[ch] += wt[k] * (double)fminf(fmaxf(mp[o + ch * pp], 0.f), 1.f);
        m += wt[k];
      }
    }
  }
  const float mf = (float)m;
  if (live) {
    const size_t plane = (size_t)S * S;
    for (int ch = 0; ch < 3; ++ch) w.adv1[((size_t)b * 3 + ch) * plane + q] = (float)a[ch];
    w.msk1[(size_t)b * plane + q] = mf;
  }
  // rows holding msk == 1 (load_data.py:1650-1664): wave min/max/count, one atomic each
  const bool one = live && mf == 1.0f;
  int rmin = one ? i : 0x7fffffff, rmax = one ? i : -1, cnt = one ? 1 : 0;
  for (int o = 32; o > 0; o >>= 1) {
    rmin = min(rmin, __shfl_xor(rmin, o));
    rmax = max(rmax, __shfl_xor(rmax, o));
    cnt += __shfl_xor(cnt, o);
  }
  if ((threadIdx.x & 63) == 0 && cnt) {
    int32_t* st = w.st + TM_ST * b;
    atomicMin(st + ST_RMIN, rmin);
    atomicMax(st + ST_RMAX, rmax);
    atomicAdd(st + ST_CNT1, cnt);
  }
}

// semi_edge and the grown label boxes in area order (load_data.py:1334-1407).
// semi_in (optional, [B]) overrides the mask extent (po_place_free_map).
__global__ __launch_bounds__(256) void tm_rects_k(const float* __restrict__ lab, const int32_t* __restrict__ nlab,
                                                  int L, int S, const float* __restrict__ semi_in, TmWork w) {
  const int b = blockIdx.x;
  int32_t* st = w.st + TM_ST * b;
  float semi;
  if (semi_in) {
    semi = semi_in[b];
  } else {
    const int cnt = st[ST_CNT1];
    // torch.min on an empty nonzero() / the squeeze of a single one: the reference raises
    semi = cnt >= 2 ? (float)(st[ST_RMAX] - st[ST_RMIN]) / 2.0f : 0.0f;
    if (threadIdx.x == 0 && cnt < 2) st[ST_FLAGS] |= F_MASK;
  }
  if (threadIdx.x == 0) {
    st[ST_K] = py_int(semi);                              // int(semi_edge), load_data.py:1361-1365
    st[ST_SEMI2] = py_int(semi * 2.0f);
  }
  const int n = rows_of(nlab, b, L);
  const float* lb = lab + (size_t)b * L * 7;
  const float fS = (float)S;
  for (int r = threadIdx.x; r < n; r += 256) {
    const int l = w.order[(size_t)b * L + r];
    const float cx = lb[l * 7 + 0] * fS, cy = lb[l * 7 + 1] * fS;   // lab_scale, 1336 / 1401-1404
    const float W = lb[l * 7 + 2] * fS, H = lb[l * 7 + 3] * fS;
    int32_t* rc = w.rect + ((size_t)b * L + r) * 4;
    rc[0] = py_slice_bound(py_int(cx - W / 2.0f - semi), S);        // 1406-1407
    rc[1] = py_slice_bound(py_int(cx + W / 2.0f + semi), S);
    rc[2] = py_slice_bound(py_int(cy - H / 2.0f - semi), S);
    rc[3] = py_slice_bound(py_int(cy + H / 2.0f + semi), S);
  }
}

__device__ __forceinline__ bool tm_border(int x, int y, int S, int k) {
  // temp_lab[:, 0:k, :], [:, -k:, :], [:, :, 0:k], [:, :, -k:] (-0: is the whole axis)
  return k <= 0 || x < k || x >= S - k || y < k || y >= S - k;
}

// first covering box per cell of the [x][y] map; M = max over non-border cells
constexpr int TM_RCHUNK = 1024;
__global__ __launch_bounds__(256) void tm_cover_k(const int32_t* __restrict__ nlab, int L, int S, TmWork w) {
  __shared__ int4 rs[TM_RCHUNK];
  const int b = blockIdx.y;
  const int q = blockIdx.x * 256 + threadIdx.x;
  const bool live = q < S * S;
  const int x = live ? q / S : 0, y = live ? q - x * S : 0;
  const int n = rows_of(nlab, b, L);
  int c = n;
  for (int r0 = 0; r0 < n; r0 += TM_RCHUNK) {
    const int nr = min(TM_RCHUNK, n - r0);
    __syncthreads();
    for (int t = threadIdx.x; t < nr; t += 256)
      rs[t] = reinterpret_cast<const int4*>(w.rect)[(size_t)b * L + r0 + t];
    __syncthreads();
    if (c == n)
      for (int t = 0; t < nr; ++t) {
        const int4 R = rs[t];
        if (x >= R.x && x < R.y && y >= R.z && y < R.w) { c = r0 + t; break; }
      }
  }
  if (!live) c = -1;
  else w.cover[(size_t)b * S * S + q] = c;
  const int k = w.st[TM_ST * b + ST_K];
  int cm = (live && !tm_border(x, y, S, k)) ? c : -1;
  for (int o = 32; o > 0; o >>= 1) cm = max(cm, __shfl_xor(cm, o));
  if ((threadIdx.x & 63) == 0 && cm >= 0) atomicMax(w.st + TM_ST * b + ST_M, cm);
}

// Free cells of inter_axis_cal's return value (load_data.py:1372-1430).  With
// c(p) the first covering box and M its max over non-border cells, the loop
// stops before box M+1 and returns the sum of layers 0..M-1 (temp_lab[0:i-1]
// at i = M+1; the full sum when M = n; layers 0..n-2 when M = n-1): its zeros
// are the non-border cells with c == M, or every cell when that sum is empty
// (M == 0, or M == -1 with n == 1).  M == -1 with n >= 2 leaves none.
__device__ __forceinline__ bool tm_free(const int32_t* cov, int q, int S, int k, int M, int n) {
  if (M == 0 || (M == -1 && n == 1)) return true;
  if (M < 0) return false;
  const int x = q / S, y = q - (q / S) * S;
  return !tm_border(x, y, S, k) && cov[q] == M;
}

constexpr int TM_PT = 1024;
__global__ __launch_bounds__(TM_PT) void tm_pick_k(const int32_t* __restrict__ nlab, int L, int S,
                                                   const float* __restrict__ upick, TmWork w,
                                                   int32_t* __restrict__ info) {
  __shared__ int wsum[TM_PT / 64];
  __shared__ int s_pick, s_n;
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  int32_t* st = w.st + TM_ST * b;
  const int n = rows_of(nlab, b, L), k = st[ST_K], M = st[ST_M];
  const int64_t NN = (int64_t)S * S;
  const int chunk = (int)((NN + TM_PT - 1) / TM_PT);
  const int lo = (int)min((int64_t)t * chunk, NN), hi = (int)min((int64_t)lo + chunk, NN);
  const int32_t* cov = w.cover + (size_t)b * NN;
  int cnt = 0;
  for (int q = lo; q < hi; ++q) cnt += tm_free(cov, q, S, k, M, n);
  // block exclusive scan of cnt
  int incl = cnt;
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  int base = 0, total = 0;
  for (int u = 0; u < TM_PT / 64; ++u) {
    if (u < wv) base += wsum[u];
    total += wsum[u];
  }
  const int excl = base + incl - cnt;
  if (t == 0) {
    // random.randint(0, len) draws from [0, len] inclusive (load_data.py:1682)
    int pick = (int)floor((double)upick[b] * (double)(total + 1));
    pick = min(pick, total);
    int flags = st[ST_FLAGS];
    if (total == 0) flags |= F_NOFREE;
    else if (pick == total) flags |= F_PICK;
    st[ST_FLAGS] = flags;
    s_pick = pick;
    s_n = total;
    int32_t* inf = info + 8 * b;
    inf[0] = flags;
    inf[1] = -1;
    inf[2] = -1;
    inf[3] = st[ST_SEMI2];
    inf[4] = M;
    inf[5] = total;
    inf[6] = pick;
    inf[7] = st[ST_CNT1];
  }
  __syncthreads();
  const int pick = s_pick;
  if (pick < s_n && pick >= excl && pick < excl + cnt) {
    int seen = excl;
    for (int q = lo; q < hi; ++q) {
      if (!tm_free(cov, q, S, k, M, n)) continue;
      if (seen == pick) {
        info[8 * b + 1] = q / S;                          // position_final[0] -> target_x
        info[8 * b + 2] = q - (q / S) * S;                // position_final[1] -> target_y
        break;
      }
      ++seen;
    }
  }
}

// inter_axis_cal's return value as a free/occupied map (0 = free), [x][y]
__global__ __launch_bounds__(256) void tm_freemap_k(const int32_t* __restrict__ nlab, int L, int S, TmWork w,
                                                    int32_t* __restrict__ layout) {
  const int b = blockIdx.y;
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= S * S) return;
  const int32_t* st = w.st + TM_ST * b;
  const size_t o = (size_t)b * S * S;
  layout[o + q] = tm_free(w.cover + o, q, S, st[ST_K], st[ST_M], rows_of(nlab, b, L)) ? 0 : 1;
}

// theta2 (load_data.py:1689-1706): ix = j + (S/2 - x), iy = i + (S/2 - y) (the
// pixel-space form of tx = (0.5 - x/S)*2, exact in float64); bilinear
// resampling of the warped patch and mask, clamp * mask (1714-1715).
__global__ __launch_bounds__(256) void tm_warp2_k(int S, TmWork w, const int32_t* __restrict__ info,
                                                  float* __restrict__ out) {
  const int b = blockIdx.y;
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= S * S) return;
  const int i = q / S, j = q - i * S;
  const size_t plane = (size_t)S * S;
  const int32_t* inf = info + 8 * b;
  float* ob = out + (size_t)b * 3 * plane + q;
  if (inf[0] != 0) {
    for (int ch = 0; ch < 3; ++ch) ob[ch * plane] = 0.f;
    return;
  }
  const double ix = (double)j + (0.5 * (double)S - (double)inf[1]);
  const double iy = (double)i + (0.5 * (double)S - (double)inf[2]);
  const float m = (float)bilin_plane(w.msk1 + (size_t)b * plane, S, ix, iy);
  for (int ch = 0; ch < 3; ++ch) {
    const float a = (float)bilin_plane(w.adv1 + ((size_t)b * 3 + ch) * plane, S, ix, iy);
    ob[ch * plane] = fminf(fmaxf(a, 0.f), 1.f) * m;
  }
}

// PatchTransformer_vanishing placement (load_data.py:1095-1178), one thread per label row
__global__ __launch_bounds__(256) void vanish_params_k(const float* __restrict__ lab, int BL, int S, int P,
                                                       float pre_scale, const float* __restrict__ angle,
                                                       const float* __restrict__ offx,
                                                       const float* __restrict__ offy, int orient,
                                                       double* __restrict__ affine, int32_t* __restrict__ roi) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= BL) return;
  const float* r = lab + (size_t)t * 5;
  const double dS = (double)S;
  const double w = (double)r[3], h = (double)r[4];
  const double hw = w * dS / (double)pre_scale, hh = h * dS / (double)pre_scale;   // 1105-1120
  const double ts = sqrt(hw * hw + hh * hh);
  double tx_ = (double)r[1], ty_ = (double)r[2];         // 1122-1123
  if (offx) tx_ += w * (double)offx[t];                  // rand_loc, 1131-1143
  if (offy) ty_ += h * (double)offy[t];
  if (orient == 1) tx_ -= w / 6.0;                       // 1158-1162
  else if (orient == 2) tx_ += w / 6.0;
  const double scale = ts / (double)P;                   // 1149
  double th[6], af[6];
  po::placement_theta(angle ? (double)angle[t] : 0.0, scale, (-tx_ + 0.5) * 2.0, (-ty_ + 0.5) * 2.0, th);
  po::theta_pixel_affine(th, dS, af);
  for (int k = 0; k < 6; ++k) affine[6 * (size_t)t + k] = af[k];
  po::footprint_roi(af, S, P, roi + 4 * (size_t)t);
}
}  // namespace

extern "C" int po_place_workspace(int B, int L, int S, int64_t* fwords, int64_t* iwords) {
  PO_REQUIRE(B > 0 && L > 0 && S > 0 && fwords && iwords, "po_place_workspace: bad argument");
  *fwords = (int64_t)4 * B * S * S + 16 * (int64_t)B;
  // carve(): cover [B*S*S] | order [B*L] | rect [B*L*4] | st [B*TM_ST], the first two rounded up to 4 words
  *iwords = (int64_t)up4((size_t)B * S * S) + (int64_t)up4((size_t)B * L) + 4 * (int64_t)B * L + (int64_t)B * TM_ST;
  return PO_OK;
}

extern "C" int po_place_test_mode(const float* patch_mp, int P, const float* lab, const int32_t* nlab, int B, int L,
                                  int S, float scale_factor, const float* angle, const float* upick, float* fwork,
                                  int32_t* iwork, float* out, int32_t* info, po_stream_t s) {
  PO_REQUIRE(patch_mp && lab && nlab && upick && fwork && iwork && out && info, "po_place_test_mode: null pointer");
  PO_REQUIRE(B > 0 && L > 0 && P > 0 && S > 1 && P <= S && (int64_t)S * S < (1LL << 30),
             "po_place_test_mode: bad shape B=%d L=%d S=%d P=%d", B, L, S, P);
  PO_REQUIRE(scale_factor > 0.f, "po_place_test_mode: scale_factor must be > 0");
  PO_REQUIRE(((uintptr_t)fwork % 8) == 0 && ((uintptr_t)iwork % 16) == 0, "po_place_test_mode: workspace alignment");
  TmWork w = carve(fwork, iwork, B, L, S);
  hipStream_t st = po::stream_of(s);
  const dim3 pix(po::ceil_div((int64_t)S * S, 256), B);
  hipLaunchKernelGGL(tm_select_k, dim3(B), dim3(64), 0, st, lab, nlab, L, S, P, scale_factor, angle, w);
  hipLaunchKernelGGL(tm_warp1_k, pix, dim3(256), 0, st, patch_mp, P, S, w);
  hipLaunchKernelGGL(tm_rects_k, dim3(B), dim3(256), 0, st, lab, nlab, L, S, (const float*)nullptr, w);
  hipLaunchKernelGGL(tm_cover_k, pix, dim3(256), 0, st, nlab, L, S, w);
  hipLaunchKernelGGL(tm_pick_k, dim3(B), dim3(TM_PT), 0, st, nlab, L, S, upick, w, info);
  hipLaunchKernelGGL(tm_warp2_k, pix, dim3(256), 0, st, S, w, info, out);
  return po::check_launch("po_place_test_mode");
}

extern "C" int po_place_free_map(const float* lab, const int32_t* nlab, int B, int L, int S, const float* semi_edge,
                                 float* fwork, int32_t* iwork, int32_t* layout, po_stream_t s) {
  PO_REQUIRE(lab && nlab && semi_edge && fwork && iwork && layout, "po_place_free_map: null pointer");
  PO_REQUIRE(B > 0 && L > 0 && S > 1 && (int64_t)S * S < (1LL << 30), "po_place_free_map: bad shape");
  PO_REQUIRE(((uintptr_t)fwork % 8) == 0 && ((uintptr_t)iwork % 16) == 0, "po_place_free_map: workspace alignment");
  TmWork w = carve(fwork, iwork, B, L, S);
  hipStream_t st = po::stream_of(s);
  const dim3 pix(po::ceil_div((int64_t)S * S, 256), B);
  hipLaunchKernelGGL(tm_select_k, dim3(B), dim3(64), 0, st, lab, nlab, L, S, 1, 2.0f, (const float*)nullptr, w);
  hipLaunchKernelGGL(tm_rects_k, dim3(B), dim3(256), 0, st, lab, nlab, L, S, semi_edge, w);
  hipLaunchKernelGGL(tm_cover_k, pix, dim3(256), 0, st, nlab, L, S, w);
  hipLaunchKernelGGL(tm_freemap_k, pix, dim3(256), 0, st, nlab, L, S, w, layout);
  return po::check_launch("po_place_free_map");
}

extern "C" int po_vanishing_params(const float* lab, int B, int L, int S, int P, float pre_scale, const float* angle,
                                   const float* offx, const float* offy, int orient, double* affine, int32_t* roi,
                                   po_stream_t s) {
  PO_REQUIRE(lab && affine && roi, "po_vanishing_params: null pointer");
  PO_REQUIRE(B > 0 && L > 0 && S > 1 && P > 0 && P <= S, "po_vanishing_params: bad shape");
  PO_REQUIRE(pre_scale > 0.f && orient >= 0 && orient <= 2, "po_vanishing_params: bad pre_scale/orient");
  PO_REQUIRE(!offx == !offy, "po_vanishing_params: offx and offy go together");
  const int BL = B * L;
  hipLaunchKernelGGL(vanish_params_k, dim3(po::ceil_div(BL, 256)), dim3(256), 0, po::stream_of(s), lab, BL, S, P,
                     pre_scale, angle, offx, offy, orient, affine, roi);
  return po::check_launch("po_vanishing_params");
}
