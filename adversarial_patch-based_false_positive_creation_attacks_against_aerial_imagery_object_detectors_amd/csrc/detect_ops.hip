// Patch evaluation on the device: YOLO head decode +
// confidence threshold (reference utils.py:125-245 get_region_boxes, with
// do_detect's normalisation, utils.py:495-517) and greedy NMS (utils.py:93-112,
// bbox_iou 27-57 in centre form).
//
// po_region_boxes: one workgroup per image walks the head's candidates in the
// reference's loop order (cy, cx, anchor), decodes them in fp32 in the
// reference's operation order, and compacts the ones above the threshold in
// that order with a workgroup prefix sum (so box indices match the
// reference's list positions).
// po_nms: per image (1) sort by key = fp32(1 - det_conf) ascending, ties by
// candidate index (one workgroup, bitonic sort of packed 64-bit keys in a
// global workspace); (2) suppression bit matrix: bit (s, t) = [t > s and
// iou(sorted s, sorted t) > thresh] (64x64 blocks, fp32 IoU in the
// reference's order, no FMA); (3) one wave scans the sorted boxes, keeping a
// box unless a kept box suppressed it, OR-ing the kept box's row into the
// removed set.  Deterministic; no atomics on the result.
#pragma clang fp contract(off)
#include "common.h"

namespace {
constexpr int BOXF = 8;      // floats per box record: x y w h det cls_conf cls_id, source index (int bits)

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

struct RegionArgs {
  float aw[4], ah[4];        // scaled anchors (anchor / stride, fp32)
  int B, A, C, h, w, cap, only_obj;
  float stride_w, stride_h, norm_w, norm_h, thresh;
};

__global__ __launch_bounds__(256) void region_boxes_k(const RegionArgs a, const float* __restrict__ head,
                                                      float* __restrict__ boxes, int32_t* __restrict__ counts,
                                                      int32_t* __restrict__ overflow) {
  __shared__ int wsum[4];
  __shared__ int base;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int F = 5 + a.C, hw = a.h * a.w;
  const int n = hw * a.A;
  const float* hb = head + (size_t)b * a.A * F * hw;
  if (tid == 0) base = counts[b];
  __syncthreads();
  for (int k0 = 0; k0 < n; k0 += 256) {
    const int k = k0 + tid;
    bool keep = false;
    float rec[7];
    int src = 0;
    if (k < n) {
      const int i = k % a.A, cell = k / a.A;
      src = i * hw + cell;                             // the head element (anchor, cy, cx) of the record
      const int cy = cell / a.w, cx = cell - cy * a.w;
      const float* f = hb + (size_t)i * F * hw + cell;
      const float det = sigm(f[4 * hw]);
      float cmax = -1.f;
      int cid = 0;
      for (int c = 0; c < a.C; ++c) {
        const float p = sigm(f[(5 + c) * hw]);
        if (p > cmax) { cmax = p; cid = c; }             // torch.max: first index on ties
      }
      const float conf = a.only_obj ? det : det * cmax;
      keep = conf > a.thresh;
      if (keep) {
        float xs = (sigm(f[0]) + (float)cx) * a.stride_w;
        float ys = (sigm(f[hw]) + (float)cy) * a.stride_h;
        float ws = (expf(f[2 * hw]) * a.aw[i]) * a.stride_w;
        float hs = (expf(f[3 * hw]) * a.ah[i]) * a.stride_h;
        if (a.norm_w != 1.f) { xs = xs / a.norm_w; ws = ws / a.norm_w; }
        if (a.norm_h != 1.f) { ys = ys / a.norm_h; hs = hs / a.norm_h; }
        rec[0] = xs; rec[1] = ys; rec[2] = ws; rec[3] = hs; rec[4] = det; rec[5] = cmax; rec[6] = (float)cid;
      }
    }
    // ordered compaction: wave ballot prefix, then the waves in order
    const uint64_t bal = __ballot(keep);
    const int pre = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wave] = __popcll(bal);
    __syncthreads();
    int off = base;
    for (int w2 = 0; w2 < wave; ++w2) off += wsum[w2];
    if (keep) {
      const int pos = off + pre;
      if (pos < a.cap) {
        float* o = boxes + ((size_t)b * a.cap + pos) * BOXF;
#pragma unroll
        for (int q = 0; q < 7; ++q) o[q] = rec[q];
        o[7] = __int_as_float(src);
      } else {
        atomicOr(overflow, 1);
      }
    }
    __syncthreads();
    if (tid == 0) base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  if (tid == 0) counts[b] = base;
}

// ---- NMS (1): per image, sort packed keys (fp32 bits of 1 - det) << 32 | index
__global__ __launch_bounds__(1024) void nms_sort_k(const float* __restrict__ boxes, const int32_t* __restrict__ counts,
                                                   int cap, int nmax, int n2, uint64_t* __restrict__ keys) {
  const int b = blockIdx.x;
  const int n = min(counts[b], nmax);   // keys / mask / LDS are sized for nmax
  uint64_t* kb = keys + (size_t)b * n2;
  for (int j = threadIdx.x; j < n2; j += 1024) {
    uint64_t v = ~0ull;
    if (j < n) {
      const float key = 1.f - boxes[((size_t)b * cap + j) * BOXF + 4];    // utils.py:98-99
      v = ((uint64_t)__float_as_uint(key) << 32) | (uint32_t)j;
    }
    kb[j] = v;
  }
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int j = threadIdx.x; j < n2; j += 1024) {
        const int p = j ^ stride;
        if (p > j) {
          const uint64_t x = kb[j], y = kb[p];
          const bool up = (j & size) == 0;
          if ((x > y) == up) { kb[j] = y; kb[p] = x; }
        }
      }
      __syncthreads();
    }
}

// bbox_iou(box1, box2, x1y1x2y2=False) > thresh, fp32, reference order (utils.py:37-57)
__device__ __forceinline__ bool iou_over(const float* b1, const float* b2, float thresh) {
  const float mx = fminf(b1[0] - b1[2] / 2.0f, b2[0] - b2[2] / 2.0f);
  const float Mx = fmaxf(b1[0] + b1[2] / 2.0f, b2[0] + b2[2] / 2.0f);
  const float my = fminf(b1[1] - b1[3] / 2.0f, b2[1] - b2[3] / 2.0f);
  const float My = fmaxf(b1[1] + b1[3] / 2.0f, b2[1] + b2[3] / 2.0f);
  const float uw = Mx - mx, uh = My - my;
  const float cw = b1[2] + b2[2] - uw, ch = b1[3] + b2[3] - uh;
  if (cw <= 0.f || ch <= 0.f) return 0.f > thresh;
  const float area1 = b1[2] * b1[3], area2 = b2[2] * b2[3];
  const float carea = cw * ch;
  const float uarea = area1 + area2 - carea;
  return carea / uarea > thresh;
}

// ---- NMS (2): suppression matrix, block (row block rb, word wd) of 64 x 64
__global__ __launch_bounds__(64) void nms_mask_k(const float* __restrict__ boxes, const int32_t* __restrict__ counts,
                                                 const uint64_t* __restrict__ keys, int cap, int nmax, int n2, int nwords,
                                                 float thresh, uint64_t* __restrict__ mask) {
  __shared__ float cb[64][BOXF];
  const int b = blockIdx.z, rb = blockIdx.y, wd = blockIdx.x, t = threadIdx.x;
  const int n = min(counts[b], nmax);   // keys / mask / LDS are sized for nmax
  if (rb * 64 >= n || wd * 64 >= n || wd < rb) {
    // blocks below the diagonal hold no bit (t > s only); rows past n are never read
    if (rb * 64 < n && wd < rb) mask[((size_t)b * n2 + rb * 64 + t) * nwords + wd] = 0ull;
    return;
  }
  const uint64_t* kb = keys + (size_t)b * n2;
  const float* bb = boxes + (size_t)b * cap * BOXF;
  const int ct = wd * 64 + t;
  if (ct < n) {
    const int src = (int)(uint32_t)kb[ct];
#pragma unroll
    for (int q = 0; q < BOXF; ++q) cb[t][q] = bb[(size_t)src * BOXF + q];
  }
  __syncthreads();
  const int s = rb * 64 + t;
  if (s >= n) return;
  float me[BOXF];
  const int si = (int)(uint32_t)kb[s];
#pragma unroll
  for (int q = 0; q < BOXF; ++q) me[q] = bb[(size_t)si * BOXF + q];
  uint64_t bits = 0;
  const int lim = min(64, n - wd * 64);
  for (int c = 0; c < lim; ++c) {
    const int tt = wd * 64 + c;
    if (tt > s && iou_over(me, cb[c], thresh)) bits |= 1ull << c;
  }
  mask[((size_t)b * n2 + s) * nwords + wd] = bits;
}

// ---- NMS (3): one wave per image scans the sorted boxes
__global__ __launch_bounds__(64) void nms_scan_k(const float* __restrict__ boxes, const int32_t* __restrict__ counts,
                                                 const uint64_t* __restrict__ keys, const uint64_t* __restrict__ mask,
                                                 int cap, int nmax, int n2, int nwords, int32_t* __restrict__ keep,
                                                 int32_t* __restrict__ nkeep) {
  extern __shared__ uint64_t removed[];
  const int b = blockIdx.x, lane = threadIdx.x;
  const int n = min(counts[b], nmax);   // keys / mask / LDS are sized for nmax
  for (int w = lane; w < nwords; w += 64) removed[w] = 0ull;
  __syncthreads();
  const uint64_t* kb = keys + (size_t)b * n2;
  int nk = 0;
  for (int s = 0; s < n; ++s) {
    const bool gone = (removed[s >> 6] >> (s & 63)) & 1ull;
    if (gone) continue;                                   // uniform: every lane reads the same word
    const int src = (int)(uint32_t)kb[s];
    if (!(boxes[((size_t)b * cap + src) * BOXF + 4] > 0.f)) continue;   // utils.py:105
    if (lane == 0) keep[(size_t)b * cap + nk] = src;
    ++nk;
    const uint64_t* row = mask + ((size_t)b * n2 + s) * nwords;
    for (int w = (s >> 6) + lane; w < nwords; w += 64) removed[w] |= row[w];
    __syncthreads();
  }
  if (lane == 0) nkeep[b] = nk;
}
}  // namespace

extern "C" int po_region_boxes(const float* head, int B, int A, int C, int h, int w, const float* anchors_scaled,
                               float stride_w, float stride_h, float norm_w, float norm_h, float conf_thresh,
                               int only_objectness, int cap, float* boxes, int32_t* counts, int32_t* overflow,
                               po_stream_t s) {
  PO_REQUIRE(head && anchors_scaled && boxes && counts && overflow, "po_region_boxes: null pointer");
  PO_REQUIRE(B >= 1 && A >= 1 && A <= 4 && C >= 1 && h >= 1 && w >= 1 && cap >= 1,
             "po_region_boxes: bad sizes (B=%d A=%d C=%d h=%d w=%d cap=%d)", B, A, C, h, w, cap);
  RegionArgs a;
  for (int i = 0; i < 4; ++i) {
    a.aw[i] = i < A ? anchors_scaled[2 * i] : 0.f;
    a.ah[i] = i < A ? anchors_scaled[2 * i + 1] : 0.f;
  }
  a.B = B; a.A = A; a.C = C; a.h = h; a.w = w; a.cap = cap; a.only_obj = only_objectness;
  a.stride_w = stride_w; a.stride_h = stride_h; a.norm_w = norm_w; a.norm_h = norm_h; a.thresh = conf_thresh;
  hipLaunchKernelGGL(region_boxes_k, dim3(B), dim3(256), 0, po::stream_of(s), a, head, boxes, counts, overflow);
  return po::check_launch("po_region_boxes");
}

extern "C" int po_nms(const float* boxes, const int32_t* counts, int B, int cap, int nmax, float nms_thresh,
                      uint64_t* keys, uint64_t* mask, int32_t* keep, int32_t* nkeep, po_stream_t s) {
  PO_REQUIRE(boxes && counts && keys && mask && keep && nkeep, "po_nms: null pointer");
  PO_REQUIRE(B >= 1 && cap >= 1 && nmax >= 1 && nmax <= cap && nmax <= 65536, "po_nms: bad sizes (B=%d cap=%d nmax=%d)",
             B, cap, nmax);
  int n2 = 1;
  while (n2 < nmax) n2 <<= 1;
  const int nwords = (nmax + 63) / 64;
  hipStream_t st = po::stream_of(s);
  hipLaunchKernelGGL(nms_sort_k, dim3(B), dim3(1024), 0, st, boxes, counts, cap, nmax, n2, keys);
  int rc = po::check_launch("po_nms (sort)");
  if (rc) return rc;
  hipLaunchKernelGGL(nms_mask_k, dim3(nwords, nwords, B), dim3(64), 0, st, boxes, counts, keys, cap, nmax, n2, nwords,
                     nms_thresh, mask);
  rc = po::check_launch("po_nms (mask)");
  if (rc) return rc;
  hipLaunchKernelGGL(nms_scan_k, dim3(B), dim3(64), nwords * sizeof(uint64_t), st, boxes, counts, keys, mask, cap,
                     nmax, n2, nwords, keep, nkeep);
  return po::check_launch("po_nms (scan)");
}

// workspace sizes of po_nms for nmax boxes per image: keys B*n2 uint64,
// mask B*n2*nwords uint64 (n2 = next power of two >= nmax, nwords = ceil(nmax/64))
extern "C" int po_nms_workspace(int B, int nmax, int64_t* key_words, int64_t* mask_words) {
  PO_REQUIRE(key_words && mask_words && B >= 1 && nmax >= 1 && nmax <= 65536, "po_nms_workspace: bad arguments");
  int n2 = 1;
  while (n2 < nmax) n2 <<= 1;
  *key_words = (int64_t)B * n2;
  *mask_words = (int64_t)B * n2 * ((nmax + 63) / 64);
  return PO_OK;
}
