// Winograd F(2x2,3x3) po_conv tile 70 (staging 15): conv_wino5_k, the
// persistent form of conv_wino4_k<stagger> (tile 68, conv_wino.hip).
#pragma clang fp contract(off)
#include "conv_common.h"
#include "wino_common.h"

namespace {

// ---------------------------------------------------------------------------
// Tile 70 (staging 15): conv_wino5_k -- tile 68 made persistent.
//
// Tile 68 spends a fixed ~10.5 us per workgroup outside its k-loop: the
// prologue's offset set-up and first input round trip, the last k-step's
// wasted prefetches, the epilogue's input loads and its store issue
// (DESIGN.md §6), and with one 512-thread workgroup per CU nothing overlaps
// it -- 54% / 35% / 21% of a workgroup at 2 / 4 / 8 k-steps.  Here one
// workgroup per CU walks the launch's units (64 2x2-tiles x 64 channels x one
// split-K slice, unit u -> slice u / mn, n-block fastest) and pipelines
// across them:
//   * the last k-step of a unit is peeled: no prefetch past the unit;
//   * once the accumulators are staged through LDS and inverse-transformed,
//     the NEXT unit's first input rows are requested, and only then are this
//     unit's outputs computed and stored -- at the top of the next iteration,
//     so the stores drain while the next unit's transform and MFMAs run;
//   * every epilogue memory operation is an unconditional buffer load or
//     store (an absent tensor: a zero-extent resource; a masked element: an
//     out-of-range offset), so the vmcnt counts the compiler places stay
//     exact around the loop and the transform waits for its input rows only,
//     not for the stores issued after them.
// Per unit the arithmetic is tile 68's (same transforms, MFMA order, inverse
// transform and epilogue operations, in the same order): bit-identical outputs.
template <int MODE, int EF>   // MODE 0: po_conv epilogue (fields EF), 1: raw split-K partials, 2: fused max pool
__global__ __launch_bounds__(512, 1) void conv_wino5_k(const ConvArgs a, const float* __restrict__ U, int Ht, int Wt,
                                                       int units, int mn) {
  constexpr int CPW = 2;                 // components per wave
  constexpr int TH = 32;                 // tiles per epilogue pass (one M-block)
  __shared__ __attribute__((aligned(16))) float smem[2 * V4_FLOATS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int h = lane >> 5;
  const int G = gridDim.x;
  const int kc_n = a.Cin_p / WK;
  const int wpp = a.Cout_p >> 5;

  // ---- buffer resources (host: every extent < 2^31 bytes)
  const uint32_t npix = (uint32_t)a.B * (uint32_t)a.Hout * (uint32_t)a.Wout;
  const uint32_t dst_bytes = npix * (uint32_t)a.Cout_p * 4u;
  const uint32_t bits_bytes = npix * (uint32_t)wpp * 4u;
  const uint32_t in_bytes = (uint32_t)__builtin_amdgcn_readfirstlane(a.in_bytes);
  const __amdgpu_buffer_rsrc_t in_rs = rsrc(a.in, in_bytes);
  __amdgpu_buffer_rsrc_t rs_out = in_rs, rs_aux = in_rs, rs_bias = in_rs;
  if constexpr (MODE == 0) rs_out = rsrc(a.y, (EF & (EF_Y | EF_ACC)) ? dst_bytes : 0u);
  if constexpr (MODE == 1) rs_out = rsrc(a.ws, (uint32_t)a.ksplit * (uint32_t)a.M * (uint32_t)a.N * 4u);
  const uint32_t pool_px = MODE == 2 ? (uint32_t)a.B * (uint32_t)(a.Hout >> 1) * (uint32_t)(a.Wout >> 1) : 0u;
  if constexpr (MODE == 2) {
    rs_out = rsrc(a.pool_y, pool_px * (uint32_t)a.Cout_p * 4u);
    rs_aux = rsrc(a.pool_am, pool_px * (uint32_t)a.Cout_p);
  }
  if constexpr (MODE != 1) rs_bias = rsrc(a.bias, a.bias ? (uint32_t)a.N * 4u : 0u);

  // ---- unit u -> (first tile row m0, n-block tn, split-K slice s and its k-steps [ks0, ks1)), wave-uniform
  // (divisions by host magic numbers: ConvArgs mg_mn / mg_ntn / mg_ks)
  auto unit = [&](int u, int& m0, int& tn, int& s, int& ks0, int& ks1) {
    s = po::div_by(u, a.mg_mn, a.sh_mn);
    const int rem = u - s * mn;
    const int tm = po::div_by(rem, a.mg_ntn, a.sh_ntn);
    tn = rem - tm * a.ntiles_n;
    m0 = tm * T4;
    ks0 = po::div_by(s * kc_n, a.mg_ks, a.sh_ks);
    ks1 = po::div_by((s + 1) * kc_n, a.mg_ks, a.sh_ks);
  };

  // ---- input staging: thread (tile r, channel pair tc) loads its 4x4 patch, 2 channels
  const int r = tid >> 3, tc = tid & 7;
  uint32_t off[16];
  auto offsets = [&](int m0) {
    int b, ti, tj;
    const bool ok_t = tile_point_magic(a, Ht, Wt, m0 + r, b, ti, tj);
    const uint32_t pix_bytes = (uint32_t)a.Cin_p * 4u;
    // (one row product per patch row, the columns as uniform steps: the same
    // offsets modulo 2^32 with 4 instead of 16 pairs of quarter-rate multiplies)
    const int y0 = 2 * ti - 1, x0 = 2 * tj - 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int y = y0 + i;
      const bool rok = ok_t && (unsigned)y < (unsigned)a.Hin;
      const uint32_t rb = (((uint32_t)b * a.Hin + y) * a.Win + x0) * pix_bytes + 8u * tc;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = rok && (unsigned)(x0 + j) < (unsigned)a.Win;
        off[4 * i + j] = ok ? rb + (uint32_t)j * pix_bytes : kOOB;
      }
    }
  };
  f2v d[16];
  auto gload = [&](int ks) {
    const uint32_t cb = (uint32_t)__builtin_amdgcn_readfirstlane(ks * (WK * 4));
#pragma unroll
    for (int p = 0; p < 16; ++p) d[p] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(in_rs, off[p], cb, 0));
  };
  auto transform = [&](float* Vb) {
    f2v t[4][4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const f2v d0 = d[v], d1 = d[4 + v], d2 = d[8 + v], d3 = d[12 + v];
      t[0][v] = d0 - d2;
      t[1][v] = d1 + d2;
      t[2][v] = d2 - d1;
      t[3][v] = d1 - d3;
    }
    const int sub = (tc & 1) * 2;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f2v e[4] = {t[u][0] - t[u][2], t[u][1] + t[u][2], t[u][2] - t[u][1], t[u][1] - t[u][3]};
#pragma unroll
      for (int v = 0; v < 4; ++v) *reinterpret_cast<f2v*>(Vb + v4idx(u * 4 + v, r, tc >> 1) + sub) = e[v];
    }
  };

  // ---- B operand (fragment-ordered U) per component, one k-step ahead: buffer
  // loads with a per-lane 16-byte offset and the block offset in a scalar
  // register (no 64-bit per-lane pointer held across the unit loop)
  const __amdgpu_buffer_rsrc_t u_rs = rsrc(U, (uint32_t)a.N * 16u * (uint32_t)a.Cin_p * 4u);
  const uint32_t u_lane = (uint32_t)lane * 16u;
  float4 bq[CPW][2][2];
  int tn = 0;
  auto bload = [&](int c, int ks) {
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const uint32_t blk = (uint32_t)__builtin_amdgcn_readfirstlane(
          ((((2 * tn + nb) * kc_n + ks) * 16 + wave_u * CPW + c) * 512) * 4);
      bq[c][nb][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(u_rs, u_lane, blk, 0));
      bq[c][nb][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(u_rs, u_lane + 1024u, blk, 0));
    }
  };
  floatx16 acc[CPW][2][2];
  auto mfma_c = [&](int c, const float* Vb) {
    const int xi = wave_u * CPW + c;
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      const int t = 32 * mb + (lane & 31);
      const float4 a0 = *reinterpret_cast<const float4*>(Vb + v4idx(xi, t, 2 * h));
      const float4 a1 = *reinterpret_cast<const float4*>(Vb + v4idx(xi, t, 2 * h + 1));
      const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const float bv[8] = {bq[c][nb][0].x, bq[c][nb][0].y, bq[c][nb][0].z, bq[c][nb][0].w,
                             bq[c][nb][1].x, bq[c][nb][1].y, bq[c][nb][1].z, bq[c][nb][1].w};
#pragma unroll
        for (int s8 = 0; s8 < 8; ++s8)        // MFMA step s, half h <-> channel 8h + s
          acc[c][mb][nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s8], bv[s8], acc[c][mb][nb], 0, 0, 0);
      }
    }
  };

  // ---- epilogue state of the staged unit: inverse-transformed sums, positions, loaded inputs
  constexpr bool RES = MODE == 0 && (EF & EF_RES), ACC = MODE == 0 && (EF & EF_ACC);
  constexpr bool MB = MODE == 0 && (EF & EF_MB), Y2 = MODE == 0 && (EF & EF_Y2);
  float4 yv[2][2][2];                    // [pass][p >> 1][p & 1]
  float4 pin[2][4];                      // the shortcut operand or the accumulated destination
  uint32_t pm[2][4], pm2[2][4];          // leaky-mask sign-bit words
  uint32_t vpix[2], vok[2];              // per pass: first pixel (MODE 1: workspace row) of the tile, output mask
  uint32_t vslice = 0u;
  int vn4 = 0;
  float4 bias4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int ps = 0; ps < 2; ++ps) {
    vpix[ps] = vok[ps] = 0u;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      yv[ps][p >> 1][p & 1] = pin[ps][p] = make_float4(0.f, 0.f, 0.f, 0.f);
      pm[ps][p] = pm2[ps][p] = 0u;
    }
  }

  // outputs of the staged unit (the same stores every time; masked ones out of range)
  auto emit = [&]() {
#pragma unroll
    for (int ps = 0; ps < 2; ++ps) {
      if constexpr (MODE == 1) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const bool ok = (vok[ps] >> p) & 1u;
          const uint32_t row = vpix[ps] + (uint32_t)(p >> 1) * a.Wg + (p & 1);
          const uint32_t o = ((vslice * (uint32_t)a.M + row) * (uint32_t)a.N + vn4) * 4u;
          bst4(yv[ps][p >> 1][p & 1], rs_out, ok ? o : kOOB);
        }
      } else if constexpr (MODE == 2) {
        // tile 68's fused pool (even map): the 2x2 tile is pool window (vti, vtj)
        float pv[4] = {0.f, 0.f, 0.f, 0.f};
        uint32_t arg[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float4 v = yv[ps][k >> 1][k & 1];
          float x[4] = {v.x + bias4.x, v.y + bias4.y, v.z + bias4.z, v.w + bias4.w};
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            x[c] = po::leaky_or_id(x[c], po::act_slope(a.act));
            if (k == 0 || x[c] > pv[c] || isnan(x[c])) { pv[c] = x[c]; arg[c] = (uint32_t)k; }
          }
        }
        uint32_t code = 0u;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (a.act) arg[c] |= 8u | (pv[c] > 0.f ? 0u : 4u);
          code |= arg[c] << (8 * c);
        }
        const bool ok = vok[ps] == 0xFu;
        const uint32_t po = vpix[ps] * (uint32_t)a.Cout_p + vn4;     // vpix: the pooled pixel
        bst4(make_float4(pv[0], pv[1], pv[2], pv[3]), rs_out, ok ? po * 4u : kOOB);
        bst1(code, rs_aux, ok ? po : kOOB);
      } else {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const bool ok = (vok[ps] >> p) & 1u;
          const uint32_t pix = vpix[ps] + (uint32_t)(p >> 1) * a.Wout + (p & 1);
          const uint32_t o = (pix * (uint32_t)a.Cout_p + vn4) * 4u;
          const float4 v = yv[ps][p >> 1][p & 1];
          float x[4] = {v.x + bias4.x, v.y + bias4.y, v.z + bias4.z, v.w + bias4.w};
#pragma unroll
          for (int c = 0; c < 4; ++c) x[c] = po::leaky_or_id(x[c], po::act_slope(a.act));
          if constexpr (ACC) {
            x[0] += pin[ps][p].x; x[1] += pin[ps][p].y; x[2] += pin[ps][p].z; x[3] += pin[ps][p].w;
          }
          float4 out = make_float4(x[0], x[1], x[2], x[3]);
          if constexpr (MB) {
            const float4 g = po::leaky_grad_bits(pm[ps][p], vn4);
            out = make_float4(x[0] * g.x, x[1] * g.y, x[2] * g.z, x[3] * g.w);
          }
          if constexpr ((EF & EF_Y) != 0) bst4(out, rs_out, ok ? o : kOOB);
          if constexpr (RES) {
            const float4 rr = pin[ps][p];
            bst4(make_float4(x[0] + rr.x, x[1] + rr.y, x[2] + rr.z, x[3] + rr.w), rsrc(a.sum, dst_bytes), ok ? o : kOOB);
          }
          if constexpr (Y2) {
            const float4 g2 = po::leaky_grad_bits(pm2[ps][p], vn4);
            bst4(make_float4(x[0] * g2.x, x[1] * g2.y, x[2] * g2.z, x[3] * g2.w), rsrc(a.y2, dst_bytes), ok ? o : kOOB);
          }
          if constexpr ((EF & EF_YB) != 0) {
            // sign bits: 8 lanes hold the 32 channels of one word
            // (masked, not branched: a divergent branch here costs an exec save/restore per pixel)
            const uint32_t nib = ((out.x > 0.f ? 1u : 0u) | (out.y > 0.f ? 2u : 0u) | (out.z > 0.f ? 4u : 0u) |
                                  (out.w > 0.f ? 8u : 0u)) & (0u - (uint32_t)ok);
            // (OR of lanes i..i+7 into lane i by DPP row shifts, dst[i] = src[i + n] within
            // a 16-lane row: VALU-rate, where __shfl_xor's three dependent LDS crossbar
            // round trips per pixel were ~1 us of every unit's emit)
            uint32_t w = nib << (4 * (lane & 7));
            w |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x101, 0xF, 0xF, false);   // row_shl:1
            w |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x102, 0xF, 0xF, false);   // row_shl:2
            w |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x104, 0xF, 0xF, false);   // row_shl:4
            bst1(w, rsrc(a.ybits, bits_bytes),
                 (ok && (lane & 7) == 0) ? (pix * (uint32_t)wpp + (uint32_t)(vn4 >> 5)) * 4u : kOOB);
          }
        }
      }
    }
  };

  // ---- the unit loop
  int u = po::xcd_remap();               // host: gridDim.x <= units
  int m0, s, ks0, ks1;
  unit(u, m0, tn, s, ks0, ks1);
  offsets(m0);
  gload(ks0);
  float* M = smem;
  for (;;) {
    emit();                              // the previous unit's outputs (none on the first pass)
    __syncthreads();                     // its M reads are done everywhere: V0 may be rewritten
    transform(smem);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < CPW; ++c)
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[c][mb][nb][e] = 0.f;
    int ks = ks0;
    if (wave_u >= 4) {
      // tile 68's stagger: waves 4-7 transform the next step before their MFMAs
      gload(ks0 + 1);
      __builtin_amdgcn_sched_barrier(0);
      bload(0, ks0);
      __builtin_amdgcn_sched_barrier(0);
      bload(1, ks0);
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
      do {                                 // steps ks0 .. ks1-2 (host: ks1 - ks0 >= 2)
        float* Vc = smem + ((ks - ks0) & 1) * V4_FLOATS;
        float* Vn = smem + (((ks - ks0) & 1) ^ 1) * V4_FLOATS;
        const int k1 = ks + 1, k2 = min(ks + 2, ks1 - 1);
        transform(Vn);
        __builtin_amdgcn_sched_barrier(0);
        gload(k2);
        __builtin_amdgcn_sched_barrier(0);
        mfma_c(0, Vc);
        __builtin_amdgcn_sched_barrier(0);
        bload(0, k1);
        __builtin_amdgcn_sched_barrier(0);
        mfma_c(1, Vc);
        __builtin_amdgcn_sched_barrier(0);
        bload(1, k1);
        __syncthreads();
      } while (++ks < ks1 - 1);
    } else {
      bload(0, ks0);
      __builtin_amdgcn_sched_barrier(0);
      gload(ks0 + 1);
      __builtin_amdgcn_sched_barrier(0);
      bload(1, ks0);
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
      do {
        float* Vc = smem + ((ks - ks0) & 1) * V4_FLOATS;
        float* Vn = smem + (((ks - ks0) & 1) ^ 1) * V4_FLOATS;
        const int k1 = ks + 1, k2 = min(ks + 2, ks1 - 1);
        mfma_c(0, Vc);
        __builtin_amdgcn_sched_barrier(0);
        bload(0, k1);
        __builtin_amdgcn_sched_barrier(0);
        transform(Vn);
        __builtin_amdgcn_sched_barrier(0);
        gload(k2);
        __builtin_amdgcn_sched_barrier(0);
        mfma_c(1, Vc);
        __builtin_amdgcn_sched_barrier(0);
        bload(1, k1);
        __syncthreads();
      } while (++ks < ks1 - 1);
    }
    {                                      // the last step, peeled: nothing prefetched past the unit
      const float* Vc = smem + ((ks1 - 1 - ks0) & 1) * V4_FLOATS;
      mfma_c(0, Vc);
      __builtin_amdgcn_sched_barrier(0);
      mfma_c(1, Vc);
      __builtin_amdgcn_sched_barrier(0);
    }
    const int cur_m0 = m0, cur_tn = tn, cur_s = s;
    // ---- the next unit's first input rows, requested under the last MFMAs so
    // they arrive during the staging (the last unit re-reads its own: branch-free)
    const int nu = u + G;
    const bool more = nu < units;
    unit(more ? nu : u, m0, tn, s, ks0, ks1);
    offsets(m0);
    gload(ks0);

    // ---- this unit's epilogue positions (tile 68's per pass: tile tid >> 4, channels n4 .. n4+3)
    const int n4 = cur_tn * N4 + 4 * (lane & 15);
    uint32_t cpix[2], cok[2];
#pragma unroll
    for (int ps = 0; ps < 2; ++ps) {
      int vb = 0, vti = 0, vtj = 0;
      const bool tl = tile_point_magic(a, Ht, Wt, cur_m0 + TH * ps + (tid >> 4), vb, vti, vtj);
      uint32_t ok4 = 0u;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int i = 2 * vti + (p >> 1), j = 2 * vtj + (p & 1);
        if (tl && i < a.Hout && j < a.Wout) ok4 |= 1u << p;
      }
      cok[ps] = ok4;
      cpix[ps] = MODE == 2 ? ((uint32_t)vb * (a.Hout >> 1) + vti) * (a.Wout >> 1) + vtj
               : MODE == 1 ? (uint32_t)vb * a.mrows + (uint32_t)(2 * vti) * a.Wg + 2 * vtj
                           : ((uint32_t)vb * a.Hout + 2 * vti) * a.Wout + 2 * vtj;
    }

    // ---- stage the accumulators through LDS and inverse-transform (tile 68's two passes)
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      __syncthreads();                     // the k-loop's (or the previous pass's) LDS reads are done
      // LDS indices made opaque here, per unit: the compiler would otherwise keep
      // (or spill) a dozen precomputed addresses across the whole k-loop
      int wrow = (wave * CPW * TH + 4 * h) * N4 + (lane & 31);
      asm volatile("" : "+v"(wrow));
#pragma unroll
      for (int c = 0; c < CPW; ++c)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int t = (e & 3) + 8 * (e >> 2);
            M[wrow + (c * TH + t) * N4 + nb * 32] = acc[c][pass][nb][e];
          }
      __syncthreads();
      // this pass's epilogue inputs, issued before the next unit's input rows so
      // the emit's wait for them leaves those rows in flight
      if (pass == 0 && MODE != 1) bias4 = bld4(rs_bias, (uint32_t)n4 * 4u);
      if constexpr (RES || ACC || MB || Y2) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const bool ok = (cok[pass] >> p) & 1u;
          const uint32_t pix = cpix[pass] + (uint32_t)(p >> 1) * a.Wout + (p & 1);
          const uint32_t o = (pix * (uint32_t)a.Cout_p + n4) * 4u;
          const uint32_t wo = (pix * (uint32_t)wpp + (uint32_t)(n4 >> 5)) * 4u;
          if constexpr (RES) pin[pass][p] = bld4(rsrc(a.res, dst_bytes), ok ? o : kOOB);
          if constexpr (ACC) pin[pass][p] = bld4(rs_out, ok ? o : kOOB);
          if constexpr (MB) pm[pass][p] = bld1(rsrc(a.mbits, bits_bytes), ok ? wo : kOOB);
          if constexpr (Y2) pm2[pass][p] = bld1(rsrc(a.m2bits, bits_bytes), ok ? wo : kOOB);
        }
      }
      int rrow = (tid >> 4) * N4 + 4 * (lane & 15);
      asm volatile("" : "+v"(rrow));
      float4 s0[4], s1[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float4 m[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          m[q] = *reinterpret_cast<const float4*>(M + (q * 4 + v) * TH * N4 + rrow);
        s0[v] = f4add(f4add(m[0], m[1]), m[2]);
        s1[v] = f4sub(f4sub(m[1], m[2]), m[3]);
      }
      yv[pass][0][0] = f4add(f4add(s0[0], s0[1]), s0[2]);
      yv[pass][0][1] = f4sub(f4sub(s0[1], s0[2]), s0[3]);
      yv[pass][1][0] = f4add(f4add(s1[0], s1[1]), s1[2]);
      yv[pass][1][1] = f4sub(f4sub(s1[1], s1[2]), s1[3]);
    }
    vpix[0] = cpix[0];
    vpix[1] = cpix[1];
    vok[0] = cok[0];
    vok[1] = cok[1];
    vn4 = n4;
    vslice = (uint32_t)cur_s;
    if (!more) break;
    u = nu;
  }
  emit();
}
}  // namespace

namespace po {
// po_conv tile staging 15 (tile 70): conv_wino5_k, tile 68 as a persistent
// kernel (one workgroup per CU) pipelined across its units (see above).
int launch_wino5(const ConvArgs& a, const float* U, hipStream_t st) {
  PO_REQUIRE(U, "po_conv: Winograd tile needs the transformed weights (Wwino)");
  PO_REQUIRE(a.prec == 0 && a.ntaps == 9 && a.tkw == 3 && (a.sdh == 1 || a.sdh == -1) && (a.sdw == 1 || a.sdw == -1) &&
                 a.dh0 == -a.sdh && a.dw0 == -a.sdw,
             "po_conv: Winograd tile needs a full 3x3 neighbourhood of taps");
  PO_REQUIRE(a.in_step == 1 && a.out_step == 1 && a.out_oy == 0 && a.out_ox == 0 && !a.in_org && !a.out_org && !a.gbox,
             "po_conv: tile 70 needs stride 1 on full maps without boxes");
  PO_REQUIRE(a.Hg == a.Hout && a.Wg == a.Wout && a.Hin == a.Hout && a.Win == a.Wout,
             "po_conv: Winograd tile needs source, grid and destination of one size");
  PO_REQUIRE(a.N % N4 == 0 && a.Cin_p % WK == 0, "po_conv: tile 70 needs N %% 64 == 0 and Cin_p %% 16 == 0");
  PO_REQUIRE(a.Cin_p / WK >= 2 * a.ksplit, "po_conv: tile 70 needs at least two k-steps per slice");
  PO_REQUIRE(a.ksplit == 1 || (!a.pool_y && a.ws && (int64_t)a.ksplit * a.M * a.N * 4 < (1LL << 31)),
             "po_conv: tile 70 split-K needs a workspace of < 2^31 bytes");
  PO_REQUIRE(!a.pool_y || (a.Hout % 2 == 0 && a.Wout % 2 == 0), "po_conv: a fused pool needs an even map");
  PO_REQUIRE(!a.mask && !a.mask2 && !a.y_amax && !a.sum_amax && !a.y2_amax,
             "po_conv: tile 70 takes leaky masks as sign bits and no max|x| slots");
  PO_REQUIRE((int64_t)a.B * a.Hout * a.Wout * a.Cout_p * 4 < (1LL << 31),
             "po_conv: tile 70 addresses the destination with 32-bit byte offsets (< 2^31 bytes)");
  const int Ht = (a.Hout + 1) / 2, Wt = (a.Wout + 1) / 2;
  ConvArgs b = a;
  b.ntiles_n = a.N / N4;
  div_magic(Ht * Wt, b.mg_tiles, b.sh_tiles);
  div_magic(Wt, b.mg_wt, b.sh_wt);
  const int ntm = ceil_div((int64_t)a.B * Ht * Wt, T4);
  const int mn = ntm * b.ntiles_n;
  div_magic(mn, b.mg_mn, b.sh_mn);
  div_magic(b.ntiles_n, b.mg_ntn, b.sh_ntn);
  div_magic(a.ksplit, b.mg_ks, b.sh_ks);
  PO_REQUIRE((int64_t)mn * a.ksplit < (1LL << 31), "po_conv: too many tiles");
  const int units = mn * a.ksplit;
  PO_REQUIRE(!(a.res && a.accumulate), "po_conv: tile 70 does not accumulate a shortcut launch");
  const int ef = (a.y ? EF_Y : 0) | (a.res ? EF_RES : 0) | (a.accumulate ? EF_ACC : 0) | (a.mbits ? EF_MB : 0) |
                 (a.y2 ? EF_Y2 : 0) | (a.ybits ? EF_YB : 0);
  const void* k = nullptr;
  int which = 0;
  // the epilogue-field combinations po_conv launches on full-map Winograd tiles
#define PO_W5(MODE, EF)                                             \
  case (MODE) * 64 + (EF):                                          \
    k = reinterpret_cast<const void*>(conv_wino5_k<MODE, EF>);      \
    break;
  which = a.ksplit > 1 ? 64 : a.pool_y ? 128 : ef;
  switch (which) {
    PO_W5(1, 0)
    PO_W5(2, 0)
    PO_W5(0, EF_Y)
    PO_W5(0, EF_Y | EF_YB)
    PO_W5(0, EF_RES | EF_YB)
    PO_W5(0, EF_Y | EF_RES)
    PO_W5(0, EF_Y | EF_RES | EF_YB)
    PO_W5(0, EF_Y | EF_ACC)
    PO_W5(0, EF_Y | EF_MB)
    PO_W5(0, EF_Y | EF_ACC | EF_MB)
    PO_W5(0, EF_Y | EF_Y2)
    PO_W5(0, EF_Y | EF_ACC | EF_Y2)
    PO_W5(0, EF_Y | EF_MB | EF_Y2)
    PO_W5(0, EF_Y | EF_ACC | EF_MB | EF_Y2)
    default:
      break;
  }
#undef PO_W5
  PO_REQUIRE(k, "po_conv: tile 70 has no kernel for epilogue fields 0x%x", which);
  // one workgroup per CU (the occupancy of this build), at most one per unit
  const int resident = resident_groups_cached(k, 512);
  const int grid = units < resident ? units : resident;
  void* args[] = {&b, const_cast<float**>(&U), const_cast<int*>(&Ht), const_cast<int*>(&Wt),
                  const_cast<int*>(&units), const_cast<int*>(&mn)};
  PO_REQUIRE(hipLaunchKernel(k, dim3(grid), dim3(512), args, 0, st) == hipSuccess, "po_conv: tile 70 launch failed");
  return check_launch("po_conv (winograd persistent)");
}
}  // namespace po
