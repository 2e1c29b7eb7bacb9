// Row-marching variant of the fused 2-D PDS iteration (separable convolution, fp32) for the
// column-interior 64-column strips; the boundary strips run the tile kernel (pds_tile.hpp).
//
// Same arithmetic per pixel as the tile kernel, organised so that the vertical halos of the
// two column passes are not recomputed: one workgroup owns a 64-column strip of a row segment
// [s0, s1) and marches down it TS = 16 rows per step, keeping
//   XR  x rows                 in a 32-row LDS ring
//   RR  residual r = h*x - y   in a 32-row LDS ring (rows [a-H, a+TS+H] live at step a)
// so every x row is read from HBM once per strip and every residual row is computed once.
// Step k (a = s0 + 16k; residual chunk k = rows [a+H+1, a+H+1+TS)):
//   top   issue loads: x rows of chunk k+1, y of chunk k+1, x on the U rows, z of step k
//   P1    A  = column conv of x             (chunk k)           XR -> A
//   P2    r  = row conv of A - y            (chunk k)           A, RR(y) -> RR  (0 outside the image)
//   P3    B  = column corr of r             U rows [a, a+TS]    RR -> B
//         land z -> Z0/Z1 and x rows of chunk k+1 -> XR
//   P45   g = row corr of B (= Conv^T r), x_t = prox_G(x - tau g - tau K^T z), u = 2x_t - x,
//         x' = rho x_t + (1-rho) x; park y of chunk k+1 in RR
//   P6    z' = rho fenchel(z + sigma K u) + (1-rho) z
// Global loads are issued once per step, unconditionally (clamped items, clamped rows with a
// zero select), so hipcc's wait counting stays exact and each load is first used two phases
// after its issue; barriers are raw s_barrier after lgkmcnt(0) (no vmcnt drain).
// Reference: PrimalDualSplitting.update_iterand, pycsou/opt/proxalgs.py:343-355, with
// grad F = Conv^T((2 (Conv x - y)) 0.5) (core/map.py:609-610) and Conv from
// pycsou/linop/conv.py:167-295 (separable PSF: conv along axis 0 then axis 1).
#pragma once

#include "pds_tile.hpp"

namespace pcs {

template <int H>
struct March {
  static constexpr int TW = 64, TS = 16, RING = 32, UROWS = TS + 1;
  static constexpr int H4 = RU4<H>::value, SH = H4 - H;
  static constexpr int WG = TW + 4, GG = WG / 4;       // U / Z columns [c0, c0 + WG) (col c0 + TW: u only)
  static constexpr int WR = WG + 2 * H4, GR = WR / 4;  // residual / B columns [c0 - H4, c0 + WG + H4)
  static constexpr int WX = WG + 4 * H4, GX = WX / 4;  // x / A columns [c0 - 2 H4, c0 + WG + 2 H4)
  // P2 items: 1 row x 2 groups; per row pair, the first 8 items of each row go to the 16 lanes
  // of one ds_read_b128 lane group, the remaining NX2 of each row to the other lane group
  static constexpr int NG2 = 2, NPR2 = (GR + 1) / 2, NX2 = NPR2 - 8;
  static constexpr int NZ0 = UROWS * GG, NZ1 = UROWS * (GG + 1);
  static constexpr int NXN = TS * GX;           // new x rows per step
  static constexpr int NXP = (TS + 2 * H) * GX;  // prologue x rows
  // LDS layout (elements)
  static constexpr int O_XR = 0, SZ_XR = RING * WX;
  static constexpr int O_RR = O_XR + SZ_XR, SZ_RR = RING * WR;
  static constexpr int O_A = O_RR + SZ_RR, SZ_A = TS * WX + 4 * NG2;  // P2's last item reads 4 past a row
  static constexpr int O_U = O_A + SZ_A, SZ_U = UROWS * WG;             // u ring: row r in slot (r - s0) % 17
  static constexpr int O_B = O_U + SZ_U, SZ_B = TS * WR;
  static constexpr int O_Z0 = O_B + SZ_B, SZ_Z0 = UROWS * WG;
  static constexpr int O_Z1 = O_Z0 + SZ_Z0, SZ_Z1 = UROWS * (WG + 4);
  static constexpr int O_W = O_Z1 + SZ_Z1, SZ_W = 32;  // taps w0, w1 zero-padded to the tier, 16 each
  static constexpr int SZ = O_W + SZ_W;
  static_assert(H == 3 || H == 7, "tiers 3 and 7 (the 5-column row correlation of P45 needs H = H4 - 1)");
  static_assert(TS + 2 * H + 1 <= RING, "x ring holds rows [a - 1, a + TS + 2H + 1)");
  static_assert(TS >= 2 * H + 1 && 2 * TS <= RING, "residual ring holds [a + 1 - H, a + TS + H]");
  static_assert(GX <= 32 && GR <= 32 && NX2 >= 1 && NX2 <= 8, "row blocks fit 32 lanes");
  static_assert((GX & 1) && (GR & 1), "odd slot pitches: P2's row pairs hit distinct b128 slots");
};

// Diagnostic build only (-DPCS_STAMPS): per-segment s_memtime totals of waves 0 and 3 of
// every block -> g_pcs_stamps (read by pcs_debug_stamps); never compiled into the product.
#ifdef PCS_STAMPS
__device__ unsigned long long g_pcs_stamps[4096][16];
__device__ __forceinline__ unsigned long long pcs_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define PCS_ST(i)                              \
  do {                                         \
    const unsigned long long t_ = pcs_stamp(); \
    st_acc[i] += t_ - st_last;                 \
    st_last = t_;                              \
  } while (0)
#else
#define PCS_ST(i) \
  do {            \
  } while (0)
#endif


// Own-row bands of one launch: segments [ra0, rb0) first (nseg0 of them), then [ra1, rb1).
// The whole slab is {seg_len, nseg, 0, rows, rows, rows}; the multi-GPU loop launches the
// two boundary bands (the rows its neighbours' halos need) apart from the interior band so
// that the halo exchange overlaps the interior.
struct Bands {
  int seg_len, nseg0, ra0, rb0, ra1, rb1;
};
// Border-strip split of a row-march launch (the stencil march): tasks [0, nint) run the interior strips
// [ilo, ilo + iw) with segments bd, tasks [nint, ntasks) the border strips bs[0 .. nbs) with the shorter
// segments bdb.  nint < 0: one segmentation for every strip (task = seg * tiles_x + strip).
struct StripSplit {
  int nint, ilo, iw, nbs;
  int bs[3];
  Bands bdb;
};
__device__ __forceinline__ void band_rows(const Bands& bd, int seg, int& s0, int& s1) {
  if (seg < bd.nseg0) {
    s0 = bd.ra0 + seg * bd.seg_len;
    s1 = min(s0 + bd.seg_len, bd.rb0);
  } else {
    s0 = bd.ra1 + (seg - bd.nseg0) * bd.seg_len;
    s1 = min(s0 + bd.seg_len, bd.rb1);
  }
}

#ifndef PCS_ABL
#define PCS_ABL 0
#endif
// 32-bit slab geometry (the host checks (rows + 2 halo) * n1 < 2^31 for this kernel)
struct Slab32 {
  int n0, n1, row0, rows, hx, hy, hz, vec;
};

// a uniform value held in a VGPR (keeps the taps out of the 102-SGPR budget)
__device__ __forceinline__ float to_vgpr(float v) {
  float r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

// Bounds-checked 16-B loads through a buffer descriptor: a byte offset at or past the
// descriptor's size reads 0 (hardware range check), so rows outside the image / the stored
// slab and columns outside [0, n1) cost no branch and no select -- their offset carries kOOB.
// Each part (row, column) is either valid or kOOB; with every view <= 2^30 bytes a sum with
// any kOOB part is >= the size and two kOOB parts (2^31) cannot wrap.
__device__ __forceinline__ G4<float> bload4(Rsrc r, uint32_t off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return {{__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3])}};
}
// 16-B store through a descriptor: an offset carrying kOOB is dropped by the range check
// AUX: cache-policy bits of the store (0 = plain; 16 = sc1, written through and dropped from L2)
template <int AUX = 0>
__device__ __forceinline__ void bstore4(Rsrc r, uint32_t off, const G4<float>& g) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const u4 d = {__float_as_uint(g.v[0]), __float_as_uint(g.v[1]), __float_as_uint(g.v[2]), __float_as_uint(g.v[3])};
#if PCS_ABL & 1024
  if (PCS_ABL) off = kOOB;
#endif
  __builtin_amdgcn_raw_buffer_store_b128(d, r, (int)off, 0, AUX);
}

// Element-typed forms for kernels templated on the element type: a 4-column group is one 16-B
// access in fp32 and two (off, off + 16) in fp64; a single element is a b32 / b64 access.  A kOOB
// offset stays out of range in the second half too (kOOB + 16 < 2^31 is still >= every size).
template <typename T>
__device__ __forceinline__ G4<T> bload4t(Rsrc r, uint32_t off);
template <>
__device__ __forceinline__ G4<float> bload4t<float>(Rsrc r, uint32_t off) {
  return bload4(r, off);
}
template <>
__device__ __forceinline__ G4<double> bload4t<double>(Rsrc r, uint32_t off) {
  const auto a = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  const auto b = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(off + 16u), 0, 0);
  G4<double> g;
  __builtin_memcpy(&g.v[0], &a, 16);
  __builtin_memcpy(&g.v[2], &b, 16);
  return g;
}
template <typename T>
__device__ __forceinline__ T bload1t(Rsrc r, uint32_t off);
template <>
__device__ __forceinline__ float bload1t<float>(Rsrc r, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
template <>
__device__ __forceinline__ double bload1t<double>(Rsrc r, uint32_t off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0);
  double d;
  __builtin_memcpy(&d, &v, 8);
  return d;
}
template <typename T, int AUX = 0>
__device__ __forceinline__ void bstore4t(Rsrc r, uint32_t off, const G4<T>& g) {
  if constexpr (sizeof(T) == 4) {
    bstore4<AUX>(r, off, g);
  } else {
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    u4 a, b;
    __builtin_memcpy(&a, &g.v[0], 16);
    __builtin_memcpy(&b, &g.v[2], 16);
    __builtin_amdgcn_raw_buffer_store_b128(a, r, (int)off, 0, AUX);
    __builtin_amdgcn_raw_buffer_store_b128(b, r, (int)(off + 16u), 0, AUX);
  }
}

// Diagnostic ablation builds only (-DPCS_ABL=bits, tools/build_var.sh): 1 = z not landed in LDS,
// 2 = y not parked, 4 = new x rows not stored, 8/16/32 = P1/P2/P3 skipped, 64/128 = P45/P6 reduced to
// their stores, 256 = without those stores, 512 = no LDS barriers, 1024 = loads from 4 rows (L2-resident) and
// stores dropped: compute with almost no HBM traffic, 2048 = normal-operator kernel without its two
// conv passes (results wrong; timing only).
// z of step k+1 is loaded at the top of step k and landed in LDS at the top of step k+1, so its
// latency hides behind a whole step (0: loaded and landed within the step, behind P1-P3 only)
#ifndef PCS_ZAHEAD
#define PCS_ZAHEAD 1
#endif
#if PCS_ABL & 512
#define PCS_MB() do { } while (0)
#else
#define PCS_MB() lds_barrier()
#endif
__device__ __forceinline__ void keep4(const G4<float>& g) {
  asm volatile("" ::"v"(g.v[0]), "v"(g.v[1]), "v"(g.v[2]), "v"(g.v[3]));
}

// One halo'd array: its descriptor, row pitch in bytes, and the local rows it can supply
// (stored AND inside the image): [lo, hi].
struct View {
  Rsrc r;
  int halo, lo, hi;
  uint32_t pitch;
  __device__ __forceinline__ uint32_t row_off(int lr) const {
#if PCS_ABL & 1024
    if (PCS_ABL) return ((unsigned)(lr - lo) <= (unsigned)(hi - lo)) ? (uint32_t)((lr & 3) + halo) * pitch : kOOB;
#endif
    return ((unsigned)(lr - lo) <= (unsigned)(hi - lo)) ? (uint32_t)(lr + halo) * pitch : kOOB;
  }
};
// esz: element size in bytes (4: fp32, 8: fp64)
__device__ __forceinline__ View make_view(const void* base, const Slab32& s, int halo, uint32_t esz = 4u) {
  View v;
  v.halo = halo;
  v.lo = max(-halo, -s.row0);
  v.hi = min(s.rows + halo, s.n0 - s.row0) - 1;
  v.pitch = (uint32_t)s.n1 * esz;
  v.r = rsrc_of(base, (uint32_t)(s.rows + 2 * halo) * v.pitch);
  return v;
}
// byte offset of column c inside a row (kOOB outside the image; 4-groups are wholly in/out)
__device__ __forceinline__ uint32_t col_off(int c, int n1, uint32_t esz = 4u) {
  return ((unsigned)c < (unsigned)n1) ? (uint32_t)c * esz : kOOB;
}

// A loop-invariant value re-materialised in a VGPR every step, so tests on it stay inside the
// loop instead of being hoisted into 64-bit lane masks (SGPR spills).
__device__ __forceinline__ int launder(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// Column (vertical) pass over a 32-row LDS ring for one 4-column group: acc[m] (m < RR) =
// sum_t w[REV ? 2H-t : t] * ring[sl + m + t].  The RR + 2H input rows are read once each with
// PF reads in flight (explicit read-ahead: a read is consumed PF reads after its issue, which
// covers the LDS latency that a read-then-use order leaves exposed).
template <typename T, int H, int RR, bool REV, int PF>
__device__ __forceinline__ void vpass(const T* __restrict__ ring, int pitch, int sl, int col,
                                      const T (&w)[2 * H + 1], G4<T> (&acc)[RR]) {
  constexpr int NR = RR + 2 * H, NT2 = 2 * H + 1;
  G4<T> buf[PF];
#pragma unroll
  for (int m = 0; m < RR; ++m)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[m].v[e] = T(0);
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (p < NR) buf[p] = lds4(ring + ((sl + p) & 31) * pitch + col);
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const G4<T> v = buf[j % PF];
    if (j + PF < NR) buf[j % PF] = lds4(ring + ((sl + j + PF) & 31) * pitch + col);
#pragma unroll
    for (int m = 0; m < RR; ++m) {
      const int t = j - m;
      if (t >= 0 && t < NT2) {
        const T wt = w[REV ? 2 * H - t : t];
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[m].v[e] += wt * v.v[e];
      }
    }
  }
}

template <typename T, int H, int HK, int NT>
__device__ __forceinline__ void march_task(const T* __restrict__ x, T* __restrict__ xn, const T* __restrict__ z,
                                           T* __restrict__ zn, const T* __restrict__ y, const T* __restrict__ taps0,
                                           const T* __restrict__ taps1, int half, const Slab32& s, const Params<T>& P, int gk,
                                           int s0, int s1, int c0, T* sm, double (&part)[4]) {
  static_assert(sizeof(T) == 4 && NT == 256, "the march kernel is fp32, 256 threads (8 row pairs x 32 lanes)");
  using M = March<H>;
  constexpr int TS = M::TS, TW = M::TW, H4 = M::H4, SH = M::SH, NT2 = 2 * H + 1;
  constexpr int WX = M::WX, WR = M::WR, WG = M::WG, GX = M::GX, GR = M::GR, GG = M::GG;
  constexpr int NG2 = M::NG2, NX2 = M::NX2;
  constexpr int KXN = cdiv(M::NXN, NT), KXP = cdiv(M::NXP, NT), KZ0 = cdiv(M::NZ0, NT), KZ1 = cdiv(M::NZ1, NT);
  T* XR = sm + M::O_XR;
  T* RR = sm + M::O_RR;
  T* A = sm + M::O_A;
  T* U = sm + M::O_U;
  T* B = sm + M::O_B;
  T* Z0 = sm + M::O_Z0;
  T* Z1 = sm + M::O_Z1;
  T* W = sm + M::O_W;
  const int tid = threadIdx.x;
  if (tid < 32) {  // centred taps, zero-padded from `half` to the tier H (visible after the first barrier)
    const int t = tid & 15;
    const bool ok = t < NT2 && (t - H >= -half) && (t - H <= half);
    W[tid] = ok ? (tid < 16 ? taps0 : taps1)[t - H + half] : T(0);
  }
  // taps are re-read from LDS at the top of every phase that uses them (uniform broadcast
  // reads into VGPRs): 30 taps held in SGPRs across the loop would spill the SGPR file
  auto ldtaps = [&](int k, T(&w)[NT2]) {
#pragma unroll
    for (int q = 0; q < (NT2 + 3) / 4; ++q) {
      const G4<T> t4 = lds4(W + 16 * k + 4 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (4 * q + e < NT2) w[4 * q + e] = t4.v[e];
    }
  };
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hb = tid >> 5, l5 = tid & 31;  // every phase: 32 lanes per row pair / row block hb
  const int lgrp = lane_grp(l5), lidx = lane_idx(l5);
  const int n0 = s.n0, n1 = s.n1;
  const int zstride = (s.rows + 2 * s.hz) * n1;
  const int xb = s0 - TS + 1;      // x ring base row (smallest row ever stored)
  const int rb = s0 - TS + H + 1;  // residual ring base row
  const int xc0 = c0 - 2 * H4;     // first column of the x / A region
  const int rc0 = c0 - H4;         // first column of the residual region
  const View vx = make_view(x, s, s.hx), vy = make_view(y, s, s.hy), vz0 = make_view(z, s, s.hz),
             vz1 = make_view(z + zstride, s, s.hz);
  const uint32_t pitch = (uint32_t)n1 * 4u;
  const Rsrc rxn = rsrc_of(xn, (uint32_t)(s.rows + 2 * s.hx) * pitch);
  const Rsrc rzn0 = rsrc_of(zn, (uint32_t)zstride * 4u), rzn1 = rsrc_of(zn + zstride, (uint32_t)zstride * 4u);
#define PCS_WAVE_ON(k, N) ((k) * NT + wv * 64 < (N))
#define PCS_ITEM(k, N) min((k) * NT + tid, (N) - 1)

  // ---- fixed per-thread geometry
  const int g1 = row_lane_group<GX>(l5);  // P1: rows [2 hb, 2 hb + 2) of the chunk, group g1
  const int g3 = row_lane_group<GR>(l5);  // P3: B rows [2 hb, 2 hb + 2), group g3
  int p2_sub, p2_j;                       // P2: row 2 hb + p2_sub, groups 2 p2_j, 2 p2_j + 1
  if (lgrp == 0) {
    p2_sub = lidx >> 3;
    p2_j = lidx & 7;
  } else {  // lanes past the 2 NX2 items repeat one of them (broadcast reads, identical writes)
    const int e = lidx % (2 * NX2);
    p2_sub = e / NX2;
    p2_j = 8 + e - p2_sub * NX2;
  }
  const int p2_r = 2 * hb + p2_sub, p2_g0 = 2 * p2_j;
  const int ui = 2 * hb + lgrp, ug = lidx;  // P45 / P6: row ui of the step, column group ug
  const int ucg = c0 + 4 * ug;
  const uint32_t co_u = col_off(ucg, n1);
  uint32_t co_y[NG2], co_xn[KXN], co_z0[KZ0], co_z1[KZ1];
  int rr_xn[KXN], rr_z0[KZ0], rr_z1[KZ1];  // row (relative) of each load item
  // bit q: P2 group q in the image; 2: U group in; 3: U column c + 4 in; 4: U group is the last
  int flags = 0;
#pragma unroll
  for (int q = 0; q < NG2; ++q) {
    co_y[q] = col_off(rc0 + 4 * min(p2_g0 + q, GR - 1), n1);
    flags |= ((unsigned)(rc0 + 4 * (p2_g0 + q)) < (unsigned)n1) << q;
  }
  flags |= (ucg < n1) << 2;
  flags |= (ucg + 4 < n1) << 3;
  flags |= (ucg == n1 - 4) << 4;
#pragma unroll
  for (int k = 0; k < KXN; ++k) {
    const int e = PCS_ITEM(k, M::NXN);
    rr_xn[k] = e / GX;
    co_xn[k] = col_off(xc0 + 4 * (e - (e / GX) * GX), n1);
  }
#pragma unroll
  for (int k = 0; k < KZ0; ++k) {
    const int e = PCS_ITEM(k, M::NZ0);
    rr_z0[k] = e / GG;
    co_z0[k] = col_off(c0 + 4 * (e - (e / GG) * GG), n1);
  }
#pragma unroll
  for (int k = 0; k < KZ1; ++k) {
    const int e = PCS_ITEM(k, M::NZ1);
    rr_z1[k] = e / (GG + 1);
    co_z1[k] = col_off(c0 - 4 + 4 * (e - (e / (GG + 1)) * (GG + 1)), n1);
  }

  auto load_y = [&](G4<T>(&yv)[NG2], int cs) {  // y of residual chunk rows [cs, cs + TS)
    const uint32_t ro = vy.row_off(cs + p2_r);
#pragma unroll
    for (int q = 0; q < NG2; ++q) yv[q] = bload4(vy.r, ro + co_y[q]);
  };
  auto store_y = [&](const G4<T>(&yv)[NG2], int cs) {  // parked where P2 writes r
    T* dst = RR + ((cs + p2_r - rb) & 31) * WR;
#if PCS_ABL & 2
    if (PCS_ABL) {
      for (int q = 0; q < NG2; ++q) keep4(yv[q]);
      return;
    }
#endif
#pragma unroll
    for (int q = 0; q < NG2; ++q)
      if (GR % NG2 == 0 || p2_g0 + q < GR) st4(dst + 4 * (p2_g0 + q), yv[q]);
  };
  auto load_xn = [&](G4<T>(&xv)[KXN], int r0) {  // x rows [r0, r0 + TS) of the X region
#pragma unroll
    for (int k = 0; k < KXN; ++k) xv[k] = bload4(vx.r, vx.row_off(r0 + rr_xn[k]) + co_xn[k]);
  };
  auto store_xn = [&](const G4<T>(&xv)[KXN], int r0) {
#if PCS_ABL & 4
    if (PCS_ABL) {
      for (int k = 0; k < KXN; ++k) keep4(xv[k]);
      return;
    }
#endif
#pragma unroll
    for (int k = 0; k < KXN; ++k) {
      if (!PCS_WAVE_ON(k, M::NXN)) continue;
      const int e = PCS_ITEM(k, M::NXN);
      const int r = e / GX, g = e - (e / GX) * GX;
      st4(XR + ((r0 + r - xb) & 31) * WX + 4 * g, xv[k]);
    }
  };
  // z0 rows [a, a + TS], cols [c0, c0 + WG) -> Z0 (pitch WG); z1 rows [a, a + TS], cols from c0 - 4 -> Z1
  auto load_z = [&](G4<T>(&zr0)[KZ0], G4<T>(&zr1)[KZ1], int a) {
#pragma unroll
    for (int k = 0; k < KZ0; ++k) zr0[k] = bload4(vz0.r, vz0.row_off(a + rr_z0[k]) + co_z0[k]);
#pragma unroll
    for (int k = 0; k < KZ1; ++k) zr1[k] = bload4(vz1.r, vz1.row_off(a + rr_z1[k]) + co_z1[k]);
  };
  auto land_z = [&](const G4<T>(&zr0)[KZ0], const G4<T>(&zr1)[KZ1]) {
#if PCS_ABL & 1
    if (PCS_ABL) {
      for (int k = 0; k < KZ0; ++k) keep4(zr0[k]);
      for (int k = 0; k < KZ1; ++k) keep4(zr1[k]);
      return;
    }
#endif
#pragma unroll
    for (int k = 0; k < KZ0; ++k)
      if (PCS_WAVE_ON(k, M::NZ0)) st4(Z0 + 4 * PCS_ITEM(k, M::NZ0), zr0[k]);
#pragma unroll
    for (int k = 0; k < KZ1; ++k)
      if (PCS_WAVE_ON(k, M::NZ1)) st4(Z1 + 4 * PCS_ITEM(k, M::NZ1), zr1[k]);
  };
  // ---- P1: A rows [cs, cs + TS) = column conv of x (forward: out[i] = sum_t w0[2H - t] x[i - H + t])
  auto p1 = [&](int cs) {
#if PCS_ABL & 8
    if (PCS_ABL) return;
#endif
    const int sl = (cs + 2 * hb - H - xb) & 31;
    T w0[NT2];
    ldtaps(0, w0);
    G4<T> acc[2];
    vpass<T, H, 2, true, 4>(XR, WX, sl, 4 * g1, w0, acc);
#pragma unroll
    for (int m = 0; m < 2; ++m) st4(A + (2 * hb + m) * WX + 4 * g1, acc[m]);
  };
  // ---- P2: residual rows [cs, cs + TS) = row conv of A - y (y parked in RR), 0 outside the image
  auto p2 = [&](int cs, int fl) {
#if PCS_ABL & 16
    if (PCS_ABL) return;
#endif
    constexpr int NV = NG2 + H4 / 2;
    T w1[NT2];
    ldtaps(1, w1);
    T v[4 * NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const G4<T> t4 = lds4(A + p2_r * WX + 4 * (p2_g0 + q));
#pragma unroll
      for (int ee = 0; ee < 4; ++ee) v[4 * q + ee] = t4.v[ee];
    }
    const int lr = cs + p2_r, gr = s.row0 + lr;
    const bool rin = gr >= 0 && gr < n0;
    T* dst = RR + ((lr - rb) & 31) * WR;
#pragma unroll
    for (int q = 0; q < NG2; ++q) {
      if (GR % NG2 == 0 || p2_g0 + q < GR) {
        const G4<T> yq = lds4(dst + 4 * (p2_g0 + q));
        const bool in = rin && ((fl >> q) & 1);
        G4<T> o;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          T acc = T(0);
#pragma unroll
          for (int t = 0; t < NT2; ++t) acc += w1[2 * H - t] * v[4 * q + m + SH + t];
          asm volatile("" : "+v"(acc));  // keep the select below a select (no branch around the taps)
          // r = Conv x - y   (grad = Conv^T((2*(r + (-y)))*0.5), map.py:609-610: exact)
          o.v[m] = in ? (acc - yq.v[m]) : T(0);
        }
        st4(dst + 4 * (p2_g0 + q), o);
      }
    }
  };
  // ---- P3: B rows [a + 1, a + 1 + TS) = column correlation of r (out[i] = sum_t w0[t] r[i - H + t])
  auto p3 = [&](int a) {
#if PCS_ABL & 32
    if (PCS_ABL) return;
#endif
    const int sl = (a + 1 + 2 * hb - H - rb) & 31;
    T w0[NT2];
    ldtaps(0, w0);
    G4<T> acc[2];
    vpass<T, H, 2, false, 4>(RR, WR, sl, 4 * g3, w0, acc);
#pragma unroll
    for (int m = 0; m < 2; ++m) st4(B + (2 * hb + m) * WR + 4 * g3, acc[m]);
  };
  // ---- P45: row lr = a + 1 + ui: grad F = row correlation of B, x_t = prox_G(x - tau g - tau K^T z),
  //      u = 2 x_t - x on columns [c, c + 5) (column c + 4 = the next group's first: only group 15
  //      stores it, for P6's right neighbour), x' = rho x_t + (1 - rho) x
  auto p45 = [&](int a, int fl, int ub) {
#if PCS_ABL & 64
    if (PCS_ABL) {
      const int lr = a + 1 + ui;
      const G4<T> xv4 = lds4(XR + ((lr - xb) & 31) * WX + 2 * H4 + 4 * ug);
      const bool own = lr >= s0 && lr < s1 && s.row0 + lr < s.n0 && ((fl >> 2) & 1);
      if (PCS_ABL & 256) keep4(xv4);
      else bstore4(rxn, (own ? (uint32_t)(lr + s.hx) * pitch : kOOB) + co_u, xv4);
      return;
    }
#endif
    const int i = ui, g = ug;
    const int lr = a + 1 + i, gr = s.row0 + lr;
    int slot = i + 1 + ub;
    slot = slot >= 17 ? slot - 17 : slot;
    constexpr int NV = 1 + H4 / 2;
    T w1[NT2];
    ldtaps(1, w1);
    T v[4 * NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const G4<T> t4 = lds4(B + i * WR + 4 * g + 4 * q);
#pragma unroll
      for (int ee = 0; ee < 4; ++ee) v[4 * q + ee] = t4.v[ee];
    }
    const T* xrow = XR + ((lr - xb) & 31) * WX + 2 * H4 + 4 * g;
    const G4<T> xv4 = lds4(xrow);
    const G4<T> za = lds4(Z0 + i * WG + 4 * g);              // z0[lr - 1]
    const G4<T> zb = lds4(Z0 + (i + 1) * WG + 4 * g);        // z0[lr]
    const G4<T> z1a = lds4(Z1 + (i + 1) * (WG + 4) + 4 * g);  // z1[lr][c - 4 .. c - 1]
    const G4<T> z1b = lds4(Z1 + (i + 1) * (WG + 4) + 4 * g + 4);  // z1[lr][c .. c + 3]
    const T xe = xrow[4], zae = Z0[i * WG + 4 * g + 4], zbe = Z0[(i + 1) * WG + 4 * g + 4];
    const T z1e = Z1[(i + 1) * (WG + 4) + 4 * g + 8];
    const bool r_last = gr >= n0 - 1, r_first = gr <= 0;
    const bool rrow = gr < n0 && lr <= s.rows;
    const bool cin = (fl >> 2) & 1, cin_e = (fl >> 3) & 1, clast = (fl >> 4) & 1;
    const bool own = lr >= s0 && lr < s1 && gr < n0 && cin;
    G4<T> uo, xo;
    T ue = T(0), sdx = T(0), sx = T(0);
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      T gd = T(0);
#pragma unroll
      for (int t = 0; t < NT2; ++t) gd += w1[t] * v[m + SH + t];
      const T xv = m < 4 ? xv4.v[m] : xe;
      // K^T z for forward differences, VStack order: (0 + D0^T z0) + D1^T z1; z1 left of the
      // image loads as 0; z1 on the last column is not used (forward difference there is 0)
      const T zl = (m == 0) ? z1a.v[3] : z1b.v[m - 1];
      const T zr = m < 4 ? z1b.v[m] : z1e;
      T d0 = r_first ? T(0) : (m < 4 ? za.v[m] : zae);
      if (!r_last) d0 -= (m < 4 ? zb.v[m] : zbe);
      const T d1 = zl - ((m == 3 && clast) ? T(0) : zr);
      const T xt = prox_g((xv - P.tau * gd) - P.tau * (d0 * P.inv_step0 + d1 * P.inv_step1), gk, P.seg_a, P.seg_b);
      const bool in = rrow && (m < 4 ? cin : cin_e);
      const T u = in ? (T(2) * xt - xv) : T(0);
      if (m < 4) {
        uo.v[m] = u;
        const T xnew = P.rho * xt + P.omr * xv;
        xo.v[m] = xnew;
        const T dx = xv - xnew;
        sdx += dx * dx;
        sx += xv * xv;
      } else {
        ue = u;
      }
    }
    if (own) {  // per-item partials: 4 terms in fp32, accumulated in fp64
      part[0] += (double)sdx;
      part[1] += (double)sx;
    }
    st4(U + slot * WG + 4 * g, uo);
    if (g == TW / 4 - 1) U[slot * WG + TW] = ue;
    bstore4(rxn, (own ? (uint32_t)(lr + s.hx) * pitch : kOOB) + co_u, xo);
  };
  // ---- P6: z' on row lr = a + ui
  auto p6 = [&](int a, int fl, int ub) {
#if PCS_ABL & 128
    if (PCS_ABL) {
      const int lr = a + ui;
      const G4<T> zv0 = lds4(Z0 + ui * WG + 4 * ug);
      const bool own = lr < s1 && s.row0 + lr < s.n0 && ((fl >> 2) & 1);
      const uint32_t off = (own ? (uint32_t)(lr + s.hz) * pitch : kOOB) + co_u;
      if (PCS_ABL & 256) {
        keep4(zv0);
      } else {
        bstore4(rzn0, off, zv0);
        bstore4(rzn1, off, zv0);
      }
      return;
    }
#endif
    const int i = ui, g = ug;
    const int lr = a + i, gr = s.row0 + lr;
    int sl0 = i + ub, sl1 = i + 1 + ub;
    sl0 = sl0 >= 17 ? sl0 - 17 : sl0;
    sl1 = sl1 >= 17 ? sl1 - 17 : sl1;
    const G4<T> uc = lds4(U + sl0 * WG + 4 * g);
    const G4<T> ud = lds4(U + sl1 * WG + 4 * g);
    const G4<T> zv0 = lds4(Z0 + i * WG + 4 * g);
    const G4<T> zv1 = lds4(Z1 + i * (WG + 4) + 4 * g + 4);
    const T une = U[sl0 * WG + 4 * g + 4];
    const bool cin = (fl >> 2) & 1, clast = (fl >> 4) & 1;
    const bool r_last = gr >= n0 - 1;
    const bool own = lr < s1 && gr < n0 && cin;
    G4<T> o0, o1;
    T sdz = T(0), sz = T(0);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const T uright = (m < 3) ? uc.v[m + 1] : une;
      const T d0 = r_last ? T(0) : (ud.v[m] - uc.v[m]);
      const T d1 = (m == 3 && clast) ? T(0) : (uright - uc.v[m]);
      const T w0v = zv0.v[m] + P.sigma * (d0 * P.inv_step0), w1v = zv1.v[m] + P.sigma * (d1 * P.inv_step1);
      const T v0 = w0v * P.inv_sigma, v1 = w1v * P.inv_sigma;
      T zt0, zt1;
      if (HK == PCS_H_L21) {  // w - sigma * (max(1 - t/||v||, 0) v), penalty.py:551-557
        T f = T(1) - P.t_h * fast_rsqrt(v0 * v0 + v1 * v1);
        f = f > T(0) ? f : T(0);
        zt0 = w0v - P.sigma * (f * v0);
        zt1 = w1v - P.sigma * (f * v1);
      } else {  // w - sigma * (v - t*clip(v/t)), func/base.py:239-240
        zt0 = w0v - P.sigma * (v0 - P.t_h * clip1(v0 * P.inv_t_h));
        zt1 = w1v - P.sigma * (v1 - P.t_h * clip1(v1 * P.inv_t_h));
      }
      o0.v[m] = P.rho * zt0 + P.omr * zv0.v[m];
      o1.v[m] = P.rho * zt1 + P.omr * zv1.v[m];
      const T e0 = zv0.v[m] - o0.v[m], e1 = zv1.v[m] - o1.v[m];
      sdz += e0 * e0 + e1 * e1;
      sz += zv0.v[m] * zv0.v[m] + zv1.v[m] * zv1.v[m];
    }
    if (own) {
      part[2] += (double)sdz;
      part[3] += (double)sz;
    }
    const uint32_t off = (own ? (uint32_t)(lr + s.hz) * pitch : kOOB) + co_u;
    bstore4(rzn0, off, o0);
    bstore4(rzn1, off, o1);
  };

  // ================= prologue: residual chunk -1 (rows [rb, rb + TS)), u on row s0, chunk 0's inputs
  G4<T> ynx[NG2], xnx[KXN], zr0[KZ0], zr1[KZ1];
  {
    G4<T> xv[KXP];
#pragma unroll
    for (int k = 0; k < KXP; ++k) {  // x rows [s0 - TS + 1, s0 + 2H + 1) = chunk -1's reach
      const int e = PCS_ITEM(k, M::NXP);
      const int r = e / GX, g = e - (e / GX) * GX;
      xv[k] = bload4(vx.r, vx.row_off(xb + r) + col_off(xc0 + 4 * g, n1));
    }
    load_y(ynx, rb);
    load_xn(xnx, s0 + 2 * H + 1);  // chunk 0's new x rows (land after the prologue's P45)
#pragma unroll
    for (int k = 0; k < KXP; ++k) {
      if (!PCS_WAVE_ON(k, M::NXP)) continue;
      const int e = PCS_ITEM(k, M::NXP);
      const int r = e / GX, g = e - (e / GX) * GX;
      st4(XR + (r & 31) * WX + 4 * g, xv[k]);
    }
    store_y(ynx, rb);
    load_y(ynx, rb + TS);  // chunk 0's y
    load_z(zr0, zr1, s0 - TS);
  }
  PCS_MB();
  p1(rb);
  PCS_MB();
  store_y(ynx, rb + TS);
  p2(rb, launder(flags));
  PCS_MB();
  p3(s0 - TS);  // B row TS - 1 = row s0 (the rows above it read stale ring rows: unused)
  land_z(zr0, zr1);
  if (PCS_ZAHEAD) load_z(zr0, zr1, s0);  // step 0's z (landed at the top of step 0)
  PCS_MB();
  p45(s0 - TS, launder(flags), 1);  // u on row s0 -> ring slot 0, x' on row s0 (other rows: not own)
  PCS_MB();
  store_xn(xnx, s0 + 2 * H + 1);

  // ================= march: step k covers B / u / x' rows [a + 1, a + TS], z' rows [a, a + TS)
#ifdef PCS_STAMPS
  unsigned long long st_acc[13] = {0}, st_last = pcs_stamp();
#endif
  const int nsteps = (s1 - s0 + TS - 1) / TS;
  int ub = 0;  // (-k) mod 17: row r = a + j sits in u ring slot (j + ub) mod 17
  for (int k = 0; k < nsteps; ++k) {
    const int a = s0 + k * TS;
    const int cs = a + H + 1;  // residual chunk k rows [cs, cs + TS)
    PCS_ST(0);
    PCS_MB();  // step k-1 done with U, Z, B and with the XR rows landed in its P6
    PCS_ST(1);
    const int fl = launder(flags);
    // ---- this step's global loads, all issued here (first use: after P3 / in P6, or next step)
    if (PCS_ZAHEAD) land_z(zr0, zr1);  // z of this step, loaded during the previous one
    load_xn(xnx, a + TS + 2 * H + 1);  // chunk k+1's new x rows
    load_y(ynx, cs + TS);              // chunk k+1's y
    load_z(zr0, zr1, PCS_ZAHEAD ? a + TS : a);
    PCS_ST(2);
    p1(cs);
    PCS_ST(3);
    PCS_MB();
    PCS_ST(4);
    p2(cs, fl);
    PCS_ST(5);
    PCS_MB();
    PCS_ST(6);
    p3(a);
    PCS_ST(7);
    if (!PCS_ZAHEAD) land_z(zr0, zr1);
    PCS_ST(8);
    PCS_MB();
    PCS_ST(9);
    store_y(ynx, cs + TS);  // RR slots of chunk k+1 held chunk k-1, last read by P3 above
    p45(a, fl, ub);
    PCS_ST(10);
    PCS_MB();
    PCS_ST(11);
    p6(a, fl, ub);
    store_xn(xnx, a + TS + 2 * H + 1);  // XR slots of rows P45 read above
    ub = ub == 0 ? 16 : ub - 1;
    PCS_ST(12);
  }
#ifdef PCS_STAMPS
  PCS_ST(0);
  if ((tid & 63) == 0 && (wv == 0 || wv == 3)) {
    const int row = 2 * (int)blockIdx.x + (wv == 3);
    if (row < 4096) {
#pragma unroll
      for (int i = 0; i < 13; ++i) g_pcs_stamps[row][i] = st_acc[i];
      g_pcs_stamps[row][13] = nsteps;
    }
  }
#endif
#undef PCS_WAVE_ON
#undef PCS_ITEM
}

// One block per task (64-column strip x row segment); with `hist` the last workgroups also
// reduce the partials and run the loop control, with `ro.sums` they only reduce.
template <typename T, int H, int HK, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(3))) void k_pds2d_march(
    const T* __restrict__ x, T* __restrict__ xn, const T* __restrict__ z, T* __restrict__ zn,
    const T* __restrict__ y, const T* __restrict__ taps0, const T* __restrict__ taps1, int half, Slab32 s,
    Params<T> P, int gk, double* __restrict__ partials, Ctrl* ctrl, double* hist, void* ws, RedOut ro,
    int tiles_x, Bands bd, int ntasks) {
  using M = March<H>;
  __shared__ __attribute__((aligned(16))) T sm[M::SZ];
  __shared__ double red[4 * (NT / 64)];
  __shared__ int flag[2];
  if (fin_slot(ro, ntasks, ctrl, hist, red, flag)) return;  // deferred finalization (pds_ctrl.hpp)
  const bool stopped = stop_requested(ctrl, ro, flag);
  if (stopped && ro.sums == nullptr) return;  // loop already stopped (solver.py:65-66)

  // XCD-aware bijective remap: blocks b, b+8, ... share an XCD -> adjacent strips of a segment
  int task;
  {
    const int b = (int)blockIdx.x - fin_shift(ro), q = ntasks / 8, r = ntasks % 8, xcd = b % 8, k = b / 8;
    task = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  const int seg = task / tiles_x, strip = task - seg * tiles_x;
  int s0, s1;
  band_rows(bd, seg, s0, s1);
  const int c0 = strip * M::TW;

  double part[4] = {0.0, 0.0, 0.0, 0.0};
  if (!stopped) march_task<T, H, HK, NT>(x, xn, z, zn, y, taps0, taps1, half, s, P, gk, s0, s1, c0, sm, part);
  block_sum<4>(part, red);
  publish_partials(part, partials, ntasks, ws, ctrl, hist, flag, ro);
}

}  // namespace pcs
