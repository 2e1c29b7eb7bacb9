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
  static constexpr int TW = 64, TS = 16, UR = TS + 1, RING = 32;
  static constexpr int H4 = RU4<H>::value;
  static constexpr int WG = TW + 4, GG = WG / 4;          // U cols [c0, c0 + WG)
  static constexpr int WR = WG + 2 * H4, GR = WR / 4;     // residual cols [c0 - H4, c0 + WG + H4)
  static constexpr int WX = WG + 4 * H4, GX = WX / 4;     // x / A cols [c0 - 2 H4, c0 + WG + 2 H4)
  // P1 items: RR1 rows x 1 group, 32 lanes per row block (lanes past the row's groups redo its
  // last group) so every 16-lane ds_read_b128 group reads 16 distinct slots of one row
  static constexpr int RR1 = 2, NI1 = (TS / RR1) * 32;                         // P1
  static constexpr int NG2 = 2, NPR2 = (GR + NG2 - 1) / NG2, NI2 = TS * NPR2;  // P2: 1 row x 2 groups
  static constexpr int RR3 = 2, NQ3 = (UR + RR3 - 1) / RR3, NI3 = NQ3 * GR;    // P3: 2 rows x 1 group
  static constexpr int NI5 = UR * GG, NI6 = TS * (TW / 4);
  static constexpr int NZ0 = (UR + 1) * GG, NZ1 = UR * (GG + 1);
  static constexpr int NXN = TS * GX;                       // new x rows per step
  static constexpr int NXP = (TS + 2 * H) * GX;             // prologue x rows
  // LDS layout (elements)
  static constexpr int O_XR = 0, SZ_XR = RING * WX;
  static constexpr int O_RR = O_XR + SZ_XR, SZ_RR = RING * WR;
  static constexpr int SZ_A = TS * WX + 4 * NG2;  // P2's last item reads up to 4 (NG2 - 1) past a row
  static constexpr int SZ_U = UR * WG;
  static constexpr int O_AU = O_RR + SZ_RR, SZ_AU = SZ_A > SZ_U ? SZ_A : SZ_U;
  static constexpr int O_B = O_AU + SZ_AU, SZ_B = NQ3 * RR3 * WR;  // P3 writes rows up to NQ3*RR3
  static constexpr int O_Z0 = O_B + SZ_B, SZ_Z0 = (UR + 1) * WG;
  static constexpr int O_Z1 = O_Z0 + SZ_Z0, SZ_Z1 = UR * (WG + 4);
  static constexpr int SZ = O_Z1 + SZ_Z1;
  static_assert(TS + 2 * H + 1 <= RING, "x ring holds rows [a+1, a+TS+2H+1) plus the next chunk's rows");
  static_assert(TS >= 2 * H + 1 && 2 * TS <= RING, "residual ring holds two chunks covering [a - H, a + TS + H]");
  static_assert(GX <= 32 && GR <= 32, "a row block fits 32 lanes");
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

// Workgroup barrier for LDS hand-offs only: LDS ops drained, global loads and stores left in
// flight (__syncthreads()' release fence waits vmcnt(0)).  No wave of this kernel reads
// global data another wave of the launch wrote.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

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
constexpr uint32_t kOOB = 0x40000000u;
typedef __amdgpu_buffer_rsrc_t Rsrc;

__device__ __forceinline__ Rsrc rsrc_of(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ G4<float> bload4(Rsrc r, uint32_t off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return {{__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3])}};
}

// One halo'd array: its descriptor, row pitch in bytes, and the local rows it can supply
// (stored AND inside the image): [lo, hi].
struct View {
  Rsrc r;
  int halo, lo, hi;
  uint32_t pitch;
  __device__ __forceinline__ uint32_t row_off(int lr) const {
    return ((unsigned)(lr - lo) <= (unsigned)(hi - lo)) ? (uint32_t)(lr + halo) * pitch : kOOB;
  }
};
__device__ __forceinline__ View make_view(const void* base, const Slab32& s, int halo) {
  View v;
  v.halo = halo;
  v.lo = max(-halo, -s.row0);
  v.hi = min(s.rows + halo, s.n0 - s.row0) - 1;
  v.pitch = (uint32_t)s.n1 * 4u;
  v.r = rsrc_of(base, (uint32_t)(s.rows + 2 * halo) * v.pitch);
  return v;
}
// byte offset of column c inside a row (kOOB outside the image; 4-groups are wholly in/out)
__device__ __forceinline__ uint32_t col_off(int c, int n1) {
  return ((unsigned)c < (unsigned)n1) ? (uint32_t)c * 4u : kOOB;
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

template <typename T, int H, int NT>
__device__ __forceinline__ void march_task(const T* __restrict__ x, T* __restrict__ xn, const T* __restrict__ z,
                                           T* __restrict__ zn, const T* __restrict__ y, const T (&w0)[2 * H + 1],
                                           const T (&w1)[2 * H + 1], const Slab32& s, const Params<T>& P, int hk,
                                           int gk, int s0, int s1, int c0, T* sm, double (&part)[4]) {
  static_assert(sizeof(T) == 4, "the march kernel is fp32");
  using M = March<H>;
  constexpr int TS = M::TS, TW = M::TW, H4 = M::H4, SH = H4 - H, NT2 = 2 * H + 1;
  constexpr int WX = M::WX, WR = M::WR, WG = M::WG, GX = M::GX, GR = M::GR, GG = M::GG;
  constexpr int RR1 = M::RR1, NG2 = M::NG2, NPR2 = M::NPR2, RR3 = M::RR3;
  constexpr int KXN = cdiv(M::NXN, NT), KXP = cdiv(M::NXP, NT), KZ0 = cdiv(M::NZ0, NT), KZ1 = cdiv(M::NZ1, NT);
  constexpr int K5 = cdiv(M::NI5, NT), K6 = cdiv(M::NI6, NT);
  static_assert(M::NI1 <= NT && M::NI2 <= NT && M::NI3 <= NT, "one item per thread in P1-P3");
  static_assert(2 * NG2 + 2 * K5 + 2 * K6 <= 31, "column flags fit one word");
  T* XR = sm + M::O_XR;
  T* RR = sm + M::O_RR;
  T* A = sm + M::O_AU;
  T* U = sm + M::O_AU;
  T* B = sm + M::O_B;
  T* Z0 = sm + M::O_Z0;
  T* Z1 = sm + M::O_Z1;
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n0 = s.n0, n1 = s.n1;
  const int zstride = (s.rows + 2 * s.hz) * n1;
  const int xb = s0 - TS + 1;      // x ring base row (smallest row ever stored)
  const int rb = s0 - TS + H + 1;  // residual ring base row
  const int xc0 = c0 - 2 * H4;     // first column of the x / A region
  const int rc0 = c0 - H4;         // first column of the residual region
  const View vx = make_view(x, s, s.hx), vy = make_view(y, s, s.hy), vz0 = make_view(z, s, s.hz),
             vz1 = make_view(z + zstride, s, s.hz);
  // is batch k of an N-item phase non-empty for this wave (uniform)?  clamped item of this lane
#define PCS_WAVE_ON(k, N) ((k) * NT + wv * 64 < (N))
#define PCS_ITEM(k, N) min((k) * NT + tid, (N) - 1)

  // ---- fixed per-thread item geometry (clamped items) and the column part of every load
  const int p2_e = PCS_ITEM(0, M::NI2);
  const int p2_r = p2_e / NPR2, p2_g0 = (p2_e - (p2_e / NPR2) * NPR2) * NG2;
  const bool p2_wave = PCS_WAVE_ON(0, M::NI2);
  uint32_t co_y[NG2], co_xn[KXN], co_xu[K5], co_z0[KZ0], co_z1[KZ1];
  int rr_xn[KXN], rr_xu[K5], rr_z0[KZ0], rr_z1[KZ1];  // row (relative) of each load item
  int flags = 0;  // bit q: P2 group q in the image; 2NG2+kk: P45 item in; +K5: P45 last group; P6 likewise
#pragma unroll
  for (int q = 0; q < NG2; ++q) {
    const int g = (GR % NG2 == 0) ? p2_g0 + q : min(p2_g0 + q, GR - 1);
    co_y[q] = col_off(rc0 + 4 * g, n1);
    flags |= ((unsigned)(rc0 + 4 * (p2_g0 + q)) < (unsigned)n1) << q;
  }
#pragma unroll
  for (int k = 0; k < KXN; ++k) {
    const int e = PCS_ITEM(k, M::NXN);
    rr_xn[k] = e / GX;
    co_xn[k] = col_off(xc0 + 4 * (e - (e / GX) * GX), n1);
  }
#pragma unroll
  for (int k = 0; k < K5; ++k) {
    const int e = PCS_ITEM(k, M::NI5);
    rr_xu[k] = e / GG;
    const int cg = c0 + 4 * (e - (e / GG) * GG);
    co_xu[k] = col_off(cg, n1);
    flags |= (cg < n1) << (NG2 + k);
    flags |= (cg == n1 - 4) << (NG2 + K5 + k);
  }
#pragma unroll
  for (int k = 0; k < K6; ++k) {
    const int e = PCS_ITEM(k, M::NI6);
    const int cg = c0 + 4 * (e - (e / (TW / 4)) * (TW / 4));
    flags |= (cg < n1) << (NG2 + 2 * K5 + k);
    flags |= (cg == n1 - 4) << (NG2 + 2 * K5 + K6 + k);
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
    if (p2_wave) {
      T* dst = RR + ((cs + p2_r - rb) & 31) * WR;
#pragma unroll
      for (int q = 0; q < NG2; ++q)
        if (GR % NG2 == 0 || p2_g0 + q < GR) st4(dst + 4 * (p2_g0 + q), yv[q]);
    }
  };
  auto load_xn = [&](G4<T>(&xv)[KXN], int r0) {  // x rows [r0, r0 + TS) of the X region
#pragma unroll
    for (int k = 0; k < KXN; ++k) xv[k] = bload4(vx.r, vx.row_off(r0 + rr_xn[k]) + co_xn[k]);
  };
  auto store_xn = [&](const G4<T>(&xv)[KXN], int r0) {
#pragma unroll
    for (int k = 0; k < KXN; ++k) {
      if (!PCS_WAVE_ON(k, M::NXN)) continue;
      const int e = PCS_ITEM(k, M::NXN);
      const int r = e / GX, g = e - (e / GX) * GX;
      st4(XR + ((r0 + r - xb) & 31) * WX + 4 * g, xv[k]);
    }
  };
  // ---- P1: A rows [cs, cs + TS) = column conv of x (forward: out[i] = sum_t w0[2H - t] x[i - H + t])
  auto p1 = [&](int cs) {
    if (PCS_WAVE_ON(0, M::NI1)) {
      const int e = PCS_ITEM(0, M::NI1);
      const int q = e >> 5, g = min(e & 31, GX - 1);
      const int sl = (cs + q * RR1 - H - xb) & 31;
      G4<T> acc[RR1];
      vpass<T, H, RR1, true, 4>(XR, WX, sl, 4 * g, w0, acc);
#pragma unroll
      for (int m = 0; m < RR1; ++m) st4(A + (q * RR1 + m) * WX + 4 * g, acc[m]);
    }
  };
  // ---- P2: residual rows [cs, cs + TS) = row conv of A - y (y parked in RR), 0 outside the image
  auto p2 = [&](int cs, int fl) {
    if (p2_wave) {
      constexpr int NV = NG2 + H4 / 2;
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
            // r = Conv x - y   (grad = Conv^T((2*(r + (-y)))*0.5), map.py:609-610: exact)
            o.v[m] = in ? (acc - yq.v[m]) : T(0);
          }
          st4(dst + 4 * (p2_g0 + q), o);
        }
      }
    }
  };

  // ================= prologue: residual chunk -1 (rows [rb, rb + TS)) and chunk 0's inputs
  G4<T> ynx[NG2], xnx[KXN];
  {
    G4<T> xv[KXP];
#pragma unroll
    for (int k = 0; k < KXP; ++k) {  // x rows [s0 - TS + 1, s0 + 2H + 1) = chunk -1's reach
      const int e = PCS_ITEM(k, M::NXP);
      const int r = e / GX, g = e - (e / GX) * GX;
      xv[k] = bload4(vx.r, vx.row_off(xb + r) + col_off(xc0 + 4 * g, n1));
    }
    load_y(ynx, rb);
    load_xn(xnx, s0 + 2 * H + 1);  // chunk 0's new x rows (land after P1 of chunk -1)
#pragma unroll
    for (int k = 0; k < KXP; ++k) {
      if (!PCS_WAVE_ON(k, M::NXP)) continue;
      const int e = PCS_ITEM(k, M::NXP);
      const int r = e / GX, g = e - (e / GX) * GX;
      st4(XR + (r & 31) * WX + 4 * g, xv[k]);
    }
    store_y(ynx, rb);
    load_y(ynx, rb + TS);  // chunk 0's y
  }
  lds_barrier();
  p1(rb);
  lds_barrier();
  store_xn(xnx, s0 + 2 * H + 1);
  store_y(ynx, rb + TS);
  p2(rb, launder(flags));

  // ================= march
#ifdef PCS_STAMPS
  unsigned long long st_acc[13] = {0}, st_last = pcs_stamp();
#endif
  const int nsteps = (s1 - s0 + TS - 1) / TS;
  for (int k = 0; k < nsteps; ++k) {
    const int a = s0 + k * TS;
    const int cs = a + H + 1;  // residual chunk k rows [cs, cs + TS)
    PCS_ST(0);
    lds_barrier();  // step k-1 done with U, Z, and with the XR / RR rows landing below
    PCS_ST(1);
    const int fl = launder(flags);
    // ---- this step's global loads, all issued here (first use: after P3)
    load_xn(xnx, a + TS + 2 * H + 1);  // chunk k+1's new x rows
    load_y(ynx, cs + TS);              // chunk k+1's y
    G4<T> xu[K5], zr0[KZ0], zr1[KZ1];
#pragma unroll
    for (int kk = 0; kk < K5; ++kk) xu[kk] = bload4(vx.r, vx.row_off(a + rr_xu[kk]) + co_xu[kk]);  // U rows
#pragma unroll
    for (int kk = 0; kk < KZ0; ++kk) zr0[kk] = bload4(vz0.r, vz0.row_off(a - 1 + rr_z0[kk]) + co_z0[kk]);
#pragma unroll
    for (int kk = 0; kk < KZ1; ++kk) zr1[kk] = bload4(vz1.r, vz1.row_off(a + rr_z1[kk]) + co_z1[kk]);
    PCS_ST(2);
    p1(cs);
    PCS_ST(3);
    lds_barrier();
    PCS_ST(4);
    p2(cs, fl);
    PCS_ST(5);
    lds_barrier();
    PCS_ST(6);
    // ---- P3: B rows [a, a + NQ3*RR3) = column correlation of r (out[i] = sum_t w0[t] r[i - H + t]);
    //      rows past UR land in B's padding
    if (PCS_WAVE_ON(0, M::NI3)) {
      const int e = PCS_ITEM(0, M::NI3);
      const int q = e / GR, g = e - (e / GR) * GR;
      const int i0 = q * RR3;
      const int sl = (a + i0 - H - rb) & 31;
      G4<T> acc[RR3];
      vpass<T, H, RR3, false, 4>(RR, WR, sl, 4 * g, w0, acc);
#pragma unroll
      for (int m = 0; m < RR3; ++m) st4(B + (i0 + m) * WR + 4 * g, acc[m]);
    }
    PCS_ST(7);
    // ---- land z (Z0: z0 rows [a-1, a+TS], pitch WG; Z1: z1 rows [a, a+TS], cols from c0-4,
    //      pitch WG+4) and chunk k+1's x rows (their ring slots held rows P1 of this step read)
#pragma unroll
    for (int kk = 0; kk < KZ0; ++kk) {
      if (!PCS_WAVE_ON(kk, M::NZ0)) continue;
      st4(Z0 + 4 * PCS_ITEM(kk, M::NZ0), zr0[kk]);
    }
#pragma unroll
    for (int kk = 0; kk < KZ1; ++kk) {
      if (!PCS_WAVE_ON(kk, M::NZ1)) continue;
      st4(Z1 + 4 * PCS_ITEM(kk, M::NZ1), zr1[kk]);
    }
    store_xn(xnx, a + TS + 2 * H + 1);
    PCS_ST(8);
    lds_barrier();
    PCS_ST(9);
    store_y(ynx, cs + TS);  // RR slots of chunk k+1 held chunk k-1, last read by P3 above
    // ---- P45: grad F = row correlation of B, primal update on the U rows, x' on own rows
#pragma unroll
    for (int kk = 0; kk < K5; ++kk) {
      if (!PCS_WAVE_ON(kk, M::NI5)) continue;
      const int e = PCS_ITEM(kk, M::NI5);
      const bool real = kk * NT + tid < M::NI5;
      const int i = e / GG, g = e - (e / GG) * GG;
      const int lr = a + i, gr = s.row0 + lr;
      const bool cin = (fl >> (NG2 + kk)) & 1, clast = (fl >> (NG2 + K5 + kk)) & 1;
      G4<T> gd;
      {
        constexpr int NV = 1 + H4 / 2;
        T v[4 * NV];
#pragma unroll
        for (int q = 0; q < NV; ++q) {
          const G4<T> t4 = lds4(B + i * WR + 4 * g + 4 * q);
#pragma unroll
          for (int ee = 0; ee < 4; ++ee) v[4 * q + ee] = t4.v[ee];
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          T acc = T(0);
#pragma unroll
          for (int t = 0; t < NT2; ++t) acc += w1[t] * v[m + SH + t];
          gd.v[m] = acc;
        }
      }
      const G4<T> za = lds4(Z0 + i * WG + 4 * g);             // z0[lr-1]
      const G4<T> zb = lds4(Z0 + (i + 1) * WG + 4 * g);       // z0[lr]
      const G4<T> z1a = lds4(Z1 + i * (WG + 4) + 4 * g);      // z1[c-4 .. c-1]
      const G4<T> z1b = lds4(Z1 + i * (WG + 4) + 4 * g + 4);  // z1[c .. c+3]
      const bool r_last = gr >= n0 - 1, r_first = gr <= 0;
      const bool rin = gr >= 0 && gr < n0 && lr <= s.rows && cin;
      const bool own = (i < TS) && (lr < s1) && gr < n0 && (4 * g < TW) && cin;
      G4<T> uo, xo;
      T sdx = T(0), sx = T(0);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const T xv = xu[kk].v[m];
        // K^T z for forward differences, VStack order: (0 + D0^T z0) + D1^T z1; z1 left of the
        // image loads as 0; z1 on the last column is not used (forward difference there is 0)
        const T zl = (m == 0) ? z1a.v[3] : z1b.v[m - 1];
        T d0 = r_first ? T(0) : za.v[m];
        if (!r_last) d0 -= zb.v[m];
        const T d1 = zl - ((m == 3 && clast) ? T(0) : z1b.v[m]);
        const T a0 = P.unit0 ? d0 : d0 * P.inv_step0;
        const T a1 = P.unit1 ? d1 : d1 * P.inv_step1;
        const T xt = prox_g((xv - P.tau * gd.v[m]) - P.tau * (a0 + a1), gk, P.seg_a, P.seg_b);
        uo.v[m] = rin ? (T(2) * xt - xv) : T(0);
        const T xnew = P.rho * xt + P.omr * xv;
        xo.v[m] = xnew;
        const T dx = xv - xnew;
        sdx += dx * dx;
        sx += xv * xv;
      }
      if (own && real) {  // per-item partials: 4 terms in fp32, accumulated in fp64
        part[0] += (double)sdx;
        part[1] += (double)sx;
      }
      st4(U + i * WG + 4 * g, uo);
      if (own) st4(xn + (lr + s.hx) * n1 + c0 + 4 * g, xo);
    }
    PCS_ST(10);
    lds_barrier();
    PCS_ST(11);
    // ---- P6: dual update on own rows
#pragma unroll
    for (int kk = 0; kk < K6; ++kk) {
      if (!PCS_WAVE_ON(kk, M::NI6)) continue;
      const int e = PCS_ITEM(kk, M::NI6);
      const bool real = kk * NT + tid < M::NI6;
      const int i = e / (TW / 4), g = e - (e / (TW / 4)) * (TW / 4);
      const int lr = a + i, gr = s.row0 + lr;
      const bool cin = (fl >> (NG2 + 2 * K5 + kk)) & 1, clast = (fl >> (NG2 + 2 * K5 + K6 + kk)) & 1;
      const bool own = lr < s1 && gr < n0 && cin;
      const G4<T> uc = lds4(U + i * WG + 4 * g);
      const G4<T> un = lds4(U + i * WG + 4 * g + 4);
      const G4<T> ud = lds4(U + (i + 1) * WG + 4 * g);
      const G4<T> zv0 = lds4(Z0 + (i + 1) * WG + 4 * g);
      const G4<T> zv1 = lds4(Z1 + i * (WG + 4) + 4 * g + 4);
      const bool r_last = gr >= n0 - 1;
      G4<T> o0, o1;
      T sdz = T(0), sz = T(0);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const T uright = (m < 3) ? uc.v[m + 1] : un.v[0];
        const T d0 = r_last ? T(0) : (ud.v[m] - uc.v[m]);
        const T d1 = (m == 3 && clast) ? T(0) : (uright - uc.v[m]);
        const T ku0 = P.unit0 ? d0 : d0 * P.inv_step0;
        const T ku1 = P.unit1 ? d1 : d1 * P.inv_step1;
        const T w0v = zv0.v[m] + P.sigma * ku0, w1v = zv1.v[m] + P.sigma * ku1;
        const T v0 = w0v * P.inv_sigma, v1 = w1v * P.inv_sigma;
        T zt0, zt1;
        if (hk == PCS_H_L21) {  // w - sigma * (max(1 - t/||v||, 0) v), penalty.py:551-557
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
      if (own && real) {
        part[2] += (double)sdz;
        part[3] += (double)sz;
      }
      if (own) {
        T* r0 = zn + (lr + s.hz) * n1 + c0 + 4 * g;
        st4(r0, o0);
        st4(r0 + zstride, o1);
      }
    }
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

// One block per task (64-column strip x row segment, strips strip0 .. strip0 + tiles_x - 1);
// with `hist` the last workgroups also reduce the partials and run the loop control.
template <typename T, int H, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(3))) void k_pds2d_march(
    const T* __restrict__ x, T* __restrict__ xn, const T* __restrict__ z, T* __restrict__ zn,
    const T* __restrict__ y, const T* __restrict__ taps0, const T* __restrict__ taps1, int half, Slab32 s,
    Params<T> P, int hk, int gk, double* __restrict__ partials, Ctrl* ctrl, double* hist, void* ws, int strip0,
    int tiles_x, int seg_len, int ntasks) {
  using M = March<H>;
  __shared__ __attribute__((aligned(16))) T sm[M::SZ];
  __shared__ double red[4 * (NT / 64)];
  __shared__ int flag[2];
  if (ctrl != nullptr && ctrl->stopped != 0) return;  // loop already stopped (solver.py:65-66)

  // XCD-aware bijective remap: blocks b, b+8, ... share an XCD -> adjacent strips of a segment
  int task;
  {
    const int b = blockIdx.x, q = ntasks / 8, r = ntasks % 8, xcd = b % 8, k = b / 8;
    task = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  const int seg = task / tiles_x, strip = task - seg * tiles_x;
  const int s0 = seg * seg_len;
  const int s1 = min(s0 + seg_len, s.rows);
  const int c0 = (strip0 + strip) * M::TW;

  T w0[2 * H + 1], w1[2 * H + 1];
#pragma unroll
  for (int t = 0; t < 2 * H + 1; ++t) {  // centred taps, zero-padded from `half` to the tier H
    const bool ok = (t - H >= -half) && (t - H <= half);
    w0[t] = ok ? taps0[t - H + half] : T(0);
    w1[t] = ok ? taps1[t - H + half] : T(0);
  }
  double part[4] = {0.0, 0.0, 0.0, 0.0};
  march_task<T, H, NT>(x, xn, z, zn, y, w0, w1, s, P, hk, gk, s0, s1, c0, sm, part);
  block_sum<4>(part, red);
  if (hist != nullptr) {  // single launch per iteration: the last workgroups reduce + finalize
    reduce_and_finalize(part, partials, ntasks, ws, ctrl, hist, flag);
  } else if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) partials[(int64_t)blockIdx.x * 4 + k] = part[k];
  }
}

}  // namespace pcs
