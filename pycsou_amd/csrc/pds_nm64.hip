// Fused fp64 PDS iteration through the NORMAL operator of a separable blur (round 5): the fp64 form
// of pds_nmarch.hpp, for every Gradient kind (forward, backward, the reference's default centred).
//   grad F = Conv^T (Conv x - y) = N x - b,  N = N_v (x) N_h (two (4H+1)-tap passes),  b = Conv^T y
// PrimalDualSplitting.update_iterand / update_diagnostics (pycsou/opt/proxalgs.py:343-394) with the
// reference's default fp64 dtype (x0 / z0 np.float, proxalgs.py:327,341; Gradient / Convolve2D
// dtype='float64', linop/diff.py:777, linop/conv.py:167):
//   x_t = prox_G((x - tau (N x - b)) - tau K^T z),  u = 2 x_t - x,  x' = rho x_t + (1 - rho) x
//   z'  = rho H.fenchel_prox(z + sigma K u, sigma) + (1 - rho) z
// ONE launch per iteration, 7 words of HBM traffic per pixel (x, b, z0, z1 in; x', z0', z1' out) --
// the split form (grad F by k_sep2d_nrmm into a buffer, then k_pds2d_smarch<double>) moves 10.
//
// A 512-thread workgroup (one per CU: 141 KB of LDS) owns a strip of TO = 60 columns [c0, c0 + 60) of a
// row segment [s0, s1) and computes 64 columns [c0 - 2, c0 + 62) of t, g, u -- the strip's own columns
// and the one each side that K u / K^T z reach, on whole 16-B chunks (2 doubles): every phase is a
// regular 32-chunk pass, no extra-column code.  It marches down the segment 32 rows per step (a =
// s0 + 32 k):
//   top   issue the z tiles of rows [a, a + 34) (LDS-DMA), b of the step's U rows, the next step's x rows
//   PH    t = N_h x on rows [a + 2H + 1, a + 2H + 33)          x ring (48 rows) -> t ring (+ mirror)
//   PV/U  g = N_v t - b on rows [a + 1, a + 33), in the same thread: x_t, u -> u ring, x' -> HBM
//   Z     z' on rows [a, a + 32); the next step's x rows land in the x ring
// Three barriers per step.  Items: PH one row x 4 columns (512 = 32 rows x 16), PV / U / Z two rows x one
// chunk (512 = 16 row pairs x 32 chunks); lane layouts conflict-free in the LDS lane-group model of
// MI355X_MICROARCH.md (ds_read_b128 16-lane groups, ds_write_b128 8-lane groups; checked offline).
// The PV window (2 + 4H rows) is contiguous through the t ring's mirror rows: immediate offsets.
// The operations and their order per element are those of the split form (k_sep2d_nrmm's passes and
// subtraction, k_pds2d_smarch's update through stencil.hpp), so the iterates are the split form's.
#include "pds_host.hpp"

namespace pcs {

template <int H>
struct NM64 {
  static constexpr int NT = 512, TS = 32, TO = 60, CW = 64, CC = CW / 2;  // own / computed columns, chunks
  static constexpr int NQ = 4 * H + 1;
  static constexpr int XOFF = 16, XW = CW + 2 * XOFF, XCH = XW / 2;  // x region [cb - 16, cb + 80), cb = c0 - 2
  static constexpr int XRING = 48, XP = XW + 2;                      // 49 slots per row (odd)
  static constexpr int TRING = TS + 4 * H, TMIR = 4 * H + 1, TP = CW + 2;  // PV window 2 + 4H rows; 33 slots
  static constexpr int URING = TS + 2, UP = CW + 2;                  // u rows [a - 1, a + 33)
  static constexpr int ZR = TS + 2, ZCH = CC + 2;                    // z tiles: rows [a, a + 34), cols [cb - 2, cb + 66)
  static constexpr int ZSL = ZR * ZCH, ZINS = (ZSL + 63) / 64;       // 16-B slots per component, DMA instructions
  static constexpr int NW = 64 + 32 * H;                             // the N tables (pcs_pds2d_args.ntaps)
  static constexpr int NXL = (TS * XCH + NT - 1) / NT;               // x loads per thread and step
  static constexpr int O_X = 0, O_T = O_X + XRING * XP, O_U = O_T + (TRING + TMIR) * TP, O_Z = O_U + URING * UP,
                       O_W = O_Z + 2 * (ZINS * 64 * 2), SZ = O_W + NW;
  static_assert(XRING >= TS + 2 * H, "x ring holds the U rows and the PH rows of a step");
  static_assert(NT == 16 * CC && NT == TS * 16, "one PH item and one PV / U / Z item per thread");
  static __device__ __forceinline__ int xslot(int r) { return (int)((unsigned)(r + XRING * (1 << 20)) % XRING); }
  static __device__ __forceinline__ int tslot(int r) { return (int)((unsigned)(r + TRING * (1 << 20)) % TRING); }
  static __device__ __forceinline__ int uslot(int r) { return (int)((unsigned)(r + URING * (1 << 20)) % URING); }
};

typedef unsigned int nm64_u4 __attribute__((ext_vector_type(4)));
struct D2 {
  double v[2];
};
__device__ __forceinline__ D2 nm64_lds(const double* p) {  // one ds_read_b128
  typedef __attribute__((address_space(3))) const volatile nm64_u4* lds_u4;
  const nm64_u4 v = *((lds_u4)(p));
  D2 r;
  __builtin_memcpy(r.v, &v, 16);
  return r;
}
__device__ __forceinline__ void nm64_st(double* p, const D2& d) {
  nm64_u4 v;
  __builtin_memcpy(&v, d.v, 16);
  *reinterpret_cast<nm64_u4*>(p) = v;
}
__device__ __forceinline__ D2 nm64_bload(Rsrc r, uint32_t off) {
  const nm64_u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  D2 d;
  __builtin_memcpy(d.v, &v, 16);
  return d;
}
__device__ __forceinline__ void nm64_bstore(Rsrc r, uint32_t off, const D2& d) {
  nm64_u4 v;
  __builtin_memcpy(&v, d.v, 16);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 0);
}
__device__ __forceinline__ void nm64_fence() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int H, int HK, int KK>
__device__ __forceinline__ void nm64_task(const double* __restrict__ x, double* __restrict__ xn,
                                          const double* __restrict__ z, double* __restrict__ zn,
                                          const double* __restrict__ b, const double* __restrict__ tq, const Slab32& s,
                                          const Params<double>& P, int gk, int edge, int s0, int s1, int c0,
                                          double* sm, double (&part)[4], int stop_raw) {
  using T = double;
  using M = NM64<H>;
  constexpr int NT = M::NT, TS = M::TS, NQ = M::NQ, XP = M::XP, TP = M::TP, UP = M::UP, ZCH = M::ZCH;
  constexpr int NXL = M::NXL, XCH = M::XCH, TO = M::TO;
  T* XR = sm + M::O_X;
  T* TR = sm + M::O_T;
  T* UR = sm + M::O_U;
  T* Z0 = sm + M::O_Z;               // z0 tile: slot (row, chunk) at 2 (row ZCH + chunk)
  T* Z1 = Z0 + M::ZINS * 64 * 2;     // z1 tile
  T* W = sm + M::O_W;
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  for (int i = tid; i < M::NW; i += NT) W[i] = tq[i];  // visible after the first barrier
  const int n0 = s.n0, n1 = s.n1, cb = c0 - 2;
  const int zstride = (s.rows + 2 * s.hz) * n1;
  const View vx = make_view(x, s, s.hx, 8u), vb = make_view(b, s, s.hy, 8u), vz0 = make_view(z, s, s.hz, 8u),
             vz1 = make_view(z + zstride, s, s.hz, 8u);
  const uint32_t pitch = (uint32_t)n1 * 8u;
  const Rsrc rxn = rsrc_of(xn, (uint32_t)(s.rows + 2 * s.hx) * pitch);
  const Rsrc rzn0 = rsrc_of(zn, (uint32_t)zstride * 8u), rzn1 = rsrc_of(zn + zstride, (uint32_t)zstride * 8u);
  // the window taps a[|q - 2H|] of both axes, 2H + 1 distinct values each (registers)
  T av[2 * H + 1], ah[2 * H + 1];
  // ---- per-thread items
  // PH: row pr of the step's 32, columns cb + 4 pg .. + 3 (lane layout r2: rows 4 wv + (lane & 1) + 2 (lane >> 5))
  const int pr = 4 * wv + (lane & 1) + 2 * (lane >> 5), pg = (lane >> 1) & 15;
  // PV / U / Z: rows 2 vi, 2 vi + 1 of the step, chunk vg (columns cb + 2 vg, cb + 2 vg + 1)
  const int vi = tid >> 5, vg = tid & 31;
  const int vc = cb + 2 * vg;  // the item's first column
  const bool c_in = (unsigned)vc < (unsigned)n1;                      // chunks wholly in / out (n1 % 4 == 0)
  const bool c_own = vg >= 1 && vg <= TO / 2 && c_in;                 // columns [c0, c0 + 60)
  const uint32_t co_v = col_off(vc, n1, 8u);
  // x loads: item e = l NT + tid -> row e / XCH of the 32, chunk e % XCH (columns cb - 16 + 2 chunk)
  uint32_t co_x[NXL];
  int rr_x[NXL];
#pragma unroll
  for (int l = 0; l < NXL; ++l) {
    const int e = min(l * NT + tid, TS * XCH - 1);
    rr_x[l] = e / XCH;
    co_x[l] = col_off(cb - M::XOFF + 2 * (e - rr_x[l] * XCH), n1, 8u);
  }
  auto load_x = [&](D2 (&xv)[NXL], int r0, int nrows) {  // x rows [r0, r0 + nrows) of the x region
#pragma unroll
    for (int l = 0; l < NXL; ++l)
      xv[l] = nm64_bload(vx.r, (rr_x[l] < nrows ? vx.row_off(r0 + rr_x[l]) : kOOB) + co_x[l]);
  };
  auto store_x = [&](const D2 (&xv)[NXL], int r0, int nrows) {
#pragma unroll
    for (int l = 0; l < NXL; ++l) {
      const int e = l * NT + tid;
      if (e < TS * XCH && rr_x[l] < nrows) {
        const int k = e - rr_x[l] * XCH;
        nm64_st(XR + M::xslot(r0 + rr_x[l]) * XP + 2 * k, xv[l]);
      }
    }
  };
  // z tiles: rows [a, a + 34), chunks [cb - 2, cb + 66) of both components, straight into LDS (buffer_load ...
  // lds, lane-linear: lane l of instruction j fills slot 64 j + l); tile rows below `rmin` read as 0
  auto load_z = [&](int a, int rmin) {
    for (int j = wv; j < 2 * M::ZINS; j += NT / 64) {
      const int comp = j >= M::ZINS, jj = comp ? j - M::ZINS : j;
      const int e = 64 * jj + lane, tr = e / ZCH, k = e - tr * ZCH;
      const View& vz = comp ? vz1 : vz0;
      const uint32_t o = (tr >= M::ZR || tr < rmin ? kOOB : vz.row_off(a + tr)) + col_off(cb - 2 + 2 * k, n1, 8u);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(vz.r, (__attribute__((address_space(3))) void*)((comp ? Z1 : Z0) + 128 * jj),
                                               16, o, 0, 0, 0);
    }
  };
  auto zt = [&](const T* Zt, int tr, int k) { return nm64_lds(Zt + 2 * (tr * ZCH + k)); };

  // ---- PH: t row lr = N_h x row lr on columns cb + 4 pg .. + 3 -> t ring (+ the mirror copy)
  auto ph = [&](int lr) {
    const T* xrow = XR + M::xslot(lr) * XP;
    T v[4 + 4 * H];  // x-region columns 16 + 4 pg - 2H .. 16 + 4 pg + 3 + 2H
#pragma unroll
    for (int u = 0; u < 2 + 2 * H; ++u) {
      const D2 d = nm64_lds(xrow + 2 * (8 - H + 2 * pg + u));
      v[2 * u] = d.v[0];
      v[2 * u + 1] = d.v[1];
    }
    T acc[4] = {T(0), T(0), T(0), T(0)};
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[m] += ah[q < 2 * H ? 2 * H - q : q - 2 * H] * v[m + q];
    const int col = cb + 4 * pg;
    if (col < H || col + 3 >= n1 - H) {  // the exact rows of N_h on the H columns nearest an image edge
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int j = col + m;
        if (j >= 0 && j < H) {
          for (int k = 0; k < H; ++k) acc[m] -= W[64 + 16 * H + 8 * k + j] * xrow[M::XOFF - cb + k];
        } else if (j >= n1 - H && j < n1) {
          for (int k = 0; k < H; ++k)
            acc[m] -= W[64 + 24 * H + 8 * k + (j - (n1 - 8))] * xrow[M::XOFF - cb + n1 - H + k];
        }
      }
    }
    const int sl = M::tslot(lr);
    T* trow = TR + sl * TP + 4 * pg;
    nm64_st(trow, D2{{acc[0], acc[1]}});
    nm64_st(trow + 2, D2{{acc[2], acc[3]}});
    if (sl < M::TMIR) {
      nm64_st(trow + M::TRING * TP, D2{{acc[0], acc[1]}});
      nm64_st(trow + M::TRING * TP + 2, D2{{acc[2], acc[3]}});
    }
  };

  // ---- PV + U: rows lr0 = a + 1 + 2 vi, lr0 + 1, chunk vg; bv: b of those rows; za: the z tiles' first row
  // I (std::true_type): every row and column the phase touches lies >= 2 samples inside the image -- the
  // stencils without their edge rules (stencil.hpp: the same bits)
  // (intr: the row axis; intc: the column axis)
  auto pvu = [&](auto intr, auto intc, int a, const D2 (&bv)[2], int za) {
    constexpr bool I0 = decltype(intr)::value, I1 = decltype(intc)::value;
    const int lr0 = a + 1 + 2 * vi;
    // g = N_v t - b: t rows lr0 - 2H .. lr0 + 1 + 2H, contiguous through the mirror (immediate offsets)
    const T* p0 = TR + M::tslot(lr0 - 2 * H) * TP + 2 * vg;
    D2 acc[2] = {{{T(0), T(0)}}, {{T(0), T(0)}}};
    constexpr int NV = NQ + 1, CH = 4, NCH = (NV + CH - 1) / CH;
    D2 w[2][CH];
    auto rd = [&](int c, D2 (&wc)[CH]) {
#pragma unroll
      for (int j = 0; j < CH; ++j)
        if (c * CH + j < NV) wc[j] = nm64_lds(p0 + (c * CH + j) * TP);
    };
    rd(0, w[0]);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (c + 1 < NCH) rd(c + 1, w[(c + 1) & 1]);
      nm64_fence();
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int q0 = c * CH + j;
        if (q0 < NV) {
#pragma unroll
          for (int r = 0; r < 2; ++r) {
            const int q = q0 - r;
            if (q >= 0 && q < NQ) {
              const T h = av[q < 2 * H ? 2 * H - q : q - 2 * H];
              acc[r].v[0] += h * w[c & 1][j].v[0];
              acc[r].v[1] += h * w[c & 1][j].v[1];
            }
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 2; ++r) asm volatile("" : "+v"(acc[r].v[0]), "+v"(acc[r].v[1]));
      nm64_fence();
    }
    T gv[2][2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int gr = s.row0 + lr0 + r;
      if (gr < H || (gr >= n0 - H && gr < n0)) {  // the exact rows of N_v on the H rows nearest an image edge
        const bool top = gr < H;
        const int kr0 = (top ? 0 : n0 - H) - s.row0;  // local row of the band's first image row
        const T* d = W + 64 + (top ? 8 * gr : 8 * H + 8 * (gr - (n0 - H)));
        for (int k = 0; k < H; ++k) {
          const D2 t2 = nm64_lds(TR + M::tslot(kr0 + k) * TP + 2 * vg);
          acc[r].v[0] -= d[k] * t2.v[0];
          acc[r].v[1] -= d[k] * t2.v[1];
        }
      }
      gv[r][0] = acc[r].v[0] - bv[r].v[0];
      gv[r][1] = acc[r].v[1] - bv[r].v[1];
    }
    // ---- U: K^T z from the z tiles: z0 rows lr0 - 1 .. lr0 + 2 (chunk vg + 1), z1 rows lr0, lr0 + 1 at
    // columns vc - 2 .. vc + 3 (chunks vg .. vg + 2)
    const int t0 = lr0 - za;  // tile row of lr0
    D2 z0w[4], z1w[2][3];
#pragma unroll
    for (int k = 0; k < 4; ++k) z0w[k] = zt(Z0, t0 - 1 + k, vg + 1);
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int k = 0; k < 3; ++k) z1w[r][k] = zt(Z1, t0 + r, vg + k);
    T sdx = T(0), sx = T(0);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int lr = lr0 + r, gr = s.row0 + lr;
      const D2 xv2 = nm64_lds(XR + M::xslot(lr) * XP + 2 * (8 + vg));
      const bool rin = (unsigned)gr < (unsigned)n0 && lr <= s.rows;
      const bool own = lr >= s0 && lr < s1 && gr < n0 && c_own;
      D2 uo, xo;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int c = vc + m;
        const T w0[5] = {T(0), z0w[r].v[m], z0w[r + 1].v[m], z0w[r + 2].v[m], T(0)};  // rows lr - 1 .. lr + 1
        const T z1c[6] = {z1w[r][0].v[0], z1w[r][0].v[1], z1w[r][1].v[0], z1w[r][1].v[1], z1w[r][2].v[0], z1w[r][2].v[1]};
        const T w1[5] = {T(0), z1c[1 + m], z1c[2 + m], z1c[3 + m], T(0)};  // columns c - 1 .. c + 1
        const T kt = pcs_fma(sw_d1_adj<KK, I0>(w0, gr, n0, edge), P.inv_step0,
                             sw_d1_adj<KK, I1>(w1, c, n1, edge) * P.inv_step1);
        const T xvm = xv2.v[m];
        const T xt = prox_g((xvm - P.tau * gv[r][m]) - P.tau * kt, gk, P.seg_a, P.seg_b);
        uo.v[m] = (rin && c_in) ? (T(2) * xt - xvm) : T(0);
        const T xnew = pcs_fma(P.rho, xt, P.omr * xvm);
        xo.v[m] = xnew;
        const T dx = xvm - xnew;
        sdx += dx * dx;
        sx += xvm * xvm;
      }
      nm64_st(UR + M::uslot(lr) * UP + 2 * vg, uo);
      nm64_bstore(rxn, (own ? (uint32_t)(lr + s.hx) * pitch : kOOB) + co_v, xo);
      if (!own) sdx = sx = T(0);
      part[0] += (double)sdx;
      part[1] += (double)sx;
      sdx = sx = T(0);
    }
  };

  // ---- Z: z' on rows lz0 = a + 2 vi, lz0 + 1, chunk vg; K u from u rows lz0 - 1 .. lz0 + 2 and columns
  // vc - 2 .. vc + 3 of rows lz0, lz0 + 1
  auto zph = [&](auto intr, auto intc, int a) {
    constexpr bool I0 = decltype(intr)::value, I1 = decltype(intc)::value;
    const int lz0 = a + 2 * vi;
    D2 uw[4], uh[2][3];
#pragma unroll
    for (int k = 0; k < 4; ++k) uw[k] = nm64_lds(UR + M::uslot(lz0 - 1 + k) * UP + 2 * vg);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const T* urow = UR + M::uslot(lz0 + r) * UP + 2 * vg;
      uh[r][0] = nm64_lds(urow - 2);
      uh[r][1] = uw[1 + r];
      uh[r][2] = nm64_lds(urow + 2);
    }
    T sdz = T(0), sz = T(0);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int lr = lz0 + r, gr = s.row0 + lr;
      const D2 zv0 = zt(Z0, lr - a, vg + 1), zv1 = zt(Z1, lr - a, vg + 1);
      const bool own = lr >= s0 && lr < s1 && gr < n0 && c_own;
      D2 o0, o1;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int c = vc + m;
        const T w0[5] = {T(0), uw[r].v[m], uw[r + 1].v[m], uw[r + 2].v[m], T(0)};  // rows lr - 1 .. lr + 1
        const T uc[6] = {uh[r][0].v[0], uh[r][0].v[1], uh[r][1].v[0], uh[r][1].v[1], uh[r][2].v[0], uh[r][2].v[1]};
        const T w1[5] = {T(0), uc[1 + m], uc[2 + m], uc[3 + m], T(0)};  // columns c - 1 .. c + 1
        const T ku0 = sw_d1_fwd<KK, I0>(w0, gr, n0, P.inv_step0, edge);
        const T ku1 = sw_d1_fwd<KK, I1>(w1, c, n1, P.inv_step1, edge);
        const T wz0 = zv0.v[m] + P.sigma * ku0, wz1 = zv1.v[m] + P.sigma * ku1;
        const T q0 = wz0 * P.inv_sigma, q1 = wz1 * P.inv_sigma;
        T zt0, zt1;
        if constexpr (HK == PCS_H_L21) {  // w - sigma * (max(1 - t/||v||, 0) v), penalty.py:551-557
          T f = T(1) - P.t_h * fast_rsqrt(pcs_fma(q0, q0, q1 * q1));
          f = f > T(0) ? f : T(0);
          zt0 = wz0 - P.sigma * (f * q0);
          zt1 = wz1 - P.sigma * (f * q1);
        } else {  // w - sigma * (v - t*clip(v/t)), func/base.py:239-240
          zt0 = wz0 - P.sigma * (q0 - P.t_h * clip1(q0 * P.inv_t_h));
          zt1 = wz1 - P.sigma * (q1 - P.t_h * clip1(q1 * P.inv_t_h));
        }
        o0.v[m] = pcs_fma(P.rho, zt0, P.omr * zv0.v[m]);
        o1.v[m] = pcs_fma(P.rho, zt1, P.omr * zv1.v[m]);
        const T e0 = zv0.v[m] - o0.v[m], e1 = zv1.v[m] - o1.v[m];
        sdz += e0 * e0;
        sz += zv0.v[m] * zv0.v[m];
        sdz += e1 * e1;
        sz += zv1.v[m] * zv1.v[m];
      }
      const uint32_t off = (own ? (uint32_t)(lr + s.hz) * pitch : kOOB) + co_v;
      nm64_bstore(rzn0, off, o0);
      nm64_bstore(rzn1, off, o1);
      if (!own) sdz = sz = T(0);
      part[2] += (double)sdz;
      part[3] += (double)sz;
      sdz = sz = T(0);
    }
  };
  auto load_b = [&](D2 (&bv)[2], int lr0, bool on) {
#pragma unroll
    for (int r = 0; r < 2; ++r) bv[r] = nm64_bload(vb.r, (on ? vb.row_off(lr0 + r) : kOOB) + co_v);
  };

  // ================= prologue: t rows [s0 - 1 - 2H, s0 + 2H + 1), u on rows s0 - 1, s0, x' on row s0 (the
  // PV / U of a pseudo-step at a = s0 - 32 whose row pair vi = 15 holds rows s0 - 1, s0)
  D2 xnx[NXL], bv[2];
  {
    constexpr int NPRO = 4 * H + 2;
    D2 xv[NXL];
    load_x(xv, s0 - 1 - 2 * H, NPRO);
    load_z(s0 - TS, M::ZR - 4);  // tile rows s0 - 2 .. s0 + 1
    load_b(bv, s0 - 1, vi == 15);
    load_x(xnx, s0 + 2 * H + 1, TS);  // step 0's PH rows, landed after the prologue's U
    __builtin_amdgcn_s_waitcnt((NXL & 15) | ((NXL >> 4) << 14) | (7 << 4) | (15 << 8));
    store_x(xv, s0 - 1 - 2 * H, NPRO);
    if (stop_raw) {  // loop already stopped (solver.py:65-66): every load drained, nothing stored
      __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));
      return;
    }
    lds_barrier();
#pragma unroll
    for (int e = 0; e < 2 * H + 1; ++e) {  // the taps from LDS: VGPRs (uniform global loads would take SGPRs)
      av[e] = W[2 * H + e];
      ah[e] = W[32 + 2 * H + e];
    }
    if (pr < NPRO) ph(s0 - 1 - 2 * H + pr);
    lds_barrier();
    if (vi == 15) pvu(std::false_type{}, std::false_type{}, s0 - TS, bv, s0 - TS);
    __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));  // step 0's x rows (and row pair 15's x' stores)
    lds_barrier();  // the prologue's U is done with the x ring rows the landing overwrites
    store_x(xnx, s0 + 2 * H + 1, TS);
  }
  // ================= march
  const int nsteps = (s1 - s0 + TS - 1) / TS;
#ifndef PCS_NM64_ALLINT  // diagnostics (timing only, wrong border values): every strip and step on the interior form
#define PCS_NM64_ALLINT 0
#endif
  const bool cint = PCS_NM64_ALLINT || (cb >= 2 && cb + M::CW + 2 <= n1);  // the strip's columns [cb, cb + 64) >= 2 inside
  // one step; RI: its U rows [a + 1, a + 33) and Z rows [a, a + 32) >= 2 inside the image
  auto step = [&](int a, auto ri, auto ci) {
    lds_barrier();  // step k - 1 done with the z tiles and the u ring; this step's x rows have landed
    __builtin_amdgcn_s_setprio(3);  // the step's loads issue ahead of other waves' VALU
    load_z(a, 0);
    load_b(bv, a + 1 + 2 * vi, true);
    load_x(xnx, a + TS + 2 * H + 1, TS);
    __builtin_amdgcn_s_setprio(0);
    // the wait below counts the NXL x loads as issued after the z tiles and b: pin the issue order (the
    // x rows are only consumed by store_x, so the scheduler could otherwise sink them past the wait --
    // the hazard of the round-5 GEN race)
    nm64_fence();
    ph(a + 2 * H + 1 + pr);
    __builtin_amdgcn_s_waitcnt((NXL & 15) | ((NXL >> 4) << 14) | (7 << 4) | (15 << 8));  // z tiles and b landed
    lds_barrier();
    pvu(ri, ci, a, bv, a);
    lds_barrier();
    zph(ri, ci, a);
    // the next step's x rows (in flight behind: 2 x' and 4 z' stores) into the slots of rows [a + 2H - 15,
    // a + 2H + 17), which this step's PH and U were the last to read
    __builtin_amdgcn_s_waitcnt((6 & 15) | (7 << 4) | (15 << 8));
    store_x(xnx, a + TS + 2 * H + 1, TS);
  };
  auto rows_in = [&](int a) { return PCS_NM64_ALLINT || (s.row0 + a >= 2 && s.row0 + a + TS + 3 <= n0); };
#ifndef PCS_NM64_PEEL  // diagnostics: 0 = one loop choosing the form per step
#define PCS_NM64_PEEL 1
#endif
// the border strips' interior-row steps on a form with the row axis interior (0: the all-axes edge form)
#ifndef PCS_NM64_ROWFORM
#define PCS_NM64_ROWFORM 1
#endif
  using Tt = std::true_type;
  using Ff = std::false_type;
  const bool peel = PCS_NM64_PEEL && rows_in(s0) && rows_in(s0 + (nsteps - 1) * TS);
  if (cint) {
    if (peel) {
      // every step of the task interior (uniform): a loop holding the interior form only -- with both
      // forms in the loop body the interior steps ran slower (profiles/r5_nm64_split_ab.txt)
      for (int k = 0; k < nsteps; ++k) step(s0 + k * TS, Tt{}, Tt{});
    } else {
      for (int k = 0; k < nsteps; ++k) {
        const int a = s0 + k * TS;
        if (rows_in(a)) step(a, Tt{}, Tt{});
        else step(a, Ff{}, Ff{});
      }
    }
  } else if (PCS_NM64_ROWFORM && peel) {  // a border strip whose rows are all interior: the column rules only
    for (int k = 0; k < nsteps; ++k) step(s0 + k * TS, Tt{}, Ff{});
  } else {
    for (int k = 0; k < nsteps; ++k) step(s0 + k * TS, Ff{}, Ff{});
  }
}

// One block per task (a 60-column strip x a row segment); with `hist` the last workgroups also reduce the
// partials and run the loop control, with `ro.sums` they only reduce (slab mode)
template <int H, int HK, int KK>
__global__ __launch_bounds__(512, 1) void k_pds2d_nmarch64(const double* __restrict__ x, double* __restrict__ xn,
                                                           const double* __restrict__ z, double* __restrict__ zn,
                                                           const double* __restrict__ b, const double* __restrict__ tq,
                                                           Slab32 s, Params<double> P, int gk, int edge,
                                                           double* __restrict__ partials, Ctrl* ctrl, double* hist,
                                                           void* ws, RedOut ro, int tiles_x, Bands bd, int ntasks) {
  using M = NM64<H>;
  extern __shared__ __attribute__((aligned(16))) unsigned char nm64_smem[];
  double* sm = reinterpret_cast<double*>(nm64_smem);
  __shared__ double red[4 * (M::NT / 64)];
  __shared__ int flag[2];
  if (fin_slot(ro, ntasks, ctrl, hist, red, flag)) return;  // deferred finalization (pds_ctrl.hpp)
  const int stop_raw = stop_flag_early(ctrl, ro);  // consumed in the task (PCS_DEFER_STOP)
  const bool stopped = !stop_deferred(ro) && stop_requested(ctrl, ro, flag);
  if (stopped && ro.sums == nullptr) return;  // loop already stopped (solver.py:65-66)
  int task;  // XCD-aware bijective remap: blocks b, b+8, ... share an XCD -> adjacent strips
  {
    const int bb = (int)blockIdx.x - fin_shift(ro), q = ntasks / 8, r = ntasks % 8, xcd = bb % 8, k = bb / 8;
    task = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  const int seg = task / tiles_x, strip = task - seg * tiles_x;
  int s0, s1;
  band_rows(bd, seg, s0, s1);
  double part[4] = {0.0, 0.0, 0.0, 0.0};
  if (!stopped) nm64_task<H, HK, KK>(x, xn, z, zn, b, tq, s, P, gk, edge, s0, s1, strip * M::TO, sm, part, stop_raw);
  if (stop_raw) return;  // the task returned before any store
  block_sum<4>(part, red);
  publish_partials(part, partials, ntasks, ws, ctrl, hist, flag, ro);
}

// ---------------------------------------------------------------- host side
template <int H, int HK, int KK>
static void nm64_attr() {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pds2d_nmarch64<H, HK, KK>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)(NM64<H>::SZ * sizeof(double)));
    (void)hipGetLastError();
    done = true;
  }
}

// resident workgroups of the kernel on the device (one per CU at 141 KB of LDS; queried once)
int nm64_slots() {
  static int slots = 0;
  if (slots == 0) {
    int dev = 0, cus = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || cus < 1)
      cus = 256;
    nm64_attr<7, PCS_H_L21, PCS_CENTERED>();
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_pds2d_nmarch64<7, PCS_H_L21, PCS_CENTERED>, 512,
                                                     NM64<7>::SZ * sizeof(double)) != hipSuccess ||
        nb < 1)
      nb = 1;
    (void)hipGetLastError();
    slots = cus * nb;
    const char* e = getenv("PCS_NM64_SLOTS");  // diagnostics: grid-size sweep
    if (e && atoi(e) > 0) slots = atoi(e);
  }
  return slots;
}

// tasks = 60-column strips x row segments of whole 32-row steps; the segment count minimises the rounds of
// resident workgroups times the steps per task (+1 for the segment prologue)
bool nm64_plan(const pcs_pds2d_args* a, RowBands rb, MarchPlan* p) {
  const int tiles_x = (int)((a->n1 + 59) / 60);
  if (tiles_x < 2) return false;
  if (rb.rb0 == rb.ra0) rb = RowBands{rb.ra1, rb.rb1, rb.rb1, rb.rb1};
  const int64_t L0 = rb.rb0 - rb.ra0, L1 = rb.rb1 - rb.ra1;
  const int64_t steps = (L0 + 31) / 32 + (L1 + 31) / 32;
  const int64_t bands = (L0 > 0) + (L1 > 0);
  const int64_t slots = nm64_slots();
  int64_t best = -1, seg_len = 32;
  for (int64_t nseg = bands; nseg <= steps && nseg <= 64; ++nseg) {
    const int64_t len = ((steps + nseg - 1) / nseg) * 32;
    const int64_t n = (L0 + len - 1) / len + (L1 + len - 1) / len;
    const int64_t rounds = (n * tiles_x + slots - 1) / slots;
    const int64_t cost = rounds * (len / 32 + 1);
    if (best < 0 || cost < best) {
      best = cost;
      seg_len = len;
    }
  }
  const int64_t n0s = (L0 + seg_len - 1) / seg_len, n1s = (L1 + seg_len - 1) / seg_len;
  p->tiles_x = tiles_x;
  p->bd = Bands{(int)seg_len, (int)n0s, (int)rb.ra0, (int)rb.rb0, (int)rb.ra1, (int)rb.rb1};
  p->ntasks = (int)(tiles_x * (n0s + n1s));
  return true;
}

template <int H, int HK, int KK>
static int nm64_go(const pcs_pds2d_args* a, const MarchPlan& p, hipStream_t st) {
  const Slab s64 = make_slab(a);
  const Slab32 s{(int)s64.n0, (int)s64.n1, (int)s64.row0, (int)s64.rows, s64.hx, s64.hy, s64.hz, s64.vec};
  const Params<double> P = make_params<double>(a);
  nm64_attr<H, HK, KK>();
  k_pds2d_nmarch64<H, HK, KK><<<(unsigned)p.ntasks + fin_extra(a), 512, NM64<H>::SZ * sizeof(double), st>>>(
      (const double*)a->x, (double*)a->xn, (const double*)a->z, (double*)a->zn, (const double*)a->cty,
      (const double*)a->ntaps, s, P, a->gkind, a->edge, a->partials, (Ctrl*)a->ctrl, a->hist, a->ws, red_out(a),
      p.tiles_x, p.bd, p.ntasks);
  return launch_status();
}

template <int H, int HK>
static int nm64_k(const pcs_pds2d_args* a, const MarchPlan& p, hipStream_t st) {
  switch (a->kkind) {
    case PCS_K_GRAD_FORWARD: return nm64_go<H, HK, PCS_FORWARD>(a, p, st);
    case PCS_K_GRAD_BACKWARD: return nm64_go<H, HK, PCS_BACKWARD>(a, p, st);
    case PCS_K_GRAD_CENTERED: return nm64_go<H, HK, PCS_CENTERED>(a, p, st);
    default: return PCS_EUNSUPPORTED;
  }
}

int launch_nmarch64(const pcs_pds2d_args* a, RowBands rb, hipStream_t st) {
  MarchPlan p;
  if (!nm64_plan(a, rb, &p)) return PCS_EINVAL;
  if (p.ntasks == 0) return PCS_OK;
  const bool l21 = a->hkind == PCS_H_L21;
  if (tier_for(a->half) == 3) return l21 ? nm64_k<3, PCS_H_L21>(a, p, st) : nm64_k<3, PCS_H_L1>(a, p, st);
  return l21 ? nm64_k<7, PCS_H_L21>(a, p, st) : nm64_k<7, PCS_H_L1>(a, p, st);
}

}  // namespace pcs
