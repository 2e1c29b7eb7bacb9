// Fused PrimalDualSplitting update for 3-D volumes (K = Gradient(kind='forward') in 3-D; the
// backward / centred kinds in k_pds3d_gen below).
//
//   x_t = prox_G((x - tau g) - tau K^T z)        g = grad F (precomputed buffer, x - y, or 0)
//   u   = 2 x_t - x
//   z_t = H.fenchel_prox(z + sigma K u, sigma)   H = lam*L1 or lam*L21 over the 3 gradient components
//   z'  = rho z_t + (1-rho) z ;  x' = rho x_t + (1-rho) x
// plus the four norm partials of update_diagnostics -- pycsou/opt/proxalgs.py:343-394 with
// K from pycsou/linop/diff.py:777-882 (PyLops Gradient: VStack of forward FirstDerivatives,
// last sample 0; adjoint accumulated in axis order).
//
// Layout: C-order volume (n0 planes of n1 x n2); z = [D0 x; D1 x; D2 x], each component with
// the same (halo'd) plane layout.  A workgroup owns an 8 x 128 in-plane tile and marches down a
// segment of planes: at plane p it lands z(p) in LDS, computes x_t / u on the tile plus one
// row / one 4-group of halo (u of plane p in a 2-plane LDS ring), writes x'(p), and then
// z'(p-1), whose axis-0 difference needs u(p).  Loads for plane p+1 are issued before plane
// p's work.  Every load goes through a buffer descriptor of ONE plane (num_records = 0 for a
// plane outside the image or the stored slab, so those read 0) with in-plane rows / columns
// outside the image pushed past the range: no branches, no selects.
#include <type_traits>

#include "pds_march.hpp"
#include "stencil.hpp"

#ifndef PCS_3D_PRIO  // wave priority 3 while the next plane's loads issue; diagnostics
#define PCS_3D_PRIO 0
#endif


namespace pcs {

template <typename T>
struct P3 {
  T tau, sigma, inv_sigma, rho, omr, t_h, inv_t_h, inv_step[3], seg_a, seg_b;
  int unit[3];
};

struct Vol {
  int n0, n1, n2, plane0, planes, hx, hz, hg;
  uint32_t pitch1, plane_bytes;  // bytes per row (n2 * elem), per plane
};

template <typename T>
__device__ __forceinline__ G4<T> bload(Rsrc r, uint32_t off);
template <>
__device__ __forceinline__ G4<float> bload<float>(Rsrc r, uint32_t off) {
  return bload4(r, off);
}
template <>
__device__ __forceinline__ G4<double> bload<double>(Rsrc r, uint32_t off) {
  const auto a = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  const auto b = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(off + 16), 0, 0);
  G4<double> g;
  g.v[0] = __hiloint2double((int)a[1], (int)a[0]);
  g.v[1] = __hiloint2double((int)a[3], (int)a[2]);
  g.v[2] = __hiloint2double((int)b[1], (int)b[0]);
  g.v[3] = __hiloint2double((int)b[3], (int)b[2]);
  return g;
}

// descriptor of local plane p of an array stored with `halo` planes on each side (0 records
// when the plane is outside the image or the stored planes)
template <typename T>
__device__ __forceinline__ Rsrc plane_rsrc(const T* base, const Vol& v, int halo, int p) {
  const int gp = v.plane0 + p;
  const bool ok = gp >= 0 && gp < v.n0 && p >= -halo && p < v.planes + halo;
  const T* pl = base + (int64_t)(ok ? p + halo : 0) * v.n1 * v.n2;
  return rsrc_of(pl, ok ? v.plane_bytes : 0u);
}
// in-plane byte offset of (row i1, column i2) -- kOOB parts outside the image
template <typename T>
__device__ __forceinline__ uint32_t inplane(const Vol& v, int i1, int i2) {
  const uint32_t ro = ((unsigned)i1 < (unsigned)v.n1) ? (uint32_t)i1 * v.pitch1 : kOOB;
  const uint32_t co = ((unsigned)i2 < (unsigned)v.n2) ? (uint32_t)i2 * (uint32_t)sizeof(T) : kOOB;
  return ro + co;
}

// one element (odd widths: n2 % 4 != 0)
template <typename T>
__device__ __forceinline__ T bload1(Rsrc r, uint32_t off);
template <>
__device__ __forceinline__ float bload1<float>(Rsrc r, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
template <>
__device__ __forceinline__ double bload1<double>(Rsrc r, uint32_t off) {
  const auto a = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0);
  return __hiloint2double((int)a[1], (int)a[0]);
}

// In-plane offsets of a 4-column group: one 16-B access when n2 % 4 == 0 (VEC: groups are
// wholly inside or outside the image), four element accesses otherwise.
template <typename T, bool VEC>
struct GOff {
  uint32_t o[VEC ? 1 : 4];
};
template <typename T, bool VEC>
__device__ __forceinline__ GOff<T, VEC> goff(const Vol& v, int i1, int c) {
  GOff<T, VEC> g;
#pragma unroll
  for (int m = 0; m < (VEC ? 1 : 4); ++m) g.o[m] = inplane<T>(v, i1, c + m);
  return g;
}
template <typename T, bool VEC>
__device__ __forceinline__ G4<T> gload(Rsrc r, const GOff<T, VEC>& g) {
  if constexpr (VEC) {
    return bload<T>(r, g.o[0]);
  } else {
    G4<T> out;
#pragma unroll
    for (int m = 0; m < 4; ++m) out.v[m] = bload1<T>(r, g.o[m]);
    return out;
  }
}
// store the in-image elements of a group (row i1 inside the image)
template <typename T, bool VEC>
__device__ __forceinline__ void gstore(T* p, const G4<T>& g, int c, int n2) {
  if constexpr (VEC) {
    st4(p, g);
  } else {
#pragma unroll
    for (int m = 0; m < 4; ++m)
      if (c + m < n2) p[m] = g.v[m];
  }
}

// LDS tiles of 4-groups with a row pitch of W elements.  fp32: plain rows (group g of row r at r W + 4 g).
// fp64: every row is stored as two half-rows of W / 2 doubles -- half h of group g (its elements 2 h, 2 h + 1)
// at (2 r + h) W / 2 + 2 g -- so the two 16-B reads / writes of a group by consecutive lanes on consecutive
// groups are each contiguous (ds_read_b128 / ds_write_b128 without bank conflicts).  The plain layout's 32-B
// lane stride cost 0.85 G (forward K) / 1.18 G (centred K) bank-conflict cycles per C5 update launch
// (profiles/r6_prof_c5*).
template <int W>
__device__ __forceinline__ G4<float> tl_ld(const float* a, int r, int g) {
  return lds4(a + r * W + 4 * g);
}
template <int W>
__device__ __forceinline__ void tl_st(float* a, int r, int g, const G4<float>& v) {
  st4(a + r * W + 4 * g, v);
}
template <int W>
__device__ __forceinline__ G4<double> tl_ld(const double* a, int r, int g) {
  static_assert(W % 4 == 0, "16-B aligned half-rows");
  typedef double d2 __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) const volatile d2* lds_d2;
  const double* p = a + 2 * r * (W / 2) + 2 * g;
  const d2 lo = *(lds_d2)(p), hi = *(lds_d2)(p + W / 2);
  return {{lo.x, lo.y, hi.x, hi.y}};
}
template <int W>
__device__ __forceinline__ void tl_st(double* a, int r, int g, const G4<double>& v) {
  double* p = a + 2 * r * (W / 2) + 2 * g;
  *reinterpret_cast<double2*>(p) = make_double2(v.v[0], v.v[1]);
  *reinterpret_cast<double2*>(p + W / 2) = make_double2(v.v[2], v.v[3]);
}

#ifndef PCS_K3TW
#define PCS_K3TW 128
#endif
// 8 x 128 tiles: a 64-column tile's one-group right halo costs a third 128-B line per row
// (PMC: 1.53x the algorithmic reads); at 128 columns it is one line in five
constexpr int k3T1 = 8;
// fp64 forward-K tile rows (diagnostics builds override): 12 (113.5 KB of LDS, one 512-thread workgroup per
// CU as at 8) -- C5 update 13.83 against 14.22 ms at 8 (profiles/r6_f3rows_ab.txt)
#ifndef PCS_3D_ROWS64
#define PCS_3D_ROWS64 12
#endif
template <typename T>
constexpr int k3_rows() { return sizeof(T) == 8 ? PCS_3D_ROWS64 : k3T1; }
// fp64 forward-K tile width (diagnostics builds override): 64 columns = 256-thread workgroups, three of
// them per CU at the fp64 kernel's 157-169 VGPRs instead of one 512-thread one -- measured slower (C5
// update 17.0 against 14.9 ms, profiles/r4_c5_tile64_ab.txt): 128 stays
#ifndef PCS_K3TW64
#define PCS_K3TW64 PCS_K3TW
#endif
template <typename T>
struct K3 {
  static constexpr int TW = sizeof(T) == 8 ? PCS_K3TW64 : PCS_K3TW;
  static constexpr int NT = TW == 64 ? 256 : TW == 128 ? 512 : 1024;
};

// fkind PCS_F_CONV0: grad F = C0^T (C0 t - w) along axis 0 inside the update, t (the `g` array) the
// in-plane normal operator C12^T C12 x and w = C12^T y: per U item two 15-plane register rings
// (t, and the residual r = C0 t - w), the arithmetic of k_conv0_rta (conv.hip) sample for sample
constexpr int k3C0K = 15;
// PCS_F_CONV0 ring item width: 3 voxels per ring thread on waves 8-15, or 2 voxels on waves 6-15 (the
// update loop's waves 6-7 have no items: U / z1 / z2 / z' items end in wave 5).  Measured C4 512^3:
// 614-619 it/s at 3 against 562-570 at 2 (alternating, profiles/r3_ck39_ring_ab.txt)
#ifndef PCS_3D_RV
#define PCS_3D_RV 3
#endif
// planes of t / C12^T y in flight while the ring prologue fills the rings (loads issued that many
// pushes ahead; 4 measured the same as 1, r3_ck39)
#ifndef PCS_3D_RPD
#define PCS_3D_RPD 1
#endif
// (a packed-pair form of the rings -- v_pk_fma_f32 on voxels 0 and 1 -- measured 529 against 611 it/s on
// C4, profiles/r4_c4_packed_ring_ab.txt: removed in round 5)

template <typename T, int FK, bool VEC>
// minimum resident workgroups per CU the register budget targets (non-fold kernels; diagnostics knob):
// at 1 the fp64 kernel takes 157-169 VGPRs, 3 waves / SIMD = one 512-thread workgroup per CU
#ifndef PCS_3D_MINB
#define PCS_3D_MINB 1
#endif
__global__ __launch_bounds__(FK == PCS_F_CONV0 ? 2 * K3<T>::NT : K3<T>::NT, FK == PCS_F_CONV0 ? 1 : PCS_3D_MINB) void k_pds3d(const T* __restrict__ x, T* __restrict__ xn,
                                                 const T* __restrict__ z, T* __restrict__ zn,
                                                 const T* __restrict__ g, Vol v, P3<T> P, int hk, int gk,
                                                 double* __restrict__ partials, Ctrl* ctrl, double* hist, void* ws,
                                                 int tiles1, int tiles2, Bands bd, int ntasks,
                                                 const T* __restrict__ w0, const T* __restrict__ taps0, int k0,
                                                 int off0) {
  // PCS_F_CONV0: a second set of k3NT threads (waves 8-15) runs the axis-0 rings beside the update
  constexpr bool FOLD = FK == PCS_F_CONV0;
  constexpr int T1 = k3_rows<T>(), TW = K3<T>::TW, NT = FOLD ? 2 * K3<T>::NT : K3<T>::NT;
  constexpr int UR = T1 + 1, WG = TW + 4, GG = WG / 4;
  constexpr int NU = UR * GG;                 // U items (x_t / u), 153
  constexpr int NZ = T1 * (TW / 4);           // z' items, 128
  constexpr int NZ1 = (T1 + 2) * GG;          // z1 rows [r1-1, r1+T1]
  constexpr int NZ2 = UR * (GG + 1);          // z2 cols [c2-4, c2+WG)
  constexpr int SZU = UR * WG, SZ0 = UR * WG, SZ1 = (T1 + 2) * WG, SZ2 = UR * (WG + 4);
  static_assert(NU <= NT && NZ <= NT && NZ1 <= NT && NZ2 <= NT, "one item per thread");
  __shared__ __attribute__((aligned(16))) T U[2][SZU];
  __shared__ __attribute__((aligned(16))) T Z0[2][SZ0];
  __shared__ __attribute__((aligned(16))) T Z1[2][SZ1];
  __shared__ __attribute__((aligned(16))) T Z2[2][SZ2];
  __shared__ double red[4 * (NT / 64)];
  __shared__ int flag[2];
  if (ctrl != nullptr && ctrl->stopped != 0) return;  // loop already stopped (solver.py:65-66)

  int task;
  {  // XCD-aware bijective remap: consecutive tasks (neighbouring tiles of a segment) share an XCD
    const int b = blockIdx.x, q = ntasks / 8, r = ntasks % 8, xcd = b % 8, k = b / 8;
    task = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  const int per_plane = tiles1 * tiles2;
  const int seg = task / per_plane, t12 = task - seg * per_plane;
  const int ty = t12 / tiles2, tx = t12 - ty * tiles2;
  const int r1 = ty * T1, c2 = tx * TW;
  int p_start, p_end;  // own planes [p_start, p_end)
  band_rows(bd, seg, p_start, p_end);
  const int tid = threadIdx.x;
  const int64_t zstride = (int64_t)(v.planes + 2 * v.hz) * v.n1 * v.n2;
  const int64_t pl = (int64_t)v.n1 * v.n2;

  // fixed per-thread item geometry
  const int ue = min(tid, NU - 1), ui = ue / GG, ug = ue - (ue / GG) * GG;  // U item: row ui, group ug
  const bool u_real = tid < NU;
  const int ze = min(tid, NZ - 1), zi = ze / (TW / 4), zg = ze - (ze / (TW / 4)) * (TW / 4);
  const int e1 = min(tid, NZ1 - 1), e1r = e1 / GG, e1g = e1 - (e1 / GG) * GG;
  const int e2 = min(tid, NZ2 - 1), e2r = e2 / (GG + 1), e2g = e2 - (e2 / (GG + 1)) * (GG + 1);
  const GOff<T, VEC> off_u = goff<T, VEC>(v, r1 + ui, c2 + 4 * ug);
  const GOff<T, VEC> off_z1 = goff<T, VEC>(v, r1 - 1 + e1r, c2 + 4 * e1g);
  const GOff<T, VEC> off_z2 = goff<T, VEC>(v, r1 + e2r, c2 - 4 + 4 * e2g);
  // column flags (loop-invariant): U item inside the image / on the last 4-group; z' item likewise
  const int i1u = r1 + ui, c_u = c2 + 4 * ug, i1z = r1 + zi, c_z = c2 + 4 * zg;
  // bits: 0 row in image, 1 group starts in image, 2 group is the last one, 3 last row; 4-7 the
  // same for the z' item
  const int flags = ((i1u < v.n1) ? 1 : 0) | ((c_u < v.n2) ? 2 : 0) | ((c_u == v.n2 - 4) ? 4 : 0) |
                    ((i1u == v.n1 - 1) ? 8 : 0) | ((i1z < v.n1) ? 16 : 0) | ((c_z < v.n2) ? 32 : 0) |
                    ((c_z == v.n2 - 4) ? 64 : 0) | ((i1z == v.n1 - 1) ? 128 : 0);

  G4<T> xr, gr, z0r, z1r, z2r;
  // ---- PCS_F_CONV0 ring waves: ring item = 3 consecutive voxels of the U tile (rows [r1, r1 + T1],
  // cols [c2, c2 + WG)), two 15-plane register rings per voxel, tw[KR-1-j] = t(P - j) and
  // rw[KR-1-j] = r(P - off0 - j), the taps zero-padded to 15 (g(P - 14) from the push of t(P));
  // g(p + 1) lands in GS while the update waves work on plane p
  constexpr int KR = FOLD ? k3C0K : 1, RV = PCS_3D_RV;
  constexpr int UWAVES = (NU + 63) / 64, NRI = UR * WG / RV;
  // first ring thread: the update loop's item-free waves join the ring waves when RV = 2
  constexpr int IWAVES = (cmax(cmax(NU, NZ), cmax(NZ1, NZ2)) + 63) / 64;  // waves holding update items
  constexpr int RBASE = RV == 2 ? 64 * IWAVES : K3<T>::NT;
  static_assert(!FOLD || (WG % RV == 0 && NRI <= NT - RBASE && RBASE <= K3<T>::NT && 64 * IWAVES <= RBASE),
                "ring items: whole rows, one per ring thread, none on a wave with update items");
  __shared__ __attribute__((aligned(16))) T GS[2][FOLD ? SZU : 4];
  const bool ring_wave = FOLD && tid >= RBASE;  // wave-uniform
  const bool u_wave = (tid >> 6) < UWAVES;
  const int rr = tid - RBASE, ritem = min(max(rr, 0), NRI - 1);
  const int rrow = (ritem * RV) / WG, rcol = ritem * RV - rrow * WG;
  uint32_t roff[RV];
#pragma unroll
  for (int m = 0; m < RV; ++m) roff[m] = inplane<T>(v, r1 + rrow, c2 + rcol + m);
  T h0[KR], tw[KR][RV], rw[KR][RV], tq[RV], wq[RV];
  if constexpr (FOLD) {
#pragma unroll
    for (int j = 0; j < KR; ++j) {
      h0[j] = j < k0 ? taps0[j] : T(0);
#pragma unroll
      for (int m = 0; m < RV; ++m) tw[j][m] = rw[j][m] = T(0);
    }
  }
  auto load0 = [&](int Pl, T (&tv)[RV], T (&wv)[RV]) {  // t of plane Pl, w of plane Pl - off0
    const Rsrc rt = plane_rsrc(g, v, v.hg, Pl), rw0 = plane_rsrc(w0, v, v.hg, Pl - off0);
#pragma unroll
    for (int m = 0; m < RV; ++m) {
      tv[m] = bload1<T>(rt, roff[m]);
      wv[m] = bload1<T>(rw0, roff[m]);
    }
  };
  // push t(Pl): r(Pl - off0) = sum_j h0[j] t(Pl - j) - w (0 off the image / the stored planes);
  // o = g(Pl - KR + 1) = sum_j h0[KR-1-j] r(Pl - off0 - j) (the adjoint's flipped taps): the sums
  // of k_conv0_rta for 15 taps in its order
  auto push0 = [&](int Pl, const T (&tv)[RV], const T (&wv)[RV], T (&o)[RV]) {
#pragma unroll
    for (int j = 0; j + 1 < KR; ++j)
#pragma unroll
      for (int m = 0; m < RV; ++m) tw[j][m] = tw[j + 1][m];
#pragma unroll
    for (int m = 0; m < RV; ++m) tw[KR - 1][m] = tv[m];
    const int pr = Pl - off0, gpr = v.plane0 + pr;
    const bool rv = gpr >= 0 && gpr < v.n0 && pr >= -v.hg && pr < v.planes + v.hg;
    T acc[RV], sacc[RV];
#pragma unroll
    for (int m = 0; m < RV; ++m) acc[m] = sacc[m] = T(0);
#pragma unroll
    for (int j = 0; j < KR; ++j)
#pragma unroll
      for (int m = 0; m < RV; ++m) acc[m] += h0[j] * tw[KR - 1 - j][m];
#pragma unroll
    for (int j = 0; j + 1 < KR; ++j)
#pragma unroll
      for (int m = 0; m < RV; ++m) rw[j][m] = rw[j + 1][m];
#pragma unroll
    for (int m = 0; m < RV; ++m) {
      const T rm = acc[m] - wv[m];
      rw[KR - 1][m] = rv ? rm : T(0);
    }
#pragma unroll
    for (int j = 0; j < KR; ++j)
#pragma unroll
      for (int m = 0; m < RV; ++m) sacc[m] += h0[KR - 1 - j] * rw[KR - 1 - j][m];
#pragma unroll
    for (int m = 0; m < RV; ++m) o[m] = sacc[m];
  };
  auto gstore3 = [&](int slot, const T (&o)[RV]) {
    if (rr < NRI) {
#pragma unroll
      for (int m = 0; m < RV; ++m) GS[slot][rrow * WG + rcol + m] = o[m];
    }
  };
  auto prefetch = [&](int p) {
    const Rsrc rx = plane_rsrc(x, v, v.hx, p), rz0 = plane_rsrc(z, v, v.hz, p),
               rz1 = plane_rsrc(z + zstride, v, v.hz, p), rz2 = plane_rsrc(z + 2 * zstride, v, v.hz, p);
    xr = gload<T, VEC>(rx, off_u);
    if constexpr (FK != PCS_F_NULL && !FOLD) gr = gload<T, VEC>(plane_rsrc(g, v, v.hg, p), off_u);
    z0r = gload<T, VEC>(rz0, off_u);
    z1r = gload<T, VEC>(rz1, off_z1);
    z2r = gload<T, VEC>(rz2, off_z2);
  };
  auto land = [&](int slot) {
    if (tid < NU) tl_st<WG>(Z0[slot], ui, ug, z0r);
    if (tid < NZ1) tl_st<WG>(Z1[slot], e1r, e1g, z1r);
    if (tid < NZ2) tl_st<WG + 4>(Z2[slot], e2r, e2g, z2r);
  };

  double part[4] = {0.0, 0.0, 0.0, 0.0};
  if (ring_wave) {  // the ring waves' own loop: the update loop's three barriers per plane
    T o[RV];
    {  // fill the rings up to t(p_start + KR - 1): g(p_start) -> GS; the 2 KR - 1 pushes run in
      // blocks of D with the loads of planes D ahead in flight (D register sets)
      constexpr int D = PCS_3D_RPD, NP = 2 * KR - 1;
      T tb[D][RV], wb[D][RV];
#pragma unroll
      for (int j = 0; j < D; ++j) load0(p_start - KR + 1 + j, tb[j], wb[j]);
      int Pl = p_start - KR + 1;
      for (int i = 0; i < NP / D; ++i) {
#pragma unroll
        for (int j = 0; j < D; ++j, ++Pl) {
          T tc[RV], wc[RV];
#pragma unroll
          for (int m = 0; m < RV; ++m) {
            tc[m] = tb[j][m];
            wc[m] = wb[j][m];
          }
          load0(Pl + D, tb[j], wb[j]);
          push0(Pl, tc, wc, o);
        }
      }
#pragma unroll
      for (int j = 0; j < NP % D; ++j, ++Pl) push0(Pl, tb[j], wb[j], o);
      // Pl = p_start + KR: its t / w sit in set NP % D (the last one issued for it)
      gstore3(p_start & 1, o);
#pragma unroll
      for (int m = 0; m < RV; ++m) {
        tq[m] = tb[NP % D][m];
        wq[m] = wb[NP % D][m];
      }
    }
    for (int p = p_start; p <= p_end; ++p) {
      lds_barrier();
      lds_barrier();
      if (p < p_end) {  // g(p + 1) -> GS while the update waves work on plane p
        T tc[RV], wc[RV];
#pragma unroll
        for (int m = 0; m < RV; ++m) {
          tc[m] = tq[m];
          wc[m] = wq[m];
        }
        load0(p + KR + 1, tq, wq);
        push0(p + KR, tc, wc, o);
        gstore3((p + 1) & 1, o);
      }
      lds_barrier();
    }
  } else {
  // prologue: z0 of plane p_start - 1 (for D0^T z0 at p_start), then plane p_start's data
  {
    const Rsrc rz0 = plane_rsrc(z, v, v.hz, p_start - 1);
    const G4<T> zp = gload<T, VEC>(rz0, off_u);
    if (tid < NU) tl_st<WG>(Z0[(p_start - 1) & 1], ui, ug, zp);
  }
  prefetch(p_start);
  for (int p = p_start; p <= p_end; ++p) {
    const int slot = p & 1, prev = slot ^ 1;
    const int gp = v.plane0 + p;
    lds_barrier();  // plane p-1's z' items are done with U[slot], Z*[slot]
    const G4<T> xv4 = xr;
    G4<T> gv4;
    if constexpr (FK != PCS_F_NULL && !FOLD) gv4 = gr;
    land(slot);
#if PCS_3D_PRIO
    __builtin_amdgcn_s_setprio(3);
#endif
    if (p < p_end) prefetch(p + 1);
#if PCS_3D_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    lds_barrier();
    const int fl = launder(flags);
    // ---- U items: x_t, u on rows [r1, r1 + T1], cols [c2, c2 + WG) of plane p; x' on own cells
    if (!FOLD || u_wave) {  // every thread runs an item (surplus threads redo the last one; only
      // real items store); with FOLD the waves without real items skip it
      if constexpr (FOLD) gv4 = lds4(&GS[slot][ui * WG + 4 * ug]);  // g(p)
      const G4<T> zb = tl_ld<WG>(Z0[slot], ui, ug);           // z0(p)
      const G4<T> za = tl_ld<WG>(Z0[prev], ui, ug);           // z0(p-1)
      const G4<T> z1a = tl_ld<WG>(Z1[slot], ui, ug);          // z1(p, i1-1)
      const G4<T> z1b = tl_ld<WG>(Z1[slot], ui + 1, ug);      // z1(p, i1)
      const G4<T> z2a = tl_ld<WG + 4>(Z2[slot], ui, ug);      // z2(p, c-4 .. c-1)
      const G4<T> z2b = tl_ld<WG + 4>(Z2[slot], ui, ug + 1);
      const bool rin = fl & 1, gin = fl & 2, glast = fl & 4, rlast = fl & 8;
      const bool p_first = gp <= 0, p_last = gp >= v.n0 - 1;
      const bool in = rin && gin && gp >= 0 && gp < v.n0 && p <= v.planes;
      const bool own = in && u_real && ui < T1 && ug < TW / 4 && p < p_end;
      G4<T> uo, xo;
      T sdx = T(0), sx = T(0);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const T xv = xv4.v[m];
        T gf;
        if constexpr (FK == PCS_F_NULL) gf = T(0);
        else if constexpr (FK == PCS_F_DENOISE) gf = xv - gv4.v[m];
        else gf = gv4.v[m];
        // K^T z, VStack order: ((0 + D0^T z0) + D1^T z1) + D2^T z2; neighbours outside the
        // image load as 0, the last sample of each forward difference is not used
        T d0 = p_first ? T(0) : za.v[m];
        if (!p_last) d0 -= zb.v[m];
        T d1 = z1a.v[m];
        if (!rlast) d1 -= z1b.v[m];
        const T z2l = (m == 0) ? z2a.v[3] : z2b.v[m - 1];
        const bool lastc = VEC ? (m == 3 && glast) : (c_u + m == v.n2 - 1);
        const bool cm = VEC ? true : (c_u + m < v.n2);  // element inside the image (group known in)
        const T d2 = z2l - (lastc ? T(0) : z2b.v[m]);
        const T a0 = P.unit[0] ? d0 : d0 * P.inv_step[0];
        const T a1 = P.unit[1] ? d1 : d1 * P.inv_step[1];
        const T a2 = P.unit[2] ? d2 : d2 * P.inv_step[2];
        const T xt = prox_g((xv - P.tau * gf) - P.tau * ((a0 + a1) + a2), gk, P.seg_a, P.seg_b);
        uo.v[m] = (in && cm) ? (T(2) * xt - xv) : T(0);
        const T xnew = P.rho * xt + P.omr * xv;
        xo.v[m] = xnew;
        const T dx = xv - xnew;
        sdx += cm ? dx * dx : T(0);
        sx += cm ? xv * xv : T(0);
      }
      if (own) {
        part[0] += (double)sdx;
        part[1] += (double)sx;
        gstore<T, VEC>(xn + (int64_t)(p + v.hx) * pl + (int64_t)i1u * v.n2 + c_u, xo, c_u, v.n2);
      }
      if (tid < NU) tl_st<WG>(U[slot], ui, ug, uo);
    }
    lds_barrier();
    // ---- z' items for plane p - 1 (own tile)
    if (p > p_start && tid < NZ) {
      const int q = p - 1, gq = gp - 1;
      const bool rin = fl & 16, gin = fl & 32, glast = fl & 64, rlast = fl & 128;
      const bool own = rin && gin && gq < v.n0;
      const G4<T> uc = tl_ld<WG>(U[prev], zi, zg);
      const G4<T> un = tl_ld<WG>(U[prev], zi, zg + 1);
      const G4<T> ud = tl_ld<WG>(U[prev], zi + 1, zg);
      const G4<T> up = tl_ld<WG>(U[slot], zi, zg);  // u(p)
      const G4<T> zv0 = tl_ld<WG>(Z0[prev], zi, zg);
      const G4<T> zv1 = tl_ld<WG>(Z1[prev], zi + 1, zg);
      const G4<T> zv2 = tl_ld<WG + 4>(Z2[prev], zi, zg + 1);
      const bool q_last = gq >= v.n0 - 1;
      G4<T> o0, o1, o2;
      T sdz = T(0), sz = T(0);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const T uright = (m < 3) ? uc.v[m + 1] : un.v[0];
        const T d0 = q_last ? T(0) : (up.v[m] - uc.v[m]);
        const T d1 = rlast ? T(0) : (ud.v[m] - uc.v[m]);
        const bool lastc = VEC ? (m == 3 && glast) : (c_z + m == v.n2 - 1);
        const bool cm = VEC ? true : (c_z + m < v.n2);
        const T d2 = lastc ? T(0) : (uright - uc.v[m]);
        const T k0 = P.unit[0] ? d0 : d0 * P.inv_step[0];
        const T k1 = P.unit[1] ? d1 : d1 * P.inv_step[1];
        const T k2 = P.unit[2] ? d2 : d2 * P.inv_step[2];
        const T w0 = zv0.v[m] + P.sigma * k0, w1 = zv1.v[m] + P.sigma * k1, w2 = zv2.v[m] + P.sigma * k2;
        const T v0 = w0 * P.inv_sigma, v1 = w1 * P.inv_sigma, v2 = w2 * P.inv_sigma;
        T t0, t1, t2;
        if (hk == PCS_H_L21) {  // w - sigma * (max(1 - t/||v||, 0) v), penalty.py:551-557
          T f = T(1) - P.t_h * fast_rsqrt((v0 * v0 + v1 * v1) + v2 * v2);
          f = f > T(0) ? f : T(0);
          t0 = w0 - P.sigma * (f * v0);
          t1 = w1 - P.sigma * (f * v1);
          t2 = w2 - P.sigma * (f * v2);
        } else {  // w - sigma * (v - t*clip(v/t)), func/base.py:239-240
          t0 = w0 - P.sigma * (v0 - P.t_h * clip1(v0 * P.inv_t_h));
          t1 = w1 - P.sigma * (v1 - P.t_h * clip1(v1 * P.inv_t_h));
          t2 = w2 - P.sigma * (v2 - P.t_h * clip1(v2 * P.inv_t_h));
        }
        o0.v[m] = P.rho * t0 + P.omr * zv0.v[m];
        o1.v[m] = P.rho * t1 + P.omr * zv1.v[m];
        o2.v[m] = P.rho * t2 + P.omr * zv2.v[m];
        const T e0 = zv0.v[m] - o0.v[m], e1 = zv1.v[m] - o1.v[m], e2 = zv2.v[m] - o2.v[m];
        sdz += cm ? (e0 * e0 + e1 * e1) + e2 * e2 : T(0);
        sz += cm ? (zv0.v[m] * zv0.v[m] + zv1.v[m] * zv1.v[m]) + zv2.v[m] * zv2.v[m] : T(0);
      }
      if (own) {
        part[2] += (double)sdz;
        part[3] += (double)sz;
        T* d = zn + (int64_t)(q + v.hz) * pl + (int64_t)i1z * v.n2 + c_z;
        gstore<T, VEC>(d, o0, c_z, v.n2);
        gstore<T, VEC>(d + zstride, o1, c_z, v.n2);
        gstore<T, VEC>(d + 2 * zstride, o2, c_z, v.n2);
      }
    }
  }
  }  // update waves
  block_sum<4>(part, red);
  if (hist != nullptr) {
    reduce_and_finalize(part, partials, ntasks, ws, ctrl, hist, flag);
  } else if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) partials[(int64_t)blockIdx.x * 4 + k] = part[k];
  }
}


// ---------------------------------------------------------------- general first-derivative K
// K = Gradient(kind = 'backward' | 'centered', edge, sampling) in 3-D (pycsou/linop/diff.py:777-882;
// 'centered' is the reference's default Gradient(shape)): D_a reaches one sample both ways, so
// K^T z at plane p needs z0 of planes p-1 .. p+1 and K u at plane q needs u of planes q-1 .. q+1.
// A workgroup owns a T1 x 128 tile and marches down its plane segment; iteration p:
//   land   z0(p+1) -> 3-plane z0 ring, z1(p) / z2(p) -> 2-plane rings, x(p), g(p) from registers;
//          issue the loads of iteration p+1
//   U      x_t, u on the tile +- 1 row / one 4-group (u(p) -> 3-plane u ring), x'(p) on own voxels
//   Z      z'(p-1): K u from u(p-2 .. p), fenchel prox, relaxation
// The segment's first iteration is plane p_start - 1 (u there feeds K u at p_start), its last is
// p_end (u for K u at p_end - 1).  Per-element stencils: stencil.hpp's window forms (sw_d1_*), the
// same arithmetic for every voxel (no interior specialisation), so slabs are bitwise the whole
// volume.  Traffic per voxel: x, g, z (3) in; x', z' (3) out = 9 words (the forward kernel's),
// plus the tile halos (rows +- 1, one 4-group per side).
// Tiles: fp64 12 x 128 (155.5 KB of LDS; 16 rows would need 202 KB.  C5 centred: 17.1 ms against 18.4 at
// 8 rows, reads 1.45x -> ~1.33x the algorithmic; 10 rows measured 20.0 ms, profiles/r6_g64rows_ab.txt).
// fp32 12 x 256 in 1024-thread workgroups with one prefetch register set (150 KB, 109-128 VGPRs): every
// row segment a tile reads is 1 KB, as the fp64 tiles' are -- C4 centred 1.075 ms against 1.267 for 16 x 128
// (512 threads, two sets; 512-B segments, about the same halo share) and 1.22 for 8 x 256
// (profiles/r6_g32w_ab.txt); 16 x 128 at 1024 threads alone changed nothing (r6_g32nt_ab.txt), so the row
// segment length, not latency hiding, was what held the fp32 kernel at ~4.4 TB/s
#ifndef PCS_3DG_NT32  // fp32 workgroup size (diagnostics builds override)
#define PCS_3DG_NT32 1024
#endif
#ifndef PCS_3DG_TW32  // fp32 tile columns (diagnostics builds override)
#define PCS_3DG_TW32 256
#endif
template <typename T>
constexpr int k3g_tw() { return sizeof(T) == 4 ? PCS_3DG_TW32 : 128; }
#ifndef PCS_3DG_NT64  // fp64 workgroup size (diagnostics builds override; 1024 with one set spills 98-202 VGPRs)
#define PCS_3DG_NT64 512
#endif
template <typename T>
constexpr int k3g_nt() { return sizeof(T) == 4 ? PCS_3DG_NT32 : PCS_3DG_NT64; }
#ifndef PCS_3DG_SETS32  // fp32 prefetch register sets (diagnostics builds override)
#define PCS_3DG_SETS32 1
#endif
#ifndef PCS_3DG_SETS64  // fp64 prefetch register sets (diagnostics builds override)
#define PCS_3DG_SETS64 2
#endif
template <typename T>
constexpr int k3g_sets() { return sizeof(T) == 4 ? PCS_3DG_SETS32 : PCS_3DG_SETS64; }
#ifndef PCS_3DG_ROWS32  // fp32 tile rows (diagnostics builds override)
#define PCS_3DG_ROWS32 12
#endif
#ifndef PCS_3DG_ROWS64  // fp64 tile rows (diagnostics builds override)
#define PCS_3DG_ROWS64 12
#endif
template <typename T>
constexpr int k3g_rows() { return sizeof(T) == 4 ? PCS_3DG_ROWS32 : PCS_3DG_ROWS64; }

#ifndef PCS_3DG_ROWFORM  // column-border tiles with the row axis interior get their own code form (A/B knob)
#define PCS_3DG_ROWFORM 1
#endif
#ifndef PCS_3DG_MINB  // workgroups per CU the register budget targets (diagnostics builds override)
#define PCS_3DG_MINB 1
#endif
template <typename T, int KK, int FK, bool VEC>
__global__ __launch_bounds__(k3g_nt<T>(), PCS_3DG_MINB) void k_pds3d_gen(const T* __restrict__ x, T* __restrict__ xn,
                                                     const T* __restrict__ z, T* __restrict__ zn,
                                                     const T* __restrict__ g, Vol v, P3<T> P, int hk, int gk, int edge,
                                                     double* __restrict__ partials, Ctrl* ctrl, double* hist, void* ws,
                                                     int tiles1, int tiles2, Bands bd, int ntasks) {
  constexpr int T1 = k3g_rows<T>(), TW = k3g_tw<T>(), NT = k3g_nt<T>();
  constexpr int UR = T1 + 2, UG = TW / 4 + 2, WU = 4 * UG;  // u / z0 region: rows r1-1 .. r1+T1, cols c2-4 ..
  constexpr int R1 = T1 + 4, W2G = UG + 2, W2 = 4 * W2G;    // z1 rows r1-2 .. r1+T1+1; z2 cols c2-8 .. c2+TW+8
  constexpr int NU = UR * UG, NZ1 = R1 * UG, NZ2 = UR * W2G, NZ = T1 * (TW / 4);
  constexpr int KU = (NU + NT - 1) / NT, K1 = (NZ1 + NT - 1) / NT, K2 = (NZ2 + NT - 1) / NT;
  static_assert(NZ <= NT, "one z' item per thread");
  __shared__ __attribute__((aligned(16))) T U[3][UR * WU];
  __shared__ __attribute__((aligned(16))) T Z0[3][UR * WU];
  __shared__ __attribute__((aligned(16))) T Z1[2][R1 * WU];
  __shared__ __attribute__((aligned(16))) T Z2[2][UR * W2];
  __shared__ double red[4 * (NT / 64)];
  __shared__ int flag[2];
  if (ctrl != nullptr && ctrl->stopped != 0) return;  // loop already stopped (solver.py:65-66)

  int task;
  {  // XCD-aware bijective remap: consecutive tasks (neighbouring tiles of a segment) share an XCD
    const int b = blockIdx.x, q = ntasks / 8, r = ntasks % 8, xcd = b % 8, k = b / 8;
    task = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  }
  const int per_plane = tiles1 * tiles2;
  const int seg = task / per_plane, t12 = task - seg * per_plane;
  const int ty = t12 / tiles2, tx = t12 - ty * tiles2;
  const int r1 = ty * T1, c2 = tx * TW;
  int p_start, p_end;  // own planes [p_start, p_end)
  band_rows(bd, seg, p_start, p_end);
  const int tid = threadIdx.x;
  const int64_t zstride = (int64_t)(v.planes + 2 * v.hz) * v.n1 * v.n2;
  const int64_t pl = (int64_t)v.n1 * v.n2;

  // item geometry (fixed per thread): U / z0 items (row ui, group ug of the u region), z1 / z2 load
  // items, the z' item (own row zi, own group zg)
  int ui[KU], ug[KU];
  GOff<T, VEC> off_u[KU], off_1[K1], off_2[K2];
#pragma unroll
  for (int k = 0; k < KU; ++k) {
    const int e = min(k * NT + tid, NU - 1);
    ui[k] = e / UG;
    ug[k] = e - ui[k] * UG;
    off_u[k] = goff<T, VEC>(v, r1 - 1 + ui[k], c2 - 4 + 4 * ug[k]);
  }
#pragma unroll
  for (int k = 0; k < K1; ++k) {
    const int e = min(k * NT + tid, NZ1 - 1), r = e / UG;
    off_1[k] = goff<T, VEC>(v, r1 - 2 + r, c2 - 4 + 4 * (e - r * UG));
  }
#pragma unroll
  for (int k = 0; k < K2; ++k) {
    const int e = min(k * NT + tid, NZ2 - 1), r = e / W2G;
    off_2[k] = goff<T, VEC>(v, r1 - 1 + r, c2 - 8 + 4 * (e - r * W2G));
  }
  const int ze = min(tid, NZ - 1), zi = ze / (TW / 4), zg = ze - zi * (TW / 4);
  const int i1z = r1 + zi, c_z = c2 + 4 * zg;
  // the tile's u region (rows r1-1 .. r1+T1, cols c2-4 .. c2+TW+3) >= 2 samples inside the plane
  // the tile's u region (rows r1-1 .. r1+T1, cols c2-4 .. c2+TW+3) >= 2 samples inside the plane
  const bool row_int = r1 - 1 >= 2 && r1 + T1 <= v.n1 - 3, col_int = c2 - 4 >= 2 && c2 + TW + 3 <= v.n2 - 3;
  const bool tile_int = row_int && col_int;
  // a tile on a column border only (most border tiles: every plane row has two) keeps the row axis interior
  const bool row_only = PCS_3DG_ROWFORM && row_int && !col_int;

  // loads run two planes ahead: iteration p lands set p & 1 and refills it with plane p + 2's data
  // (C4 centred: 1.41 ms with one set; the wait for the next plane's loads was exposed at two waves
  // per SIMD)
  constexpr int NSET = k3g_sets<T>();  // register sets of prefetched planes (loads run NSET planes ahead)
  G4<T> xr[NSET][KU], gr[NSET][KU], z0r[NSET][KU], z1r[NSET][K1], z2r[NSET][K2];
  auto prefetch = [&](int p, auto sc) {  // x, g, z1, z2 of plane p; z0 of plane p + 1 -> set sc
    constexpr int S = decltype(sc)::value;
    const Rsrc rx = plane_rsrc(x, v, v.hx, p), rz0 = plane_rsrc(z, v, v.hz, p + 1),
               rz1 = plane_rsrc(z + zstride, v, v.hz, p), rz2 = plane_rsrc(z + 2 * zstride, v, v.hz, p);
#pragma unroll
    for (int k = 0; k < KU; ++k) {
      xr[S][k] = gload<T, VEC>(rx, off_u[k]);
      if constexpr (FK != PCS_F_NULL) gr[S][k] = gload<T, VEC>(plane_rsrc(g, v, v.hg, p), off_u[k]);
      z0r[S][k] = gload<T, VEC>(rz0, off_u[k]);
    }
#pragma unroll
    for (int k = 0; k < K1; ++k) z1r[S][k] = gload<T, VEC>(rz1, off_1[k]);
#pragma unroll
    for (int k = 0; k < K2; ++k) z2r[S][k] = gload<T, VEC>(rz2, off_2[k]);
  };
  auto land = [&](int s3, int s2, auto sc) {  // z0 slot s3 (plane p + 1), z1 / z2 slot s2 (plane p)
    constexpr int S = decltype(sc)::value;
#pragma unroll
    for (int k = 0; k < KU; ++k)
      if (k * NT + tid < NU) tl_st<WU>(Z0[s3], ui[k], ug[k], z0r[S][k]);
#pragma unroll
    for (int k = 0; k < K1; ++k)
      if (k * NT + tid < NZ1) tl_st<WU>(Z1[s2], (k * NT + tid) / UG, (k * NT + tid) % UG, z1r[S][k]);
#pragma unroll
    for (int k = 0; k < K2; ++k)
      if (k * NT + tid < NZ2) tl_st<W2>(Z2[s2], (k * NT + tid) / W2G, (k * NT + tid) % W2G, z2r[S][k]);
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;

  double part[4] = {0.0, 0.0, 0.0, 0.0};
  // ring slots: plane j lives in slot (j + 3 * 2^20) % 3 of the 3-plane rings, (j & 1) of the others
  auto slot3 = [](int j) { return (int)((unsigned)(j + 3 * (1 << 20)) % 3u); };
  {  // prologue: z0 of planes p_start - 2 and p_start - 1
    const int pa = p_start - 2;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const Rsrc r0 = plane_rsrc(z, v, v.hz, pa + j);
#pragma unroll
      for (int k = 0; k < KU; ++k) {
        const G4<T> zz = gload<T, VEC>(r0, off_u[k]);
        if (k * NT + tid < NU) tl_st<WU>(Z0[slot3(pa + j)], ui[k], ug[k], zz);
      }
    }
  }
  prefetch(p_start - 1, S0{});
  if constexpr (NSET == 2)
    if (p_start <= p_end) prefetch(p_start, S1{});
  auto iter = [&](int p, auto sc) {
    constexpr int S = decltype(sc)::value;
    const int sm1 = slot3(p - 1), s0 = slot3(p), sp1 = slot3(p + 1), sm2 = slot3(p - 2);
      const int b2 = p & 1;
      const int gp = v.plane0 + p;
      lds_barrier();  // iteration p-1's z' items are done with the slots landed / written below
      G4<T> xv4[KU], gv4[KU];
#pragma unroll
      for (int k = 0; k < KU; ++k) {
        xv4[k] = xr[S][k];
        if constexpr (FK != PCS_F_NULL) gv4[k] = gr[S][k];
      }
      land(sp1, b2, sc);
      if (p + NSET <= p_end) prefetch(p + NSET, sc);
      lds_barrier();
      // ---- U items: x_t, u on the u region of plane p; x' on own voxels (I: every sample of the
      // tile's u region and plane p lies >= 2 samples inside the volume -- no edge rules)
      auto u_items = [&](auto ic0, auto ic12, auto ic2) {  // interior along axis 0 / axis 1 / axis 2
        constexpr bool I0 = decltype(ic0)::value, I1 = decltype(ic12)::value, I2 = decltype(ic2)::value;
#pragma unroll
        for (int k = 0; k < KU; ++k) {
          if (k * NT + tid >= NU) continue;
          const int i1 = r1 - 1 + ui[k], c = c2 - 4 + 4 * ug[k];
          const int ur = ui[k], uq = ug[k];
          const G4<T> za = tl_ld<WU>(Z0[sm1], ur, uq), zb = tl_ld<WU>(Z0[s0], ur, uq), zc = tl_ld<WU>(Z0[sp1], ur, uq);
          // z1 region rows ur .. ur + 2 = rows i1 - 1 .. i1 + 1; z2 region groups uq .. uq + 2 = c - 4 .. c + 7
          const G4<T> y0 = tl_ld<WU>(Z1[b2], ur, uq), y1 = tl_ld<WU>(Z1[b2], ur + 1, uq), y2 = tl_ld<WU>(Z1[b2], ur + 2, uq);
          const G4<T> wl = tl_ld<W2>(Z2[b2], ur, uq), wc = tl_ld<W2>(Z2[b2], ur, uq + 1), wr = tl_ld<W2>(Z2[b2], ur, uq + 2);
          const T h2[6] = {wl.v[3], wc.v[0], wc.v[1], wc.v[2], wc.v[3], wr.v[0]};
          const bool rin = (unsigned)i1 < (unsigned)v.n1, pin = gp >= 0 && gp < v.n0;
          const bool own = rin && pin && ui[k] >= 1 && ui[k] <= T1 && ug[k] >= 1 && ug[k] <= TW / 4 && c < v.n2 &&
                           p >= p_start && p < p_end;
          G4<T> uo, xo;
          T sdx = T(0), sx = T(0);
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            const int i2 = c + m;
            const bool in = rin && pin && (unsigned)i2 < (unsigned)v.n2;
            const T w0[5] = {T(0), za.v[m], zb.v[m], zc.v[m], T(0)};
            const T w1[5] = {T(0), y0.v[m], y1.v[m], y2.v[m], T(0)};
            const T w2[5] = {T(0), h2[m], h2[m + 1], h2[m + 2], T(0)};
            // K^T z, VStack order ((D0^T z0 + D1^T z1) + D2^T z2), each sum scaled by 1/h once
            const T kt = pcs_fma(sw_d1_adj<KK, I2>(w2, i2, v.n2, edge), P.inv_step[2],
                                 pcs_fma(sw_d1_adj<KK, I1>(w1, i1, v.n1, edge), P.inv_step[1],
                                         sw_d1_adj<KK, I0>(w0, gp, v.n0, edge) * P.inv_step[0]));
            const T xv = xv4[k].v[m];
            T gf;
            if constexpr (FK == PCS_F_NULL) gf = T(0);
            else if constexpr (FK == PCS_F_DENOISE) gf = xv - gv4[k].v[m];
            else gf = gv4[k].v[m];
            const T xt = prox_g((xv - P.tau * gf) - P.tau * kt, gk, P.seg_a, P.seg_b);
            uo.v[m] = in ? (T(2) * xt - xv) : T(0);
            const T xnew = pcs_fma(P.rho, xt, P.omr * xv);
            xo.v[m] = xnew;
            const T dx = xv - xnew;
            sdx += in ? dx * dx : T(0);
            sx += in ? xv * xv : T(0);
          }
          if (own) {
            part[0] += (double)sdx;
            part[1] += (double)sx;
            gstore<T, VEC>(xn + (int64_t)(p + v.hx) * pl + (int64_t)i1 * v.n2 + c, xo, c, v.n2);
          }
          tl_st<WU>(U[s0], ur, uq, uo);
        }
      };
      // three forms: interior; the edge rules on the row and column axes only (the tiles along the plane's
      // border, on every plane but the first / last two); the edge rules on every axis.  With one task per
      // CU the kernel ends with its slowest task: the border row tiles on the all-axes form held C4 centred
      // at 1.37-1.42 ms against 1.11 with every tile interior (profiles/r5_g3d_edge_ab.txt)
      using Tt = std::true_type;
      using Ff = std::false_type;
      const bool pint_u = gp >= 2 && gp <= v.n0 - 3;
      if (tile_int && pint_u) u_items(Tt{}, Tt{}, Tt{});
      else if (row_only && pint_u) u_items(Tt{}, Tt{}, Ff{});
      else if (pint_u) u_items(Tt{}, Ff{}, Ff{});
      else u_items(Ff{}, Ff{}, Ff{});
      lds_barrier();
      // ---- z' items for plane q = p - 1 (own tile)
      auto z_items = [&](auto ic0, auto ic12, auto ic2) {
        constexpr bool I0 = decltype(ic0)::value, I1 = decltype(ic12)::value, I2 = decltype(ic2)::value;
        if (p > p_start && tid < NZ) {
          const int q = p - 1, gq = gp - 1;
          const int orr = zi + 1, og = zg + 1;  // the u region's row / group of the item
          const G4<T> ua = tl_ld<WU>(U[sm2], orr, og), ub = tl_ld<WU>(U[sm1], orr, og),
                      uc = tl_ld<WU>(U[s0], orr, og);                                         // u(q-1), u(q), u(q+1)
          const G4<T> un = tl_ld<WU>(U[sm1], orr - 1, og), us = tl_ld<WU>(U[sm1], orr + 1, og);  // rows i1-1, i1+1
          const G4<T> ul = tl_ld<WU>(U[sm1], orr, og - 1), ur = tl_ld<WU>(U[sm1], orr, og + 1);  // groups left / right
          const T h2[6] = {ul.v[3], ub.v[0], ub.v[1], ub.v[2], ub.v[3], ur.v[0]};
          const G4<T> zv0 = tl_ld<WU>(Z0[sm1], orr, og);
          const G4<T> zv1 = tl_ld<WU>(Z1[b2 ^ 1], zi + 2, zg + 1);
          const G4<T> zv2 = tl_ld<W2>(Z2[b2 ^ 1], zi + 1, zg + 2);
          const bool own = i1z < v.n1 && gq >= 0 && gq < v.n0 && c_z < v.n2;
          G4<T> o0, o1, o2;
          T sdz = T(0), sz = T(0);
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            const int i2 = c_z + m;
            const bool cm = VEC ? true : (i2 < v.n2);
            const T w0[5] = {T(0), ua.v[m], ub.v[m], uc.v[m], T(0)};
            const T w1[5] = {T(0), un.v[m], ub.v[m], us.v[m], T(0)};
            const T w2[5] = {T(0), h2[m], h2[m + 1], h2[m + 2], T(0)};
            const T k0 = sw_d1_fwd<KK, I0>(w0, gq, v.n0, P.inv_step[0], edge);
            const T k1 = sw_d1_fwd<KK, I1>(w1, i1z, v.n1, P.inv_step[1], edge);
            const T k2 = sw_d1_fwd<KK, I2>(w2, i2, v.n2, P.inv_step[2], edge);
            const T w0v = zv0.v[m] + P.sigma * k0, w1v = zv1.v[m] + P.sigma * k1, w2v = zv2.v[m] + P.sigma * k2;
            const T v0 = w0v * P.inv_sigma, v1 = w1v * P.inv_sigma, v2 = w2v * P.inv_sigma;
            T t0, t1, t2;
            if (hk == PCS_H_L21) {  // w - sigma * (max(1 - t/||v||, 0) v), penalty.py:551-557
              T f = T(1) - P.t_h * fast_rsqrt(pcs_fma(v0, v0, pcs_fma(v1, v1, v2 * v2)));
              f = f > T(0) ? f : T(0);
              t0 = w0v - P.sigma * (f * v0);
              t1 = w1v - P.sigma * (f * v1);
              t2 = w2v - P.sigma * (f * v2);
            } else {  // w - sigma * (v - t*clip(v/t)), func/base.py:239-240
              t0 = w0v - P.sigma * (v0 - P.t_h * clip1(v0 * P.inv_t_h));
              t1 = w1v - P.sigma * (v1 - P.t_h * clip1(v1 * P.inv_t_h));
              t2 = w2v - P.sigma * (v2 - P.t_h * clip1(v2 * P.inv_t_h));
            }
            o0.v[m] = pcs_fma(P.rho, t0, P.omr * zv0.v[m]);
            o1.v[m] = pcs_fma(P.rho, t1, P.omr * zv1.v[m]);
            o2.v[m] = pcs_fma(P.rho, t2, P.omr * zv2.v[m]);
            const T e0 = zv0.v[m] - o0.v[m], e1 = zv1.v[m] - o1.v[m], e2 = zv2.v[m] - o2.v[m];
            sdz += cm ? pcs_fma(e0, e0, pcs_fma(e1, e1, e2 * e2)) : T(0);
            sz += cm ? pcs_fma(zv0.v[m], zv0.v[m], pcs_fma(zv1.v[m], zv1.v[m], zv2.v[m] * zv2.v[m])) : T(0);
          }
          if (own) {
            part[2] += (double)sdz;
            part[3] += (double)sz;
            T* d = zn + (int64_t)(q + v.hz) * pl + (int64_t)i1z * v.n2 + c_z;
            gstore<T, VEC>(d, o0, c_z, v.n2);
            gstore<T, VEC>(d + zstride, o1, c_z, v.n2);
            gstore<T, VEC>(d + 2 * zstride, o2, c_z, v.n2);
          }
        }
      };
      const bool pint_z = gp - 1 >= 2 && gp - 1 <= v.n0 - 3;
      if (tile_int && pint_z) z_items(Tt{}, Tt{}, Tt{});
      else if (row_only && pint_z) z_items(Tt{}, Tt{}, Ff{});
      else if (pint_z) z_items(Tt{}, Ff{}, Ff{});
      else z_items(Ff{}, Ff{}, Ff{});
  };
  if constexpr (NSET == 2) {
    for (int p = p_start - 1; p <= p_end; p += 2) {
      iter(p, S0{});
      if (p + 1 <= p_end) iter(p + 1, S1{});
    }
  } else {
    for (int p = p_start - 1; p <= p_end; ++p) iter(p, S0{});
  }
  block_sum<4>(part, red);
  if (hist != nullptr) {
    reduce_and_finalize(part, partials, ntasks, ws, ctrl, hist, flag);
  } else if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) partials[(int64_t)blockIdx.x * 4 + k] = part[k];
  }
}

// ---------------------------------------------------------------- host side
struct Plan3 {
  int tiles1, tiles2, ntasks;
  Bands bd;
};

// own-plane bands [a0, b0) u [a1, b1) of one launch (the whole slab: {0, planes, planes, planes})
struct PlaneBands {
  int64_t a0, b0, a1, b1;
};

// update-tile rows of the launch: the forward kernel's 8, or the general-K kernel's (k3g_rows)
static int tile_rows3(const pcs_pds3d_args* a) {
  if (a->kkind == PCS_BACKWARD || a->kkind == PCS_CENTERED) return a->dtype == PCS_F32 ? k3g_rows<float>() : k3g_rows<double>();
  return a->dtype == PCS_F32 ? k3_rows<float>() : k3_rows<double>();
}

static Plan3 plan3(const pcs_pds3d_args* a, PlaneBands pb) {
  Plan3 p;
  if (pb.b0 == pb.a0) pb = PlaneBands{pb.a1, pb.b1, pb.b1, pb.b1};
  const int t1 = tile_rows3(a);
  p.tiles1 = (int)((a->n1 + t1 - 1) / t1);
  const bool gen = a->kkind == PCS_BACKWARD || a->kkind == PCS_CENTERED, f32 = a->dtype == PCS_F32;
  const int tw = gen ? (f32 ? k3g_tw<float>() : k3g_tw<double>()) : f32 ? K3<float>::TW : K3<double>::TW;
  p.tiles2 = (int)((a->n2 + tw - 1) / tw);
  const int64_t per_plane = (int64_t)p.tiles1 * p.tiles2;
  const int64_t L0 = pb.b0 - pb.a0, L1 = pb.b1 - pb.a1, L = L0 + L1;
  const int64_t bands = (L0 > 0) + (L1 > 0);
  // as few plane segments as give one workgroup per CU (the device's CU count): long marches amortise the
  // two-plane ring prologue; C4 512^3: 0.92 ms at 256 tasks against 0.95 at 1024 (paired runs)
  // (profiles/r1_3d_grid_sweep.txt); never segments shorter than 8 planes
  static const int64_t target = [] {
    const char* e = getenv("PCS_3D_TARGET");  // diagnostics: grid-size sweep
    if (e && atoll(e) > 0) return (int64_t)atoll(e);
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
      cus = 256;
    (void)hipGetLastError();
    return (int64_t)cus;  // one 512-thread workgroup per CU
  }();
  // the segment count minimises the makespan: (rounds of `target` workgroups) x (segment length + the
  // two-plane prologue).  A plane of tiles that is not a multiple of the CU count otherwise leaves a
  // partial last round: C5 at 12-row fp64 tiles is 688 tiles per plane = 2.69 rounds of 1024 planes run
  // as 3; 7 segments of 147 planes run 19 rounds of 147 (2793 plane-times against 3072)
  const int64_t max_seg = (L + 7) / 8;
  int64_t lo = (target + per_plane - 1) / per_plane;
  lo = lo > max_seg ? max_seg : lo;
  lo = lo < bands ? bands : lo;
  lo = lo < 1 ? 1 : lo;
  int64_t nseg = lo, best = -1;
  for (int64_t ns = lo; ns <= max_seg && ns <= lo + 15; ++ns) {
    const int64_t sl = (L + ns - 1) / ns;
    const int64_t tasks = per_plane * ((L0 + sl - 1) / sl + (L1 + sl - 1) / sl);
    const int64_t cost = (tasks + target - 1) / target * (sl + 2);
    if (best < 0 || cost < best) best = cost, nseg = ns;
  }
  static const int64_t force_seg = [] {
    const char* e = getenv("PCS_3D_NSEG");  // diagnostics: segment-count sweep
    return e ? (int64_t)atoll(e) : (int64_t)0;
  }();
  if (force_seg > 0) nseg = force_seg < bands ? bands : force_seg > max_seg ? max_seg : force_seg;
  const int64_t seg_len = (L + nseg - 1) / nseg;
  const int64_t n0 = seg_len ? (L0 + seg_len - 1) / seg_len : 0, n1 = seg_len ? (L1 + seg_len - 1) / seg_len : 0;
  p.bd = Bands{(int)seg_len, (int)n0, (int)pb.a0, (int)pb.b0, (int)pb.a1, (int)pb.b1};
  p.ntasks = (int)(per_plane * (n0 + n1));
  return p;
}
static PlaneBands full3(const pcs_pds3d_args* a) { return PlaneBands{0, a->planes, a->planes, a->planes}; }

static bool aligned16_3(const void* q) { return q == nullptr || ((uintptr_t)q & 15) == 0; }

template <typename T, int FK, bool VEC>
static int launch3(const pcs_pds3d_args* a, PlaneBands pb, hipStream_t st) {
  const Plan3 p = plan3(a, pb);
  if (p.ntasks == 0) return PCS_OK;
  Vol v;
  v.n0 = (int)a->n0;
  v.n1 = (int)a->n1;
  v.n2 = (int)a->n2;
  v.plane0 = (int)a->plane0;
  v.planes = (int)a->planes;
  v.hx = a->halo_x;
  v.hz = a->halo_z;
  v.hg = a->halo_g;
  v.pitch1 = (uint32_t)(a->n2 * sizeof(T));
  v.plane_bytes = (uint32_t)(a->n1 * a->n2 * sizeof(T));
  P3<T> P;
  P.tau = (T)a->tau;
  P.sigma = (T)a->sigma;
  P.inv_sigma = (T)(1.0 / a->sigma);
  P.rho = (T)a->rho;
  P.omr = (T)(1.0 - a->rho);
  const double t_h = (1.0 / a->sigma) * a->lam;  // ProxFuncPostComp: tau*scale with tau = 1/sigma
  P.t_h = (T)t_h;
  P.inv_t_h = (T)(1.0 / t_h);
  const double steps[3] = {a->step0, a->step1, a->step2};
  for (int k = 0; k < 3; ++k) {
    P.inv_step[k] = (T)(1.0 / steps[k]);
    P.unit[k] = steps[k] == 1.0;
  }
  P.seg_a = (T)a->seg_a;
  P.seg_b = (T)a->seg_b;
  if constexpr (FK != PCS_F_CONV0) {
    if (a->kkind == PCS_BACKWARD || a->kkind == PCS_CENTERED) {
      auto kern =
          a->kkind == PCS_BACKWARD ? k_pds3d_gen<T, PCS_BACKWARD, FK, VEC> : k_pds3d_gen<T, PCS_CENTERED, FK, VEC>;
      kern<<<(unsigned)p.ntasks, k3g_nt<T>(), 0, st>>>((const T*)a->x, (T*)a->xn, (const T*)a->z, (T*)a->zn, (const T*)a->g,
                                                 v, P, a->hkind, a->gkind, a->edge, a->partials, (Ctrl*)a->ctrl,
                                                 a->hist, a->ws, p.tiles1, p.tiles2, p.bd, p.ntasks);
      return launch_status();
    }
  }
  k_pds3d<T, FK, VEC><<<(unsigned)p.ntasks, FK == PCS_F_CONV0 ? 2 * K3<T>::NT : K3<T>::NT, 0, st>>>(
      (const T*)a->x, (T*)a->xn, (const T*)a->z, (T*)a->zn, (const T*)a->g, v, P, a->hkind, a->gkind, a->partials,
      (Ctrl*)a->ctrl, a->hist, a->ws, p.tiles1, p.tiles2, p.bd, p.ntasks, (const T*)a->conv0_w,
      (const T*)a->conv0_taps, a->conv0_k, a->conv0_off);
  return launch_status();
}

template <typename T, bool VEC>
static int pds3d_v(const pcs_pds3d_args* a, PlaneBands pb, hipStream_t st) {
  switch (a->fkind) {
    case PCS_F_NULL: return launch3<T, PCS_F_NULL, VEC>(a, pb, st);
    case PCS_F_DENOISE: return launch3<T, PCS_F_DENOISE, VEC>(a, pb, st);
    case PCS_F_GRADBUF: return launch3<T, PCS_F_GRADBUF, VEC>(a, pb, st);
    case PCS_F_CONV0:
      if constexpr (std::is_same<T, float>::value) return launch3<T, PCS_F_CONV0, VEC>(a, pb, st);
      return PCS_EUNSUPPORTED;
    default: return PCS_EINVAL;
  }
}

template <typename T>
static int pds3d(const pcs_pds3d_args* a, PlaneBands pb, hipStream_t st) {
  const bool vec = a->n2 % 4 == 0 && aligned16_3(a->x) && aligned16_3(a->xn) && aligned16_3(a->z) &&
                   aligned16_3(a->zn) && aligned16_3(a->g) && aligned16_3(a->conv0_w);
  return vec ? pds3d_v<T, true>(a, pb, st) : pds3d_v<T, false>(a, pb, st);
}

}  // namespace pcs

using namespace pcs;

extern "C" {

int64_t pcs_pds3d_nblocks(const pcs_pds3d_args* a) {
  if (!a || a->planes < 1 || a->n1 < 1 || a->n2 < 1) return -1;
  return plan3(a, full3(a)).ntasks;
}

int64_t pcs_pds3d_ws_bytes(const pcs_pds3d_args* a) {
  const int64_t nb = pcs_pds3d_nblocks(a);
  return nb < 0 ? -1 : red_ws_bytes(nb);
}

static int check3(const pcs_pds3d_args* a) {
  if (!a || !a->x || !a->xn || !a->z || !a->zn || !a->partials) return PCS_EINVAL;
  if (a->n0 < 1 || a->n1 < 1 || a->n2 < 1 || a->planes < 1 || a->plane0 < 0 || a->plane0 + a->planes > a->n0)
    return PCS_EINVAL;
  if (a->hkind != PCS_H_L1 && a->hkind != PCS_H_L21) return PCS_EINVAL;
  if (a->gkind < PCS_G_NULL || a->gkind > PCS_G_SEGMENT) return PCS_EINVAL;
  if (!(a->sigma > 0) || !(a->step0 != 0) || !(a->step1 != 0) || !(a->step2 != 0)) return PCS_EINVAL;
  if ((a->fkind == PCS_F_DENOISE || a->fkind == PCS_F_GRADBUF) && !a->g) return PCS_EINVAL;
  if (a->halo_x < 0 || a->halo_z < 0 || a->halo_g < 0) return PCS_EINVAL;
  if (a->kkind != PCS_FORWARD && a->kkind != PCS_BACKWARD && a->kkind != PCS_CENTERED) return PCS_EINVAL;
  const bool multi = a->planes < a->n0;
  if (multi && (a->halo_x < 1 || a->halo_z < 1 || (a->fkind != PCS_F_NULL && a->halo_g < 1))) return PCS_EINVAL;
  // backward / centred K: K^T z reads z0 one plane past u's planes [-1, planes] on both sides
  if (multi && a->kkind != PCS_FORWARD && a->halo_z < 2) return PCS_EINVAL;
  const int64_t esz = a->dtype == PCS_F64 ? 8 : 4;
  if (a->n1 * a->n2 * esz > (1LL << 30) || a->n0 >= (1LL << 30)) return PCS_EUNSUPPORTED;  // one plane <= 1 GiB
  if (a->hist && (!a->ws || !a->ctrl || !aligned16_3(a->ws) || !aligned16_3(a->partials))) return PCS_EINVAL;
  if (a->dtype != PCS_F32 && a->dtype != PCS_F64) return PCS_EINVAL;
  if (a->fkind == PCS_F_CONV0) {  // the axis-0 pass inside the forward-K update (fp32)
    if (!a->g || !a->conv0_w || !a->conv0_taps || a->conv0_k < 1 || a->conv0_k > k3C0K || a->conv0_off < 0 ||
        a->conv0_off >= a->conv0_k)
      return PCS_EINVAL;
    if (multi && a->halo_g < a->conv0_k) return PCS_EINVAL;  // t planes [-(k - 1), planes + k - 1]
    if (a->kkind != PCS_FORWARD || a->dtype != PCS_F32) return PCS_EUNSUPPORTED;
  }
  return PCS_OK;
}

static int step3(const pcs_pds3d_args* a, PlaneBands pb, hipStream_t st) {
  return a->dtype == PCS_F32 ? pds3d<float>(a, pb, st) : pds3d<double>(a, pb, st);
}

static bool bands3_ok(const pcs_pds3d_args* a, int64_t a0, int64_t b0, int64_t a1, int64_t b1) {
  return 0 <= a0 && a0 <= b0 && b0 <= a1 && a1 <= b1 && b1 <= a->planes;
}

int pcs_pds3d_step(const pcs_pds3d_args* a, hipStream_t st) {
  const int rc = check3(a);
  return rc != PCS_OK ? rc : step3(a, full3(a), st);
}

int64_t pcs_pds3d_nblocks_bands(const pcs_pds3d_args* a, int64_t a0, int64_t b0, int64_t a1, int64_t b1) {
  if (check3(a) != PCS_OK || !bands3_ok(a, a0, b0, a1, b1)) return -1;
  return plan3(a, PlaneBands{a0, b0, a1, b1}).ntasks;
}

int pcs_pds3d_step_bands(const pcs_pds3d_args* a, int64_t a0, int64_t b0, int64_t a1, int64_t b1, hipStream_t st) {
  const int rc = check3(a);
  if (rc != PCS_OK) return rc;
  if (a->hist || !bands3_ok(a, a0, b0, a1, b1)) return PCS_EINVAL;
  return step3(a, PlaneBands{a0, b0, a1, b1}, st);
}



}  // extern "C"
