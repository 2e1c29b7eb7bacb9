// In-plane normal operator of a separable 3-D blur, every plane in one pass:
//
//   out = C_a^T C_b^T C_b C_a in        (C_a: Convolve1D along axis 1, C_b: along axis 2)
//
// i.e. the in-plane half of grad F = C^T (C x - y) for the reference's 3-D deconvolution
// (pycsou/linop/conv.py:20-164 per axis; residual and adjoint of core/map.py:609-610).  The
// axis-0 pass commutes with the in-plane ones, so the 3-D engine computes
//   g = C_0^T (C_0 (C_12^T C_12 x) - C_12^T y)
// with C_12^T y formed once at setup: two sub-volume passes per iteration (this kernel, then
// pcs_conv0_residual_adjoint) instead of three, 5 words per voxel of traffic instead of 7.
//
// Four 15-tap passes per plane, marched down a 128-column strip 32 rows per step:
//   P1  horizontal conv  (staging  -> ring A, 144 columns: the strip + the reach of P4)
//   P2  vertical conv    (ring A   -> ring B, rows outside the image forced to 0)
//   P3  vertical corr    (ring B   -> P3 rows, aliasing the staging buffer)
//   P4  horizontal corr  (P3 rows  -> HBM, the strip's 128 columns)
// Rings hold 48 rows (the 14-row reach of the vertical passes above a step), so no row is
// filtered twice; a strip's horizontal halo (16 columns) is recomputed by P1-P3 (1.125x).
// Zero boundary: input outside the plane reads 0, and P1 / P2 outputs outside the plane
// are 0 (the truncation between C and C^T).  Taps are zero-padded to 15 (out[j] =
// sum_t h'[t] in[j + o - t], h'[t] = h[t - pad], o = off + pad); the adjoint passes use
// h'[14 - t] with offset 14 - o.  Persistent grid, tasks (plane, row segment, strip) with the
// strip fastest and an XCD-aware task map, as k_sep2d_march.
#include <cstring>
#include <type_traits>

#include "vecio.hpp"

namespace pcs {

struct AtaG {
  static constexpr int KT = 15, TX = 128, GX = TX / 4, GE = GX + 4, WE = 4 * GE, GI = GE + 4, WI = 4 * GI;
  static constexpr int RS = 32, RING = 48, NT = 576;
  static constexpr int NIN = RS * GI, NL = (NIN + NT - 1) / NT;  // staging loads per thread
  static constexpr int NP1 = RS * GE, NP4 = RS * GX;             // P1 / P4 items
  static_assert((RS / 2) * GE == NT, "at most one vertical item (2 or 4 rows x 4 columns) per thread");
  static_assert(RING >= RS + KT - 1, "ring holds the 14 rows above a step");
};


#ifndef PCS_ATA_RB
#define PCS_ATA_RB 2
#endif
#ifndef PCS_ATA_HREG
#define PCS_ATA_HREG 0
#endif

// one vertical 15-tap pass over a ring of rows: acc[r] = sum_t h(t) ring[(base + r0 + r - t) mod RING]
// at 4-column group q, h(t) = hv[t] (conv) or hv[14 - t] (FLIP: correlation); each of the RB + 14
// ring rows is read once
template <typename T, int RB, bool FLIP>
__device__ __forceinline__ void vert_pass(const T* ring, int base, int r0, int q, const T* hv, Q4<T> (&acc)[RB]) {
  using A = AtaG;
  constexpr int KT = A::KT, RING = A::RING, WE = A::WE;
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[r].v[m] = T(0);
#pragma unroll 2
  for (int j = 0; j < KT - 1 + RB; ++j) {  // ring rows base + r0 - 14 + j
    int slot = base + r0 - (KT - 1) + j;
    slot = slot < 0 ? slot + RING : (slot >= RING ? slot - RING : slot);
    const Q4<T> v = ldsq(ring + slot * WE + 4 * q);
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int t = r + KT - 1 - j;
      if (t >= 0 && t < KT) {
        const T h = FLIP ? hv[KT - 1 - t] : hv[t];
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[r].v[m] += h * v.v[m];
      }
    }
  }
}

template <typename T, int SH4>
__global__ __launch_bounds__(AtaG::NT) void k_sep2d_ata(const T* __restrict__ in, T* __restrict__ out, int n1, int n2,
                                                         int nstrips, int nseg, int seg_len, int64_t ntasks,
                                                         const T* __restrict__ ha_, int ka, const T* __restrict__ hb_,
                                                         int kb, int o1, int padb, int o2) {
  using A = AtaG;
  constexpr int KT = A::KT, TX = A::TX, GE = A::GE, WE = A::WE, WI = A::WI, GI = A::GI, RS = A::RS, RING = A::RING,
                NT = A::NT, NL = A::NL;
  constexpr int SH1 = 2 - SH4;  // P1's window shift: the staged input starts 16 columns left of the strip
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  T* stg = reinterpret_cast<T*>(smem_raw);  // RS x WI input rows; P3 rows (RS x WE) after P1
  T* ringA = stg + RS * WI;                 // RING x WE
  T* ringB = ringA + RING * WE;             // RING x WE
  // taps in LDS (broadcast reads, re-read per phase): 30 fp64 taps in registers spill at the
  // 168-VGPR budget of 9 waves per workgroup.  hv: [0, 15), hh: [16, 31)
  T* hv = ringB + RING * WE;
  T* hh = hv + 16;
  if (threadIdx.x < 16) {
    const int t = threadIdx.x;
    hv[t] = t < ka ? ha_[t] : T(0);
    hh[t] = (t >= padb && t - padb < kb) ? hb_[t - padb] : T(0);
  }
#if PCS_ATA_HREG
  T hreg[KT];  // horizontal taps in registers (P1 / P4 read each once per 4 outputs)
#pragma unroll
  for (int t = 0; t < KT; ++t) hreg[t] = (t >= padb && t - padb < kb) ? hb_[t - padb] : T(0);
#define PCS_HH(t) hreg[t]
#else
#define PCS_HH(t) hh[t]
#endif
  int64_t t0, t_end, t_stride;
  {  // XCD x owns a contiguous share of the task list; its blocks take consecutive tasks
    const int64_t b = blockIdx.x, nb = gridDim.x, xcd = b % 8, k = b / 8, q = nb / 8, r = nb % 8;
    const int64_t nbx = q + (xcd < r ? 1 : 0);
    const int64_t before = xcd * q + (xcd < r ? xcd : r);
    const int64_t lo = ntasks * before / nb, hi = ntasks * (before + nbx) / nb;
    t0 = lo + k;
    t_end = hi;
    t_stride = nbx;
  }
  if (t0 >= t_end) return;
  const int tid = threadIdx.x;
  struct Cur {
    int64_t t, plane;
    int strip, a, b, s, ns;
  };
  auto task_at = [&](int64_t t) {
    Cur c;
    c.t = t;
    const int64_t per_plane = (int64_t)nseg * nstrips;
    c.plane = t / per_plane;
    const int rem = (int)(t - c.plane * per_plane), seg = rem / nstrips;
    c.strip = rem - seg * nstrips;
    c.a = seg * seg_len;
    c.b = min(n1, c.a + seg_len);
    c.s = 0;
    c.ns = (c.b - c.a + 2 * (KT - 1) + RS - 1) / RS;
    return c;
  };
  Q4<T> q[NL];
  // staging rows of step c: input rows L1 + s RS + r (L1 = a - 14), columns c0 - 16 + 4 g
  auto prefetch = [&](const Cur& c) {
    const T* src = in + c.plane * (int64_t)n1 * n2;
    const int kmax = c.b - c.a + 2 * (KT - 1) - 1;  // last staged row any output of [a, b) needs
    const int gc0 = c.strip * TX - 16;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int e = min(l * NT + tid, A::NIN - 1);
      const int rr = e / GI, g = e - rr * GI;
      const int k = c.s * RS + rr, gi = c.a - (KT - 1) + k, gc = gc0 + 4 * g;
      const bool ok = gi >= 0 && gi < n1 && k <= kmax && gc >= 0 && gc + 4 <= n2;
      const Q4<T> v = ldq(src + (ok ? (int64_t)gi * n2 + gc : 0));
#pragma unroll
      for (int m = 0; m < 4; ++m) q[l].v[m] = ok ? v.v[m] : T(0);
    }
  };
  Cur cur = task_at(t0);
  prefetch(cur);
  constexpr int RB = PCS_ATA_RB, NV = (RS / RB) * GE;  // vertical items: RB rows x one 4-column group
  const int vrb = tid / GE, vq = tid - (tid / GE) * GE;  // vertical item: rows RB vrb .. + RB - 1; group vq
  for (;;) {
    lds_barrier();  // the previous step's P4 is done with the P3 rows (staging)
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int e = l * NT + tid;
      if (e < A::NIN) stq(stg + 4 * e, q[l]);
    }
    Cur nxt = cur;
    bool more = true;
    if (cur.s + 1 < cur.ns) {
      nxt.s = cur.s + 1;
    } else {
      more = cur.t + t_stride < t_end;
      if (more) nxt = task_at(cur.t + t_stride);
    }
    if (more) prefetch(nxt);
    const int c0 = cur.strip * TX;
    const int e0 = c0 - o2 - SH4;  // first P1 column (E0, a multiple of 4); E0 + WE covers P4's reach
    const int base = (cur.s * RS) % RING;  // ring slot of the step's first row
    lds_barrier();
    // ---- P1: horizontal conv of the RS staged rows, columns [E0, E0 + WE) -> ring A
#pragma unroll 1
    for (int l = 0; l < (A::NP1 + NT - 1) / NT; ++l) {
      const int e = l * NT + tid;
      if (e < A::NP1) {
        const int r = e / GE, g = e - r * GE;
        T w[20];
#pragma unroll
        for (int u = 0; u < 5; ++u) {
          const Q4<T> v = ldsq(stg + r * WI + 4 * (g + u));
#pragma unroll
          for (int m = 0; m < 4; ++m) w[4 * u + m] = v.v[m];
        }
        Q4<T> o;
        const int col = e0 + 4 * g;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          T acc = T(0);
#pragma unroll
          for (int t = 0; t < KT; ++t) acc += PCS_HH(t) * w[SH1 + m + (KT - 1 - t)];
          o.v[m] = (unsigned)(col + m) < (unsigned)n2 ? acc : T(0);
        }
        int slot = base + r;
        slot = slot >= RING ? slot - RING : slot;
        stq(ringA + slot * WE + 4 * g, o);
      }
    }
    lds_barrier();
    // ---- P2: vertical conv, P2 row (rel. L1 - o1) s RS + r reads ring A rows s RS + r - t
    if (tid < NV) {
      Q4<T> acc[RB];
      vert_pass<T, RB, false>(ringA, base, RB * vrb, vq, hv, acc);
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int row = cur.a - (KT - 1) - o1 + cur.s * RS + RB * vrb + r;  // image row of this P2 output
        if ((unsigned)row >= (unsigned)n1) {
#pragma unroll
          for (int m = 0; m < 4; ++m) acc[r].v[m] = T(0);
        }
        int slot = base + RB * vrb + r;
        slot = slot >= RING ? slot - RING : slot;
        stq(ringB + slot * WE + 4 * vq, acc[r]);
      }
    }
    lds_barrier();
    // ---- P3: vertical correlation (taps hv[14 - t], offset 14 - o1): P3 row s RS + r (rel.
    // a - 28) reads ring B rows s RS + r - t -> P3 rows in the staging buffer (pitch WE)
    if (tid < NV) {
      Q4<T> acc[RB];
      vert_pass<T, RB, true>(ringB, base, RB * vrb, vq, hv, acc);
#pragma unroll
      for (int r = 0; r < RB; ++r) stq(stg + (RB * vrb + r) * WE + 4 * vq, acc[r]);
    }
    lds_barrier();
    // ---- P4: horizontal correlation (taps hh[14 - t], offset 14 - o2) -> output row
    // a - 28 + s RS + r, columns c0 + 4 g .. + 3
    {
      T* dst = out + cur.plane * (int64_t)n1 * n2;
#pragma unroll 1
      for (int l = 0; l < (A::NP4 + NT - 1) / NT; ++l) {
        const int e = l * NT + tid;
        if (e < A::NP4) {
          const int r = e / A::GX, g = e - r * A::GX;
          const int row = cur.a - 2 * (KT - 1) + cur.s * RS + r, gc = c0 + 4 * g;
          T w[20];
#pragma unroll
          for (int u = 0; u < 5; ++u) {
            const Q4<T> v = ldsq(stg + r * WE + 4 * (g + u));
#pragma unroll
            for (int m = 0; m < 4; ++m) w[4 * u + m] = v.v[m];
          }
          Q4<T> o;
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            T acc = T(0);
#pragma unroll
            for (int s = 0; s < KT; ++s) acc += PCS_HH(s) * w[SH4 + m + s];
            o.v[m] = acc;
          }
          if (row >= cur.a && row < cur.b && gc < n2) stq(dst + (int64_t)row * n2 + gc, o);
        }
      }
    }
    if (!more) break;
    cur = nxt;
  }
#undef PCS_HH
}

template <typename T>
static size_t ata_lds_bytes() {
  using A = AtaG;
  return sizeof(T) * (size_t)(A::RS * A::WI + 2 * A::RING * A::WE + 32);
}

// the kernel's LDS (> 64 KB) is dynamic: raise the function's limit once per instantiation
template <typename T, int SH4>
static void ata_attr() {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sep2d_ata<T, SH4>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)ata_lds_bytes<T>());
    (void)hipGetLastError();
    done = true;
  }
}

// resident workgroups of k_sep2d_ata<T> on the device (queried once per type)
template <typename T>
static int ata_slots() {
  static int slots = 0;
  if (slots == 0) {
    int dev = 0, cus = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || cus < 1)
      cus = 256;
    const size_t lds = ata_lds_bytes<T>();
    ata_attr<T, 1>();
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_sep2d_ata<T, 1>, AtaG::NT, lds) != hipSuccess || nb < 1)
      nb = 1;
    (void)hipGetLastError();
    slots = cus * nb;
    const char* e = getenv("PCS_ATA_SLOTS");  // diagnostics: grid-size sweep
    if (e && atoi(e) > 0) slots = atoi(e);
  }
  return slots;
}

// horizontal tap padding that makes both horizontal windows fit the strip layout: the padded
// offset o2 = offb + pad must satisfy o2 % 4 != 1 (SH4 = (-o2) mod 4 <= 2); -1 if none exists
static int ata_padb(int kb, int offb) {
  for (int pad = 0; pad <= AtaG::KT - kb; ++pad)
    if ((offb + pad) % 4 != 1) return pad;
  return -1;
}

// ---------------------------------------------------------------------------------------------
// The same operator as TWO 29-tap passes (the default when the taps reach <= 7 samples either
// side and the plane is >= 16 x 16): per axis C^T C is the autocorrelation of the taps,
//   (C^T C)[j, k] = a[j - k] - E[j][k],  a[e] = sum_m c(m) c(m + e),  c(d) = h[d + off],
// E the terms of the samples outside the plane (rows i < 0 / i >= n), nonzero only for j, k in
// the 7 samples nearest each edge (the zero boundary of the reference's Convolve1D, PyLops 1.x
// `Convolve1D` truncation between C and C^T).  A 128-column (fp32) / 64-column (fp64) strip
// marches down a row segment 32 rows per step:
//   PH  horizontal 29-tap pass of the 32 staged input rows (+ the left / right edge terms)
//       -> a ring of RS + 28 rows (each input row filtered once: no vertical halo recomputed)
//   PV  vertical 29-tap pass, RB rows x 4 columns per thread (RB + 28 ring reads per 4 RB
//       outputs) + the top / bottom edge terms -> HBM
// Two barriers per step; the next step's input rows are in flight (registers) during PH and PV.
// The tables (a for both axes, the four 7x7 edge blocks) are built per workgroup from the taps
// in fp64.  2 words of HBM traffic per voxel, like one k_sep2d_march pass, for the work of two.
// fp32 geometry (fp64 takes k_sep2d_nrmm below): 128-column strips, 32-row steps, PV items of 4 rows x
// 4 columns, PH items of 16 outputs (0.433-0.449 against 0.469 ms for 8 at 512^3, C4 642-645 against
// 633-635 it/s, profiles/r4_nrm_cfg6_ab.txt).  Measured without gain and removed in round 5: loads two
// steps ahead, packed-FMA PV, PH unroll, PV chunks of 2 / 8 rows, lane-rotated LDS writes
// (profiles/r4_nrm_var_ab*.txt, r4_nrm_swz_ab.txt)
struct NrmF {
  static constexpr int PQ = 4;  // PH item: 4 PQ outputs of one row
  static constexpr int TX = 128, RS = 32, RB = 4, RING = RS + 28, GX = TX / 4, GI = GX + 8;
  // the lanes of a b128 group read every fourth 16-B slot of rows r .. r + 3, so the staged rows take an
  // odd slot pitch (22.4 M bank-conflict cycles per 512^3 launch without it at 8 outputs,
  // profiles/r4_prof_nrm32_pmc_summary.txt)
  static constexpr int SPAD = 4, WI = 4 * GI + SPAD, TP = TX;
  static constexpr int NT = (RS / RB) * GX, NIN = RS * GI, NL = (NIN + NT - 1) / NT, NPH = RS * GX / PQ;
  static constexpr int NST = RB;  // 16-B stores per thread per step
  static constexpr int NTAB = 288;  // a_v[0..29), a_h[32..61), E_v lo / hi, E_h lo / hi (7 x 8 each)
  static_assert(NPH % NT == 0, "whole PH items per thread");
  static constexpr size_t lds_bytes() { return 4 * ((size_t)RS * WI + (size_t)RING * TP + NTAB); }
};

// compiler fences of the PV chunks: no LDS read or FMA moves across (bounds the registers held
// by hoisted window reads) ...
__device__ __forceinline__ void nrm_fence() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// ... and the chunk's FMAs stay before the fence (not sunk below the later reads)
template <typename T>
__device__ __forceinline__ void nrm_pin(Q4<T>& a) {
  asm volatile("" : "+v"(a.v[0]), "+v"(a.v[1]), "+v"(a.v[2]), "+v"(a.v[3]));
}

// 4 elements through a descriptor (16-B stores; an offset carrying kOOB is dropped)
template <typename T>
__device__ __forceinline__ void nrm_bstore(Rsrc r, uint32_t off, const Q4<T>& a) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  constexpr int VN = V16<T>::N;
#pragma unroll
  for (int h = 0; h < 4 / VN; ++h) {
    u4 d;
    __builtin_memcpy(&d, a.v + h * VN, 16);
    __builtin_amdgcn_raw_buffer_store_b128(d, r, (int)(off + 16 * h), 0, 0);
  }
}

// a += h w on 4 columns
template <typename T>
__device__ __forceinline__ void nrm_fma4(Q4<T>& a, T h, const Q4<T>& w) {
#pragma unroll
  for (int m = 0; m < 4; ++m) a.v[m] += h * w.v[m];
}

// tap d of a filter stored as h[0..k) with offset off (zero outside)
__device__ __forceinline__ double nrm_tap(const double* h, int k, int off, int d) {
  const int t = d + off;
  return (t >= 0 && t < k) ? h[t] : 0.0;
}

// 4 elements through a descriptor (16-B loads; an offset carrying kOOB reads 0)
template <typename T>
__device__ __forceinline__ Q4<T> nrm_bload(Rsrc r, uint32_t off) {
  constexpr int VN = V16<T>::N;
  Q4<T> a;
#pragma unroll
  for (int h = 0; h < 4 / VN; ++h) {
    const auto d = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(off + 16 * h), 0, 0);
    __builtin_memcpy(a.v + h * VN, &d, 16);
  }
  return a;
}

// SUB: out = C^T C in - sub (sub laid out as in / out; a 2-D step's grad F = N x - Conv^T y formed here, so
// the step reads one buffer instead of two -- the same subtraction, bit for bit).  fp32 (T = float): 53 KB of
// LDS, 3 workgroups / CU
template <typename T, bool SUB>
__global__ __launch_bounds__(NrmF::NT, 3) void k_sep2d_nrm(const T* __restrict__ in, T* __restrict__ out, int n1,
                                                                 int n2, int nstrips, int nseg, int seg_len,
                                                                 int64_t ntasks, const T* __restrict__ ha_, int ka,
                                                                 int offa, const T* __restrict__ hb_, int kb, int offb,
                                                                 const T* __restrict__ sub) {
  static_assert(sizeof(T) == 4, "fp32 (fp64: k_sep2d_nrmm)");
  using G = NrmF;
  constexpr int TX = G::TX, RS = G::RS, RB = G::RB, RING = G::RING, GX = G::GX, GI = G::GI, WI = G::WI, NT = G::NT,
                NL = G::NL, TP = G::TP;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  T* stg = reinterpret_cast<T*>(smem_raw);  // RS x WI staged input rows
  T* ring = stg + RS * WI;                  // RING rows (pitch TP) of the horizontal pass
  T* tab = ring + RING * TP;                // NTAB
  const int tid = threadIdx.x;
  {
    __shared__ double hs[32];  // the two filters in fp64
    if (tid < 16) hs[tid] = tid < ka ? (double)ha_[tid] : 0.0;
    else if (tid < 32) hs[tid] = tid - 16 < kb ? (double)hb_[tid - 16] : 0.0;
    __syncthreads();
    for (int e = tid; e < G::NTAB; e += NT) {
      double v = 0.0;
      if (e < 64) {
        const int q = e & 31;
        const double* h = e < 32 ? hs : hs + 16;
        const int k = e < 32 ? ka : kb, off = e < 32 ? offa : offb;
        if (q < 29)
          for (int m = -7; m <= 7; ++m) v += nrm_tap(h, k, off, m) * nrm_tap(h, k, off, m + q - 14);
      } else {
        const int idx = e - 64, tb = idx / 56, r = idx - 56 * tb, j = r >> 3, c = r & 7;
        const double* h = tb < 2 ? hs : hs + 16;
        const int k = tb < 2 ? ka : kb, off = tb < 2 ? offa : offb;
        if (c < 7) {
          if ((tb & 1) == 0)  // rows / columns i = -7..-1 before the plane: E[j][c], j, c < 7
            for (int i = -7; i < 0; ++i) v += nrm_tap(h, k, off, i - j) * nrm_tap(h, k, off, i - c);
          else  // after it: j = n - 7 + jj, c = n - 7 + cc, i = n + ii
            for (int ii = 0; ii < 7; ++ii) v += nrm_tap(h, k, off, 7 + ii - j) * nrm_tap(h, k, off, 7 + ii - c);
        }
      }
      tab[e] = (T)v;
    }
    __syncthreads();
  }
  // the autocorrelation is symmetric: window tap q is a[|q - 14|], 15 registers per axis
  T av[15], ah[15];
#pragma unroll
  for (int e = 0; e < 15; ++e) {
    av[e] = tab[14 + e];
    ah[e] = tab[32 + 14 + e];
  }
  const T* evl = tab + 64;
  const T* evh = tab + 120;
  const T* ehl = tab + 176;
  const T* ehh = tab + 232;
  int64_t t0, t_end, t_stride;
  {  // XCD x owns a contiguous share of the task list; its blocks take consecutive tasks
    const int64_t b = blockIdx.x, nb = gridDim.x, xcd = b % 8, k = b / 8, q = nb / 8, r = nb % 8;
    const int64_t nbx = q + (xcd < r ? 1 : 0);
    const int64_t before = xcd * q + (xcd < r ? xcd : r);
    const int64_t lo = ntasks * before / nb, hi = ntasks * (before + nbx) / nb;
    t0 = lo + k;
    t_end = hi;
    t_stride = nbx;
  }
  if (t0 >= t_end) return;
  struct Cur {
    int64_t t, plane;
    int strip, a, b, s, ns;
  };
  auto task_at = [&](int64_t t) {
    Cur c;
    c.t = t;
    const int64_t per_plane = (int64_t)nseg * nstrips;
    c.plane = t / per_plane;
    const int rem = (int)(t - c.plane * per_plane), seg = rem / nstrips;
    c.strip = rem - seg * nstrips;
    c.a = seg * seg_len;
    c.b = min(n1, c.a + seg_len);
    c.s = 0;
    c.ns = (c.b - c.a + 28 + RS - 1) / RS;
    return c;
  };
  // staged rows of step s: input rows a - 14 + s RS + rr, columns c0 - 16 + 4 gg (0 outside)
  auto prefetch = [&](const Cur& c, Q4<T>(&q)[NL]) {
    const T* src = in + c.plane * (int64_t)n1 * n2;
    const int kmax = c.b - c.a + 27;  // last staged row any output of [a, b) reads
    const int gc0 = c.strip * TX - 16;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int e = min(l * NT + tid, G::NIN - 1);
      const int rr = e / GI, gg = e - rr * GI;
      const int k = c.s * RS + rr, gi = c.a - 14 + k, gc = gc0 + 4 * gg;
      const bool ok = gi >= 0 && gi < n1 && k <= kmax && gc >= 0 && gc + 4 <= n2;
      const Q4<T> v = ldq(src + (ok ? (int64_t)gi * n2 + gc : 0));
#pragma unroll
      for (int m = 0; m < 4; ++m) q[l].v[m] = ok ? v.v[m] : T(0);
    }
  };
  // the staged rows have landed (WAITN: the memory ops issued after them that may stay in flight --
  // vector memory ops retire in order); rows -> LDS
  auto stage = [&](const Q4<T>(&q)[NL], auto waitn) {
    constexpr int WN = decltype(waitn)::value;
    __builtin_amdgcn_s_waitcnt((WN & 15) | ((WN >> 4) << 14) | (7 << 4) | (15 << 8));
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int e = l * NT + tid, rr = e / GI, gg = e - rr * GI;
      if (e < G::NIN) stq(stg + rr * WI + 4 * gg, q[l]);
    }
  };
  // one step on the staged rows of cur: PH into the ring, PV from it -> HBM
  auto body = [&](const Cur cur) {
    const int vi = tid / GX, vg = tid - vi * GX;  // PV item: rows RB vi .. + RB - 1 of the step, group vg
    const int c0 = cur.strip * TX;
    Q4<T> bsub[SUB ? RB : 1];  // SUB: the PV outputs' sub values, loaded before PH (a phase to land)
    if constexpr (SUB) {
      const Rsrc rs = rsrc_of(sub + cur.plane * (int64_t)n1 * n2, (uint32_t)((int64_t)n1 * n2 * sizeof(T)));
      const int gc = c0 + 4 * vg;
#pragma unroll
      for (int rr = 0; rr < RB; ++rr) {
        const int i = cur.a - 28 + cur.s * RS + RB * vi + rr;
        const bool live = i >= cur.a && i < cur.b && gc < n2;
        bsub[rr] = nrm_bload<T>(rs, live ? (uint32_t)(((int64_t)i * n2 + gc) * sizeof(T)) : kOOB);
      }
    }
    const int sb = (cur.s * RS) % RING;  // ring slot of the step's first staged row
    lds_barrier();
    // ---- PH: t[row][c0 + j] = sum_q a_h[q] x[row][c0 + j - 14 + q] (staged column j + 2 + q);
    // an item is 4 PQ consecutive outputs of one row (PQ + 8 window reads)
#pragma unroll 1
    for (int l = 0; l < G::NPH / NT; ++l) {
      constexpr int PQ = G::PQ, GQ = GX / PQ;
      const int e = l * NT + tid, r = e / GQ, g = PQ * (e - r * GQ);
      const T* srow = stg + r * WI;
      T acc[4 * PQ];
#pragma unroll
      for (int o = 0; o < 4 * PQ; ++o) acc[o] = T(0);
#pragma unroll
      for (int u = 0; u < PQ + 8; ++u) {
        const Q4<T> v = ldsq(srow + 4 * (g + u));
#pragma unroll
        for (int ee = 0; ee < 4; ++ee)
#pragma unroll
          for (int o = 0; o < 4 * PQ; ++o) {
            const int qq = 4 * u + ee - o - 2;
            if (qq >= 0 && qq < 29) acc[o] += ah[qq < 14 ? 14 - qq : qq - 14] * v.v[ee];
          }
      }
      const int col = c0 + 4 * g;
      if (col < 7 || col + 4 * PQ - 1 >= n2 - 7) {  // the edge terms of the first / last 7 columns
#pragma unroll
        for (int o = 0; o < 4 * PQ; ++o) {
          const int j = col + o;
          if (j < 7) {
            for (int c = 0; c < 7; ++c) acc[o] -= ehl[8 * j + c] * srow[16 + c];
          } else if (j >= n2 - 7 && j < n2) {
            const int jj = j - (n2 - 7), s0 = n2 - 7 - c0 + 16;
            for (int c = 0; c < 7; ++c) acc[o] -= ehh[8 * jj + c] * srow[s0 + c];
          }
        }
      }
      int slot = sb + r;
      slot = slot >= RING ? slot - RING : slot;
#pragma unroll
      for (int k = 0; k < PQ; ++k) {
        Q4<T> c;
#pragma unroll
        for (int m = 0; m < 4; ++m) c.v[m] = acc[4 * k + m];
        stq(ring + slot * TP + 4 * (g + k), c);
      }
    }
    lds_barrier();
    // ---- PV: out row i = a - 28 + s RS + r reads t rows i - 14 .. i + 14 (staged s RS + r - 28 ..)
    {
      const int r0 = RB * vi;
      const int base = (cur.s * RS + r0 - 28 + RING) % RING;
      Q4<T> acc[RB];
#pragma unroll
      for (int rr = 0; rr < RB; ++rr)
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[rr].v[m] = T(0);
      // RB + 28 window rows in chunks of CH, the next chunk's reads in flight during this one's FMAs
      // 4-row chunks: 0.543 against 0.565-0.573 ms for 8 (512^3 fp32, profiles/r2_nrm_ablation.txt)
      constexpr int NV = RB + 28, CH = 4, NCH = (NV + CH - 1) / CH;
      const T* rcol = ring + 4 * vg;
      // window row v sits at ring slot base + v, wrapped once at most: two bases (the second one ring
      // length back) and a per-row select, the row offset an immediate of the LDS read -- instead of
      // recomputing the wrapped slot and its address for every row (round 6)
      const T* rb0 = rcol + base * TP;
      const T* rb1 = rb0 - RING * TP;
      const int wrap = RING - base;  // the first window row past the ring's end
      Q4<T> w[2][CH];  // chunk c in w[c & 1] (static after unrolling: no register copies)
      auto rd = [&](int c, Q4<T>(&wc)[CH]) {
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          const int v = c * CH + j;
          if (v < NV) wc[j] = ldsq((v < wrap ? rb0 : rb1) + v * TP);
        }
      };
      rd(0, w[0]);
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if (c + 1 < NCH) rd(c + 1, w[(c + 1) & 1]);
        nrm_fence();
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          const int v = c * CH + j;
          if (v < NV) {
#pragma unroll
            for (int rr = 0; rr < RB; ++rr) {
              const int qq = v - rr;
              if (qq >= 0 && qq < 29) nrm_fma4(acc[rr], av[qq < 14 ? 14 - qq : qq - 14], w[c & 1][j]);
            }
          }
        }
#pragma unroll
        for (int rr = 0; rr < RB; ++rr) nrm_pin(acc[rr]);
        nrm_fence();
      }
      const int gc = c0 + 4 * vg;
      // every thread issues RB stores per step (rows outside [a, b) dropped by the range check),
      // so the next step's wait for its staged rows leaves these stores in flight
      const Rsrc dst = rsrc_of(out + cur.plane * (int64_t)n1 * n2, (uint32_t)((int64_t)n1 * n2 * sizeof(T)));
#pragma unroll
      for (int rr = 0; rr < RB; ++rr) {
        const int i = cur.a - 28 + cur.s * RS + r0 + rr;
        const bool live = i >= cur.a && i < cur.b && gc < n2;
        if (live) {
          if (i < 7 || i >= n1 - 7) {  // the edge terms of the first / last 7 rows
            const bool top = i < 7;
            const int jr = top ? i : i - (n1 - 7), row0 = top ? 0 : n1 - 7;
            const T* e = top ? evl : evh;
            for (int c = 0; c < 7; ++c) {
              const Q4<T> w = ldsq(ring + ((row0 + c - cur.a + 14) % RING) * TP + 4 * vg);
              const T ec = e[8 * jr + c];
#pragma unroll
              for (int m = 0; m < 4; ++m) acc[rr].v[m] -= ec * w.v[m];
            }
          }
        }
        if constexpr (SUB) {
#pragma unroll
          for (int m = 0; m < 4; ++m) acc[rr].v[m] = acc[rr].v[m] - bsub[rr].v[m];
        }
        nrm_bstore(dst, live ? (uint32_t)(((int64_t)i * n2 + gc) * sizeof(T)) : kOOB, acc[rr]);
      }
    }
  };
  Q4<T> q[NL];
  Cur cur = task_at(t0);
  prefetch(cur, q);
  for (;;) {
    // the previous step's RB row stores may still be in flight
    stage(q, std::integral_constant<int, G::NST>{});
    Cur nxt = cur;
    bool more = true;
    if (cur.s + 1 < cur.ns) {
      nxt.s = cur.s + 1;
    } else {
      more = cur.t + t_stride < t_end;
      if (more) nxt = task_at(cur.t + t_stride);
    }
    prefetch(nxt, q);  // unconditional (the last step re-reads its own rows): the wait for these
                    // loads at the next step then leaves this step's stores in flight
    body(cur);
    if (!more) break;
    cur = nxt;
  }
}

// ---------------------------------------------------------------------------------------------
// k_sep2d_nrmm: the same two 29-tap passes on a MIRRORED ring (round 5).  The vertical window of a PV
// item spans RB + 28 ring rows; with the ring's first RB + 27 rows duplicated past its end (PH writes
// those rows twice) every window is contiguous, so its reads are one base address plus immediate
// offsets -- the old kernel recomputed a wrapped slot and its row offset for each of the 30 window rows
// (about 7 VALU per row pair, 227 VALU beside 232 FMAs in the fp64 PV block).  PV items are RB = 4 rows x
// one 16-B chunk (4 floats / 2 doubles): RB + 28 = 32 b128 reads per 4 x VN outputs (fp64: 4 reads per
// output instead of 7.5).  LDS layouts, all conflict-free in the lane-group model of MI355X_MICROARCH.md
// (ds_read_b128: 16-lane groups, 64 banks; ds_write_b128: 8-lane groups, 32 banks):
//   staged rows  pitch WI = the row's 4-column groups + 4 16-B slots, row r shifted by (r & 3) slots;
//                staging items in row-major order (fp32) / 8-lane groups of 4 groups x 2 rows (fp64)
//   PH items     lane l of wave w: row 8 w + (l & 7), item (l >> 3) & 7 of the row's 8 (4 PQ outputs, 4
//                chunks each): the 8 lanes of a write group hold 8 rows of one item column
//   ring         pitch TP = TX + one 16-B slot (an odd number of slots: those 8 rows hit 8 banks)
//   PV items     the 32 lanes of a half-wave read 32 consecutive chunks of one ring row
// one 16-B chunk from LDS as a single ds_read_b128 (volatile LDS access, as ldsq)
template <typename T>
__device__ __forceinline__ V16<T> nrm_ldsv(const T* p) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) const volatile u4* lds_u4;
  V16<T> r;
  const u4 v = *((lds_u4)(p));
  __builtin_memcpy(r.v, &v, 16);
  return r;
}

template <typename T>
struct NrmM {
  static constexpr int ES = sizeof(T), VN = 16 / ES;
  static constexpr int TX = ES == 4 ? 128 : 64, PQ = ES == 4 ? 4 : 2;  // 8 PH items of 4 chunks per row
  static constexpr int RS = 32, RB = 4, RING = RS + 28, MIR = RB + 27;
  static constexpr int GX = TX / 4, GI = GX + 8, GQ = GX / PQ, GV = TX / VN;
  static constexpr int NT = (RS / RB) * GV;
  static constexpr int WI = 4 * GI + 4 * VN;  // staged pitch (elements): the groups + 4 slots of shift room
  static constexpr int TP = TX + VN;          // ring pitch
  static constexpr int NIN = RS * GI, NL = (NIN + NT - 1) / NT;
  static constexpr int NTAB = 288;
  static_assert(GQ == 8 && NT == 256 && RS * GQ == NT && GI % 4 == 0, "one PH item per thread");
  static constexpr size_t lds_bytes() { return ES * ((size_t)RS * WI + (size_t)(RING + MIR) * TP + NTAB); }
  // staging item e -> staged row / 4-column group
  static __device__ __forceinline__ void stage_item(int e, int& rr, int& gg) {
    if constexpr (ES == 4) {
      rr = e / GI;
      gg = e - rr * GI;
    } else {
      const int e8 = e & 7, eh = e >> 3, q = eh / (GI / 4);
      rr = 2 * q + (e8 >> 2);
      gg = 4 * (eh - q * (GI / 4)) + (e8 & 3);
    }
  }
  static __device__ __forceinline__ int srow(int r) { return r * WI + (r & 3) * VN; }
};

template <typename T, bool SUB>
__global__ __launch_bounds__(256, 2) void k_sep2d_nrmm(const T* __restrict__ in, T* __restrict__ out, int n1, int n2,
                                                       int nstrips, int nseg, int seg_len, int64_t ntasks,
                                                       const T* __restrict__ ha_, int ka, int offa,
                                                       const T* __restrict__ hb_, int kb, int offb,
                                                       const T* __restrict__ sub) {
  using G = NrmM<T>;
  constexpr int TX = G::TX, RS = G::RS, RB = G::RB, RING = G::RING, GV = G::GV, VN = G::VN, NT = G::NT,
                NL = G::NL, TP = G::TP, PQ = G::PQ;
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  T* stg = reinterpret_cast<T*>(smem_raw);  // RS staged input rows (pitch WI, shifted)
  T* ring = stg + RS * G::WI;               // RING + MIR rows of the horizontal pass (pitch TP)
  T* tab = ring + (RING + G::MIR) * TP;     // NTAB
  const int tid = threadIdx.x;
  {
    __shared__ double hs[32];  // the two filters in fp64
    if (tid < 16) hs[tid] = tid < ka ? (double)ha_[tid] : 0.0;
    else if (tid < 32) hs[tid] = tid - 16 < kb ? (double)hb_[tid - 16] : 0.0;
    __syncthreads();
    for (int e = tid; e < G::NTAB; e += NT) {
      double v = 0.0;
      if (e < 64) {
        const int q = e & 31;
        const double* h = e < 32 ? hs : hs + 16;
        const int k = e < 32 ? ka : kb, off = e < 32 ? offa : offb;
        if (q < 29)
          for (int m = -7; m <= 7; ++m) v += nrm_tap(h, k, off, m) * nrm_tap(h, k, off, m + q - 14);
      } else {
        const int idx = e - 64, tb = idx / 56, r = idx - 56 * tb, j = r >> 3, c = r & 7;
        const double* h = tb < 2 ? hs : hs + 16;
        const int k = tb < 2 ? ka : kb, off = tb < 2 ? offa : offb;
        if (c < 7) {
          if ((tb & 1) == 0)  // rows / columns i = -7..-1 before the plane: E[j][c], j, c < 7
            for (int i = -7; i < 0; ++i) v += nrm_tap(h, k, off, i - j) * nrm_tap(h, k, off, i - c);
          else  // after it: j = n - 7 + jj, c = n - 7 + cc, i = n + ii
            for (int ii = 0; ii < 7; ++ii) v += nrm_tap(h, k, off, 7 + ii - j) * nrm_tap(h, k, off, 7 + ii - c);
        }
      }
      tab[e] = (T)v;
    }
    __syncthreads();
  }
  // the autocorrelation is symmetric: window tap q is a[|q - 14|], 15 registers per axis
  T av[15], ah[15];
#pragma unroll
  for (int e = 0; e < 15; ++e) {
    av[e] = tab[14 + e];
    ah[e] = tab[32 + 14 + e];
  }
  const T* evl = tab + 64;
  const T* evh = tab + 120;
  const T* ehl = tab + 176;
  const T* ehh = tab + 232;
  int64_t t0, t_end, t_stride;
  {  // XCD x owns a contiguous share of the task list; its blocks take consecutive tasks
    const int64_t b = blockIdx.x, nb = gridDim.x, xcd = b % 8, k = b / 8, q = nb / 8, r = nb % 8;
    const int64_t nbx = q + (xcd < r ? 1 : 0);
    const int64_t before = xcd * q + (xcd < r ? xcd : r);
    const int64_t lo = ntasks * before / nb, hi = ntasks * (before + nbx) / nb;
    t0 = lo + k;
    t_end = hi;
    t_stride = nbx;
  }
  if (t0 >= t_end) return;
  struct Cur {
    int64_t t, plane;
    int strip, a, b, s, ns;
  };
  auto task_at = [&](int64_t t) {
    Cur c;
    c.t = t;
    const int64_t per_plane = (int64_t)nseg * nstrips;
    c.plane = t / per_plane;
    const int rem = (int)(t - c.plane * per_plane), seg = rem / nstrips;
    c.strip = rem - seg * nstrips;
    c.a = seg * seg_len;
    c.b = min(n1, c.a + seg_len);
    c.s = 0;
    c.ns = (c.b - c.a + 28 + RS - 1) / RS;
    return c;
  };
  // this thread's staging items (fixed): staged row / group and their LDS offsets
  int st_rr[NL], st_gg[NL], st_off[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    G::stage_item(min(l * NT + tid, G::NIN - 1), st_rr[l], st_gg[l]);
    st_off[l] = G::srow(st_rr[l]) + 4 * st_gg[l];
  }
  // staged rows of step s: input rows a - 14 + s RS + rr, columns c0 - 16 + 4 gg (0 outside)
  auto prefetch = [&](const Cur& c, Q4<T>(&q)[NL]) {
    const T* src = in + c.plane * (int64_t)n1 * n2;
    const int kmax = c.b - c.a + 27;  // last staged row any output of [a, b) reads
    const int gc0 = c.strip * TX - 16;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int k = c.s * RS + st_rr[l], gi = c.a - 14 + k, gc = gc0 + 4 * st_gg[l];
      const bool ok = gi >= 0 && gi < n1 && k <= kmax && gc >= 0 && gc + 4 <= n2;
      const Q4<T> v = ldq(src + (ok ? (int64_t)gi * n2 + gc : 0));
#pragma unroll
      for (int m = 0; m < 4; ++m) q[l].v[m] = ok ? v.v[m] : T(0);
    }
  };
  // the staged rows have landed (WN: the memory ops issued after them that may stay in flight --
  // vector memory ops retire in order); rows -> LDS
  auto stage = [&](const Q4<T>(&q)[NL], auto waitn) {
    constexpr int WN = decltype(waitn)::value;
    __builtin_amdgcn_s_waitcnt((WN & 15) | ((WN >> 4) << 14) | (7 << 4) | (15 << 8));
#pragma unroll
    for (int l = 0; l < NL; ++l)
      if (l * NT + tid < G::NIN) stq(stg + st_off[l], q[l]);
  };
  // PH item: row pr, outputs 4 PQ pg .. + 4 PQ - 1 of the strip
  const int pr = ((tid >> 6) << 3) | (tid & 7), pg = PQ * ((tid >> 3) & 7);
  const T* psrow = stg + G::srow(pr);
  // PV item: rows RB vi .. + RB - 1 of the step, chunk vg (columns VN vg .. VN vg + VN - 1)
  const int vi = tid / GV, vg = tid - vi * GV, r0 = RB * vi;
  auto body = [&](const Cur cur) {
    const int c0 = cur.strip * TX;
    const int gc = c0 + VN * vg;
    V16<T> bsub[SUB ? RB : 1];  // SUB: the PV outputs' sub values, loaded before PH (a phase to land)
    if constexpr (SUB) {
      const Rsrc rs = rsrc_of(sub + cur.plane * (int64_t)n1 * n2, (uint32_t)((int64_t)n1 * n2 * sizeof(T)));
#pragma unroll
      for (int rr = 0; rr < RB; ++rr) {
        const int i = cur.a - 28 + cur.s * RS + r0 + rr;
        const bool live = i >= cur.a && i < cur.b && gc < n2;
        const u4 d = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(live ? (uint32_t)(((int64_t)i * n2 + gc) * sizeof(T)) : kOOB), 0, 0);
        __builtin_memcpy(bsub[rr].v, &d, 16);
      }
    }
    lds_barrier();
    // ---- PH: t[row][c0 + j] = sum_q a_h[q] x[row][c0 + j - 14 + q] (staged column j + 2 + q)
    {
      T acc[4 * PQ];
#pragma unroll
      for (int o = 0; o < 4 * PQ; ++o) acc[o] = T(0);
#pragma unroll
      for (int u = 0; u < PQ + 8; ++u) {
        const Q4<T> v = ldsq(psrow + 4 * (pg + u));
#pragma unroll
        for (int ee = 0; ee < 4; ++ee)
#pragma unroll
          for (int o = 0; o < 4 * PQ; ++o) {
            const int qq = 4 * u + ee - o - 2;
            if (qq >= 0 && qq < 29) acc[o] += ah[qq < 14 ? 14 - qq : qq - 14] * v.v[ee];
          }
      }
      const int col = c0 + 4 * pg;
      if (col < 7 || col + 4 * PQ - 1 >= n2 - 7) {  // the edge terms of the first / last 7 columns
#pragma unroll
        for (int o = 0; o < 4 * PQ; ++o) {
          const int j = col + o;
          if (j < 7) {
            for (int c = 0; c < 7; ++c) acc[o] -= ehl[8 * j + c] * psrow[16 + c];
          } else if (j >= n2 - 7 && j < n2) {
            const int jj = j - (n2 - 7), s0 = n2 - 7 - c0 + 16;
            for (int c = 0; c < 7; ++c) acc[o] -= ehh[8 * jj + c] * psrow[s0 + c];
          }
        }
      }
      int slot = (cur.s * RS) % RING + pr;
      slot = slot >= RING ? slot - RING : slot;
      T* dst = ring + slot * TP + 4 * pg;
#pragma unroll
      for (int k = 0; k < 4 * PQ / VN; ++k) {
        V16<T> c;
#pragma unroll
        for (int e = 0; e < VN; ++e) c.v[e] = acc[k * VN + e];
        stv(dst + k * VN, c);
      }
      if (slot < G::MIR) {  // the ring's first RB + 27 rows again past its end
#pragma unroll
        for (int k = 0; k < 4 * PQ / VN; ++k) {
          V16<T> c;
#pragma unroll
          for (int e = 0; e < VN; ++e) c.v[e] = acc[k * VN + e];
          stv(dst + RING * TP + k * VN, c);
        }
      }
    }
    lds_barrier();
    // ---- PV: out row i = a - 28 + s RS + r0 + rr reads t rows i - 14 .. i + 14 (staged s RS + r0 + rr - 28 ..)
    {
      const int base = (cur.s * RS + r0 - 28 + RING) % RING;
      const T* rcol = ring + base * TP + VN * vg;  // window row j at rcol + j TP (contiguous: the mirror)
      V16<T> acc[RB];
#pragma unroll
      for (int rr = 0; rr < RB; ++rr)
#pragma unroll
        for (int m = 0; m < VN; ++m) acc[rr].v[m] = T(0);
      constexpr int NV = RB + 28, CH = 4, NCH = NV / CH;
      static_assert(NV % CH == 0, "whole chunks");
      V16<T> w[2][CH];  // chunk c in w[c & 1]; the next chunk's reads in flight during this one's FMAs
      auto rd = [&](int c, V16<T>(&wc)[CH]) {
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          wc[j] = nrm_ldsv(rcol + (c * CH + j) * TP);
        }
      };
      rd(0, w[0]);
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if (c + 1 < NCH) rd(c + 1, w[(c + 1) & 1]);
        nrm_fence();
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          const int v = c * CH + j;
#pragma unroll
          for (int rr = 0; rr < RB; ++rr) {
            const int qq = v - rr;
            if (qq >= 0 && qq < 29) {
              const T h = av[qq < 14 ? 14 - qq : qq - 14];
#pragma unroll
              for (int m = 0; m < VN; ++m) acc[rr].v[m] += h * w[c & 1][j].v[m];
            }
          }
        }
#pragma unroll
        for (int rr = 0; rr < RB; ++rr)
#pragma unroll
          for (int m = 0; m < VN; ++m) asm volatile("" : "+v"(acc[rr].v[m]));
        nrm_fence();
      }
      // every thread issues RB stores per step (rows outside [a, b) dropped by the range check),
      // so the next step's wait for its staged rows leaves these stores in flight
      const Rsrc dst = rsrc_of(out + cur.plane * (int64_t)n1 * n2, (uint32_t)((int64_t)n1 * n2 * sizeof(T)));
#pragma unroll
      for (int rr = 0; rr < RB; ++rr) {
        const int i = cur.a - 28 + cur.s * RS + r0 + rr;
        const bool live = i >= cur.a && i < cur.b && gc < n2;
        if (live && (i < 7 || i >= n1 - 7)) {  // the edge terms of the first / last 7 rows
          const bool top = i < 7;
          const int jr = top ? i : i - (n1 - 7), row0 = top ? 0 : n1 - 7;
          const T* e = top ? evl : evh;
          for (int c = 0; c < 7; ++c) {
            const V16<T> wv = ldv(ring + ((row0 + c - cur.a + 14) % RING) * TP + VN * vg);
            const T ec = e[8 * jr + c];
#pragma unroll
            for (int m = 0; m < VN; ++m) acc[rr].v[m] -= ec * wv.v[m];
          }
        }
        if constexpr (SUB) {
#pragma unroll
          for (int m = 0; m < VN; ++m) acc[rr].v[m] = acc[rr].v[m] - bsub[rr].v[m];
        }
        u4 d;
        __builtin_memcpy(&d, acc[rr].v, 16);
        __builtin_amdgcn_raw_buffer_store_b128(d, dst, (int)(live ? (uint32_t)(((int64_t)i * n2 + gc) * sizeof(T)) : kOOB), 0, 0);
      }
    }
  };
  auto advance = [&](const Cur& c, bool& more) {  // the step after c (more = false: none)
    Cur n = c;
    more = true;
    if (c.s + 1 < c.ns) {
      n.s = c.s + 1;
    } else {
      more = c.t + t_stride < t_end;
      if (more) n = task_at(c.t + t_stride);
    }
    return n;
  };
  Q4<T> q[NL];
  Cur cur = task_at(t0);
  prefetch(cur, q);
  for (;;) {
    // the previous step's RB row stores may still be in flight (with SUB the wait also covers its RB
    // sub loads, issued before the stores)
    stage(q, std::integral_constant<int, RB>{});
    bool more;
    const Cur nxt = advance(cur, more);
    prefetch(nxt, q);  // unconditional (the last step re-reads its own rows): the wait for these
                       // loads at the next step then leaves this step's stores in flight
    body(cur);
    if (!more) break;
    cur = nxt;
  }
}

// fp32: k_sep2d_nrm (53 KB of LDS, 3 workgroups / CU); fp64: k_sep2d_nrmm (77 KB, 2 / CU).  The mirrored ring
// in fp32 needs 72 KB (2 / CU) and measured slower there: 512^3 0.41-0.48 against 0.36-0.43 ms, 4096^2 equal;
// in fp64 it took 1024^3 from 5.19-5.22 to 4.59-4.67 ms, 4096^2 from 0.108-0.111 to 0.098-0.100 ms (bitwise the
// same output; loading two steps ahead: no further change, profiles/r5_nrm_ab.txt)
template <typename T, bool SUB>
static const void* nrm_fn() {
  if constexpr (sizeof(T) == 8) return reinterpret_cast<const void*>(&k_sep2d_nrmm<T, SUB>);
  else return reinterpret_cast<const void*>(&k_sep2d_nrm<T, SUB>);
}
template <typename T>
static size_t nrm_lds() {
  if constexpr (sizeof(T) == 8) return NrmM<T>::lds_bytes();
  else return NrmF::lds_bytes();
}

template <typename T, bool SUB>
static void nrm_attr() {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute(nrm_fn<T, SUB>(), hipFuncAttributeMaxDynamicSharedMemorySize, (int)nrm_lds<T>());
    (void)hipGetLastError();
    done = true;
  }
}

template <typename T>
static int nrm_slots() {
  static int slots = 0;
  if (slots == 0) {
    int dev = 0, cus = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess || cus < 1)
      cus = 256;
    nrm_attr<T, false>();
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, nrm_fn<T, false>(), 256, nrm_lds<T>()) != hipSuccess ||
        nb < 1)
      nb = 1;
    (void)hipGetLastError();
    slots = cus * nb;
    const char* e = getenv("PCS_ATA_SLOTS");  // diagnostics: grid-size sweep
    if (e && atoi(e) > 0) slots = atoi(e);
  }
  return slots;
}

// the two-pass kernel takes taps reaching <= 7 samples either side (any centred filter of
// <= 15 taps) on planes of >= 16 x 16; PCS_ATA_KERNEL=4pass pins the four-pass kernel (diagnostics)
static bool nrm_fits(int64_t n1, int64_t n2, int ka, int offa, int kb, int offb) {
  const char* e = getenv("PCS_ATA_KERNEL");
  if (e && strcmp(e, "4pass") == 0) return false;
  return n1 >= 16 && n2 >= 16 && n2 % 4 == 0 && offa <= 7 && ka - 1 - offa <= 7 && offb <= 7 && kb - 1 - offb <= 7;
}

template <typename T>
static int sep_nrm(const void* in, void* out, int64_t np, int64_t n1, int64_t n2, const void* ha, int ka, int offa,
                   const void* hb, int kb, int offb, hipStream_t st, const void* sub = nullptr) {
  constexpr int TX = sizeof(T) == 8 ? NrmM<T>::TX : NrmF::TX;
  if (np == 0) return PCS_OK;
  const int64_t nstrips = (n2 + TX - 1) / TX, pieces = np * nstrips;
  const int64_t slots = nrm_slots<T>();
  // row segments: the fewest (each task re-reads a 28-row prologue) whose tasks fill the resident
  // workgroup slots once, segments of >= 64 rows; then one task per workgroup, later workgroups
  // starting as earlier ones finish.  Against the resident grid (a contiguous run of tasks per
  // workgroup, segments by a waves x rows cost): 512^3 fp32 0.49 against 0.57-0.58 ms, 1024^3 fp64
  // 5.96 (4 tasks per workgroup) against 7.33-7.44 ms, 4096^2 fp64 0.113 either way
  // (profiles/r4_nrm_slots_sweep*.txt).  PCS_NRM_GRIDX=k (diagnostics): k x the resident slots, each
  // workgroup a contiguous run of tasks
  const int64_t max_seg = n1 / 64 > 1 ? n1 / 64 : 1;
  int64_t nseg = 1;
  while (nseg < max_seg && pieces * nseg < slots) ++nseg;
  const int64_t seg_len = (n1 + nseg - 1) / nseg;
  nseg = (n1 + seg_len - 1) / seg_len;
  const int64_t ntasks = pieces * nseg;
  static int gridx = -1;
  if (gridx < 0) {
    const char* e = getenv("PCS_NRM_GRIDX");
    gridx = e && atoi(e) > 0 ? atoi(e) : 0;
  }
  const int64_t gslots = gridx > 0 ? slots * gridx : ntasks;
  const int64_t grid = ntasks < gslots ? ntasks : gslots;
  const size_t lds = nrm_lds<T>();
  auto go = [&](auto kern) {
    kern<<<(unsigned)grid, 256, lds, st>>>((const T*)in, (T*)out, (int)n1, (int)n2, (int)nstrips, (int)nseg,
                                           (int)seg_len, ntasks, (const T*)ha, ka, offa, (const T*)hb, kb, offb,
                                           (const T*)sub);
  };
  if (sub != nullptr) {
    nrm_attr<T, true>();
    if constexpr (sizeof(T) == 8) go(k_sep2d_nrmm<T, true>);
    else go(k_sep2d_nrm<T, true>);
  } else {
    nrm_attr<T, false>();
    if constexpr (sizeof(T) == 8) go(k_sep2d_nrmm<T, false>);
    else go(k_sep2d_nrm<T, false>);
  }
  return launch_status();
}

template <typename T>
static int sep_ata(const void* in, void* out, int64_t np, int64_t n1, int64_t n2, const void* ha, int ka, int offa,
                   const void* hb, int kb, int offb, hipStream_t st) {
  using A = AtaG;
  if (!in || !out || !ha || !hb || np < 0 || n1 < 1 || n2 < 1 || ka < 1 || ka > A::KT || kb < 1 || kb > A::KT ||
      offa < 0 || offa >= ka || offb < 0 || offb >= kb || in == out)
    return PCS_EINVAL;
  if ((uintptr_t)in % 16 || (uintptr_t)out % 16) return PCS_EINVAL;
  if (nrm_fits(n1, n2, ka, offa, kb, offb) && n1 * n2 * (int64_t)sizeof(T) < (1LL << 30))
    return sep_nrm<T>(in, out, np, n1, n2, ha, ka, offa, hb, kb, offb, st);
  const int padb = ata_padb(kb, offb);
  if (padb < 0 || n2 % 4 != 0 || n1 >= (1LL << 30) || n2 >= (1LL << 30)) return PCS_EUNSUPPORTED;
  if (np == 0) return PCS_OK;
  const int o2 = offb + padb, sh4 = (4 - o2 % 4) % 4;
  const int64_t nstrips = (n2 + A::TX - 1) / A::TX, pieces = np * nstrips;
  const int64_t slots = ata_slots<T>();
  // row segments: the count minimising (waves of resident workgroups) x (rows per task + the
  // 28-row prologue of the two vertical passes), segments of >= 64 rows
  const int64_t max_seg = n1 / 64 > 1 ? n1 / 64 : 1;
  int64_t nseg = 1, best = -1;
  for (int64_t c = 1; c <= max_seg; ++c) {
    const int64_t len = (n1 + c - 1) / c, waves = (pieces * c + slots - 1) / slots;
    const int64_t cost = waves * (len + 2 * (A::KT - 1));
    if (best < 0 || cost < best) {
      best = cost;
      nseg = c;
    }
  }
  const int64_t seg_len = (n1 + nseg - 1) / nseg;
  nseg = (n1 + seg_len - 1) / seg_len;
  const int64_t ntasks = pieces * nseg;
  const int64_t grid = ntasks < slots ? ntasks : slots;
  const size_t lds = ata_lds_bytes<T>();
  auto go = [&](auto kern) {
    kern<<<(unsigned)grid, A::NT, lds, st>>>((const T*)in, (T*)out, (int)n1, (int)n2, (int)nstrips, (int)nseg,
                                             (int)seg_len, ntasks, (const T*)ha, ka, (const T*)hb, kb, offa, padb, o2);
  };
  switch (sh4) {
    case 0: ata_attr<T, 0>(); go(k_sep2d_ata<T, 0>); break;
    case 1: ata_attr<T, 1>(); go(k_sep2d_ata<T, 1>); break;
    default: ata_attr<T, 2>(); go(k_sep2d_ata<T, 2>); break;
  }
  return launch_status();
}

}  // namespace pcs

using namespace pcs;

namespace pcs {
// N x - sub by the two-pass kernel (the fp64 2-D march's gradient buffer, pds.hip); PCS_EUNSUPPORTED when
// the two-pass kernel does not take the taps / layout (the caller then forms N x and subtracts in the step)
int sep_normal_minus(int dt, const void* in, void* out, const void* sub, int64_t np, int64_t n1, int64_t n2,
                     const void* ha, int ka, int offa, const void* hb, int kb, int offb, hipStream_t st) {
  if (!in || !out || !sub || !ha || !hb || np < 0 || n1 < 1 || n2 < 1 || in == out || sub == out) return PCS_EINVAL;
  // a buffer off the 16-B grid is a layout this kernel does not take: the caller's fallback (N x, then the
  // subtraction inside the step) runs it
  if ((uintptr_t)in % 16 || (uintptr_t)out % 16 || (uintptr_t)sub % 16) return PCS_EUNSUPPORTED;
  const int64_t esz = dt == PCS_F64 ? 8 : 4;
  if (!nrm_fits(n1, n2, ka, offa, kb, offb) || n1 * n2 * esz >= (1LL << 30)) return PCS_EUNSUPPORTED;
  if (np == 0) return PCS_OK;
  if (dt == PCS_F32) return sep_nrm<float>(in, out, np, n1, n2, ha, ka, offa, hb, kb, offb, st, sub);
  if (dt == PCS_F64) return sep_nrm<double>(in, out, np, n1, n2, ha, ka, offa, hb, kb, offb, st, sub);
  return PCS_EINVAL;
}
}  // namespace pcs

extern "C" {

int pcs_conv2d_sep_ata_planes(int dt, const void* in, void* out, int64_t nplanes, int64_t n1, int64_t n2,
                              const void* ha, int ka, int offa, const void* hb, int kb, int offb, hipStream_t st) {
  if (dt == PCS_F32) return sep_ata<float>(in, out, nplanes, n1, n2, ha, ka, offa, hb, kb, offb, st);
  if (dt == PCS_F64) return sep_ata<double>(in, out, nplanes, n1, n2, ha, ka, offa, hb, kb, offb, st);
  return PCS_EINVAL;
}

}  // extern "C"
