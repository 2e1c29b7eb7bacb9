// Row-marching fused 2-D PDS iteration through the NORMAL operator of the separable blur
// (fp32, tiers H = 3 / 7): grad F = Conv^T (Conv x - y) = N x - b with
//   N = Conv^T Conv = N_v (x) N_h        (the column and row passes commute, so N factors)
//   b = Conv^T y                          (formed once per problem by the host: pcs_pds2d_args.cty)
// so an iteration applies two (4H+1)-tap passes instead of four (2H+1)-tap passes, with no
// residual ring and one LDS round trip per pass.  Away from the image edges N_v / N_h are the
// autocorrelation of the taps; on the H rows (columns) nearest an edge the zero-boundary
// truncation between Conv and Conv^T changes the window taps -- the host tables
// (pcs_pds2d_args.ntaps, below) hold the exact rows of N there.  Same update as the 4-pass
// march kernel (pds_march.hpp); the iterates differ from it only by fp32 rounding.
//
// One workgroup (256 threads: 4 rows x 16 column groups per wave) owns a 64-column strip of a row
// segment [s0, s1) (strips on 256-B boundaries) and marches down it 16 rows per step; each item
// also computes the column after its 4 (t, g, u): the strip's 65th column, whose u K u of the 64th
// needs, comes from the last group's fifth column:
//   top   land z of this step (loaded during the previous one); issue the next step's loads:
//         x rows [a+2H+17, a+2H+33), b rows [a+17, a+33), z rows [a+16, a+33)
//   PH    t = N_h x on rows [a+2H+1, a+2H+17)           x ring (32 rows) -> t ring (64 rows)
//   PV    g = N_v t - b on rows [a+1, a+17); x_t = prox_G(x - tau g - tau K^T z),
//         u = 2 x_t - x -> u ring, x' = rho x_t + (1 - rho) x
//   P6    z' = rho fenchel(z + sigma K u) + (1 - rho) z on rows [a, a+16)
//         park the next step's x rows in the x ring
// Three barriers per step (the 4-pass kernel has five).
//
// ntaps (fp32, 64 + 32 H values): [0, 32) N_v window taps tv[q] (q = 0..4H: row r - 2H + q) =
// the autocorrelation of the axis-0 taps, [32, 64) the same along axis 1, then the truncation
// corrections E (H x 8 each, N = window - E on the edge band): E_v for rows 0..H-1 against rows
// 0..H-1, E_v for rows n0-H+j against rows n0-H+k, E_h for columns 0..H-1, E_h for the last H.
// Reference: PrimalDualSplitting.update_iterand, pycsou/opt/proxalgs.py:343-355, with
// grad F = Conv^T((2 (Conv x - y)) 0.5) (core/map.py:609-610), Conv from
// pycsou/linop/conv.py:167-295.
#pragma once
// waves per SIMD the register budget targets (diagnostics builds override)
#ifndef PCS_NM_WPE
#define PCS_NM_WPE 3
#endif
// window rows per PV read chunk (2 chunks in flight)
#ifndef PCS_NM_PF
#define PCS_NM_PF 2
#endif
#ifndef PCS_NM_EDGE
#define PCS_NM_EDGE 1
#endif
// cache-policy bits of the x' / z' stores (16 = sc1: written through, not left dirty in L2)
// C2 2048^2: 31.4 against 32.3 us per iteration, C3 4096^2: 112.7 against 113.9 us (two alternating
// reps each, profiles/r3_store_policy_ab.txt)
#ifndef PCS_NM_SAUX
#define PCS_NM_SAUX 16
#endif

#include <type_traits>

#include "pds_march.hpp"
#include "stencil.hpp"

namespace pcs {

// compiler-only fence: no memory access (LDS reads included) moves across it, at IR or MIR level
// (bounds the reads in flight, hence the registers they occupy); emits no instruction
__device__ __forceinline__ void pcs_fence() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// the value is live (computed) at this point: arithmetic is not sunk past it
__device__ __forceinline__ void pin4(G4<float>& g) {
  asm volatile("" : "+v"(g.v[0]), "+v"(g.v[1]), "+v"(g.v[2]), "+v"(g.v[3]));
}

__device__ __forceinline__ void pin1(float& v) { asm volatile("" : "+v"(v)); }

// one LDS float (a volatile read: never widened or merged with its neighbours)
__device__ __forceinline__ float lds1(const float* p) {
  typedef __attribute__((address_space(3))) const volatile float* lds_f1;
  return *(lds_f1)(p);
}

// wave priority 3 while a step's loads issue (s_setprio), 0 for its LDS / VALU phases: the loads
// of every wave go out ahead of the other waves' FMAs -- 113.1-113.6 against 115.9-116.5 us
// back to back (4 alternating reps, tools/march_ablate.py); PCS_NM_PRIO=0 drops it
#ifndef PCS_NM_PRIO
#define PCS_NM_PRIO 1
#endif

// s_waitcnt vmcnt(N) alone (expcnt / lgkmcnt left at their maxima)
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// cache-policy bits of the march's steady-state x / z / b loads (0: default; 2 = nt, streaming: measured
// 113.6-115.9 against 109.9-112.2 us on C3, no change on the centred-K C3, profiles/r3_ck38_nt_*ab.txt)
#ifndef PCS_NM_LAUX
#define PCS_NM_LAUX 0
#endif
template <int AUX>
__device__ __forceinline__ G4<float> bload4a(Rsrc r, uint32_t off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, AUX);
  return {{__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3])}};
}

// step 0's x rows loaded with the prologue's own rows (1: one exposed load latency per segment instead of
// two) or after the prologue's PV (0).  C3 106.7-106.9 against 107.0-107.8 us back to back, c3_cen
// 135.7-136.0 against 138.0-138.1 (profiles/r3_ck43_xe_*ab.txt)
#ifndef PCS_NM_XEARLY
#define PCS_NM_XEARLY 1
#endif

// forward kernel: the strip's 65th column by 16 lanes per output (1) or by the last group's 4 lanes
// per wave in a serial 29-read branch (0)
#ifndef PCS_NM_COOP65
#define PCS_NM_COOP65 1
#endif

// sum over the 16-lane DPP row holding the lane (every lane of the row gets the sum; the lanes of a
// row add in different orders, so only one lane's value is used): row_ror 8, 4, 2, 1
__device__ __forceinline__ float row_sum16(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xf, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xf, 0xf, false));
  return v;
}

// forward kernel: PV / update / P6 in the column layout (1: a thread owns one column of the wave's four
// rows -- b32 LDS reads, each t row of the window read once for four outputs, taps in VGPRs) or in the
// row layout of PH (0: four columns of one row, every output row reading its own 29-row window).
// Measured: parity green, but 123.8-125.0 against 107.1-111.0 us back to back (4 alternating reps,
// profiles/r3_ck35_cols_ab.txt): the b32 stores / loads (12 + 4 VMEM instructions per thread and step
// instead of 3 + 1) and the extra update reads cost more than the PV's halved LDS cycles save -- kept off
#ifndef PCS_NM_COLS
#define PCS_NM_COLS 0
#endif

// 4-B store through a descriptor (kOOB offsets dropped), cache-policy bits AUX as bstore4
template <int AUX = 0>
__device__ __forceinline__ void bstore1(Rsrc r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)off, 0, AUX);
}

// GEN: the extra columns' 8-lane reduction by DPP (quad_perm xor 1, xor 2, row_half_mirror: VALU
// latency) or by three ds_bpermute shuffles (0: LDS latency each); the same sums bit for bit
#ifndef PCS_NMG_DPP
#define PCS_NMG_DPP 1
#endif
// sum over the 8-lane group holding the lane (lanes 8 g .. 8 g + 7); every lane gets the same value, the
// sums of __shfl_xor by 1, 2, 4 (fp addition commutes, and after the quad steps a quad holds one value)
__device__ __forceinline__ float oct_sum8(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xf, 0xf, false));   // [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xf, 0xf, false));   // [2,3,0,1]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xf, 0xf, false));  // half mirror
  return v;
}

// diagnostics builds (timing only, wrong results): 1 = GEN without its extra columns, 2 = GEN with
// interior stencils everywhere, 4 = the forward kernel without its 65th column
#ifndef PCS_NMG_ABL
#define PCS_NMG_ABL 0
#endif
// GEN: the border strips' steps with interior rows take a form with the row axis interior (only the column
// axis on the edge rules) -- 0: every non-interior step on the all-axes form (A/B knob)
#ifndef PCS_NMG_ROWFORM
#define PCS_NMG_ROWFORM 1
#endif
// GEN: backward / centred K (KK != PCS_FORWARD) -- K^T z reads z rows lr - 1 .. lr + 1 and columns
// c - 1 .. c + 1, K u reads u rows r - 1 .. r + 1 and columns c - 1 .. c + 1: z tiles of 18 rows (the
// z0 tile from column c0 - 4 too), an 18-row u ring, and a sixth u / t / g column c0 - 1 (group 0,
// slot SLM1 of the t and u rows) beside the 65th
template <int H, bool GEN = false>
struct NMarch {
  static constexpr int TW = 64, TS = 16, NQ = 4 * H + 1;
  static constexpr int XL = RU4<2 * H>::value, SHX = XL - 2 * H;  // x region [c0 - XL, c0 + TW + XL)
  static constexpr int GXL = (TW + 2 * XL) / 4;                    // loaded x groups per row (24 / 20)
  static constexpr int WX = TW + 2 * XL + 4;                       // x ring pitch (odd slot count)
  // t ring: 48 rows (a step's window + new rows: 4H + 2 TS <= 48 + TS) + a mirror of its first 4H
  // (rows 48..48+4H-1 repeat rows 0..4H-1), so any (4H+1)-row window starting in the ring is contiguous
  // (forward, PCS_NM_COLS: 4H + 3, so the 4H + 4 rows of a wave's four-row window are contiguous too)
  static constexpr int XRING = 32, TRING = 48, TMIR = (GEN || !PCS_NM_COLS) ? 4 * H : 4 * H + 3;
  static constexpr int WT = TW + 4, WU = TW + 4;  // t / u rows: 65 columns used (272 B; GEN: 66)
  static constexpr int SLM1 = TW + 1;             // GEN: slot of column c0 - 1 in a t / u row
  // z tiles (own __shared__ arrays, filled by LDS-DMA, lane-linear): z0 rows of 17 groups (from
  // column c0; GEN: 18 from c0 - 4), z1 rows of 18 groups (from column c0 - 4); ZR rows from row a;
  // 5 (GEN: 6) wave-instructions of 64 x 16 B each
  static constexpr int ZR = GEN ? TS + 2 : TS + 1, Z0C = GEN ? 4 : 0, Z0G = GEN ? 18 : 17;
  static constexpr int WZ0 = 4 * Z0G, WZ1 = TW + 8, ZSLOTS = (GEN ? 6 : 5) * 64;
  static constexpr int UR = GEN ? TS + 2 : TS + 1;  // u ring rows: [a, a+16] (GEN: [a-1, a+16])
  static constexpr int NVH = (SHX + 3 + 4 * H) / 4 + 1;  // b128 groups a PH item reads
  static constexpr int NXN = TS * GXL;                   // x items per step
  static constexpr int NXP = (4 * H + 1 + (GEN ? 1 : 0)) * GXL;  // prologue x items
  static constexpr int O_XR = 0, O_T = O_XR + XRING * WX, O_U = O_T + (TRING + TMIR) * WT, O_W = O_U + UR * WU,
                       NW = 64 + 32 * H, SZ = O_W + NW;  // W: the ntaps table
  static_assert(ZR * (WZ0 / 4) <= ZSLOTS && ZR * (WZ1 / 4) <= ZSLOTS, "z tiles");
  static_assert(H == 3 || H == 7, "tiers 3 and 7");
  static_assert(TS + 2 * H + 1 + TS <= XRING + 1 + 2 * H, "x ring holds rows [a+1, a+2H+17)");
  static_assert(4 * H + TS <= TRING, "t ring holds a step's PV window (the rows PH writes are its newest)");
  static __device__ __forceinline__ int tslot(int r) { return (int)((unsigned)(r + TRING * (1 << 20)) % TRING); }
  static_assert(4 * (NVH - 1) + 3 >= SHX + 4 + 4 * H, "PH window (5 outputs)");
  static_assert((WX / 4) % 2 == 1, "odd x slot pitch");
};

template <typename T, int H, int HK, int NT, int KK>
__device__ __forceinline__ void nmarch_task(const T* __restrict__ x, T* __restrict__ xn, const T* __restrict__ z,
                                            T* __restrict__ zn, const T* __restrict__ b,
                                            const T* __restrict__ tq, const Slab32& s, const Params<T>& P, int gk,
                                            int edge, int s0, int s1, int c0, T* sm, T* Z0, T* Z1,
                                            double (&part)[4], int stop_raw) {
  static_assert(sizeof(T) == 4 && NT == 256, "fp32, 256 threads (4 rows x 16 column groups per wave)");
  constexpr bool GEN = KK != PCS_FORWARD;
  using M = NMarch<H, GEN>;
  constexpr int TS = M::TS, TW = M::TW, NQ = M::NQ, XL = M::XL, SHX = M::SHX, NVH = M::NVH;
  constexpr int WX = M::WX, WT = M::WT, WU = M::WU, WZ0 = M::WZ0, WZ1 = M::WZ1, GXL = M::GXL;
  constexpr int UR = M::UR, ZR = M::ZR, SLM1 = M::SLM1;
  constexpr int KXN = cdiv(M::NXN, NT), KXP = cdiv(M::NXP, NT);
  constexpr int GG = TW / 4;
  T* XR = sm + M::O_XR;
  T* TR = sm + M::O_T;
  T* U = sm + M::O_U;
  T* W = sm + M::O_W;  // taps (broadcast reads, re-read per phase: none live across the loop)
  int wz = 0;          // 0, laundered every step: taps read at W + wz are not loop-invariant
  const T* Wq = W;     // (so no tap read is hoisted out of the loop into registers)
  for (int i = threadIdx.x; i < M::NW; i += NT) W[i] = tq[i];  // visible after the first barrier
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hb = tid >> 5, l5 = tid & 31;
  const int ui = 2 * hb + lane_grp(l5), ug = lane_idx(l5);  // every phase: row ui, column group ug
  const int n0 = s.n0, n1 = s.n1;
  const int zstride = (s.rows + 2 * s.hz) * n1;
  const int xc0 = c0 - XL;
  const View vx = make_view(x, s, s.hx), vb = make_view(b, s, s.hy), vz0 = make_view(z, s, s.hz),
             vz1 = make_view(z + zstride, s, s.hz);
  const uint32_t pitch = (uint32_t)n1 * 4u;
  const Rsrc rxn = rsrc_of(xn, (uint32_t)(s.rows + 2 * s.hx) * pitch);
  const Rsrc rzn0 = rsrc_of(zn, (uint32_t)zstride * 4u), rzn1 = rsrc_of(zn + zstride, (uint32_t)zstride * 4u);
#define PCS_WAVE_ON(k, N) ((k) * NT + wv * 64 < (N))
#define PCS_ITEM(k, N) min((k) * NT + tid, (N) - 1)

  // ---- per-thread geometry
  const int ucg = c0 + 4 * ug;
  const uint32_t co_u = col_off(ucg, n1);
  const bool cin = ucg < n1;                        // group in the image (4-groups wholly in / out)
  const bool clast = ucg == n1 - 4;                 // holds the image's last column
  const bool cown = cin;                            // stored by this workgroup
  // GEN: the strip's columns c0 - 1 .. c0 + 64 >= 2 samples inside the image (no column edge rules)
  const bool cint = c0 >= 4 && c0 + TW + 3 <= n1 - 3;
  // GEN extra columns: lane l of wave wv works on output (row 4 wv + (eo & 3), column c0 - 1 (eo < 4) or
  // c0 + 64), eo = l / 8, window taps l % 8 + 8 j; its b value is loaded with the step's b (bm1)
  const int elane = tid & 63, eo = elane >> 3, esub = elane & 7, eur = 4 * wv + (eo & 3);
  const bool eright = eo >= 4;
  const int ecol = eright ? c0 + TW : c0 - 1, ets = eright ? TW : SLM1, eti = eright ? TW + 4 : 3;
  const uint32_t co_bx = GEN ? col_off(ecol, n1) : kOOB;
  // forward, PCS_NM_COOP65: lane l of wave wv works on the 65th column of row 4 wv + l / 16, window taps
  // l % 16 + 16 j
  const int fur = 4 * wv + (elane >> 4), fsub = elane & 15;
  (void)fur;
  (void)fsub;
  uint32_t co_xn[KXN];
  int rr_xn[KXN];
#pragma unroll
  for (int k = 0; k < KXN; ++k) {
    const int e = PCS_ITEM(k, M::NXN);
    rr_xn[k] = e / GXL;
    co_xn[k] = col_off(xc0 + 4 * (e - (e / GXL) * GXL), n1);
  }

  auto load_xn = [&](G4<T>(&xv)[KXN], int r0) {  // x rows [r0, r0 + TS) of the x region
#pragma unroll
    for (int k = 0; k < KXN; ++k) xv[k] = bload4a<PCS_NM_LAUX>(vx.r, vx.row_off(r0 + rr_xn[k]) + co_xn[k]);
  };
  auto store_xn = [&](const G4<T>(&xv)[KXN], int r0) {
#pragma unroll
    for (int k = 0; k < KXN; ++k) {
      if (!PCS_WAVE_ON(k, M::NXN)) continue;
      const int e = PCS_ITEM(k, M::NXN);
      const int r = e / GXL, g = e - (e / GXL) * GXL;
      st4(XR + ((r0 + r) & 31) * WX + 4 * g, xv[k]);
    }
  };
  // z0 rows [a, a + ZR), cols [c0 - Z0C, c0 + TW + 4) -> Z0; z1 rows [a, a + ZR), cols [c0 - 4, c0 + TW + 4) -> Z1,
  // straight into LDS (buffer_load ... lds: no VGPRs, no ds_write).  Wave w issues tile
  // instructions w and w + 4 of each tile (5 / 6 each): lane l of instruction j fills slot 64 j + l (rows
  // past the tile and rows below `rmin` read as 0).  The issuing waves wait for them (vmcnt) before the
  // barrier that precedes the first read.
  const int lane = tid & 63;
  auto load_z = [&](int a, int rmin) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = wv + 4 * jj;
      if (j < M::ZSLOTS / 64) {
        const int e = 64 * j + lane;
        constexpr int G0 = M::Z0G;
        const int r0 = e / G0, g0 = e - G0 * (e / G0);  // z0: 17 (GEN: 18) groups per row
        const int r1 = e / 18, g1 = e - 18 * (e / 18);  // z1: 18 groups per row (cols c0 - 4 .. c0 + 67)
        const uint32_t o0 = (r0 >= ZR || r0 < rmin ? kOOB : vz0.row_off(a + r0)) + col_off(c0 - M::Z0C + 4 * g0, n1);
        const uint32_t o1 = (r1 >= ZR || r1 < rmin ? kOOB : vz1.row_off(a + r1)) + col_off(c0 - 4 + 4 * g1, n1);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(vz0.r, (__attribute__((address_space(3))) void*)(Z0 + 256 * j), 16,
                                                 o0, 0, 0, PCS_NM_LAUX);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(vz1.r, (__attribute__((address_space(3))) void*)(Z1 + 256 * j), 16,
                                                 o1, 0, 0, PCS_NM_LAUX);
      }
    }
  };
  // ---- PH: t row lr = N_h x row lr on columns [c0 + 4 ug, + 5) -> t ring (the fifth column is
  // kept by the last group only: the strip's 65th column)
  auto ph = [&](int lr) {
    const T* xrow = XR + (lr & 31) * WX;
    T v[4 * NVH];
#pragma unroll
    for (int q = 0; q < NVH; ++q) {
      const G4<T> t4 = lds4(xrow + 4 * ug + 4 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * q + e] = t4.v[e];
    }
    G4<T> o;
    T o4 = T(0), om1 = T(0);  // om1 (GEN): column c0 - 1 (kept by group 0)
#pragma unroll
    for (int m = 0; m < 4; ++m) o.v[m] = T(0);
    // taps 4 at a time (broadcast LDS reads), the next 4 read while the current ones are used
    constexpr int NQ4 = (PCS_ABL & 2048) ? 1 : (NQ + 3) / 4;
    G4<T> wc = lds4(Wq + 32), wn;
#pragma unroll
    for (int q4 = 0; q4 < NQ4; ++q4) {
      if (q4 + 1 < NQ4) wn = lds4(Wq + 32 + 4 * (q4 + 1));
      pcs_fence();
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int q = 4 * q4 + e;
        if (q < NQ) {
#pragma unroll
          for (int m = 0; m < 4; ++m) o.v[m] += wc.v[e] * v[SHX + m + q];
          o4 += wc.v[e] * v[SHX + 4 + q];
          if constexpr (GEN) om1 += wc.v[e] * v[SHX - 1 + q];
        }
      }
      pin4(o);
      pin1(o4);
      if constexpr (GEN) pin1(om1);
      pcs_fence();
      wc = wn;
    }
    if (PCS_NM_EDGE && c0 < H) {  // exact rows of N_h on the H columns nearest the left image edge
      const G4<T> x0 = lds4(xrow + XL), x1 = lds4(xrow + XL + 4);  // image columns 0..7
      const T xe[8] = {x0.v[0], x0.v[1], x0.v[2], x0.v[3], x1.v[0], x1.v[1], x1.v[2], x1.v[3]};
      const bool on = ug < 2;
      const T* et = Wq + 64 + 16 * H + 4 * (on ? ug : 0);
#pragma unroll
      for (int k = 0; k < H; ++k) {
        const G4<T> e4 = lds4(et + 8 * k);
#pragma unroll
        for (int m = 0; m < 4; ++m) o.v[m] -= (on ? e4.v[m] : T(0)) * xe[k];
      }
    }
    if (PCS_NM_EDGE && c0 + TW + 1 > n1 - H) {  // ... and the right one (image columns n1 - 8 .. n1 - 1)
      const T* xr8 = xrow + (n1 - 8 - xc0);
      const G4<T> x0 = lds4(xr8), x1 = lds4(xr8 + 4);
      const T xf[8] = {x0.v[0], x0.v[1], x0.v[2], x0.v[3], x1.v[0], x1.v[1], x1.v[2], x1.v[3]};
      const int j = ucg - (n1 - 8);
      const bool on = j == 0 || j == 4;
      const bool on5 = ug == GG - 1 && ucg + 4 == n1 - 4;  // the 65th column is column n1 - 4
      const T* et = Wq + 64 + 24 * H + (on ? j : 0);
#pragma unroll
      for (int k = 0; k < H; ++k) {
        const G4<T> e4 = lds4(et + 8 * k);
#pragma unroll
        for (int m = 0; m < 4; ++m) o.v[m] -= (on ? e4.v[m] : T(0)) * xf[8 - H + k];
        o4 -= (on5 ? et[8 * k + 4 - j] : T(0)) * xf[8 - H + k];
      }
    }
    const int sl = M::tslot(lr);
    T* trow = TR + sl * WT + 4 * ug;
    st4(trow, o);
    if (ug == GG - 1) trow[4] = o4;
    if constexpr (GEN) {  // column c0 - 1 (>= H columns inside the image, or outside it: no edge rows of N_h)
      if (ug == 0) trow[SLM1] = om1;
    }
    if (sl < M::TMIR) {  // the mirror copy
      st4(trow + M::TRING * WT, o);
      if (ug == GG - 1) trow[M::TRING * WT + 4] = o4;
      if constexpr (GEN) {
        if (ug == 0) trow[M::TRING * WT + SLM1] = om1;
      }
    }
  };
  // ---- PV + update: row lr = a + 1 + ui, columns [c, c + 4); the last group also column c + 4
  // (the strip's 65th), in a branch of its own lanes (4 per wave: conflict-free b32 reads)
  auto pv = [&](int a, const G4<T>& bv, T b5, T bm1, int ub) {
    const int lr = a + 1 + ui, gr = s.row0 + lr;
    // GEN: the step's update rows [a+1, a+16] and z' rows [a, a+16) >= 2 samples inside the image
    const bool rint = s.row0 + a >= 2 && s.row0 + a + TS <= n0 - 3;
    int slot = ui + 1 + ub;
    slot = slot >= UR ? slot - UR : slot;
    // g = N_v t - b: rows lr - 2H .. lr + 2H of the t ring, window row q at p0 + q rows (no
    // address arithmetic: immediate offsets); reads are issued in chunks of PF behind a compiler
    // fence (at most 2 PF in flight)
    G4<T> g;
#pragma unroll
    for (int m = 0; m < 4; ++m) g.v[m] = T(0);
    const T* p0 = TR + M::tslot(lr - 2 * H) * WT + 4 * ug;  // the window is contiguous (mirror rows)
    constexpr int PF = PCS_NM_PF, NCH = (PCS_ABL & 2048) ? 1 : (NQ + PF - 1) / PF;  // window rows per chunk
    G4<T> buf[2][PF];
#pragma unroll
    for (int j = 0; j < PF; ++j)
      if (j < NQ) buf[0][j] = lds4(p0 + j * WT);
    // taps 4 at a time, the next 4 read one chunk ahead of their use (as the window rows)
    static_assert(4 % PF == 0, "a tap group spans whole chunks");
    G4<T> w4 = lds4(Wq), w4n;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (c + 1 < NCH) {
#pragma unroll
        for (int j = 0; j < PF; ++j)
          if ((c + 1) * PF + j < NQ) buf[(c + 1) & 1][j] = lds4(p0 + ((c + 1) * PF + j) * WT);
        if (((c + 1) * PF) % 4 == 0) w4n = lds4(Wq + (c + 1) * PF);
      }
      pcs_fence();
#pragma unroll
      for (int j = 0; j < PF; ++j) {
        if (c * PF + j < NQ) {
#pragma unroll
          for (int m = 0; m < 4; ++m) g.v[m] += w4.v[(c * PF + j) & 3] * buf[c & 1][j].v[m];
        }
      }
      pin4(g);  // the chunk's FMAs stay here (not sunk below the later reads)
      pcs_fence();
      if (c + 1 < NCH && ((c + 1) * PF) % 4 == 0) w4 = w4n;
    }
    const int wrow0 = s.row0 + a + 1 + 4 * wv;  // the wave's first global row
    const bool vedge = PCS_NM_EDGE && (wrow0 < H || wrow0 + 3 >= n0 - H);  // rows of N_v near an image edge
    const bool top = gr >= 0 && gr < H, bot = gr >= n0 - H && gr < n0;
    const T* d = Wq + 64 + (top ? 8 * gr : 8 * H + 8 * (gr - (n0 - H)));
    const int kr0 = (wrow0 < H ? 0 : n0 - H) - s.row0;  // local row of the band's first image row
    if (vedge) {
#pragma unroll
      for (int k = 0; k < H; ++k) {
        const G4<T> t4 = lds4(TR + (M::tslot(kr0) + k) * WT + 4 * ug);  // contiguous through the mirror
        const T w = (top || bot) ? d[k] : T(0);
#pragma unroll
        for (int m = 0; m < 4; ++m) g.v[m] -= w * t4.v[m];
      }
    }
    if constexpr (!GEN) {
      const G4<T> xv4 = lds4(XR + (lr & 31) * WX + XL + 4 * ug);
      const G4<T> za = lds4(Z0 + ui * WZ0 + 4 * ug);               // z0[lr - 1]
      const G4<T> zb = lds4(Z0 + (ui + 1) * WZ0 + 4 * ug);         // z0[lr]
      const G4<T> z1a = lds4(Z1 + (ui + 1) * WZ1 + 4 * ug);        // z1[lr][c - 4 .. c - 1]
      const G4<T> z1b = lds4(Z1 + (ui + 1) * WZ1 + 4 * ug + 4);    // z1[lr][c .. c + 3]
      const bool r_last = gr >= n0 - 1, r_first = gr <= 0;
      const bool rrow = gr < n0 && lr <= s.rows;
      const bool own = lr >= s0 && lr < s1 && gr < n0 && cown;
      // x_t = prox_G((x - tau g) - tau K^T z); K^T z for forward differences, VStack order:
      // (0 + D0^T z0) + D1^T z1
      auto xt_of = [&](T gd, T xv, T za_, T zb_, T zl, T zr, bool last_col) {
        T d0 = r_first ? T(0) : za_;
        if (!r_last) d0 -= zb_;
        const T d1 = zl - (last_col ? T(0) : zr);
        return prox_g((xv - P.tau * gd) - P.tau * (d0 * P.inv_step0 + d1 * P.inv_step1), gk, P.seg_a, P.seg_b);
      };
      G4<T> uo, xo;
      T sdx = T(0), sx = T(0);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const T xv = xv4.v[m];
        const T xt = xt_of(g.v[m] - bv.v[m], xv, za.v[m], zb.v[m], (m == 0) ? z1a.v[3] : z1b.v[m - 1], z1b.v[m],
                           m == 3 && clast);
        uo.v[m] = (rrow && cin) ? (T(2) * xt - xv) : T(0);
        const T xnew = P.rho * xt + P.omr * xv;
        xo.v[m] = xnew;
        const T dx = xv - xnew;
        sdx += dx * dx;
        sx += xv * xv;
      }
      if (own) {
        part[0] += (double)sdx;
        part[1] += (double)sx;
      }
      T* urow = U + slot * WU + 4 * ug;
      st4(urow, uo);
      bstore4<PCS_NM_SAUX>(rxn, (own ? (uint32_t)(lr + s.hx) * pitch : kOOB) + co_u, xo);
#if PCS_NM_COOP65
      // the strip's 65th column c0 + 64 (never the image's last: n1 % 4 == 0), cooperatively: the wave's 4
      // outputs (its rows 4 wv + f, f = lane / 16) take 16 lanes each, lane fsub summing window taps
      // fsub and fsub + 16 (and edge term fsub), a row_ror DPP reduction inside the 16-lane row, then
      // every lane evaluates the update and lane fsub == 0 stores u (b65: the step's b at the column,
      // loaded per lane with bv)
      if (!(PCS_NMG_ABL & 4)) {
        const int flr = a + 1 + fur, fgr = s.row0 + flr;
        const T* q0 = TR + M::tslot(flr - 2 * H) * WT + TW;  // the window is contiguous (mirror rows)
        T pg = T(0);
#pragma unroll
        for (int j = 0; j < (NQ + 15) / 16; ++j) {
          const int q = fsub + 16 * j;
          if (q < NQ) pg += Wq[q] * q0[q * WT];
        }
        if (vedge) {  // the exact rows of N_v near an image edge: term k = fsub
          const bool ftop = fgr >= 0 && fgr < H, fbot = fgr >= n0 - H && fgr < n0;
          const T* fd = Wq + 64 + (ftop ? 8 * fgr : 8 * H + 8 * (fgr - (n0 - H)));
          if (fsub < H && (ftop || fbot)) pg -= fd[fsub] * TR[(M::tslot(kr0) + fsub) * WT + TW];
        }
        pg = row_sum16(pg);
        const T xe = XR[(flr & 31) * WX + XL + TW];
        const bool f_last = fgr >= n0 - 1, f_first = fgr <= 0;
        T d0 = f_first ? T(0) : Z0[fur * WZ0 + TW];
        if (!f_last) d0 -= Z0[(fur + 1) * WZ0 + TW];
        const T d1 = Z1[(fur + 1) * WZ1 + TW + 3] - Z1[(fur + 1) * WZ1 + TW + 4];
        const T xt = prox_g((xe - P.tau * (pg - b5)) - P.tau * (d0 * P.inv_step0 + d1 * P.inv_step1), gk, P.seg_a,
                            P.seg_b);
        int fslot = fur + 1 + ub;
        fslot = fslot >= UR ? fslot - UR : fslot;
        const bool frow = fgr < n0 && flr <= s.rows;
        if (fsub == 0) U[fslot * WU + TW] = (frow && c0 + TW < n1) ? (T(2) * xt - xe) : T(0);
      }
#else
      if (!(PCS_NMG_ABL & 4) && ug == GG - 1) {  // the strip's 65th column c0 + 64 (never the image's last: n1 % 4 == 0)
        const T* q0 = p0 + 4;
        T g4 = T(0);
#pragma unroll
        for (int q4 = 0; q4 < (NQ + 3) / 4; ++q4) {
          const G4<T> w = lds4(Wq + 4 * q4);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (4 * q4 + e < NQ) g4 += w.v[e] * lds1(q0 + (4 * q4 + e) * WT);
        }
        if (vedge) {
#pragma unroll
          for (int k = 0; k < H; ++k) g4 -= ((top || bot) ? d[k] : T(0)) * lds1(TR + (M::tslot(kr0) + k) * WT + TW);
        }
        const T xe = lds1(XR + (lr & 31) * WX + XL + TW);
        const T xt = xt_of(g4 - b5, xe, lds1(Z0 + ui * WZ0 + TW), lds1(Z0 + (ui + 1) * WZ0 + TW), z1b.v[3],
                           lds1(Z1 + (ui + 1) * WZ1 + TW + 4), false);
        urow[4] = (rrow && ucg + 4 < n1) ? (T(2) * xt - xe) : T(0);
      }
#endif
    } else {  // backward / centred K: K^T z from z rows lr - 1 .. lr + 1, columns c - 1 .. c + 1
      const G4<T> xv4 = lds4(XR + (lr & 31) * WX + XL + 4 * ug);
      const T* z0p = Z0 + ui * WZ0 + 4 * ug + 4;  // tile row ui = row lr - 1, column c
      const G4<T> za = lds4(z0p), zb = lds4(z0p + WZ0), zc = lds4(z0p + 2 * WZ0);
      const T* z1p = Z1 + (ui + 1) * WZ1 + 4 * ug;  // row lr, columns c - 4 ..
      const G4<T> z1a = lds4(z1p), z1b = lds4(z1p + 4);
      const T z1r = lds4(z1p + 8).v[0];
      const T zh[6] = {z1a.v[3], z1b.v[0], z1b.v[1], z1b.v[2], z1b.v[3], z1r};
      const bool rrow = (unsigned)gr < (unsigned)n0 && lr <= s.rows;
      const bool own = lr >= s0 && lr < s1 && gr < n0 && cown;
      // x_t = prox_G((x - tau (g - b)) - tau K^T z), K^T z = D0^T z0 + D1^T z1 (stencil.hpp windows;
      // I: rows and columns >= 2 samples inside the image, no edge rules -- the same bits)
      // (intr: the row axis interior; intc: the column axis)
      auto xt_of = [&](auto intr, auto intc, T gd, T xv, const T (&w0)[5], const T (&w1)[5], int i1) {
        constexpr bool I0 = decltype(intr)::value || (PCS_NMG_ABL & 2);
        constexpr bool I1 = decltype(intc)::value || (PCS_NMG_ABL & 2);
        const T kt = pcs_fma(sw_d1_adj<KK, I0>(w0, gr, n0, edge), P.inv_step0,
                             sw_d1_adj<KK, I1>(w1, i1, n1, edge) * P.inv_step1);
        return prox_g((xv - P.tau * gd) - P.tau * kt, gk, P.seg_a, P.seg_b);
      };
      G4<T> uo, xo;
      T sdx = T(0), sx = T(0);
      auto items = [&](auto intr, auto intc) {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const T xv = xv4.v[m];
          const T w0[5] = {T(0), za.v[m], zb.v[m], zc.v[m], T(0)};
          const T w1[5] = {T(0), zh[m], zh[m + 1], zh[m + 2], T(0)};
          const T xt = xt_of(intr, intc, g.v[m] - bv.v[m], xv, w0, w1, ucg + m);
          uo.v[m] = (rrow && cin) ? (T(2) * xt - xv) : T(0);
          const T xnew = pcs_fma(P.rho, xt, P.omr * xv);
          xo.v[m] = xnew;
          const T dx = xv - xnew;
          sdx += dx * dx;
          sx += xv * xv;
        }
      };
      if (rint && cint) items(std::true_type{}, std::true_type{});
      else if (PCS_NMG_ROWFORM && rint) items(std::true_type{}, std::false_type{});
      else items(std::false_type{}, std::false_type{});
      if (own) {
        part[0] += (double)sdx;
        part[1] += (double)sx;
      }
      T* urow = U + slot * WU + 4 * ug;
      st4(urow, uo);
      bstore4<PCS_NM_SAUX>(rxn, (own ? (uint32_t)(lr + s.hx) * pitch : kOOB) + co_u, xo);
      // the two extra columns, cooperatively: the wave's 8 outputs (its 4 rows x columns c0 - 1 and
      // c0 + 64) take 8 lanes each, lane `esub` summing window taps esub, esub + 8, .. (and edge term
      // esub), a 3-step xor reduction, then all 8 lanes evaluate the update and lane 0 of the group
      // stores u.  Column c0 - 1 is >= H inside the image or outside it, c0 + 64 is < n1 - H or the
      // image's last group (no edge rows of N_h); every lane of the wave does useful work instead of
      // 8 lanes issuing a 29-read serial pass
      if (!(PCS_NMG_ABL & 1)) {
        const int elr = a + 1 + eur, egr = s.row0 + elr;
        const T* q0 = TR + M::tslot(elr - 2 * H) * WT + ets;  // the window is contiguous (mirror rows)
        T part_g = T(0);
#pragma unroll
        for (int j = 0; j < (NQ + 7) / 8; ++j) {
          const int q = esub + 8 * j;
          if (q < NQ) part_g += Wq[q] * q0[q * WT];
        }
        if (vedge) {  // the exact rows of N_v near an image edge: term k = esub
          const bool etop = egr >= 0 && egr < H, ebot = egr >= n0 - H && egr < n0;
          const T* ed = Wq + 64 + (etop ? 8 * egr : 8 * H + 8 * (egr - (n0 - H)));
          if (esub < H && (etop || ebot)) part_g -= ed[esub] * TR[(M::tslot(kr0) + esub) * WT + ets];
        }
#if PCS_NMG_DPP
        part_g = oct_sum8(part_g);
#else
        part_g += __shfl_xor(part_g, 1, 64);
        part_g += __shfl_xor(part_g, 2, 64);
        part_g += __shfl_xor(part_g, 4, 64);
#endif
        const T xe = XR[(elr & 31) * WX + XL + (ecol - c0)];
        const T w0[5] = {T(0), Z0[eur * WZ0 + eti], Z0[(eur + 1) * WZ0 + eti], Z0[(eur + 2) * WZ0 + eti], T(0)};
        const T* z1e = Z1 + (eur + 1) * WZ1 + eti;
        const T w1[5] = {T(0), z1e[-1], z1e[0], z1e[1], T(0)};
        // K^T z on the extra column's row (egr) through xt_of's row index: recompute with egr
        const T kt = pcs_fma(sw_d1_adj<KK, false>(w0, egr, n0, edge), P.inv_step0,
                             sw_d1_adj<KK, false>(w1, ecol, n1, edge) * P.inv_step1);
        const T xt = prox_g((xe - P.tau * (part_g - bm1)) - P.tau * kt, gk, P.seg_a, P.seg_b);
        int eslot = eur + 1 + ub;
        eslot = eslot >= UR ? eslot - UR : eslot;
        const bool erow = (unsigned)egr < (unsigned)n0 && elr <= s.rows;
        if (esub == 0) U[eslot * WU + ets] = (erow && (unsigned)ecol < (unsigned)n1) ? (T(2) * xt - xe) : T(0);
      }
    }
  };
  // ---- P6: z' on row lr = a + ui
  auto p6f = [&](int a, int ub) {
    const int lr = a + ui, gr = s.row0 + lr;
    int sl0 = ui + ub, sl1 = ui + 1 + ub;
    sl0 = sl0 >= 17 ? sl0 - 17 : sl0;
    sl1 = sl1 >= 17 ? sl1 - 17 : sl1;
    const G4<T> uc = lds4(U + sl0 * WU + 4 * ug);
    const G4<T> ud = lds4(U + sl1 * WU + 4 * ug);
    const G4<T> zv0 = lds4(Z0 + ui * WZ0 + 4 * ug);
    const G4<T> zv1 = lds4(Z1 + ui * WZ1 + 4 * ug + 4);
    const T une = lds4(U + sl0 * WU + 4 * ug + 4).v[0];  // u[c + 4] (a b128 read: conflict-free)
    const bool r_last = gr >= n0 - 1;
    const bool own = lr >= s0 && lr < s1 && gr < n0 && cown;
    G4<T> o0, o1;
    T sdz = T(0), sz = T(0);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const T uright = (m < 3) ? uc.v[m + 1] : une;
      const T d0 = r_last ? T(0) : (ud.v[m] - uc.v[m]);
      const T d1 = (m == 3 && clast) ? T(0) : (uright - uc.v[m]);
      const T w0v = zv0.v[m] + P.sigma * (d0 * P.inv_step0), w1v = zv1.v[m] + P.sigma * (d1 * P.inv_step1);
      T zt0, zt1;
      if (HK == PCS_H_L21) {
        // w - sigma prox_{L21, t}(w / sigma) (penalty.py:551-557, t = lam / sigma) = w min(1, lam / ||w||)
        const T sc = fminf(T(1), P.lam * fast_rsqrt(w0v * w0v + w1v * w1v));
        zt0 = w0v * sc;
        zt1 = w1v * sc;
      } else {  // w - sigma (v - t clip(v / t)), v = w / sigma (func/base.py:239-240) = clip(w, -lam, lam)
        zt0 = fminf(fmaxf(w0v, -P.lam), P.lam);
        zt1 = fminf(fmaxf(w1v, -P.lam), P.lam);
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
    bstore4<PCS_NM_SAUX>(rzn0, off, o0);
    bstore4<PCS_NM_SAUX>(rzn1, off, o1);
  };
  // ---- P6 (GEN): z' on row lr = a + ui; K u from u rows lr - 1 .. lr + 1 (ring rows [a - 1, a + 16]) and
  // columns c - 1 .. c + 4 (c0 - 1 at SLM1, c0 + 64 at slot TW)
  auto p6g = [&](int a, int ub) {
    const int lr = a + ui, gr = s.row0 + lr;
    int slm = ui - 1 + ub, sl0 = ui + ub, sl1 = ui + 1 + ub;
    slm = slm < 0 ? slm + UR : (slm >= UR ? slm - UR : slm);
    sl0 = sl0 >= UR ? sl0 - UR : sl0;
    sl1 = sl1 >= UR ? sl1 - UR : sl1;
    const T* u0 = U + sl0 * WU;
    const G4<T> uc = lds4(u0 + 4 * ug), ud = lds4(U + sl1 * WU + 4 * ug), uu = lds4(U + slm * WU + 4 * ug);
    const T ur4 = lds4(u0 + 4 * ug + 4).v[0];               // u[c + 4] (a b128 read: conflict-free)
    const T ul = lds1(u0 + (ug == 0 ? SLM1 : 4 * ug - 1));  // u[c - 1]
    const T uh[6] = {ul, uc.v[0], uc.v[1], uc.v[2], uc.v[3], ur4};
    const G4<T> zv0 = lds4(Z0 + ui * WZ0 + 4 * ug + 4);
    const G4<T> zv1 = lds4(Z1 + ui * WZ1 + 4 * ug + 4);
    const bool own = lr >= s0 && lr < s1 && gr < n0 && cown;
    const bool rint = s.row0 + a >= 2 && s.row0 + a + TS <= n0 - 3;
    G4<T> o0, o1;
    T sdz = T(0), sz = T(0);
    auto items = [&](auto intr, auto intc) {
      constexpr bool I0 = decltype(intr)::value || (PCS_NMG_ABL & 2);
      constexpr bool I1 = decltype(intc)::value || (PCS_NMG_ABL & 2);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const T w0[5] = {T(0), uu.v[m], uc.v[m], ud.v[m], T(0)};
        const T w1[5] = {T(0), uh[m], uh[m + 1], uh[m + 2], T(0)};
        const T k0 = sw_d1_fwd<KK, I0>(w0, gr, n0, P.inv_step0, edge);
        const T k1 = sw_d1_fwd<KK, I1>(w1, ucg + m, n1, P.inv_step1, edge);
        const T w0v = zv0.v[m] + P.sigma * k0, w1v = zv1.v[m] + P.sigma * k1;
        T zt0, zt1;
        if (HK == PCS_H_L21) {  // w min(1, lam / ||w||), as p6f
          const T sc = fminf(T(1), P.lam * fast_rsqrt(pcs_fma(w0v, w0v, w1v * w1v)));
          zt0 = w0v * sc;
          zt1 = w1v * sc;
        } else {
          zt0 = fminf(fmaxf(w0v, -P.lam), P.lam);
          zt1 = fminf(fmaxf(w1v, -P.lam), P.lam);
        }
        o0.v[m] = pcs_fma(P.rho, zt0, P.omr * zv0.v[m]);
        o1.v[m] = pcs_fma(P.rho, zt1, P.omr * zv1.v[m]);
        const T e0 = zv0.v[m] - o0.v[m], e1 = zv1.v[m] - o1.v[m];
        sdz += pcs_fma(e0, e0, e1 * e1);
        sz += pcs_fma(zv0.v[m], zv0.v[m], zv1.v[m] * zv1.v[m]);
      }
    };
    if (rint && cint) items(std::true_type{}, std::true_type{});
    else if (PCS_NMG_ROWFORM && rint) items(std::true_type{}, std::false_type{});
    else items(std::false_type{}, std::false_type{});
    if (own) {
      part[2] += (double)sdz;
      part[3] += (double)sz;
    }
    const uint32_t off = (own ? (uint32_t)(lr + s.hz) * pitch : kOOB) + co_u;
    bstore4<PCS_NM_SAUX>(rzn0, off, o0);
    bstore4<PCS_NM_SAUX>(rzn1, off, o1);
  };
  auto p6 = [&](int a, int ub) {
    if constexpr (GEN) p6g(a, ub);
    else p6f(a, ub);
  };

  // ---- forward, PCS_NM_COLS: the column layout.  Lane `lane` of wave wv owns column cc = c0 + lane of
  // the wave's rows: PV / update rows a + 1 + 4 wv + o, P6 rows a + 4 wv + o (o = 0..3).  PV reads the
  // 4H + 4 window rows once each (b32, contiguous through the mirror) and feeds every row to the
  // outputs it reaches; each output sums its taps in ascending order, as the row layout does
  const int cc = c0 + lane;
  const uint32_t co_cc = col_off(cc, n1);
  const bool ccin = cc < n1, cclast = cc == n1 - 1;
  auto pvc = [&](int a, const T (&bc)[4], T b5, int ub) {
    const int lr0 = a + 1 + 4 * wv;
    const T* p0 = TR + M::tslot(lr0 - 2 * H) * WT + lane;
    constexpr int NR = NQ + 3, CH = 4, NCH = (NR + CH - 1) / CH;
    static_assert(CH == 4, "chunk c's rows 4c .. 4c + 3 take taps of groups c - 1 and c");
    T g[4] = {T(0), T(0), T(0), T(0)};
    T buf[2][CH];
    // taps 4 at a time (broadcast b128 reads, group c + 1 read one chunk ahead)
    G4<T> wprev = {{T(0), T(0), T(0), T(0)}}, wcur = lds4(Wq), wnext;
#pragma unroll
    for (int j = 0; j < CH; ++j) buf[0][j] = lds1(p0 + j * WT);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (c + 1 < NCH) {
#pragma unroll
        for (int j = 0; j < CH; ++j)
          if ((c + 1) * CH + j < NR) buf[(c + 1) & 1][j] = lds1(p0 + ((c + 1) * CH + j) * WT);
        if (4 * (c + 1) < NQ) wnext = lds4(Wq + 4 * (c + 1));
      }
      pcs_fence();
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int q = c * CH + j;
#pragma unroll
        for (int o = 0; o < 4; ++o) {
          const int k = q - o;
          if (q < NR && k >= 0 && k < NQ) {
            const T w = k >= 4 * c ? wcur.v[k - 4 * c] : wprev.v[k - 4 * (c - 1)];
            g[o] += w * buf[c & 1][j];
          }
        }
      }
#pragma unroll
      for (int o = 0; o < 4; ++o) pin1(g[o]);
      pcs_fence();
      wprev = wcur;
      if (c + 1 < NCH && 4 * (c + 1) < NQ) wcur = wnext;
    }
    const int wrow0 = s.row0 + lr0;  // the wave's first global row
    const bool vedge = PCS_NM_EDGE && (wrow0 < H || wrow0 + 3 >= n0 - H);
    const int kr0 = (wrow0 < H ? 0 : n0 - H) - s.row0;  // local row of the band's first image row
    if (vedge) {  // exact rows of N_v near an image edge
      T te[H];
#pragma unroll
      for (int k = 0; k < H; ++k) te[k] = lds1(TR + (M::tslot(kr0) + k) * WT + lane);  // contiguous (mirror)
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        const int gr = wrow0 + o;
        const bool top = gr >= 0 && gr < H, bot = gr >= n0 - H && gr < n0;
        const T* d = Wq + 64 + (top ? 8 * gr : bot ? 8 * H + 8 * (gr - (n0 - H)) : 0);
#pragma unroll
        for (int k = 0; k < H; ++k) g[o] -= ((top || bot) ? d[k] : T(0)) * te[k];
      }
    }
    // update: z0 tile rows 4 wv .. 4 wv + 4 (row lr - 1 of output o at tile row 4 wv + o), z1 tile rows
    // 4 wv + 1 + o at columns cc - 1 (index lane + 3) and cc (lane + 4)
    T z0c[5];
#pragma unroll
    for (int o = 0; o < 5; ++o) z0c[o] = lds1(Z0 + (4 * wv + o) * WZ0 + lane);
    T sdx = T(0), sx = T(0);
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const int lr = lr0 + o, gr = s.row0 + lr;
      const T xv = lds1(XR + (lr & 31) * WX + XL + lane);
      const T zl = lds1(Z1 + (4 * wv + 1 + o) * WZ1 + 3 + lane), zc = lds1(Z1 + (4 * wv + 1 + o) * WZ1 + 4 + lane);
      const bool r_last = gr >= n0 - 1, r_first = gr <= 0;
      const bool rrow = gr < n0 && lr <= s.rows;
      const bool own = lr >= s0 && lr < s1 && gr < n0 && ccin;
      T d0 = r_first ? T(0) : z0c[o];
      if (!r_last) d0 -= z0c[o + 1];
      const T d1 = zl - (cclast ? T(0) : zc);
      const T xt = prox_g((xv - P.tau * (g[o] - bc[o])) - P.tau * (d0 * P.inv_step0 + d1 * P.inv_step1), gk,
                          P.seg_a, P.seg_b);
      int slot = 4 * wv + o + 1 + ub;
      slot = slot >= UR ? slot - UR : slot;
      U[slot * WU + lane] = (rrow && ccin) ? (T(2) * xt - xv) : T(0);
      const T xnew = P.rho * xt + P.omr * xv;
      bstore1<PCS_NM_SAUX>(rxn, (own ? (uint32_t)(lr + s.hx) * pitch : kOOB) + co_cc, xnew);
      if (own) {
        const T dx = xv - xnew;
        sdx += dx * dx;
        sx += xv * xv;
      }
    }
    part[0] += (double)sdx;
    part[1] += (double)sx;
#if PCS_NM_COOP65
    if (!(PCS_NMG_ABL & 4)) {  // the strip's 65th column, 16 lanes per output (as in pv)
      const int flr = a + 1 + fur, fgr = s.row0 + flr;
      const T* q0 = TR + M::tslot(flr - 2 * H) * WT + TW;
      T pg = T(0);
#pragma unroll
      for (int j = 0; j < (NQ + 15) / 16; ++j) {
        const int q = fsub + 16 * j;
        if (q < NQ) pg += Wq[q] * q0[q * WT];
      }
      if (vedge) {
        const bool ftop = fgr >= 0 && fgr < H, fbot = fgr >= n0 - H && fgr < n0;
        const T* fd = Wq + 64 + (ftop ? 8 * fgr : fbot ? 8 * H + 8 * (fgr - (n0 - H)) : 0);
        if (fsub < H && (ftop || fbot)) pg -= fd[fsub] * TR[(M::tslot(kr0) + fsub) * WT + TW];
      }
      pg = row_sum16(pg);
      const T xe = XR[(flr & 31) * WX + XL + TW];
      const bool f_last = fgr >= n0 - 1, f_first = fgr <= 0;
      T d0 = f_first ? T(0) : Z0[fur * WZ0 + TW];
      if (!f_last) d0 -= Z0[(fur + 1) * WZ0 + TW];
      const T d1 = Z1[(fur + 1) * WZ1 + TW + 3] - Z1[(fur + 1) * WZ1 + TW + 4];
      const T xt = prox_g((xe - P.tau * (pg - b5)) - P.tau * (d0 * P.inv_step0 + d1 * P.inv_step1), gk, P.seg_a,
                          P.seg_b);
      int fslot = fur + 1 + ub;
      fslot = fslot >= UR ? fslot - UR : fslot;
      const bool frow = fgr < n0 && flr <= s.rows;
      if (fsub == 0) U[fslot * WU + TW] = (frow && c0 + TW < n1) ? (T(2) * xt - xe) : T(0);
    }
#else
    static_assert(PCS_NM_COOP65 || !PCS_NM_COLS, "the column layout computes the 65th column cooperatively");
#endif
  };
  // P6 in the column layout: z' on rows lr = a + 4 wv + o, column cc; u rows 4 wv + o .. 4 wv + 4 of the step
  auto p6c = [&](int a, int ub) {
    T uc[5];
#pragma unroll
    for (int o = 0; o < 5; ++o) {
      int sl = 4 * wv + o + ub;
      sl = sl >= 17 ? sl - 17 : sl;
      uc[o] = lds1(U + sl * WU + lane);
    }
    T sdz = T(0), sz = T(0);
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const int lr = a + 4 * wv + o, gr = s.row0 + lr;
      int sl = 4 * wv + o + ub;
      sl = sl >= 17 ? sl - 17 : sl;
      const T uright = lds1(U + sl * WU + lane + 1);
      const T zv0 = lds1(Z0 + (4 * wv + o) * WZ0 + lane), zv1 = lds1(Z1 + (4 * wv + o) * WZ1 + 4 + lane);
      const bool r_last = gr >= n0 - 1;
      const bool own = lr >= s0 && lr < s1 && gr < n0 && ccin;
      const T d0 = r_last ? T(0) : (uc[o + 1] - uc[o]);
      const T d1 = cclast ? T(0) : (uright - uc[o]);
      const T w0v = zv0 + P.sigma * (d0 * P.inv_step0), w1v = zv1 + P.sigma * (d1 * P.inv_step1);
      T zt0, zt1;
      if (HK == PCS_H_L21) {  // as p6f
        const T sc = fminf(T(1), P.lam * fast_rsqrt(w0v * w0v + w1v * w1v));
        zt0 = w0v * sc;
        zt1 = w1v * sc;
      } else {
        zt0 = fminf(fmaxf(w0v, -P.lam), P.lam);
        zt1 = fminf(fmaxf(w1v, -P.lam), P.lam);
      }
      const T o0 = P.rho * zt0 + P.omr * zv0, o1 = P.rho * zt1 + P.omr * zv1;
      const uint32_t off = (own ? (uint32_t)(lr + s.hz) * pitch : kOOB) + co_cc;
      bstore1<PCS_NM_SAUX>(rzn0, off, o0);
      bstore1<PCS_NM_SAUX>(rzn1, off, o1);
      if (own) {
        const T e0 = zv0 - o0, e1 = zv1 - o1;
        sdz += e0 * e0 + e1 * e1;
        sz += zv0 * zv0 + zv1 * zv1;
      }
    }
    part[2] += (double)sdz;
    part[3] += (double)sz;
  };
  constexpr bool COLS = !GEN && PCS_NM_COLS;
  // b of the column layout: rows r0 + 4 wv + o, column cc
  auto load_bc = [&](T (&bc)[4], int r0) {
#pragma unroll
    for (int o = 0; o < 4; ++o)
      bc[o] = __uint_as_float(
          __builtin_amdgcn_raw_buffer_load_b32(vb.r, (int)(vb.row_off(r0 + 4 * wv + o) + co_cc), 0, 0));
  };

  // ================= prologue: t rows [s0 - 2H, s0 + 2H], u / x' on row s0 (GEN: t rows from s0 - 2H - 1,
  // u on rows s0 - 1 and s0)
  // b of a group = its 4 columns (bv) and, for the last group, the strip's 65th column (b5; GEN: the
  // lane's extra-column output, bm1)
  const uint32_t co_b5 = ug == GG - 1 ? col_off(c0 + TW, n1) : kOOB;
  // forward, PCS_NM_COOP65: every lane loads b of its 65th-column output (row r0 + fur), else the last
  // group's lanes b of their own row's 65th column
  const uint32_t co_f65 = col_off(c0 + TW, n1);
  auto load_b5 = [&](int r0) -> T {
    if constexpr (!GEN && PCS_NM_COOP65)
      return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vb.r, (int)(vb.row_off(r0 + fur) + co_f65), 0, 0));
    else
      return bload4(vb.r, vb.row_off(r0 + ui) + co_b5).v[0];
  };
  constexpr int PR = GEN ? 1 : 0;  // extra prologue rows
  G4<T> xnx[KXN], bv;
  T b5, bm1 = T(0);
  T bc[4];  // COLS: b of the lane's column on the wave's four update rows
  {
    G4<T> xv[KXP];
#pragma unroll
    for (int k = 0; k < KXP; ++k) {
      const int e = PCS_ITEM(k, M::NXP);
      const int r = e / GXL, g = e - (e / GXL) * GXL;
      xv[k] = bload4(vx.r, vx.row_off(s0 - 2 * H - PR + r) + col_off(xc0 + 4 * g, n1));
    }
    // z rows s0 - 1, s0 only (GEN: s0 - 3 .. s0 + 1) for the prologue's update rows; b on those rows
    load_z(s0 - TS, GEN ? TS - 3 : TS - 1);
    if constexpr (GEN) {  // rows s0 - 1 (ui 14) and s0 (ui 15)
      const uint32_t rbp = ui >= TS - 2 ? vb.row_off(s0 - TS + 1 + ui) : kOOB;
      bv = bload4(vb.r, rbp + co_u);
      b5 = bload4(vb.r, rbp + co_b5).v[0];
      bm1 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vb.r, (int)(vb.row_off(s0 - TS + 1 + eur) + co_bx), 0, 0));
    } else {
      if constexpr (COLS) load_bc(bc, s0 - TS + 1);  // wave 3: rows s0 - 3 .. s0
      else bv = bload4(vb.r, (ui == TS - 1 ? vb.row_off(s0) : kOOB) + co_u);
      if constexpr (PCS_NM_COOP65) b5 = load_b5(s0 - TS + 1);  // row s0: wave 3's last output row
      else b5 = bload4(vb.r, (ui == TS - 1 ? vb.row_off(s0) : kOOB) + co_b5).v[0];
    }
#pragma unroll
    for (int k = 0; k < KXP; ++k) {
      if (!PCS_WAVE_ON(k, M::NXP)) continue;
      const int e = PCS_ITEM(k, M::NXP);
      const int r = e / GXL, g = e - (e / GXL) * GXL;
      st4(XR + ((s0 - 2 * H - PR + r) & 31) * WX + 4 * g, xv[k]);
    }
#if PCS_NM_XEARLY
    load_xn(xnx, s0 + 2 * H + 1);  // step 0's x rows: in flight with the prologue's (parked after PH)
#endif
    vm_wait<0>();
  }
  if (stop_raw) return;  // loop already stopped (solver.py:65-66): loads landed, nothing stored
  lds_barrier();
  ph(s0 - 2 * H - PR + ui);  // t rows [s0 - 2H - PR, s0 - 2H - PR + 16)
  if (ui + TS < 4 * H + 1 + PR) ph(s0 - 2 * H - PR + TS + ui);  // t rows [.. + 16, s0 + 2H]
  lds_barrier();
  // u on row s0 (GEN: s0 - 1 too) -> the ring slots of step 0's rows a - 1, a; x' on row s0 (rows above: not own)
  if (wv == 3) {
    if constexpr (COLS) pvc(s0 - TS, bc, b5, UR - TS);
    else pv(s0 - TS, bv, b5, bm1, UR - TS);
  }
#if !PCS_NM_XEARLY
  load_xn(xnx, s0 + 2 * H + 1);        // step 0's x rows [s0 + 2H + 1, s0 + 2H + 17)
#endif
  lds_barrier();
  store_xn(xnx, s0 + 2 * H + 1);  // slots of rows [s0 + 2H - 31, s0 + 2H - 15): read by PH above only

  // ================= march: step k covers t rows [a+2H+1, a+2H+17), u / x' rows [a+1, a+17), z' rows [a, a+16)
  const int nsteps = (s1 - s0 + TS - 1) / TS;
  int ub = 0;  // (16 k) mod UR: row r = a + j sits in u ring slot (j + ub) mod UR
  for (int k = 0; k < nsteps; ++k) {
    const int a = s0 + k * TS;
    lds_barrier();  // step k-1 done with U, Z and the t / x ring rows it read; its x rows landed
    asm volatile("" : "+v"(wz));
    Wq = W + wz;
    // this step's z tiles (LDS-DMA) and b, the next step's x rows (registers, landed after P6)
#if PCS_NM_PRIO
    __builtin_amdgcn_s_setprio(3);  // the step's loads issue ahead of other waves' VALU
#endif
    // The z tiles land through LDS-DMA loads; before the barrier that precedes their first read the wave
    // waits until only the loads it issued after them are outstanding.  Forward K: b (bv, b5) and the x
    // rows, counted.  GEN: its b values (bm1 of the extra-column lanes, b5 of the last group) are used on
    // subsets of lanes only, and the compiler sinks those loads to their uses past the wait -- counted,
    // they left the last tile load in flight when the tiles were read (a race: the C3 centred iterate
    // differed between runs from the second iteration on).  GEN therefore issues every load ahead of the
    // tiles and waits for all of them (tools/vmcnt_check.py checks the counts in the assembly).
#ifndef PCS_NM_LOADFIRST  // diagnostics: the forward kernel with GEN's load order and full wait
#define PCS_NM_LOADFIRST 0
#endif
    constexpr bool LF = GEN || (PCS_NM_LOADFIRST && !COLS);
    if constexpr (LF) {
      if constexpr (GEN) bm1 = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vb.r, (int)(vb.row_off(a + 1 + eur) + co_bx), 0, 0));
      bv = bload4a<PCS_NM_LAUX>(vb.r, vb.row_off(a + 1 + ui) + co_u);
      b5 = load_b5(a + 1);
      load_xn(xnx, a + 2 * H + 1 + TS);
      load_z(a, 0);
    } else {
      load_z(a, 0);
      if constexpr (COLS) {
        load_bc(bc, a + 1);
      } else {
        const uint32_t rb = vb.row_off(a + 1 + ui);
        bv = bload4a<PCS_NM_LAUX>(vb.r, rb + co_u);
      }
      b5 = load_b5(a + 1);
      load_xn(xnx, a + 2 * H + 1 + TS);
    }
#if PCS_NM_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    ph(a + 2 * H + 1 + ui);
    if constexpr (LF) vm_wait<0>();
    else vm_wait<KXN + (COLS ? 5 : 2)>();  // this wave's z tile loads have landed (b and the x rows may be in flight)
    lds_barrier();
    if constexpr (COLS) pvc(a, bc, b5, ub);
    else pv(a, bv, b5, bm1, ub);
    lds_barrier();
    if constexpr (COLS) p6c(a, ub);
    else p6(a, ub);
    store_xn(xnx, a + 2 * H + 1 + TS);  // x ring slots of rows [a + 2H - 15, a + 2H + 1): read above
    if constexpr (GEN) ub = ub + TS >= UR ? ub + TS - UR : ub + TS;
    else ub = ub == 0 ? 16 : ub - 1;
  }
#undef PCS_WAVE_ON
#undef PCS_ITEM
}

// One block per task (64-column strip x row segment); with `hist` the last workgroups also
// reduce the partials and run the loop control, with `ro.sums` they only reduce.  The C3 kernel
// (forward K):
template <typename T, int H, int HK, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(PCS_NM_WPE))) void k_pds2d_nmarch(
    const T* __restrict__ x, T* __restrict__ xn, const T* __restrict__ z, T* __restrict__ zn,
    const T* __restrict__ b, const T* __restrict__ tq, Slab32 s, Params<T> P, int gk, double* __restrict__ partials,
    Ctrl* ctrl, double* hist, void* ws, RedOut ro, int tiles_x, Bands bd, int ntasks) {
  using M = NMarch<H, false>;
  __shared__ __attribute__((aligned(16))) T sm[M::SZ];
  __shared__ __attribute__((aligned(16))) T zs0[4 * M::ZSLOTS];  // z tiles: own arrays, so the LDS-DMA
  __shared__ __attribute__((aligned(16))) T zs1[4 * M::ZSLOTS];  // into them never aliases a ring read
  __shared__ double red[4 * (NT / 64)];
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
  const int c0 = strip * M::TW;

  double part[4] = {0.0, 0.0, 0.0, 0.0};
  if (!stopped)
    nmarch_task<T, H, HK, NT, PCS_FORWARD>(x, xn, z, zn, b, tq, s, P, gk, 0, s0, s1, c0, sm, zs0, zs1, part, stop_raw);
  if (stop_raw) return;  // the task returned before any store
  block_sum<4>(part, red);
  publish_partials(part, partials, ntasks, ws, ctrl, hist, flag, ro);
}

// backward / centred K (KK; `edge` = Gradient(edge=...) of the centred kind): the GEN geometry
template <typename T, int H, int HK, int NT, int KK>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(PCS_NM_WPE))) void k_pds2d_nmarch_gen(
    const T* __restrict__ x, T* __restrict__ xn, const T* __restrict__ z, T* __restrict__ zn,
    const T* __restrict__ b, const T* __restrict__ tq, Slab32 s, Params<T> P, int gk, int edge,
    double* __restrict__ partials, Ctrl* ctrl, double* hist, void* ws, RedOut ro, int tiles_x, Bands bd,
    int ntasks) {
  static_assert(KK == PCS_BACKWARD || KK == PCS_CENTERED, "k_pds2d_nmarch is the forward kernel");
  using M = NMarch<H, true>;
  __shared__ __attribute__((aligned(16))) T sm[M::SZ];
  __shared__ __attribute__((aligned(16))) T zs0[4 * M::ZSLOTS];
  __shared__ __attribute__((aligned(16))) T zs1[4 * M::ZSLOTS];
  __shared__ double red[4 * (NT / 64)];
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
  const int c0 = strip * M::TW;

  double part[4] = {0.0, 0.0, 0.0, 0.0};
  if (!stopped) nmarch_task<T, H, HK, NT, KK>(x, xn, z, zn, b, tq, s, P, gk, edge, s0, s1, c0, sm, zs0, zs1, part, stop_raw);
  if (stop_raw) return;  // the task returned before any store
  block_sum<4>(part, red);
  publish_partials(part, partials, ntasks, ws, ctrl, hist, flag, ro);
}

}  // namespace pcs
