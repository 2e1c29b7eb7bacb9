/*
 * pycsou_hip.h -- C ABI of libpycsou_hip.so, the gfx950 (MI355X) engine behind
 * the pycsou PrimalDualSplitting / APGD hot path.
 *
 * Conventions
 *  - Buffers are caller-allocated DEVICE pointers, contiguous, C order (the
 *    flat-vector layout pycsou uses: a d-dimensional image of `shape` is the
 *    C-order ravel; a gradient is the concatenation [d_0 x; d_1 x; (d_2 x)],
 *    pycsou/linop/diff.py:855-875).
 *  - `dtype` is PCS_F32 or PCS_F64.  Scalars are passed as double and rounded
 *    to `dtype` inside, exactly as NumPy does for `array * python_float`.
 *  - Every entry point returns PCS_OK (0) or a negative status; nothing is
 *    thrown across the ABI.  No entry point allocates, frees or synchronises:
 *    all of them are hipGraph-capturable on `stream`.
 *  - Workspaces (`ws`) are caller-allocated device buffers of the size the
 *    matching *_ws_bytes() query returns.
 *
 * Each entry point names the reference interface it replaces (file:line in
 * dhamm97/pycsou; PyLops 1.x for the operators pycsou delegates to it).
 */
#ifndef PYCSOU_HIP_H
#define PYCSOU_HIP_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { PCS_F32 = 0, PCS_F64 = 1 };
enum { PCS_OK = 0, PCS_EINVAL = -1, PCS_ELAUNCH = -2, PCS_EUNSUPPORTED = -3 };
/* derivative kinds (pycsou/linop/diff.py:24 `kind`) */
enum { PCS_FORWARD = 0, PCS_BACKWARD = 1, PCS_CENTERED = 2 };
/* H functional kinds in the fused step */
enum { PCS_H_L1 = 0, PCS_H_L21 = 1 };
/* G functional kinds in the fused step */
enum { PCS_G_NULL = 0, PCS_G_NONNEG = 1, PCS_G_SEGMENT = 2 };
/* F kinds in the fused step */
enum { PCS_F_NULL = 0, PCS_F_DENOISE = 1, PCS_F_SEPCONV = 2, PCS_F_GRADBUF = 3, PCS_F_CONV2D = 4, PCS_F_CONV0 = 5 };
/* finite-difference K of the fused 2-D steps */
enum { PCS_K_GRAD_FORWARD = 0, PCS_K_GRAD_BACKWARD = 1, PCS_K_GRAD_CENTERED = 2, PCS_K_LAPLACIAN = 3 };

int pcs_abi_version(void);

/* ---------------------------------------------------------------- operators */

/* FirstDerivative along `axis` (pycsou/linop/diff.py:24-130 -> pylops.FirstDerivative):
 * out = D_axis x.  ndim in 1..32, dims[ndim], step = sampling. */
int pcs_deriv1_fwd(int dtype, const void* x, void* out, int ndim, const int64_t* dims, int axis, double step,
                   int kind, int edge, hipStream_t stream);
/* Adjoint of the above (pylops FirstDerivative.rmatvec). */
int pcs_deriv1_adj(int dtype, const void* y, void* out, int ndim, const int64_t* dims, int axis, double step,
                   int kind, int edge, hipStream_t stream);

/* SecondDerivative along `axis` (pycsou/linop/diff.py:133-219 -> pylops.SecondDerivative):
 * out[i] = (x[i+1] - 2 x[i] + x[i-1]) / step^2 inside; ends 0, or the one-sided second-order
 * stencils with `edge`.  ndim in 1..32. */
int pcs_deriv2_fwd(int dtype, const void* x, void* out, int ndim, const int64_t* dims, int axis, double step,
                   int edge, hipStream_t stream);
int pcs_deriv2_adj(int dtype, const void* y, void* out, int ndim, const int64_t* dims, int axis, double step,
                   int edge, hipStream_t stream);

/* Gradient (pycsou/linop/diff.py:777-882 -> pylops.Gradient = VStack of FirstDerivative):
 * out[k*N:(k+1)*N] = D_k x for k < ndim (1..32; one launch per axis beyond 3).  steps[ndim]. */
int pcs_grad_fwd(int dtype, const void* x, void* out, int ndim, const int64_t* dims, const double* steps,
                 int kind, int edge, hipStream_t stream);
/* Gradient.adjoint: out = sum_k D_k^T z_k (accumulated in axis order, pylops VStack.rmatvec). */
int pcs_grad_adj(int dtype, const void* z, void* out, int ndim, const int64_t* dims, const double* steps,
                 int kind, int edge, hipStream_t stream);

/* Laplacian 2-D (pycsou/linop/diff.py:885-957 -> pylops.Laplacian):
 * out = w0 * D2_0 x + w1 * D2_1 x.  dims[2], weights[2], steps[2]. */
int pcs_lap_fwd(int dtype, const void* x, void* out, const int64_t* dims, const double* weights,
                const double* steps, int edge, hipStream_t stream);
int pcs_lap_adj(int dtype, const void* y, void* out, const int64_t* dims, const double* weights,
                const double* steps, int edge, hipStream_t stream);

/* Convolve2D (pycsou/linop/conv.py:167-295 -> pylops Convolve2D, 'same', zero boundary):
 * out[i] = sum_j h[j] x[i + off - j] (+ beta * b[i] if b != NULL).  `psf` is a device
 * buffer kh*kw of dtype.  The adjoint (correlation) is this call with the flipped PSF
 * and offsets (kh-1-off0, kw-1-off1). */
int pcs_conv2d(int dtype, const void* x, void* out, int64_t n0, int64_t n1, const void* psf, int kh, int kw,
               int off0, int off1, const void* b, double beta, hipStream_t stream);
/* x == out is rejected (PCS_EINVAL); b == out is allowed.  Odd square PSFs centred at
 * (kh/2, kw/2) of size 3..15 or 31 run the register-blocked marching kernel (corr2d.hip);
 * other shapes run the LDS-tiled kernel, or use the plan entry points below. */

/* Convolve2D through a packed plan (same operator, any PSF up to 31 x 31): every call is
 * one correlation with a K x K window centred at K/2, K = the "tier" (odd, 3..15 or 31)
 * returned by pcs_conv2d_plan_tier (< 0: unsupported).  pcs_conv2d_plan_pack is a HOST
 * function: it writes the forward (adjoint = 0) or adjoint (adjoint = 1) window of the
 * fp64 host PSF into a host buffer of pcs_conv2d_plan_bytes bytes of `dtype`, which the
 * caller copies to the device once.  pcs_conv2d_planned then computes
 *   out = Conv(x) (+ beta * b)  (plan of adjoint = 0)  or  Conv^T(x) (+ beta * b)  (adjoint = 1)
 * Same arithmetic as pcs_conv2d up to floating-point summation order.  x != out. */
int pcs_conv2d_plan_tier(int kh, int kw, int off0, int off1);
int64_t pcs_conv2d_plan_bytes(int dtype, int kh, int kw, int off0, int off1);
int pcs_conv2d_plan_pack(int dtype, const double* psf, int kh, int kw, int off0, int off1, int adjoint,
                         void* plan_host);
int pcs_conv2d_planned(int dtype, const void* x, void* out, int64_t n0, int64_t n1, const void* plan, int tier,
                       const void* b, double beta, hipStream_t stream);

/* Convolve1D along `axis` of a 1..32-D array (pycsou/linop/conv.py:20-164 -> pylops Convolve1D):
 * out[i] = sum_t h[t] x[i + (off - t) e_axis].  Adjoint = flipped taps, off' = k-1-off. */
int pcs_conv1d(int dtype, const void* x, void* out, int ndim, const int64_t* dims, int axis, const void* taps,
               int k, int off, hipStream_t stream);

/* Two Convolve1D of a 3-D array's planes in one pass (pycsou/linop/conv.py:20-164 along axes 1
 * and 2): C_a along axis 1 (taps ha, ka, offa), C_b along axis 2 (taps hb, kb, offb), both with
 * pcs_conv1d's definition; out = C_b(C_a(in)) if vfirst else C_a(C_b(in)) (the two pcs_conv1d
 * calls in that order, same per-output sums to rounding).  in != out, 16-B aligned; ka, kb <= 15. */
int pcs_conv2d_sep_planes(int dtype, const void* in, void* out, int64_t nplanes, int64_t n1, int64_t n2,
                          const void* ha, int ka, int offa, const void* hb, int kb, int offb, int vfirst,
                          hipStream_t stream);

/* In-plane normal operator of a separable blur, every plane in one pass (pycsou/linop/conv.py:20-164
 * along axes 1 and 2; the in-plane half of grad F = C^T (C x - y), core/map.py:609-610):
 *   out = C_a^T C_b^T C_b C_a in   (C_a along axis 1: ha, ka, offa; C_b along axis 2: hb, kb, offb;
 *                                   zero boundary between the passes, as the four pcs_conv1d calls)
 * in != out, 16-B aligned, ka, kb <= 15.  PCS_EUNSUPPORTED when n2 % 4 != 0 or the horizontal
 * offset cannot be fitted to the strip layout (15-tap filter with offb % 4 == 1); nplanes == 0
 * only validates. */
int pcs_conv2d_sep_ata_planes(int dtype, const void* in, void* out, int64_t nplanes, int64_t n1, int64_t n2,
                              const void* ha, int ka, int offa, const void* hb, int kb, int offb, hipStream_t stream);

/* FFT-domain Convolve2D (pycsou/linop/conv.py:167-295, method='fft': scipy.signal.fftconvolve,
 * mode 'same' at pycsou's offset), for PSFs of any size at a cost independent of the PSF:
 *   forward out[i] = sum_j h[j] x[i + off - j] (+ beta b[i]);  adjoint out[i] = sum_j h[j] x[i - off + j]
 * (zero boundary; kh x kw PSF h in host fp64, row-major; offsets off0 < kh, off1 < kw).  Overlap-add
 * over blocks of at most 2048 x 2048 samples: the plan holds batched rocFFT R2C / C2R plans on a
 * zero-padded P0 x P1 grid per block (P = pcs_fftconv2d_grid(n, k): the smallest even 2-3-5-7-smooth
 * size >= block + k - 1, so the circular transforms are exact linear ones), their work buffer and
 * the PSF spectrum (formed at creation; create synchronises).
 * pcs_fftconv2d_apply: x != out, device arrays of n0*n1 (b may be NULL); stream-ordered, no
 * allocation (graph-capturable).  One plan per (dtype, shape, PSF); not thread-safe per plan. */
int64_t pcs_fftconv2d_grid(int64_t n, int k);
int pcs_fftconv2d_create(int dtype, int64_t n0, int64_t n1, const double* h, int kh, int kw, int off0, int off1,
                         void** handle);
int pcs_fftconv2d_apply(void* handle, const void* x, void* out, int adjoint, const void* b, double beta,
                        hipStream_t stream);
int pcs_fftconv2d_destroy(void* handle);

/* The axis-0 stage of grad F = C^T (C x - y) for a 3-D Convolve1D chain, in one pass
 * (pycsou/linop/conv.py:20-164 along axis 0, residual of core/map.py:609-610): on sub-volumes
 * of nsub planes of `plane` elements,
 *   r[p] = sum_t h[t] t[p + off - t] - y[p]  for p in [img_lo, img_hi) n [0, nsub) (0 elsewhere;
 *          t = 0 outside [0, nsub)),
 *   s[q] = sum_t h[k-1-t] r[q + k-1-off - t]  written for q in [q0, q1) only.
 * = pcs_conv1d(axis 0) + pcs_axpby(1, -1) + pcs_conv1d(axis 0, flipped) with 3 instead of 7
 * sub-volume passes.  k <= 15. */
int pcs_conv0_residual_adjoint(int dtype, const void* t, const void* y, void* s, int64_t nsub, int64_t plane,
                               const void* taps, int k, int off, int64_t img_lo, int64_t img_hi, int64_t q0,
                               int64_t q1, hipStream_t stream);

/* Masking / DownSampling / SubSampling (pycsou/linop/sampling.py:25-391).
 * pcs_gather:          out[i] = x[idx[i]], i < m         (Masking.__call__, sampling.py:192-193)
 * pcs_gather_or_zero:  out[p] = inv[p] >= 0 ? y[inv[p]] : 0, p < n
 *                      = (x = 0; x[idx] = y) with inv the inverse index map (Masking.adjoint,
 *                      sampling.py:195-198).  Indices are int32 (n < 2^31). */
int pcs_gather(int dtype, const void* x, const int32_t* idx, void* out, int64_t m, hipStream_t stream);
int pcs_gather_or_zero(int dtype, const void* y, const int32_t* inv, void* out, int64_t n, hipStream_t stream);

/* ---------------------------------------------------------------- prox / functionals */

/* L1Norm.prox (pycsou/func/penalty.py:194-245 via LpNorm.prox, func/base.py:239-240):
 * out = x - tau*clip(x/tau, -1, 1). */
int pcs_prox_l1(int dtype, const void* x, void* out, int64_t n, double tau, hipStream_t stream);
/* (lam*L1Norm).fenchel_prox (core/functional.py:207, 264-265):
 * out = w - sigma * prox_l1(w/sigma, (1/sigma)*lam). */
int pcs_fenchel_l1(int dtype, const void* w, void* out, int64_t n, double sigma, double lam, hipStream_t stream);
/* L21Norm.prox with pixel groups tile(arange(npix), d) (func/penalty.py:551-557):
 * out_g = max(1 - tau/||x_g||, 0) x_g. */
int pcs_prox_l21_pixel(int dtype, const void* x, void* out, int64_t npix, int d, double tau, hipStream_t stream);
int pcs_fenchel_l21_pixel(int dtype, const void* w, void* out, int64_t npix, int d, double sigma, double lam,
                          hipStream_t stream);
/* L21Norm.prox with arbitrary labels: `gid[n]` = index of the element's group in
 * [0, ngroups) (np.unique order); ws = ngroups doubles. */
int pcs_prox_l21_labels(int dtype, const void* x, void* out, int64_t n, const int32_t* gid, int64_t ngroups,
                        double tau, void* ws, hipStream_t stream);
/* The same prox with run-to-run identical group sums (ABI 10; replaces pcs_prox_l21_labels in
 * L21Norm.prox, func/penalty.py:525-560): `order[n]` lists the elements group by group (a stable
 * argsort of gid), `off[ngroups + 1]` the group boundaries in it, `maxlen` the largest group; each
 * group's sum of squares is taken in ascending element order (fp64) without atomics. */
int pcs_prox_l21_groups(int dtype, const void* x, void* out, int64_t n, const int32_t* gid, int64_t ngroups,
                        const int32_t* order, const int64_t* off, int64_t maxlen, double tau, void* ws,
                        hipStream_t stream);
/* L2Norm.prox (func/penalty.py:23-70 via LpNorm.prox + proj_l2_ball, math/prox.py:207-210):
 * v = x/tau; out = x - tau*(||v|| <= 1 ? v : v/||v||), with ||x||^2 read from the device
 * double `sumsq_dev` (pcs_reduce kind 0). */
int pcs_prox_l2(int dtype, const void* x, void* out, int64_t n, double tau, const double* sumsq_dev,
                hipStream_t stream);
/* SquaredL2Norm prox (new API, core/functional.py:100-103): out = x / (1 + 2 tau). */
int pcs_prox_sql2(int dtype, const void* x, void* out, int64_t n, double tau, hipStream_t stream);
/* NonNegativeOrthant / Segment projections (math/prox.py:295-297, 340-343). */
int pcs_proj_nonneg(int dtype, const void* x, void* out, int64_t n, hipStream_t stream);
int pcs_proj_segment(int dtype, const void* x, void* out, int64_t n, double a, double b, hipStream_t stream);

/* ---------------------------------------------------------------- algebra / reductions */

/* out = a*x + b*y (y may be NULL -> out = a*x).  Numpy-order: (a*x) + (b*y). */
int pcs_axpby(int dtype, const void* x, const void* y, void* out, int64_t n, double a, double b,
              hipStream_t stream);
/* out = (x - a*y) - b*w  (the PDS primal argument, proxalgs.py:348). */
int pcs_sub2(int dtype, const void* x, const void* y, const void* w, void* out, int64_t n, double a, double b,
             hipStream_t stream);
/* out = d * x elementwise (DiagonalOperator with a vector diagonal, pycsou/linop/base.py:551-579). */
int pcs_mul(int dtype, const void* x, const void* d, void* out, int64_t n, hipStream_t stream);
/* The two sums of one relative improvement ||old - new|| / ||old|| (proxalgs.py:370-383) in one
 * pass, fixed order: out_dev[0] = sum (old - new)^2, out_dev[1] = sum old^2 (the layout
 * pcs_pds_finalize reads).  ws >= pcs_reduce_ws_bytes(). */
int pcs_rel_sums(int dtype, const void* old, const void* nw, int64_t n, double* out_dev, void* ws,
                 hipStream_t stream);
/* Deterministic fp64 reductions into out_dev[0]: kind 0 = sum x^2, 1 = sum |x|,
 * 2 = sum (x-y)^2, 3 = sum x*y.  ws >= pcs_reduce_ws_bytes(). */
int64_t pcs_reduce_ws_bytes(void);
int pcs_reduce(int dtype, int kind, const void* x, const void* y, int64_t n, double* out_dev, void* ws,
               hipStream_t stream);

/* One fused AcceleratedProximalGradientDescent.update_iterand + update_diagnostics
 * (pycsou/opt/proxalgs.py:586-601 and 612-622), given g = grad F(x):
 *   x_t = G.prox(x - tau g, tau)   gkind PCS_G_NULL / PCS_G_NONNEG / PCS_G_SEGMENT [seg_a, seg_b] /
 *                                  PCS_APGD_G_L1 (lam * L1Norm: soft threshold tau*lam)
 *   x'  = x_t + a (x_t - aux)      aux = the previous x_t ('past_aux'), a = (t_old - 1) / t
 * writes x' -> xn, x_t -> aux_n (no aliasing) and sums_dev[0..1] = ||x - x'||^2, ||x||^2 (fp64,
 * fixed order).  ws >= pcs_reduce_ws_bytes(). */
enum { PCS_APGD_G_L1 = 3 };
int pcs_apgd_step(int dtype, const void* x, const void* g, const void* aux, void* xn, void* aux_n, int64_t n,
                  double tau, double a, int gkind, double lam, double seg_a, double seg_b, double* sums_dev,
                  void* ws, hipStream_t stream);

/* ---------------------------------------------------------------- fused PDS iteration */

/* One fused PrimalDualSplitting.update_iterand + update_diagnostics
 * (pycsou/opt/proxalgs.py:343-394) for 2-D images, K = Gradient(kind='forward'):
 *   g   = grad F(x)           (F kind: 0, x - y, Conv^T(Conv x - y) separable, or read from gbuf)
 *   x_t = prox_G((x - tau g) - tau K^T z)
 *   u   = 2 x_t - x
 *   z_t = H.fenchel_prox(z + sigma K u, sigma)      (H = lam*L1 or lam*L21 pixel groups)
 *   z'  = rho z_t + (1-rho) z ;  x' = rho x_t + (1-rho) x
 * plus per-block partials of ||x-x'||^2, ||x||^2, ||z-z'||^2, ||z||^2.
 * Slab form: the local arrays hold rows [row0 - halo, row0 + rows + halo) of a
 * global n0 x n1 image (halo rows of x >= pcs_pds2d_halo_x(half), of each z component >= 1,
 * of y >= (pcs_pds2d_halo_x(half) - 1)/2 + 1); only the slab's own rows of xn/zn are written. */
typedef struct {
  int dtype;          /* PCS_F32 / PCS_F64 */
  int fkind;          /* PCS_F_* */
  int hkind;          /* PCS_H_* */
  int gkind;          /* PCS_G_* */
  int64_t n0, n1;     /* global image */
  int64_t row0, rows; /* this slab: global rows [row0, row0+rows) */
  int halo_x, halo_z, halo_y; /* halo rows stored above/below the slab in x/xn, z/zn, y/gbuf */
  int half;           /* separable conv half width H (taps 2H+1, centred) */
  const void* taps0;  /* 2H+1 taps along axis 0 (rows), device */
  const void* taps1;  /* 2H+1 taps along axis 1 (cols), device */
  double tau, sigma, rho, lam, step0, step1, seg_a, seg_b;
  const void* x; void* xn; const void* z; void* zn; const void* y; const void* gbuf;
  double* partials;       /* [nblocks][4] */
  void* ctrl;             /* device control block (pcs_ctrl_*) ; NULL = always run */
  double* hist;           /* non-NULL: reduce the partials and run pcs_pds_finalize inside the
                             step launch (single GPU); NULL: only write `partials` */
  void* ws;               /* with hist or sums_out: pcs_pds2d_ws_bytes() bytes, zeroed once before first use */
  double* sums_out;       /* hist NULL, sums_out non-NULL (slab mode): the last workgroups reduce the
                             partials, then add pre_partials, into sums_out[4] (no loop control) */
  const double* pre_partials; /* [n_pre][4] partials of an earlier launch of the same iteration */
  int64_t n_pre;
  /* optional, fkind PCS_F_SEPCONV (fp32, half <= 7): grad F = N x - cty with N = Conv^T Conv
   * applied as two (4 tier + 1)-tap passes (the normal-operator row-marching kernel).  cty: Conv^T y
   * in y's layout (halo_y rows); ntaps: pcs_pds2d_ntaps_len(half) fp32 values, the window taps of
   * N along axis 0 and axis 1 and their exact rows on the tier rows / columns nearest each image
   * edge (layout in pds_nmarch.hpp; pycsou_amd.opt.engine.nmarch_taps builds it).  NULL: grad F
   * = Conv^T (Conv x - y) as four (2 tier + 1)-tap passes. */
  const void* cty;
  const void* ntaps;
  /* K (appended in ABI 2; all zero = the forward Gradient of the fields above).  kkind
   * PCS_K_GRAD_{FORWARD,BACKWARD,CENTERED}: K = Gradient(kind, edge, step0/1), z = [D0 x; D1 x];
   * PCS_K_LAPLACIAN: K = w0 D2_0 + w1 D2_1 (Laplacian(weights, step, edge), z has rows*n1
   * elements, H = lam*L1).  Non-forward K: the general-stencil row-marching kernel (fp32, F = NULL /
   * DENOISE / GRADBUF / SEPCONV with cty (grad F = N x - cty, N x into gbuf first) / CONV2D,
   * n1 % 4 == 0, 16-B aligned, at least two 64-column strips; slabs need halo rows x >= 2,
   * y >= 2, z >= 4); PCS_EUNSUPPORTED otherwise (pcs_pds2d_stencil_step covers the rest). */
  int kkind, edge;
  double w0, w1;
  /* fkind PCS_F_CONV2D (ABI 3): a general (non-separable) Convolve2D in F, grad F = Conv^T (Conv x - y)
   * by two pcs_conv2d_planned passes (conv_fwd / conv_adj: packed windows of tier conv_tier) over
   * the stored rows of x clipped to the image, into rbuf (the residual) and gbuf, inside this call
   * before the step (any K).  y, rbuf and gbuf share x's layout (halo_y == halo_x); a slab needs
   * halo_x >= conv_tier + 1 so that the rows the step reads are exact.  With fkind PCS_F_SEPCONV,
   * cty and a non-forward K, N x goes to gbuf the same way (halo_y == halo_x, halo_x >= 2 + 2 tier).
   * Neither runs banded (pcs_pds2d_step_bands: PCS_EUNSUPPORTED). */
  const void* conv_fwd;
  const void* conv_adj;
  int conv_tier, pad3;
  void* rbuf;
  /* ABI 6: a masked data-fidelity block (mkind PCS_M_L1LOSS), the reference notebook's TV-LAD
   * inpainting solved by ChambollePockSplitting (pycsou/opt/proxalgs.py:628-716):
   *   K = LinOpVStack(Masking(mask), K_s)  (linop/base.py:259-279, linop/sampling.py:125-196),
   *   H = ProxFuncHStack(L1Loss(dim=m, data=y), lam * L1Norm | lam * L21Norm on K_s x)
   *       (func/base.py:21-89, func/loss.py:222-268), K_s the kkind stencil above, F = 0 (fkind
   *       PCS_F_NULL), whole images only (rows == n0), the general-stencil row march (n1 % 4 == 0,
   *       at least two 64-column strips).
   * The masked dual block z_m is held EXPANDED to the image: zm / zmn are n0*n1 arrays (0 where the
   * mask is False, the sampled entries in image order elsewhere); ym is y expanded the same way
   * with NaN where the mask is False.  z / zn hold the K_s block only.  pcs_pds2d_run swaps zm / zmn
   * with x / xn.  The partials' z sums cover both blocks (= the reference's ||z|| over [z_m; z_s]). */
  int mkind, pad4;
  const void* ym;
  const void* zm;
  void* zmn;
  /* ABI 8: deferred finalization (with hist; NULL = finalize inside the launch).  The launch stores
   * its partials into `partials` without reducing them and finalizes the PREVIOUS launch's partials,
   * `fin_partials` (the other of two [nblocks][4] arrays, swapped with the iterate parity -- as
   * pcs_pds2d_run does), in a workgroup of its own while its tasks run: the reduction leaves the
   * critical path of every launch.  The stopping rule then acts one launch later (the extra iterate
   * goes to the buffer the engine does not select: the iterate after Ctrl.it iterations), and the
   * last launch's partials are finalized by pcs_pds_finalize_pending at the end of a run. */
  const double* fin_partials;
} pcs_pds2d_args;
enum { PCS_M_NONE = 0, PCS_M_L1LOSS = 1 };
/* 1 if pcs_pds2d_step runs these arguments (0: PCS_EUNSUPPORTED / invalid). */
int pcs_pds2d_supported(const pcs_pds2d_args* a);
/* Which kernel family pcs_pds2d_step runs for these arguments (-1: none), so an engine can tell the fused
 * normal-operator marches (one launch per iteration) from the split forms: */
enum {
  PCS_PATH_TILE = 1,      /* the tile kernel (pds_tile.hpp)                                         */
  PCS_PATH_MARCH = 2,     /* fp32 separable PSF, four-pass row march (pds_march.hpp)                */
  PCS_PATH_NMARCH = 3,    /* fp32 separable PSF, normal-operator march (pds_nmarch.hpp)             */
  PCS_PATH_PT = 4,        /* fp32 pointwise grad F, forward K (pds_pt.hpp)                          */
  PCS_PATH_SMARCH = 5,    /* general-stencil march, pointwise grad F (pds_smarch.hpp)               */
  PCS_PATH_SMARCH_NX = 6, /* N x pass into gbuf, then the general-stencil march (two launches)      */
  PCS_PATH_NM64 = 7,      /* fp64 separable PSF, fused normal-operator march (pds_nm64.hip)         */
  PCS_PATH_CONV2D = 8     /* two correlation passes, then the step with grad F from gbuf            */
};
int pcs_pds2d_path(const pcs_pds2d_args* a);
int pcs_pds2d_ntaps_len(int half); /* 64 + 32 * tier(half); -1 beyond tier 7 */

int pcs_pds2d_halo_x(int half);
int64_t pcs_pds2d_nblocks(const pcs_pds2d_args* a);
int64_t pcs_pds2d_ws_bytes(const pcs_pds2d_args* a);
/* One iteration (x, z -> xn, zn).  With fin_partials the launch finalizes the previous launch's
 * partials, not its own: see pcs_pds2d_run for the stop semantics and pcs_pds_finalize_pending. */
int pcs_pds2d_step(const pcs_pds2d_args* a, hipStream_t stream);
/* pcs_pds2d_step restricted to the slab's own rows [ra0, rb0) u [ra1, rb1)
 * (0 <= ra0 <= rb0 <= ra1 <= rb1 <= rows): writes x', z' on those rows and one partials row per
 * block (pcs_pds2d_nblocks_bands of them); hist must be NULL.  Same arithmetic per pixel as the
 * whole-slab step, so any split of the rows into launches gives bitwise the same x', z'.  The
 * multi-GPU loop runs the boundary bands and the interior band as separate launches so that the
 * halo exchange overlaps the interior.  Row-marching kernels only (fp32, L1/L21; F separable
 * conv of half width <= 7, or pointwise): PCS_EUNSUPPORTED otherwise. */
int64_t pcs_pds2d_nblocks_bands(const pcs_pds2d_args* a, int64_t ra0, int64_t rb0, int64_t ra1, int64_t rb1);
int pcs_pds2d_step_bands(const pcs_pds2d_args* a, int64_t ra0, int64_t rb0, int64_t ra1, int64_t rb1,
                         hipStream_t stream);
/* n iterations of pcs_pds2d_step launched back to back, ping-ponging (x, z) <-> (xn, zn) (and
 * partials <-> fin_partials); requires hist/ctrl/ws (in-kernel loop control).  The host-side form of
 * GenericIterativeAlgorithm.iterate's loop (pycsou/core/solver.py:55-76).
 * Without fin_partials an even n leaves the iterate in (x, z).  With fin_partials (deferred
 * finalization) the stopping rule acts one launch late: after a natural stop at iteration j the
 * next launch has already written iterate j + 1 into the other buffer pair, and the stop flag is
 * written mid-launch by that launch's finalizer workgroup.  The caller must then (1) call
 * pcs_pds_finalize_pending once the run is done, before reading ctrl or hist, and (2) select the
 * result by the parity of Ctrl.it (iterations done: even -> x, z; odd -> xn, zn), not by n. */
int pcs_pds2d_run(const pcs_pds2d_args* a, int64_t n, hipStream_t stream);

/* One fused PrimalDualSplitting.update_iterand + update_diagnostics (pycsou/opt/proxalgs.py:343-394)
 * for a 2-D image with a general finite-difference K (single GPU, whole image):
 *   kkind PCS_K_GRAD_{FORWARD,BACKWARD,CENTERED}: K = Gradient(kind, edge, step)  (diff.py:777-882),
 *         z = [D0 x; D1 x] (2 N), H = lam*L1 or lam*L21 over the two components;
 *   kkind PCS_K_LAPLACIAN: K = w0 D2_0 + w1 D2_1 (Laplacian(weights, step, edge), diff.py:885-957),
 *         z has N elements, H = lam*L1.
 *   fkind PCS_F_NULL: grad F = 0; PCS_F_DENOISE: grad F = x - g (g holds y); PCS_F_GRADBUF: g.
 * Same update and partials as pcs_pds2d_step (x_t = prox_G((x - tau g) - tau K^T z), ...); the
 * stencils are the standalone operators' (pcs_grad_fwd/adj, pcs_lap_fwd/adj) per element.  With
 * hist/ctrl/ws the last workgroups reduce the partials and run the stopping rule (as
 * pcs_pds2d_step); else only `partials` ([nblocks][4]) is written. */
typedef struct {
  int dtype, kkind, fkind, hkind, gkind, edge;
  int64_t n0, n1;
  double tau, sigma, rho, lam, step0, step1, w0, w1, seg_a, seg_b;
  const void* x; void* xn; const void* z; void* zn; const void* g;
  double* partials;
  void* ctrl;
  double* hist;
  void* ws; /* pcs_pds2d_stencil_ws_bytes() bytes, zeroed once before first use */
} pcs_pds2d_stencil_args;
int64_t pcs_pds2d_stencil_nblocks(const pcs_pds2d_stencil_args* a);
int64_t pcs_pds2d_stencil_ws_bytes(const pcs_pds2d_stencil_args* a);
int pcs_pds2d_stencil_step(const pcs_pds2d_stencil_args* a, hipStream_t stream);
/* n steps back to back, ping-ponging (x, z) <-> (xn, zn); requires hist/ctrl/ws. */
int pcs_pds2d_stencil_run(const pcs_pds2d_stencil_args* a, int64_t n, hipStream_t stream);

/* ---------------------------------------------------------------- multi-GPU row slabs
 * Native per-rank loop of the row-slab 2-D PDS (one process per GPU, RCCL over xGMI):
 * GenericIterativeAlgorithm.iterate (pycsou/core/solver.py:55-76) around
 * PrimalDualSplitting.update_iterand / update_diagnostics (pycsou/opt/proxalgs.py:343-394) for an
 * image split into contiguous row slabs.  Per iteration: the fused slab step, the four norm sums
 * all-gathered (4 doubles per rank, added in rank order, so every rank takes the same stop
 * decision) and the boundary rows of x', z' exchanged with the two neighbour ranks.
 * RCCL is bound at run time (dlopen librccl.so.1); pcs_comm_available() says whether it was. */
int pcs_comm_available(void);
int pcs_comm_id_bytes(void); /* size of the opaque unique id (ncclUniqueId) */
int pcs_comm_unique_id(void* id);                               /* rank 0; broadcast id to the others */
int pcs_comm_init(const void* id, int world, int rank, void** comm); /* collective over the ranks */
int pcs_comm_destroy(void* comm);

/* Halo buffers written by one parity of the ping-pong (up to 4 arrays, e.g. x', z0', z1'):
 * send_lo[k] (own first rows) goes to rank-1's recv_hi[k]; send_hi[k] (own last rows) to
 * rank+1's recv_lo[k]; bytes[k] bytes each.  Pointers toward a missing neighbour may be NULL. */
typedef struct {
  int nbuf;
  int pad;
  void* send_lo[4];
  void* recv_lo[4];
  void* send_hi[4];
  void* recv_hi[4];
  int64_t bytes[4];
} pcs_halo_set;

/* One grouped RCCL send/recv of the halo rows/planes with the two neighbour ranks on `stream`
 * (the exchange step of SURVEY 8(e)): send_lo -> rank-1's recv_hi, send_hi -> rank+1's recv_lo.
 * world == 1: no-op.  Graph-capturable (no allocation, no host synchronisation). */
int pcs_halo_exchange(void* comm, int rank, int world, const pcs_halo_set* h, hipStream_t stream);
/* dst[r * count .. (r + 1) * count) = src of rank r (RCCL all-gather over `comm` on `stream`; the
 * norm-sums step of SURVEY 8(e)); comm NULL (world 1 only): a device copy.  Graph-capturable. */
int pcs_allgather_f64(void* comm, int world, const double* src, double* dst, int64_t count, hipStream_t stream);

typedef struct {
  int world, rank;
  pcs_pds2d_args step[2]; /* parity p: x = X[p] -> xn = X[1-p] (hist/ws ignored, partials owned by the plan) */
  pcs_halo_set halo[2];   /* halo[p]: the buffers step[p] writes (X[1-p], Z[1-p]) */
  void* ctrl;             /* loop control block (pcs_ctrl_init2), identical on every rank */
  double* hist;
  int64_t band;           /* boundary band rows (>= the x halo depth) for the overlapped schedule */
  int overlap;            /* 1: boundary bands, then the halo exchange on a side stream while the
                             interior band runs (row-marching kernels only; else the serial schedule) */
  int pad2;
} pcs_slab2d_desc;

/* comm may be NULL when world == 1.  The plan owns its partials/sums buffers, a side stream and
 * events (allocated here, not in pcs_slab2d_run). */
int pcs_slab2d_create(const pcs_slab2d_desc* d, void* comm, void** plan);
int pcs_slab2d_overlapped(const void* plan);
/* n iterations starting at parity p0 (no host synchronisation; the stop flag in ctrl makes the
 * iterations after the reference loop's exit return at once). */
int pcs_slab2d_run(void* plan, int64_t n, int p0, hipStream_t stream);
int pcs_slab2d_destroy(void* plan);

/* Communication-avoiding form of the row-slab loop (ABI 9; the same iteration as pcs_slab2d_run,
 * GenericIterativeAlgorithm.iterate of pycsou/core/solver.py:55-76 across ranks): the halos of x, z, y
 * are stored `depth` iterations deep and exchanged once per chunk of `depth` iterations.  Iteration j of
 * a chunk computes the own rows plus (m - j) * reach redundant rows of each halo (clipped at the image),
 * so the own rows after the chunk are bitwise the single-GPU iterate; the m x 4 norm sums of a chunk are
 * all-gathered once and pcs_pds_reduce_finalize_k runs the loop control over them in iteration order.
 * Buffers rotate through nbuf sets (step[b]: X[b] -> X[(b + 1) % nbuf]); after n iterations from set 0
 * the iterate is set n % nbuf, and after a natural stop set (Ctrl.it % nbuf).  Needs the banded
 * (row-marching) step: PCS_EUNSUPPORTED at create otherwise. */
#define PCS_DEEP_MAX 8
typedef struct {
  int world, rank;
  int depth;              /* 1 <= depth <= PCS_DEEP_MAX: iterations per exchange */
  int nbuf;               /* buffer sets in the rotation, >= max(2, depth) */
  int reach;              /* even, >= the rows one iteration reads past its own (x and z) */
  int local;              /* 1: no communicator -- the plan runs only under pcs_slab2d_deep_run_local */
  pcs_pds2d_args step[PCS_DEEP_MAX]; /* plain slabs with the deep halos (>= (depth - 1) reach + 1 rows) */
  pcs_halo_set halo[PCS_DEEP_MAX];   /* the deep halos of X[b], Z[b] */
  void* ctrl;
  double* hist;
} pcs_slab2d_deep_desc;
int pcs_slab2d_deep_create(const pcs_slab2d_deep_desc* d, void* comm, void** plan);
/* n iterations from buffer set b0: chunks of depth (the last one shorter), each followed by the
 * all-gather, the loop control and the deep-halo exchange. */
int pcs_slab2d_deep_run(void* plan, int64_t n, int b0, hipStream_t stream);
/* The same chunks for all `nplans` ranks of one image in ONE process (plans[i] of ranks 0..nplans-1,
 * one stream): the all-gather and the halo exchange as device copies -- the parity tests' transport. */
int pcs_slab2d_deep_run_local(void* const* plans, int nplans, int64_t n, int b0, hipStream_t stream);
int pcs_slab2d_deep_destroy(void* plan);
/* Loop control over k iterations' sums gathered as [world][k][4] (rank r's k rows of 4 sums, each summed
 * across ranks in the order pcs_pds_reduce_finalize uses), in iteration order. */
int pcs_pds_reduce_finalize_k(const double* gathered, int world, int k, void* ctrl_dev, double* hist,
                              hipStream_t stream);

/* One fused PrimalDualSplitting.update_iterand + update_diagnostics for 3-D volumes
 * (pycsou/opt/proxalgs.py:343-394), K = Gradient(kind='forward') in 3-D
 * (pycsou/linop/diff.py:777-882): the same update as pcs_pds2d_step with three gradient
 * components (z = [D0 x; D1 x; D2 x]) and grad F taken from `g`:
 *   fkind PCS_F_NULL: 0;  PCS_F_DENOISE: x - g (g holds y);  PCS_F_GRADBUF: g.
 * Volume n0 x n1 x n2 (C order, n2 % 4 == 0); slab form as in 2-D along axis 0: the local
 * arrays hold planes [plane0 - halo, plane0 + planes + halo); `g` must supply planes
 * [0, planes] (one past the slab) when planes < n0 -- [-1, planes] for the backward / centred
 * kinds (kkind), which also need halo_z >= 2 (K^T z at plane p reads z0 of p - 1 .. p + 1). */
typedef struct {
  int dtype, fkind, hkind, gkind;
  int64_t n0, n1, n2;
  int64_t plane0, planes;
  int halo_x, halo_z, halo_g;
  int pad;
  double tau, sigma, rho, lam, step0, step1, step2, seg_a, seg_b;
  const void* x; void* xn; const void* z; void* zn; const void* g;
  double* partials;       /* [nblocks][4] */
  void* ctrl;             /* device control block; NULL = always run */
  double* hist;           /* non-NULL: in-launch reduce + loop control (single GPU) */
  void* ws;               /* with hist: pcs_pds3d_ws_bytes() bytes, zeroed once */
  int kkind;              /* PCS_FORWARD (0), PCS_BACKWARD or PCS_CENTERED: Gradient(kind) */
  int edge;               /* Gradient(edge=...): the centred kind's one-sided end samples */
  /* fkind PCS_F_CONV0 (ABI 5; fp32, forward K): the axis-0 Convolve1D of a separable 3-D PSF inside
   * the step, grad F = C0^T (C0 g - conv0_w) along axis 0 with `g` holding the in-plane normal
   * operator C12^T C12 x and conv0_w = C12^T y (both with halo_g planes; halo_g >= conv0_k when
   * planes < n0); conv0_taps: conv0_k <= 15 device taps, conv0_off the Convolve1D offset.  Replaces
   * the pcs_conv0_residual_adjoint pass (pycsou/linop/conv.py:20-164 along axis 0). */
  const void* conv0_w;
  const void* conv0_taps;
  int conv0_k, conv0_off;
} pcs_pds3d_args;

int64_t pcs_pds3d_nblocks(const pcs_pds3d_args* a);
int64_t pcs_pds3d_ws_bytes(const pcs_pds3d_args* a);
int pcs_pds3d_step(const pcs_pds3d_args* a, hipStream_t stream);
/* pcs_pds3d_step restricted to the slab's own planes [a0, b0) u [a1, b1)
 * (0 <= a0 <= b0 <= a1 <= b1 <= planes): writes x', z' on those planes and one partials row per
 * block (pcs_pds3d_nblocks_bands of them); hist must be NULL.  Per-voxel arithmetic is that of
 * the whole-slab step (bitwise the same x', z' for any split).  The multi-GPU loop updates the
 * boundary bands first, starts their halo exchange, and updates the interior meanwhile. */
int64_t pcs_pds3d_nblocks_bands(const pcs_pds3d_args* a, int64_t a0, int64_t b0, int64_t a1, int64_t b1);
int pcs_pds3d_step_bands(const pcs_pds3d_args* a, int64_t a0, int64_t b0, int64_t a1, int64_t b1,
                         hipStream_t stream);

/* Device control block for the hipGraph-captured loop:
 * int32 [0]=it (next iteration), [1]=stopped, [2]=min_iter, [3]=max_iter, [4]=has_dual,
 * [5]=hist_len, [6]=pend (deferred finalization: the last launch's partials wait); double at byte 32:
 * accuracy_threshold.
 * hist: double[2*(max(min_iter,max_iter)+1)+2] = (primal, dual) relative improvement per iteration. */
int64_t pcs_ctrl_bytes(void);
int pcs_ctrl_init(void* ctrl_dev, int min_iter, int max_iter, double thr, int has_dual, hipStream_t stream);
/* Reduce [nparts][4] partials (fixed order, fp64) into sums[4]. */
int pcs_reduce_partials(const double* partials, int64_t nparts, double* sums, hipStream_t stream);
/* From sums[4] (global), write hist[it], advance it, set stopped per
 * GenericIterativeAlgorithm.iterate's loop condition (pycsou/core/solver.py:65-66). */
int pcs_pds_finalize(const double* sums, void* ctrl_dev, double* hist, hipStream_t stream);
/* Single-GPU shortcut: pcs_reduce_partials + pcs_pds_finalize in one launch. */
int pcs_pds_reduce_finalize(const double* partials, int64_t nparts, void* ctrl_dev, double* hist,
                            hipStream_t stream);
/* End of a deferred-finalization run (pcs_pds2d_args.fin_partials): finalize the last launch's
 * [nparts][4] partials if they are pending and the loop has not stopped (a no-op otherwise), in the
 * summation order of the in-launch finalizer. */
int pcs_pds_finalize_pending(const double* partials, int64_t nparts, void* ctrl_dev, double* hist,
                             hipStream_t stream);
/* pcs_ctrl_init with an explicit history length (doubles in `hist`). */
int pcs_ctrl_init2(void* ctrl_dev, int min_iter, int max_iter, double thr, int has_dual, int hist_len,
                   hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* PYCSOU_HIP_H */
